#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_k1_variants_gpu.py tests/test_i32_gpu.py tests/test_tsplib.py tests/test_bench_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r05/k1_tests.log 2>&1; echo k1 tests rc=$?; tail -3 gpurun_out/r05/k1_tests.log
