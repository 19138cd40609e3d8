set -o pipefail
cd /root/repo
timeout -k 10 800 python -u -m pytest tests/test_search_gpu.py tests/test_tsplib.py -x -v --timeout 300 --timeout-method thread > gpurun_out/k2_tests.log 2>&1 || exit 1
TSPGPU_SEARCH_DEBUG=1 timeout -k 10 120 python tools/k2_solve_time.py 10 > gpurun_out/k2_solve_time.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /root/repo/gpurun_out/k2prof -o k2 -- python3 /root/repo/tools/k2_solve_time.py 5 > /root/repo/gpurun_out/k2_prof.log 2>&1 || exit 3
