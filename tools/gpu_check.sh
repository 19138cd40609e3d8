#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Each GPU step has its own time limit; a fault / abort / timeout ends the
# script (no further GPU work in the same call).  Usage:
#   gpurun -- 'bash tools/gpu_check.sh [tag] [steps...]'   steps: tests smoke bench prof
set -u
cd "$(dirname "$0")/.."
TAG=${1:-r01}
shift || true
STEPS=${*:-tests smoke bench prof}
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp

run() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -n 25 "$OUT/$name.log" >&2
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "== stopping after $name (rc=$rc)" >&2
        exit $rc
    fi
    return $rc
}

for s in $STEPS; do
    case $s in
    tests) run gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ;;
    smoke) run smoke 180 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python -u bench.py ;;
    prof)
        rm -rf $OUT/prof_$TAG
        run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
            python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-tto ;;
    esac
done
exit 0
