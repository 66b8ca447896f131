#!/bin/bash
# Guarded GPU session for gpurun: every GPU step has its own time limit; the
# script stops at the first step that faults, aborts or times out (statuses
# other than 0 and pytest's 1 = "tests failed").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # step <name> <timeout-seconds> <cmd...>
    local name=$1 secs=$2; shift 2
    echo "=== $name ($(date +%T))"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
    return 0
}
for s in "$@"; do
    case $s in
        tests) step gpu_tests 600 python -m pytest tests -m gpu -x -q ;;
        testsall) step gpu_tests 900 python -m pytest tests -m gpu -q ;;
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        bench) step bench 600 python bench.py ;;
        benchq) step bench 400 python bench.py --steps 44 --warmup 22 --cpu-seconds 5 ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 44 --warmup 22 --no-cpu ;;
        benchab) step bench_lane 300 env TRX_KERNEL=lane python bench.py --steps 44 --warmup 22 --no-cpu
                 step bench_quad 300 python bench.py --steps 44 --warmup 22 --no-cpu ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
