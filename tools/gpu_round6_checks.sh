#!/bin/bash
# Round-6 GPU checks, each step under its own limit; the batched-GEMM fault probe runs
# last (a fault there ends the call).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/gpu_ab_pair.sh prev sparse || exit $?
timeout -k 10 900 python -u -m pytest -v --timeout 700 --timeout-method thread tests/test_pk_hazard.py tests/test_dist_gpu.py -rxX > gpurun_out/t2.log 2>&1
rc=$?; tail -25 gpurun_out/t2.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/bmm_fault_probe.py > gpurun_out/bmm_probe.log 2>&1
echo "probe rc=$?"; cat gpurun_out/bmm_probe.log
