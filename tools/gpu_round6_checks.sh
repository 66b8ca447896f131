cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 700 --timeout-method thread tests/test_pk_hazard.py tests/test_dist_gpu.py -rxX > gpurun_out/t2.log 2>&1
rc=$?; tail -25 gpurun_out/t2.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/bmm_fault_probe.py > gpurun_out/bmm_probe.log 2>&1
echo "probe rc=$?"; cat gpurun_out/bmm_probe.log
