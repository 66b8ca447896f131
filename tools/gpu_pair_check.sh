set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_gpu_fallback.py tests/test_known_answers.py > gpurun_out/p1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then tail -40 gpurun_out/p1.log; exit $rc; fi
timeout -k 10 180 python tools/ab_env.py sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl.so 4096 20 > gpurun_out/ab_pair.log 2>&1 && \
TRX_KERNEL=sparse timeout -k 10 180 python tools/ab_env.py sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl.so 4096 20 > gpurun_out/ab_sparse.log 2>&1 && \
timeout -k 10 180 python tools/ab_env.py sac-gat-her_transportationrl_amd/trafficrl/libtrafficrl.so 4096 20 >> gpurun_out/ab_pair.log 2>&1
rc=$?
cat gpurun_out/ab_pair.log gpurun_out/ab_sparse.log | grep -v Warn
tail -3 gpurun_out/p1.log
exit $rc
