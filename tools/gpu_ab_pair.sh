#!/bin/bash
# A/B of env-kernel library variants (tools/ab_env.py, one process per library, alternated),
# after the env parity tests of the main library.  usage: gpu_ab_pair.sh <variant-name>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=sac-gat-her_transportationrl_amd/trafficrl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py tests/test_gpu_parity.py tests/test_known_answers.py > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in main "$@"; do
    lib=$T/libtrafficrl.so; [ "$v" = main ] || lib=$T/libtrafficrl_$v.so
    if [ "$v" = sparse ]; then lib=$T/libtrafficrl.so; export TRX_KERNEL=sparse; else unset TRX_KERNEL; fi
    timeout -k 10 120 python tools/ab_env.py $lib 4096 30 2>&1 | grep -v amdgpu.ids | sed "s/^/[$v] /" | tee -a gpurun_out/ab.log
    [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
  done
done
