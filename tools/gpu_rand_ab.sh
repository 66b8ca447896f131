#!/bin/bash
# Random-damage A/B: env parity tests, tools/ab_env.py per library, then the random-damage
# env bench per library (alternated).  usage: gpu_rand_ab.sh <variant>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=$PWD/sac-gat-her_transportationrl_amd/trafficrl
bash tools/gpu_ab_pair.sh "$@" || exit $?
for rep in 1 2; do
  for v in main "$@"; do
    if [ "$v" = main ]; then unset TRX_LIB; else export TRX_LIB=$T/libtrafficrl_$v.so; fi
    timeout -k 10 300 python bench.py --workload env --damage random --steps 66 --warmup 22 --no-cpu > gpurun_out/rand_$v.log 2>&1 || exit 1
    python - "$v" gpurun_out/rand_$v.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
b = d["breakdown_ms_per_step"] if d.get("breakdown_ms_per_step") else {}
print(f"[{sys.argv[1]}] random-damage env: {d['value']:.0f} env steps/s, {d['ms_per_step']:.3f} ms/step, "
      f"step kernel {d['env_launches']['step_mean_ms']:.3f} ms, reset {d['env_launches']['reset_mean_ms']:.2f} ms")
PY
  done
done
unset TRX_LIB
