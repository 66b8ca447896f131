#!/bin/bash
# A/B of two builds on the graphed SAC update (tools/agent_profile.py update wall time),
# alternated: bash tools/ab_upd.sh <variant-suffix>   (trafficrl/libtrafficrl<suffix>.so vs the shipped one)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out && export TMPDIR=/tmp
L=sac-gat-her_transportationrl_amd/trafficrl
for r in 1 2; do for v in "$1" ""; do
  TRX_LIB=$PWD/$L/libtrafficrl$v.so timeout -k 10 200 python tools/agent_profile.py 4096 update > gpurun_out/abupd$v.$r.log 2>&1 || exit 1
  echo "libtrafficrl$v: $(tail -1 gpurun_out/abupd$v.$r.log)"
done; done
