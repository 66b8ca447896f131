#!/bin/bash
# Cross-process determinism probe (tests/det_worker.py): two runs per setting,
# first differing iteration printed.  Settings: default, serial update streams.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/det
for mode in default serial; do
    for k in 1 2; do
        if [ $mode = serial ]; then export TRX_DET_SERIAL=1; else unset TRX_DET_SERIAL; fi
        timeout -k 10 200 python tests/det_worker.py gpurun_out/det/${mode}_$k.pt 8 > gpurun_out/det/${mode}_$k.log 2>&1 || exit 1
    done
    python - "$mode" <<'PY'
import sys, torch
m = sys.argv[1]
a = torch.load(f"gpurun_out/det/{m}_1.pt", weights_only=True); b = torch.load(f"gpurun_out/det/{m}_2.pt", weights_only=True)
diff = [(i, [k for k in ra if ra[k] != rb.get(k)]) for i, (ra, rb) in enumerate(zip(a["trace"], b["trace"])) if ra != rb]
print(m, "identical" if not diff else f"first difference at iteration {diff[0][0]}: {diff[0][1]}")
PY
done
