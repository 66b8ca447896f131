#!/bin/bash
# Cross-process determinism probe (tests/det_worker.py): two runs per setting,
# first differing iteration printed.  Settings (DET_MODES): default, serial (no side
# streams in the update), fwd / bwd (only that phase of the fused update serial),
# nan (default, fresh float blocks NaN-poisoned: tests/det_worker.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/det
for mode in ${DET_MODES:-default serial}; do
    for k in 1 2; do
        unset TRX_DET_SERIAL TRX_DET_FWD_GROUPS TRX_DET_NOGRAPH
        export TRX_DET_CONCURRENT=1   # the probe studies the concurrent default
        fill=0
        case $mode in
            serial) export TRX_DET_SERIAL=1 ;;
            fwd|bwd) export TRX_DET_SERIAL=$mode ;;
            nan) fill=1 ;;
            nograph) export TRX_DET_NOGRAPH=1 ;;
            g*) export TRX_DET_FWD_GROUPS=$(echo ${mode#g} | tr _ '|') ;;
        esac
        timeout -k 10 200 python tests/det_worker.py gpurun_out/det/${mode}_$k.pt ${DET_ITERS:-8} $fill > gpurun_out/det/${mode}_$k.log 2>&1 || exit 1
    done
    python - "$mode" <<'PY'
import sys, torch
m = sys.argv[1]
a = torch.load(f"gpurun_out/det/{m}_1.pt", weights_only=True); b = torch.load(f"gpurun_out/det/{m}_2.pt", weights_only=True)
diff = [(i, [k for k in ra if ra[k] != rb.get(k)]) for i, (ra, rb) in enumerate(zip(a["trace"], b["trace"])) if ra != rb]
print(m, "identical" if not diff else f"first difference at iteration {diff[0][0]}: {diff[0][1]}")
PY
    rm -f gpurun_out/det/${mode}_*.pt
done
