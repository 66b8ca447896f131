#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc1..4) for the env kernel
into profiles/<tag>_pmc.json.

HBM traffic per launch = (FETCH_SIZE + WRITE_SIZE) x 1024 B (rocprofv3 reports
KB).  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads exactly half the
bytes of a wide (16 B/lane) coalesced stream; other widths are uncalibrated.
This kernel's loads are 4-byte per lane (SoA link arrays), so the raw value is
reported and the x2 wide-stream correction is given as an upper bound.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src_glob = sys.argv[2] if len(sys.argv) > 2 else "pmc[0-9]"
agg = defaultdict(list)
names = defaultdict(int)
for f in sorted(glob.glob(os.path.join(root, "gpurun_out", src_glob, "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "env_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
            names[r["Kernel_Name"].split("(")[0].replace("void ", "")] += 1
mean = {k: sum(v) / len(v) for k, v in agg.items()}
out = {"kernel": max(names, key=names.get) if names else None, "dispatches": {k: len(v) for k, v in agg.items()},
       "per_dispatch_mean": mean}
if "SQ_INSTS_VALU" in mean and "GRBM_GUI_ACTIVE" in mean:
    # VALU issue: a wave64 VALU instruction holds its SIMD 4 cycles; GRBM_GUI_ACTIVE
    # is summed over the 8 XCDs; 256 CUs x 4 SIMDs
    cyc = mean["GRBM_GUI_ACTIVE"] / 8
    out["valu_busy_frac"] = 4 * mean["SQ_INSTS_VALU"] / (cyc * 1024)
if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_ACTIVE_INST_LDS"):
    out["lds_bank_conflict_frac"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_ACTIVE_INST_LDS"]
if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
    raw = (mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
    out["hbm_bytes_per_launch_raw"] = raw
    out["hbm_bytes_per_launch_fetch_x2_upper"] = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
if "SQ_WAVE_CYCLES" in mean:
    w = mean["SQ_WAVE_CYCLES"]
    out["wait_any_frac"] = mean.get("SQ_WAIT_ANY", 0) / w
    out["active_inst_any_frac"] = mean.get("SQ_ACTIVE_INST_ANY", 0) / w
    out["wait_inst_any_frac"] = mean.get("SQ_WAIT_INST_ANY", 0) / w
# the library the passes ran (tools/gpu_session.sh writes its hash on the box);
# bench.py attaches these counters only to runs of the same binary
sha_file = os.path.join(root, "gpurun_out", "lib_sha16.txt")
if os.path.exists(sha_file):
    out["lib_sha16"] = open(sha_file).read().split()[0]
path = os.path.join(root, "profiles", f"{tag}_pmc.json")
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out, indent=1))
