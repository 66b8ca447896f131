#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes into profiles/<tag>_pmc.json, per kernel.

usage: pmc_summary.py <tag> <pass-dir glob under gpurun_out/> [kernel-substring ...]

Every kernel whose demangled name contains one of the substrings (default:
"env_kernel") gets its per-dispatch mean of every counter and the derived
shares below, plus `code_sha16`: trafficrl.codeobj.kernel_code_hash of that
kernel's machine code in the library the passes ran (the in-tree
libtrafficrl.so, whose whole-file hash gpu_session.sh records as
lib_sha16).  bench.py attaches counters to a run only when the kernel it
times has the same code hash: another kernel changing does not drop them.

HBM traffic per launch = (FETCH_SIZE + WRITE_SIZE) x 1024 B (rocprofv3 reports
KB).  MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE reads exactly half the
bytes of a wide (16 B/lane) coalesced stream; other widths are uncalibrated,
so the raw sum is reported and the x2 read correction is given beside it.
Time-like SQ counters count quad-cycles (§Per-instruction cycle constants).
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sac-gat-her_transportationrl_amd"))

from trafficrl import codeobj  # noqa: E402

LIB = os.path.join(ROOT, "sac-gat-her_transportationrl_amd", "trafficrl", "libtrafficrl.so")


def short_name(kernel_name):
    """'void trx::env_kernel_s<24, 2>(trx::DevGraph, ...)' -> 'trx::env_kernel_s<24, 2>'."""
    s = kernel_name.replace("void ", "", 1).replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return s[:i]
    return s


def mangled_key(short):
    """Mangled-name substring of a trx:: kernel: 'trx::k<24, 2>' -> '1kILi24ELi2EE'
    (length-prefixed identifier + integer template arguments)."""
    m = re.match(r"(?:trx::)?(\w+)(?:<(.*)>)?$", short)
    if not m:
        return None
    name, targs = m.group(1), m.group(2)
    key = f"{len(name)}{name}"
    if targs is not None:
        args = [a.strip() for a in targs.split(",")]
        if not all(re.fullmatch(r"-?\d+|true|false", a) for a in args):
            return None
        enc = {"true": "Lb1E", "false": "Lb0E"}
        key += "I" + "".join(enc.get(a) or (f"Li{a}E" if not a.startswith("-") else f"Lin{a[1:]}E")
                             for a in args) + "E"
    return key


def derive(mean):
    out = {}
    if "SQ_INSTS_VALU" in mean and "GRBM_GUI_ACTIVE" in mean:
        # a wave64 VALU instruction holds its SIMD 4 cycles; GRBM_GUI_ACTIVE is
        # summed over the 8 XCDs; 256 CUs x 4 SIMDs
        cyc = mean["GRBM_GUI_ACTIVE"] / 8
        out["valu_busy_frac"] = 4 * mean["SQ_INSTS_VALU"] / (cyc * 1024)
        out["gpu_cycles"] = cyc
    if "SQ_LDS_BANK_CONFLICT" in mean and mean.get("SQ_ACTIVE_INST_LDS"):
        out["lds_bank_conflict_frac"] = mean["SQ_LDS_BANK_CONFLICT"] / mean["SQ_ACTIVE_INST_LDS"]
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        out["hbm_bytes_per_launch_raw"] = (mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
        out["hbm_bytes_per_launch_fetch_x2"] = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024
        out["fetch_bytes"] = mean["FETCH_SIZE"] * 1024
        out["write_bytes"] = mean["WRITE_SIZE"] * 1024
    if mean.get("SQ_WAVE_CYCLES"):
        w = mean["SQ_WAVE_CYCLES"]
        for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_INST_CYCLES_VMEM", "SQ_WAIT_INST_LDS"):
            if k in mean:
                out[k.lower().replace("sq_", "") + "_frac"] = mean[k] / w
    if mean.get("SQ_WAVES") and mean.get("SQ_WAVE_CYCLES") and "GRBM_GUI_ACTIVE" in mean:
        # mean resident waves per SIMD over the kernel's span (SQ_WAVE_CYCLES in quad-cycles)
        out["mean_waves_per_simd"] = 4 * mean["SQ_WAVE_CYCLES"] / (mean["GRBM_GUI_ACTIVE"] / 8) / 1024
    if mean.get("SQ_INSTS_VALU") and mean.get("SQ_WAVES"):
        out["valu_insts_per_wave"] = mean["SQ_INSTS_VALU"] / mean["SQ_WAVES"]
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04_sf"
    src_glob = sys.argv[2] if len(sys.argv) > 2 else "pmc[0-9]"
    subs = sys.argv[3:] or ["env_kernel"]
    agg = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", src_glob, "**", "*counter_collection.csv"),
                              recursive=True)):
        for r in csv.DictReader(open(f)):
            short = short_name(r["Kernel_Name"])
            if not any(s in short for s in subs):
                continue
            # one record per (kernel, grid): the acting pass's 4096-graph launches and the
            # update's 256-graph launches of the same kernel are different workloads
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
            agg[(short, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", src_glob, "**", "*kernel_trace.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            short = short_name(r["Kernel_Name"])
            if any(s in short for s in subs):
                grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
                dur[(short, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    sha_file = os.path.join(ROOT, "gpurun_out", "lib_sha16.txt")
    out = {"lib_sha16": open(sha_file).read().split()[0] if os.path.exists(sha_file) else None,
           "source": f"gpurun_out/{src_glob}", "kernels": {}}
    import hashlib
    local = hashlib.sha256(open(LIB, "rb").read()).hexdigest()[:16]
    if out["lib_sha16"] and out["lib_sha16"] != local:
        sys.exit(f"the passes ran libtrafficrl.so {out['lib_sha16']}, the in-tree library is {local}: "
                 "code hashes would describe another build")
    for (short, grid), cnt in sorted(agg.items()):
        mean = {k: sum(v) / len(v) for k, v in cnt.items()}
        key = mangled_key(short)
        rec = {"kernel": short, "grid_threads": grid, "mangled_key": key,
               "code_sha16": codeobj.kernel_code_hash(LIB, key) if key else None,
               "dispatches": {k: len(v) for k, v in cnt.items()}, "per_dispatch_mean": mean}
        if dur.get((short, grid)):
            rec["mean_duration_us_under_pmc"] = sum(dur[(short, grid)]) / len(dur[(short, grid)])
        rec.update(derive(mean))
        out["kernels"][f"{short} grid={grid}"] = rec
    path = os.path.join(ROOT, "profiles", f"{tag}_pmc.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
