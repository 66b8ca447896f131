"""Static scan for the packed-FP32 -> DPP pattern (DESIGN §5 "determinism") in
gfx950 code objects that this repo does not build: hipBLASLt's Tensile
libraries and the gfx950 code objects inside torch's HIP library.

For every kernel it counts packed-FP32 results (v_pk_add_f32 / v_pk_mul_f32 /
v_pk_fma_f32) and reports each one whose destination register pair is read by a
DPP instruction within WINDOW instructions -- the pattern whose last 16 lanes
were seen to arrive late in round 5.  CPU only (llvm-objdump).

usage: python tools/pk_dpp_scan.py [--window 8] [--torch] [glob ...]
       (default globs: the bf16 Tensile libraries, Type_BB* / Type_BS*)"""
import argparse
import glob
import os
import re
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
PK = re.compile(r"\bv_pk_(add|mul|fma)_f32\s+v\[(\d+):(\d+)\]")
DPP = re.compile(r"(quad_perm|row_shl|row_shr|row_ror|row_mirror|row_half_mirror|row_bcast|wave_sh|wave_ro|"
                 r"row_share|row_xmask|_dpp)")
VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def regs_read(line):
    """VGPR numbers named after the destination operand of an instruction line."""
    parts = line.split(None, 1)
    if len(parts) < 2:
        return set()
    ops = parts[1].split(",", 1)
    if len(ops) < 2:
        return set()
    out = set()
    for m in VREG.finditer(ops[1]):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def scan_text(text, window):
    kernels, cur, insts = {}, None, []

    def flush():
        if cur is None:
            return
        n_pk, hits = 0, []
        for i, ln in enumerate(insts):
            m = PK.search(ln)
            if not m:
                continue
            n_pk += 1
            dst = set(range(int(m.group(2)), int(m.group(3)) + 1))
            for j in range(i + 1, min(len(insts), i + 1 + window)):
                nxt = insts[j]
                if DPP.search(nxt) and regs_read(nxt) & dst:
                    hits.append((i, j - i, ln.strip()[:60], nxt.strip()[:80]))
                    break
        kernels[cur] = (len(insts), n_pk, hits)

    for ln in text.splitlines():
        if ln.endswith(">:") and "<" in ln:
            flush()
            cur = ln[ln.index("<") + 1:-2]
            insts = []
        elif cur is not None and ln.startswith("\t") and ln.strip() and not ln.strip().startswith(";"):
            insts.append(ln.split("//")[0])
    flush()
    return kernels


def disasm(path, tmp):
    """Disassembly of a gfx950 code object; Tensile's .co files are offload bundles."""
    r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", path], capture_output=True, text=True)
    if r.returncode == 0:
        return r.stdout
    dst = os.path.join(tmp, os.path.basename(path) + ".elf")
    subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={path}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--output={dst}"], capture_output=True)
    r = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", dst], capture_output=True, text=True)
    return r.stdout


def torch_code_objects(tmp):
    """gfx950 code objects of torch's HIP library: its .hip_fatbin section is a run of
    clang offload bundles (one per translation unit, plain or compressed), each unbundled
    for the gfx950 target."""
    import torch
    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_hip.so")
    sec = os.path.join(tmp, "fatbin.bin")
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", "--dump-section", f".hip_fatbin={sec}", lib,
                    os.path.join(tmp, "discard.so")], check=True, capture_output=True)
    data = open(sec, "rb").read()
    spans, o = [], 0
    while True:  # compressed bundles ("CCOB", version 2: u32 total size at byte 8) back to back
        o = data.find(b"CCOB", o)
        if o < 0:
            break
        ver = int.from_bytes(data[o + 4:o + 6], "little")
        size = int.from_bytes(data[o + 8:o + (12 if ver == 2 else 16)], "little")
        if size <= 0 or o + size > len(data):
            o += 4
            continue
        spans.append((o, o + size))
        o += size
    out = []
    for k, (st, end) in enumerate(spans):
        b = os.path.join(tmp, f"b{k}.bundle")
        with open(b, "wb") as f:
            f.write(data[st:end])
        dst = os.path.join(tmp, f"b{k}.gfx950.co")
        r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={b}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dst}"], capture_output=True)
        os.remove(b)
        if r.returncode == 0 and os.path.exists(dst) and os.path.getsize(dst) > 0:
            out.append(dst)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--torch", action="store_true")
    ap.add_argument("globs", nargs="*")
    args = ap.parse_args()
    pats = args.globs or ["/opt/rocm/lib/hipblaslt/library/TensileLibrary*Type_BB*gfx950.co",
                          "/opt/rocm/lib/hipblaslt/library/TensileLibrary*Type_BS*gfx950.co"]
    files = sorted({f for p in pats for f in glob.glob(p)})
    tot_k = tot_pk = tot_hit = 0
    with tempfile.TemporaryDirectory() as tmp:
        if args.torch:
            files += torch_code_objects(tmp)
        for f in files:
            ks = scan_text(disasm(f, tmp), args.window)
            nk = len(ks)
            npk = sum(1 for v in ks.values() if v[1])
            hits = [(k, h) for k, v in ks.items() for h in v[2]]
            tot_k += nk
            tot_pk += npk
            tot_hit += len(hits)
            print(f"{os.path.basename(f)[:90]}: {nk} kernels, {npk} with packed FP32, {len(hits)} pk->DPP within "
                  f"{args.window}")
            for k, h in hits[:3]:
                print(f"    {k[:70]}: +{h[1]}  {h[2]}  ->  {h[3]}")
    print(f"TOTAL: {tot_k} kernels, {tot_pk} with packed FP32, {tot_hit} packed results read by DPP within "
          f"{args.window} instructions")


if __name__ == "__main__":
    sys.exit(main())
