"""Per-update kernel breakdown from a rocprofv3 kernel trace of
tools/agent_profile.py ... update: the last N updates (split at the first
kernel of each graph replay: the PER sample gather) -> kernels per update,
busy time per update (union of kernel intervals), top kernels.
Usage: python tools/update_trace.py gpurun_out/upd/run_kernel_trace.csv [first_kernel_substring] [N]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "per32_sample"
    nlast = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    if len(starts) < nlast + 1:
        print("not enough updates found:", len(starts))
        return
    segs = [(starts[j], starts[j + 1]) for j in range(len(starts) - nlast - 1, len(starts) - 1)]
    per = collections.defaultdict(float)
    cnt = collections.Counter()
    spans, busys, nk = [], [], []
    for a, b in segs:
        ks = rows[a:b]
        t0, t1 = int(ks[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in ks)
        spans.append((t1 - t0) / 1e3)
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        busys.append(busy / 1e3)
        nk.append(len(ks))
        for r in ks:
            per[r["Kernel_Name"]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[r["Kernel_Name"]] += 1
    n = len(segs)
    print(f"{n} updates: kernels/update {sum(nk) / n:.1f}, span {sum(spans) / n:.1f} us, busy {sum(busys) / n:.1f} us")
    tot = sum(per.values())
    for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:40]:
        print(f"{v / n:8.1f} us {100 * v / tot:5.1f}% x{cnt[k] / n:5.1f}  {k[:110]}")


if __name__ == "__main__":
    main()
