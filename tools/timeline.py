"""Per-step kernel timeline of a rocprofv3 kernel trace (bench.py steps): each kernel's start and end
relative to the step's first kernel, and the idle gaps on the GPU between kernels.
Usage: python3 tools/timeline.py TRACE.csv [first-kernel-substring] [step index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_gray_strips"
want = int(sys.argv[3]) if len(sys.argv) > 3 else -2
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows))
starts = [i for i, k in enumerate(ks) if first in k[2]]
i0 = starts[want]
i1 = starts[want + 1] if want + 1 < len(starts) and want != -1 else len(ks)
t0 = ks[i0][0]
busy_end = t0
for s, e, name, q in ks[i0:i1]:
    gap = (s - busy_end) / 1e3
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {gap:6.1f} q{q} {name[:70]}")
    busy_end = max(busy_end, e)
print(f"step span {(busy_end - t0) / 1e3:.1f} us")
