"""Report for tools/ubench_after.py: step-kernel duration grouped by the kernel that ran before it."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
by = collections.defaultdict(list)
prev = None
for r in rows:
    name = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "d2d_step_kernel" in name and prev is not None:
        key = prev["Kernel_Name"][:40] + " grid=" + prev.get("Grid_Size", prev.get("Grid_Size_X", "?"))
        by[key].append(d)
    prev = r
for k, v in sorted(by.items()):
    v.sort()
    print(f"{k:70s} n={len(v):4d} median {v[len(v) // 2]:6.1f} min {v[0]:6.1f} max {v[-1]:6.1f}")
