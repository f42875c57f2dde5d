"""Kernel timeline of one NPG update from a rocprofv3 kernel trace of tools/npg_time.py: every
kernel from the update's VPG pass (k_npg<0, ...>) up to (not including) the next update's, with
offset, gap and duration (us); then per-kernel totals of that update.
usage: python tools/npg_timeline.py <run_kernel_trace.csv> [which=-3]  (the which-th VPG launch)"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -3
idx = [i for i, x in enumerate(rows) if "k_npg<0," in x["Kernel_Name"]]
i0 = idx[which]
i1 = idx[which + 1] if which + 1 < 0 else len(rows)
t0 = prev = int(rows[i0]["Start_Timestamp"])
tot = defaultdict(lambda: [0, 0.0])
for x in rows[i0:i1]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    n = x["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:64]
    print(f"{(s - t0) / 1000:8.1f} gap {(s - prev) / 1000:5.1f} dur {(e - s) / 1000:7.1f} {n}")
    tot[n][0] += 1
    tot[n][1] += (e - s) / 1000
    prev = e
print(f"update span {(prev - t0) / 1000:.1f} us")
for n, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print(f"{n:64s} {c:4d} {d:9.1f} us {d / c:8.2f} us/call")
