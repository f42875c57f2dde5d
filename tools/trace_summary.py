"""Summarise a rocprofv3 kernel trace: per-kernel stats over the last timed rollouts."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
n_last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if n_last:
    rows = rows[-n_last:]
agg = defaultdict(lambda: [0, 0.0])
for x in rows:
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000
    k = x["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    k = k.split("(")[0][:60]
    agg[k][0] += 1
    agg[k][1] += d
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1000
tot = sum(v[1] for v in agg.values())
print(f"span {span:.1f} us, busy {tot:.1f} us ({100 * tot / span:.1f}%)")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:60s} {n:5d} {t:10.1f} us {t / n:9.2f} us/call {100 * t / tot:5.1f}%")
