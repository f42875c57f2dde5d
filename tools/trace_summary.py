"""Summarise a rocprofv3 kernel trace: per-kernel stats over the rollout region (from the
first policy launch on: excludes the one-off init work such as the ensemble threshold pass
over the offline set), plus the average duration of the ensemble-layer GEMM launches
(k_gemm_nt with the BIAS_ACT/UNNORM epilogues) to set beside bench.py's HIP-event
`roofline.avg_launch_us`.

usage: python tools/trace_summary.py <run_kernel_trace.csv> [timed_launches]
(timed_launches: the GEMM launches of bench's timed region = steps * sync_steps * (L+1),
e.g. 5 * 5 * 5 = 125 for `bench.py --steps 5`; their average is what the HIP events see)
"""
import csv
import re
import sys
from collections import defaultdict

path = sys.argv[1]
rows = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
first = next((i for i, x in enumerate(rows) if "k_policy" in x["Kernel_Name"]), 0)
rows = rows[first:]
agg = defaultdict(lambda: [0, 0.0])
gemm = []
for x in rows:
    d = (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1000
    name = x["Kernel_Name"]
    k = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
    agg[k][0] += 1
    agg[k][1] += d
    if re.search(r"k_gemm_(nt|x6|h3|lb)<[01],", name):
        gemm.append(d)
span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1000
tot = sum(v[1] for v in agg.values())
print(f"rollout region: span {span:.1f} us, kernels busy {tot:.1f} us ({100 * tot / span:.1f}%)")
if gemm:
    print(f"ensemble-layer GEMM launches: {len(gemm)}, average {sum(gemm) / len(gemm):.2f} us")
    if len(sys.argv) > 2:
        n = int(sys.argv[2])
        print(f"  last {n} (bench's timed region): average {sum(gemm[-n:]) / len(gemm[-n:]):.2f} us")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{k:60s} {n:5d} {t:10.1f} us {t / n:9.2f} us/call {100 * t / tot:5.1f}%")
