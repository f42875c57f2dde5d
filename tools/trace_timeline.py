"""Print the kernel timeline of one rollout from a rocprofv3 kernel trace: offset, gap to the
previous kernel's end and duration (us) of every kernel between two consecutive policy launches.
usage: python tools/trace_timeline.py <run_kernel_trace.csv> [which=-2]  (which: the n-th policy
launch from the end that starts the rollout; a rollout of T steps spans T policy launches)
      python tools/trace_timeline.py <csv> -2 5   (5 steps per rollout)"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
T = int(sys.argv[3]) if len(sys.argv) > 3 else 1
idx = [i for i, x in enumerate(rows) if "k_policy" in x["Kernel_Name"]]
i0, i1 = idx[which - T + 1], idx[which + 1] if which + 1 < 0 else len(rows) - 1
t0 = prev = int(rows[i0]["Start_Timestamp"])
busy = 0.0
for x in rows[i0:i1]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    n = x["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:64]
    print(f"{(s - t0) / 1000:8.1f} gap {(s - prev) / 1000:5.1f} dur {(e - s) / 1000:7.1f} {n}")
    busy += (e - s) / 1000
    prev = e
print(f"rollout span {(prev - t0) / 1000:.1f} us, kernels {busy:.1f} us")
