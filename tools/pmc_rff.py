"""HBM traffic of the RFF pass (k_gemm_h3 with the EPI_RFF epilogue, EPI 2) from two rocprofv3
PMC passes over tools/rff_ab.py: bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch (the
gfx950 correction of MI355X_MICROARCH.md's HBM section), against the algorithmic bytes: the
[s, s'] rows read once (rows x K fp32), the split weights (F x K x 2 fp16), the phi rows written
(rows x F fp32) and the fp64 column partials.
usage: python tools/pmc_rff.py <fetch_dir> <write_dir> [rows] [K] [F]"""
import csv
import glob
import os
import re
import sys


def per_dispatch(d, counter):
    path = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not re.search(r"k_gemm_h3<2", r["Kernel_Name"]):
            continue
        k = int(r["Dispatch_Id"])
        out[k] = out.get(k, 0.0) + float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    rows = int(sys.argv[3]) if len(sys.argv) > 3 else 40960
    K = int(sys.argv[4]) if len(sys.argv) > 4 else 416
    F = int(sys.argv[5]) if len(sys.argv) > 5 else 512
    f = per_dispatch(sys.argv[1], "FETCH_SIZE")
    w = per_dispatch(sys.argv[2], "WRITE_SIZE")
    n = min(len(f), len(w))
    f, w = sorted(f[-n:]), sorted(w[-n:])
    fm, wm = f[n // 2], w[n // 2]
    alg = rows * K * 4 + F * K * 4 + rows * F * 4 + (rows // 32) * F * 8
    hbm = (2 * fm + wm) * 1024
    print(f"RFF pass {rows} rows K {K} F {F}: {n} dispatches; median FETCH_SIZE {fm:.0f} KB (x2 = "
          f"{2 * fm / 1024:.1f} MB), WRITE_SIZE {wm:.0f} KB ({wm / 1024:.1f} MB); HBM {hbm / 1e6:.1f} MB per launch "
          f"vs algorithmic {alg / 1e6:.1f} MB (ratio {hbm / alg:.3f}); A panel {rows * K * 4 / 1e6:.1f} MB, "
          f"phi {rows * F * 4 / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
