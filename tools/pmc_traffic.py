"""HBM traffic of the ensemble GEMM from rocprofv3 PMC passes -> amp_extensions_amd/data/gemm_traffic_<gemm>.json
(bench.py reads it there; keyed to the GEMM sources' hash).

Two separate counter passes over the same bench command (MI355X_MICROARCH.md, HBM section:
one counter per pass, FETCH_SIZE counts half of the wide coalesced loads on gfx950 -> x2):

  cd /tmp && export TMPDIR=/tmp
  rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc_fetch -o run --output-format csv -- \
      python $R/bench.py --no-cpu-baseline --steps 3 --warmup 1
  rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmc_write -o run --output-format csv -- \
      python $R/bench.py --no-cpu-baseline --steps 3 --warmup 1
  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write [lanes] [S] [A] [f16x3|bf16x6|f32] \
      > profiles/gemm_traffic_<gemm>.json

The last L+1 ensemble-layer dispatches (k_gemm_h3 / k_gemm_x6 / k_gemm_nt with the BIAS_ACT / UNNORM epilogues, i.e.
the final step's forward) are taken; bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch,
against the algorithmic bytes (activation panel read + weights + output write).
"""
import csv
import glob
import json
import os
import re
import sys


def per_dispatch(d, counter, kernel):
    path = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(kernel + r"<(\d)", r["Kernel_Name"])
        if not m or m.group(1) == "2":  # skip the RFF (EPI 2) GEMM
            continue
        k = int(r["Dispatch_Id"])
        out[k] = out.get(k, 0.0) + float(r["Counter_Value"])
    return [out[k] for k in sorted(out)]


def main():
    fetch_dir, write_dir = sys.argv[1], sys.argv[2]
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
    S = int(sys.argv[4]) if len(sys.argv) > 4 else 197
    A = int(sys.argv[5]) if len(sys.argv) > 5 else 36
    M, H, L = 4, 512, 4
    k0 = (S + A + 31) // 32 * 32
    n_out_pad = (S + 127) // 128 * 128
    rows = M * B
    gemm = sys.argv[6] if len(sys.argv) > 6 else "f16x3"
    kernel = {"f16x3": "k_gemm_h3", "bf16x6": "k_gemm_x6", "f32": "k_gemm_nt"}[gemm]
    # weight bytes per element as the kernel reads them (3 bf16 limbs / 2 fp16 limbs / fp32)
    wb = 6 if gemm == "bf16x6" else 4
    f = per_dispatch(fetch_dir, "FETCH_SIZE", kernel)[-(L + 1):]
    w = per_dispatch(write_dir, "WRITE_SIZE", kernel)[-(L + 1):]
    layers, tot_hbm, tot_alg = [], 0, 0
    # f16x3: the x0 slice is assembled once and read for all M members (k_shared), so its
    # compulsory bytes are B*k0*4, not M*B*k0*4
    a_bytes = (lambda K: (rows * (K - k0) + B * k0) * 4) if gemm == "f16x3" else (lambda K: rows * K * 4)
    for i in range(L + 1):
        K = k0 + i * H
        if i < L:
            alg = a_bytes(K) + M * H * K * wb + rows * H * 4
        else:
            alg = a_bytes(K) + M * n_out_pad * K * wb + rows * S * 4
        hbm = int((2 * f[i] + w[i]) * 1024)
        layers.append({"layer": i, "K": K, "fetch_kb": f[i], "write_kb": w[i], "hbm_bytes": hbm, "alg_bytes": alg})
        tot_hbm += hbm
        tot_alg += alg
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import gemm_source_sha16
    print(json.dumps({
        "kernel": f"{kernel} (ensemble layers)", "gemm": gemm, "gemm_source_sha16": gemm_source_sha16(), "state_dim": S, "action_dim": A, "lanes": B,
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py --steps 3, last step",
        "method": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch (gfx950: FETCH_SIZE counts 1/2 of "
                  "wide coalesced loads, MI355X_MICROARCH.md HBM section); L2<->fabric traffic (Infinity-Cache "
                  "hits included)",
        "hbm_bytes_per_launch": tot_hbm // (L + 1), "alg_bytes_per_launch": tot_alg // (L + 1),
        "ratio": round(tot_hbm / tot_alg, 3), "layers": layers}, indent=1))


if __name__ == "__main__":
    main()
