"""Run one f16x3 ensemble layer (default: hidden layer 3, K=1792) REPS times at the bench
shape, for rocprofv3 --pmc passes (tools/h3_pmc.sh); the parser mode prints the per-dispatch
averages of the collected counters.
usage: python tools/h3_pmc.py run [layer] [reps]
       python tools/h3_pmc.py parse <pmc_dir>...
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def run(layer, reps):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import amp_extensions_amd as amx
    from amp_extensions_amd import _native as N
    from amp_extensions_amd.ensemble import init_ensemble_weights
    S, A, B = 197, 36, 8192
    norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
    c = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
    e = amx.DeviceEnsemble(c, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms, gemm="f16x3")
    ob, ac = torch.randn(B, S, device="cuda"), torch.randn(B, A, device="cuda")
    e.forward_preds(ob, ac, B)
    ws = e.workspace(B)
    Bp, buf, rexp, preds = ws["Bp"], ws["act"], ws["rexp"], ws["preds"]
    out = torch.zeros_like(buf)
    scratch = torch.empty_like(rexp)
    sA, sR = Bp * c.ldk, (c.L + 1) * Bp
    for _ in range(reps):
        if layer < c.L:
            K = c.k0_pad + layer * c.Hp
            N.check(c.lib.amx_gemm_bias_act_h3(c.h, c.M, Bp, c.Hp, K, buf.data_ptr(), c.ldk, sA,
                                               e.W2[layer].data_ptr(), c.Hp * 2 * K, e.wexp[layer].data_ptr(), c.Hp,
                                               e.b[layer].data_ptr(), c.Hp, out.data_ptr(), c.ldk, sA, K,
                                               N.AMX_ACT_RELU, rexp.data_ptr(), sR, layer + 1,
                                               scratch[0, layer + 1].data_ptr(), c.k0_pad, c.stream), "h3")
        else:
            N.check(c.lib.amx_gemm_out_unnorm_h3(c.h, c.M, Bp, c.S, c.ldk, buf.data_ptr(), c.ldk, sA,
                                                 e.W2[c.L].data_ptr(), c.n_out_pad * 2 * c.ldk,
                                                 e.wexp[c.L].data_ptr(), c.n_out_pad, e.b[c.L].data_ptr(),
                                                 c.n_out_pad, preds.data_ptr(), c.S, Bp * c.S, rexp.data_ptr(), sR,
                                                 c.L + 1, c.k0_pad, c.stream), "h3 out")
    torch.cuda.synchronize()


def parse(dirs):
    tot = defaultdict(list)
    dur = []
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            for r in csv.DictReader(open(path)):
                if "k_gemm_h3" not in r["Kernel_Name"]:
                    continue
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            for (disp, name), v in per.items():
                tot[name].append(v)
    for name in sorted(tot):
        v = tot[name][len(tot[name]) // 4:]  # drop the first quarter (clock ramp)
        print(f"{name:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 3, int(sys.argv[3]) if len(sys.argv) > 3 else 40)
    else:
        parse(sys.argv[2:])
