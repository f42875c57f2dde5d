"""Counter passes over whole f16x3 forwards, the one-launch form (amx_forward_h3) against the
per-layer launches, at one lane count (tools/fwd_pmc.sh).  Counters are summed per forward (one
k_forward_h3 dispatch, or the five k_gemm_h3 dispatches of one forward).
usage: python tools/fwd_pmc.py run <fused|layers> [lanes] [reps]
       python tools/fwd_pmc.py parse <pmc_dir>..."""
import csv
import glob
import os
import sys
from collections import defaultdict


def run(mode, B, reps):
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import amp_extensions_amd as amx
    from amp_extensions_amd.ensemble import init_ensemble_weights
    S, A = 197, 36
    norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
    c = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
    e = amx.DeviceEnsemble(c, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms, gemm="f16x3")
    e.forward_mode = mode
    rs = np.random.RandomState(0)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
    ac = torch.from_numpy(rs.randn(B, A)).cuda()
    for _ in range(reps):
        e.forward_preds(ob, ac, B)
    torch.cuda.synchronize()


def parse(dirs):
    for d in dirs:
        per = defaultdict(float)
        names = set()
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                k = r["Kernel_Name"]
                if "k_gemm_h3" not in k and "k_forward_h3" not in k:
                    continue
                names.add(k.split("(")[0][:40])
                per[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        disp = sorted({k[0] for k in per})
        fused = any("k_forward_h3" in n for n in names)
        per_fwd = 1 if fused else 5
        disp = disp[len(disp) // 4 // per_fwd * per_fwd:]  # drop the first quarter (clock ramp)
        nf = max(len(disp) // per_fwd, 1)
        tot = defaultdict(float)
        for (di, name), v in per.items():
            if di in disp:
                tot[name] += v
        print(f"{d}: {'fused' if fused else 'layers'}, {nf} forwards")
        for name in sorted(tot):
            print(f"  {name:34s} {tot[name] / nf:18.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 5120, int(sys.argv[4]) if len(sys.argv) > 4 else 20)
    else:
        parse(sys.argv[2:])
