"""Same-process A/B of the f16x3 RFF feature tiles (amx__set_h3_rff_variant) on the
rollout's scoring shape: 40 960 [s, s'] rows (S=197 -> K=416), F=512.  Checks that every
variant's phi and fp64 column partials are bit-identical to the automatic tile.
usage: python tools/rff_ab.py [rows] [variants]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 40960
VS = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "-1,1,2,3").split(",")]
S = 197
ctx = amx.AmxContext(S, 36, 4, 512, 4, 512, device="cuda")
cost = amx.RBFLinearCost(torch.from_numpy(syn.expert(4096, S, 3)), feature_dim=512, bw_samples=10000,
                         lambda_b=0.0025, seed=100, ctx=ctx)
m = cost.map
x = torch.zeros(rows, m.Kp, device="cuda")
x[:, :2 * S] = torch.randn(rows, 2 * S, device="cuda") * 0.5
phi = torch.empty(rows, 512, device="cuda")
part = torch.empty(rows // 128, 512, dtype=torch.float64, device="cuda")
lib = ctx.lib
lib.amx__set_h3_rff_variant.argtypes = [ctypes.c_int]
ref = None
for v in VS:
    lib.amx__set_h3_rff_variant(v)
    m.features(x, rows, rows, phi, part)
    torch.cuda.synchronize()
    out = (phi.clone(), part.clone())
    if ref is None:
        ref = out
    print(f"r{v}: {'bit-identical' if all(torch.equal(a, b) for a, b in zip(out, ref)) else 'DIFFERS'}")
res = {v: [] for v in VS}
for _ in range(5):
    for v in VS:
        lib.amx__set_h3_rff_variant(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            m.features(x, rows, rows, phi, part)
        e1.record()
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) * 100)
for v in VS:
    print(f"r{v}: {np.median(res[v]):7.1f} us per {rows}-row pass (incl. row exponents)")
