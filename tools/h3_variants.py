"""A/B the f16x3 GEMM tile variants per ensemble layer, interleaved in one process (GPU box).

Hidden-layer variants (amx__set_h3_variant): -1 automatic (= 21) | 0 128x128 | 1 256x256 8 waves |
2 256x256 BK32 | 3 256x256 16 waves | 4 256x128 | 5 128x256 | 6 128x128 BK32 | 7 256x128 BK32 |
8 256x256 BK32 16 waves | 9 = 2, write-after-barrier | 11 = 8, write-after-barrier |
13 = 11 on 16x16x32 | 14 = 9 on 16x16x32 | 15,16 = 14 + s_setprio | 17,18 128x256 | 19 = 14, pinned reads | 20 = 19 + early first reads | 21 = 20 + split staging |
91..95 ablations (k_gemm_h3 ABL).
Output layer (amx__set_h3_out_variant): -1 automatic (= 16 + split staging) | 9 128x224 14 waves 32x32x16 BK 32 late |
16 same on 16x16x32, pinned + early reads | 17,18 (S=226) 128x256 16x16x32 pinned + early, 32x32x16 (automatic: 17 + split) |
0 same, BK 16 | 1 BK 32 | 2,3 4 waves of 32x224 | 4 7 waves | 5-8 N padded to 256 (8 = 8 waves, late) |
10 N 256, 16 waves.
Every variant's output must be bit-identical to the automatic one (same k order per element).
usage: python tools/h3_variants.py [lanes] [hidden variants] [output variants]
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import _native as N  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
HV = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "-1,0,1,2,3,4,5,6,7").split(",")]
OV = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "-1,0").split(",")]
S, A = (int(v) for v in os.environ.get("AMX_SA", "197,36").split(","))  # AMX_SA=226,28: the scene layout
ROUNDS, REPS = 5, 10

torch.manual_seed(0)
norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
w = init_ensemble_weights(S, A, [512] * 4, 4, 100)
e = amx.DeviceEnsemble(ctx, w, norms, gemm="f16x3")
lib = ctx.lib
lib.amx__set_h3_variant.argtypes = [ctypes.c_int]
lib.amx__set_h3_out_variant.argtypes = [ctypes.c_int]
ob = torch.randn(B, S, device="cuda")
ac = torch.randn(B, A, device="cuda")
e.forward_preds(ob, ac, B)  # fills the activation rows and every row-exponent slot
ws = e.workspace(B)
Bp, buf, rexp, preds = ws["Bp"], ws["act"], ws["rexp"], ws["preds"]
out = torch.zeros_like(buf)
s = ctx.stream
c = ctx
sA, sR = Bp * c.ldk, (c.L + 1) * Bp
scratch = torch.empty_like(rexp)


def layer(i):
    if i < c.L:
        K = c.k0_pad + i * c.Hp
        N.check(lib.amx_gemm_bias_act_h3(c.h, c.M, Bp, c.Hp, K, buf.data_ptr(), c.ldk, sA, e.W2[i].data_ptr(),
                                         c.Hp * 2 * K, e.wexp[i].data_ptr(), c.Hp, e.b[i].data_ptr(), c.Hp,
                                         out.data_ptr(), c.ldk, sA, K, N.AMX_ACT_RELU, rexp.data_ptr(), sR, i + 1,
                                         scratch[0, i + 1].data_ptr(), c.k0_pad, s), "h3")
    else:
        N.check(lib.amx_gemm_out_unnorm_h3(c.h, c.M, Bp, c.S, c.ldk, buf.data_ptr(), c.ldk, sA, e.W2[c.L].data_ptr(),
                                           c.n_out_pad * 2 * c.ldk, e.wexp[c.L].data_ptr(), c.n_out_pad,
                                           e.b[c.L].data_ptr(), c.n_out_pad, preds.data_ptr(), c.S, Bp * c.S,
                                           rexp.data_ptr(), sR, c.L + 1, c.k0_pad, s), "h3 out")


def result(i):
    if i < c.L:
        K = c.k0_pad + i * c.Hp
        return out[:, :B, K:K + 512].clone()
    return preds[:, :B].clone()


def flops(i):
    if i < c.L:
        return 2.0 * 4 * B * 512 * (S + A + i * 512)
    return 2.0 * 4 * B * S * (S + A + c.L * 512)


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


ref = {}
lib.amx__set_h3_variant(-1)
lib.amx__set_h3_out_variant(-1)
for i in range(c.L + 1):
    layer(i)
    torch.cuda.synchronize()
    ref[i] = result(i)
for v in HV:
    lib.amx__set_h3_variant(v)
    bad = []
    for i in range(c.L):
        layer(i)
        torch.cuda.synchronize()
        if not torch.equal(result(i), ref[i]):
            bad.append(i)
    print(f"h{v}: hidden layers {'bit-identical' if not bad else 'DIFFER at ' + str(bad)}")
lib.amx__set_h3_variant(-1)
for ov in OV:
    lib.amx__set_h3_out_variant(ov)
    layer(c.L)
    torch.cuda.synchronize()
    print(f"o{ov}: output layer {'bit-identical' if torch.equal(result(c.L), ref[c.L]) else 'DIFFERS'}")
lib.amx__set_h3_out_variant(-1)

for _ in range(40):
    for i in range(c.L + 1):
        layer(i)
torch.cuda.synchronize()
res = {}
for r in range(ROUNDS):
    for v in HV:
        lib.amx__set_h3_variant(v)
        for i in range(c.L):
            res.setdefault((f"h{v}", i), []).append(timed(lambda: layer(i)))
    lib.amx__set_h3_variant(-1)
    for ov in OV:
        lib.amx__set_h3_out_variant(ov)
        res.setdefault((f"o{ov}", c.L), []).append(timed(lambda: layer(c.L)))
    lib.amx__set_h3_out_variant(-1)
print(f"lanes {B}: us/launch (median) and f32-equivalent TF/s (median / best)")
for i in range(c.L + 1):
    names = [f"h{v}" for v in HV] if i < c.L else [f"o{v}" for v in OV]
    line = [f"layer {i}:"]
    for n in names:
        t = np.array(res[(n, i)])
        line.append(f"{n} {np.median(t):6.1f}us {flops(i) / np.median(t) / 1e6:5.0f}/{flops(i) / t.min() / 1e6:5.0f}")
    print("  ".join(line))
tot = {f"h{v}": sum(np.median(res[(f"h{v}", i)]) for i in range(c.L)) for v in HV}
print("hidden layers total (us): " + "  ".join(f"{n} {t:.0f}" for n, t in tot.items()))
