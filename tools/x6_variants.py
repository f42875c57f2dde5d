"""A/B the bf16x6 GEMM tile variants on the ensemble's layer shapes, interleaved in one
process.  Prints per-layer f32-equivalent TFLOP/s (algorithmic, unpadded K/N): median and
best over rounds, and each variant's max |diff| against the f32 MFMA path (correctness).

Hidden-layer variants (amx__set_x6_variant): 0 128x128 BK16 | 1 + two K-tiles in registers |
2 BK32 single LDS buffer | 3 BK32 double buffer (1 WG/CU) | 4 128x256 8 waves | 5 256x128 8
waves | 6 128x256 4 waves of 64x128 | 7 = 0 on pre-split activations | 8 = 4 on pre-split.  Output layer (amx__set_x6_out_variant): o0 128x224 |
oK hidden variant K-1 on N padded to 256.

usage: python tools/x6_variants.py [lanes] [hidden variants] [output variants]
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
HV = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,1,4,7,8").split(",")]
OV = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,1,5,8").split(",")]
S, A = 197, 36
ROUNDS, REPS = 5, 5

torch.manual_seed(0)
norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
w = init_ensemble_weights(S, A, [512] * 4, 4, 100)
e6 = amx.DeviceEnsemble(ctx, w, norms, gemm="bf16x6")
e32 = amx.DeviceEnsemble(ctx, w, norms, gemm="f32")
lib = ctx.lib
lib.amx__set_x6_variant.argtypes = [ctypes.c_int]
lib.amx__set_x6_out_variant.argtypes = [ctypes.c_int]
ws = e6.workspace(B)
Bp, buf = ws["Bp"], ws["act"]
buf.normal_()
buf.abs_()
out = torch.zeros_like(buf)
# pre-split activation image for the ALIMB variants (7, 8)
a3 = torch.empty(4, Bp, 3 * ctx.ldk, dtype=torch.int16, device="cuda")
N.check(lib.amx_split_bf16x3(ctx.h, 4, Bp, ctx.ldk, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk, a3.data_ptr(),
                             Bp * 3 * ctx.ldk, ctx.stream))
lib.amx__set_x6_a3.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
lib.amx__set_x6_a3(a3.data_ptr(), Bp * 3 * ctx.ldk)
preds = torch.zeros(4, Bp, S, device="cuda")
s = ctx.stream
k0 = ctx.k0_pad


def layer(i, x6=True):
    if i < ctx.L:
        K = k0 + i * ctx.Hp
        if x6:
            N.check(lib.amx_gemm_bias_act_x6(ctx.h, 4, Bp, 512, K, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk,
                                             e6.W3[i].data_ptr(), 512 * 3 * K, e6.b[i].data_ptr(), 512,
                                             out.data_ptr(), ctx.ldk, Bp * ctx.ldk, K, 1, s))
        else:
            N.check(lib.amx_gemm_bias_act(ctx.h, 4, Bp, 512, K, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk,
                                          e32.W[i].data_ptr(), K, 512 * K, e32.b[i].data_ptr(), 512, out.data_ptr(),
                                          ctx.ldk, Bp * ctx.ldk, K, 1, s))
    else:
        if x6:
            N.check(lib.amx_gemm_out_unnorm_x6(ctx.h, 4, Bp, S, ctx.ldk, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk,
                                               e6.W3[i].data_ptr(), ctx.n_out_pad * 3 * ctx.ldk, e6.b[i].data_ptr(),
                                               ctx.n_out_pad, preds.data_ptr(), S, Bp * S, s))
        else:
            N.check(lib.amx_gemm_out_unnorm(ctx.h, 4, Bp, S, ctx.ldk, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk,
                                            e32.W[i].data_ptr(), ctx.ldk, ctx.n_out_pad * ctx.ldk,
                                            e32.b[i].data_ptr(), ctx.n_out_pad, preds.data_ptr(), S, Bp * S, s))


def result(i):
    if i < ctx.L:
        K = k0 + i * ctx.Hp
        return out[:, :B, K:K + 512].clone()
    return preds[:, :B].clone()


def flops(i):
    if i < ctx.L:
        return 2.0 * 4 * B * 512 * (S + A + i * 512)
    return 2.0 * 4 * B * S * (S + A + ctx.L * 512)


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


configs = [("f32", None)] + [(f"h{v}", v) for v in HV]
ref = {}
for i in range(ctx.L + 1):
    layer(i, x6=False)
    torch.cuda.synchronize()
    ref[i] = result(i)
# correctness of every variant
for name, v in configs[1:]:
    lib.amx__set_x6_variant(v)
    errs = []
    for i in range(ctx.L):
        layer(i)
        torch.cuda.synchronize()
        errs.append(((result(i) - ref[i]).abs().max() / ref[i].abs().max()).item())
    print(f"{name}: hidden-layer max rel diff vs f32 {max(errs):.2e}")
lib.amx__set_x6_variant(-1)
for ov in OV:
    lib.amx__set_x6_out_variant(ov)
    layer(ctx.L)
    torch.cuda.synchronize()
    print(f"o{ov}: output-layer max rel diff vs f32 "
          f"{((result(ctx.L) - ref[ctx.L]).abs().max() / ref[ctx.L].abs().max()).item():.2e}")
lib.amx__set_x6_out_variant(-1)

# warm the clock
for _ in range(40):
    for i in range(ctx.L + 1):
        layer(i)
torch.cuda.synchronize()
res = {}
for r in range(ROUNDS):
    for name, v in configs:
        if v is not None:
            lib.amx__set_x6_variant(v)
        for i in range(ctx.L):
            res.setdefault((name, i), []).append(timed(lambda: layer(i, x6=v is not None)))
    for ov in OV:
        lib.amx__set_x6_out_variant(ov)
        res.setdefault((f"o{ov}", ctx.L), []).append(timed(lambda: layer(ctx.L)))
    lib.amx__set_x6_out_variant(-1)
    res.setdefault(("f32", ctx.L), []).append(timed(lambda: layer(ctx.L, x6=False)))
lib.amx__set_x6_variant(-1)
print(f"lanes {B}: us/launch (median) and f32-equivalent TF/s (median / best)")
for i in range(ctx.L + 1):
    names = [n for n, _ in configs] if i < ctx.L else ["f32"] + [f"o{v}" for v in OV]
    line = [f"layer {i}:"]
    for n in names:
        t = np.array(res[(n, i)])
        line.append(f"{n} {np.median(t):6.1f}us {flops(i) / np.median(t) / 1e6:5.0f}/{flops(i) / t.min() / 1e6:5.0f}")
    print("  ".join(line))
tot = {}
for n, _ in configs:
    tot[n] = sum(np.median(res[(n, i)]) for i in range(ctx.L))
print("hidden layers total (us): " + "  ".join(f"{n} {t:.0f}" for n, t in tot.items()))
