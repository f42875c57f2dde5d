"""bf16x6 vs f32 MFMA GEMM: error against fp64 and time per ensemble layer (GPU box).

For the bench's ensemble (4 x dense [512]x4, S=197, A=36, 8192 lanes):
  * per layer: C = A W^T with the same A (the f32 forward's activation buffer) through both
    kernels; error = |C - C64| / (|A| |W|^T) (the fp32 dot-product error scale), max + mean;
  * whole forward: preds of both paths vs an fp64 forward, relative to max(1, |ref|);
  * time per layer launch (HIP events, 20 reps, after warmup).
usage: python tools/x6_accuracy.py [lanes]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import _native as N  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.synthetic import offline  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
S, A = 197, 36
dev = torch.device("cuda:0")
s, a, s2 = offline(20000, S, A, seed=0)
norms = get_transformations(torch.from_numpy(s).float(), torch.from_numpy(a).float(), torch.from_numpy(s2).float())
w = init_ensemble_weights(S, A, [512] * 4, 4, 100)
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=dev)
e32 = amx.DeviceEnsemble(ctx, w, norms, gemm="f32")
ex6 = amx.DeviceEnsemble(ctx, w, norms, gemm="bf16x6")
ob = torch.from_numpy(s[:B]).to(dev)
ac = torch.from_numpy(a[:B]).to(dev)
p32 = e32.forward_preds(ob, ac, B).clone()
buf = e32.workspace(B)["act"].clone()  # f32 activations of every layer
p6 = ex6.forward_preds(ob, ac, B).clone()

# fp64 forward (BasicMLP dense-connect + normalisation, dynamics.py:216-233, 422-433)
mu_s, sd_s, mu_a, sd_a, mu_d, sd_d = [torch.as_tensor(x).double().to(dev) for x in norms]
x = torch.cat([(ob.float().double() - mu_s) / sd_s, (ac.float().double() - mu_a) / sd_a], 1)
ref = []
for m in range(4):
    h = x
    for i, (W, b) in enumerate(w[m]):
        y = h @ W.double().to(dev).T + b.double().to(dev)
        if i < len(w[m]) - 1:
            h = torch.cat([h, torch.relu(y)], 1)
    ref.append(y * sd_d + mu_d)
ref = torch.stack(ref)
scale = torch.clamp(ref.abs(), min=1.0)
for name, p in (("f32", p32), ("bf16x6", p6)):
    e = ((p[:, :B].double() - ref).abs() / scale)
    print(f"forward {name:7s}: max rel err {e.max().item():.3e}  mean {e.mean().item():.3e}")
e = ((p6[:, :B].double() - p32[:, :B].double()).abs() / scale)
print(f"forward bf16x6 vs f32: max {e.max().item():.3e}")

# per-layer GEMM error + timing on the same A
c = ctx
Bp = round(B / 128 + 0.4999) * 128
sA = Bp * c.ldk
out32 = torch.empty_like(buf)
out6 = torch.empty_like(buf)
print(f"{'layer':>5} {'K':>5} {'f32 max':>10} {'f32 mean':>10} {'x6 max':>10} {'x6 mean':>10} {'f32 us':>8} {'x6 us':>8} {'TF f32':>7} {'TF x6':>7}")
for i in range(c.L + 1):
    last = i == c.L
    K = c.ldk if last else c.k0_pad + i * c.Hp
    Nn = c.n_out_pad if last else c.Hp
    Wt = e32.W[i]

    def run32():
        if last:
            N.check(c.lib.amx_gemm_out_unnorm(c.h, 4, Bp, c.S, K, buf.data_ptr(), c.ldk, sA, Wt.data_ptr(), K, Nn * K,
                                              e32.b[i].data_ptr(), Nn, out32.data_ptr(), c.S, Bp * c.S, c.stream), "")
        else:
            N.check(c.lib.amx_gemm_bias_act(c.h, 4, Bp, Nn, K, buf.data_ptr(), c.ldk, sA, Wt.data_ptr(), K, Nn * K,
                                            e32.b[i].data_ptr(), Nn, out32.data_ptr(), c.ldk, sA, 0, N.AMX_ACT_NONE,
                                            c.stream), "")

    def run6():
        if last:
            N.check(c.lib.amx_gemm_out_unnorm_x6(c.h, 4, Bp, c.S, K, buf.data_ptr(), c.ldk, sA, ex6.W3[i].data_ptr(),
                                                 Nn * 3 * K, ex6.b[i].data_ptr(), Nn, out6.data_ptr(), c.S, Bp * c.S,
                                                 c.stream), "")
        else:
            N.check(c.lib.amx_gemm_bias_act_x6(c.h, 4, Bp, Nn, K, buf.data_ptr(), c.ldk, sA, ex6.W3[i].data_ptr(),
                                               Nn * 3 * K, ex6.b[i].data_ptr(), Nn, out6.data_ptr(), c.ldk, sA, 0,
                                               N.AMX_ACT_NONE, c.stream), "")

    run32()
    run6()
    torch.cuda.synchronize()
    Af = buf[:, :B, :K].double()
    C64 = torch.einsum("mbk,mnk->mbn", Af, Wt.double()) + e32.b[i].double()[:, None, :]
    den = torch.einsum("mbk,mnk->mbn", Af.abs(), Wt.double().abs()) + 1e-30
    if last:
        C64 = C64[:, :, :c.S] * sd_d + mu_d
        den = den[:, :, :c.S] * sd_d.abs()
        g32 = out32.view(-1)[:4 * Bp * c.S].view(4, Bp, c.S)[:, :B].double()
        g6 = out6.view(-1)[:4 * Bp * c.S].view(4, Bp, c.S)[:, :B].double()
    else:
        g32 = out32[:, :B, :Nn].double()
        g6 = out6[:, :B, :Nn].double()
    r32 = (g32 - C64).abs() / den
    r6 = (g6 - C64).abs() / den
    times = {}
    for name, fn in (("f32", run32), ("x6", run6)):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[name] = e0.elapsed_time(e1) * 1e3 / 20
    real_n = c.S if last else 512
    real_k = (S + A + c.L * 512) if last else (S + A + i * 512)
    fl = 2.0 * 4 * B * real_n * real_k
    print(f"{i:5d} {K:5d} {r32.max().item():10.2e} {r32.mean().item():10.2e} {r6.max().item():10.2e} "
          f"{r6.mean().item():10.2e} {times['f32']:8.1f} {times['x6']:8.1f} {fl / times['f32'] / 1e6:7.1f} "
          f"{fl / times['x6'] / 1e6:7.1f}")
