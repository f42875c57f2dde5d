"""f16x3 vs bf16x6 vs f32 MFMA ensemble forward: error against fp64 and time (GPU box).

For the bench's ensemble (4 x dense [512]x4, S=197, A=36): preds of each GEMM path vs an
fp64 forward (relative to max(1, |ref|)), on (a) the bench's synthetic states and (b) the
same rows with 1/8 of them scaled by 1e4 and 1/8 by 1e-4 (row-exponent coverage), plus the
mean time of a whole 5-launch forward (HIP events, 50 reps after warmup).
usage: python tools/h3_accuracy.py [lanes]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.synthetic import offline  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
S, A = 197, 36
dev = torch.device("cuda:0")
s, a, s2 = offline(max(B, 20000), S, A, seed=0)
norms = get_transformations(torch.from_numpy(s).float(), torch.from_numpy(a).float(), torch.from_numpy(s2).float())
w = init_ensemble_weights(S, A, [512] * 4, 4, 100)
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=dev)
ens = {g: amx.DeviceEnsemble(ctx, w, norms, gemm=g) for g in ("f32", "bf16x6", "f16x3")}
mu_s, sd_s, mu_a, sd_a, mu_d, sd_d = [torch.as_tensor(x).double().to(dev) for x in norms]


def ref_forward(ob, ac):
    # fp64 BasicMLP dense-connect + normalisation (dynamics.py:216-233, 422-433)
    x = torch.cat([(ob.float().double() - mu_s) / sd_s, (ac.float().double() - mu_a) / sd_a], 1)
    out = []
    for m in range(4):
        h = x
        for i, (W, b) in enumerate(w[m]):
            y = h @ W.double().to(dev).T + b.double().to(dev)
            if i < len(w[m]) - 1:
                h = torch.cat([h, torch.relu(y)], 1)
        out.append(y * sd_d + mu_d)
    return torch.stack(out)


for case in ("bench states", "rows x1e4 / x1e-4"):
    ob = torch.from_numpy(s[:B]).to(dev)
    ac = torch.from_numpy(a[:B]).to(dev)
    if case != "bench states":
        ob = ob.clone()
        ac = ac.clone()
        k = B // 8
        ob[:k] *= 1e4
        ac[:k] *= 1e4
        ob[k:2 * k] = mu_s.to(ob.dtype) + (ob[k:2 * k] - mu_s.to(ob.dtype)) * 1e-4
        ac[k:2 * k] = mu_a.to(ac.dtype) + (ac[k:2 * k] - mu_a.to(ac.dtype)) * 1e-4
    ref = ref_forward(ob, ac)
    scale = torch.clamp(ref.abs(), min=1.0)
    for g, e in ens.items():
        p = e.forward_preds(ob, ac, B)[:, :B].double()
        err = (p - ref).abs() / scale
        print(f"[{case}] forward {g:7s}: max rel err {err.max().item():.3e}  mean {err.mean().item():.3e}")

ob = torch.from_numpy(s[:B]).to(dev)
ac = torch.from_numpy(a[:B]).to(dev)
flops = ens["f32"].mlp_flops_per_sample() * B
for rnd in range(2):
    for g, e in ens.items():
        for _ in range(10):
            e.forward_preds(ob, ac, B)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            e.forward_preds(ob, ac, B)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        if rnd:
            print(f"forward {g:7s}: {us:8.1f} us ({flops / us / 1e6:6.1f} TF/s f32-equivalent incl. assembly)")
