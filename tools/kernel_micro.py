"""Time the per-step small kernels in isolation (HIP events, median of rounds) at the bench
shape: policy (Philox noise / injected noise / eval), assemble, step, reset, RFF features.

usage: python tools/kernel_micro.py [lanes] [S] [A]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import _native as N  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
S = int(sys.argv[2]) if len(sys.argv) > 2 else 197
A = int(sys.argv[3]) if len(sys.argv) > 3 else 36
dev = "cuda"
s_, a_, s2_ = syn.offline(4096, S, A, 0)
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
norms = get_transformations(*[torch.from_numpy(x).float() for x in (s_, a_, s2_)])
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device=dev)
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
expert = torch.from_numpy(syn.expert(4096, S, 3))
cost = amx.RBFLinearCost(expert, feature_dim=512, bw_samples=10000, lambda_b=0.0025, seed=100, ctx=ctx)
pw, ls = init_mlp_policy_params(S, A)
pol = amx.DevicePolicy(ctx, pw, ls, seed=3)
eng = amx.RolloutEngine(ens, syn.reset_table(4096, S, 1), lanes=B, policy=pol, cost=cost, max_steps=2)
eng.reset_all()
ob = eng.obs[0]
act = eng.acts[0]
noise = torch.randn(B, A, dtype=torch.float64, device=dev)
ws = ens.workspace(B)
preds = ws["preds"]
preds.normal_(std=0.01)
s = ctx.stream
mask = torch.zeros(B, dtype=torch.uint8, device=dev)
mask[::7] = 1

cases = {
    "policy(philox)": lambda: pol.act(ob, B, act, 1),
    "policy(injected)": lambda: pol.act(ob, B, act, 1, noise=noise),
    "policy(eval)": lambda: pol.act(ob, B, act, 1, eval_mode=True),
    "policy+x0(philox)": lambda: pol.act(ob, B, act, 1, x0=ws["act"]),
    "assemble": lambda: N.check(ctx.lib.amx_assemble_input(ctx.h, ob.data_ptr(), act.data_ptr(), 0,
                                                           ws["act"].data_ptr(), ws["Bp"] * ctx.ldk, ctx.ldk, B, s)),
    "step": lambda: N.check(ctx.lib.amx_step(ctx.h, preds.data_ptr(), S, preds.shape[1] * S,
                                             eng.model_idx.data_ptr(), ob.data_ptr(), eng.next_obs[0].data_ptr(),
                                             eng.num_steps.data_ptr(), eng.done[0].data_ptr(), eng.disc[0].data_ptr(),
                                             eng.cost_in.data_ptr(), ctx.k_rff_pad, None, B, s)),
    "reset(1/7)": lambda: N.check(ctx.lib.amx_reset_lanes(ctx.h, mask.data_ptr(), eng.table.data_ptr(),
                                                          eng.table.shape[0], None, 5, eng.next_obs[0].data_ptr(),
                                                          eng.obs[1].data_ptr(), eng.num_steps.data_ptr(),
                                                          eng.model_idx.data_ptr(), eng.reset_count.data_ptr(), None,
                                                          B, s)),
    "rff": lambda: cost.map.features(eng.cost_in, eng.Bp, B, eng.phi[0], eng.partials[0]),
}
res = {k: [] for k in cases}
for r in range(9):
    for k, f in cases.items():
        f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 10 * 1e3)
print(f"lanes {B} S {S} A {A}: us per call (median / min of 9 rounds x 10)")
for k, v in res.items():
    print(f"{k:18s} {np.median(v):8.2f} {np.min(v):8.2f}")
