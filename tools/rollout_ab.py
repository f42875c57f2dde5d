"""Same-process A/B of rollout-engine options on the real rollout (bench workload),
interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/rollout_ab.py [lanes] [variants, comma-separated]
variants: "base" (defaults); "s0": one x0 copy per member (DeviceEnsemble.shared_x0 off);
"r0": separate step + reset launches (RolloutEngine.fuse_reset off); "f0"/"f1": layer-by-layer GEMM launches /
the fused ensemble forward (DeviceEnsemble.fused); "a0": separate step and policy launches (RolloutEngine.fuse_step_act
off); "w8": the fused step + action at two workgroups per CU (amx_set_step_act_occupancy); "x1": the policy launch
writes the ensemble's x0 (RolloutEngine.fuse_assembly); "t1": the f16x3 forwards time themselves (amx_set_gemm_timer,
as bench.py's timed region).
"""
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
VARIANTS = (sys.argv[2] if len(sys.argv) > 2 else "base,s0").split(",")
S, A = 197, 36
dev = torch.device("cuda", 0)
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device=dev)
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
ens.compute_threshold(torch.from_numpy(s).float().to(dev), torch.from_numpy(a).float().to(dev))
cost = amx.RBFLinearCost(torch.from_numpy(syn.expert(50000, S, 3)), feature_dim=512, bw_quantile=0.1,
                         lambda_b=0.0025, seed=100, ctx=ctx)
pw, ls = init_mlp_policy_params(S, A)
pol = amx.DevicePolicy(ctx, pw, ls, seed=1)
T = math.ceil(40000 / B)
eng = amx.RolloutEngine(ens, syn.reset_table(65536, S, 1), lanes=B, policy=pol, cost=cost, seed=7, max_steps=T)
eng.reset_all()


def setv(v):
    s = str(v)
    ens.shared_x0 = s != "s0"
    eng.fuse_reset = s != "r0"
    eng.fuse_step_act = s in ("a1", "w8")
    eng.fuse_assembly = s == "x1"
    if s == "t1":
        ctx.gemm_timer()
    else:
        ctx.gemm_timer(False)
    ctx.lib.amx_set_step_act_occupancy(ctx.h, int(s == "w8"))
    if hasattr(ens, "fused"):
        ens.fused = s == "f1" or (s != "f0" and ens.fused_default)


def rollout():
    eng.rollout(T)
    eng.relabel()
    cost.get_expert_cost()


for v in VARIANTS:
    setv(v)
    rollout()
torch.cuda.synchronize()
setv("base")
t_end = time.perf_counter() + 0.5  # clock settle (tools/mfma_ceiling.hip)
while time.perf_counter() < t_end:
    rollout()
    torch.cuda.synchronize()
res = {v: [] for v in VARIANTS}
for r in range(6):
    for v in VARIANTS:
        setv(v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            rollout()
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / 4)
setv("base")
print(f"lanes {B}: ms per {T * B}-sample rollout (median / min of 6 rounds x 4)")
for v in VARIANTS:
    print(f"variant {v:>4s}: {np.median(res[v]) * 1e3:7.3f} {np.min(res[v]) * 1e3:7.3f}  -> "
          f"{T * B / np.median(res[v]) / 1e6:.3f} M env-steps/s")
