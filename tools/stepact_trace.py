"""Rollouts with the fused step + next action (amx_step_reset_act) and with separate step /
policy / assembly launches, back to back in one process, for a rocprofv3 kernel trace
(k_step_act against k_step + k_policy + k_assemble per step).  usage: python tools/stepact_trace.py [lanes]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
S, A = 197, 36
dev = torch.device("cuda", 0)
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device=dev)
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
cost = amx.RBFLinearCost(torch.from_numpy(syn.expert(50000, S, 3)), feature_dim=512, bw_quantile=0.1,
                         lambda_b=0.0025, seed=100, ctx=ctx)
pw, ls = init_mlp_policy_params(S, A)
pol = amx.DevicePolicy(ctx, pw, ls, seed=1)
T = math.ceil(40000 / B)
eng = amx.RolloutEngine(ens, syn.reset_table(65536, S, 1), lanes=B, policy=pol, cost=cost, seed=7, max_steps=T)
eng.reset_all()
for mode in ("fused", "w8", "separate"):
    eng.fuse_step_act = mode != "separate"
    ctx.lib.amx_set_step_act_occupancy(ctx.h, int(mode == "w8"))
    for _ in range(4):
        eng.rollout(T)
        eng.relabel()
    torch.cuda.synchronize()
