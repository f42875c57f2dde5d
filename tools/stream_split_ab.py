"""Experiment: does splitting the lanes into two halves on two HIP streams (so one half's
small kernels overlap the other half's GEMMs) beat one engine over all lanes?

usage: python tools/stream_split_ab.py [lanes]
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
S, A = 197, 36
dev = torch.device("cuda", 0)
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device=dev)
w = init_ensemble_weights(S, A, [512] * 4, 4, 100)
expert = torch.from_numpy(syn.expert(50000, S, 3))
pw, ls = init_mlp_policy_params(S, A)
table = syn.reset_table(65536, S, 1)
T = math.ceil(40000 / B)


def make(lanes, seed):
    ens = amx.DeviceEnsemble(ctx, w, norms)
    ens.threshold = 0.065
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100, ctx=ctx)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=seed)
    eng = amx.RolloutEngine(ens, table, lanes=lanes, policy=pol, cost=cost, seed=seed, max_steps=T)
    eng.reset_all()
    return eng, cost


one, cost1 = make(B, 1)
ha, costa = make(B // 2, 2)
hb, costb = make(B // 2, 3)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def run_one():
    one.rollout(T)
    one.relabel()
    cost1.get_expert_cost()


def run_split():
    cur = torch.cuda.current_stream(dev)
    ha.begin_rollout()
    hb.begin_rollout()
    sa.wait_stream(cur)
    sb.wait_stream(cur)
    for _ in range(T):
        with torch.cuda.stream(sa):
            ha.step()
        with torch.cuda.stream(sb):
            hb.step()
    with torch.cuda.stream(sa):
        ha.score()
        ha.relabel()
        costa.get_expert_cost()
    with torch.cuda.stream(sb):
        hb.score()
        hb.relabel()
    cur.wait_stream(sa)
    cur.wait_stream(sb)


for f in (run_one, run_split):
    f()
torch.cuda.synchronize()
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    run_one()
    torch.cuda.synchronize()
res = {"one": [], "split": []}
for r in range(6):
    for name, f in (("one", run_one), ("split", run_split)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            f()
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / 4)
print(f"lanes {B} x {T} steps: ms per rollout (median / min of 6 x 4)")
for k, v in res.items():
    print(f"{k:6s} {np.median(v) * 1e3:7.3f} {np.min(v) * 1e3:7.3f}  -> {T * B / np.median(v) / 1e6:.3f} M env-steps/s")
