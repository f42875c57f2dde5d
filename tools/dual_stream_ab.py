"""Prototype A/B: the 40 960-sample rollout as ONE engine of 8192 lanes on one stream, against
TWO engines of 4096 lanes (separate contexts, workspaces, policies, costs) whose steps are
issued alternately on two HIP streams, so one lane group's small kernels and GEMM tails can
overlap the other group's GEMMs.  Wall time per rollout (steps + scoring + relabel), medians of
interleaved rounds.  usage: python tools/dual_stream_ab.py [T]"""
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

T = int(sys.argv[1]) if len(sys.argv) > 1 else 5
S, A = 197, 36
dev = torch.device("cuda", 0)
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
wts = init_ensemble_weights(S, A, [512] * 4, 4, 100)
expert = torch.from_numpy(syn.expert(50000, S, 3))
pw, ls = init_mlp_policy_params(S, A)
table = syn.reset_table(65536, S, 1)


def engine(B, seed):
    ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device=dev)
    ens = amx.DeviceEnsemble(ctx, wts, norms)
    ens.compute_threshold(torch.from_numpy(s[:8192]).float().to(dev), torch.from_numpy(a[:8192]).float().to(dev))
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100, ctx=ctx)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=seed)
    eng = amx.RolloutEngine(ens, table, lanes=B, policy=pol, cost=cost, seed=seed + 7, max_steps=T)
    eng.reset_all()
    return eng, cost


one, c1 = engine(8192, 1)
halves = [engine(4096, 11), engine(4096, 21)]
streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def single():
    one.rollout(T)
    one.relabel()
    c1.get_expert_cost()


def dual():
    main = torch.cuda.current_stream(dev)
    for st in streams:
        st.wait_stream(main)
    for (e, _), st in zip(halves, streams):
        with torch.cuda.stream(st):
            e._rollout_begin()
    for t in range(T):
        for (e, _), st in zip(halves, streams):
            with torch.cuda.stream(st):
                e.step()
    for (e, c), st in zip(halves, streams):
        with torch.cuda.stream(st):
            e.score()
            e.relabel()
            c.get_expert_cost()
    for st in streams:
        main.wait_stream(st)


for f in (single, dual):
    for _ in range(3):
        f()
torch.cuda.synchronize()
res = {"single": [], "dual": []}
for r in range(6):
    for name, f in (("single", single), ("dual", dual)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            f()
        torch.cuda.synchronize()
        res[name].append((time.perf_counter() - t0) / 4)
for name in res:
    m = np.median(res[name])
    print(f"{name:>6s}: {m * 1e3:.3f} ms per {T * 8192}-sample rollout -> {T * 8192 / m / 1e6:.2f} M env-steps/s "
          f"(min {np.min(res[name]) * 1e3:.3f})", flush=True)
