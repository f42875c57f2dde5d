"""sample_points (40 000 samples, W = 4, 16-step chunks) + relabel_paths with the chunks replayed
as HIP graphs (graph=True, the default) vs launched eagerly (graph=False), interleaved, same
process: ms per call (median of 5 after a warm call of each) and whether the paths agree.
usage: python tools/paths_graph_ab.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402
from amp_extensions_amd.relabel import relabel_paths  # noqa: E402

S, A = 197, 36
dev = torch.device("cuda", 0)
s, a, s2 = syn.offline(100000, S, A, 0)
norms = get_transformations(*(torch.from_numpy(x).float() for x in (s, a, s2)))
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=dev)
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, base_seed=100), norms)
ens.compute_threshold(torch.from_numpy(s).float().to(dev), torch.from_numpy(a).float().to(dev))
cost = amx.RBFLinearCost(torch.from_numpy(syn.expert(50000, S, 3)), feature_dim=512, bw_quantile=0.1,
                         lambda_b=0.0025, seed=100, ctx=ctx)
pw, ls = init_mlp_policy_params(S, A)
pol = amx.DevicePolicy(ctx, pw, ls, seed=1000)
eng = amx.RolloutEngine(ens, syn.reset_table(65536, S, 1), lanes=8192, policy=pol, cost=cost, seed=7, max_steps=5)


def once(i, graph):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    paths = amx.sample_points(eng, pol, num_to_collect=40000, base_seed=i, num_workers=4, chunk=16, graph=graph)
    relabel_paths(paths, cost, ens)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, paths


times = {True: [], False: []}
for g in (True, False):
    once(0, g)
for i in range(1, 6):
    for g in (True, False):
        ms, paths = once(i, g)
        times[g].append(ms)
        if g:
            ref = paths
        else:
            same = len(ref) == len(paths) and all(np.array_equal(x["observations"], y["observations"]) and
                                                  np.array_equal(x["actions"], y["actions"]) for x, y in zip(ref, paths))
            print(f"call {i}: graph {times[True][-1]:.1f} ms, eager {ms:.1f} ms, paths identical {same}")
n = sum(len(p["rewards"]) for p in ref)
for g in (True, False):
    med = float(np.median(times[g]))
    print(f"{'graph' if g else 'eager'}: median {med:.1f} ms per sample_points + relabel_paths, {n / med * 1e3:.0f} env-steps/s")
