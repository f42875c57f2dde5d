"""Check of the in-kernel GEMM timer in paths mode: one warm sample_points + relabel_paths with the
timer registered before the chunk graphs are captured, then one timed call; prints the timer's
forward count and tick sum (run under rocprofv3 --kernel-trace to compare the count with the
output-layer launches of the last call).  usage: python tools/timer_count.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
timer = ctx.gemm_timer()
for i in range(2):
    paths = amx.sample_points(eng, pol, num_to_collect=40000, base_seed=i, num_workers=4)
    relabel_paths(paths, cost, ens)
    torch.cuda.synchronize()
    tv = timer.cpu().tolist()
    n = sum(len(p["rewards"]) for p in paths)
    print(f"call {i}: {n} samples, timer forwards {tv[3]}, ticks {tv[2] / 1e5:.3f} ms, arrivals left {tv[1]}",
          flush=True)
    timer.zero_()
    torch.cuda.synchronize()
