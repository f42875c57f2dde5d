"""cProfile of the reference-semantics path (bench.py --mode paths): one warm sample_points +
relabel_paths at the bench shape, then a profiled one.
usage: python tools/paths_profile.py [W] [chunk] [fuse|nofuse]  (fuse: the sampler engine's policy
launch writes the ensemble input, RolloutEngine.fuse_assembly)"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402
from amp_extensions_amd.relabel import relabel_paths  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 4
CHUNK = int(sys.argv[2]) if len(sys.argv) > 2 else 8
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


def once(i):
    t0 = time.perf_counter()
    paths = amx.sample_points(eng, pol, num_to_collect=40000, base_seed=i, num_workers=W, chunk=CHUNK)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    relabel_paths(paths, cost, ens)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    n = sum(len(p["rewards"]) for p in paths)
    print(f"W={W} chunk={CHUNK}: {n} samples, {len(paths)} paths: sample_points {1e3 * (t1 - t0):.1f} ms, relabel_paths "
          f"{1e3 * (t2 - t1):.1f} ms", flush=True)


once(1)
if len(sys.argv) > 3:
    for e in eng.__dict__.get("_sampler_engines", {}).values():
        e.fuse_assembly = sys.argv[3] == "fuse"
    print(f"fuse_assembly = {sys.argv[3] == 'fuse'}")
once(2)
once(2)
pr = cProfile.Profile()
pr.enable()
once(3)
pr.disable()
buf = io.StringIO()
pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(35)
print(buf.getvalue())
buf = io.StringIO()
pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
print(buf.getvalue())
