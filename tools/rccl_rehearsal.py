"""One-rank RCCL rehearsal of bench.py's multi-rank plumbing on a single GPU: the "nccl" process
group (RCCL) with device_id, the per-rollout all-reduce of the [sum phi | count] fp64 message in
the serial order (eager and between the two graphs of a replay) and in the overlapped order
(async_op handles), barriers and the MAX-reduce of the elapsed time.  Results must equal the
no-collective run bit for bit (a one-rank sum is the identity).
usage: torchrun --nproc-per-node 1 --master-addr 127.0.0.1 --master-port P tools/rccl_rehearsal.py"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

S, A, B, T = 197, 36, 5120, 1
dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
s, a, s2 = syn.offline(4096, S, A, 0)
norms = get_transformations(*(torch.from_numpy(x).float() for x in (s, a, s2)))
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device=dev)
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
ens.compute_threshold(torch.from_numpy(s).float().to(dev), torch.from_numpy(a).float().to(dev))
expert = torch.from_numpy(syn.expert(20000, S, 3))
pw, ls = init_mlp_policy_params(S, A)
table = syn.reset_table(4096, S, 1)


def engine():
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100, ctx=ctx)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=5)
    e = amx.RolloutEngine(ens, table, lanes=B, policy=pol, cost=cost, seed=9, max_steps=T)
    e.reset_all()
    return e, cost


ar = lambda t: dist.all_reduce(t)                       # noqa: E731
ar_async = lambda t: dist.all_reduce(t, async_op=True)  # noqa: E731
ref, cref = engine()
eg, cg = engine()
eo, co = engine()
for e, c, f in ((ref, cref, None), (eg, cg, ar), (eo, co, ar)):
    e.rollout(T); e.relabel(f); c.get_expert_cost()
replay = eg.graph_rollout(T, allreduce=ar, tail=cg.get_expert_cost)
oreplay, oflush = eo.graph_rollout_overlapped(T, ar_async, tail=co.get_expert_cost)
for _ in range(3):
    ref.rollout(T); ref.relabel(None); cref.get_expert_cost()
    replay()
    oreplay()
oflush()
dist.barrier()
torch.cuda.synchronize()
el = torch.tensor([1.0], dtype=torch.float64, device=dev)
dist.all_reduce(el, op=dist.ReduceOp.MAX)
ok = (torch.equal(ref.rewards, eg.rewards) and torch.equal(ref.rewards, eo.rewards) and
      torch.equal(ref.obs, eg.obs) and torch.equal(ref.obs, eo.obs) and
      float(ref.mb_mmd.item()) == float(eg.mb_mmd.item()) == float(eo.mb_mmd.item()) and
      float(cref._expert_mean.item()) == float(cg._expert_mean.item()) == float(co._expert_mean.item()))
print(f"rccl rehearsal: serial graph + overlapped graph == no-collective run: {ok}; mb_mmd {float(ref.mb_mmd):.6g}",
      flush=True)
dist.destroy_process_group()
sys.exit(0 if ok else 1)
