"""Worker process of tests/test_gpu_multirank.py (started fresh by the test; not collected).

usage: python multirank_worker.py RANK WORLD PORT OUT.npz

One rank of a lane-sharded rollout on the GPU (several ranks may share one card): rank r of
`world` owns lanes [r*B/world, (r+1)*B/world) of a B_TOTAL-lane rollout.  Reset rows and
policy noise are injected from global per-lane arrays, so the union of the ranks' lanes
is the same set of trajectories as one process running all B_TOTAL lanes.  The ranks'
only exchange is RolloutEngine.relabel's all-reduce of [sum phi, count] (gloo here, over
host copies; RCCL on the 8-GPU path).  Then a second engine checks the two-graph HIP-graph
replay (graph_rollout with the all-reduce between the graphs) against eager rollouts, and two
more the overlapped forms (rollout_overlapped / graph_rollout_overlapped: each all-reduce under
the next rollout's first forward).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

S, A = 197, 36
# the shape: AMX_MR_LANES lanes in total over the ranks, AMX_MR_STEPS steps per rollout,
# AMX_MR_EXPERT expert rows (default: a small case; the test also runs the N = 8 per-rank share,
# 2 x 5120 lanes x 1 step with 12 500 expert rows -> 6 250 per rank)
B_TOTAL = int(os.environ.get("AMX_MR_LANES", "512"))
K = int(os.environ.get("AMX_MR_STEPS", "4"))
N_EXPERT = int(os.environ.get("AMX_MR_EXPERT", "2048"))
HORIZON = 3


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    import amp_extensions_amd as amx
    from amp_extensions_amd import dist as D
    from amp_extensions_amd import synthetic as syn
    from amp_extensions_amd.ensemble import init_ensemble_weights
    from amp_extensions_amd.policy import init_mlp_policy_params
    allreduce = None
    if world > 1:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)

        def allreduce(t):  # gloo reduces host tensors: copy out, reduce, copy back
            h = t.cpu()
            dist.all_reduce(h)
            t.copy_(h)

    class _Done:
        def wait(self):
            pass

    class _Pending:
        """A real asynchronous gloo all-reduce of a host copy: wait() completes it and copies the
        sum back on the current stream, so the GPU-side orderings the overlapped and sharded paths
        rely on (wait before the relabel reads the message / overwrites the expert sum) are
        exercised with the collective still in flight across the ranks."""

        def __init__(self, t):
            import torch.distributed as dist
            self.t, self.h = t, t.cpu()
            self.work = dist.all_reduce(self.h, async_op=True)

        def wait(self):
            self.work.wait()
            self.t.copy_(self.h)

    def allreduce_async(t):  # the overlapped path's handle
        return _Pending(t) if allreduce is not None else _Done()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s, a, s2 = syn.offline(4096, S, A, 0)
    from amp_extensions_amd.datasets import get_transformations
    norms = get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=dev)
    ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
    ens.compute_threshold(torch.from_numpy(s).float().to(dev), torch.from_numpy(a).float().to(dev))
    expert = torch.from_numpy(syn.expert(N_EXPERT, S, 3))
    pw, ls = init_mlp_policy_params(S, A)
    table = syn.reset_table(1024, S, 1)
    lo, hi = D.shard(B_TOTAL, rank, world)
    B = hi - lo
    g = np.random.RandomState(42)  # the global per-lane inputs, identical on every rank
    rows0 = g.randint(0, 1024, B_TOTAL).astype(np.int32)
    noise = g.randn(K, B_TOTAL, A)
    rrows = g.randint(0, 1024, (K, B_TOTAL)).astype(np.int32)
    term = amx.TerminationConfig(horizon=HORIZON)

    def engine(seed):
        cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100, ctx=ctx)
        if world > 1:  # each rank scores its block of the expert rows; the partial sums all-reduced
            cost.shard_expert(rank, world, allreduce_async)
        pol = amx.DevicePolicy(ctx, pw, ls, seed=D.rank_seed(5, rank))
        return amx.RolloutEngine(ens, table, lanes=B, term=term, policy=pol, cost=cost, seed=D.rank_seed(seed, rank),
                                 max_steps=K), cost

    # ---- eager rollout with injected per-lane inputs + relabel(allreduce) --------------------
    eng, cost = engine(7)
    eng.reset_all(rows=torch.from_numpy(rows0[lo:hi]).to(dev))
    eng.begin_rollout()
    for t in range(K):
        eng.step(noise=torch.from_numpy(noise[t, lo:hi].copy()).to(dev),
                 reset_rows=torch.from_numpy(rrows[t, lo:hi].copy()).to(dev))
    info = eng.relabel(allreduce)
    mmd = float(info["mb_mmd"].item())
    res = dict(lo=lo, hi=hi, mb_mmd=mmd, rewards=eng.rewards[:K, :B].cpu().numpy(),
               next_obs=eng.next_obs.cpu().numpy(), done=eng.done.cpu().numpy(),
               phi_sum=eng.phi_sum.cpu().numpy(), expert_cost=float(cost.get_expert_cost().item()),
               expert_cost_again=float(cost.get_expert_cost().item()),  # read twice: one all-reduce
               bonus_mmd=eng.bonus_mmd(allreduce))  # global mean(-rewards) - expert cost
    # ---- HIP-graph replay of whole rollouts (two graphs around the all-reduce) vs eager -----
    if world > 1 or os.environ.get("AMX_GRAPH_SINGLE") == "1":
        e1, c1 = engine(9)
        e2, c2 = engine(9)
        for e in (e1, e2):
            e.reset_all()
        e1.rollout(); e1.relabel(allreduce); c1.get_expert_cost()
        e2.rollout(); e2.relabel(allreduce); c2.get_expert_cost()

        def graph_args(c_):  # sharded expert cost: its all-reduce around the relabel graph
            if c_.expert_sharded:
                return dict(tail=None, before_relabel=c_.wait_expert_allreduce, after=c_.expert_allreduce_replayed)
            return dict(tail=c_.get_expert_cost)
        replay = e2.graph_rollout(K, allreduce=allreduce, **graph_args(c2))
        for _ in range(2):
            e1.rollout(); e1.relabel(allreduce); c1.get_expert_cost()
            replay()
        c2.get_expert_cost()
        # the overlapped forms (each all-reduce under the next rollout's first forward, its
        # relabel after that forward; flush_relabel / flush for the last one), eager and graph
        e3, c3 = engine(9)
        e4, c4 = engine(9)
        for e, c_ in ((e3, c3), (e4, c4)):
            e.reset_all()
            e.rollout(); e.relabel(allreduce); c_.get_expert_cost()
        replay4, flush4 = e4.graph_rollout_overlapped(K, allreduce_async, **graph_args(c4))
        for _ in range(2):
            e3.rollout_overlapped(K, allreduce_async,
                                  tail=c3.expert_allreduce if c3.expert_sharded else c3.get_expert_cost)
            replay4()
        e3.flush_relabel()
        flush4()
        c3.get_expert_cost()
        c4.get_expert_cost()
        torch.cuda.synchronize()
        res.update(ovl_rewards=e3.rewards[:K, :B].cpu().numpy(), ovl_mmd=float(e3.mb_mmd.item()),
                   ovl_obs=e3.obs.cpu().numpy(), ovl_expert=float(c3._expert_mean.item()),
                   govl_rewards=e4.rewards[:K, :B].cpu().numpy(), govl_mmd=float(e4.mb_mmd.item()),
                   govl_obs=e4.obs.cpu().numpy(), govl_expert=float(c4._expert_mean.item()))
        res.update(graph_rewards=e2.rewards[:K, :B].cpu().numpy(), eager_rewards=e1.rewards[:K, :B].cpu().numpy(),
                   graph_mmd=float(e2.mb_mmd.item()), eager_mmd=float(e1.mb_mmd.item()),
                   graph_obs=e2.obs.cpu().numpy(), eager_obs=e1.obs.cpu().numpy(),
                   graph_expert=float(c2._expert_mean.item()), eager_expert=float(c1._expert_mean.item()))
    np.savez(out, **res)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
