"""The per-rank configuration the strong-scaling runs actually execute (bench.py plan_lanes):
N = 8 -> 5120 lanes x 1 step, N = 4 -> 5120 x 2, replayed as captured HIP graphs, with the
stream-K output layer (self-resetting arrival counters), the 128 x 64 RFF tiles and the
rank's 6 250-row block of a 50 000-row expert buffer (RBFLinearCost.shard_expert), the
two-graph form around the cross-rank all-reduce.  Here one process plays rank 0 of 8: the
all-reduce is the identity, so the witness is rank 0's and the expert sum is rank 0's partial.

Checks: graph replays bit-identical to the same rollouts launched eagerly (lane states,
actions, rewards, mb_mmd, the expert partial sum); the last rollout against the CPU oracle
(mb_mmd over every row and rewards on a strided subset at rtol 1e-4, next states at 2e-5,
linear_cost.py:84-152, dynamics.py:216-233); the expert partial vs an fp64 host sum of the
rank's block.  Plus the ADVICE round-2 case: a graph captured at 4096 lanes still replays
correctly after a 7168-lane forward on the same context grew the stream-K workspace."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
S, A, LAM = 197, 36, 0.0025


class _Done:
    def wait(self):
        pass


def _identity_allreduce(t):  # one process standing in for rank 0: the sum over ranks is its own
    return None


def _identity_async(t):
    return _Done()


def t32(x):
    return torch.from_numpy(np.ascontiguousarray(x)).float()


@pytest.fixture(scope="module")
def model():
    import amp_extensions_amd as amx
    from amp_extensions_amd import synthetic as syn
    n = torch.get_num_threads()
    torch.set_num_threads(16)
    s, a, s2 = syn.offline(20000, S, A, 0)
    norms = R.get_transformations(t32(s), t32(a), t32(s2))
    ens_w = R.init_ensemble_weights(S, A, [512] * 4, 4, 100)
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=DEV)
    ens = amx.DeviceEnsemble(ctx, ens_w, norms)
    thr = ens.compute_threshold(t32(s).to(DEV), t32(a).to(DEV))
    expert = torch.from_numpy(syn.expert(50000, S, 3))
    yield amx, syn, ctx, ens, ens_w, norms, thr, expert
    torch.set_num_threads(n)


def _engine(model, B, T, shard):
    amx, syn, ctx, ens, ens_w, norms, thr, expert = model
    from amp_extensions_amd.policy import init_mlp_policy_params
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, lambda_b=LAM, seed=100, ctx=ctx)
    if shard:
        cost.shard_expert(0, 8, _identity_async)
    pw, ls = init_mlp_policy_params(S, A)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=1000)
    eng = amx.RolloutEngine(ens, syn.reset_table(65536, S, 1), lanes=B, policy=pol, cost=cost, seed=(7 << 32),
                            max_steps=T)
    eng.reset_all()
    eng.num_steps.copy_(torch.randint(0, 300, (B,), generator=torch.Generator().manual_seed(11),
                                      dtype=torch.int32).to(DEV))  # the bench's steady-state spread
    return eng, cost


def _snap(eng, cost):
    return [eng.obs.clone(), eng.acts.clone(), eng.rewards.clone(), eng.mb_mmd.clone(),
            cost._expert_out[:1].clone(), eng.done.clone()]


@pytest.mark.parametrize("T", [1, 2])
def test_n8_n4_rank_share_graph_replay(model, T):
    amx, syn, ctx, ens, ens_w, norms, thr, expert = model
    B = 5120
    runs = []
    for graph in (False, True):
        eng, cost = _engine(model, B, T, shard=True)
        eng.rollout(T)
        eng.relabel(_identity_allreduce)
        out = []
        if graph:
            replay = eng.graph_rollout(T, allreduce=_identity_allreduce, tail=None,
                                       before_relabel=cost.wait_expert_allreduce, after=cost.expert_allreduce_replayed)
            for _ in range(3):
                replay()
                out.append(_snap(eng, cost))
        else:
            for _ in range(3):
                eng.rollout(T)
                eng.relabel(_identity_allreduce)
                cost.expert_allreduce()
                out.append(_snap(eng, cost))
        torch.cuda.synchronize()
        runs.append(out)
        assert getattr(ctx, "_split_ws", None) is not None  # 5120 lanes: the stream-K output layer
    for ea, eb in zip(*runs):
        for xa, xb in zip(ea, eb):
            assert torch.equal(xa, xb)
    assert not torch.equal(runs[1][0][1], runs[1][1][1])  # fresh policy noise per replay
    # the last rollout vs the oracle
    n = B * T
    obs = eng.obs[:T].cpu().numpy().reshape(-1, S)
    nxt = eng.next_obs.cpu().numpy().reshape(-1, S)
    act = eng.acts.cpu().numpy().reshape(-1, A)
    ref = R.RBFLinearCostRef(expert, feature_dim=512, bw_quantile=0.1, lambda_b=LAM, seed=100)
    mmd = ref.fit_cost(t32(np.concatenate([obs, nxt], 1)))
    np.testing.assert_allclose(float(eng.mb_mmd.item()), mmd, rtol=1e-4)
    idx = np.arange(0, n, 53)
    # the member of each transition: the lane's model index, carried across rollouts
    done_all = torch.stack([r[5] for r in runs[1]]).cpu().numpy().astype(np.int64)  # [3, T, B]
    # resets before this rollout: reset_all (1) + every done of the earlier rollouts (incl. warm-up)
    first = eng.reset_count.cpu().numpy().astype(np.int64) - done_all[-1].sum(0)
    dn = done_all[-1].astype(np.int64)
    k_step = ((first[None, :] + np.concatenate([np.zeros((1, B), np.int64), np.cumsum(dn, 0)[:-1]], 0)) % 4)
    k_step = k_step.reshape(-1)
    preds = R.ensemble_preds(ens_w, norms, t32(obs[idx]), t32(act[idx])).numpy()
    ref_next = obs[idx] + preds[k_step[idx], np.arange(idx.size)].astype(np.float64)
    # lanes that reset in the step carry the reset row in obs[t+1], but next_obs is the pre-reset s'
    err = np.abs(nxt[idx] - ref_next).max() / max(1.0, np.abs(ref_next).max())
    assert err <= 2e-5, err
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    cst, _ = ref.get_bonus_costs(t32(obs[idx]), t32(act[idx]), disc_fn, thr, next_states=t32(nxt[idx]))
    rew = eng.rewards[:T, :B].cpu().numpy().reshape(-1)
    want = -cst.numpy()[:, 0]
    np.testing.assert_allclose(rew[idx], want, rtol=1e-4, atol=1e-4 * np.abs(want).max())
    # the rank's expert block (rows [0, 6250)): fp64 partial sum of clamp(phi_E w, -1, 0)
    cost = eng.cost
    blk = cost.expert_rep[:6250].double() @ cost.w.double()
    want_sum = torch.clamp(blk, -1.0, 0.0).sum().item()
    np.testing.assert_allclose(float(cost._expert_out[0].item()), want_sum, rtol=1e-6, atol=1e-9)
    assert cost._ehi - cost._elo == 6250


def test_graph_survives_split_workspace_growth(model):
    """A rollout graph captured at 4096 lanes (stream-K scratch sized for 4096) replays with the
    same bits after a 7168-lane forward registered a larger scratch on the same context: the
    captured launches keep the old buffers, which the context keeps alive (AmxContext._retained)."""
    amx, syn, ctx, ens, ens_w, norms, thr, expert = model
    B, T = 4096, 2
    runs = []
    for graph in (False, True):
        eng, cost = _engine(model, B, T, shard=False)
        eng.rollout(T)
        eng.relabel()
        out = []
        if graph:
            replay = eng.graph_rollout(T, tail=cost.get_expert_cost)
            before = ctx._split_ws[0].data_ptr()
            rs = np.random.RandomState(4)
            ob = torch.from_numpy(0.5 * rs.randn(7168, S)).to(DEV)
            ac = torch.from_numpy(rs.randn(7168, A)).to(DEV)
            ens.forward_preds(ob, ac, 7168)
            torch.cuda.synchronize()
            assert ctx._split_ws[0].data_ptr() != before  # the workspace grew
            torch.cuda.empty_cache()
            for _ in range(3):
                replay()
                out.append(_snap(eng, cost))
        else:
            for _ in range(3):
                eng.rollout(T)
                eng.relabel()
                cost.get_expert_cost()
                out.append(_snap(eng, cost))
        torch.cuda.synchronize()
        runs.append(out)
    for ea, eb in zip(*runs):
        for xa, xb in zip(ea, eb):
            assert torch.equal(xa, xb)
    assert int(ctx._split_ws[1].abs().sum().item()) == 0
