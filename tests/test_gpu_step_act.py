"""The fused step + next action (amx_step_reset_act, RolloutEngine.fuse_step_act, an A/B option
off by default: DESIGN §6): step t's
kernel also runs the policy of step t + 1 on the observations it produced -- actions, means,
Philox noise, and the x0 + row-exponent assembly of step t + 1's f16x3 forward.  The work
decomposition of the policy is the stand-alone kernel's, so a rollout is bit-identical with the
fusion on and off: lane states, next states, actions, means, done flags, disagreement, rewards,
mb_mmd -- eager and as a captured HIP graph, with horizon/fall resets inside the rollout, at
lane counts with a partial last workgroup, in eval mode, and at the 226/28 scene layout.
Reference: gym-simenv/gym_simenv/envs/sim_env.py:140-285 (step/reset) and
mjrl/mjrl/policies/gaussian_mlp.py:95-104 (get_action) as milo/milo/sampler.py:48-65 chains them."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(S, A, B, K, eval_mode=False, graph=False, fuse=True, horizon=4):
    import amp_extensions_amd as amx
    from amp_extensions_amd.humanoid import TerminationConfig
    rs = np.random.RandomState(0)
    s = 0.5 * rs.randn(2048, S)
    s[:, 0] = rs.uniform(0.8, 0.95, 2048)
    a = rs.randn(2048, A)
    s2 = s + 0.01 * rs.randn(2048, S)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    w = R.init_ensemble_weights(S, A, [512] * 4, 4, 100)
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=DEV)
    ens = amx.DeviceEnsemble(ctx, w, norms)
    ens.compute_threshold(torch.from_numpy(s).float().to(DEV), torch.from_numpy(a).float().to(DEV))
    expert = torch.from_numpy(np.concatenate([s[:300], s2[:300]], 1)).float()
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, bw_samples=5000, lambda_b=0.0025, seed=100,
                             ctx=ctx)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
    term = TerminationConfig(horizon=horizon) if S == 197 else None
    eng = amx.RolloutEngine(ens, s[:64], lanes=B, policy=pol, cost=cost, seed=2, max_steps=K, eval_mode=eval_mode,
                            record_means=True, term=term)
    eng.fuse_step_act = fuse
    eng.reset_all()
    return eng, cost


def _snap(eng):
    T, B = eng.t, eng.B
    return [x.clone() for x in (eng.obs[:T + 1], eng.next_obs[:T], eng.acts[:T], eng.means[:T], eng.done[:T],
                                eng.disc[:T, :B], eng.rewards[:T, :B], eng.num_steps, eng.reset_count,
                                eng.model_idx)] + [torch.as_tensor(eng.mb_mmd).clone()]


def _runs(S, A, B, K, eval_mode=False, graph=False, n=3, w8=False):
    out = {}
    for fuse in (False, True):
        eng, cost = _setup(S, A, B, K, eval_mode=eval_mode, fuse=fuse)
        eng.ctx.lib.amx_set_step_act_occupancy(eng.ctx.h, int(w8))
        eng.rollout()
        eng.relabel()
        snaps = []
        if graph:
            replay = eng.graph_rollout(K, tail=cost.get_expert_cost)
            for _ in range(n):
                replay()
                snaps.append(_snap(eng))
        else:
            for _ in range(n):
                eng.rollout()
                eng.relabel()
                snaps.append(_snap(eng))
        torch.cuda.synchronize()
        out[fuse] = (snaps, eng)
    return out


@pytest.mark.parametrize("S,A,B,K,graph,eval_mode,w8", [(197, 36, 1000, 5, False, False, False),
                                                        (197, 36, 1000, 5, True, False, True),
                                                        (197, 36, 5120, 2, True, False, False),
                                                        (197, 36, 300, 4, False, True, True),
                                                        (226, 28, 257, 3, False, False, False)])
def test_fused_step_act_bit_identical(S, A, B, K, graph, eval_mode, w8):
    out = _runs(S, A, B, K, eval_mode=eval_mode, graph=graph, w8=w8)
    (ref, _), (got, eng) = out[False], out[True]
    names = ["obs", "next_obs", "acts", "means", "done", "disc", "rewards", "num_steps", "reset_count", "model_idx",
             "mb_mmd"]
    for i, (sa, sb) in enumerate(zip(ref, got)):
        for name, xa, xb in zip(names, sa, sb):
            assert torch.equal(xa, xb), f"rollout {i}: {name} differs with the fused step + action"
    if S == 197:
        assert int(ref[-1][4].sum()) > 0  # horizon resets happened inside the rollouts
    # the fused path ran: the engine's last rollout left its step-t + 1 action flags consumed
    assert eng._act_ready == -1


def test_fused_step_act_matches_policy_oracle():
    """The actions the fused kernel writes for step t + 1 are the stand-alone policy's on the
    observations it produced: means vs the oracle's FCNetwork (rel 1e-4), noise vs the oracle's
    Philox + Box-Muller (1e-12)."""
    S, A, B, K = 197, 36, 300, 3
    eng, _ = _setup(S, A, B, K, fuse=True)
    eng.rollout()
    torch.cuda.synchronize()
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    obs = eng.obs[:K].cpu().numpy()
    means = eng.means[:K].cpu().numpy()
    acts = eng.acts[:K].cpu().numpy()
    scale = np.exp(np.float64(log_std.numpy()))
    for t in range(1, K):  # slots written by the fused kernel
        ref = np.stack([R.policy_mean(pw, obs[t, b]) for b in range(B)])
        np.testing.assert_allclose(means[t], ref, rtol=1e-4, atol=1e-6)
        z = R.policy_noise(1, eng.step_counter - K + t, B, A)
        np.testing.assert_allclose(acts[t] - means[t].astype(np.float64), scale * z, rtol=1e-12, atol=1e-12)
