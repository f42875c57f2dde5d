"""amx_step_reset: the step kernel with the table reset of done lanes fused in (RolloutEngine's
default) against amx_step / amx_step_rexp followed by amx_reset_lanes(mask = done) — every
lane buffer bit-identical over rollouts with horizon and fall resets (sim_env.py:150-285)."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _engines(cost_kind, flag="fuse_reset"):
    import amp_extensions_amd as amx
    from amp_extensions_amd.humanoid import TerminationConfig
    S, A, B = 197, 36, 320
    rs = np.random.RandomState(0)
    s = 0.5 * rs.randn(2048, S)
    s[:, 0] = rs.uniform(0.8, 0.95, 2048)
    a = rs.randn(2048, A)
    s2 = s + 0.01 * rs.randn(2048, S)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=DEV)
    ctx.set_termination(TerminationConfig(horizon=3))  # horizon resets every third step
    ens = amx.DeviceEnsemble(ctx, R.init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    expert = torch.from_numpy(np.concatenate([s[:300], s2[:300]], 1)).float()
    out = []
    for fused in (False, True):
        if cost_kind == "mmd":
            cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, bw_samples=5000, lambda_b=0.0025,
                                     seed=100, ctx=ctx)
        elif cost_kind == "gail":
            cost = amx.GAILCost(expert, hidden_dims=[256, 128], lambda_b=0.4, seed=100, ctx=ctx)
        else:
            cost = None
        pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
        eng = amx.RolloutEngine(ens, s[:97], lanes=B, policy=pol, cost=cost, seed=2, max_steps=8)
        setattr(eng, flag, fused)
        out.append(eng)
    return out


@pytest.mark.parametrize("cost_kind", ["mmd", "gail", "none"])
def test_fused_step_reset_matches_step_then_reset(cost_kind):
    engs = _engines(cost_kind)
    for eng in engs:
        eng.reset_all()
        for _ in range(2):
            eng.rollout()
    torch.cuda.synchronize()
    ref, got = engs
    names = ["obs", "next_obs", "acts", "done", "disc", "num_steps", "model_idx", "reset_count", "reset_rows",
             "nonfinite", "cost_in", "cost_rexp"]
    for n in names:
        x, y = getattr(ref, n), getattr(got, n)
        if x is None:
            assert y is None
            continue
        assert torch.equal(x, y), n
    done = ref.done.bool()
    assert done.any() and not done.all()  # both branches ran
    assert (ref.reset_rows[done[:, :ref.B]] >= 0).all()


@pytest.mark.parametrize("cost_kind", ["mmd", "gail"])
def test_score_overlap_bit_identical(cost_kind):
    # (GAIL: the flag is ignored -- the discriminator GEMMs' K split depends on the row count)
    """RolloutEngine.score_overlap (each step's cost rows scored on a side stream under the next
    step's policy) against the batched pass at the rollout's end: every feature, fp64 partial,
    disagreement, reward and relabel output bit-identical over rollouts with resets."""
    engs = _engines(cost_kind, flag="score_overlap")
    outs = []
    for eng in engs:
        eng.reset_all()
        for _ in range(3):
            eng.rollout()
            outs.append(eng.relabel() if cost_kind == "mmd" else None)
    torch.cuda.synchronize()
    ref, got = engs
    names = ["cost_in", "cost_rexp", "disc", "rewards"] + (["phi", "partials", "ipm", "wbonus", "_fbuf"]
                                                          if cost_kind == "mmd" else [])
    bits = {torch.float32: torch.int32, torch.float64: torch.int64}
    for n in names:
        x, y = getattr(ref, n), getattr(got, n)
        if x.dtype in bits:  # bit patterns (the padding rows' rewards are NaN on both sides)
            x, y = x.view(bits[x.dtype]), y.view(bits[y.dtype])
        assert torch.equal(x, y), n
    if cost_kind == "mmd":
        assert [float(o["mb_mmd"]) for o in outs[:3]] == [float(o["mb_mmd"]) for o in outs[3:]]
    assert (got._side is not None) == (cost_kind == "mmd") and ref._side is None


@pytest.mark.parametrize("hidden", [(32, 32), (64, 48)])
def test_policy_fused_assembly_bit_identical(hidden):
    """k_policy writing the ensemble's x0 rows itself (fused assembly) gives the same actions and
    means as without, and the same x0 rows as the separate assembly kernel, bit for bit; the
    means follow the oracle's float32 MLP (gaussian_mlp.py:95-104)."""
    import amp_extensions_amd as amx
    S, A, B = 197, 36, 1000
    rs = np.random.RandomState(4)
    s = 0.5 * rs.randn(2048, S)
    a = rs.randn(2048, A)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s + 0.01)])
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=DEV)
    ctx.set_normalizers(norms)
    pw, log_std = R.init_policy_weights(S, A, hidden, seed=100)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).to(DEV)
    outs = []
    for fused in (False, True):
        act = torch.empty(B, A, dtype=torch.float64, device=DEV)
        mean = torch.empty(B, A, dtype=torch.float32, device=DEV)
        x0 = torch.zeros(4, 1024, ctx.ldk, dtype=torch.float32, device=DEV)
        pol.act(ob, B, act, 7, mean_out=mean, x0=x0 if fused else None)
        outs.append((act, mean, x0))
    x0_sep = torch.zeros(4, 1024, ctx.ldk, dtype=torch.float32, device=DEV)
    from amp_extensions_amd import _native as N
    N.check(ctx.lib.amx_assemble_input(ctx.h, ob.data_ptr(), outs[0][0].data_ptr(), N.AMX_IN_F64, x0_sep.data_ptr(),
                                       1024 * ctx.ldk, ctx.ldk, B, ctx.stream), "amx_assemble_input")
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[1][2][:, :B, :ctx.k0_pad], x0_sep[:, :B, :ctx.k0_pad])
    obn = ob.cpu().numpy()
    ref = np.stack([R.policy_mean(pw, obn[i]) for i in range(0, B, 37)])  # the oracle's float32 MLP
    np.testing.assert_allclose(outs[1][1].cpu().numpy()[::37], ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("cost_kind", ["mmd", "gail"])
def test_policy_fused_x0_matches_separate_assembly(cost_kind):
    """RolloutEngine.fuse_assembly (the policy launch writes the shared x0 slice and its row
    exponents, amx_policy_act with row_exp) against the separate amx_assemble_input_rexp launch:
    every lane buffer, the ensemble workspace and the rewards bit-identical over two rollouts."""
    engs = _engines(cost_kind, flag="fuse_assembly")
    for eng in engs:
        eng.reset_all()
        for _ in range(2):
            eng.rollout()
            eng.relabel()
    torch.cuda.synchronize()
    ref, got = engs
    for n in ["obs", "next_obs", "acts", "done", "disc", "num_steps", "model_idx", "cost_in", "cost_rexp",
              "rewards", "steps0"]:
        x, y = getattr(ref, n, None), getattr(got, n, None)
        if x is None:
            continue
        torch.testing.assert_close(x, y, rtol=0, atol=0, equal_nan=True, msg=n)  # (padding rows are NaN)
    wr, wg = ref.ens.workspace(ref.B), got.ens.workspace(got.B)
    assert torch.equal(wr["preds"], wg["preds"]) and torch.equal(wr["rexp"], wg["rexp"])
