"""Cost input types and cost variants on the device vs the oracle:
  * RBFLinearCost / GAILCost input_type 'sa', 'sas', 's' (linear_cost.py:115-127,
    gail_cost.py:258-268), RBFLinearCost cost_range=None (raw cost and raw disagreement
    bonus, linear_cost.py:103, 138-139), GAILCost log-likelihood loss (get_ll_costs,
    gail_cost.py:238-251);
  * the rollout engine's cost-input rows (amx_cost_rows) and rewards for those types;
  * AMP-feature cost input ('amp'): engine rows == AMP(s, s') of the recorded states, checked
    against the oracle's state_amp_obs restatement (parity unpinned vs the C++ core).
Tolerances as test_gpu_parity: rel 1e-4 on costs/rewards; the cost-input rows are exact
(fp64 -> fp32 casts) except 'amp' (device vs host libm, 1e-5 after the fp32 cast)."""
import json

import numpy as np
import pytest
import torch

from oracle import deepmimic_ref as DR
from oracle import milo_ref as R

from test_gpu_parity import A, DEV, S, make_ensemble, synthetic_offline

pytestmark = pytest.mark.gpu
TYPES = ["sa", "sas", "s"]


@pytest.fixture(scope="module")
def amx():
    import amp_extensions_amd as amx
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    return amx


@pytest.fixture(scope="module")
def norms():
    s, a, s2 = synthetic_offline(2048, 0)
    return R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])


def t32(x):
    return torch.from_numpy(np.asarray(x)).float()


def expert_rows(typ, n=512):
    es, ea, es2 = synthetic_offline(n, 3)
    return R.cost_input(typ, t32(es), t32(ea), t32(es2))


def close(x, ref, rtol=1e-4):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    np.testing.assert_allclose(x, ref, rtol=rtol, atol=rtol * max(1e-3, np.abs(ref).max()))


@pytest.mark.parametrize("cost_range", [(-1.0, 0.0), None])
@pytest.mark.parametrize("typ", TYPES + ["ss"])
def test_rbf_input_types_vs_oracle(amx, norms, typ, cost_range):
    ctx, ens_w, ens = make_ensemble(amx, [64] * 4, norms)
    expert = expert_rows(typ)
    cost = amx.RBFLinearCost(expert, feature_dim=512, input_type=typ, cost_range=cost_range, lambda_b=0.3,
                             seed=100, ctx=ctx)
    ref = R.RBFLinearCostRef(expert, feature_dim=512, input_type=typ, cost_range=cost_range, lambda_b=0.3,
                             seed=100)
    assert cost.bw == ref.bw
    ps, pa, ps2 = synthetic_offline(300, 4)
    x = R.cost_input(typ, t32(ps), t32(pa), t32(ps2))
    close(cost.fit_cost(x.to(DEV)), ref.fit_cost(x), rtol=1e-4)
    close(cost.get_costs(x.to(DEV)).cpu().numpy(), ref.get_costs(x).numpy())
    s, a, _ = synthetic_offline(2048, 0)
    thr = ens.compute_threshold(t32(s).to(DEV), t32(a).to(DEV))
    bc, info = cost.get_bonus_costs(t32(ps).to(DEV), t32(pa).to(DEV), ens, next_states=t32(ps2).to(DEV))
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    rc, ri = ref.get_bonus_costs(t32(ps), t32(pa), disc_fn, thr, next_states=t32(ps2))
    for k in ("bonus", "ipm", "v_targ", "cost"):
        close(info[k].cpu().numpy(), ri[k].numpy())
    close(bc.cpu().numpy(), rc.numpy())
    if cost_range is None:
        with pytest.raises(AttributeError):
            cost.get_expert_cost()
    else:
        close(float(cost.get_expert_cost()), float(ref.get_expert_cost()), rtol=1e-4)


@pytest.mark.parametrize("loss", ["least_squares", "logistic"])
@pytest.mark.parametrize("typ", TYPES)
def test_gail_input_types_and_loss_vs_oracle(amx, norms, typ, loss):
    ctx, ens_w, ens = make_ensemble(amx, [64] * 4, norms)
    expert = expert_rows(typ)
    gc = amx.GAILCost(expert, hidden_dims=[256, 128], input_type=typ, lambda_b=0.4, seed=100, ctx=ctx,
                      disc_loss_type=loss)
    w = R.init_disc_weights(expert.shape[1], (256, 128), seed=100)
    ps, pa, ps2 = synthetic_offline(300, 4)
    x = R.cost_input(typ, t32(ps), t32(pa), t32(ps2))
    ref_costs = R.gail_ls_costs(w, x) if loss == "least_squares" else R.gail_ll_costs(w, x)
    close(gc.get_costs(x.to(DEV)).cpu().numpy(), ref_costs.numpy())
    s, a, _ = synthetic_offline(2048, 0)
    ens.compute_threshold(t32(s).to(DEV), t32(a).to(DEV))
    bc, info = gc.get_bonus_costs(t32(ps).to(DEV), t32(pa).to(DEV), ens, next_states=t32(ps2).to(DEV))
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    rc, ri = R.gail_bonus_costs(w, t32(ps), t32(pa), t32(ps2), disc_fn, 0.4, input_type=typ, disc_loss_type=loss)
    close(bc.cpu().numpy(), rc.numpy())
    close(info["v_targ"].cpu().numpy(), ri["v_targ"].numpy())


@pytest.mark.parametrize("typ", TYPES)
def test_rollout_cost_rows_and_relabel(amx, norms, typ):
    """Engine rollout with an input_type cost: recorded rows are the fp32 casts of the lane
    buffers; MMD relabel rewards and GAIL rewards vs the oracle on the recorded samples."""
    ctx, ens_w, ens = make_ensemble(amx, [64] * 4, norms)
    s, a, _ = synthetic_offline(2048, 0)
    thr = ens.compute_threshold(t32(s).to(DEV), t32(a).to(DEV))
    expert = expert_rows(typ, 800)
    cost = amx.RBFLinearCost(expert, feature_dim=512, input_type=typ, lambda_b=0.0025, seed=100, ctx=ctx)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
    table, _, _ = synthetic_offline(128, 1)
    B, K = 200, 5
    eng = amx.RolloutEngine(ens, table, lanes=B, policy=pol, cost=cost, seed=5, max_steps=K)
    eng.reset_all()
    eng.rollout()
    info = eng.relabel()
    torch.cuda.synchronize()
    obs = eng.obs[:K].cpu().numpy().reshape(-1, S)
    nxt = eng.next_obs.cpu().numpy().reshape(-1, S)
    acts = eng.acts.cpu().numpy().reshape(-1, A)
    x = R.cost_input(typ, t32(obs), t32(acts), t32(nxt))
    rows = eng.cost_in[:, :B].cpu().reshape(K * B, -1)
    assert torch.equal(rows[:, :x.shape[1]], x) and (rows[:, x.shape[1]:] == 0).all()
    assert (eng.cost_in[:, B:] == 0).all()
    ref = R.RBFLinearCostRef(expert, feature_dim=512, input_type=typ, lambda_b=0.0025, seed=100)
    close(float(info["mb_mmd"]), ref.fit_cost(x), rtol=1e-4)
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    cst, _ = ref.get_bonus_costs(t32(obs), t32(acts), disc_fn, thr, next_states=t32(nxt))
    close(eng.rewards[:K, :B].cpu().numpy().reshape(-1), -cst.numpy()[:, 0])
    # GAIL on the same input type: rewards from the batched discriminator pass
    gc = amx.GAILCost(expert, hidden_dims=[256, 128], input_type=typ, lambda_b=0.4, seed=100, ctx=ctx)
    eng2 = amx.RolloutEngine(ens, table, lanes=B, policy=pol, cost=gc, seed=5, max_steps=K)
    eng2.reset_all()
    eng2.rollout()
    torch.cuda.synchronize()
    obs = eng2.obs[:K].cpu().numpy().reshape(-1, S)
    nxt = eng2.next_obs.cpu().numpy().reshape(-1, S)
    acts = eng2.acts.cpu().numpy().reshape(-1, A)
    w = R.init_disc_weights(expert.shape[1], (256, 128), seed=100)
    rc, _ = R.gail_bonus_costs(w, t32(obs), t32(acts), t32(nxt), disc_fn, 0.4, input_type=typ)
    close(eng2.rewards[:K, :B].cpu().numpy().reshape(-1), -rc.numpy()[:, 0])


def test_input_width_mismatch_raises(amx, norms):
    ctx, _, ens = make_ensemble(amx, [64] * 4, norms)
    cost = amx.RBFLinearCost(expert_rows("sa"), feature_dim=512, input_type="ss", seed=100, ctx=ctx)
    table, _, _ = synthetic_offline(16, 1)
    with pytest.raises(ValueError):
        amx.RolloutEngine(ens, table, lanes=8, cost=cost, max_steps=2)


def test_amp_feature_cost_in_rollout(amx, golden):
    """'amp' cost input: discriminator on AMP(s, s') of each recorded transition of a
    motion-reset rollout; rows vs the oracle's state_amp_obs, rewards vs the oracle
    discriminator on those rows."""
    from amp_extensions_amd.ensemble import init_ensemble_weights
    from amp_extensions_amd.motion import ReferenceMotion
    from amp_extensions_amd.policy import init_mlp_policy_params
    g = golden("g12_motion.npz")
    char = json.loads(str(g["character_json"]))
    motion = {"Loop": str(g["loop"]), "Frames": g["frames"].tolist()}
    ctx = amx.AmxContext(226, 28, n_models=4, hidden=128, n_hidden=2, device=DEV)
    rm = ReferenceMotion(ctx, char, motion)
    rs = np.random.RandomState(0)
    s, a = rs.randn(512, 226) * 0.5, rs.randn(512, 28)
    norms = [torch.from_numpy(x).float() for x in (s.mean(0), np.abs(s).mean(0) + 1e-8, a.mean(0),
                                                   np.abs(a).mean(0) + 1e-8, np.zeros(226), np.full(226, 0.003))]
    ens_w = init_ensemble_weights(226, 28, [128] * 2, 4, 100)
    ens = amx.DeviceEnsemble(ctx, ens_w, norms)
    ens.compute_threshold(torch.from_numpy(s).float().to(DEV), torch.from_numpy(a).float().to(DEV))
    times = rs.uniform(1.0 / 30, rm.get_motion_length(), 400)
    expert = rm.expert_amp_obs(times).float().cpu()
    gc = amx.GAILCost(expert, hidden_dims=[256, 128], input_type="amp", lambda_b=0.3, seed=100, ctx=ctx, motion=rm)
    pw, ls = init_mlp_policy_params(226, 28)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=4)
    B, K = 192, 4
    eng = amx.RolloutEngine(ens, rm, lanes=B, policy=pol, cost=gc, seed=9, max_steps=K)
    eng.reset_all()
    eng.rollout()
    torch.cuda.synchronize()
    obs, nxt = eng.obs[:K].cpu().numpy(), eng.next_obs.cpu().numpy()
    acts = eng.acts.cpu().numpy()
    J, _, _ = DR.load_character(char)
    ee = [5, 8, 11, 14]
    ref_rows = np.stack([DR.state_amp_obs(J, ee, obs[t, b], nxt[t, b]) for t in range(K) for b in range(B)])
    rows = eng.cost_in[:, :B].cpu().numpy().reshape(K * B, -1)
    np.testing.assert_allclose(rows[:, :226], ref_rows.astype(np.float32), rtol=1e-5,
                               atol=1e-5 * max(1.0, np.abs(ref_rows).max()))
    assert (rows[:, 226:] == 0).all()
    w = R.init_disc_weights(226, (256, 128), seed=100)
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    x = torch.from_numpy(rows[:, :226])
    st, ac = t32(obs.reshape(-1, 226)), t32(acts.reshape(-1, 28))
    ic = R.gail_ls_costs(w, x)
    ref_cost = (1 - 0.3) * ic - 0.3 * disc_fn(st, ac).view(-1, 1)
    close(eng.rewards[:K, :B].cpu().numpy().reshape(-1), -ref_cost.numpy()[:, 0])
    # the facade builds the same rows from (s, s')
    bc, _ = gc.get_bonus_costs(torch.from_numpy(obs.reshape(-1, 226)).to(DEV), torch.from_numpy(
        acts.reshape(-1, 28)).to(DEV), ens, next_states=torch.from_numpy(nxt.reshape(-1, 226)).to(DEV))
    close(bc.cpu().numpy(), ref_cost.numpy())
