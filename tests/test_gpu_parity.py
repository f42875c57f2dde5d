"""GPU parity of every HIP kernel of the hot path against the CPU oracle (and, where the
reference's own outputs exist, against the golden fixtures).  All calls go through the
C ABI (libamx_hip.so) via the product classes; nothing here falls back to the CPU.

Tolerances (fp32 work; the oracle runs torch-CPU fp32 with a different summation order):
  * ensemble deltas:          max|gpu-ref| <= 2e-5 * max(1, max|ref|)   (K <= 2302 fp32 dots)
  * disagreement:             rel 1e-4
  * RFF features / w / costs: abs 2e-6 on phi (|phi| <= 0.0625), rel 1e-4 on rewards
  * termination, reset rows, model index, step counters, Philox: bit-exact
  * fp64 state update given identical deltas: bit-exact
"""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu

S, A = 226, 28
DEV = "cuda"


def synthetic_offline(n, seed, S=S, A=A):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


@pytest.fixture(scope="module")
def amx():
    import amp_extensions_amd as amx
    assert torch.cuda.is_available(), "GPU tests need a ROCm GPU"
    return amx


@pytest.fixture(scope="module")
def norms():
    s, a, s2 = synthetic_offline(2048, 0)
    return R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])


def make_ensemble(amx, hidden, norms, M=4, gemm="f16x3"):
    ens_w = R.init_ensemble_weights(S, A, hidden, M, 100)
    ctx = amx.AmxContext(S, A, n_models=M, hidden=hidden[0], n_hidden=len(hidden), feat_dim=512, device=DEV)
    return ctx, ens_w, amx.DeviceEnsemble(ctx, ens_w, norms, gemm=gemm)


def rel_err(x, ref):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return np.abs(x - ref).max() / max(1.0, np.abs(ref).max())


def test_philox_matches_oracle(amx):
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, device=DEV)
    from amp_extensions_amd import _native as N
    out = torch.empty(1000 * 4, dtype=torch.int32, device=DEV)
    seed = 0x1234567890ABCDEF
    N.check(ctx.lib.amx_philox(ctx.h, seed, 5, 6, 7, out.data_ptr(), 1000, ctx.stream))
    got = out.cpu().numpy().view(np.uint32).reshape(1000, 4)
    ctr = np.stack([np.arange(1000, dtype=np.uint32), np.full(1000, 5, np.uint32), np.full(1000, 6, np.uint32),
                    np.full(1000, 7, np.uint32)], -1)
    ref = R.philox4x32_10(ctr, (seed & 0xFFFFFFFF, seed >> 32))
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("gemm", ["f16x3", "bf16x6", "f32"])
@pytest.mark.parametrize("tag", ["h64", "h512"])
def test_ensemble_vs_reference_golden(amx, golden, norms, tag, gemm):
    """Device ensemble (every GEMM path) vs the REFERENCE's own DynamicsModel.forward outputs."""
    g = golden(f"g1_ensemble_{tag}.npz")
    hidden = [int(x) for x in g["hidden"]]
    ctx, _, ens = make_ensemble(amx, hidden, norms, gemm=gemm)
    rs = np.random.RandomState(int(g["query_seed"]))
    B = int(g["B"])
    qs = torch.from_numpy(rs.randn(B, S) * 0.5).float()
    qa = torch.from_numpy(rs.randn(B, A)).float()
    preds = ens.forward_preds(qs.to(DEV), qa.to(DEV), B)[:, :B].cpu().numpy()
    assert rel_err(preds, g["preds"]) <= 2e-5
    disc = ens.get_action_discrepancy(qs, qa).cpu().numpy()
    np.testing.assert_allclose(disc, g["disc"], rtol=1e-4, atol=1e-6)
    s, a, _ = synthetic_offline(2048, 0)
    thr = ens.compute_threshold(torch.from_numpy(s).float().to(DEV), torch.from_numpy(a).float().to(DEV))
    np.testing.assert_allclose(thr, float(g["threshold"]), rtol=1e-4)


@pytest.mark.parametrize("gemm", ["f16x3", "bf16x6", "f32"])
def test_ensemble_forward_f64_padding(amx, norms, gemm):
    """fp64 state input (SimEnv's ob) with B not a multiple of 128, full [512]*4 ensemble."""
    ctx, ens_w, ens = make_ensemble(amx, [512] * 4, norms, gemm=gemm)
    rs = np.random.RandomState(11)
    B = 333
    ob = rs.randn(B, S) * 0.5
    ac = rs.randn(B, A)
    preds = ens.forward_preds(torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV), B)[:, :B].cpu().numpy()
    ref = R.ensemble_preds(ens_w, norms, torch.from_numpy(ob).float(), torch.from_numpy(ac).float()).numpy()
    assert rel_err(preds, ref) <= 2e-5


def _step_inputs(n_boundary=True, B=512, seed=3):
    """States near every fall threshold so done flips on last-bit differences."""
    rs = np.random.RandomState(seed)
    ob = np.zeros((B, S))
    ob[:, 0] = rs.uniform(0.5, 1.0, B)
    ob[:, 1:] = 0.3 * rs.randn(B, S - 1)
    pred = (0.01 * rs.randn(B, S)).astype(np.float32)
    env = R.SimEnvRef([None], None)
    for b in range(B):
        bi = b % len(R.FALL_BODIES)
        off = env.fall_contact_bodies_offset[bi]
        thr = 0.5 * env.fall_contact_bodies_params[bi][0] + 0.0001
        # put the body's next y exactly on / next to the threshold
        want = thr - (ob[b, 0] + np.float64(pred[b, 0]))
        ob[b, off + 1] = want - np.float64(pred[b, off + 1])
        k = (b // len(R.FALL_BODIES)) % 3
        ob[b, off + 1] = [np.nextafter(ob[b, off + 1], -np.inf), ob[b, off + 1],
                          np.nextafter(ob[b, off + 1], np.inf)][k]
    return ob, pred


def test_step_termination_bit_exact(amx, norms):
    ctx, _, ens = make_ensemble(amx, [64] * 4, norms)
    from amp_extensions_amd import _native as N
    for horizon in (300, 3):
        cfg = amx.TerminationConfig(horizon=horizon)
        ctx.set_termination(cfg)
        ob, pred = _step_inputs()
        B = ob.shape[0]
        M = 4
        rs = np.random.RandomState(9)
        model_idx = rs.randint(0, M, B).astype(np.int32)
        preds = np.zeros((M, B, S), np.float32)
        for m in range(M):
            preds[m] = pred + (m - model_idx[:, None]) * np.float32(0.001)
        preds[model_idx, np.arange(B)] = pred
        num_steps = rs.randint(0, 5, B).astype(np.int32)
        d_preds = torch.from_numpy(preds).to(DEV)
        d_ob = torch.from_numpy(ob).to(DEV)
        d_next = torch.empty_like(d_ob)
        d_ns = torch.from_numpy(num_steps).to(DEV)
        d_done = torch.empty(B, dtype=torch.uint8, device=DEV)
        d_disc = torch.empty(B, dtype=torch.float32, device=DEV)
        cost_in = torch.full((B, ctx.k_rff_pad), 7.0, dtype=torch.float32, device=DEV)
        N.check(ctx.lib.amx_step(ctx.h, d_preds.data_ptr(), S, B * S, torch.from_numpy(model_idx).to(DEV).data_ptr(),
                                 d_ob.data_ptr(), d_next.data_ptr(), d_ns.data_ptr(), d_done.data_ptr(),
                                 d_disc.data_ptr(), cost_in.data_ptr(), ctx.k_rff_pad, None, B, ctx.stream))
        ref_next, ref_done, ref_ns = R.step_update_terminate(ob, pred, num_steps, horizon=horizon)
        np.testing.assert_array_equal(d_next.cpu().numpy(), ref_next)
        np.testing.assert_array_equal(d_done.cpu().numpy(), ref_done)
        np.testing.assert_array_equal(d_ns.cpu().numpy(), ref_ns)
        assert 0 < ref_done.sum() < B
        ci = cost_in.cpu().numpy()
        np.testing.assert_array_equal(ci[:, :S], ob.astype(np.float32))
        np.testing.assert_array_equal(ci[:, S:2 * S], ref_next.astype(np.float32))
        assert (ci[:, 2 * S:] == 0).all()
        # disagreement of the injected members
        tp = torch.from_numpy(preds)
        ref_d = torch.stack([torch.norm(tp[i] - tp[j], dim=1) for i in range(M) for j in range(i + 1, M)]).max(0).values
        np.testing.assert_allclose(d_disc.cpu().numpy(), ref_d.numpy(), rtol=1e-5)


def test_step_velocity_check_mutates(amx, norms):
    """enable_velocity_check with RecordVelAsPos: the reference's in-place /= is kept."""
    ctx, _, ens = make_ensemble(amx, [64] * 4, norms)
    from amp_extensions_amd import _native as N
    cfg = amx.TerminationConfig(enable_velocity_check=True, record_vel_as_pos=True)
    ctx.set_termination(cfg)
    B = 256
    rs = np.random.RandomState(4)
    ob = np.zeros((B, S))
    ob[:, 0] = 2.0
    ob[:, 1:] = 0.1 * rs.randn(B, S - 1)
    ob[:, 136:] = rs.uniform(-3, 3, (B, S - 136))  # /(1/30) -> |v| <= 90 ...
    ob[1::2, 140] = 3.4                              # ... except one velocity of odd lanes (102)
    for b in range(B):  # keep every body clear of the ground
        for bi, body in enumerate(R.FALL_BODIES):
            ob[b, 9 * body + 2] = 1.0
    pred = np.zeros((B, S), np.float32)
    preds = np.stack([pred] * 4)
    model_idx = np.zeros(B, np.int32)
    d_ob = torch.from_numpy(ob).to(DEV)
    d_next = torch.empty_like(d_ob)
    d_ns = torch.zeros(B, dtype=torch.int32, device=DEV)
    d_done = torch.empty(B, dtype=torch.uint8, device=DEV)
    N.check(ctx.lib.amx_step(ctx.h, torch.from_numpy(preds).to(DEV).data_ptr(), S, B * S,
                             torch.from_numpy(model_idx).to(DEV).data_ptr(), d_ob.data_ptr(), d_next.data_ptr(),
                             d_ns.data_ptr(), d_done.data_ptr(), None, None, 0, None, B, ctx.stream))
    ref_next, ref_done, _ = R.step_update_terminate(ob, pred, np.zeros(B, np.int32), enable_velocity_check=True,
                                                    record_vel_as_pos=True)
    np.testing.assert_array_equal(d_next.cpu().numpy(), ref_next)
    np.testing.assert_array_equal(d_done.cpu().numpy(), ref_done)
    assert 0 < ref_done.sum() < B


def test_reset_rows_and_model_rotation(amx, norms):
    ctx, _, ens = make_ensemble(amx, [64] * 4, norms)
    table, _, _ = synthetic_offline(97, 1)
    eng = amx.RolloutEngine(ens, table, lanes=300, seed=77, max_steps=4)
    eng.reset_all()
    torch.cuda.synchronize()
    rows = R.reset_rows(77, np.arange(300), np.ones(300, np.int64), 97)
    np.testing.assert_array_equal(eng.obs[0].cpu().numpy(), table[rows])
    np.testing.assert_array_equal(eng.model_idx.cpu().numpy(), np.full(300, 1))  # first trajectory: member 1
    np.testing.assert_array_equal(eng.num_steps.cpu().numpy(), np.zeros(300))


@pytest.mark.parametrize("gemm", ["f16x3", "bf16x6", "f32"])
def test_rff_mmd_vs_reference_golden(amx, golden, norms, gemm):
    """Device RBFLinearCost (every feature-GEMM path) vs the REFERENCE's outputs
    (bandwidth/W/b init bit-exact)."""
    g = golden("g5_rff_mmd.npz")
    es, _, es2 = synthetic_offline(512, 3)
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], dim=1)
    ctx, ens_w, ens = make_ensemble(amx, [64] * 4, norms)
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100, ctx=ctx,
                             gemm=gemm)
    assert cost.bw == float(g["bw"])
    np.testing.assert_array_equal(cost.rff_weight.numpy()[:4, :8], g["W_head"])
    np.testing.assert_allclose(cost.phi_e.cpu().numpy(), g["phi_e"], atol=2e-6)
    ps, pa, ps2 = synthetic_offline(96, 4)
    mmd = cost.fit_cost(torch.cat([torch.from_numpy(ps), torch.from_numpy(ps2)], 1).float())
    np.testing.assert_allclose(mmd, float(g["mb_mmd"]), rtol=1e-4)
    np.testing.assert_allclose(cost.w.cpu().numpy(), g["w"], atol=3e-6)
    s, a, _ = synthetic_offline(2048, 0)
    ens.compute_threshold(torch.from_numpy(s).float().to(DEV), torch.from_numpy(a).float().to(DEV))
    bc, info = cost.get_bonus_costs(torch.from_numpy(ps).float().to(DEV), torch.from_numpy(pa).float().to(DEV), ens,
                                    next_states=torch.from_numpy(ps2).float().to(DEV))
    ref = g["cost"]
    np.testing.assert_allclose(bc.cpu().numpy(), ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max())
    np.testing.assert_allclose(info["ipm"].cpu().numpy(), g["ipm"], rtol=1e-4, atol=1e-4 * np.abs(ref).max())
    np.testing.assert_allclose(info["bonus"].cpu().numpy(), g["bonus"], rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(float(cost.get_expert_cost()), float(g["expert_cost"]), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("gemm", ["f16x3", "bf16x6", "f32"])
@pytest.mark.parametrize("tag", ["h64", "h1024"])
def test_gail_vs_reference_golden(amx, golden, norms, tag, gemm):
    g = golden(f"g6_gail_{tag}.npz")
    hid = [int(x) for x in g["hidden"]]
    es, _, es2 = synthetic_offline(512, 3)
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], dim=1)
    ctx, ens_w, ens = make_ensemble(amx, [64] * 4, norms)
    gc = amx.GAILCost(expert, hidden_dims=hid, lambda_b=float(g["lambda_b"]), seed=100, ctx=ctx, gemm=gemm)
    ps, pa, ps2 = synthetic_offline(96, 4)
    ss = torch.cat([torch.from_numpy(ps), torch.from_numpy(ps2)], 1).float()
    logits = gc.disc_logits(ss.to(DEV)).cpu().numpy()
    np.testing.assert_allclose(logits, g["logits"], rtol=1e-4, atol=1e-4 * np.abs(g["logits"]).max())
    np.testing.assert_allclose(gc.get_costs(ss.to(DEV)).cpu().numpy(), g["cost_plain"], rtol=1e-4, atol=1e-5)
    bc, info = gc.get_bonus_costs(torch.from_numpy(ps).float().to(DEV), torch.from_numpy(pa).float().to(DEV), ens,
                                  next_states=torch.from_numpy(ps2).float().to(DEV))
    np.testing.assert_allclose(bc.cpu().numpy(), g["cost"], rtol=1e-4, atol=1e-5)


def test_policy_action(amx, norms):
    ctx, _, ens = make_ensemble(amx, [64] * 4, norms)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100, init_log_std=-0.25)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=42)
    B = 200
    rs = np.random.RandomState(5)
    ob = rs.randn(B, S)
    d_ob = torch.from_numpy(ob).to(DEV)
    act = torch.empty(B, A, dtype=torch.float64, device=DEV)
    mean = torch.empty(B, A, dtype=torch.float32, device=DEV)
    noise = torch.from_numpy(rs.randn(B, A)).to(DEV)
    pol.act(d_ob, B, act, counter=3, noise=noise, mean_out=mean)
    ref_mean = np.stack([R.policy_mean(pw, ob[b]) for b in range(B)])
    np.testing.assert_allclose(mean.cpu().numpy(), ref_mean, rtol=1e-4, atol=1e-6)
    # the fp64 action algebra is exact given the device mean and the injected noise
    np.testing.assert_array_equal(act.cpu().numpy(), mean.cpu().numpy().astype(np.float64) +
                                  np.exp(np.float64(log_std.numpy())) * noise.cpu().numpy())
    pol.act(d_ob, B, act, counter=3, mean_out=mean)
    z = R.policy_noise(42, 3, B, A)
    np.testing.assert_allclose(act.cpu().numpy() - mean.cpu().numpy().astype(np.float64),
                               np.exp(np.float64(log_std.numpy())) * z, rtol=1e-12, atol=1e-12)


def test_policy_fused_assembly_bit_exact(amx, norms):
    """amx_policy_act's fused x0 rows == amx_assemble_input on the same (ob, act)."""
    from amp_extensions_amd import _native as N
    ctx, _, ens = make_ensemble(amx, [64] * 4, norms)
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100, init_log_std=-0.25)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=9)
    B = 300
    ob = torch.from_numpy(np.random.RandomState(1).randn(B, S)).to(DEV)
    act = torch.empty(B, A, dtype=torch.float64, device=DEV)
    ws = ens.workspace(B)
    ws["act"].fill_(7.0)
    pol.act(ob, B, act, counter=5, x0=ws["act"])
    fused = ws["act"][:, :B, :ctx.k0_pad].clone()
    ws["act"].fill_(-3.0)
    N.check(ctx.lib.amx_assemble_input(ctx.h, ob.data_ptr(), act.data_ptr(), 0, ws["act"].data_ptr(),
                                       ws["Bp"] * ctx.ldk, ctx.ldk, B, ctx.stream))
    ref = ws["act"][:, :B, :ctx.k0_pad]
    assert torch.equal(fused, ref)


def test_rollout_matches_simenv_oracle(amx, norms):
    """End-to-end lanes vs per-lane SimEnvRef with the same actions and reset rows."""
    ctx, ens_w, ens = make_ensemble(amx, [512] * 4, norms)
    table, _, _ = synthetic_offline(64, 1)
    B, K = 256, 12
    eng = amx.RolloutEngine(ens, table, lanes=B, term=amx.TerminationConfig(horizon=5), seed=3, max_steps=K)
    eng.reset_all()
    rs = np.random.RandomState(8)
    acts = rs.randn(K, B, A) * np.exp(-0.25)
    for t in range(K):
        eng.step(actions=torch.from_numpy(acts[t]).to(DEV))
    torch.cuda.synchronize()
    rows0 = R.reset_rows(3, np.arange(B), np.ones(B, np.int64), 64)
    rr = eng.reset_rows.cpu().numpy()
    envs = [R.SimEnvRef(ens_w, norms, horizon=5) for _ in range(B)]
    for b in range(B):
        envs[b].reset(table[rows0[b]])
    obs, nxt, done = eng.obs.cpu().numpy(), eng.next_obs.cpu().numpy(), eng.done.cpu().numpy()
    worst = 0.0
    for t in range(K):
        for b in range(B):
            e = envs[b]
            np.testing.assert_allclose(obs[t, b], e.ob, rtol=0, atol=1e-4)
            e.ob = obs[t, b].copy()  # re-anchor on the device state (per-step parity)
            no, _, d, _ = e.step(acts[t, b].copy())
            worst = max(worst, np.abs(nxt[t, b] - no).max() / max(1.0, np.abs(no).max()))
            assert bool(done[t, b]) == d, (t, b)
            if d:
                assert rr[t, b] >= 0
                e.reset(table[rr[t, b]])
    assert worst <= 2e-5


def test_rollout_relabel_mmd(amx, norms):
    """Full MILO relabel over an engine rollout vs the oracle relabel of the same samples."""
    ctx, ens_w, ens = make_ensemble(amx, [64] * 4, norms)
    es, _, es2 = synthetic_offline(1000, 3)
    expert = torch.cat([torch.from_numpy(es).float(), torch.from_numpy(es2).float()], dim=1)
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100, ctx=ctx)
    s, a, _ = synthetic_offline(2048, 0)
    thr = ens.compute_threshold(torch.from_numpy(s).float().to(DEV), torch.from_numpy(a).float().to(DEV))
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
    table, _, _ = synthetic_offline(128, 1)
    B, K = 200, 6
    eng = amx.RolloutEngine(ens, table, lanes=B, policy=pol, cost=cost, seed=5, max_steps=K)
    eng.reset_all()
    eng.rollout()
    info = eng.relabel()
    torch.cuda.synchronize()
    obs = eng.obs[:K].cpu().numpy().reshape(-1, S)
    nxt = eng.next_obs.cpu().numpy().reshape(-1, S)
    acts = eng.acts.cpu().numpy().reshape(-1, A)
    ref = R.RBFLinearCostRef(expert, feature_dim=512, bw_quantile=0.1, lambda_b=0.0025, seed=100)
    mmd = ref.fit_cost(torch.from_numpy(np.concatenate([obs, nxt], 1)).float())
    np.testing.assert_allclose(float(info["mb_mmd"]), mmd, rtol=1e-4)
    disc_fn = lambda st, ac: R.compute_discrepancy(ens_w, norms, st, ac)
    cst, ci = ref.get_bonus_costs(torch.from_numpy(obs).float(), torch.from_numpy(acts).float(), disc_fn, thr,
                                  next_states=torch.from_numpy(nxt).float())
    rew = eng.rewards[:K, :B].cpu().numpy().reshape(-1)
    ref_rew = -cst.numpy()[:, 0]
    np.testing.assert_allclose(rew, ref_rew, rtol=1e-4, atol=1e-4 * np.abs(ref_rew).max())
    bm = eng.bonus_mmd()
    ref_bm = np.mean(-ref_rew) - ref.get_expert_cost().item()
    np.testing.assert_allclose(bm, ref_bm, rtol=1e-4, atol=1e-7)
