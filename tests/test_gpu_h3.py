"""The f16x3 ensemble GEMM (power-of-two scaled operands split into two fp16 limbs, three
products on the f16 MFMA pipe, fp32 accumulation): parity with the oracle's fp32 forward
(dynamics.py:216-233, 422-433) at the f32 path's tolerance, per-row independence of the
activation scaling (extreme, zero and non-finite rows), determinism, the weight split and
the row-exponent slots, and the C ABI's argument checks."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def offline(n, seed, S, A):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


def make(S, A, hidden, gemms=("f16x3", "f32"), M=4):
    import amp_extensions_amd as amx
    s, a, s2 = offline(2048, 0, S, A)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ens_w = R.init_ensemble_weights(S, A, hidden, M, 100)
    ctx = amx.AmxContext(S, A, n_models=M, hidden=hidden[0], n_hidden=len(hidden), feat_dim=512, device=DEV)
    ens = {g: amx.DeviceEnsemble(ctx, ens_w, norms, gemm=g) for g in gemms}
    return amx, ctx, ens, ens_w, norms, (s, a)


def row_err(p, ref):
    """max |p - ref| per row over max(1, max |ref row|), over members."""
    d = np.abs(p - ref).max(axis=-1)
    return (d / np.maximum(1.0, np.abs(ref).max(axis=-1))).max(axis=0)


@pytest.mark.parametrize("S,A,hidden,B", [(197, 36, [512] * 4, 8192), (197, 36, [512] * 4, 640),
                                          (100, 20, [256] * 3, 640), (300, 40, [128] * 2, 384),
                                          (226, 28, [100] * 2, 200), (197, 36, [512] * 4, 4096),
                                          (197, 36, [512] * 4, 5120), (197, 36, [512] * 4, 6144),
                                          (197, 36, [512] * 4, 7168), (226, 28, [512] * 4, 5120)])
def test_f16x3_ensemble_matches_oracle_and_f32(S, A, hidden, B):
    """Tile paths: 8192 lanes -> 256x256 BK32 hidden tiles; 4096 / 5120 / 6144 / 7168 lanes ->
    the row-block tiles (RB x 256 hidden, RB x 112 / RB x 128 output, RB = 128 .. 224: one
    256-workgroup wave); 640 lanes at H = 512, S = 197 -> stream-K over K for the hidden
    (128 x 256) and output (128 x 224) tiles (few tiles: up to 6 workgroups per tile, combined in
    K order); other grids -> 128x128; S=197 -> the 128x224 output tile, S=100 ->
    128, S=300 -> three 128 tiles; hidden 100 -> padded columns.  Same tolerance as the f32
    path (2e-5 of max(1, |ref|)) and within 1e-6 of it."""
    amx, ctx, ens, ens_w, norms, (s, a) = make(S, A, hidden)
    rs = np.random.RandomState(1)
    ob = 0.5 * rs.randn(B, S)
    ob[:, 0] = rs.uniform(0.8, 0.95, B)
    ac = rs.randn(B, A)
    obd, acd = torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV)
    p3 = ens["f16x3"].forward_preds(obd, acd, B)[:, :B].cpu().numpy().astype(np.float64)
    p32 = ens["f32"].forward_preds(obd, acd, B)[:, :B].cpu().numpy().astype(np.float64)
    n = min(B, 1024)  # the fp32 CPU oracle on a prefix
    ref = R.ensemble_preds(ens_w, norms, torch.from_numpy(ob[:n]).float(), torch.from_numpy(ac[:n]).float()).numpy()
    scale = max(1.0, np.abs(ref).max())
    assert np.abs(p3[:, :n] - ref).max() / scale <= 2e-5
    assert np.abs(p32[:, :n] - ref).max() / scale <= 2e-5
    assert np.abs(p3 - p32).max() / max(1.0, np.abs(p32).max()) <= 1e-6


@pytest.mark.parametrize("S,A,B", [(197, 36, 8192), (197, 36, 640), (226, 28, 2048)])
def test_f16x3_shared_x0_matches_per_member_copies(S, A, B):
    """x0 assembled once (model 0's rows, amx_assemble_input_rexp with stride_m 0) and read by
    every member's GEMMs through k_shared gives the same bits as one x0 copy per member; the
    other members' x0 columns are not written."""
    amx, ctx, ens, ens_w, norms, (s, a) = make(S, A, [512] * 4, gemms=("f16x3",))
    e3 = ens["f16x3"]
    rs = np.random.RandomState(3)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).to(DEV)
    ac = torch.from_numpy(rs.randn(B, A)).to(DEV)
    e3.shared_x0 = False
    ref = e3.forward_preds(ob, ac, B)[:, :B].clone()
    buf = e3.workspace(B)["act"]
    buf[1:, :, :ctx.k0_pad].fill_(float("nan"))  # stale copies must not be read
    e3.shared_x0 = True
    got = e3.forward_preds(ob, ac, B)[:, :B].clone()
    assert torch.equal(got, ref)
    assert torch.isnan(buf[1:, :B, :ctx.k0_pad]).all()


def _f64_forward(ens_w, norms, ob, ac):
    mu_s, sd_s, mu_a, sd_a, mu_d, sd_d = [np.asarray(x, np.float64) for x in norms]
    x = np.concatenate([(ob.astype(np.float32).astype(np.float64) - mu_s) / sd_s,
                        (ac.astype(np.float32).astype(np.float64) - mu_a) / sd_a], 1)
    out = []
    for layers in ens_w:
        h = x
        for i, (W, b) in enumerate(layers):
            y = h @ np.asarray(W, np.float64).T + np.asarray(b, np.float64)
            if i < len(layers) - 1:
                h = np.concatenate([h, np.maximum(y, 0.0)], 1)
        out.append(y * sd_d + mu_d)
    return np.stack(out)


@pytest.mark.parametrize("B", [512, 5120])
def test_f16x3_extreme_and_zero_rows(B):
    """Rows 1e4x and 1e-4x the offline scale, rows exactly at the normalizer mean (x0 = 0) and
    ordinary rows in one batch: each row is scaled by its own power of two, so every row's
    error vs fp64 stays at fp32 level relative to that row, no worse than the f32 MFMA path's,
    and the ordinary rows are bit-identical to a batch without the extreme ones (B = 5120: the
    row-block tiles, RB = 160, and their per-block row-exponent reduction; fp64 check on the
    first 512 rows)."""
    S, A = 197, 36
    amx, ctx, ens, ens_w, norms, (s, a) = make(S, A, [512] * 4)
    rs = np.random.RandomState(2)
    ob = 0.5 * rs.randn(B, S)
    ob[:, 0] = rs.uniform(0.8, 0.95, B)
    ac = rs.randn(B, A)
    mu_s, mu_a = np.asarray(norms[0], np.float64), np.asarray(norms[2], np.float64)
    ob2, ac2 = ob.copy(), ac.copy()
    ob2[:64] = mu_s + (ob[:64] - mu_s) * 1e4
    ac2[:64] = mu_a + (ac[:64] - mu_a) * 1e4
    ob2[64:128] = mu_s + (ob[64:128] - mu_s) * 1e-4
    ac2[64:128] = mu_a + (ac[64:128] - mu_a) * 1e-4
    ob2[128:136] = mu_s.astype(np.float32)
    ac2[128:136] = mu_a.astype(np.float32)
    ref = _f64_forward(ens_w, norms, ob2[:512], ac2[:512])
    e3 = ens["f16x3"]
    p3 = e3.forward_preds(torch.from_numpy(ob2).to(DEV), torch.from_numpy(ac2).to(DEV), B)[:, :512].cpu().numpy()
    p32 = ens["f32"].forward_preds(torch.from_numpy(ob2).to(DEV), torch.from_numpy(ac2).to(DEV), B)[:, :512].cpu().numpy()
    r3, r32 = row_err(p3.astype(np.float64), ref), row_err(p32.astype(np.float64), ref)
    assert r3.max() <= 2e-5, r3.max()
    assert (r3 <= 2.0 * r32 + 1e-6).all()
    full = e3.forward_preds(torch.from_numpy(ob2).to(DEV), torch.from_numpy(ac2).to(DEV), B)[:, :B].cpu().numpy()
    clean = e3.forward_preds(torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV), B)[:, :B].cpu().numpy()
    np.testing.assert_array_equal(full[:, 136:], clean[:, 136:])


def test_f16x3_nonfinite_rows_stay_local_and_deterministic():
    """A NaN / inf state row propagates to that row's outputs only; the other rows match the
    finite batch bit for bit; two forwards of the same input are bit-identical (the row
    exponents come from per-layer slots, never read and written by one launch)."""
    S, A, B = 197, 36, 384
    amx, ctx, ens, ens_w, norms, (s, a) = make(S, A, [512] * 4, gemms=("f16x3",))
    e3 = ens["f16x3"]
    ob = torch.from_numpy(s[:B].copy()).to(DEV)
    ac = torch.from_numpy(a[:B].copy()).to(DEV)
    clean = e3.forward_preds(ob, ac, B)[:, :B].clone()
    again = e3.forward_preds(ob, ac, B)[:, :B].clone()
    assert torch.equal(clean, again)
    bad = ob.clone()
    bad[5, 3] = float("nan")
    bad[77, 0] = float("inf")
    got = e3.forward_preds(bad, ac, B)[:, :B].clone()
    assert torch.isnan(got[:, 5]).all() and not torch.isfinite(got[:, 77]).all()
    keep = torch.ones(B, dtype=torch.bool, device=DEV)
    keep[5] = keep[77] = False
    assert torch.equal(got[:, keep], clean[:, keep])


def test_f16x3_split_and_row_exponent_slots():
    """amx_split_f16x2: (limb0 + limb1) * 2^(E-14) reconstructs W to 2^-22 of the row max, with
    2^(E-1) <= max|W_row| < 2^E (zero rows E = -100); after a forward, slot i+1 of the row
    exponents holds the exponent of each row's largest h_i, slot 0 that of x0."""
    S, A, B = 197, 36, 256
    amx, ctx, ens, ens_w, norms, (s, a) = make(S, A, [512] * 4, gemms=("f16x3",))
    from amp_extensions_amd import _native as N
    from amp_extensions_amd.engine import split_f16x2
    rs = np.random.RandomState(5)
    W = (rs.randn(2, 128, 64) * np.exp(rs.uniform(-20, 20, (2, 128, 1)))).astype(np.float32)
    W[1, 7] = 0.0
    W2, wexp = split_f16x2(ctx, torch.from_numpy(W).to(DEV))
    torch.cuda.synchronize()
    E = wexp.cpu().numpy()
    limbs = W2.cpu().numpy().view(np.float16).astype(np.float64).reshape(2, 128, 4, 2, 16)
    rec = limbs.sum(axis=3).reshape(2, 128, 64) * np.exp2(E - 14.0)[..., None]
    rmax = np.abs(W).max(axis=-1).astype(np.float64)
    assert E[1, 7] == -100
    nz = rmax > 0
    assert (rmax[nz] < np.exp2(E[nz])).all() and (rmax[nz] >= np.exp2(E[nz] - 1.0)).all()
    assert (np.abs(rec - W).max(axis=-1) <= rmax * 2.0 ** -22).all()
    e3 = ens["f16x3"]
    ob = torch.from_numpy(s[:B]).to(DEV)
    ac = torch.from_numpy(a[:B]).to(DEV)
    e3.forward_preds(ob, ac, B)
    ws = e3.workspace(B)
    torch.cuda.synchronize()
    act, rexp = ws["act"].cpu().numpy(), ws["rexp"].cpu().numpy()
    k0, Hp = ctx.k0_pad, ctx.Hp

    def exps(x):
        m = np.abs(x).max(axis=-1)
        e = np.where(m > 0, np.frexp(m)[1], -100)
        return np.clip(e, -100, 100)

    x0_exp = exps(act[0, :B, :k0])  # the shared x0 slice lives in member 0's rows
    np.testing.assert_array_equal(rexp[:, 0, :B], np.broadcast_to(x0_exp, rexp[:, 0, :B].shape))
    for i in range(ctx.L):
        np.testing.assert_array_equal(rexp[:, i + 1, :B], exps(act[:, :B, k0 + i * Hp:k0 + (i + 1) * Hp]))


def test_f16x3_abi_checks():
    import amp_extensions_amd as amx
    ctx = amx.AmxContext(226, 28, n_models=4, hidden=128, n_hidden=2, device=DEV)
    lib, s = ctx.lib, ctx.stream
    buf = torch.zeros(1, 128, 64, dtype=torch.float32, device=DEV)
    W2 = torch.zeros(128, 128, dtype=torch.int16, device=DEV)
    we = torch.zeros(128, dtype=torch.int32, device=DEV)
    rc = lib.amx_gemm_bias_act_h3(ctx.h, 1, 128, 128, 64, buf.data_ptr(), 64, 0, W2.data_ptr(), 128 * 128,
                                  we.data_ptr(), 128, buf.data_ptr(), 0, buf.data_ptr(), 128, 0, 0, 1, None, 0, 1,
                                  None, 0, s)
    assert rc == -1 and b"null exponents" in lib.amx_last_error()
    rc = lib.amx_gemm_bias_act_h3(ctx.h, 1, 100, 128, 64, buf.data_ptr(), 64, 0, W2.data_ptr(), 128 * 128,
                                  we.data_ptr(), 128, buf.data_ptr(), 0, buf.data_ptr(), 128, 0, 0, 1, we.data_ptr(),
                                  128, 1, None, 0, s)
    assert rc == -1 and b"multiple of 128" in lib.amx_last_error()
    rc = lib.amx_gemm_bias_act_h3(ctx.h, 1, 128, 128, 64, buf.data_ptr(), 64, 0, W2.data_ptr(), 128 * 128,
                                  we.data_ptr(), 128, buf.data_ptr(), 0, buf.data_ptr(), 128, 0, 0, 1, we.data_ptr(),
                                  128, 1, None, 48, s)
    assert rc == -1 and b"k_shared" in lib.amx_last_error()
    rc = lib.amx_split_f16x2(ctx.h, 1, 128, 40, buf.data_ptr(), 64, 0, W2.data_ptr(), 128 * 128, we.data_ptr(), 128, s)
    assert rc == -1 and b"multiple of 16" in lib.amx_last_error()
    rc = lib.amx_row_exponents(ctx.h, 1, 128, 64, buf.data_ptr(), 64, 0, we.data_ptr(), 128, 2, s)
    assert rc == -1 and b"n_slots" in lib.amx_last_error()


def test_f16x3_rff_features_in_rollout():
    """The rollout's RFF pass (f16x3, row exponents written by amx_step_rexp) equals the
    same features with the exponents recomputed by amx_row_exponents bit for bit, and
    matches phi = cos(x W^T + b) sqrt(2/F) in fp64 (linear_cost.py:64-71) to fp32 level;
    the column partials are the fp64 sums of the phi rows."""
    S, A, B, K = 197, 36, 256, 3
    amx, ctx, ens, ens_w, norms, (s, a) = make(S, A, [512] * 4, gemms=("f16x3",))
    rs = np.random.RandomState(3)
    expert = torch.from_numpy(np.concatenate([s[:300], s[:300] + 0.01 * rs.randn(300, S)], 1)).float()
    cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, bw_samples=5000, lambda_b=0.0025, seed=100,
                             ctx=ctx)
    assert cost.map.W2 is not None
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
    eng = amx.RolloutEngine(ens["f16x3"], s[:64], lanes=B, policy=pol, cost=cost, seed=2, max_steps=K)
    eng.reset_all()
    eng.rollout()
    torch.cuda.synchronize()
    rows = K * eng.Bp
    x = eng.cost_in[:K].reshape(rows, -1)
    phi2 = torch.empty_like(eng.phi[:K].reshape(rows, -1))
    part2 = torch.empty_like(eng.partials[:K].reshape(rows // 32, -1))
    cost.map.features(x, rows, rows, phi2, part2)  # exponents recomputed in a separate pass
    torch.cuda.synchronize()
    phi = eng.phi[:K].reshape(rows, -1)
    assert torch.equal(phi, phi2)
    xd = x.double().cpu().numpy()[:, :2 * S]
    W = cost.rff_weight.double().numpy()
    ref = np.cos(xd @ W.T + cost.rff_bias.double().numpy()) * np.sqrt(2.0 / 512)
    # |x W^T| reaches ~1e2 here: fp32 rounding of the argument dominates (cos' <= 1)
    arg = np.abs(xd) @ np.abs(W).T
    err = np.abs(phi.double().cpu().numpy() - ref) / np.sqrt(2.0 / 512)
    assert (err <= 4e-7 * arg + 1e-6).all(), float((err - 4e-7 * arg).max())
    got = eng.partials[:K].reshape(rows // 32, -1).double().sum(0).cpu().numpy()
    np.testing.assert_allclose(got, phi.double().cpu().numpy().sum(0), rtol=1e-9, atol=1e-9)


def test_graph_replay_matches_eager_rollouts():
    """RolloutEngine.graph_rollout: replaying the captured rollout (steps, scoring, relabel,
    expert cost) gives bit-identical lane states, actions, rewards and mb_mmd to the same
    rollouts launched eagerly (the policy's Philox counter is device-resident)."""
    S, A, B, K = 197, 36, 256, 3
    amx, ctx, ens, ens_w, norms, (s, a) = make(S, A, [512] * 4, gemms=("f16x3",))
    rs = np.random.RandomState(3)
    expert = torch.from_numpy(np.concatenate([s[:300], s[:300] + 0.01 * rs.randn(300, S)], 1)).float()
    pw, log_std = R.init_policy_weights(S, A, (32, 32), seed=100)
    runs = []
    for graph in (False, True):
        cost = amx.RBFLinearCost(expert, feature_dim=512, bw_quantile=0.1, bw_samples=5000, lambda_b=0.0025,
                                 seed=100, ctx=ctx)
        pol = amx.DevicePolicy(ctx, pw, log_std, seed=1)
        eng = amx.RolloutEngine(ens["f16x3"], s[:64], lanes=B, policy=pol, cost=cost, seed=2, max_steps=K)
        eng.reset_all()
        eng.rollout()
        eng.relabel()
        out = []
        if graph:
            replay = eng.graph_rollout(K, tail=cost.get_expert_cost)
            for _ in range(3):
                replay()
                out.append([x.clone() for x in (eng.obs, eng.acts, eng.rewards, eng.mb_mmd)])
        else:
            for _ in range(3):
                eng.rollout()
                eng.relabel()
                cost.get_expert_cost()
                out.append([x.clone() for x in (eng.obs, eng.acts, eng.rewards, eng.mb_mmd)])
        torch.cuda.synchronize()
        runs.append(out)
    for ea, eb in zip(*runs):
        for xa, xb in zip(ea, eb):
            assert torch.equal(xa, xb)
    # successive replays draw fresh policy noise
    assert not torch.equal(runs[1][0][1], runs[1][1][1])


@pytest.mark.parametrize("B", [8192, 5120, 640])
def test_gemm_timer_counts_every_forward(B):
    """amx_set_gemm_timer: one start stamp per forward (first hidden layer) and one tick sum per
    output layer, eager and inside a captured graph; the arrival counter is left zero, the
    forward's results are unchanged."""
    amx, ctx, ens, ens_w, norms, (s, a) = make(197, 36, [512] * 4, gemms=("f16x3",))
    e = ens["f16x3"]
    rs = np.random.RandomState(2)
    obd = torch.from_numpy(0.5 * rs.randn(B, 197)).to(DEV)
    acd = torch.from_numpy(rs.randn(B, 36)).to(DEV)
    ref = e.forward_preds(obd, acd, B).clone()
    timer = ctx.gemm_timer()
    for _ in range(3):
        out = e.forward_preds(obd, acd, B)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    tv = timer.cpu().numpy()
    assert tv[3] == 3 and tv[1] == 0 and 0 < tv[2] < 3 * 100000  # < 1 ms per forward at 100 MHz
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            e.forward_preds(obd, acd, B)
    torch.cuda.synchronize()
    timer.zero_()
    for _ in range(4):
        g.replay()
    torch.cuda.synchronize()
    tv = timer.cpu().numpy()
    assert tv[3] == 4 and tv[1] == 0 and tv[2] > 0
    ctx.gemm_timer(False)


@pytest.mark.parametrize("B", [4096, 5120, 6144, 7168])
def test_output_stream_k_deterministic_and_close_to_unsplit(B):
    """4096-7168 lanes x 4 members (128-224 output tiles of 128 x 224, fewer than the CUs): the
    output layer runs stream-K (the tiles' K-tiles dealt evenly over one workgroup per CU; each
    tile's 1-3 segments summed in K order by the last arriver): repeated forwards give the same
    bits, the arrival counters are left zero, and the result is within fp32 rounding of the
    unsplit row-block tiles (amx_set_split_workspace unset)."""
    amx, ctx, ens, ens_w, norms, (s, a) = make(197, 36, [512] * 4, gemms=("f16x3",))
    e = ens["f16x3"]
    rs = np.random.RandomState(3)
    obd = torch.from_numpy(0.5 * rs.randn(B, 197)).to(DEV)
    acd = torch.from_numpy(rs.randn(B, 36)).to(DEV)
    p1 = e.forward_preds(obd, acd, B).clone()
    assert getattr(ctx, "_split_ws", None) is not None, f"{B} lanes should register the stream-K workspace"
    p2 = e.forward_preds(obd, acd, B).clone()
    torch.cuda.synchronize()
    assert torch.equal(p1, p2)
    assert int(ctx._split_ws[1].abs().sum().item()) == 0
    ctx.lib.amx_set_split_workspace(ctx.h, None, 0, None, 0)
    p0 = e.forward_preds(obd, acd, B).clone()
    scratch, counters = ctx._split_ws
    ctx.lib.amx_set_split_workspace(ctx.h, scratch.data_ptr(), scratch.numel(), counters.data_ptr(), counters.numel())
    torch.cuda.synchronize()
    d = (p1 - p0).abs().max().item()
    assert d <= 1e-6 * max(1.0, p0.abs().max().item()), d


@pytest.mark.parametrize("rows", [40960, 21504, 20480, 12288, 10240, 5120, 2048])
def test_rff_features_every_tile_shape(rows):
    """amx_rff_features_h3 on each of its tiles -- 40 960 / 20 480 rows: 160 x 256 (whole rounds at
    one per CU, the epilogue staged in 64-row passes); 21 504: 128 x 128 at three per CU; 12 288 /
    10 240: 128 x 128 at two; 5 120 / 2 048: 128 x 64 --
    against phi = cos(x W^T + b) sqrt(2/F) in fp64 (linear_cost.py:64-71, tolerance as
    test_f16x3_rff_features_in_rollout), the column partials against the fp64 sums of the valid
    phi rows of each 32-row group (AMX_RFF_PART_ROWS; n_valid and row_mask both applied), and
    bit-identical on a second launch."""
    import amp_extensions_amd as amx
    K, F = 416, 512
    ctx = amx.AmxContext(197, 36, n_models=1, hidden=128, n_hidden=1, feat_dim=F, device=DEV)
    lib, h = ctx.lib, ctx.h
    g = torch.Generator(device="cpu").manual_seed(rows)
    x = (0.5 * torch.randn(rows, K, generator=g)).float()
    x[:, 394:] = 0
    W = (torch.rand(F, K, generator=g) / 14.0).float()
    W[:, 394:] = 0
    b = ((torch.rand(F, generator=g) - 0.5) * 6.28).float()
    mask = (torch.rand(rows, generator=g) > 0.1).to(torch.uint8)
    n_valid = rows - 77 if rows != 20480 else 16000  # 20 480: n_valid well inside the rows
    xd, Wd, bd, md = x.to(DEV), W.to(DEV), b.to(DEV), mask.to(DEV)
    W2 = torch.empty(F * 2 * K, dtype=torch.int16, device=DEV)
    wexp = torch.empty(F, dtype=torch.int32, device=DEV)
    rexp = torch.empty(rows, dtype=torch.int32, device=DEV)
    st = ctx.stream
    assert lib.amx_split_f16x2(h, 1, F, K, Wd.data_ptr(), K, 0, W2.data_ptr(), F * 2 * K, wexp.data_ptr(), F, st) == 0
    assert lib.amx_row_exponents(h, 1, rows, K, xd.data_ptr(), K, 0, rexp.data_ptr(), rows, 1, st) == 0
    scale = float(np.float32(np.sqrt(2.0 / F)))
    outs = []
    for _ in range(2):
        phi = torch.empty(rows, F, device=DEV)
        part = torch.empty(rows // 32, F, dtype=torch.float64, device=DEV)
        assert lib.amx_rff_features_h3(h, rows, n_valid, F, K, xd.data_ptr(), K, W2.data_ptr(), wexp.data_ptr(),
                                       rexp.data_ptr(), bd.data_ptr(), ctypes.c_float(scale), phi.data_ptr(), F,
                                       part.data_ptr(), md.data_ptr(), st) == 0
        torch.cuda.synchronize()
        outs.append((phi.cpu(), part.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    phi, part = outs[0][0].double().numpy(), outs[0][1].numpy()
    xn, Wn = x.double().numpy(), W.double().numpy()
    ref = np.cos(xn @ Wn.T + b.double().numpy()) * scale
    arg = np.abs(xn) @ np.abs(Wn).T
    err = np.abs(phi - ref) / scale
    assert (err <= 4e-7 * arg + 1e-6).all(), float((err - 4e-7 * arg).max())
    valid = (mask.numpy() > 0) & (np.arange(rows) < n_valid)
    want = (phi * valid[:, None]).reshape(rows // 32, 32, F).sum(1)
    np.testing.assert_allclose(part, want, rtol=1e-12, atol=1e-12)
