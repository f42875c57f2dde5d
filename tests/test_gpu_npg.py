"""Device NPG policy update (amx_npg_pass / DeviceNPG) vs the reference's NPG (G11 golden,
mjrl/mjrl/algos/npg_cg.py) and vs the oracle's restatement at rollout sizes.

Tolerances (fp32 per-sample math in a different order, fp64 block reductions, fp64 CG):
  * VPG gradient and a single Fisher-vector product: |x - ref| <= 1e-4 * max|ref|
  * the 10-iteration CG solution, the updated parameters: <= 2e-3 * max|ref| (CG on a
    damping-1e-4 Fisher amplifies the last-bit differences of each HVP)
  * surr_after: rel 1e-3
"""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def close(x, ref, tol):
    x, ref = np.asarray(x, np.float64), np.asarray(ref, np.float64)
    return np.abs(x - ref).max() <= tol * np.abs(ref).max()


def make(S, A, params):
    import amp_extensions_amd as amx
    from amp_extensions_amd.npg import unpack_policy
    ctx = amx.AmxContext(S, A, n_models=1, hidden=128, n_hidden=1, device=DEV)
    layers, ls = unpack_policy(params, S, A)
    return amx.DeviceNPG(ctx, layers, ls, normalized_step_size=0.1, FIM_invert_args={"iters": 10, "damping": 1e-4},
                         min_log_std=-2.0)


def test_npg_vs_reference_golden(golden):
    g = golden("g11_npg.npz")
    S, A = 226, 28
    npg = make(S, A, g["params0"])
    obs, act = g["observations"].astype(np.float64), g["actions"]
    vpg = npg.flat_vpg(obs, act, g["adv_whitened"]).cpu().numpy()
    assert close(vpg, g["vpg"], 1e-4), np.abs(vpg - g["vpg"]).max()
    hv = npg.HVP(obs, act, g["hvp_v"]).cpu().numpy()
    assert close(hv, g["hvp"], 1e-4), np.abs(hv - g["hvp"]).max()
    out = npg.train_from_arrays(obs, act, g["advantages"])
    np.testing.assert_allclose(out["advantages"].cpu().numpy(), g["adv_whitened"], rtol=1e-12)
    assert close(out["npg_grad"].cpu().numpy(), g["npg"], 2e-3)
    assert close(npg.get_param_values() - g["params0"], g["params1"] - g["params0"], 2e-3)
    np.testing.assert_allclose(out["surr_after"], float(g["surr_after"]), rtol=1e-3)
    # the log_std clamp and the flat order: log_std is the last A entries
    assert (npg.get_param_values()[-A:] >= -2.0).all()


@pytest.mark.parametrize("S,A,N,conditioned", [(197, 36, 4096, True), (226, 28, 1000, True), (111, 8, 2048, True),
                                                (11, 3, 1000, False), (256, 64, 700, False)])
def test_npg_vs_oracle_rollout_size(S, A, N, conditioned):
    """Rollout-sized batches (ragged last block), f64 inputs as the engine holds them; every
    layer-1 depth the pass kernel is compiled for (S = 11, 111, 197, 226, 256: 1, 7, 13, 15, 16
    K-steps) and A = 3..64.  The per-product parity (VPG, Fisher-vector product) is 1e-4 of max
    at every shape.  Where 10 CG iterations on an ill-conditioned Fisher (S = 11; N = 700 samples
    for 11 456 parameters) amplify fp32 rounding of the products -- the reference's as well as
    this pass's -- past the 2e-3 solution check, the solutions are checked for direction and size."""
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    p0 = pack_policy(layers, ls)
    rs = np.random.RandomState(7)
    obs = (0.5 * rs.randn(N, S)).astype(np.float32).astype(np.float64)
    h = torch.from_numpy(obs).float()
    for i, (W, b) in enumerate(layers):
        h = torch.nn.functional.linear(h, W, b)
        h = torch.tanh(h) if i < len(layers) - 1 else h
    act = h.numpy().astype(np.float64) + np.exp(-0.25) * rs.randn(N, A)
    adv = rs.randn(N) * 1.5 + 0.2
    shapes = R.policy_param_shapes(S, A, (32, 32))
    ref = R.npg_update(p0, shapes, obs, act, adv, step=0.1, damping=1e-4, cg_iters=10, min_log_std=-2.0)
    npg = make(S, A, p0)
    vpg = npg.flat_vpg(obs, act, ref["adv_whitened"]).cpu().numpy()
    assert close(vpg, ref["vpg"], 1e-4)
    v = rs.randn(p0.size)
    hv = npg.HVP(obs, act, v).cpu().numpy()
    hv_ref = R.npg_hvp(p0, shapes, obs, act, v, 1e-4)
    assert close(hv, hv_ref, 1e-4), np.abs(hv - hv_ref).max() / np.abs(hv_ref).max()
    out = npg.train_from_arrays(obs, act, adv)
    x = out["npg_grad"].cpu().numpy()
    if conditioned:
        assert close(x, ref["npg"], 2e-3)
        assert close(npg.get_param_values() - p0, ref["params1"] - p0, 2e-3)
        np.testing.assert_allclose(out["surr_after"], ref["surr_after"], rtol=1e-3)
    else:
        # the reference's own fp32 solution is 12 % (max-relative) from the fp64 ground truth at
        # S = 11 (fp64 autograd HVP + fp64 CG, measured with this oracle): the solutions agree in
        # direction and size, not to 2e-3
        xr = ref["npg"].astype(np.float64)
        cos = np.dot(x, xr) / (np.linalg.norm(x) * np.linalg.norm(xr))
        assert cos > 0.98 and abs(np.linalg.norm(x) / np.linalg.norm(xr) - 1) < 0.1, (cos, np.linalg.norm(x),
                                                                                       np.linalg.norm(xr))


def test_npg_engine_path_refreshes_policy():
    """train_from_engine on the rollout buffers updates the device sampler's policy."""
    import amp_extensions_amd as amx
    from amp_extensions_amd import synthetic as syn
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.ensemble import init_ensemble_weights
    S, A = 197, 36
    s, a, s2 = syn.offline(2048, S, A, 0)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    ctx = amx.AmxContext(S, A, n_models=4, hidden=128, n_hidden=2, device=DEV)
    ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [128] * 2, 4, 100), norms)
    layers, ls = init_mlp_policy_params(S, A)
    pol = amx.DevicePolicy(ctx, layers, ls, seed=3)
    eng = amx.RolloutEngine(ens, syn.reset_table(512, S, 1), lanes=256, policy=pol, seed=5, max_steps=4)
    eng.reset_all()
    eng.rollout()
    adv = torch.randn(4, 256, dtype=torch.float64, device=DEV)
    npg = amx.DeviceNPG(ctx, layers, ls, normalized_step_size=0.1, min_log_std=-2.0, policy=pol)
    blob0 = pol.blob.clone()
    out = npg.train_from_engine(eng, adv)
    assert np.isfinite(out["alpha"]) and out["kl_dist"] > 0
    # the KL of the step is about half the normalized step size (2 * kl_dist = 0.1)
    assert 0.01 < out["kl_dist"] < 0.2
    assert not torch.equal(blob0, pol.blob)


def test_npg_device_cg_early_stop():
    """amx_npg_cg_step's device-side `live` flag is cg_solve's break (mjrl/mjrl/utils/cg_solve.py:
    9-21): with a residual_tol the solve reaches after 3 of 10 iterations, the device solve returns
    the reference loop's x, the loop run in fp64 numpy with the device HVP as f_Ax."""
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy
    S, A, N = 197, 36, 2048
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    p0 = pack_policy(layers, ls)
    rs = np.random.RandomState(3)
    obs = (0.5 * rs.randn(N, S)).astype(np.float32)
    act = rs.randn(N, A).astype(np.float32)
    adv = rs.randn(N)
    npg = make(S, A, p0)
    b = npg.flat_vpg(obs, act, adv).cpu().numpy()

    def cg_ref(tol):
        x, r = np.zeros_like(b), b.copy()
        p, rdotr, hist = r.copy(), r @ r, []
        for _ in range(10):
            z = npg.HVP(obs, act, p).cpu().numpy()
            v = rdotr / (p @ z)
            x += v * p
            r -= v * z
            newrdotr = r @ r
            mu = newrdotr / rdotr
            p = r + mu * p
            rdotr = newrdotr
            hist.append(rdotr)
            if rdotr < tol:
                break
        return x, hist

    _, hist = cg_ref(0.0)
    assert len(hist) == 10 and hist[2] < hist[1]
    tol = float(np.sqrt(hist[2] * hist[1]))  # reached at iteration 3
    x_ref, hist3 = cg_ref(tol)
    assert len(hist3) == 3
    o, a, _ = npg._inputs(obs, act)
    npg.residual_tol = tol
    x_dev = npg.cg_solve(o, a, torch.from_numpy(b).to(DEV)).cpu().numpy()
    assert close(x_dev, x_ref, 1e-7), np.abs(x_dev - x_ref).max()
    npg.residual_tol = 0.0
    x10 = npg.cg_solve(o, a, torch.from_numpy(b).to(DEV)).cpu().numpy()
    assert not close(x10, x_ref, 1e-7)  # the stop mattered


def test_npg_gated_fvp_pass_skips_after_stop():
    """amx_npg_pass_gated / amx_npg_reduce_gated (the FVP products of cg_solve): with the CG
    state's live flag 1 they equal the ungated pass bit for bit; with live 0 (the solve stopped,
    cg_solve.py:19-20) neither the partials nor the output are written."""
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy, NPG_FVP
    S, A, N = 197, 36, 1024
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    npg = make(S, A, pack_policy(layers, ls))
    rs = np.random.RandomState(5)
    o, a, _ = npg._inputs((0.5 * rs.randn(N, S)).astype(np.float32), rs.randn(N, A).astype(np.float32))
    vec = torch.from_numpy(rs.randn(npg.P).astype(np.float32)).to(DEV)
    h0 = npg._pass(NPG_FVP, o, a, None, vec)
    live = torch.tensor([1.0, 1.0], dtype=torch.float64, device=DEV)
    h1 = npg._pass(NPG_FVP, o, a, None, vec, gate=live)
    assert torch.equal(h0, h1)
    c, lib = npg.ctx, npg.ctx.lib
    rpb = npg._rows_per_block(N)
    nb = (N + rpb - 1) // rpb
    part = torch.full((nb, npg.P), 7.0, dtype=torch.float64, device=DEV)
    out = torch.full((npg.P,), 9.0, dtype=torch.float64, device=DEV)
    dead = torch.tensor([1.0, 0.0], dtype=torch.float64, device=DEV)
    assert lib.amx_npg_pass_gated(c.h, NPG_FVP, N, o.data_ptr(), 1, o.stride(0), a.data_ptr(), 1, a.stride(0), None,
                                  npg.theta.data_ptr(), vec.data_ptr(), rpb, part.data_ptr(), dead.data_ptr(),
                                  c.stream) == 0
    assert lib.amx_npg_reduce_gated(c.h, part.data_ptr(), nb, npg.P, out.data_ptr(), dead.data_ptr(), c.stream) == 0
    torch.cuda.synchronize()
    assert bool((part == 7.0).all()) and bool((out == 9.0).all())


@pytest.mark.parametrize("N", [2048, 1000])
def test_npg_fvp_theta_cache_bit_identical(N):
    """amx_npg_pass_ex: the VPG pass writes the policy's forward at theta (H1 | H2 per sample) and
    the Fisher-vector pass that reads it (layers 1-2 at theta skipped, the tangent's chains dealt
    over all eight waves) gives the uncached pass's partials bit for bit -- N = 1000 leaves a
    ragged last chunk; the VPG result is unchanged by writing the cache."""
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy, NPG_FVP, NPG_VPG
    S, A = 197, 36
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    npg = make(S, A, pack_policy(layers, ls))
    rs = np.random.RandomState(7)
    o, a, adv = npg._inputs((0.5 * rs.randn(N, S)).astype(np.float32), rs.randn(N, A).astype(np.float32),
                            rs.randn(N))
    hc = torch.full((N, 64), float("nan"), dtype=torch.float32, device=DEV)
    v0 = npg._pass(NPG_VPG, o, a, adv, None).clone()
    v1 = npg._pass(NPG_VPG, o, a, adv, None, hcache=hc).clone()
    assert torch.equal(v0, v1)
    assert not torch.isnan(hc).any()
    for seed in (1, 2):
        vec = torch.from_numpy(np.random.RandomState(seed).randn(npg.P).astype(np.float32)).to(DEV)
        h0 = npg._pass(NPG_FVP, o, a, None, vec).clone()
        h1 = npg._pass(NPG_FVP, o, a, None, vec, hcache=hc).clone()
        assert torch.equal(h0, h1), float((h0 - h1).abs().max())


def test_npg_cg_tail_matches_separate():
    """amx_npg_cg_tail (the FVP partials' column sums + the CG vector step in two launches spread
    over the chip) against amx_npg_reduce + amx_npg_cg_step from the same state, three iterations:
    the same h (the reduction's order is kept), p.z and r.r summed from fixed-order block parts
    instead of the 1024-thread tree -- x, r, p within 1e-12 of the scale; a second solve from the
    same start reproduces the first bit for bit (deterministic: every block forms the same v and
    r.r); a stopped solve (tol above r.r) carries the stop over and leaves x, r, p untouched."""
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy, NPG_FVP
    S, A, N = 197, 36, 3000
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    npg = make(S, A, pack_policy(layers, ls))
    rs = np.random.RandomState(11)
    o, a, _ = npg._inputs((0.5 * rs.randn(N, S)).astype(np.float32), rs.randn(N, A).astype(np.float32))
    c, lib, P = npg.ctx, npg.ctx.lib, npg.P
    b = torch.from_numpy(rs.randn(P)).to(DEV)
    curv = npg._ls_curvature()
    work = torch.empty(int(lib.amx_npg_cg_tail_work(P)), dtype=torch.float64, device=DEV)

    def solve(fused, iters=3, tol=0.0):
        x, r, p, r2 = (torch.empty(P, dtype=torch.float64, device=DEV) for _ in range(4))
        p32 = torch.empty(P, dtype=torch.float32, device=DEV)
        st, st2 = (torch.empty(2, dtype=torch.float64, device=DEV) for _ in range(2))
        assert lib.amx_npg_cg_init(c.h, P, b.data_ptr(), x.data_ptr(), r.data_ptr(), p.data_ptr(), p32.data_ptr(),
                                   st.data_ptr(), c.stream) == 0
        for _ in range(iters):
            if fused:
                part = npg._pass(NPG_FVP, o, a, None, p32, gate=st, reduce=False)
                assert lib.amx_npg_cg_tail(c.h, part.data_ptr(), part.shape[0], P, A, curv.data_ptr(), npg.damping,
                                           tol, x.data_ptr(), r.data_ptr(), r2.data_ptr(), p.data_ptr(),
                                           p32.data_ptr(), st.data_ptr(), st2.data_ptr(), work.data_ptr(),
                                           c.stream) == 0
                r, r2, st, st2 = r2, r, st2, st
            else:
                h = npg._pass(NPG_FVP, o, a, None, p32, gate=st)
                assert lib.amx_npg_cg_step(c.h, P, A, h.data_ptr(), curv.data_ptr(), npg.damping, tol, x.data_ptr(),
                                           r.data_ptr(), p.data_ptr(), p32.data_ptr(), st.data_ptr(), c.stream) == 0
        torch.cuda.synchronize()
        return [t.cpu().double().numpy() for t in (x, r, p, st)]

    sep, fus, fus2 = solve(False), solve(True), solve(True)
    for u, v in zip(sep[:3], fus[:3]):
        assert close(v, u, 1e-12), np.abs(u - v).max()
    assert sep[3][1] == fus[3][1] and close(fus[3][:1], sep[3][:1], 1e-12)
    for u, v in zip(fus, fus2):
        assert np.array_equal(u, v)
    # early stop: with tol above the first r.r the first tail stops the solve; the later
    # iterations (gated FVP passes, tails that only carry the state) change nothing
    one = solve(True, iters=1, tol=1e300)
    four = solve(True, iters=4, tol=1e300)
    assert one[3][1] == 0.0 and four[3][1] == 0.0
    for u, v in zip(one[:3], four[:3]):
        assert np.array_equal(u, v)


@pytest.mark.parametrize("iters,stop_at,cache", [(1, None, True), (2, None, False), (10, None, True),
                                                 (10, 3, True), (4, 1, False)])
def test_npg_cg_fold_bit_identical(iters, stop_at, cache):
    """amx_npg_pass_cg (the CG vector step folded into the next Fisher-vector pass, one launch per
    iteration fewer) against the round-5 form (pass on p32 + amx_npg_cg_tail): the same x bit for
    bit -- the fold forms v, r'.r' and p' in k_npg_cg_xrp's summation orders -- over 1, 2 and 10
    iterations, with the theta cache and without it (fp64 observations: the uncached pass), and
    with the solve stopping at iteration 1 or 3 (residual_tol between two r.r values: the stop
    found by the fold itself, then carried through the later passes and the final step)."""
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy, NPG_VPG
    S, A, N = 197, 36, 3000
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    npg = make(S, A, pack_policy(layers, ls))
    npg.cg_iters = iters
    rs = np.random.RandomState(13)
    o, a, adv = npg._inputs((0.5 * rs.randn(N, S)).astype(np.float32), rs.randn(N, A).astype(np.float32),
                            rs.randn(N))
    hc = None
    if cache:
        hc = npg._hcache(N)
        b = npg._pass(NPG_VPG, o, a, adv, None, hcache=hc).clone()
    else:
        o = o.double()
        b = npg._pass(NPG_VPG, o, a, adv, None).clone()

    def solve(fold, tol):
        npg.cg_fold, npg.residual_tol = fold, tol
        x = npg.cg_solve(o, a, b, hcache=hc).clone()
        torch.cuda.synchronize()
        return x.cpu().numpy()

    tol = 0.0
    if stop_at is not None:  # r.r after each step from a numpy CG with the device HVP as f_Ax
        bn = b.cpu().numpy()
        x_, r_, p_ = np.zeros_like(bn), bn.copy(), bn.copy()
        hist = [float(bn @ bn)]
        for _ in range(stop_at):
            z = npg.HVP(o, a, p_).cpu().numpy()
            v = hist[-1] / (p_ @ z)
            r_ = r_ - v * z
            nr = float(r_ @ r_)
            p_ = r_ + nr / hist[-1] * p_
            hist.append(nr)
        tol = float(np.sqrt(hist[-1] * hist[-2]))  # reached at step `stop_at`, not before
    x0 = solve(False, tol)
    x1 = solve(True, tol)
    assert np.array_equal(x0, x1), np.abs(x0 - x1).max()
    assert np.array_equal(x1, solve(True, tol))
    if stop_at is not None:
        npg.cg_iters = stop_at
        assert np.array_equal(x1, solve(False, 0.0))  # the stop took effect after `stop_at` steps


def test_npg_pass_input_dtypes_bit_identical():
    """amx_npg_pass on fp64 and fp32 inputs (the fp64 C-ABI path: 16 layer-1 K-steps compiled; the
    fp32 path DeviceNPG takes: ceil(S / 16) rounded to 4 / 8 / 13 / 16) gives the same bits in all
    three modes -- the kernels read float32(obs) either way and the extra K-steps add exact zeros."""
    from amp_extensions_amd import npg as NP
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy
    S, A, N = 197, 36, 2000
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=5, init_log_std=-0.4)
    p0 = pack_policy(layers, ls)
    npg = make(S, A, p0)
    rs = np.random.RandomState(11)
    obs64 = torch.from_numpy(0.5 * rs.randn(N, S)).to(DEV)
    act64 = torch.from_numpy(rs.randn(N, A)).to(DEV)
    adv = torch.from_numpy(rs.randn(N)).to(DEV)
    vec = torch.from_numpy(rs.randn(npg.P).astype(np.float32)).to(DEV)
    newp = (npg.theta + 0.01 * vec).contiguous()
    for mode, v in ((NP.NPG_VPG, None), (NP.NPG_FVP, vec), (NP.NPG_EVAL, newp)):
        a64 = npg._pass(mode, obs64, act64, adv, v).cpu().numpy()
        a32 = npg._pass(mode, obs64.float().contiguous(), act64.float().contiguous(), adv, v).cpu().numpy()
        np.testing.assert_array_equal(a64, a32)


def test_npg_cg_init_ls_matches_separate():
    """amx_npg_cg_init_ls (the CG start + the log_std curvature in one launch) writes the same
    bits as amx_npg_cg_init followed by amx_npg_curvature."""
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd.npg import pack_policy
    S, A = 197, 36
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=7, init_log_std=-0.4)
    npg = make(S, A, pack_policy(layers, ls))
    c, lib, P = npg.ctx, npg.ctx.lib, npg.P
    b = torch.from_numpy(np.random.RandomState(3).randn(P)).to(DEV)
    outs = []
    for fused in (False, True):
        x, r, p = (torch.full((P,), 7.0, dtype=torch.float64, device=DEV) for _ in range(3))
        p32 = torch.empty(P, dtype=torch.float32, device=DEV)
        st = torch.empty(2, dtype=torch.float64, device=DEV)
        if fused:
            curv = torch.empty(A, dtype=torch.float64, device=DEV)
            assert lib.amx_npg_cg_init_ls(c.h, P, A, npg.theta.data_ptr(), curv.data_ptr(), b.data_ptr(),
                                          x.data_ptr(), r.data_ptr(), p.data_ptr(), p32.data_ptr(), st.data_ptr(),
                                          c.stream) == 0
        else:
            assert lib.amx_npg_cg_init(c.h, P, b.data_ptr(), x.data_ptr(), r.data_ptr(), p.data_ptr(),
                                       p32.data_ptr(), st.data_ptr(), c.stream) == 0
            curv = npg._ls_curvature()
        torch.cuda.synchronize()
        outs.append([t.cpu().double().numpy() for t in (x, r, p, p32, st, curv)])
    for u, v in zip(*outs):
        assert np.array_equal(u, v)
