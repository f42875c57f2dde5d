"""The one-launch f16x3 forward (amx_forward_h3, csrc/experimental/amx_fwd.hip; an AMX_EXPERIMENTAL=1
build) against the per-layer launches
(amx_gemm_bias_act_h3 x L + amx_gemm_out_unnorm_h3) it replaces: the same K order, limb products
and row exponents, so preds, every hidden slice of the dense rows and the row-exponent slots
must be BIT-identical, at every rows-per-workgroup it instantiates (64..128 rows: 4096, 5120,
6144, 7168 and 8192 lanes x 4 members on 256 CUs; 10 240 lanes = two CU rounds), for fp32 and
fp64 inputs; plus the oracle (BasicMLP.forward, milo/milo/dynamics.py:216-233, 422-433) at
2e-5, and lane counts the fused form does not take (the per-layer launches run)."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

pytestmark = [pytest.mark.gpu, pytest.mark.experimental]
DEV = "cuda"
S, A = 197, 36


def t32(x):
    return torch.from_numpy(np.ascontiguousarray(x)).float()


@pytest.fixture(scope="module")
def model():
    import amp_extensions_amd as amx
    from amp_extensions_amd import synthetic as syn
    s, a, s2 = syn.offline(4000, S, A, 0)
    norms = R.get_transformations(t32(s), t32(a), t32(s2))
    ens_w = R.init_ensemble_weights(S, A, [512] * 4, 4, 100)
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=DEV)
    ens = amx.DeviceEnsemble(ctx, ens_w, norms)
    yield amx, ctx, ens, ens_w, norms


def _run(ens, ob, ac, B, mode):
    ens.forward_mode = mode
    preds = ens.forward_preds(ob, ac, B).clone()
    ws = ens.workspace(B)
    torch.cuda.synchronize()
    return preds, ws["act"].clone(), ws["rexp"].clone()


# exact: the per-layer output layer runs whole-K tiles at this lane count (5120: the 80 x 224
# one-tile-per-CU tile).  At 4096 / 6144 lanes it runs stream-K (a tile's K range in 2-3 segments
# added in K order by the last arriver), whose sum of partial sums rounds differently from the
# fused form's single K chain: there preds agree to fp32 rounding (|d| <= 1e-5 of max |p|; the
# oracle bound is 2e-5) and the hidden slices / exponents stay bit-identical.
@pytest.mark.parametrize("B,dtype,exact", [(5120, torch.float64, True), (5000, torch.float32, True),
                                           (4096, torch.float32, False), (6144, torch.float64, False)])
def test_fused_forward_bit_identical(model, B, dtype, exact):
    amx, ctx, ens, ens_w, norms = model
    Bp = (B + 127) // 128 * 128
    assert ens.fused_rows(Bp) > 0, "the fused forward should take this lane count"
    rs = np.random.RandomState(B)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).to(DEV, dtype)
    ac = torch.from_numpy(rs.randn(B, A)).to(DEV, dtype)
    try:
        p_l, act_l, rexp_l = _run(ens, ob, ac, B, "layers")
        p_f, act_f, rexp_f = _run(ens, ob, ac, B, "fused")
    finally:
        ens.forward_mode = "fused"
    d = (p_f - p_l).abs().max().item()
    if exact:
        assert torch.equal(p_f, p_l), f"preds differ: max |d| {d:.3g}"
    else:
        assert d <= 1e-5 * p_l.abs().max().item(), f"preds differ: max |d| {d:.3g}"
    assert torch.equal(act_f, act_l), "hidden slices differ"
    assert torch.equal(rexp_f, rexp_l), "row-exponent slots differ"


def test_fused_forward_vs_oracle(model):
    amx, ctx, ens, ens_w, norms = model
    B = 5120
    rs = np.random.RandomState(7)
    ob = 0.5 * rs.randn(B, S)
    ac = rs.randn(B, A)
    ens.forward_mode = "fused"
    p = ens.forward_preds(torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV), B)[:, :B].cpu().numpy()
    rows = np.arange(0, B, 37)
    for m in range(4):
        ref = R.dynamics_forward(ens_w[m], norms, t32(ob[rows]), t32(ac[rows])).detach().numpy()
        scale = np.abs(ref).max()
        assert np.abs(p[m, rows] - ref).max() <= 2e-5 * scale, f"member {m}"


@pytest.mark.parametrize("B", [8192, 7168, 10240, 1000, 640, 3000])
def test_unfused_lane_counts_still_run(model, B):
    """Lane counts whose row blocks are not one CU round of 64-96-row blocks take the per-layer
    launches (fused_rows 0); the result equals the per-layer mode's exactly (it IS that path)."""
    amx, ctx, ens, ens_w, norms = model
    Bp = (B + 127) // 128 * 128
    rs = np.random.RandomState(B)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).to(DEV)
    ac = torch.from_numpy(rs.randn(B, A)).to(DEV)
    if ens.fused_rows(Bp):
        pytest.skip(f"{B} lanes are fused on this device")
    p_f = _run(ens, ob, ac, B, "fused")[0]
    p_l = _run(ens, ob, ac, B, "layers")[0]
    ens.forward_mode = "fused"
    assert torch.equal(p_f, p_l)


def test_fused_forward_rejects_bad_shapes(model):
    amx, ctx, ens, ens_w, norms = model
    assert ctx.lib.amx_forward_h3_rows(ctx.h, 4, 1024) == 0  # 256 blocks of 16: one row block per CU is < 64 rows
    assert ctx.lib.amx_forward_h3_rows(ctx.h, 4, 8192) == 0  # 128-row blocks: the per-layer launches
    assert ctx.lib.amx_forward_h3_rows(ctx.h, 4, 5120) == 80  # 256 CUs: 1280 blocks of 16 rows, 5 per CU
    ws = ens.workspace(1024)
    rc = ctx.lib.amx_forward_h3(ctx.h, 4, 1024, ctx.k0_pad, ctx.Hp, ctx.L, ws["act"].data_ptr(), ctx.ldk,
                                1024 * ctx.ldk, *ens._fw_ptrs, ctx.n_out_pad, ws["preds"].data_ptr(), S, 1024 * S,
                                ws["rexp"].data_ptr(), (ctx.L + 1) * 1024, 0, ctx.stream)
    assert rc == -1  # AMX_E_INVAL
    assert b"whole CU round" in ctx.lib.amx_last_error()


def test_fwd_weight_image(model):
    """amx_fwd_weight_image = the row-major amx_split_f16x2 image re-ordered to [g][N/16][K/32][limb]
    [lane = 32 granule + 16 half + row][8] (a permutation: every 16-B unit moved, none changed)."""
    amx, ctx, ens, ens_w, norms = model
    assert ens.W2f is not None and len(ens.W2f) == ctx.L + 1
    for w, wf in zip(ens.W2, ens.W2f):
        M, n, k2 = w.shape
        x = w.view(M, n // 16, 16, k2 // 64, 2, 2, 2, 8)  # [g][block][row][kt][granule][limb][half][8]
        ref = x.permute(0, 1, 3, 5, 4, 6, 2, 7).contiguous()  # [g][block][kt][limb][granule][half][row][8]
        assert torch.equal(wf.reshape(-1), ref.reshape(-1))
