"""The limb-format ensemble forward (amx_assemble_input_limbs + amx_gemm_*_lb, DeviceEnsemble
act_format='limbs'): activations stored as scaled fp16 limb pairs with one exponent per row and
128-column chunk, split once by their producer; the consumers' K loops copy bytes (LDS-DMA) and
rescale the fp32 accumulators at chunk boundaries.  Parity with the oracle's fp32 forward
(dynamics.py:216-233, 422-433) at the f32 path's tolerance and within 1e-6 of the native f32
MFMA path, on every tile regime; the stored limbs decode to the f32-format path's activations;
chunks that are all zero or 2^70 below the row's other chunks (the accumulator's clamped
rescale) stay at fp32-level error against an fp64 forward."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

# experimental A/B path: runs against an AMX_EXPERIMENTAL=1 build, skipped on the shipped library
pytestmark = [pytest.mark.gpu, pytest.mark.experimental]
DEV = "cuda"


def offline(n, seed, S, A):
    rs = np.random.RandomState(seed)
    s = 0.5 * rs.randn(n, S)
    s[:, 0] = rs.uniform(0.8, 0.95, n)
    a = rs.randn(n, A)
    s2 = s + 0.01 * rs.randn(n, S)
    return s, a, s2


def make(S, A, hidden, ens_w=None, M=4):
    import amp_extensions_amd as amx
    s, a, s2 = offline(2048, 0, S, A)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    if ens_w is None:
        ens_w = R.init_ensemble_weights(S, A, hidden, M, 100)
    ctx = amx.AmxContext(S, A, n_models=M, hidden=hidden[0], n_hidden=len(hidden), feat_dim=512, device=DEV)
    ens = {"lb": amx.DeviceEnsemble(ctx, ens_w, norms, act_format="limbs"),
           "h3": amx.DeviceEnsemble(ctx, ens_w, norms, act_format="f32"),
           "f32": amx.DeviceEnsemble(ctx, ens_w, norms, gemm="f32")}
    assert ens["lb"].limbs and not ens["h3"].limbs
    return amx, ctx, ens, ens_w, norms


def inputs(B, S, A, seed=1):
    rs = np.random.RandomState(seed)
    ob = 0.5 * rs.randn(B, S)
    ob[:, 0] = rs.uniform(0.8, 0.95, B)
    return ob, rs.randn(B, A)


def f64_forward(ens_w, norms, ob, ac):
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


@pytest.mark.parametrize("S,A,hidden,B", [(197, 36, [512] * 4, 8192), (197, 36, [512] * 4, 640),
                                          (197, 36, [512] * 4, 5120), (197, 36, [512] * 4, 7168),
                                          (197, 36, [512] * 4, 4096), (197, 36, [512] * 4, 2048),
                                          (226, 28, [512] * 4, 1024), (100, 20, [256] * 3, 640),
                                          (300, 40, [256] * 2, 384), (11, 3, [256] * 2, 256)])
def test_lb_forward_matches_oracle_and_f32(S, A, hidden, B):
    """Tile regimes: 8192 lanes -> 256 x 256 hidden tiles, 128 x 224 output tiles; 4096-7168 ->
    row-block hidden tiles (128-224 rows), stream-K output; 640 / 2048 -> stream-K hidden (few
    tiles) and output; S = 226 -> 128 x 256 output tiles; S = 100 -> 128; S = 300 -> two 256-wide
    tiles... (round_up(300, 128) = 384: three 128-wide); k0 = 32 (S + A = 14)."""
    amx, ctx, ens, ens_w, norms = make(S, A, hidden)
    ob, ac = inputs(B, S, A)
    obd, acd = torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV)
    p = {k: e.forward_preds(obd, acd, B)[:, :B].cpu().numpy().astype(np.float64) for k, e in ens.items()}
    n = min(B, 1024)
    ref = R.ensemble_preds(ens_w, norms, torch.from_numpy(ob[:n]).float(), torch.from_numpy(ac[:n]).float()).numpy()
    scale = max(1.0, np.abs(ref).max())
    assert np.abs(p["lb"][:, :n] - ref).max() / scale <= 2e-5
    assert np.abs(p["lb"] - p["f32"]).max() / max(1.0, np.abs(p["f32"]).max()) <= 1e-6
    assert np.abs(p["lb"] - p["h3"]).max() / max(1.0, np.abs(p["h3"]).max()) <= 1e-6
    again = ens["lb"].forward_preds(obd, acd, B)[:, :B].cpu().numpy().astype(np.float64)
    np.testing.assert_array_equal(again, p["lb"])  # deterministic (stream-K sums in K order)


def _decode(act_row_words, exps, k0, chunk=128):
    """fp32 values of limb-format rows: [rows, ldk] u32 words -> [rows, ldk] float64."""
    rows, ldk = act_row_words.shape
    h = act_row_words.view(np.float16).reshape(rows, ldk // 16, 2, 16).astype(np.float64)
    v = (h[:, :, 0] + h[:, :, 1]).reshape(rows, ldk)
    col_slot = np.concatenate([np.zeros(k0, np.int64), 1 + np.arange(ldk - k0) // chunk])
    return v * np.exp2(exps[col_slot, :].T.astype(np.float64) - 14.0)


def test_lb_limbs_decode_to_the_f32_activations():
    """The stored rows: x0 and every hidden slice decode ((limb0 + limb1) 2^(E - 14)) to the
    f32-format path's fp32 activations within 2^-21 of each chunk's max; each chunk's exponent
    is that of its max |value| (2^(E-1) <= max < 2^E, all-zero chunks -100)."""
    S, A, B = 197, 36, 512
    amx, ctx, ens, ens_w, norms = make(S, A, [512] * 4)
    ob, ac = inputs(B, S, A, 4)
    obd, acd = torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV)
    ens["h3"].shared_x0 = ens["lb"].shared_x0 = False  # every member's x0 copy written
    ens["h3"].forward_preds(obd, acd, B)
    ens["lb"].forward_preds(obd, acd, B)
    torch.cuda.synchronize()
    ref = ens["h3"].workspace(B)["act"].cpu().numpy()[:, :B].astype(np.float64)
    ws = ens["lb"].workspace(B)
    words = ws["act"].cpu().numpy()[:, :B].view(np.uint32)
    rexp = ws["rexp"].cpu().numpy()[:, :, :B]
    k0 = ctx.k0_pad
    for m in range(4):
        got = _decode(words[m], rexp[m], k0)
        bounds = [(0, k0)] + [(k0 + 128 * c, k0 + 128 * (c + 1)) for c in range((ctx.ldk - k0) // 128)]
        for c, (lo, hi) in enumerate(bounds):
            mx = np.abs(ref[m, :, lo:hi]).max(axis=1)
            err = np.abs(got[:, lo:hi] - ref[m, :, lo:hi]).max(axis=1)
            tol = np.maximum(mx, 1e-30) * 2.0 ** -21 + 1e-6 * np.abs(ref[m, :, lo:hi]).max(axis=1)
            assert (err <= tol).all(), (m, c, float((err / np.maximum(mx, 1e-30)).max()))
            E = rexp[m, c]
            nz = mx > 0
            assert (E[~nz] == -100).all()
            assert (mx[nz] < np.exp2(E[nz])).all() and (mx[nz] >= np.exp2(E[nz] - 1.0) * (1 - 1e-6)).all()


def test_lb_zero_and_tiny_chunks():
    """Hidden chunks that are all zero (weights and biases of a 128-unit block zeroed: E = -100,
    an accumulator rescale of up to 2^60 with nothing to scale) or 2^70 below the row's other
    chunks (block scaled by 2^-70: the clamped rescale) next to ordinary ones: fp32-level error
    against an fp64 forward, no worse than the native f32 path's, finite everywhere."""
    S, A, B = 197, 36, 512
    ens_w = R.init_ensemble_weights(S, A, [512] * 4, 4, 100)
    for m in range(4):
        W, b = ens_w[m][0]
        W[128:256] = 0.0
        b[128:256] = 0.0
        W, b = ens_w[m][1]
        W[256:384] *= 2.0 ** -70
        b[256:384] *= 2.0 ** -70
    amx, ctx, ens, _, norms = make(S, A, [512] * 4, ens_w=ens_w)
    ob, ac = inputs(B, S, A, 6)
    obd, acd = torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV)
    ref = f64_forward(ens_w, norms, ob, ac)
    scale = np.maximum(1.0, np.abs(ref).max(axis=-1, keepdims=True))
    plb = ens["lb"].forward_preds(obd, acd, B)[:, :B].cpu().numpy().astype(np.float64)
    p32 = ens["f32"].forward_preds(obd, acd, B)[:, :B].cpu().numpy().astype(np.float64)
    assert np.isfinite(plb).all()
    elb, e32 = (np.abs(plb - ref) / scale).max(), (np.abs(p32 - ref) / scale).max()
    assert elb <= 2e-5 and elb <= 2.0 * e32 + 1e-6, (elb, e32)
    rexp = ens["lb"].workspace(B)["rexp"].cpu().numpy()[:, :, :B]
    assert (rexp[:, 1 + 1] == -100).all()  # h0 columns 128..255: chunk slot 2


def test_lb_graph_replay_and_timer():
    """A captured forward replays bit-identically, and the in-kernel GEMM timer counts one
    forward per eager forward (first hidden layer's start stamp, output layer's tick sum)."""
    S, A, B = 197, 36, 5120
    amx, ctx, ens, ens_w, norms = make(S, A, [512] * 4)
    e = ens["lb"]
    ob, ac = inputs(B, S, A, 8)
    obd, acd = torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV)
    ref = e.forward_preds(obd, acd, B).clone()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            e.forward_preds(obd, acd, B)
    torch.cuda.synchronize()
    e.workspace(B)["preds"].zero_()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(e.workspace(B)["preds"], ref)
    timer = ctx.gemm_timer()
    for _ in range(2):
        e.forward_preds(obd, acd, B)
    torch.cuda.synchronize()
    tv = timer.cpu().numpy()
    assert tv[3] == 2 and tv[1] == 0 and 0 < tv[2] < 2 * 100000
    ctx.gemm_timer(False)


def test_lb_abi_checks():
    import amp_extensions_amd as amx
    ctx = amx.AmxContext(197, 36, n_models=4, hidden=512, n_hidden=4, device=DEV)
    lib, s = ctx.lib, ctx.stream
    buf = torch.zeros(4, 256, ctx.ldk, dtype=torch.float32, device=DEV)
    W2 = torch.zeros(4, 512, 2 * ctx.ldk, dtype=torch.int16, device=DEV)
    we = torch.zeros(4, 512, dtype=torch.int32, device=DEV)
    b = torch.zeros(4, 512, dtype=torch.float32, device=DEV)
    rx = torch.zeros(4, 17, 256, dtype=torch.int32, device=DEV)
    k0 = ctx.k0_pad
    args = lambda K, col_off, k0_, out: (ctx.h, 4, 256, 512, K, buf.data_ptr(), ctx.ldk, 256 * ctx.ldk, W2.data_ptr(),
                                         512 * 2 * K, we.data_ptr(), 512, b.data_ptr(), 512, buf.data_ptr(), ctx.ldk,
                                         256 * ctx.ldk, col_off, 1, rx.data_ptr(), 17 * 256, 256, out, k0_, 0, s)
    assert lib.amx_gemm_bias_act_lb(*args(k0 + 64, k0 + 64, k0, rx.data_ptr())) == -1
    assert b"multiple of 128" in lib.amx_last_error()
    assert lib.amx_gemm_bias_act_lb(*args(k0, k0, k0, None)) == -1
    assert b"row_exp_out" in lib.amx_last_error()
    assert lib.amx_gemm_bias_act_lb(*args(k0, k0 + 128, 48, rx.data_ptr())) == -1
