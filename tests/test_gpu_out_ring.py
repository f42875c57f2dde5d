"""The output layer's LDS-DMA ring tile (amx_set_out_tile 2/3: k_gemm_ring, an A/B option:
DESIGN §6) against the register-staged tiles (the default) on the same f16x3 forward: every lane count the engine
and the strong-scaling shares use -- one tile per workgroup, stream-K (4096-7168 lanes, K
segments combined in K order), the row-block shapes and small partial grids -- and the scene
layout S = 226 (15 column blocks).  The ring issues the same three limb products per 16 x 16
block and K-tile in the same order, over the same K segments, so the predictions are
bit-identical (at 5120 lanes, where the default is the 80 x 224 one-tile-per-CU tile and the
ring keeps the stream-K segments, equal to fp32 rounding); and against the oracle's fp64-accumulated forward at rel 2e-5 of the scale.
Reference: milo/milo/dynamics.py:216-233, 422-433 (BasicMLP output layer + un-normalisation)."""
import numpy as np
import pytest
import torch

from oracle import milo_ref as R

# experimental A/B path: runs against an AMX_EXPERIMENTAL=1 build, skipped on the shipped library
pytestmark = [pytest.mark.gpu, pytest.mark.experimental]
DEV = "cuda"


def _ensemble(S, A):
    import amp_extensions_amd as amx
    rs = np.random.RandomState(S)
    s = 0.5 * rs.randn(4096, S)
    a = rs.randn(4096, A)
    s2 = s + 0.01 * rs.randn(4096, S)
    norms = R.get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
    w = R.init_ensemble_weights(S, A, [512] * 4, 4, 100)
    ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=DEV)
    return ctx, amx.DeviceEnsemble(ctx, w, norms), w, norms


@pytest.mark.parametrize("S,A,lanes", [(197, 36, 8192), (197, 36, 5120), (197, 36, 4096), (197, 36, 7168),
                                       (197, 36, 6144), (197, 36, 1000), (197, 36, 128), (197, 36, 10240),
                                       (226, 28, 8192), (226, 28, 300)])
def test_ring_output_layer_bit_identical(S, A, lanes):
    ctx, ens, _, _ = _ensemble(S, A)
    rs = np.random.RandomState(lanes)
    ob = torch.from_numpy(0.5 * rs.randn(lanes, S)).to(DEV)
    ac = torch.from_numpy(rs.randn(lanes, A)).to(DEV)
    outs = {}
    for tile in (0, 2, 3):
        ctx.set_out_tile(tile)
        outs[tile] = ens.forward_preds(ob, ac, lanes).clone()
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0][:, :lanes]).all()
    rows = 4 * ((lanes + 127) // 128 * 128)
    if S == 197 and rows % 80 == 0 and rows // 80 == torch.cuda.get_device_properties(0).multi_processor_count:
        # the default is the 80 x 224 one-tile-per-CU output tile here (one K chain per element),
        # the ring tiles keep the stream-K segments: equal to fp32 rounding of the K split
        for t in (2, 3):
            d = (outs[t][:, :lanes] - outs[0][:, :lanes]).abs() / outs[0][:, :lanes].abs().clamp_min(1.0)
            assert float(d.max()) < 2e-6, (t, float(d.max()))
    else:
        assert torch.equal(outs[2][:, :lanes], outs[0][:, :lanes]), "ring 16-row waves differ from the staged tile"
        assert torch.equal(outs[3][:, :lanes], outs[0][:, :lanes]), "ring 32x112 differs from the staged tile"
    # repeated launches of the ring (its DMA ring and stream-K counters) give the same bits
    ctx.set_out_tile(2)
    again = ens.forward_preds(ob, ac, lanes)
    assert torch.equal(again[:, :lanes], outs[2][:, :lanes])


@pytest.mark.parametrize("lanes", [8192, 5120])
def test_ring_output_layer_matches_oracle(lanes):
    S, A = 197, 36
    ctx, ens, w, norms = _ensemble(S, A)
    ctx.set_out_tile(2)
    rs = np.random.RandomState(7)
    ob = 0.5 * rs.randn(lanes, S)
    ac = rs.randn(lanes, A)
    preds = ens.forward_preds(torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV), lanes)
    got = preds[:, :lanes].cpu().numpy()
    idx = np.arange(0, lanes, 61)  # a strided subset through the oracle's torch-CPU fp32 forward
    ref = R.ensemble_preds(w, norms, torch.from_numpy(ob[idx]).float(), torch.from_numpy(ac[idx]).float()).numpy()
    scale = np.maximum(1.0, np.abs(ref).max(axis=2, keepdims=True))
    assert np.max(np.abs(got[:, idx] - ref) / scale) < 2e-5


@pytest.mark.parametrize("lanes", [8192, 7168, 5120, 4096, 1000])
def test_out_tile4_streamk_256(lanes):
    """amx_set_out_tile 4: 256 x 224 output tiles, K-tiles dealt over the CUs (stream-K, segments
    summed in K order by the last arriver).  Its K segments differ from the one-tile-per-workgroup
    staged tile's single chain, so it matches it (and the oracle) to fp32 rounding, not bit for
    bit; repeated launches are bit-identical (deterministic combine, self-resetting counters)."""
    S, A = 197, 36
    ctx, ens, w, norms = _ensemble(S, A)
    rs = np.random.RandomState(lanes + 3)
    ob = 0.5 * rs.randn(lanes, S)
    ac = rs.randn(lanes, A)
    obt, act = torch.from_numpy(ob).to(DEV), torch.from_numpy(ac).to(DEV)
    ctx.set_out_tile(1)
    staged = ens.forward_preds(obt, act, lanes)[:, :lanes].clone()
    ctx.set_out_tile(4)
    got = ens.forward_preds(obt, act, lanes)[:, :lanes].clone()
    again = ens.forward_preds(obt, act, lanes)[:, :lanes]
    assert torch.equal(again, got), "256 x 224 stream-K is not deterministic"
    scale = torch.clamp(staged.abs().amax(dim=2, keepdim=True), min=1.0)
    assert ((got - staged).abs() / scale).max().item() < 2e-6
    idx = np.arange(0, lanes, 61)
    ref = R.ensemble_preds(w, norms, torch.from_numpy(ob[idx]).float(), torch.from_numpy(ac[idx]).float()).numpy()
    g = got.cpu().numpy()[:, idx]
    sc = np.maximum(1.0, np.abs(ref).max(axis=2, keepdims=True))
    assert np.max(np.abs(g - ref) / sc) < 2e-5
