"""Output-layer tile A/B (amx_set_out_tile): one f16x3 ensemble forward (assembly + 4 hidden
layers + output layer) at B lanes with the register-staged tiles (1), the LDS-DMA ring with
16-row waves (2), with 32 x 112 waves (3) and the 256 x 224 stream-K tile (4); HIP-event medians
over 30 forwards, rounds alternating in one process.
usage: [OUT_TILES=1,4] python tools/out_ab.py [B ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402

lanes = [int(x) for x in sys.argv[1:]] or [8192, 5120]
S, A = 197, 36
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*(torch.from_numpy(x).float() for x in (s, a, s2)))
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, base_seed=100), norms)


def timed(ob, ac, B, n=30):
    for _ in range(5):
        ens.forward_preds(ob, ac, B)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for e0, e1 in ev:
        e0.record()
        ens.forward_preds(ob, ac, B)
        e1.record()
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]))


for B in lanes:
    rs = np.random.RandomState(1)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
    ac = torch.from_numpy(rs.randn(B, A)).cuda()
    tiles = [int(x) for x in os.environ.get("OUT_TILES", "1,2,3,4").split(",")]
    names = {1: "staged", 2: "ring16", 3: "ring32x112", 4: "256x224-streamK"}
    for rnd in range(3):
        res = {}
        for tile in tiles:
            ctx.set_out_tile(tile)
            res[tile] = timed(ob, ac, B)
        print(f"lanes {B} round {rnd}: forward " + ", ".join(f"{names[t]} {res[t]:.1f} us" for t in tiles),
              flush=True)
    ctx.set_out_tile(1)
    ref = ens.forward_preds(ob, ac, B).clone()
    for tile in tiles:
        ctx.set_out_tile(tile)
        d = (ens.forward_preds(ob, ac, B) - ref)[:, :B].abs().max().item()
        print(f"lanes {B}: tile {tile} max |diff| vs staged {d:.3e}", flush=True)
