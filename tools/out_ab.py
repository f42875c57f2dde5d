"""Output-layer tile A/B (amx_set_out_tile): one f16x3 ensemble forward (assembly + 4 hidden
layers + output layer) at B lanes with the register-staged tiles (1), the LDS-DMA ring with
16-row waves (2) and with 32 x 112 waves (3); HIP-event medians over 30 forwards, rounds
alternating in one process.  usage: python tools/out_ab.py [B ...]"""
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
    for rnd in range(3):
        res = {}
        for tile in (1, 2, 3):
            ctx.set_out_tile(tile)
            res[tile] = timed(ob, ac, B)
        print(f"lanes {B} round {rnd}: forward staged {res[1]:.1f} us, ring16 {res[2]:.1f} us, ring32x112 "
              f"{res[3]:.1f} us", flush=True)
