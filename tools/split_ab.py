"""Output-layer split-K A/B: one f16x3 ensemble forward at B lanes with the split workspace
registered (the 5120-lane output layer as 3 K-slices of 128 x 224 tiles) and without it (the
160 x 112 row-block tiles), HIP-event medians over 30 forwards, same process.
usage: python tools/split_ab.py [B]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 5120
S, A = 197, 36
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*(torch.from_numpy(x).float() for x in (s, a, s2)))
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, base_seed=100), norms)
rs = np.random.RandomState(1)
ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
ac = torch.from_numpy(rs.randn(B, A)).cuda()
ens.forward_preds(ob, ac, B)
ws = getattr(ctx, "_split_ws", None)


def timed(n=30):
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


for rnd in range(3):
    ctx.lib.amx_set_split_workspace(ctx.h, None, 0, None, 0)
    t0 = timed()
    if ws is not None:
        ctx.lib.amx_set_split_workspace(ctx.h, ws[0].data_ptr(), ws[0].numel(), ws[1].data_ptr(), ws[1].numel())
    t1 = timed()
    print(f"lanes {B}: forward (assembly + 5 GEMMs) unsplit {t0:.1f} us, split-K output {t1:.1f} us "
          f"(workspace {'registered' if ws is not None else 'not applicable'})", flush=True)
