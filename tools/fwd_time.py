"""Median HIP-event time of one f16x3 ensemble forward (assembly + 5 GEMM launches) at the given
lane counts, plus the output layer alone (rocprof gives per-kernel times; this is the quick A/B).
usage: python tools/fwd_time.py [B ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402

S, A = 197, 36
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*(torch.from_numpy(x).float() for x in (s, a, s2)))
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, base_seed=100), norms)
for B in [int(x) for x in sys.argv[1:]] or [8192, 5120]:
    rs = np.random.RandomState(1)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
    ac = torch.from_numpy(rs.randn(B, A)).cuda()
    for _ in range(10):
        ens.forward_preds(ob, ac, B)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
    for e0, e1 in ev:
        e0.record()
        ens.forward_preds(ob, ac, B)
        e1.record()
    torch.cuda.synchronize()
    t = np.median([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev])
    print(f"lanes {B}: forward {t:.1f} us", flush=True)
