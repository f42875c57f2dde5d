"""Time one f16x3 ensemble forward (assembly + 5 GEMM launches) at the given lane counts:
every member on every lane (forward_preds) and, for lane counts that are multiples of 4 x 128,
one member per lane (forward_blocked, the reference-semantics sampler's form).  Each form is
timed eagerly (HIP events, median of 40) and as 20 forwards replayed back to back from one
captured HIP graph (the sampler's chunk graphs), and the blocked preds are checked against the
matching member's rows of forward_preds.
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


def eager(fn):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
    for e0, e1 in ev:
        e0.record()
        fn()
        e1.record()
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]))


def graphed(fn, n=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        g.capture_begin()
        for _ in range(n):
            fn()
        g.capture_end()
    torch.cuda.current_stream().wait_stream(st)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / n)
    return float(np.median(ts))


M = ctx.M
for B in [int(x) for x in sys.argv[1:]] or [512, 640, 1024, 2048]:
    rs = np.random.RandomState(1)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
    ac = torch.from_numpy(rs.randn(B, A)).cuda()
    full = lambda: ens.forward_preds(ob, ac, B)
    line = f"lanes {B:5d}: all members {eager(full):7.1f} us eager, {graphed(full):7.1f} us graphed"
    if B % (M * 128) == 0:
        Bq = B // M
        blk = lambda: ens.forward_blocked(ob, ac, Bq)
        ref = ens.forward_preds(ob, ac, B).clone()
        got = ens.forward_blocked(ob, ac, Bq).clone()
        want = torch.cat([ref[g, g * Bq:(g + 1) * Bq] for g in range(M)])
        err = float(((got - want).abs().max() / want.abs().max()).item())
        line += f" | one member {eager(blk):7.1f} us eager, {graphed(blk):7.1f} us graphed (max rel diff {err:.1e})"
    print(line, flush=True)
