"""Per-phase timing of the f16x3 forward's five launches from an H3_TRACE build (thread 0 of
every workgroup stamps the 100 MHz device clock: entry, row exponents read, K loop entered /
done, epilogue issued, its stores drained).  Prints, per layer, the medians over workgroups of
each phase and the launch's span (first entry -> last drain), and the gap to the next launch.

usage: tools/src_variant.sh amx_gemm.hip h3t -DH3_TRACE=1, install it as libamx_hip.so, then
       python tools/h3_trace.py [lanes ...]"""
import ctypes
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
# "b512": 512 lanes through the member-blocked forward (forward_blocked, 128 rows per member)
lanes = [x for x in sys.argv[1:]] or ["5120", "8192"]
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*(torch.from_numpy(x).float() for x in (s, a, s2)))
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, base_seed=100), norms)
lib = ctx.lib
if not hasattr(lib, "amx_h3_trace_read"):
    raise SystemExit("not an H3_TRACE build (tools/src_variant.sh amx_gemm.hip h3t -DH3_TRACE=1)")
lib.amx_h3_trace_read.argtypes = [ctypes.c_void_p]
buf = np.zeros((5, 1024, 8), np.uint64)
names = ["L0", "L1", "L2", "L3", "out"]
for spec in lanes:
    blocked = spec.startswith("b")
    B = int(spec.lstrip("b"))
    rs = np.random.RandomState(B)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
    ac = torch.from_numpy(rs.randn(B, A)).cuda()
    for rep in range(6):
        buf[:] = 0
        if blocked:
            ens.forward_blocked(ob, ac, B // 4)
        else:
            ens.forward_preds(ob, ac, B)
        torch.cuda.synchronize()
        assert lib.amx_h3_trace_read(buf.ctypes.data) == 0
    print(f"lanes {spec}: medians over workgroups, us (100 MHz stamps; last of 6 forwards)")
    print(f"  {'layer':5s} {'wgs':>4s} {'start':>7s} {'rexp':>6s} {'prolog':>6s} {'kloop':>7s} {'epi':>6s} "
          f"{'drain':>6s} | {'span':>7s} {'entry spread':>12s} {'gap->next':>9s}")
    t0 = None
    prev_end = None
    rows = []
    for li in range(5):
        st = buf[li].astype(np.int64)
        used = st[:, 0] > 0
        st = st[used]
        if len(st) == 0:
            continue
        if t0 is None:
            t0 = st[:, 0].min()
        d = np.diff(st[:, :6], axis=1) / 100.0  # us
        med = np.median(d, axis=0)
        span = (st[:, 5].max() - st[:, 0].min()) / 100.0
        spread = (st[:, 0].max() - st[:, 0].min()) / 100.0
        rows.append((li, st[:, 0].min(), st[:, 5].max()))
        print(f"  {names[li]:5s} {len(st):4d} {(st[:, 0].min() - t0) / 100.0:7.1f} {med[0]:6.2f} {med[1]:6.2f} "
              f"{med[2]:7.2f} {med[3]:6.2f} {med[4]:6.2f} | {span:7.1f} {spread:12.2f}", end="")
        print()
    for (la, _, e), (lb, s_, _) in zip(rows, rows[1:]):
        print(f"  gap {names[la]} last drain -> {names[lb]} first entry: {(s_ - e) / 100.0:.2f} us")
    # the spread of K-loop ends and drain ends within a launch
    for li in range(5):
        st = buf[li].astype(np.int64)
        st = st[st[:, 0] > 0]
        if len(st):
            ke = (st[:, 3] - st[:, 3].min()) / 100.0
            de = (st[:, 5] - st[:, 5].min()) / 100.0
            print(f"  {names[li]}: K-loop end spread p50/p90/max {np.median(ke):.2f}/{np.percentile(ke, 90):.2f}/"
                  f"{ke.max():.2f}, drain end spread {np.median(de):.2f}/{np.percentile(de, 90):.2f}/{de.max():.2f}")
