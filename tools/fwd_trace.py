"""Per-layer phase times of the one-launch forward from an FW_TRACE build (thread 0 of every
workgroup: K loop entered / done, layer done), medians over workgroups, at the given lane counts.
usage: tools/src_variant.sh amx_fwd.hip fwt -DFW_TRACE=1, install it as libamx_hip.so, then
       python tools/fwd_trace.py [lanes ...]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402

S, A = 197, 36
lanes = [int(x) for x in sys.argv[1:]] or [5120, 8192]
norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms, gemm="f16x3")
lib = ctx.lib
if not hasattr(lib, "amx_fwd_trace_read"):
    raise SystemExit("not an FW_TRACE build (tools/src_variant.sh amx_fwd.hip fwt -DFW_TRACE=1)")
lib.amx_fwd_trace_read.argtypes = [ctypes.c_void_p]
buf = np.zeros((1024, 9, 3), np.uint64)
names = ["L0", "L1", "L2", "L3", "out"]
Ks = [256, 768, 1280, 1792, 2304]
for B in lanes:
    rs = np.random.RandomState(B)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
    ac = torch.from_numpy(rs.randn(B, A)).cuda()
    for _ in range(6):
        ens.forward_preds(ob, ac, B)
        torch.cuda.synchronize()
    assert lib.amx_fwd_trace_read(buf.ctypes.data) == 0
    st = buf.astype(np.int64)
    used = st[:, 0, 0] > 0
    st = st[used]
    t0 = st[:, 0, 0].min()
    print(f"lanes {B}: {len(st)} workgroups, rows/wg {ens.fused_rows((B + 127) // 128 * 128)}; us, medians (max)")
    for li in range(5):
        kl = (st[:, li, 1] - st[:, li, 0]) / 100.0
        ep = (st[:, li, 2] - st[:, li, 1]) / 100.0
        print(f"  {names[li]:4s} K {Ks[li]:5d}: start {np.median(st[:, li, 0] - t0) / 100.0:7.1f}  K loop "
              f"{np.median(kl):7.2f} ({kl.max():7.2f}) = {np.median(kl) / (Ks[li] // 32):.3f} per K-tile   "
              f"epilogue+sync {np.median(ep):6.2f} ({ep.max():6.2f})")
    end = (st[:, 4, 2].max() - t0) / 100.0
    print(f"  span {end:.1f} us (first start -> last drained); ends spread {np.ptp(st[:, 4, 2]) / 100.0:.2f} us")
