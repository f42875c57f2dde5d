"""Shader clock and matrix-pipe efficiency of the bf16x6 hidden-layer GEMM, from inside the
kernel (same probe as tools/gemm_clock.py).  Ideal main-loop cycles per workgroup = its
bf16 MFMAs (6 limb products x 32x32x16 blocks) x 32 cycles x co-resident WGs / 4 SIMDs.

usage: python tools/x6_clock.py [lanes] [variants]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import _native as N  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
VARIANTS = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,4").split(",")]
S, A = 197, 36
# variant -> (BM, BN, co-resident WGs per CU)
TILES = {0: (128, 128, 2), 1: (128, 128, 2), 2: (128, 128, 2), 3: (128, 128, 1), 4: (128, 256, 1),
         5: (256, 128, 1), 6: (128, 256, 1), 9: (256, 256, 1), -1: (256, 256, 1)}
norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms, gemm="bf16x6")
lib = ctx.lib
lib.amx__set_x6_variant.argtypes = [ctypes.c_int]
lib.amx__set_gemm_clock_probe.argtypes = [ctypes.c_void_p]
ws = ens.workspace(B)
Bp, buf = ws["Bp"], ws["act"]
buf.normal_()
s = ctx.stream
probe = torch.zeros(4 * 4096, dtype=torch.int64, device="cuda")


def layer(i):
    K = ctx.k0_pad + i * ctx.Hp
    N.check(lib.amx_gemm_bias_act_x6(ctx.h, 4, Bp, 512, K, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk,
                                     ens.W3[i].data_ptr(), 512 * 3 * K, ens.b[i].data_ptr(), 512, buf.data_ptr(),
                                     ctx.ldk, Bp * ctx.ldk, K, 1, s))


t_end = time.perf_counter() + 1.0  # clock settle
while time.perf_counter() < t_end:
    for i in range(ctx.L):
        layer(i)
    torch.cuda.synchronize()
print(f"lanes {B}: per hidden layer, mean over workgroups (3 runs)")
print("variant layer     K   clock_GHz  span_us  loop_cycles  ideal_cycles  mfma_eff")
for v in VARIANTS:
    lib.amx__set_x6_variant(v)
    BM, BN, occ = TILES[v]
    for i in range(ctx.L):
        K = ctx.k0_pad + i * ctx.Hp
        nwg = (Bp // BM) * (512 // BN) * 4
        clocks, spans, cyc = [], [], []
        for _ in range(3):
            for _ in range(3):
                layer(i)
            probe.zero_()
            lib.amx__set_gemm_clock_probe(probe.data_ptr())
            layer(i)
            lib.amx__set_gemm_clock_probe(None)
            torch.cuda.synchronize()
            p = probe[:4 * nwg].view(nwg, 4).cpu().numpy().astype(np.float64)
            dc, dr = p[:, 2] - p[:, 0], (p[:, 3] - p[:, 1]) / 100e6
            clocks.append(np.mean(dc / dr) / 1e9)
            spans.append(np.mean(dr) * 1e6)
            cyc.append(np.mean(dc))
        ideal = (BM // 32) * (BN // 32) * (K // 16) * 6 * 32 * occ / 4
        print(f"{v:7d} {i:5d} {K:5d} {np.median(clocks):10.3f} {np.median(spans):8.1f} {np.median(cyc):12.0f} "
              f"{ideal:13.0f} {ideal / np.median(cyc):9.3f}")
lib.amx__set_x6_variant(-1)
