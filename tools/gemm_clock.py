"""Shader clock and MFMA-pipe efficiency of the ensemble GEMM, from inside the kernel.

Each workgroup records s_memtime (shader cycles) and s_memrealtime (100 MHz) at its start
and at the end of its main loop (amx__set_gemm_clock_probe).  Per layer this prints the
mean shader clock the workgroups ran at, and the main-loop span in cycles against the
MFMA-only ideal (per-WG MFMAs x co-resident WGs x 64 cycles / 4 SIMDs), which separates
clock (DVFS) from schedule losses in the gap to the 157.3 TF spec.

usage: python tools/gemm_clock.py [lanes] [variants, comma-separated; -1 = automatic]
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
# variant -> (BM, BN, co-resident WGs per CU) for the hidden layers
TILES = {0: (128, 128, 2), 1: (128, 256, 1), 3: (256, 256, 1), 4: (256, 128, 1), 9: (256, 128, 1), -1: (128, 128, 2)}

torch.manual_seed(0)
norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
lib = ctx.lib
lib.amx__set_gemm_variant.argtypes = [ctypes.c_int]
lib.amx__set_gemm_clock_probe.argtypes = [ctypes.c_void_p]
ws = ens.workspace(B)
Bp, buf = ws["Bp"], ws["act"]
buf.normal_()
s = ctx.stream
probe = torch.zeros(4 * 4096, dtype=torch.int64, device="cuda")


def layer(i):
    K = ctx.k0_pad + i * ctx.Hp
    N.check(lib.amx_gemm_bias_act(ctx.h, 4, Bp, 512, K, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk, ens.W[i].data_ptr(),
                                  K, 512 * K, ens.b[i].data_ptr(), 512, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk, K,
                                  1, s))


t_end = time.perf_counter() + 0.5  # clock settle
while time.perf_counter() < t_end:
    for i in range(ctx.L):
        layer(i)
    torch.cuda.synchronize()

print(f"lanes {B}: per hidden layer, mean over workgroups (3 runs)")
print("variant layer     K   clock_GHz  span_us  loop_cycles  ideal_cycles  mfma_eff")
for v in VARIANTS:
    lib.amx__set_gemm_variant(v)
    BM, BN, occ = TILES[v]
    for i in range(ctx.L):
        K = ctx.k0_pad + i * ctx.Hp
        nwg = (Bp // BM) * (512 // BN) * 4
        clocks, spans, cyc = [], [], []
        for _ in range(3):
            for _ in range(3):
                layer(i)  # keep the pipe busy before the probed launch
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
        ideal = BM * BN * K / (32 * 32 * 2) * occ * 64 / 4
        print(f"{v:7d} {i:5d} {K:5d} {np.median(clocks):10.3f} {np.median(spans):8.1f} {np.median(cyc):12.0f} "
              f"{ideal:13.0f} {ideal / np.median(cyc):9.3f}")
lib.amx__set_gemm_variant(-1)
