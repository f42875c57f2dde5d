"""A/B the GEMM tile variants on the ensemble's layer shapes, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24).  Prints per-layer TFLOP/s (algorithmic, unpadded
K/N) for each variant: median and best over rounds.

usage: python tools/gemm_variants.py [lanes] [S] [A]
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
S = int(sys.argv[2]) if len(sys.argv) > 2 else 197
A = int(sys.argv[3]) if len(sys.argv) > 3 else 36
VARIANTS = sys.argv[4].split(",") if len(sys.argv) > 4 else ["0", "4", "9"]
ROUNDS, REPS = 7, 5

torch.manual_seed(0)
norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
lib = ctx.lib
_setv = lib.amx__set_gemm_variant
_setv.argtypes = [ctypes.c_int]
lib.amx__set_gemm_persistent.argtypes = [ctypes.c_int]

def setv(v):
    """'4' -> tile variant 4; a trailing 'p' -> persistent workgroups; 'auto'/'-1' -> automatic."""
    s = str(v)
    lib.amx__set_gemm_persistent(int(s.endswith("p")))
    s = s.rstrip("p")
    _setv(-1 if s in ("auto", "-1", "") else int(s))

ws = ens.workspace(B)
Bp, buf, preds = ws["Bp"], ws["act"], ws["preds"]
buf.normal_()
s = ctx.stream
k0 = ctx.k0_pad


def layer(i):
    if i < ctx.L:
        K = k0 + i * ctx.Hp
        N.check(lib.amx_gemm_bias_act(ctx.h, 4, Bp, 512, K, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk, ens.W[i].data_ptr(),
                                      K, 512 * K, ens.b[i].data_ptr(), 512, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk, K,
                                      1, s))
    else:
        N.check(lib.amx_gemm_out_unnorm(ctx.h, 4, Bp, S, ctx.ldk, buf.data_ptr(), ctx.ldk, Bp * ctx.ldk,
                                        ens.W[i].data_ptr(), ctx.ldk, ctx.n_out_pad * ctx.ldk, ens.b[i].data_ptr(),
                                        ctx.n_out_pad, preds.data_ptr(), S, Bp * S, s))


def alg_flops(i):
    Kalg = S + A + 512 * i
    Nalg = 512 if i < ctx.L else S
    return 2.0 * 4 * B * Nalg * Kalg


# every variant must reproduce variant 0 bit for bit (same per-element k order)
buf0 = buf.clone()
ref = None
for v in ["0"] + VARIANTS + ["auto"]:
    setv(v)
    buf.copy_(buf0)
    preds.zero_()
    for i in range(ctx.L + 1):
        layer(i)
    torch.cuda.synchronize()
    if ref is None:
        ref = (buf.clone(), preds.clone())
    else:
        ok = torch.equal(buf, ref[0]) and torch.equal(preds, ref[1])
        print(f"variant {v}: {'bit-exact vs variant 0' if ok else 'MISMATCH vs variant 0'}", flush=True)
        if not ok:
            raise SystemExit(1)

# settle the clock: the chip ramps its clock over tens of ms of sustained MFMA load
# (tools/mfma_ceiling.hip), so measure only after ~0.5 s of back-to-back work
setv(-1)
t_end = time.perf_counter() + 0.5
while time.perf_counter() < t_end:
    for i in range(ctx.L + 1):
        layer(i)
    torch.cuda.synchronize()

res = {(v, i): [] for v in VARIANTS + ["auto"] for i in range(ctx.L + 1)}
seq = {v: [] for v in VARIANTS + ["auto"]}
for r in range(ROUNDS):
    # whole-forward sequence per variant (what the rollout runs)
    for v in VARIANTS + ["auto"]:
        setv(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(REPS):
            for i in range(ctx.L + 1):
                layer(i)
        e1.record()
        torch.cuda.synchronize()
        seq[v].append(e0.elapsed_time(e1) / REPS * 1e-3)
    for v in VARIANTS + ["auto"]:
        setv(v)
        for i in range(ctx.L + 1):
            layer(i)  # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(REPS):
                layer(i)
            e1.record()
            torch.cuda.synchronize()
            res[(v, i)].append(e0.elapsed_time(e1) / REPS * 1e-3)
setv(-1)
print(f"lanes {B}, S {S}, A {A}: TFLOP/s algorithmic (median / best of {ROUNDS})")
print("variant " + " ".join(f"{'L' + str(i) if i < ctx.L else 'out':>14s}" for i in range(ctx.L + 1)) + "   total_us")
for v in VARIANTS + ["auto"]:
    row, tot = [], 0.0
    for i in range(ctx.L + 1):
        ts = np.array(res[(v, i)])
        tot += np.median(ts)
        row.append(f"{alg_flops(i) / np.median(ts) / 1e12:6.1f}/{alg_flops(i) / ts.min() / 1e12:6.1f}")
    print(f"{str(v):>7s} " + " ".join(f"{x:>14s}" for x in row) + f"   {tot * 1e6:8.1f}"
          f"   sequence {np.median(seq[v]) * 1e6:8.1f} us")
