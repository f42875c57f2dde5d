"""Same-process A/B of GEMM tile variants on the real rollout (bench workload), interleaved
rounds (cdna_hip_programming.md §5.4 rule 24).

usage: python tools/rollout_ab.py [lanes] [variants, comma-separated]
variant: f16x3 (default GEMM path) "h<hidden>o<output>" -> amx__set_h3_variant / amx__set_h3_out_variant
(-1 = automatic, e.g. "h-1o-1", "h9o1"); "s0"/"s1": automatic tiles without / with the shared x0
slice (DeviceEnsemble.shared_x0); "r0"/"r1": separate / fused step + reset (RolloutEngine.fuse_reset); "p16"/"p32": policy kernel with 16 / 32
threads per lane (amx__set_policy_tpl); "o0"/"o1": batched / per-step side-stream scoring; f32 path (--gemm f32 ensembles) "<k>[p]" -> amx__set_gemm_variant.
"""
import re
import ctypes
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
VARIANTS = (sys.argv[2] if len(sys.argv) > 2 else "h-1o-1,h9o1").split(",")
S, A = 197, 36
dev = torch.device("cuda", 0)
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
ctx = amx.AmxContext(S, A, 4, 512, 4, 512, device=dev)
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
ens.compute_threshold(torch.from_numpy(s).float().to(dev), torch.from_numpy(a).float().to(dev))
cost = amx.RBFLinearCost(torch.from_numpy(syn.expert(50000, S, 3)), feature_dim=512, bw_quantile=0.1,
                         lambda_b=0.0025, seed=100, ctx=ctx)
pw, ls = init_mlp_policy_params(S, A)
pol = amx.DevicePolicy(ctx, pw, ls, seed=1)
T = math.ceil(40000 / B)
eng = amx.RolloutEngine(ens, syn.reset_table(65536, S, 1), lanes=B, policy=pol, cost=cost, seed=7, max_steps=T)
eng.reset_all()
lib = ctx.lib
_setv = lib.amx__set_gemm_variant
_setv.argtypes = [ctypes.c_int]
lib.amx__set_gemm_persistent.argtypes = [ctypes.c_int]

lib.amx__set_h3_variant.argtypes = [ctypes.c_int]
lib.amx__set_h3_out_variant.argtypes = [ctypes.c_int]
lib.amx__set_policy_tpl.argtypes = [ctypes.c_int]


def setv(v):
    """'h9o1' -> f16x3 hidden variant 9, output variant 1; '4' -> f32 tile variant 4; a trailing
    'p' -> persistent workgroups; 'auto'/'-1' -> automatic."""
    s = str(v)
    ens.shared_x0 = s != "s0"  # "s0": one x0 copy per member (no k_shared)
    eng.fuse_reset = s != "r0"  # "r0": amx_step + amx_reset_lanes instead of amx_step_reset
    lib.amx__set_policy_tpl(16 if s == "p16" else (32 if s == "p32" else 0))  # policy threads per lane
    if s in ("o0", "o1"):  # per-step scoring on a side stream (RolloutEngine.overlap_score)
        eng.overlap_score = s == "o1"
    if s in ("s0", "s1", "r0", "r1", "p16", "p32", "o0", "o1"):
        s = "h-1o-1"
    m = re.fullmatch(r"h(-?\d+)o(-?\d+)", s)
    if m:
        lib.amx__set_h3_variant(int(m.group(1)))
        lib.amx__set_h3_out_variant(int(m.group(2)))
        return
    lib.amx__set_h3_variant(-1)
    lib.amx__set_h3_out_variant(-1)
    lib.amx__set_gemm_persistent(int(s.endswith("p")))
    s = s.rstrip("p")
    _setv(-1 if s in ("auto", "-1", "") else int(s))



def rollout():
    eng.rollout(T)
    eng.relabel()
    cost.get_expert_cost()


for v in VARIANTS:
    setv(v)
    rollout()
torch.cuda.synchronize()
setv(-1)
t_end = time.perf_counter() + 0.5  # clock settle (tools/mfma_ceiling.hip)
while time.perf_counter() < t_end:
    rollout()
    torch.cuda.synchronize()
res = {v: [] for v in VARIANTS}
for r in range(6):
    for v in VARIANTS:
        setv(v)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(4):
            rollout()
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t0) / 4)
setv(-1)
print(f"lanes {B}: ms per {T * B}-sample rollout (median / min of 6 rounds x 4)")
for v in VARIANTS:
    print(f"variant {v:>4s}: {np.median(res[v]) * 1e3:7.3f} {np.min(res[v]) * 1e3:7.3f}  -> "
          f"{T * B / np.median(res[v]) / 1e6:.3f} M env-steps/s")
