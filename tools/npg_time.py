"""Time the device NPG update (DeviceNPG.train_from_arrays: VPG + 10 CG Fisher-vector
products + eval) on a 40 960-sample rollout, against the oracle's restatement of the
reference's torch-CPU NPG on the same data (host cores, torch threads as given).

usage: python tools/npg_time.py [N] [S] [A] [cpu_threads]
"""
import hashlib
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd.npg import pack_policy  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402
from oracle import milo_ref as R  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40960
S = int(sys.argv[2]) if len(sys.argv) > 2 else 197
A = int(sys.argv[3]) if len(sys.argv) > 3 else 36
threads = int(sys.argv[4]) if len(sys.argv) > 4 else 16
layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
rs = np.random.RandomState(0)
obs = (0.5 * rs.randn(N, S))
act = rs.randn(N, A)
adv = rs.randn(N)
ctx = amx.AmxContext(S, A, n_models=1, hidden=128, n_hidden=1, device="cuda")
obs_d, act_d, adv_d = (torch.from_numpy(x).cuda() for x in (obs, act, adv))
npg = amx.DeviceNPG(ctx, layers, ls, normalized_step_size=0.1, min_log_std=-2.0)
p0 = npg.get_param_values()
for _ in range(3):
    npg.set_param_values(p0)
    npg.train_from_arrays(obs_d, act_d, adv_d)
torch.cuda.synchronize()
reps = 10
t0 = time.perf_counter()
for _ in range(reps):
    npg.set_param_values(p0)
    out = npg.train_from_arrays(obs_d, act_d, adv_d)
torch.cuda.synchronize()
gpu_ms = (time.perf_counter() - t0) / reps * 1e3
# the update alone, as a training loop runs it: consecutive updates, no parameter restore in
# between (set_param_values' copies, clamp and policy re-sync are the harness's, not the update's)
t0 = time.perf_counter()
for _ in range(reps):
    npg.train_from_arrays(obs_d, act_d, adv_d)
torch.cuda.synchronize()
upd_ms = (time.perf_counter() - t0) / reps * 1e3
# one Fisher-vector product alone
v = torch.randn(npg.P, dtype=torch.float64, device="cuda")
obs32 = obs_d.contiguous()
npg._hvp(obs32, act_d, v)  # the fp64-observation pass kernel's first launch loads its code object
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    npg._hvp(obs32, act_d, v)
e1.record()
torch.cuda.synchronize()
fvp_us = e0.elapsed_time(e1) / 20 * 1e3
print(f"device NPG update, N={N} S={S} A={A}: {gpu_ms:.2f} ms per update (VPG + 10 CG FVPs + eval), "
      f"{fvp_us:.1f} us per public HVP call (fp64 observations); alpha {out['alpha']:.4g}, kl {out['kl_dist']:.4g}")
print(f"  consecutive updates (no set_param_values between them): {upd_ms:.3f} ms per update, its one host sync "
      f"(the infos' python floats) included")
npg.set_param_values(p0)  # the comparison below: one update from p0
npg.train_from_arrays(obs_d, act_d, adv_d)
torch.cuda.synchronize()
print(f"  parameters after one update from p0: sha1 {hashlib.sha1(npg.get_param_values().tobytes()).hexdigest()[:16]} "
      f"(equal across builds = bit-identical updates)")
torch.set_num_threads(threads)
shapes = R.policy_param_shapes(S, A, (32, 32))
t0 = time.perf_counter()
ref = R.npg_update(pack_policy(layers, ls), shapes, obs, act, adv, step=0.1, damping=1e-4, cg_iters=10,
                   min_log_std=-2.0)
cpu_s = time.perf_counter() - t0
print(f"oracle (reference torch-CPU NPG restated), {threads} threads: {cpu_s * 1e3:.1f} ms per update "
      f"-> x{cpu_s * 1e3 / gpu_ms:.0f}; max |dparams| GPU vs CPU "
      f"{np.abs((npg.get_param_values() - p0) - (ref['params1'] - p0)).max():.3g} "
      f"(step max {np.abs(ref['params1'] - p0).max():.3g})")
