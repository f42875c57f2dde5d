"""A/B of the CG fold (DeviceNPG.cg_fold: the vector step at the head of the next Fisher-vector
pass, amx_npg_pass_cg) against the round-5 tail (amx_npg_cg_tail's two launches), same process,
alternating: the 10-iteration cg_solve alone (HIP events, 20 solves) and the whole update as a
training loop runs it (consecutive train_from_arrays, 10 updates); x compared bit for bit.
usage: python tools/npg_fold_ab.py [N] [rounds]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd.npg import NPG_VPG  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40960
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
S, A = 197, 36
layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
rs = np.random.RandomState(0)
obs_d, act_d, adv_d = (torch.from_numpy(x).cuda() for x in (0.5 * rs.randn(N, S), rs.randn(N, A), rs.randn(N)))
ctx = amx.AmxContext(S, A, n_models=1, hidden=128, n_hidden=1, device="cuda")
npg = amx.DeviceNPG(ctx, layers, ls, normalized_step_size=0.1, min_log_std=-2.0)
o, a, adv = npg._inputs(obs_d, act_d, adv_d)
hc = npg._hcache(N)
b = npg._pass(NPG_VPG, o, a, adv, None, hcache=hc).clone()
xs = {}
for fold in (False, True):
    npg.cg_fold = fold
    xs[fold] = npg.cg_solve(o, a, b, hcache=hc).clone()
print("x bit-identical:", bool(torch.equal(xs[False], xs[True])), flush=True)
p0 = npg.get_param_values()
for r in range(rounds):
    for fold in (False, True):
        npg.cg_fold = fold
        for _ in range(3):
            npg.cg_solve(o, a, b, hcache=hc)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            npg.cg_solve(o, a, b, hcache=hc)
        e1.record()
        torch.cuda.synchronize()
        cg_us = e0.elapsed_time(e1) * 1e3 / 20
        npg.set_param_values(p0)
        npg.train_from_arrays(obs_d, act_d, adv_d)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            npg.train_from_arrays(obs_d, act_d, adv_d)
        torch.cuda.synchronize()
        upd_ms = (time.perf_counter() - t0) / 10 * 1e3
        npg.set_param_values(p0)
        print(f"round {r} fold={int(fold)}: cg_solve {cg_us:7.1f} us ({cg_us / npg.cg_iters:5.1f} per iteration), "
              f"update {upd_ms:6.3f} ms", flush=True)
