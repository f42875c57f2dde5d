"""Time the device policy kernel (amx_policy_act: staging, three MFMA layers, Gaussian noise) at
8192 and 5120 lanes in three forms -- Philox + Box-Muller noise (the rollout's), injected noise
(read from a tensor) and eval mode (no noise) -- HIP events over 200 back-to-back launches, to
price the noise phase.  usage: python tools/policy_time.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

S, A = 197, 36
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
pw, ls = init_mlp_policy_params(S, A)
pol = amx.DevicePolicy(ctx, pw, ls, seed=5)
for B in (8192, 5120):
    ob = torch.from_numpy(syn.reset_table(B, S, 2)).cuda()
    out = torch.empty(B, A, dtype=torch.float64, device="cuda")
    noise = torch.randn(B, A, dtype=torch.float64, device="cuda")
    ctr = torch.zeros(1, dtype=torch.int64, device="cuda")
    forms = {"philox": dict(), "philox_dev": dict(counter_dev=ctr), "injected": dict(noise=noise),
             "eval": dict(eval_mode=True)}
    for name, kw in forms.items():
        def launch(i):
            pol.act(ob, B, out, i, **kw)
        for i in range(10):
            launch(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(200):
            launch(i)
        e1.record()
        torch.cuda.synchronize()
        print(f"lanes {B} {name:10s}: {e0.elapsed_time(e1) * 1e3 / 200:6.2f} us/launch", flush=True)
