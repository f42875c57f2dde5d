"""k_policy timing at B lanes: Philox noise (the rollout's), injected noise, eval mode (no
noise), HIP-event medians over 50 launches.  usage: python tools/policy_ab.py [B]"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd.policy import init_mlp_policy_params  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
S, A = 197, 36
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
pw, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
pol = amx.DevicePolicy(ctx, pw, ls, seed=1)
ob = torch.randn(B, S, dtype=torch.float64, device="cuda") * 0.5
act = torch.empty(B, A, dtype=torch.float64, device="cuda")
noise = torch.randn(B, A, dtype=torch.float64, device="cuda")


def timed(**kw):
    for _ in range(5):
        pol.act(ob, B, act, 3, **kw)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for e0, e1 in ev:
        e0.record()
        pol.act(ob, B, act, 3, **kw)
        e1.record()
    torch.cuda.synchronize()
    return float(np.median([e0.elapsed_time(e1) * 1e3 for e0, e1 in ev]))


for _ in range(2):
    print(f"B={B}: philox {timed():.1f} us, injected noise {timed(noise=noise):.1f} us, "
          f"eval mode {timed(eval_mode=True):.1f} us", flush=True)
