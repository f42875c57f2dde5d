"""amx_feature_message over the rollout's RFF column partials ([rows / 32][512] fp64: 1280 rows at
the 40 960-sample rollout, 160 at the N = 8 share): us per launch (HIP events over 200
back-to-back launches) and a hash of the message bits.  usage: python tools/msg_time.py"""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402

ctx = amx.AmxContext(197, 36, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
for n_parts in (1280, 160):
    g = torch.Generator(device="cpu").manual_seed(n_parts)
    parts = torch.randn(n_parts, 512, generator=g, dtype=torch.float64).cuda()
    msg = torch.empty(513, dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(10):
        ctx.lib.amx_feature_message(ctx.h, parts.data_ptr(), n_parts, 512, 40960.0, msg.data_ptr(), s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        ctx.lib.amx_feature_message(ctx.h, parts.data_ptr(), n_parts, 512, 40960.0, msg.data_ptr(), s)
    e1.record()
    torch.cuda.synchronize()
    ref = parts.sum(0)
    print(f"feature message, {n_parts} partial rows: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per launch; "
          f"max |msg - torch sum| {(msg[:512] - ref).abs().max().item():.3g}; "
          f"bits {hashlib.sha1(msg.cpu().numpy().tobytes()).hexdigest()[:12]}")
