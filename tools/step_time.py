"""Time the fused step kernel (amx_step_reset: fp64 update, termination, 4-member disagreement,
[s, s'] cost row + row exponent, table reset of done lanes) at 8192 and 5120 lanes, with and
without the disagreement (disc = null), HIP events over 200 back-to-back launches; algorithmic
HBM bytes per lane: 4 S f32 preds + S f64 ob read, 2 S f64 (ob', carried ob) + 2S f32 cost row
written.  usage: python tools/step_time.py"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402

S, A = 197, 36
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
ctx.set_termination(amx.TerminationConfig())
lib, h, st = ctx.lib, ctx.h, ctx.stream
table = torch.from_numpy(syn.reset_table(65536, S, 1)).cuda()
for B in (8192, 5120):
    Bp = (B + 127) // 128 * 128
    g = torch.Generator(device="cpu").manual_seed(0)
    ob = torch.from_numpy(syn.reset_table(B, S, 2)).cuda()
    preds = (torch.randn(4, Bp, S, generator=g) * 1e-3).cuda()
    ob_next = torch.empty_like(ob)
    ob_out = torch.empty_like(ob)
    kc = (2 * S + 31) // 32 * 32
    cost_in = torch.zeros(Bp, kc, device="cuda")
    rexp = torch.zeros(Bp, dtype=torch.int32, device="cuda")
    z = lambda dt: torch.zeros(B, dtype=dt, device="cuda")
    model_idx, num_steps, reset_count, row_out = z(torch.int32), z(torch.int32), z(torch.int32), z(torch.int32)
    done, nonf = z(torch.uint8), z(torch.uint8)
    disc = torch.zeros(Bp, device="cuda")
    for with_disc in (True, False):
        def launch():
            rc = lib.amx_step_reset(h, preds.data_ptr(), S, Bp * S, model_idx.data_ptr(), ob.data_ptr(),
                                    ob_next.data_ptr(), num_steps.data_ptr(), done.data_ptr(),
                                    disc.data_ptr() if with_disc else None, cost_in.data_ptr(), kc, rexp.data_ptr(),
                                    nonf.data_ptr(), table.data_ptr(), table.shape[0], None, 5, ob_out.data_ptr(),
                                    reset_count.data_ptr(), row_out.data_ptr(), None, None, 0, None, B, st)
            assert rc == 0, lib.amx_last_error()
        for _ in range(10):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(200):
            launch()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 200
        byts = B * (4 * S * 4 + S * 8 + 2 * S * 8 + kc * 4)
        print(f"lanes {B} disc={with_disc}: {us:6.2f} us/launch, {byts / us / 1e6:5.2f} TB/s algorithmic", flush=True)
