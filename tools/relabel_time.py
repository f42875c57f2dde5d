"""Time amx_mmd_relabel (witness + per-sample rewards + 50 000-row expert cost in one launch) at the
rollout sizes of the bench (40 960 rows, N = 1) and of the 8-GPU strong-scaling share (5 120 rows):
HIP events around 200 back-to-back launches; algorithmic bytes = 4 F per rollout row and per expert
row (+ disc/reward/ipm/bonus 16 B per rollout row).  usage: python tools/relabel_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import amp_extensions_amd as amx
from amp_extensions_amd import _native as N

F = 512
ctx = amx.AmxContext(197, 36, n_models=4, hidden=512, n_hidden=4, feat_dim=F, device="cuda")
lib, h, s = ctx.lib, ctx.h, ctx.stream
g = torch.Generator(device="cpu").manual_seed(0)
sc = (2.0 / F) ** 0.5
erows_all = (torch.cos(torch.rand(50000, F, generator=g) * 6.3) * sc).cuda()
counter = torch.zeros(4, dtype=torch.int32, device="cuda")
eo = torch.zeros(1025, dtype=torch.float64, device="cuda")
em = torch.zeros(1, dtype=torch.float32, device="cuda")
for n, NE in ((40960, 50000), (5120, 50000), (5120, 6250), (10240, 12500)):
    erows = erows_all[:NE]
    phi_e = erows.double().mean(0).float()
    phi = (torch.cos(torch.rand(n, F, generator=g) * 6.3) * sc).cuda()
    disc = torch.rand(n, generator=g).cuda() * 0.1
    msg = torch.cat([phi.double().sum(0), torch.tensor([float(n)], dtype=torch.float64, device="cuda")])
    w, m = torch.empty(F, device="cuda"), torch.empty(1, device="cuda")
    r, ip, wb = (torch.empty(n, device="cuda") for _ in range(3))

    def launch():
        N.check(lib.amx_mmd_relabel(h, msg.data_ptr(), 0.0, phi_e.data_ptr(), F, w.data_ptr(), m.data_ptr(),
                                    phi.data_ptr(), F, disc.data_ptr(), 0.07, 0.0025, 1, -1.0, 0.0, r.data_ptr(),
                                    ip.data_ptr(), wb.data_ptr(), n, erows.data_ptr(), F, NE, eo.data_ptr(),
                                    em.data_ptr(), counter.data_ptr(), s), "relabel")
    for _ in range(20):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    byts = 4 * F * (n + NE) + 16 * n
    print(f"rollout rows {n:6d} + expert rows {NE:5d}: {us:7.2f} us/launch, {byts / us / 1e6:6.2f} TB/s algorithmic")
