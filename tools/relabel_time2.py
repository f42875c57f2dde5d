"""amx_mmd_relabel at the bench shape (40 960 rollout rows + the 50 000-row expert buffer, and the
N = 8 share: 5120 + 6250): us per launch (HIP events over 100 launches) and a hash of the rewards
and the expert sum.  usage: python tools/relabel_time2.py"""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import amp_extensions_amd as amx  # noqa: E402

ctx = amx.AmxContext(197, 36, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
lib, h = ctx.lib, ctx.h
F = 512
for n, n_e in ((40960, 50000), (5120, 6250)):
    g = torch.Generator(device="cpu").manual_seed(n)
    sc = float(np.sqrt(2.0 / F))
    phi = (torch.cos(torch.rand(n, F, generator=g) * 6.3) * sc).cuda()
    erows = (torch.cos(torch.rand(n_e, F, generator=g) * 6.3 + 0.3) * sc).cuda()
    phi_e = erows.double().mean(0).float()
    msg = torch.cat([phi.double().sum(0), torch.tensor([float(n)], dtype=torch.float64, device="cuda")])
    disc = (torch.rand(n, generator=g) * 0.2).cuda()
    w, mmd = torch.empty(F, device="cuda"), torch.empty(1, device="cuda")
    rew, ipm, wb = (torch.empty(n, device="cuda") for _ in range(3))
    eout = torch.zeros(1025, dtype=torch.float64, device="cuda")
    emean = torch.empty(1, device="cuda")
    cnt = torch.zeros(4, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream

    def run():
        lib.amx_mmd_relabel(h, msg.data_ptr(), 0.0, phi_e.data_ptr(), F, w.data_ptr(), mmd.data_ptr(), phi.data_ptr(),
                            F, disc.data_ptr(), 0.07, 0.0025, 1, -1.0, 0.0, rew.data_ptr(), ipm.data_ptr(),
                            wb.data_ptr(), n, erows.data_ptr(), F, n_e, eout.data_ptr(), emean.data_ptr(),
                            cnt.data_ptr(), s)
    for _ in range(5):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        run()
    e1.record()
    torch.cuda.synchronize()
    hsh = hashlib.sha1(rew.cpu().numpy().tobytes() + eout[:1].cpu().numpy().tobytes()).hexdigest()[:12]
    print(f"relabel {n} rollout + {n_e} expert rows: {e0.elapsed_time(e1) / 100 * 1e3:.2f} us per launch; bits {hsh}")
