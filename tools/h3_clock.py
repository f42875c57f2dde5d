"""Where a f16x3 ensemble-layer launch spends its time, from inside the kernel: per workgroup
s_memrealtime (100 MHz) at start, at the end of the K loop and after its epilogue's stores
have drained (s_waitcnt 0), plus the loop's shader clocks (amx__set_gemm_clock_probe, LATE
tiles).  Against the launch's wall time (20 back-to-back launches) this splits a layer into
dispatch skew, K loop, epilogue + store drain and the rest (launch / teardown).

usage: python tools/h3_clock.py [lanes]
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
S, A = (int(v) for v in os.environ.get("AMX_SA", "197,36").split(","))
torch.manual_seed(0)
norms = [torch.zeros(S), torch.ones(S), torch.zeros(A), torch.ones(A), torch.zeros(S), torch.ones(S)]
c = amx.AmxContext(S, A, 4, 512, 4, 512, device="cuda")
e = amx.DeviceEnsemble(c, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms, gemm="f16x3")
lib = c.lib
lib.amx__set_gemm_clock_probe.argtypes = [ctypes.c_void_p]
ob = torch.randn(B, S, device="cuda")
ac = torch.randn(B, A, device="cuda")
e.forward_preds(ob, ac, B)  # activation rows + row-exponent slots of a real forward
ws = e.workspace(B)
Bp, buf, rexp, preds = ws["Bp"], ws["act"], ws["rexp"], ws["preds"]
out = torch.zeros_like(buf)
scratch = torch.empty_like(rexp)
s = c.stream
sA, sR = Bp * c.ldk, (c.L + 1) * Bp
probe = torch.zeros(4 * 8192, dtype=torch.int64, device="cuda")


def layer(i):
    if i < c.L:
        K = c.k0_pad + i * c.Hp
        N.check(lib.amx_gemm_bias_act_h3(c.h, c.M, Bp, c.Hp, K, buf.data_ptr(), c.ldk, sA, e.W2[i].data_ptr(),
                                         c.Hp * 2 * K, e.wexp[i].data_ptr(), c.Hp, e.b[i].data_ptr(), c.Hp,
                                         out.data_ptr(), c.ldk, sA, K, N.AMX_ACT_RELU, rexp.data_ptr(), sR, i + 1,
                                         scratch[0, i + 1].data_ptr(), c.k0_pad, s), "h3")
    else:
        N.check(lib.amx_gemm_out_unnorm_h3(c.h, c.M, Bp, c.S, c.ldk, buf.data_ptr(), c.ldk, sA, e.W2[c.L].data_ptr(),
                                           c.n_out_pad * 2 * c.ldk, e.wexp[c.L].data_ptr(), c.n_out_pad,
                                           e.b[c.L].data_ptr(), c.n_out_pad, preds.data_ptr(), c.S, Bp * c.S,
                                           rexp.data_ptr(), sR, c.L + 1, c.k0_pad, s), "h3 out")


t_end = time.perf_counter() + 1.0  # clock settle
while time.perf_counter() < t_end:
    for i in range(c.L + 1):
        layer(i)
    torch.cuda.synchronize()
print(f"lanes {B}, S={S}: per layer (us; medians over 5 probed launches, workgroup means unless noted)")
print("layer     K  wall  skew(max start)  loop  loop_GHz  epi+drain  last_end  wall-last_end")
for i in range(c.L + 1):
    K = c.k0_pad + i * c.Hp if i < c.L else c.ldk
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        layer(i)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 20 * 1e6
    rows = []
    for _ in range(5):
        probe.zero_()
        lib.amx__set_gemm_clock_probe(probe.data_ptr())
        layer(i)
        lib.amx__set_gemm_clock_probe(None)
        torch.cuda.synchronize()
        p = probe.view(-1, 4).cpu().numpy().astype(np.float64)
        p = p[p[:, 0] > 0]
        t0w = p[:, 0].min()
        st, l1, l2 = (p[:, 0] - t0w) / 100.0, (p[:, 1] - t0w) / 100.0, (p[:, 2] - t0w) / 100.0
        ghz = np.mean(p[:, 3] / ((p[:, 1] - p[:, 0]) / 100e6)) / 1e9
        rows.append((st.max(), np.mean(l1 - st), ghz, np.mean(l2 - l1), l2.max(), len(p)))
    r = np.median(np.array(rows), axis=0)
    print(f"{i:5d} {K:5d} {wall:5.1f} {r[0]:16.2f} {r[1]:5.1f} {r[2]:9.2f} {r[3]:10.2f} {r[4]:9.1f} "
          f"{wall - r[4]:14.1f}   ({int(r[5])} WGs)")
