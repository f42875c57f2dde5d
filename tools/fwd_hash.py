"""Hash of the f16x3 ensemble forward (every lane-count regime: 256x256, row-block, stream-K
and small-tile shapes) and of an RFF pass, for bit-identity checks between library builds
(tools/so_ab.sh).  usage: python tools/fwd_hash.py"""
import hashlib
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import amp_extensions_amd as amx  # noqa: E402
from amp_extensions_amd import synthetic as syn  # noqa: E402
from amp_extensions_amd.datasets import get_transformations  # noqa: E402
from amp_extensions_amd.ensemble import init_ensemble_weights  # noqa: E402

S, A = 197, 36
s, a, s2 = syn.offline(20000, S, A, 0)
norms = get_transformations(*(torch.from_numpy(x).float() for x in (s, a, s2)))
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device="cuda")
ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, base_seed=100), norms)
h = hashlib.sha256()
for B in (8192, 7168, 5120, 4096, 1000, 640, 128):
    rs = np.random.RandomState(B)
    ob = torch.from_numpy(0.5 * rs.randn(B, S)).cuda()
    ac = torch.from_numpy(rs.randn(B, A)).cuda()
    p = ens.forward_preds(ob, ac, B)[:, :B].contiguous()
    h.update(p.cpu().numpy().tobytes())
    print(f"lanes {B}: preds sum {p.double().sum().item():.17g}", flush=True)
g = torch.Generator().manual_seed(3)
W = torch.randn(512, 2 * S, generator=g) / 3.0
b = torch.rand(512, generator=g) * 6.28
rff = amx.RffMap(ctx, W, b)
for rows in (40960, 5120):
    x = torch.zeros(rows, rff.Kp, device="cuda")
    x[:, :2 * S] = 0.5 * torch.randn(rows, 2 * S, generator=g).cuda()
    phi = torch.empty(rows, 512, device="cuda")
    part = torch.empty((rows + 127) // 128 * 4, 512, dtype=torch.float64, device="cuda")  # 32-row partials
    rff.features(x, rows, rows, phi, part)
    torch.cuda.synchronize()
    h.update(phi.cpu().numpy().tobytes())
    h.update(part.cpu().numpy().tobytes())
    print(f"rff {rows}: phi sum {phi.double().sum().item():.17g}", flush=True)
print("HASH", h.hexdigest(), flush=True)
