"""Policy kernel vs the CPU oracle while another process loads the GPU.

usage: python tools/corun_check.py policy      # the checker (6 s of k_policy launches vs the oracle mean)
       python tools/corun_check.py gemm|torchmm  # a co-running load (ensemble GEMMs / torch matmul, 12 s)
e.g.   (./tools/corunner 4 12 & python tools/corun_check.py policy; wait)
"""
import os, sys, numpy as np, torch, time
sys.path.insert(0, "/root/repo")
import amp_extensions_amd as amx
if os.environ.get("AMX_LIB"):
    from amp_extensions_amd import _native
    _native.load(os.environ["AMX_LIB"])
from amp_extensions_amd import synthetic as syn
from amp_extensions_amd.ensemble import init_ensemble_weights
from amp_extensions_amd.policy import init_mlp_policy_params
from amp_extensions_amd.datasets import get_transformations
S, A = 197, 36
B = 256
dev = torch.device("cuda", 0)
role = sys.argv[1]
s, a, s2 = syn.offline(4096, S, A, 0)
norms = get_transformations(*[torch.from_numpy(x).float() for x in (s, a, s2)])
ctx = amx.AmxContext(S, A, n_models=4, hidden=512, n_hidden=4, feat_dim=512, device=dev)
ob = torch.from_numpy(syn.reset_table(B, S, 2)).to(dev)
act = torch.from_numpy(np.random.RandomState(1).randn(B, A)).to(dev)
if role == "gemm":
    ens = amx.DeviceEnsemble(ctx, init_ensemble_weights(S, A, [512] * 4, 4, 100), norms)
    Bg = int(os.environ.get("BG", "256"))
    obg = torch.from_numpy(syn.reset_table(Bg, S, 2)).to(dev); actg = torch.from_numpy(np.random.RandomState(1).randn(Bg, A)).to(dev)
    t_end = time.time() + 12
    n = 0
    while time.time() < t_end:
        for _ in range(20): ens.forward_preds(obg, actg, Bg)
        torch.cuda.synchronize(); n += 1
    print("gemm done", n, flush=True)
elif role == "torchmm":
    x = torch.randn(4096, 4096, device=dev); t_end = time.time() + 12
    while time.time() < t_end:
        for _ in range(20): y = x @ x
        torch.cuda.synchronize()
    print("mm done", flush=True)
else:
    pw, ls = init_mlp_policy_params(S, A)
    pol = amx.DevicePolicy(ctx, pw, ls, seed=5)
    pa = torch.empty(B, A, dtype=torch.float64, device=dev)
    mean = torch.empty(B, A, dtype=torch.float32, device=dev)
    time.sleep(3)
    sys.path.insert(0, "/root/repo")
    from oracle import milo_ref as R
    obn = ob.cpu().numpy()
    truth = torch.from_numpy(np.stack([R.policy_mean(pw, obn[i]) for i in range(B)])).to(dev)
    nb = 0; lanes = set(); tot = 0; worst = 0.0
    t_end = time.time() + 6
    while time.time() < t_end:
        pol.act(ob, B, pa, 3, mean_out=mean)
        torch.cuda.synchronize(); tot += 1
        err = (mean - truth).abs().amax(1)
        badl = (err > 1e-4).nonzero().flatten().tolist()
        worst = max(worst, float(err.max()))
        if badl:
            nb += 1
            for r in badl: lanes.add(r % 16)
    print("policy", "bad", nb, "of", tot, "local lanes", sorted(lanes), "worst", worst, flush=True)
