import sys, os, ctypes
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from amp_extensions_amd import _native as N, _build
import amp_extensions_amd as amx
res = {}
for tag in sys.argv[1:]:
    path = _build.LIB_PATH if tag == "base" else _build.LIB_PATH.replace(".so", f"_{tag}.so")
    lib = N.load(path)
    rows = int(os.environ.get("RFF_ROWS", "40960"))
    S = 197
    K = int(os.environ.get("RFF_K", "416")); KV = min(394, K)
    ctx_h = lib.amx_create(0, S, 1, 1, 128, 0, 512)
    dev = "cuda"
    torch.manual_seed(0)
    x = (0.5 * torch.randn(rows, K, device=dev)); x[:, KV:] = 0
    W = torch.rand(512, K, device=dev) / 14.0; W[:, KV:] = 0
    b = (torch.rand(512, device=dev) - 0.5) * 6.28
    W2 = torch.empty(512 * 2 * K, dtype=torch.int16, device=dev); wexp = torch.empty(512, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    assert lib.amx_split_f16x2(ctx_h, 1, 512, K, W.data_ptr(), K, 0, W2.data_ptr(), 512 * 2 * K, wexp.data_ptr(), 512, st) == 0
    rexp = torch.empty(rows, dtype=torch.int32, device=dev)
    assert lib.amx_row_exponents(ctx_h, 1, rows, K, x.data_ptr(), K, 0, rexp.data_ptr(), rows, 1, st) == 0
    phi = torch.empty(rows, 512, device=dev); part = torch.empty(rows // 32, 512, dtype=torch.float64, device=dev)
    def run():
        assert lib.amx_rff_features_h3(ctx_h, rows, rows, 512, K, x.data_ptr(), K, W2.data_ptr(), wexp.data_ptr(),
                                       rexp.data_ptr(), b.data_ptr(), ctypes.c_float(0.0625), phi.data_ptr(), 512,
                                       part.data_ptr(), None, st) == 0
    for _ in range(5): run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(20):
        e0.record(); run(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1) * 1e3)
    print(f"{tag:8s} rff_features_h3 {rows} rows K {K}: median {np.median(ts):.1f} us, min {min(ts):.1f}; "
          f"phi sum {phi.double().sum().item():.17g} partials sum {part.sum().item():.17g}", flush=True)
