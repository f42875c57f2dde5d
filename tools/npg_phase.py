"""Where the NPG pass kernel's time goes: variants of csrc/amx_npg.hip built with phases
compiled out (-DNPG_PHASES=mask; the results of a partial variant are meaningless, only its
time is read), each timed in its own process on the same 40 960 x 197 rollout.

usage:
  python tools/npg_phase.py build            # here (CPU): tools/_npgvar/libamx_hip_<mask>.so
  python tools/npg_phase.py run [N S A]      # on the GPU box: one process per variant
  python tools/npg_phase.py time LIB N S A   # (internal) time one variant
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tools", "_npgvar")
# input dtype of the timed passes: float32 (DeviceNPG casts once per update; 64-row chunks) or
# NPG_IN=f64 (the C-ABI's fp64 path, 32-row chunks)
_F64 = os.environ.get("NPG_IN", "f32") == "f64"


def IN_CODE(NP):
    return NP.N.AMX_IN_F64 if _F64 else NP.N.AMX_IN_F32


def _in_dt():
    import torch
    return torch.float64 if _F64 else torch.float32
MASKS = {
    0x7F: "all phases",
    0x40: "chunk loads only",
    0x41: "loads + layer 1",
    0x47: "loads + forward (layers 1-3)",
    0x4F: "loads + forward + bp layer 3",
    0x5F: "loads + forward + bp layers 3, 2",
    0x3F: "all compute, no chunk loads",
    0x00: "nothing (launch, parameters, partial writes)",
}


def build():
    from amp_extensions_amd import _build as B
    B.build(verbose=False)
    os.makedirs(OUT, exist_ok=True)
    objs = [os.path.join(ROOT, "amp_extensions_amd", "build", f) for f in
            sorted(os.listdir(os.path.join(ROOT, "amp_extensions_amd", "build"))) if f.endswith(".o") and f != "amx_npg.o"]
    flags = [f for f in B.HIPCC_FLAGS if f != "-shared"]
    for m in MASKS:
        o = os.path.join(OUT, f"amx_npg_{m:02x}.o")
        subprocess.run([B._hipcc(), *flags, f"-DNPG_PHASES={m}", "-I", B.INCLUDE, "-c", "-o", o,
                        os.path.join(ROOT, "amp_extensions_amd", "csrc", "amx_npg.hip")], check=True)
        subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o",
                        os.path.join(OUT, f"libamx_hip_{m:02x}.so"), *objs, o], check=True)
        print("built", m)
    o = os.path.join(OUT, "amx_npg_trace.o")
    subprocess.run([B._hipcc(), *flags, "-DNPG_TRACE", "-I", B.INCLUDE, "-c", "-o", o,
                    os.path.join(ROOT, "amp_extensions_amd", "csrc", "amx_npg.hip")], check=True)
    subprocess.run([B._hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o",
                    os.path.join(OUT, "libamx_hip_trace.so"), *objs, o], check=True)
    for f in os.listdir(OUT):
        if f.endswith(".o"):
            os.remove(os.path.join(OUT, f))


def time_one(lib, N, S, A):
    import numpy as np
    import torch
    from amp_extensions_amd import _build as B
    B.LIB_PATH = lib
    import amp_extensions_amd as amx
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd import npg as NP
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    rs = np.random.RandomState(0)
    obs = torch.from_numpy(0.5 * rs.randn(N, S)).cuda().to(_in_dt())
    act = torch.from_numpy(rs.randn(N, A)).cuda().to(_in_dt())
    adv = torch.from_numpy(rs.randn(N)).cuda()
    ctx = amx.AmxContext(S, A, n_models=1, hidden=128, n_hidden=1, device="cuda")
    npg = amx.DeviceNPG(ctx, layers, ls)
    vec = torch.randn(npg.P, device="cuda", dtype=torch.float32)
    rpb = npg._rows_per_block(N)
    nb = (N + rpb - 1) // rpb
    part = torch.empty(nb, npg.P, dtype=torch.float64, device="cuda")
    res = {}
    for mode, name in ((NP.NPG_FVP, "fvp"), (NP.NPG_VPG, "vpg"), (NP.NPG_EVAL, "eval")):
        def call():
            NP.N.check(ctx.lib.amx_npg_pass(ctx.h, mode, N, obs.data_ptr(), IN_CODE(NP), obs.stride(0),
                                            act.data_ptr(), IN_CODE(NP), act.stride(0), adv.data_ptr(),
                                            npg.theta.data_ptr(), vec.data_ptr(), rpb, part.data_ptr(),
                                            ctx.stream), "amx_npg_pass")
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            call()
        e1.record()
        torch.cuda.synchronize()
        res[name] = e0.elapsed_time(e1) / 20 * 1e3
    if IN_CODE(NP) == NP.N.AMX_IN_F32 and hasattr(ctx.lib, "amx_npg_pass_ex"):
        # the FVP pass reading the theta forward a VPG pass cached (amx_npg_pass_ex)
        hc = torch.empty(N, 64, dtype=torch.float32, device="cuda")
        def ex(mode, h):
            NP.N.check(ctx.lib.amx_npg_pass_ex(ctx.h, mode, N, obs.data_ptr(), IN_CODE(NP), obs.stride(0),
                                               act.data_ptr(), IN_CODE(NP), act.stride(0), adv.data_ptr(),
                                               npg.theta.data_ptr(), vec.data_ptr(), rpb, part.data_ptr(), None,
                                               h.data_ptr(), ctx.stream), "amx_npg_pass_ex")
        ex(NP.NPG_VPG, hc)
        for _ in range(3):
            ex(NP.NPG_FVP, hc)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ex(NP.NPG_FVP, hc)
        e1.record()
        torch.cuda.synchronize()
        res["fvp_cached"] = e0.elapsed_time(e1) / 20 * 1e3
    print(" ".join(f"{k} {v:7.1f} us" for k, v in res.items()))


def trace(N, S, A, mode_name="fvp"):
    """Per-phase wall time (device realtime clock, 100 MHz) of blocks 0, 64, 128, 255."""
    import ctypes as C
    import numpy as np
    import torch
    from amp_extensions_amd import _build as B
    B.LIB_PATH = os.path.join(OUT, "libamx_hip_trace.so")
    import amp_extensions_amd as amx
    from amp_extensions_amd.policy import init_mlp_policy_params
    from amp_extensions_amd import npg as NP
    layers, ls = init_mlp_policy_params(S, A, (32, 32), seed=100, init_log_std=-0.25)
    rs = np.random.RandomState(0)
    obs = torch.from_numpy(0.5 * rs.randn(N, S)).cuda().to(_in_dt())
    act = torch.from_numpy(rs.randn(N, A)).cuda().to(_in_dt())
    adv = torch.from_numpy(rs.randn(N)).cuda()
    ctx = amx.AmxContext(S, A, n_models=1, hidden=128, n_hidden=1, device="cuda")
    npg = amx.DeviceNPG(ctx, layers, ls)
    vec = torch.randn(npg.P, device="cuda", dtype=torch.float32)
    rpb = npg._rows_per_block(N)
    part = torch.empty((N + rpb - 1) // rpb, npg.P, dtype=torch.float64, device="cuda")
    mode = {"fvp": NP.NPG_FVP, "vpg": NP.NPG_VPG, "eval": NP.NPG_EVAL, "fvp_cached": NP.NPG_FVP}[mode_name]
    hc = torch.empty(N, 64, dtype=torch.float32, device="cuda") if mode_name == "fvp_cached" else None
    if hc is not None:  # the VPG pass writes the theta forward the cached FVP reads
        NP.N.check(ctx.lib.amx_npg_pass_ex(ctx.h, NP.NPG_VPG, N, obs.data_ptr(), IN_CODE(NP), obs.stride(0),
                                           act.data_ptr(), IN_CODE(NP), act.stride(0), adv.data_ptr(),
                                           npg.theta.data_ptr(), vec.data_ptr(), rpb, part.data_ptr(), None,
                                           hc.data_ptr(), ctx.stream))
    for _ in range(4):
        NP.N.check(ctx.lib.amx_npg_pass_ex(ctx.h, mode, N, obs.data_ptr(), IN_CODE(NP), obs.stride(0),
                                           act.data_ptr(), IN_CODE(NP), act.stride(0), adv.data_ptr(),
                                           npg.theta.data_ptr(), vec.data_ptr(), rpb, part.data_ptr(), None,
                                           None if hc is None else hc.data_ptr(), ctx.stream))
    torch.cuda.synchronize()
    buf = (C.c_ulonglong * 256)()
    ctx.lib.amx_npg_trace_read.argtypes = [C.c_void_p]
    assert ctx.lib.amx_npg_trace_read(buf) == 0
    tr = np.array(buf, dtype=np.int64).reshape(4, 64)
    names = ["stash", "layer1", "layer2", "out", "bp3", "bp2", "bp1(w0)", "barrier"]
    rc = 32
    nch = (rpb + rc - 1) // rc
    print(f"{mode_name}: N={N} S={S} A={A}, {nch} chunks per block; microseconds (100 MHz clock)")
    for bi, blk in enumerate((0, 64, 128, 255)):
        t = tr[bi]
        t0 = t[0]
        rows = [f"setup {(t[2] - t0) / 100:5.2f} (" + " ".join(f"{(t[k] - t0) / 100:.2f}" for k in range(50, 56)) + ")"]
        per = np.zeros(8)
        for c in range(nch):
            st = [t[2 + 8 * c + k] for k in range(8)]
            nxt = t[2 + 8 * (c + 1)] if c + 1 < nch else t[1]
            seq = st + [nxt]
            for k in range(8):
                if seq[k + 1] and seq[k]:
                    per[k] += (seq[k + 1] - seq[k]) / 100
        rows += [f"{n} {v:5.2f}" for n, v in zip(names, per)]
        rows.append("chunks " + "/".join(f"{((t[2 + 8 * (c + 1)] if c + 1 < nch else t[1]) - t[2 + 8 * c]) / 100:.2f}"
                                         for c in range(nch)))
        rows.append(f"tail {(t[63] - t[1]) / 100:5.2f}")
        rows.append(f"total {(t[63] - t0) / 100:6.2f}")
        print(f"  block {blk:3d}: " + ", ".join(rows))


def run(N, S, A):
    print(f"NPG pass variants, N={N} S={S} A={A} ({'fp64' if _F64 else 'fp32'} inputs), average of 20 back-to-back launches")
    for m, what in MASKS.items():
        lib = os.path.join(OUT, f"libamx_hip_{m:02x}.so")
        r = subprocess.run([sys.executable, __file__, "time", lib, str(N), str(S), str(A)], capture_output=True,
                           text=True, timeout=120)
        line = r.stdout.strip().splitlines()[-1] if r.returncode == 0 and r.stdout.strip() else \
            f"failed ({r.returncode}): {r.stderr[-300:]}"
        print(f"  0x{m:02x} {what:46s} {line}", flush=True)


if __name__ == "__main__":
    cmd = sys.argv[1] if len(sys.argv) > 1 else "run"
    if cmd == "build":
        build()
    elif cmd == "trace":
        args = [int(x) for x in sys.argv[2:5]] or [40960, 197, 36]
        for m in ("fvp", "fvp_cached", "vpg", "eval"):
            trace(*args, mode_name=m)
    elif cmd == "time":
        time_one(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
    else:
        args = [int(x) for x in sys.argv[2:5]] or [40960, 197, 36]
        run(*args)
