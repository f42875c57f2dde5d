"""Build recipe for libamx_hip.so (the C-ABI HIP library) — in-tree, gfx950 only.

`python -m amp_extensions_amd._build` or `__graft_entry__.build()` compiles every
`csrc/*.hip` with hipcc (one object per source, in parallel, under `build/`) and links
`amp_extensions_amd/libamx_hip.so`.  The build is incremental on source/header mtimes.  -ffp-contract=off keeps the scalar state /
termination / reward algebra rounding exactly like the reference's separate IEEE ops
(the GEMM inner loops are MFMA and are unaffected).
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
ROOT = os.path.dirname(PKG_DIR)
INCLUDE = os.path.join(ROOT, "include")
LIB_NAME = "libamx_hip.so"
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)
ARCH = os.environ.get("AMX_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    "-ffp-contract=off",
    "-Wall",
    "-Wno-pass-failed",
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (need ROCm); cannot build libamx_hip.so")


def sources() -> list[str]:
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps() -> list[str]:
    return sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def up_to_date() -> bool:
    if not os.path.exists(LIB_PATH):
        return False
    t = os.path.getmtime(LIB_PATH)
    return all(os.path.getmtime(p) <= t for p in _deps())


def _obj(src: str) -> str:
    return os.path.join(PKG_DIR, "build", os.path.basename(src)[:-4] + ".o")


def build(force: bool = False, verbose: bool = True) -> str:
    """Compile libamx_hip.so in-tree; returns its path.  Each csrc/*.hip is compiled to its
    own object in parallel (recompiled when it or any header is newer), then linked."""
    if not force and up_to_date():
        return LIB_PATH
    os.makedirs(os.path.join(PKG_DIR, "build"), exist_ok=True)
    hdr_t = max((os.path.getmtime(p) for p in _deps() if not p.endswith(".hip")), default=0.0)
    cc = [_hipcc(), *[f for f in HIPCC_FLAGS if f != "-shared"], "-I", INCLUDE, "-I", CSRC]
    procs = []
    for src in sources():
        obj = _obj(src)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_t):
            cmd = [*cc, "-c", "-o", obj + ".tmp", src]
            if verbose:
                print("[amx build]", " ".join(cmd), flush=True)
            procs.append((obj, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    errs = []
    for obj, pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            errs.append(out)
        else:
            os.replace(obj + ".tmp", obj)
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB_PATH + ".tmp",
           *[_obj(s) for s in sources()]]
    if verbose:
        print("[amx build]", " ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc link failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    os.replace(LIB_PATH + ".tmp", LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    build(force="--force" in sys.argv)
