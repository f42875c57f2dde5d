#!/bin/bash
# Build amp_extensions_amd/libamx_hip_<tag>.so: amx_gemm.hip compiled with extra defines,
# linked with the in-tree objects of the other sources (A/B experiments; tools/rff_ab.py <tag>).
# usage: tools/gemm_variant.sh <tag> -DNAME=VALUE ...
set -e
tag=$1; shift
cd "$(dirname "$0")/.."
python3 -c "from amp_extensions_amd import _build; _build.build(verbose=False)"
objs=$(python3 -c "from amp_extensions_amd import _build; print(' '.join(_build._obj(s) for s in _build.sources() if not s.endswith('amx_gemm.hip')))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-pass-failed -I include -I amp_extensions_amd/csrc "$@" \
  -c -o /tmp/amx_gemm_$tag.o amp_extensions_amd/csrc/amx_gemm.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o amp_extensions_amd/libamx_hip_$tag.so $objs /tmp/amx_gemm_$tag.o
echo "built amp_extensions_amd/libamx_hip_$tag.so"
