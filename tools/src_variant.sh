#!/bin/bash
# Build amp_extensions_amd/libamx_hip_<tag>.so with one csrc source compiled with extra defines,
# linked with the in-tree objects of the others (A/B experiments; tools/so_ab.sh).
# usage: tools/src_variant.sh <source.hip> <tag> -DNAME=VALUE ...
set -e
src=$1; tag=$2; shift 2
cd "$(dirname "$0")/.."
python3 -c "from amp_extensions_amd import _build; _build.build(verbose=False)"
objs=$(python3 -c "from amp_extensions_amd import _build; print(' '.join(_build._obj(s) for s in _build.sources() if not s.endswith('/$src')))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-pass-failed -I include -I amp_extensions_amd/csrc "$@" \
  -c -o /tmp/amx_var_$tag.o amp_extensions_amd/csrc/$src
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o amp_extensions_amd/libamx_hip_$tag.so $objs /tmp/amx_var_$tag.o
echo "built amp_extensions_amd/libamx_hip_$tag.so"
