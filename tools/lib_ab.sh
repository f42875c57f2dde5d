#!/bin/bash
# A/B of library builds (tools/src_variant.sh) on one box: for each round and each tag, install
# libamx_hip_<tag>.so as the library and run the given command; restores base at the end.
# usage: tools/lib_ab.sh "<tags>" <rounds> <cmd...>   (run on the GPU box, from the repo root)
set -e
tags=$1; rounds=$2; shift 2
cp amp_extensions_amd/libamx_hip.so /tmp/libamx_hip_orig.so
for r in $(seq 1 $rounds); do
  for t in $tags; do
    cp amp_extensions_amd/libamx_hip_$t.so amp_extensions_amd/libamx_hip.so
    echo "== $t round $r"
    timeout -k 10 120 "$@"
  done
done
cp /tmp/libamx_hip_orig.so amp_extensions_amd/libamx_hip.so
