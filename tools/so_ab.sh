#!/bin/bash
# Alternate two prebuilt libraries (amp_extensions_amd/libamx_hip_{old,new}.so) under one command,
# process by process: usage tools/so_ab.sh ROUNDS CMD...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
N=$1; shift
for i in $(seq $N); do
  for v in old new; do
    cp $L/libamx_hip_$v.so $L/libamx_hip.so && echo "== $v" && timeout -k 10 200 "$@" || exit 1
  done
done
