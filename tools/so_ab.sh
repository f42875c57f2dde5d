#!/bin/bash
# Alternate prebuilt libraries (amp_extensions_amd/libamx_hip_<tag>.so, built by tools/src_variant.sh)
# under one command, process by process, and restore the in-tree library at the end:
#   tools/so_ab.sh ROUNDS "tag1 tag2 ..." CMD...      (default tags: "old new")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; L=$R/amp_extensions_amd
N=$1; shift
TAGS="old new"
if [[ "$1" != python* && "$1" != bash* ]]; then TAGS=$1; shift; fi
cp $L/libamx_hip.so /tmp/libamx_hip_restore.so
for i in $(seq $N); do
  for v in $TAGS; do
    cp $L/libamx_hip_$v.so $L/libamx_hip.so && echo "== $v" && timeout -k 10 200 "$@" || { cp /tmp/libamx_hip_restore.so $L/libamx_hip.so; exit 1; }
  done
done
cp /tmp/libamx_hip_restore.so $L/libamx_hip.so
