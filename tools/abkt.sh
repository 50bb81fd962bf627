#!/bin/bash
# Interleaved A/B of library variants on the serial C3b frame (tools/kt.py):
# usage: tools/abkt.sh ROUNDS lib1.so lib2.so ...   (paths under cpu-renderer_amd/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
n=$1; shift
for r in $(seq "$n"); do
  for l in "$@"; do
    PRK_LIB=cpu-renderer_amd/$l timeout -k 10 100 python tools/kt.py || exit $?
  done
done
