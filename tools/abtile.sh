#!/bin/bash
# Serial C3b stage times (tools/kt.py) of library variants at given tiles.
# usage: tools/abtile.sh "256x8 128x8" lib1.so lib2.so ...   (paths under cpu-renderer_amd/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
tiles=$1; shift
for t in $tiles; do
  for l in "$@"; do
    PRK_LIB=cpu-renderer_amd/$l timeout -k 10 100 python tools/kt.py 1000000 4096 4096 16 10 $t || exit $?
  done
done
