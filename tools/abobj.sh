#!/bin/bash
# Interleaved A/B of library variants on the whole-object cases (tools/time_objects.py):
# usage: tools/abobj.sh ROUNDS CASES lib1.so lib2.so ...   (CASES comma-separated; paths under cpu-renderer_amd/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
n=$1; cases=$2; shift 2
for r in $(seq "$n"); do
  for l in "$@"; do
    echo "lib=$l"
    PRK_LIB=cpu-renderer_amd/$l timeout -k 10 200 python tools/time_objects.py --frames 5 --only "$cases" || exit $?
  done
done
