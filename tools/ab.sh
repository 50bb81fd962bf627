#!/bin/bash
# A/B serial stage times of libprk_hip variants on the C3b frame (GPU box),
# interleaved twice.  usage: tools/ab.sh name1 name2 ...   ("base" = libprk_hip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
for rep in 1 2; do
for n in "$@"; do
  if [ "$n" = base ]; then lib=cpu-renderer_amd/libprk_hip.so; else lib=cpu-renderer_amd/libprk_hip_$n.so; fi
  PRK_LIB=$lib timeout -k 10 90 python tools/kt.py 1000000 4096 4096 16 10 || exit $?
done
done
