#!/bin/bash
# A/B timing of libprk_hip variants on the C3b frame (GPU box).
# usage: tools/ab.sh name1 name2 ...   ("base" = libprk_hip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
for n in "$@"; do
  if [ "$n" = base ]; then lib=cpu-renderer_amd/libprk_hip.so; else lib=cpu-renderer_amd/libprk_hip_$n.so; fi
  PRK_LIB=$lib timeout -k 10 90 python tools/time_frame.py 1000000 4096 4096 16 10 || exit $?
done
