#!/bin/bash
# Variant x tile grid on the C3b frame (GPU box).  usage: tools/abt.sh "v1 v2" "t1 t2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
for n in $1; do
  if [ "$n" = base ]; then lib=cpu-renderer_amd/libprk_hip.so; else lib=cpu-renderer_amd/libprk_hip_$n.so; fi
  for t in $2; do
    PRK_LIB=$lib timeout -k 10 90 python tools/time_frame.py 1000000 4096 4096 16 10 $t || exit $?
  done
done
