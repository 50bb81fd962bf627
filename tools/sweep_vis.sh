#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 3
for r in 1 2; do
  for l in libprk_hip.so libprk_hip_g3.so libprk_hip_g4.so libprk_hip_w8.so libprk_hip_mw5.so; do
    PRK_LIB=cpu-renderer_amd/$l timeout -k 10 100 python tools/kt.py || exit $?
  done
  for t in 128x16 512x8 256x16 128x8 512x4; do
    timeout -k 10 100 python tools/kt.py 1000000 4096 4096 16 10 $t || exit $?
  done
done
