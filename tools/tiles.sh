#!/bin/bash
# Tile-size sweep of the C3b frame (GPU box).  usage: tools/tiles.sh [lib] WxH ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
lib=cpu-renderer_amd/libprk_hip.so
for t in "$@"; do
  PRK_LIB=$lib timeout -k 10 90 python tools/time_frame.py 1000000 4096 4096 16 10 $t || exit $?
done
