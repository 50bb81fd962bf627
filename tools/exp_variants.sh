#!/bin/bash
# Build libprk_hip variants (register budget) for an A/B timing run on the GPU box.
cd "$(dirname "$0")/../cpu-renderer_amd" || exit 1
for w in "$@"; do
  make -s clean >/dev/null; make -s HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -DPRK_RASTER_MIN_WAVES=$w" && mv libprk_hip.so libprk_hip_w$w.so
done
make -s clean >/dev/null; make -s
