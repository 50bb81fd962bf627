#!/bin/bash
# Diagnostic builds (PRK_DIAG bit flags, see prk_kernels.hip) for time splits.
cd "$(dirname "$0")/../cpu-renderer_amd" || exit 1
for dg in "$@"; do
  make -s clean >/dev/null; make -s HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -DPRK_DIAG=$dg" && mv libprk_hip.so libprk_hip_d$dg.so
done
make -s clean >/dev/null; make -s
