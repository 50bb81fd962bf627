#!/bin/bash
# Build a named libprk_hip variant with extra -D flags (A/B experiments).
# usage: tools/build_variant.sh NAME "-DPRK_WAVES=1 -D..."
cd "$(dirname "$0")/../cpu-renderer_amd" || exit 1
name=$1; shift
make -s clean >/dev/null
make -s HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero $*" || exit 1
mv libprk_hip.so libprk_hip_$name.so
