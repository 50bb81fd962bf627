#!/bin/bash
# Build a named libprk_hip variant with extra -D flags on the raster kernels
# (A/B experiments): cpu-renderer_amd/libprk_hip_NAME.so
# usage: tools/build_variant.sh NAME "-DPRK_WAVES=1 -D..."
cd "$(dirname "$0")/../cpu-renderer_amd" || exit 1
name=$1; shift
make -s variant NAME="$name" VARIANT="$*"
