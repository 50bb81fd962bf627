#!/bin/bash
# Kernel timeline of pipelined band frames (tools/time_band.py under
# rocprofv3 --kernel-trace) and its GPU-busy fraction (tools/timeline.py).
# usage: tools/band_trace.sh <scene> <N> [outdir]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
sc=$1; n=$2; o=${3:-gpurun_out/bt_${1}_$2}
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d $o -o bt -- \
    python3 tools/time_band.py --scene $sc --n $n --frames 20 > $o.log 2>&1 || exit $?
f=$(find $o -name '*kernel_trace.csv' | head -n 1)
python3 tools/timeline.py "$f" 8 3
