#!/bin/bash
# Serial per-kernel averages of rank 0's band frame (tools/band_frames.py).
# usage: tools/bprof.sh <c3b|c5> <N> [outdir]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
o=${3:-gpurun_out/bprof_$1_$2}
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o b -- \
    python3 tools/band_frames.py $1 $2 20 > $o.log 2>&1 || exit $?
python3 - "$o" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for x in csv.DictReader(open(f)):
    print("%8.1f us (min %7.1f) x%4s  %s" % (float(x['AverageNs']) / 1e3, float(x['MinNs']) / 1e3, x['Calls'],
                                            x['Name'].split('(')[0][-50:]))
PY
