#!/bin/bash
# Serial per-kernel averages of one BASELINE config (rocprofv3 --kernel-trace
# --stats of tools/frames.py).  usage: tools/fprof.sh <config> [frames] [outdir]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
c=$1; n=${2:-20}; o=${3:-gpurun_out/fprof_$1}
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o f -- \
    python3 tools/frames.py $c $n > $o.log 2>&1 || exit $?
python3 - "$o" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for x in csv.DictReader(open(f)):
    n = x['Name']
    print("%8.1f us x%4s  %s" % (float(x['AverageNs']) / 1e3, x['Calls'], n.split('(')[0][-60:]))
PY
