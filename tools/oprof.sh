#!/bin/bash
# Per-kernel totals of whole-object (span path) frames: rocprofv3
# --kernel-trace --stats of tools/time_objects.py on the cases named.
# usage: tools/oprof.sh CASES [frames] [outdir]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
c=$1; n=${2:-3}; o=${3:-gpurun_out/oprof}
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o f -- \
    python3 tools/time_objects.py --frames $n --only $c > $o.log 2>&1 || exit $?
cat $o.log | grep '^{'
python3 - "$o" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for x in csv.DictReader(open(f)):
    n = x['Name']
    print("%10.1f us total %8.1f us avg x%5s  %s" % (float(x['TotalDurationNs']) / 1e3, float(x['AverageNs']) / 1e3,
                                                  x['Calls'], n.split('(')[0][-60:]))
PY
