#!/bin/bash
# Serial per-kernel averages (rocprofv3 --kernel-trace --stats of tools/kt.py)
# on the C3b frame, printed compactly.  usage: tools/ktprof.sh [outdir] [kt args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
o=${1:-gpurun_out/ktprof}; shift
export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o kt -- \
    python3 tools/kt.py ${@:-1000000 4096 4096 16 10} > $o.log 2>&1 || exit $?
python3 - "$o" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for x in csv.DictReader(open(f)):
    n = x['Name']
    print("%8.1f us x%4s  %s" % (float(x['AverageNs']) / 1e3, x['Calls'], n.split('(')[0][-60:]))
PY
grep "serial ms" $o.log
