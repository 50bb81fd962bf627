#!/bin/bash
# Interleaved A/B of library variants on pipelined band frames (tools/time_band.py).
# usage: tools/abband.sh ROUNDS SCENE NLIST lib1.so lib2.so ...   (paths under cpu-renderer_amd/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
n=$1; sc=$2; ns=$3; shift 3
for r in $(seq "$n"); do
  for l in "$@"; do
    echo "lib=$l"
    PRK_LIB=cpu-renderer_amd/$l timeout -k 10 100 python tools/time_band.py --scene $sc --n $ns --frames 50 | \
      python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); print('  N=%d ms/frame %.4f serial %s' % (d['n'], d['ms_per_frame_rank'], {k: round(v,3) for k,v in d['serial_ms'].items()}))" || exit $?
  done
done
