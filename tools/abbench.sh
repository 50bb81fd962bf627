#!/bin/bash
# Interleaved A/B of libprk_hip variants on the bench line (pipelined frames,
# no CPU baseline).  usage: tools/abbench.sh ROUNDS name1 name2 ...  ("base" = libprk_hip.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
n=$1; shift
for r in $(seq "$n"); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=cpu-renderer_amd/libprk_hip.so; else lib=cpu-renderer_amd/libprk_hip_$v.so; fi
    PRK_LIB=$lib timeout -k 10 120 python3 bench.py --cpu-baseline 0 --steps 200 2>/dev/null | tail -1 | \
      python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v ms_per_step %.4f' % d['ms_per_step'])" || exit $?
  done
done
