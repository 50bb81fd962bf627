#!/bin/bash
# A/B of runtime knobs on the C3b frame: tools/abenv.sh "VAR=a VAR=b ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
for kv in $1; do
  echo "== $kv"
  env $kv timeout -k 10 90 python tools/time_frame.py 1000000 4096 4096 16 10 ${2:-} || exit $?
done
