#!/bin/bash
# Round profile of the headline bench (GPU box): the two PMC passes
# (FETCH_SIZE, WRITE_SIZE) -> profiles-style traffic summary, then the bench
# line (which reads that summary for roofline.traffic), then rocprofv3 kernel
# stats.  Output under gpurun_out/prof_$1 (copy the summaries into profiles/).
# usage: tools/profile_round.sh r01
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
tag=${1:-r01}
o=gpurun_out/prof_$tag
mkdir -p $o
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $o/pmcf -o fetch -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $o/pmcf.log 2>&1 || exit $?
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $o/pmcw -o write -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $o/pmcw.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $o 4096x4096_T1000000_r16_N1 profiles/pmc_traffic.json > $o/pmct.log 2>&1 || exit $?
timeout -k 10 200 python3 bench.py > $o/bench.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o stats -- python3 bench.py --steps 10 --cpu-baseline 0 > $o/stats.log 2>&1 || exit $?
cp profiles/pmc_traffic.json $o/pmc_traffic.json
echo done
