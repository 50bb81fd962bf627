#!/bin/bash
# Round profile of the headline bench (GPU box), every step under its own
# time limit:
#   1. two PMC passes (FETCH_SIZE, WRITE_SIZE) -> profiles-style per-frame
#      traffic summary (tools/pmc_traffic.py),
#   2. two SQ counter passes (wave cycles, waits, VALU/LDS instruction counts,
#      lane utilisation) -> tools/sqsum.py summary,
#   3. the bench line (reads the traffic summary for roofline.traffic),
#   4. rocprofv3 --kernel-trace --stats of the bench (pipelined frames: the
#      kernels overlap the neighbouring frames' and their averages stretch),
#   5. rocprofv3 --kernel-trace --stats of tools/kt.py: the same C3b frame,
#      the host waiting after every frame, so each kernel's average is its
#      own serial duration (the roofline's dominant_frac is priced on it).
# Output under gpurun_out/prof_$1 (copy the summaries into profiles/).
# usage: tools/profile_round.sh r02
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
tag=${1:-r02}
o=gpurun_out/prof_$tag
mkdir -p $o
B="python3 bench.py --steps 3 --warmup 1 --cpu-baseline 0"
timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $o/pmcf -o fetch -- $B > $o/pmcf.log 2>&1 || exit $?
timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $o/pmcw -o write -- $B > $o/pmcw.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $o 4096x4096_T1000000_r16_N1 $tag profiles/pmc_traffic.json > $o/pmct.log 2>&1 || exit $?
timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $o/sq1 -o p1 -- $B > $o/sq1.log 2>&1 || exit $?
timeout -s KILL 100 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $o/sq2 -o p2 -- $B > $o/sq2.log 2>&1 || exit $?
python3 tools/sqsum.py $o --json profiles/sq_valu.json 4096x4096_T1000000_r16_N1 $tag > $o/sq_summary.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py > $o/bench.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/stats -o stats -- python3 bench.py --steps 10 --cpu-baseline 0 > $o/stats.log 2>&1 || exit $?
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $o/serial -o serial -- python3 tools/kt.py 1000000 4096 4096 16 20 > $o/serial.log 2>&1 || exit $?
cp profiles/pmc_traffic.json $o/pmc_traffic.json
cp profiles/sq_valu.json $o/sq_valu.json
echo done
