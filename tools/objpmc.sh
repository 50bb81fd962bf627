#!/bin/bash
# SQ counters of the object path's kernels (tools/time_objects.py, one case):
# two passes, summarised by tools/sqsum.py.
# usage: tools/objpmc.sh CASE [outdir]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
c=$1; o=${2:-gpurun_out/objpmc}
export TMPDIR=/tmp
mkdir -p $o
B="python3 tools/time_objects.py --frames 2 --only $c"
timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $o/sq1 -o p1 -- $B > $o/sq1.log 2>&1 || exit $?
timeout -s KILL 100 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $o/sq2 -o p2 -- $B > $o/sq2.log 2>&1 || exit $?
python3 tools/sqsum.py $o > $o/sq_summary.txt 2>&1 || exit $?
echo done
