#!/bin/bash
# SQ counter passes over the C3b frame (one rocprofv3 --pmc run per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
out=gpurun_out/sq; mkdir -p $out
lib=${1:-cpu-renderer_amd/libprk_hip.so}
export PRK_LIB=$lib
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-trace --output-format csv -d $out/p1 -o p1 -- python3 tools/time_frame.py 1000000 4096 4096 16 2 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d $out/p2 -o p2 -- python3 tools/time_frame.py 1000000 4096 4096 16 2 || exit $?
