#!/bin/bash
cd "${GRAFT_REPO_ROOT}" || exit 3
for v in base mw3; do
  if [ "$v" = base ]; then lib=cpu-renderer_amd/libprk_hip.so; else lib=cpu-renderer_amd/libprk_hip_$v.so; fi
  o=gpurun_out/pmcvar_$v; mkdir -p $o
  PRK_LIB=$lib timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $o/pmcf -o fetch -- python3 tools/time_frame.py 1000000 4096 4096 16 3 > $o/f.log 2>&1 || exit $?
  PRK_LIB=$lib timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $o/pmcw -o write -- python3 tools/time_frame.py 1000000 4096 4096 16 3 > $o/w.log 2>&1 || exit $?
  python3 tools/pmc_traffic.py $o x $o/t.json > $o/t.log 2>&1 || exit $?
done
