#!/bin/bash
# End-of-round measurement set (GPU box), every step under its own limit;
# outputs under gpurun_out/final_$1 (copy what is judged into profiles/).
# usage: tools/round_final.sh r05
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
tag=${1:-r05}
o=gpurun_out/final_$tag
mkdir -p $o
exec tools/gpu_run.sh \
  "600|final_gt|python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread" \
  "300|final_bench|python3 bench.py > $o/bench.log 2>&1 && tail -1 $o/bench.log" \
  "300|final_band_c3b|python3 tools/time_band.py --scene c3b --json $o/band_c3b_final.json" \
  "300|final_band_c5|python3 tools/time_band.py --scene c5 --json $o/band_c5_final.json" \
  "300|final_objects|python3 tools/time_objects.py --json $o/objects_final.json" \
  "300|final_dropin|examples/dropin_bench 5 > $o/dropin_bench.json 2>&1 && cat $o/dropin_bench.json" \
  "200|final_oprof|tools/oprof.sh sphere_1obj_avx 3 $o/oprof_sphere" \
  "200|final_oprof16|tools/oprof.sh c3b_obj16_avx 3 $o/oprof_obj16" \
  "900|final_prof|tools/profile_round.sh $tag"
