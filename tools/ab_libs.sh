#!/bin/bash
# A/B of library builds on one box: LIBS="a.so b.so" (default build = maveric-slam_amd/libmaveric_hip.so),
# each run ROUNDS times interleaved (ABAB...) with the same short bench command; prints value and the
# dominant kernel's time per run.  ARGS: bench.py arguments.
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-ab}
mkdir -p "$out"
ARGS=${ARGS:-"--steps 20 --warmup 3 --no-cpu-baseline --check 1 --extra-steps 0 --window-steps 0 --score-steps 0"}
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in ${LIBS}; do
    n=$(basename $lib .so)
    MV_LIB=$lib timeout -k 10 300 python -u bench.py $ARGS > "$out/${n}_$r.json" 2> "$out/${n}_$r.err"
    python3 -c "import json; d=json.loads(open('$out/${n}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', 'round $r', d['value'], 'k %.4f ms frac %.4f' % (r['avg_launch_ms'], r['frac']), 'pose', d['stages_ms_per_step'].get('k_pose_ransac'))" | tee -a "$out/summary.log"
  done
done
