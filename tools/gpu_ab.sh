#!/bin/bash
# A/B of library builds on the headline step (and SURVEY C1 noise): each variant's bench line
# (k_q8d_match time from HIP events) one after the other on the same box, twice in alternation.
# VARIANTS: space-separated names; "ship" = maveric-slam_amd/libmaveric_hip.so, else
# build_variants/libmaveric_<name>.so.  TESTS_FOR: variants whose all-pairs GPU tests run first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
lib() { [ "$1" = ship ] && echo maveric-slam_amd/libmaveric_hip.so || echo build_variants/libmaveric_$1.so; }
for v in ${TESTS_FOR:-}; do
  MV_LIB=$(lib $v) timeout -k 10 300 python -m pytest tests/test_gpu_allpairs.py tests/test_gpu_pipeline.py -m gpu -q -x \
      --timeout 150 --timeout-method thread > gpurun_out/ab_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -3 gpurun_out/ab_tests_$v.log
  [ $rc -eq 0 ] || exit $rc
done
ARGS="--steps ${AB_STEPS:-30} --warmup 3 --extra-steps 0 --score-steps ${AB_SCORE:-0} --window-steps 0 --no-cpu-baseline --check 1"
for rep in 1 2; do
  for v in ${VARIANTS:-ship}; do
    for nz in ${AB_NOISE:-0.01875 0.05}; do
      MV_LIB=$(lib $v) timeout -k 10 200 python bench.py $ARGS --noise $nz > gpurun_out/ab_${v}_n${nz}_$rep.log 2>&1
      rc=$?
      [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 gpurun_out/ab_${v}_n${nz}_$rep.log; exit $rc; }
      python3 - "$v" "$nz" "$rep" gpurun_out/ab_${v}_n${nz}_$rep.log <<'PY'
import json, sys
v, nz, rep, f = sys.argv[1:]
d = json.loads([l for l in open(f) if l.startswith("{")][-1])
r = d["roofline"]
print("%-12s noise %-8s rep %s  %10.0f pairs/s  k_q8d %.4f ms  frac %.4f  pose %.4f%s" % (
    v, nz, rep, d["value"], r["avg_launch_ms"], r["frac"], d["stages_ms_per_step"].get("k_pose_ransac", 0),
    ("  scores %.4f ms" % d["with_scores"]["k_q8d_match_ms"]) if d.get("with_scores") else ""))
PY
    done
  done
done
