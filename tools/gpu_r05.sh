#!/bin/bash
# Round-5 GPU call: the GPU test suite, smoke(), the default bench line (and optionally the
# rocprofv3 profiles of the headline and of the sigma-0.05 line).  Every GPU step has its own time
# limit and the steps are chained: the first failure ends the call.
#   TAG=r05a [PROF=1] bash tools/gpu_r05.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
      -p no:cacheprovider > gpurun_out/${TAG}_pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench.err; exit $rc; }
  python3 - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("headline %.0f pairs/s  %s %.4f ms  frac %.4f  traffic_ratio %s  stages %s" % (d["value"], r["kernel"], r["avg_launch_ms"], r["frac"], r["traffic_ratio"], d["stages_ms_per_step"]))
for k in ("with_scores", "near_threshold", "realistic", "noisy_pose", "i8_allpairs", "sequence", "superpoint", "image_to_pose", "keypoints", "window_frontend"):
    v = d.get(k)
    if v: print(k, json.dumps({kk: vv for kk, vv in v.items() if kk in ("value", "ms_per_step", "stages_ms", "k_q8d_match_ms", "k_q8t_match_ms", "hbm_frac_8d", "roofline", "mfma_roofline", "hbm_roofline", "pose_ok", "rot_err_deg", "tdir_err_deg", "matches_per_pair")})[:600])
PY
fi
if [ "${PROF:-0}" = 1 ]; then
  bash tools/profile.sh ${TAG} || exit $?
  PROF_BENCH_ARGS="--steps 10 --warmup 2 --no-cpu-baseline --check 0 --noise 0.05" bash tools/profile.sh ${TAG}_nt || exit $?
fi
