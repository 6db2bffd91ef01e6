#!/bin/bash
# pose kernel: GN solved per wave (PE_RSOLVE) -- parity tests, determinism under 3 streams, timing A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05p}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_pose.py tests/test_gpu_image_to_pose.py tests/test_gpu_pipeline.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
NP=3 SYNC=0 ROUNDS=8 timeout -k 10 200 python tools/dbg_pipelines.py 2>&1 | grep -v amdgpu.ids || exit 1
for rep in 1 2; do
  for v in default ${POSE_VARIANTS:-rsolve0}; do
    if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
    echo "== $v rep $rep"
    MV_LIB=$L POSE_BATCHES=8192 POSE_NOISE=1 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py 2>&1 | grep "B=" || exit 1
    MV_LIB=$L POSE_BATCHES=8192 POSE_HYPS=256 POSE_ITERS=10 timeout -k 10 200 python tools/pose_timing.py 2>&1 | grep "B=" || exit 1
  done
done
MV_LIB=build_variants/libmaveric_posetrace.so POSE_BATCHES=256 POSE_NOISE=1 POSE_HYPS=256 POSE_ITERS=10 \
  timeout -k 10 200 python tools/pose_timing.py 2>&1 | grep -m 3 "pose phases"
