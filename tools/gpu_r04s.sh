#!/bin/bash
# round 4: SuperPoint with the frames pre-resized once (SP_PRERESIZE, shipping) against each
# conv1 workgroup resizing its own tile (sp0 variant): the SuperPoint / image->pose GPU tests on
# the shipping build, then bench_superpoint alternating twice on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
lib() { [ "$1" = ship ] && echo maveric-slam_amd/libmaveric_hip.so || echo build_variants/libmaveric_$1.so; }
timeout -k 10 400 python -m pytest tests/test_gpu_superpoint.py tests/test_gpu_image_to_pose.py -m gpu -q -x \
    --timeout 200 --timeout-method thread > gpurun_out/sp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/sp_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in ${VARIANTS:-ship sp0}; do
    MV_LIB=$(lib $v) timeout -k 10 200 python tools/bench_superpoint.py --batch 64 --steps 20 --check 1 \
        > gpurun_out/sp_${v}_$rep.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 gpurun_out/sp_${v}_$rep.log; exit $rc; }
    echo "$v rep $rep: $(tail -1 gpurun_out/sp_${v}_$rep.log | cut -c1-300)"
  done
done
