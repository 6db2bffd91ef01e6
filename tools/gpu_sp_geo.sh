#!/bin/bash
# SuperPoint 24 x 16 tiles for the 24 x 80 layers (SP_GEO): parity tests, then frames/s and the
# image -> pose line against the 16 x 32-only build (build_variants/libmaveric_spgeo0.so), twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_superpoint.py tests/test_gpu_image_to_pose.py > gpurun_out/${TAG}_geo_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_geo_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in default spgeo0 ${EXTRA_VARIANTS:-}; do
    if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
    MV_LIB=$L timeout -k 10 200 python tools/bench_superpoint.py --batch 64 --steps 10 --check 0 > gpurun_out/${TAG}_geo_sp_${v}_$rep.log 2>&1 || exit $?
    echo "$v rep $rep superpoint: $(tail -1 gpurun_out/${TAG}_geo_sp_${v}_$rep.log | cut -c1-300)"
  done
done
for pl in 1 2 3; do
  timeout -k 10 200 python tools/bench_image_pose.py --pipelines $pl > gpurun_out/${TAG}_geo_image_pose_p$pl.json 2>gpurun_out/${TAG}_geo_image_pose.err || exit $?
  cat gpurun_out/${TAG}_geo_image_pose_p$pl.json
done
