#!/bin/bash
# image -> pose A/B: VARIANTS (build_variants/libmaveric_<name>.so; "default" = the shipping
# build), the chain's tests on the default build first, then tools/bench_image_pose.py twice,
# interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05z}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_superpoint.py tests/test_gpu_image_to_pose.py tests/test_keypoints.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in ${VARIANTS}; do
    if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
    MV_LIB=$L timeout -k 10 200 python tools/bench_image_pose.py --pipelines ${PIPES:-2} > gpurun_out/${TAG}_ip_${v}_$rep.json 2>gpurun_out/${TAG}_ip.err || exit $?
    echo "$v rep $rep: $(python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_ip_${v}_$rep.json'));print(d['value'],d['stages_ms_per_step'])")"
  done
done
