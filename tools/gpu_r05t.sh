#!/bin/bash
# k_i8t_match hand-backs: int8 parity tests, the network-descriptor timing (default / k_i8_match /
# deep rows in k_i8t), the synthetic bench line default vs the no-hand-back build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05t}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu -k "i8 or int8" \
  tests/test_gpu_allpairs.py tests/test_gpu_superpoint.py > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ab_real_i8.py 2>&1 | grep "^{" || exit 1
MV_I8_KERNEL=m timeout -k 10 200 python tools/ab_real_i8.py 2>&1 | grep "^{" || exit 1
MV_LIB=build_variants/libmaveric_i8deep.so timeout -k 10 200 python tools/ab_real_i8.py 2>&1 | grep "^{" || exit 1
for rep in 1 2; do
  for v in default i8deep; do
    if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
    MV_LIB=$L timeout -k 10 200 python tools/bench_i8.py > gpurun_out/${TAG}_i8_${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/${TAG}_i8_${v}_$rep.json') if l.startswith('{')][-1]); print('$v', $rep, d['value'], d['stages_ms'], d['mfma_roofline']['frac'])"
  done
done
