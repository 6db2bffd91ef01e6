#!/bin/bash
# Wide-row re-screen of k_q8t_match: parity tests, SuperPoint-descriptor timing (default / q8d /
# traced), and the headline against the build without it (build_variants/libmaveric_norescreen.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_allpairs.py tests/test_gpu_image_to_pose.py > gpurun_out/${TAG}_rs_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_rs_pytest.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/${TAG}_rs_real.jsonl
timeout -k 10 200 python tools/ab_real.py >> gpurun_out/${TAG}_rs_real.jsonl 2>gpurun_out/${TAG}_rs_err.log || exit $?
MV_LIB=build_variants/libmaveric_trace.so timeout -k 10 200 python tools/ab_real.py >> gpurun_out/${TAG}_rs_real.jsonl 2>>gpurun_out/${TAG}_rs_err.log || exit $?
MV_LIB=build_variants/libmaveric_norescreen.so timeout -k 10 200 python tools/ab_real.py >> gpurun_out/${TAG}_rs_real.jsonl 2>>gpurun_out/${TAG}_rs_err.log || exit $?
cat gpurun_out/${TAG}_rs_real.jsonl
ARGS="--steps 20 --warmup 3 --extra-steps 0 --score-steps 5 --window-steps 0 --no-cpu-baseline --check 1"
for rep in 1 2; do
  for v in default norescreen; do
    f=gpurun_out/${TAG}_rs_${v}_$rep.json
    if [ $v = default ]; then timeout -k 10 200 python bench.py $ARGS > $f 2>/dev/null
    else MV_LIB=build_variants/libmaveric_$v.so timeout -k 10 200 python bench.py $ARGS > $f 2>/dev/null; fi
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
    python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['roofline']
print('$v rep $rep %10.0f pairs/s %s %.4f ms frac %.4f scores %s' % (d['value'], r['kernel'], r['avg_launch_ms'], r['frac'], (d.get('with_scores') or {}).get('value')))"
  done
done
