#!/bin/bash
# round 4: int8 all-pairs with integer keys (shipping) against the float screen (I8_KEYS=0
# variant): the i8 parity tests on both, then bench_i8 alternating twice on one box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
lib() { [ "$1" = ship ] && echo maveric-slam_amd/libmaveric_hip.so || echo build_variants/libmaveric_$1.so; }
for v in ${TESTS_FOR:-ship}; do
  MV_LIB=$(lib $v) timeout -k 10 300 python -m pytest tests/test_gpu_allpairs.py -m gpu -q -x -k i8 \
      --timeout 150 --timeout-method thread > gpurun_out/i8_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -3 gpurun_out/i8_tests_$v.log
  [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in ${VARIANTS:-ship}; do
    MV_LIB=$(lib $v) timeout -k 10 200 python tools/bench_i8.py --steps 20 --warmup 3 --check ${I8_CHECK:-1} --cpu-seconds 0 \
        > gpurun_out/i8_${v}_$rep.json 2> gpurun_out/i8_${v}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -5 gpurun_out/i8_${v}_$rep.err; exit $rc; }
    python3 - "$v" "$rep" gpurun_out/i8_${v}_$rep.json <<'PY'
import json, sys
v, rep, f = sys.argv[1:]
d = json.loads([l for l in open(f) if l.startswith("{")][-1])
print("%-6s rep %s  %9.0f pairs/s  %s  frac %.4f" % (v, rep, d["value"], json.dumps(d["stages_ms"]),
      d["mfma_roofline"]["frac"]))
PY
  done
done
