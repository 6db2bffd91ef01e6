#!/bin/bash
# A/B on one box: the one-workgroup-per-pair k_q8t_match (default) against k_q8d_match
# (MV_Q8_KERNEL=d), headline data and SURVEY C1 noise, twice in alternation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
ARGS="--steps ${AB_STEPS:-20} --warmup 3 --extra-steps 0 --score-steps ${AB_SCORE:-5} --window-steps 0 --no-cpu-baseline --check 1"
for rep in 1 2; do
  for k in t d; do
    for nz in 0.01875 0.05; do
      f=gpurun_out/${TAG}_ab_${k}_n${nz}_$rep.json
      if [ $k = d ]; then MV_Q8_KERNEL=d timeout -k 10 200 python bench.py $ARGS --noise $nz > $f 2>/dev/null
      else timeout -k 10 200 python bench.py $ARGS --noise $nz > $f 2>/dev/null; fi
      rc=$?; [ $rc -eq 0 ] || { echo "bench $k $nz rc=$rc"; exit $rc; }
      python3 - $k $nz $rep $f <<'PY'
import json, sys
k, nz, rep, f = sys.argv[1:]
d = json.loads([l for l in open(f) if l.startswith("{")][-1])
r = d["roofline"]
ws = d.get("with_scores") or {}
print("%s noise %-8s rep %s  %10.0f pairs/s  %s %.4f ms  frac %.4f  scores %s" % (
    k, nz, rep, d["value"], r["kernel"], r["avg_launch_ms"], r["frac"],
    {kk: vv for kk, vv in ws.items() if kk.endswith("_ms")}))
PY
    done
  done
done
