#!/bin/bash
# One GPU call: the whole -m gpu suite, smoke(), then the default bench line (TAG names the outputs).
#   TAG=r06d bash tools/gpu_suite.sh            (EXTRA: more shell run after the bench, same rules)
set -eu -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-r06x}
mkdir -p "$out"
(while sleep 50; do date >> "$out/heartbeat"; done) &  # long steps print nothing for minutes
hb=$!
trap 'kill $hb 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$out/pytest_gpu.log" 2>&1 \
  || { tail -30 "$out/pytest_gpu.log"; exit 1; }
tail -2 "$out/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
if [ -z "${NOBENCH:-}" ]; then
  timeout -k 10 600 python -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'frac', d['roofline']['frac'], 'k', d['roofline']['avg_launch_ms'], 'secondary_errors', d.get('secondary_errors'))"
fi
if [ -n "${EXTRA:-}" ]; then bash -c "$EXTRA"; fi
