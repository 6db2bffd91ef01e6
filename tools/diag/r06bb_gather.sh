#!/bin/bash
# the per-step result all-gather (--gather-every 1, round 5) against one per pipeline cycle (default),
# one GPU with a forced RCCL group, and without any group
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r06bb2
mkdir -p "$out"
A="--steps 20 --warmup 3 --extra-steps 0 --window-steps 0 --score-steps 0 --no-cpu-baseline --check 1"
for r in 1 2; do
  for mode in "--force-gather --gather-every 1" "--force-gather" ""; do
    tag=$(echo "x$mode" | tr -d ' -')
    timeout -k 10 300 python -u bench.py $mode $A > "$out/$tag.json" 2> "$out/$tag.err" || { tail -20 "$out/$tag.err"; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/$tag.json').read().strip().splitlines()[-1]); g=d.get('result_gather') or {}; print('round $r [$mode]', d['value'], d['ms_per_step'], 'k', d['roofline']['avg_launch_ms'], 'gathers', g.get('gathers_in_timed_steps'), g.get('steps_per_gather'))"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 240 --timeout-method thread > "$out/pytest.log" 2>&1 || { tail -30 "$out/pytest.log"; exit 1; }
tail -1 "$out/pytest.log"
