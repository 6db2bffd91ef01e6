#!/bin/bash
# the multi-rank bench path on one GPU: (a) 2 ranks over gloo sharing the device, (b) one rank with
# the RCCL group and the per-step result all-gather forced (--force-gather)
set -u -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r06bb
mkdir -p "$out"
A="--steps 5 --warmup 1 --extra-steps 0 --window-steps 0 --score-steps 0 --no-cpu-baseline --check 1"
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo $A > "$out/gloo2.json" 2> "$out/gloo2.err" || { tail -20 "$out/gloo2.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$out/gloo2.json').read().strip().splitlines()[-1]); print('gloo x2:', d['value'], d['n_gpus'], json.dumps(d.get('result_gather'))[:400])"
timeout -k 10 300 python -u bench.py --force-gather $A > "$out/nccl1.json" 2> "$out/nccl1.err" || { tail -20 "$out/nccl1.err"; exit 1; }
python3 -c "import json; d=json.loads(open('$out/nccl1.json').read().strip().splitlines()[-1]); print('nccl x1 forced gather:', d['value'], d['n_gpus'], json.dumps(d.get('result_gather'))[:400])"
