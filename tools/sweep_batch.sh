#!/bin/bash
# bench.py knob sweep on the GPU box (headline only, no secondaries): CFGS is a ';'-separated
# list of bench.py argument sets, each run REPS times.
set -u
mkdir -p gpurun_out
IFS=';' read -ra LIST <<< "${CFGS:---batch 8192 --pipeline 2;--batch 8192 --pipeline 3}"
for rep in $(seq 1 ${REPS:-1}); do
for cfg in "${LIST[@]}"; do
  timeout -k 10 240 python bench.py $cfg --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --score-steps 0 --extra-steps 0 --window-steps 0 --check 1 > gpurun_out/sw.log 2>&1 || { tail -5 gpurun_out/sw.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]); print('$cfg', d['value'], d['ms_per_step'], d['stages_ms_per_step'])"
done
done
