#!/bin/bash
# the out-of-kernel re-screen: parity + real-descriptor timing + headline A/B; then the
# concurrent-pipeline determinism probe and the pose scan
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05i}
TAG=$TAG bash tools/gpu_rescreen.sh || exit $?
NP=3 timeout -k 10 200 python tools/dbg_pipelines.py > gpurun_out/${TAG}_dbgpipe.log 2>&1 || { tail -5 gpurun_out/${TAG}_dbgpipe.log; exit 1; }
cat gpurun_out/${TAG}_dbgpipe.log | grep -v amdgpu.ids
TAG=$TAG bash tools/gpu_pose_scan.sh || exit $?
