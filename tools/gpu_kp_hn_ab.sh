set -u
for v in kptrace kptrace8; do
  echo "$v chain: $(MV_LIB=build_variants/libmaveric_$v.so timeout -k 10 120 python tools/bench_image_pose.py --steps 1 --warmup 0 --check 0 --pipelines 1 2>&1 | grep 'nms phases' | head -1)"
  echo "$v fullres: $(MV_LIB=build_variants/libmaveric_$v.so timeout -k 10 120 python tools/bench_keypoints.py --batch 64 --steps 1 --warmup 0 --check 0 2>&1 | grep 'nms phases' | head -1)"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_keypoints.py tests/test_gpu_image_to_pose.py 2>&1 | tail -1 || exit 1
for rep in 1 2; do for v in default kphn8; do
  if [ $v = default ]; then L=""; else L="build_variants/libmaveric_$v.so"; fi
  echo "$v $rep ip: $(MV_LIB=$L timeout -k 10 200 python tools/bench_image_pose.py --check 0 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["stages_ms_per_step"]["k_kp_nms"])')"
  echo "$v $rep kp: $(MV_LIB=$L timeout -k 10 200 python tools/bench_keypoints.py --batch 1024 --steps 10 --check 0 | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["stages_ms"]["k_kp_nms"])')"
done; done
