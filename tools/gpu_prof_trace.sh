set -u
bash tools/profile.sh r02a || exit $?
touch maveric-slam_amd/csrc/hip/k_allpairs_q8.hip
make -s -C maveric-slam_amd/csrc -j16 EXTRA=-DQ8_EXP_TRACE > gpurun_out/trace_build.log 2>&1 || exit 2
timeout -k 10 120 python tools/trace_q8.py > gpurun_out/trace_q8.log 2>&1; rc=$?
cat gpurun_out/trace_q8.log | tail -30
exit $rc
