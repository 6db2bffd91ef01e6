set -eu -o pipefail
bash tools/diag/r06d_sensitivity.sh
TAG=r06d_ab LIBS="maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_apipe.so" ROUNDS=2 bash tools/ab_libs.sh
TAG=r06e_window bash tools/gpu_window_prof.sh
