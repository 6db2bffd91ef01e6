bash tools/diag/r06f_extra.sh
TAG=$TAG/abw ROUNDS=2 LIBS="maveric-slam_amd/libmaveric_hip.so build_variants/libmaveric_feold.so build_variants/libmaveric_win2.so build_variants/libmaveric_win4.so" bash tools/ab_window.sh
