#!/bin/bash
# Build a variant of libmaveric_hip.so (extra compile flags) beside the shipping build, on the CPU:
#   tools/build_variant.sh NAME "-DMV_TRACE ..."  ->  build_variants/libmaveric_NAME.so
# Load it with MV_LIB=build_variants/libmaveric_NAME.so (mvtrack.LIB_PATH).
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p build_variants
make -s -C maveric-slam_amd/csrc -j8 EXTRA="$*" OUT="$PWD/build_variants/libmaveric_$name.so" \
    OBJDIR="$PWD/build_variants/obj_$name"
echo "build_variants/libmaveric_$name.so"
