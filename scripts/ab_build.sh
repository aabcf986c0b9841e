#!/bin/bash
# Builds an A/B variant of librtamd.so with extra kernel defines into
# real-time-opencl-raytracer_amd/lib/ab/NAME/librtamd.so (travels to the GPU box; bench.py
# and the tests load it with RTAMD_LIB=...).  Usage: scripts/ab_build.sh NAME [-DKNOB=V ...]
set -e
name=$1; shift
cd "$(dirname "$0")/../real-time-opencl-raytracer_amd"
make -j8 OUT=lib/ab/$name/librtamd.so BUILD=build/ab/$name KDEFS="$*" lib/ab/$name/librtamd.so
