#!/bin/bash
# A/B library of the fp64 kernels: build_ab_f64.sh NAME "EXTRA FLAGS"
# Recompiles the fp64 tb_kernel units with the extra flags into build_ab/NAME/ and links them
# with the default build's other objects (make all first). Load it with HEAT2D_LIB=build_ab/NAME/libheat2d.so.
set -e
cd "$(dirname "$0")/../cuda-hip-mpi-heat-equation-test_amd/csrc"
NAME=$1; FLAGS=$2
D=../../build_ab/$NAME; mkdir -p $D/obj
HIPCC=/opt/rocm/bin/hipcc
CF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -I/opt/rocm/include -Wall -Wno-unused-function -munsafe-fp-atomics $FLAGS"
ls kernels/tb_f64_*.hip | xargs -P 8 -I{} sh -c "$HIPCC $CF -c {} -o $D/obj/\$(basename {} .hip).o"
OTHERS=$(ls ../_native/obj/kernels/*.o ../_native/obj/runtime/*.o ../_native/obj/cpu/*.o ../_native/obj/capi/*.o | grep -v '/tb_f64_')
$HIPCC --offload-arch=gfx950 -shared -o $D/libheat2d.so $OTHERS $D/obj/*.o -L/opt/rocm/lib -lamdhip64 -lrccl \
  -lrocprofiler-sdk-roctx -lhiprtc -lpthread -Wl,-rpath,/opt/rocm/lib
echo built $D/libheat2d.so
