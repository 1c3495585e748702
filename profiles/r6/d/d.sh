#!/bin/bash
# r6 run D: VERDICT r5 item 3 (host abort) under host AddressSanitizer, and
# item 2's host share of a one-cycle timed step: the first step after
# prepare() with the HSA runtime's interrupt-driven waits (default) against
# busy-polled waits (HSA_ENABLE_INTERRUPT=0), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6d
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }

# (1) host share of the one-cycle step
for i in 1 2; do
  for v in default nointr; do
    if [ $v = nointr ]; then export HSA_ENABLE_INTERRUPT=0; else unset HSA_ENABLE_INTERRUPT; fi
    timeout -k 10 200 python3 $R/tools/first_step.py --transport rccl --rows 4096 --reps 6 --json $O/fs_${v}_$i.json > /dev/null 2> $O/fs_${v}_$i.err
    rc=$?; echo "first_step $v $i rc=$rc"; fatal $rc
    b slab_${v}_$i --rehearse-comm --rows 4096 --steps 20 --warmup 5 --transport rccl
    b whole_${v}_$i --steps 20 --warmup 5 --field-check off
  done
done
export HSA_ENABLE_INTERRUPT=0
b share2_nointr --gpus 2 --share-gpu --grid 8192 --steps 20 --warmup 5 --check
unset HSA_ENABLE_INTERRUPT

# (2) VERDICT r5 item 3: the 1-GPU and shared-GPU bench --check paths (where the
# round-5 host abort "free(): invalid pointer" happened once) under host
# AddressSanitizer: an interpreter with ASan's runtime linked in and the
# library's host code instrumented (csrc/Makefile asan-python); every malloc /
# free of the process goes through ASan's allocator, device code is not
# instrumented (host sanitizers only on this pool)
A=$R/cuda-hip-mpi-heat-equation-test_amd/_native/asan
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:exitcode=99:protect_shadow_gap=0 PYTHONMALLOC=malloc HEAT2D_LIB=$A/libheat2d.so
for i in 1 2; do
  timeout -k 10 400 $A/python $R/bench.py --grid 8192 --steps 20 --warmup 5 --check > $O/asan1_$i.json 2> $O/asan1_$i.err
  rc=$?; echo "asan 1-gpu $i rc=$rc $(grep -c AddressSanitizer $O/asan1_$i.err) asan reports"; fatal $rc
  timeout -k 10 400 $A/python $R/bench.py --gpus 4 --share-gpu --grid 8192 --steps 20 --warmup 5 --check > $O/asan4_$i.json 2> $O/asan4_$i.err
  rc=$?; echo "asan share4 $i rc=$rc $(grep -c AddressSanitizer $O/asan4_$i.err) asan reports"; fatal $rc
done
echo done
