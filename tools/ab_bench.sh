#!/bin/bash
# A/B timing of kernel builds: ab_bench.sh OUTFILE "LIB1 LIB2 ..." "ARGS1;ARGS2;..."
# each (lib, args) pair is one bench.py process under its own time limit.
out=$1; libs=$2; IFS=';' read -ra argsets <<< "$3"
mkdir -p gpurun_out
for a in "${argsets[@]}"; do
  for l in $libs; do
    if [ "$l" = default ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$l; fi
    echo "== lib=$l args=$a" >> "$out"
    timeout -k 10 120 python bench.py $a >> "$out" 2>&1 || { echo "FAILED rc=$?" >> "$out"; exit 1; }
  done
done
