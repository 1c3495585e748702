#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/weak
timeout -k 10 300 python bench.py --weak --dtype fp32 --n 173056 --steps 64 --warmup 16 > gpurun_out/weak/w1.json 2>gpurun_out/weak/w1.err || { tail gpurun_out/weak/w1.err; exit 1; }
cat gpurun_out/weak/w1.json
# one rank of the 8-GPU weak run (global 489481^2 fp32, 61185 rows per rank), with the RCCL self-exchange rehearsal
timeout -k 10 300 python bench.py --dtype fp32 --n 489481 --rows 61186 --rehearse-comm --steps 64 --warmup 16 > gpurun_out/weak/w8rank.json 2>gpurun_out/weak/w8rank.err || { tail gpurun_out/weak/w8rank.err; exit 1; }
cat gpurun_out/weak/w8rank.json
timeout -k 10 300 python bench.py --weak --n 122368 --steps 48 --warmup 12 > gpurun_out/weak/w1_f64.json 2>gpurun_out/weak/w1f64.err || { tail gpurun_out/weak/w1f64.err; exit 1; }
cat gpurun_out/weak/w1_f64.json
