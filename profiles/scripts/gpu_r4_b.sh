# Round 4, first measured tree: GPU suite + smoke, headline, sigma = 0.2
# (fast / exact), the reference's literal 25000-step CLI run (auto = r = 1/4
# form, with and without --time-transfers), strong-scaling slab rehearsals
# (rccl, ipc) and the small grid.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4b
mkdir -p $O
BIN=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --sigma 0.2 --arith fast > $O/s02_fast.json 2> $O/s02_fast.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --sigma 0.2 > $O/s02_auto.json 2> $O/s02_auto.err || exit 1
mkdir -p $O/ref && cd $O/ref && printf "32768 0.25 0.05 1.0 25000 0\n" > input.dat
timeout -k 10 300 $BIN input.dat --output none --json auto.json > auto.txt 2>&1 && tail -4 auto.txt || exit 1
timeout -k 10 300 $BIN input.dat --output none --time-transfers --json auto_tt.json > auto_tt.txt 2>&1 && tail -4 auto_tt.txt || exit 1
timeout -k 10 300 $BIN input.dat --output none --arith fma --json fma.json > fma.txt 2>&1 && tail -3 fma.txt || exit 1
cd $GRAFT_REPO_ROOT
for t in rccl ipc; do
  timeout -k 10 200 python -u bench.py --rehearse-comm --transport $t --rows 4096 --steps 20 --warmup 5 --phase-timers > $O/reh64_$t.json 2> $O/reh64_$t.err || exit 1
  timeout -k 10 200 python -u bench.py --dtype fp32 --rehearse-comm --transport $t --rows 4096 --steps 480 --warmup 20 > $O/reh32_$t.json 2> $O/reh32_$t.err || exit 1
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_$i.json 2> $O/small_$i.err || exit 1
done
# prepare(): staged screening + prescan (new) vs the round-3 search (old), cache off
timeout -k 10 400 python -u bench.py --steps 480 --warmup 48 > $O/b480_new.json 2> $O/b480_new.err || exit 1
HEAT2D_TUNE_STAGED=0 HEAT2D_SCHED_PRESCAN=0 timeout -k 10 400 python -u bench.py --steps 480 --warmup 48 > $O/b480_old.json 2> $O/b480_old.err || exit 1
timeout -k 10 400 python -u bench/configs.py --only gpu-max-fp32 gpu-32768-fp64-s0.2 > $O/configs_new.jsonl 2> $O/configs_new.err || exit 1
python tools/summarize_json.py $O/*.json $O/*.jsonl
# thin-slab band phase: the fused cycle (band items first in the interior launch,
# exchange gated on their count) against the autotuned order, r = 1/4 kernels
for t in rccl ipc; do
  HEAT2D_SPLIT_ORDER=fused timeout -k 10 200 python -u bench.py --rehearse-comm --transport $t --rows 4096 --steps 20 --warmup 5 --phase-timers > $O/reh64_fused_$t.json 2> $O/reh64_fused_$t.err || exit 1
  HEAT2D_FUSED=1 timeout -k 10 200 python -u bench.py --rehearse-comm --transport $t --rows 4096 --steps 20 --warmup 5 > $O/reh64_fusedcand_$t.json 2> $O/reh64_fusedcand_$t.err || exit 1
done
python tools/summarize_json.py $O/reh64*.json
