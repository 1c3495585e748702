# Round 4, run C: the exchange-aware autotuner on the strong-scaling slab
# rehearsals (against the whole grid on the same box), the small grid with the
# sub-ms stage-A screening, then profiles: kernel trace + stats of the headline
# and achieved DRAM traffic (FETCH_SIZE / WRITE_SIZE) of the headline pass and
# of the sigma = 0.2 fast pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
timeout -k 10 300 python -u bench.py --steps 480 --warmup 20 --dtype fp32 > $O/b32_480.json 2> $O/b32_480.err || exit 1
for t in rccl ipc; do
  timeout -k 10 200 python -u bench.py --rehearse-comm --transport $t --rows 4096 --steps 20 --warmup 5 --phase-timers > $O/reh64_$t.json 2> $O/reh64_$t.err || exit 1
  timeout -k 10 200 python -u bench.py --dtype fp32 --rehearse-comm --transport $t --rows 4096 --steps 480 --warmup 20 > $O/reh32_$t.json 2> $O/reh32_$t.err || exit 1
done
for r in 8192 16384; do
  timeout -k 10 200 python -u bench.py --rehearse-comm --transport ipc --rows $r --steps 20 --warmup 5 > $O/reh64_ipc_$r.json 2> $O/reh64_ipc_$r.err || exit 1
done
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_$i.json 2> $O/small_$i.err || exit 1
done
python tools/summarize_json.py $O/*.json
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --verify off > $P/trace_bench.json 2> $P/trace.err || exit 1
run() {  # tag dtype n k cycles env...
  tag=$1; shift; dt=$1; n=$2; k=$3; c=$4; shift 4
  env "$@" timeout -k 10 120 python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py $dt $n $k $c 1 0 > $P/$tag.json || return 1
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env "$@" timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $P/${tag}_$ctr -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py $dt $n $k $c 1 0 > /dev/null || return 1
  done
}
run b20 fp64 32768 20 2 CP_ARITH=jacobi HEAT2D_BANDS=8 HEAT2D_TB_RING=4 HEAT2D_DYNAMIC=1 || exit 1
run fast20 fp64 32768 20 2 CP_ARITH=fast CP_SIGMA=0.2 HEAT2D_BANDS=8 HEAT2D_TB_RING=4 HEAT2D_DYNAMIC=1 || exit 1
cd $GRAFT_REPO_ROOT
for t in b20 fast20; do
  python tools/prof_summary.py hbm $P/${t}_FETCH_SIZE $P/${t}_WRITE_SIZE $P/$t.json > $P/${t}_hbm.json && echo $t && cat $P/${t}_hbm.json
  python -c "import json; d=json.load(open('$P/$t.json')); print('$t', round(d['ms']/d['cycles'],3), 'ms/cycle', round(d['gpts']), 'Gpts/s')"
done
python tools/prof_summary.py trace $P/trace > $P/trace_summary.txt; head -40 $P/trace_summary.txt
