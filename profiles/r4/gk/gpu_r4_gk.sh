# Round 4, run GK: fp64 chained march (K 17..20, default) vs one chain
# (build_ab/nochain: -DHEAT2D_CHAIN_F64=0; tools/build_ab_f64.sh) with the
# r = 1/4 form — headline x3 and 16384^2 / 32768^2 per-depth tuned cycles,
# interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4gk
mkdir -p $O
NC=$GRAFT_REPO_ROOT/build_ab/nochain/libheat2d.so
for i in 1 2 3; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $O/b20_chain_$i.json 2> $O/b20_chain_$i.err || exit 1
  HEAT2D_LIB=$NC timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $O/b20_nochain_$i.json 2> $O/b20_nochain_$i.err || exit 1
done
export CP_AUTOTUNE=1 CP_TIMERS=1 CP_ARITH=jacobi
for n in 16384 32768; do
  for k in 17 18 20; do
    timeout -k 10 120 python -u tools/cycle_probe.py fp64 $n $k 6 >> $O/probe_chain.jsonl 2>> $O/probe.err || exit 1
    HEAT2D_LIB=$NC timeout -k 10 120 python -u tools/cycle_probe.py fp64 $n $k 6 >> $O/probe_nochain.jsonl 2>> $O/probe.err || exit 1
  done
done
python tools/summarize_json.py $O/*.json
