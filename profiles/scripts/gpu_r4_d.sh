# Round 4, run D: GPU suite + smoke on the fused-cycle rewrite (band items
# first, the interior's short bands last), the headline, and the 4096-row
# middle-slab rehearsals (fp64 20 steps, fp32 480 steps) per order: the
# autotuner's default, fused candidates admitted (HEAT2D_FUSED=1), fused forced
# with and without the short-band balance; kernel traces of one rehearsal per order.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
reh() {  # tag transport dtype steps env...
  tag=$1; t=$2; dt=$3; st=$4; shift 4
  env "$@" timeout -k 10 200 python -u bench.py --dtype $dt --rehearse-comm --transport $t --rows 4096 --steps $st --warmup 5 > $O/$tag.json 2> $O/$tag.err
}
for t in rccl ipc; do
  reh r64_${t}_auto $t fp64 20 || exit 1
  reh r64_${t}_fcand $t fp64 20 HEAT2D_FUSED=1 || exit 1
  reh r64_${t}_fused $t fp64 20 HEAT2D_SPLIT_ORDER=fused || exit 1
  reh r64_${t}_fused_eq $t fp64 20 HEAT2D_SPLIT_ORDER=fused HEAT2D_FUSED_BALANCE=0 || exit 1
done
reh r32_rccl_auto rccl fp32 480 || exit 1
reh r32_rccl_fcand rccl fp32 480 HEAT2D_FUSED=1 || exit 1
reh r64_rccl_auto_2 rccl fp64 20 || exit 1
reh r64_rccl_fused_2 rccl fp64 20 HEAT2D_SPLIT_ORDER=fused || exit 1
python tools/summarize_json.py $O/*.json
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
for o in edge-first fused; do
  HEAT2D_SPLIT_ORDER=$o timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $P/tr_$o -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rehearse-comm --transport rccl --rows 4096 --steps 20 --warmup 5 --verify off > $P/tr_$o.json 2> $P/tr_$o.err || exit 1
done
echo done
