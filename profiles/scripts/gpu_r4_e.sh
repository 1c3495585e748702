# Round 4, run E: why the autotuner rejects the fused cycle on the 4096-row
# middle slab (HEAT2D_TUNE_LOG rankings), and the fused cycle forced at the
# edge-first winner's shape (ring 6, 8 interior bands), balance on / off, with
# a kernel trace of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4e
mkdir -p $O
reh() {  # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --rehearse-comm --transport rccl --rows 4096 --steps 20 --warmup 5 > $O/$tag.json 2> $O/$tag.err
}
reh fcand HEAT2D_FUSED=1 HEAT2D_TUNE_LOG=1 || exit 1
reh ef HEAT2D_SPLIT_ORDER=edge-first HEAT2D_BANDS=8 HEAT2D_TB_RING=6 || exit 1
reh f8 HEAT2D_SPLIT_ORDER=fused HEAT2D_BANDS=8 HEAT2D_TB_RING=6 || exit 1
reh f8eq HEAT2D_SPLIT_ORDER=fused HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_FUSED_BALANCE=0 || exit 1
reh f10 HEAT2D_SPLIT_ORDER=fused HEAT2D_BANDS=10 HEAT2D_TB_RING=6 || exit 1
reh ef_2 HEAT2D_SPLIT_ORDER=edge-first HEAT2D_BANDS=8 HEAT2D_TB_RING=6 || exit 1
reh f8_2 HEAT2D_SPLIT_ORDER=fused HEAT2D_BANDS=8 HEAT2D_TB_RING=6 || exit 1
python tools/summarize_json.py $O/*.json
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
for b in 1 0; do
  HEAT2D_SPLIT_ORDER=fused HEAT2D_BANDS=8 HEAT2D_TB_RING=6 HEAT2D_FUSED_BALANCE=$b timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $P/tr_f8_$b -o run -- python3 $GRAFT_REPO_ROOT/bench.py --rehearse-comm --transport rccl --rows 4096 --steps 20 --warmup 5 --verify off > $P/tr_f8_$b.json 2> $P/tr_f8_$b.err || exit 1
done
cd $GRAFT_REPO_ROOT
for b in 1 0; do echo "== balance $b"; python tools/trace_tail.py $P/tr_f8_$b/run_kernel_trace.csv 6; done
grep "heat2d tune" $O/fcand.err | tail -20
