# Round 4, run GM: frame launch first on runs without an exchange
# (HEAT2D_LEAD_SELF=1) vs the concurrent order's interior-first issue,
# interleaved: headline x4, 32768^2 fp32 480 steps x2, small grid x2; plus the
# headline-depth kernel timeline with the knob.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4gm
mkdir -p $O
for i in 1 2 3 4; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $O/b20_base_$i.json 2> $O/b20_base_$i.err || exit 1
  HEAT2D_LEAD_SELF=1 timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 > $O/b20_lead_$i.json 2> $O/b20_lead_$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_base_$i.json 2> $O/b32_base_$i.err || exit 1
  HEAT2D_LEAD_SELF=1 timeout -k 10 240 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_lead_$i.json 2> $O/b32_lead_$i.err || exit 1
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_base_$i.json 2> $O/small_base_$i.err || exit 1
  HEAT2D_LEAD_SELF=1 timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_lead_$i.json 2> $O/small_lead_$i.err || exit 1
done
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
HEAT2D_LEAD_SELF=1 CP_AUTOTUNE=1 CP_ARITH=jacobi timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $P/t_lead -o run -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp64 32768 20 6 > $P/probe_lead.json 2> $P/probe_lead.err || exit 1
f=$(ls $P/t_lead/*/run_kernel_trace.csv 2>/dev/null || ls $P/t_lead/run_kernel_trace.csv)
python3 $GRAFT_REPO_ROOT/tools/trace_tail.py $f 14 > $P/tail_lead.txt || exit 1
cd $GRAFT_REPO_ROOT && python tools/summarize_json.py $O/*.json && cat $O/tail_lead.txt
