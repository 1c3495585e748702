# Round 4, run GL: kernel timelines of 16384^2 fp64 cycles (r = 1/4 form,
# autotuned plans) at K = 16 vs 18 — is the frame (general) kernel, 1 wave/SIMD
# from K = 17, the cycle's tail? Plus the 32768^2 K = 20 cycle for reference.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off CP_AUTOTUNE=1 CP_ARITH=jacobi
O=gpurun_out/r4gl
mkdir -p $O
P=$GRAFT_REPO_ROOT/$O
cd /tmp && export TMPDIR=/tmp
for cfg in "16384 16" "16384 18" "32768 20"; do
  set -- $cfg
  timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $P/t_$1_$2 -o run -- python3 $GRAFT_REPO_ROOT/tools/cycle_probe.py fp64 $1 $2 6 > $P/probe_$1_$2.json 2> $P/probe_$1_$2.err || exit 1
  f=$(ls $P/t_$1_$2/*/run_kernel_trace.csv 2>/dev/null || ls $P/t_$1_$2/run_kernel_trace.csv)
  python3 $GRAFT_REPO_ROOT/tools/trace_tail.py $f 14 > $P/tail_$1_$2.txt || exit 1
done
cat $P/tail_*.txt
