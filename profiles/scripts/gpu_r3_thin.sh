# Thin-slab rehearsals (one rank of 8 at 32768^2): per-rank efficiency of the
# exchange schemes vs the slab alone and the whole grid (VERDICT r2 task 6).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r3t
mkdir -p $O
export HEAT2D_PLAN_CACHE=$PWD/$O/plans.txt
run() { name=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/$name.json')); c=d['config']; print('$name', d['value'], c['cycles'], c['transport'], c['graph'], {k:(v['order'],v['main_bands']) for k,v in (c['launch_plans'] or {}).items()}, d.get('phase_ms'))"; }
for dt in fp64 fp32; do
  if [ $dt = fp64 ]; then S="--steps 20 --warmup 5"; else S="--steps 480 --warmup 48"; fi
  run whole_$dt $S --dtype $dt
  run slab_$dt $S --dtype $dt --rows 4096
  run rccl_$dt $S --dtype $dt --rows 4096 --rehearse-comm
  run ipc_$dt $S --dtype $dt --rows 4096 --rehearse-comm --transport peer
  run ipc_eager_$dt $S --dtype $dt --rows 4096 --rehearse-comm --transport peer --graph off
  run rccl_ph_$dt $S --dtype $dt --rows 4096 --rehearse-comm --phase-timers
done
