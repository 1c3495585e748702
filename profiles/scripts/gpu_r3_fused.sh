# Fused cycles: bitwise (IPC rank processes on one GPU) + middle-slab rehearsals.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_distributed.py -m gpu -k ipc -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "ipc/fused tests rc=$rc"; grep -E "PASS|FAIL|Error" $O/tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
export HEAT2D_PLAN_CACHE=off
run() { name=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/$name.json')); c=d['config']; print('$name', d['value'], c['cycles'], c['transport'], c['graph'], {k:(v['order'],v['ring'],v['main_bands']) for k,v in (c['launch_plans'] or {}).items()}, d.get('phase_ms'))"; }
S="--steps 20 --warmup 5 --rows 4096 --rehearse-comm"
run rccl_auto $S
HEAT2D_SPLIT_ORDER=fused run rccl_fused $S
HEAT2D_SPLIT_ORDER=fused run rccl_fused_ph $S --phase-timers
run ipc_auto $S --transport peer
HEAT2D_SPLIT_ORDER=fused run ipc_fused $S --transport peer
HEAT2D_SPLIT_ORDER=fused run ipc_fused_eager $S --transport peer --graph off
run whole20 --steps 20 --warmup 5
S32="--steps 480 --warmup 48 --rows 4096 --rehearse-comm --dtype fp32"
run rccl32_auto $S32
HEAT2D_SPLIT_ORDER=fused run rccl32_fused $S32
S480="--steps 480 --warmup 48 --rows 4096 --rehearse-comm"
run rccl480_auto $S480
HEAT2D_SPLIT_ORDER=fused run rccl480_fused $S480
