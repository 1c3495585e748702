set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r3p
mkdir -p $O
export HEAT2D_PLAN_CACHE=off
timeout -k 10 400 python -u -m pytest tests/test_persistent.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "persist tests rc=$rc"; tail -4 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() { name=$1; shift; timeout -k 10 200 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -3 $O/$name.err; exit 1; }; python -c "import json; d=json.load(open('$O/$name.json')); print('$name', d['value'], d['config']['cycles'])"; }
for mode in 0 1; do
  export HEAT2D_PERSIST=$mode
  b s4096_p$mode --grid 4096 --dtype fp32 --steps 1000 --warmup 100
  b d4096_p$mode --grid 4096 --dtype fp64 --steps 1000 --warmup 100
  b s8192_p$mode --grid 8192 --dtype fp32 --steps 1000 --warmup 100
done
unset HEAT2D_PERSIST
b s4096_auto --grid 4096 --dtype fp32 --steps 1000 --warmup 100
for seg in 1536 2014; do HEAT2D_PERSIST=1 HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=$seg b s4096_p1_seg$seg --grid 4096 --dtype fp32 --steps 1000 --warmup 100; done
