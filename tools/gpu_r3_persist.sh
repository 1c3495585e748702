set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r3p
mkdir -p $O
export HEAT2D_PLAN_CACHE=off
timeout -k 10 400 python -u -m pytest tests/test_persistent.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "persist tests rc=$rc"; tail -15 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100"
for mode in 0 1; do
  HEAT2D_PERSIST=$mode timeout -k 10 200 $B > $O/s4096_p$mode.json 2> $O/s4096_p$mode.err || exit 1; echo "persist=$mode"; cat $O/s4096_p$mode.json | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['config']['cycles'], d['config']['launch_plans'])"
done
timeout -k 10 200 $B > $O/s4096_auto.json 2> $O/s4096_auto.err || exit 1; echo auto; python -c "import json; d=json.load(open('$O/s4096_auto.json')); print(d['value'], d['config']['cycles'])"
for seg in 1007 1536 2014; do
  HEAT2D_PERSIST=1 HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=$seg timeout -k 10 200 $B > $O/s4096_p1_seg$seg.json 2> $O/s4096_p1_seg$seg.err || exit 1; echo "seg=$seg"; python -c "import json; d=json.load(open('$O/s4096_p1_seg$seg.json')); print(d['value'], d['config']['cycles'])"
done
for mode in 0 1; do
  HEAT2D_PERSIST=$mode timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 100 > $O/d4096_p$mode.json 2> $O/d4096_p$mode.err || exit 1; echo "fp64 persist=$mode"; python -c "import json; d=json.load(open('$O/d4096_p$mode.json')); print(d['value'], d['config']['cycles'])"
  HEAT2D_PERSIST=$mode timeout -k 10 200 python -u bench.py --grid 8192 --dtype fp32 --steps 1000 --warmup 100 > $O/s8192_p$mode.json 2> $O/s8192_p$mode.err || exit 1; echo "fp32 8192 persist=$mode"; python -c "import json; d=json.load(open('$O/s8192_p$mode.json')); print(d['value'], d['config']['cycles'])"
done
