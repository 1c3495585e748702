# Final tree: full GPU suite, smoke, driver bench, every BASELINE config, rehearsals, kernel-trace profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && cat $O/bench20.json || exit 1
HEAT2D_DYNAMIC=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20_static.json 2> $O/bench20_static.err && cat $O/bench20_static.json || exit 1
timeout -k 10 900 python -u bench/configs.py > $O/configs.jsonl 2> $O/configs.err || exit 1
cat $O/configs.jsonl | python -c "import sys,json; [print(d['config'], d['gpts'], d['cycles'], d['prepare_s']) for d in map(json.loads, sys.stdin)]"
timeout -k 10 200 python -u bench.py --rehearse-comm --rows 4096 --steps 20 --warmup 5 > $O/reh64_20.json 2> $O/reh64_20.err || exit 1
timeout -k 10 200 python -u bench.py --dtype fp32 --rehearse-comm --rows 4096 --steps 480 --warmup 20 > $O/reh32_480.json 2> $O/reh32_480.err || exit 1
timeout -k 10 200 python -u bench.py --gpus 4 --share-gpu --transport peer --grid 8192 --steps 40 --check > $O/ipc4.json 2> $O/ipc4.err || exit 1
timeout -k 10 200 python -u bench.py --grid 8192 --steps 40 --check > $O/ipc1.json 2> $O/ipc1.err || exit 1
for f in $O/reh64_20.json $O/reh32_480.json $O/ipc4.json $O/ipc1.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['transport'], d.get('field_stats', {}).get('sum'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err
echo "prof rc=$?"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_small -o run -- python3 $GRAFT_REPO_ROOT/bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $GRAFT_REPO_ROOT/$O/prof_small.json 2> $GRAFT_REPO_ROOT/$O/prof_small.err
echo "prof small rc=$?"
