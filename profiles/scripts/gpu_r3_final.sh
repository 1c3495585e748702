# Full GPU suite, smoke, the driver's bench (20 steps), then a kernel-trace
# profile of the same bench (last: rocprofv3 may fault at its own exit).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/final
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && cat $O/bench20.json || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --arith auto > $O/bench20_fma.json 2> $O/bench20_fma.err && cat $O/bench20_fma.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$O/prof_bench.json 2> $GRAFT_REPO_ROOT/$O/prof.err
echo "prof rc=$?"
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -1 | xargs -r head -8 | cut -c1-250
