# Round-4 start tree baseline: headline, the reference's literal 25000-step run
# (CLI, auto and jacobi arithmetic), strong-scaling slab rehearsals (rccl, peer)
# and the small grid, all on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r4base
mkdir -p $O
BIN=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && cat $O/bench20.json || exit 1
mkdir -p $O/ref && cd $O/ref && printf "32768 0.25 0.05 1.0 25000 0\n" > input.dat
timeout -k 10 300 $BIN input.dat --output none --json auto.json > auto.txt 2>&1 && tail -3 auto.txt || exit 1
timeout -k 10 300 $BIN input.dat --output none --arith jacobi --json jacobi.json > jacobi.txt 2>&1 && tail -3 jacobi.txt || exit 1
cd $GRAFT_REPO_ROOT
for t in rccl peer; do
  timeout -k 10 200 python -u bench.py --rehearse-comm --transport $t --rows 4096 --steps 20 --warmup 5 > $O/reh64_$t.json 2> $O/reh64_$t.err || exit 1
  timeout -k 10 200 python -u bench.py --dtype fp32 --rehearse-comm --transport $t --rows 4096 --steps 480 --warmup 20 > $O/reh32_$t.json 2> $O/reh32_$t.err || exit 1
done
timeout -k 10 200 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_480.json 2> $O/b32_480.err || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/small_$i.json 2> $O/small_$i.err || exit 1
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['transport'], d['config']['cycles'], d['config']['prepare_s'])"; done
