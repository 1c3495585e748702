# Round 4, first measured tree: GPU suite + smoke, headline, sigma = 0.2
# (fast / exact), the reference's literal 25000-step CLI run (auto = r = 1/4
# form, with and without --time-transfers), strong-scaling slab rehearsals
# (rccl, ipc) and the small grid.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r4a
mkdir -p $O
BIN=$GRAFT_REPO_ROOT/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && cat $O/bench20.json || exit 1
# prepare(): staged screening + prescan (new) vs the exhaustive search (old), interleaved
for i in 1 2; do
  HEAT2D_TUNE_STAGED=0 HEAT2D_SCHED_PRESCAN=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_old_$i.json 2> $O/b20_old_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_new_$i.json 2> $O/b20_new_$i.err || exit 1
done
HEAT2D_TUNE_STAGED=0 HEAT2D_SCHED_PRESCAN=0 timeout -k 10 400 python -u bench.py --steps 480 --warmup 48 > $O/b480_old.json 2> $O/b480_old.err || exit 1
timeout -k 10 400 python -u bench.py --steps 480 --warmup 48 > $O/b480_new.json 2> $O/b480_new.err || exit 1
timeout -k 10 400 python -u bench/configs.py --only gpu-max-fp32 > $O/max_new.json 2> $O/max_new.err || exit 1
python tools/summarize_json.py $O/*.json
