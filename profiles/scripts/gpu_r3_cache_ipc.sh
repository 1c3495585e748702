set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/r3c
mkdir -p $O
export HEAT2D_PLAN_CACHE=$PWD/$O/plans.txt
timeout -k 10 300 python -u -m pytest tests/test_bench_contract.py -m gpu -k plan_cache -x -v --timeout 280 --timeout-method thread > $O/cache_test.log 2>&1; echo "cache test rc=$?"; tail -3 $O/cache_test.log
# headline twice: the second run's prepare() from the cache
for i in 1 2; do timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_$i.json 2> $O/b20_$i.err || exit 1; cat $O/b20_$i.json; done
# thin-slab rehearsal (one rank of 8 at 32768^2): RCCL self-exchange, exchange of the cycle depth
timeout -k 10 300 python -u bench.py --rehearse-comm --rows 4096 --steps 20 --warmup 5 > $O/reh_f64_20.json 2> $O/reh_f64_20.err && cat $O/reh_f64_20.json
timeout -k 10 300 python -u bench.py --rehearse-comm --rows 4096 --steps 480 --warmup 48 --dtype fp32 > $O/reh_f32_480.json 2> $O/reh_f32_480.err && cat $O/reh_f32_480.json
# IPC transport, 4 processes on one GPU vs 1 rank
timeout -k 10 300 python -u bench.py --gpus 1 --grid 8192 --steps 40 --warmup 5 --check > $O/ipc1.json 2> $O/ipc1.err && cat $O/ipc1.json
timeout -k 10 300 python -u bench.py --gpus 4 --share-gpu --transport peer --grid 8192 --steps 40 --warmup 5 --check > $O/ipc4.json 2> $O/ipc4.err && cat $O/ipc4.json
timeout -k 10 300 python -u bench.py --gpus 4 --share-gpu --transport peer --grid 8192 --steps 40 --warmup 5 --check --graph off > $O/ipc4_eager.json 2> $O/ipc4_eager.err && cat $O/ipc4_eager.json
