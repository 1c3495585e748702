#!/bin/bash
# Round-end state of this session's tree: GPU suite, smoke, the driver's bench command (plain and under torchrun
# with one rank, as the scaling driver launches it), and bench.py --gpus 2 on a 1-GPU box (must refuse, rc 2).
set -o pipefail
O=gpurun_out/s3final
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail $O/bench20.err; exit 1; }
cat $O/bench20.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_torchrun.json 2> $O/bench20_torchrun.err || { tail $O/bench20_torchrun.err; exit 1; }
cat $O/bench20_torchrun.json
set +e
timeout -k 10 120 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/gpus2.out 2> $O/gpus2.err
echo "bench.py --gpus 2 on one GPU: rc=$? $(tail -1 $O/gpus2.err)"
