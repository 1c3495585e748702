#!/bin/bash
# r6 FINAL 4 (the round's last tree: the IPC field allocation fix): the GPU
# suite and smoke again, the headline twice, and the native CLI's peer-
# transport ranks on one GPU with and without an edge shift against a 1-GPU
# run of the same input (bitwise, npy outputs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6final4
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc $(tail -1 $O/gpu_tests.log)"; fatal $rc; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc
for i in 1 2; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/h20_$i.json 2> $O/h20_$i.err
  rc=$?; echo "h20_$i rc=$rc $(head -c 80 $O/h20_$i.json | tail -c 30)"; fatal $rc
done
CLI=$R/cuda-hip-mpi-heat-equation-test_amd/_native/heat2d
for v in one p3 p3s p5s; do mkdir -p $O/cli_$v; printf "4096 0.25 0.05 1.0 100 1\n" > $O/cli_$v/input.dat; done
(cd $O/cli_one && timeout -k 10 120 $CLI --gpus 1 --output npy --quiet --json m.json > out.txt 2>&1); rc=$?; echo "cli one rc=$rc"; fatal $rc
(cd $O/cli_p3 && timeout -k 10 120 $CLI --gpus 3 --share-gpu --transport peer --output npy --quiet --json m.json > out.txt 2>&1); rc=$?; echo "cli p3 rc=$rc"; fatal $rc
(cd $O/cli_p3s && timeout -k 10 120 $CLI --gpus 3 --share-gpu --transport peer --edge-shift 200 --output npy --quiet --json m.json > out.txt 2>&1); rc=$?; echo "cli p3s rc=$rc"; fatal $rc
(cd $O/cli_p5s && timeout -k 10 120 $CLI --gpus 5 --share-gpu --transport peer --edge-shift 100 --output npy --quiet --json m.json > out.txt 2>&1); rc=$?; echo "cli p5s rc=$rc"; fatal $rc
timeout -k 10 120 python3 - $O <<'PY' > $O/cli_compare.json
import glob, json, os, sys
import numpy as np
O = sys.argv[1]
def field(d):
    fs = sorted(glob.glob(os.path.join(O, d, "soln*.npy")))
    return np.concatenate([np.load(f, allow_pickle=False) for f in fs], axis=0), [np.load(f, allow_pickle=False).shape[0] for f in fs]
ref, _ = field("cli_one")
out = {}
for d in ("cli_p3", "cli_p3s", "cli_p5s"):
    a, rows = field(d)
    out[d] = {"rows": rows, "bitwise_equal_to_1gpu": bool(a.shape == ref.shape and np.array_equal(a, ref))}
print(json.dumps(out))
PY
rc=$?; echo "compare rc=$rc $(cat $O/cli_compare.json)"; fatal $rc
rm -f $O/cli_*/*.npy  # 134 MB each: gpurun_out/ must stay under 64 MiB
echo done
