#!/bin/bash
# r6 run H: the edge-balanced decomposition.
# (1) the GPU bench-contract tests (the 4-rank shared-GPU run now rehearses
#     every rank's slab, one after another, before choosing the shift);
# (2) the calibration of a 32768^2 fp64 node run at N = 8 and N = 4, rehearsed
#     on the one GPU (ranks take turns, so each slab is timed alone as on its
#     own GPU); the IPC attach of 4 or 8 ranks at 32768^2 then stalls on this
#     box (profiles/r6/c/) and ends the run with exit 3 — the calibration
#     line on stderr is what this step records;
# (3) the driver's transport: RCCL-loop rehearsals of the three slab positions
#     with the uniform rows and with the calibrated rows, medians of 3,
#     interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6h
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }

timeout -k 10 900 python3 -u -m pytest tests/test_bench_contract.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $O/tests.log)"; fatal $rc

for P in 8 4; do
  HEAT2D_IPC_ATTACH_TIMEOUT=15 timeout -k 10 400 python3 $R/bench.py --gpus $P --share-gpu --transport ipc --steps 20 --warmup 5 --field-check off --verify off > $O/cal$P.json 2> $O/cal$P.err
  rc=$?; echo "calibration N=$P rc=$rc: $(grep -h 'edge balance' $O/cal$P.err | head -c 600)"; fatal $rc
done

# rows of the three slab positions, uniform and calibrated
rows() { python3 - "$1" "$2" <<'EOF'
import json, re, sys
P, path = int(sys.argv[1]), sys.argv[2]
line = [l for l in open(path) if "edge balance" in l][0]
rep = json.loads(line.split(" rows: ", 1)[1])
sh = rep.get("shifted_rows") or rep["uniform_rows"]
print(rep["uniform_rows"][0], rep["uniform_rows"][1], sh[0], sh[P // 2 - 1 if P > 2 else 1], sh[-1])
EOF
}
for P in 8 4; do
  read U0 UM S0 SM SL < <(rows $P $O/cal$P.err) || { echo "no calibration line for N=$P"; continue; }
  echo "N=$P uniform $U0/$UM shifted first $S0 middle $SM last $SL"
  for i in 1 2 3; do
    b u${P}_first_$i --rehearse-comm --rows $U0 --slab-pos first --steps 20 --warmup 5 --transport rccl --verify off
    b u${P}_middle_$i --rehearse-comm --rows $UM --slab-pos middle --steps 20 --warmup 5 --transport rccl --verify off
    b s${P}_first_$i --rehearse-comm --rows $S0 --slab-pos first --steps 20 --warmup 5 --transport rccl --verify off
    b s${P}_middle_$i --rehearse-comm --rows $SM --slab-pos middle --steps 20 --warmup 5 --transport rccl --verify off
    b s${P}_last_$i --rehearse-comm --rows $SL --slab-pos last --steps 20 --warmup 5 --transport rccl --verify off
  done
done
echo done
