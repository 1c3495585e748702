#!/bin/bash
# r6 run I: the edge-balance calibration on the RCCL loop (the exchange a node
# run uses), and the slab medians at the shift it picks.
# (1) 8 rank processes on the one GPU at 32768^2 fp64 (ranks take turns for the
#     slab rehearsals, each a 1-rank RCCL loop; IPC attaches at N = 8 on this
#     box, run H) — the calibration line and the shift it keeps;
# (2) RCCL-loop rehearsals of the three slab positions, uniform and at the
#     calibrated rows, medians of 3, interleaved; the whole grid beside them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6i
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 300 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 150 $O/$tag.json | tail -c 70)"; fatal $rc; }

for P in 8; do
  HEAT2D_IPC_ATTACH_TIMEOUT=15 timeout -k 10 400 python3 $R/bench.py --gpus $P --share-gpu --transport ipc --balance-loop rccl --steps 20 --warmup 5 --field-check off --verify off > $O/cal$P.json 2> $O/cal$P.err
  rc=$?; echo "calibration N=$P rc=$rc: $(grep -h 'edge balance' $O/cal$P.err | head -c 700)"; fatal $rc
done

rows() { python3 - "$1" "$2" <<'EOF'
import json, sys
P, path = int(sys.argv[1]), sys.argv[2]
line = [l for l in open(path) if "edge balance" in l][0]
rep = json.loads(line.split(" rows: ", 1)[1])
sh = rep.get("shifted_rows") or rep["uniform_rows"]
print(sh[0], sh[P // 2 - 1], sh[-1])
EOF
}
read S0 SM SL < <(rows 8 $O/cal8.err) || { echo "no calibration line"; exit 1; }
echo "N=8 shifted first $S0 middle $SM last $SL"
for i in 1 2 3; do
  b whole_$i --steps 20 --warmup 5 --field-check off --verify off
  for pos in first middle last; do
    b u8_${pos}_$i --rehearse-comm --rows 4096 --slab-pos $pos --steps 20 --warmup 5 --transport rccl --verify off
  done
  b s8_first_$i --rehearse-comm --rows $S0 --slab-pos first --steps 20 --warmup 5 --transport rccl --verify off
  b s8_middle_$i --rehearse-comm --rows $SM --slab-pos middle --steps 20 --warmup 5 --transport rccl --verify off
  b s8_last_$i --rehearse-comm --rows $SL --slab-pos last --steps 20 --warmup 5 --transport rccl --verify off
done
echo done
