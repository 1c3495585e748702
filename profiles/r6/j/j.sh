#!/bin/bash
# r6 run J: edge balance for the fp32 8-rank slab (VERDICT r5 item 2's fp32
# target), 32768^2 fp32, 480 steps, RCCL loop: uniform first / middle / last
# slabs (medians of 3), the shift estimated from them (parallel/select.py
# edge_shift_estimate, the bench's own rule), then the shifted slabs (medians
# of 3); the whole grid beside them.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6j
mkdir -p $O
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1: stopping"; exit $1;; esac; }
b() { tag=$1; shift; timeout -k 10 400 python3 $R/bench.py "$@" > $O/$tag.json 2> $O/$tag.err; rc=$?; echo "$tag rc=$rc $(head -c 80 $O/$tag.json | tail -c 30)"; fatal $rc; }
C="--dtype fp32 --steps 480 --warmup 48 --transport rccl --verify off"
b whole --dtype fp32 --steps 480 --warmup 48 --field-check off --verify off
for i in 1 2 3; do
  for pos in first middle last; do b u_${pos}_$i --rehearse-comm --rows 4096 --slab-pos $pos $C; done
done
read S0 SM SL < <(python3 - $O <<'PY'
import json, statistics, sys
sys.path.insert(0, ".")
from heat2d.parallel import select
from heat2d.ops import _native as N
O = sys.argv[1]
ms = {p: statistics.median(json.load(open(f"{O}/u_{p}_{i}.json"))["ms_per_step"] for i in (1, 2, 3))
      for p in ("first", "middle", "last")}
slab = [ms["first"]] + [ms["middle"]] * 6 + [ms["last"]]
d = select.edge_shift_estimate(slab, [4096] * 8, cap=1024)
rows = [N.decompose(32768, 8, r, d)[1] for r in range(8)]
json.dump({"uniform_ms_per_step": ms, "shift": d, "rows": rows}, open(f"{O}/estimate.json", "w"))
print(rows[0], rows[3], rows[7])
PY
) || { echo "no estimate"; exit 1; }
echo "shifted rows $S0 $SM $SL"
for i in 1 2 3; do
  b s_first_$i --rehearse-comm --rows $S0 --slab-pos first $C
  b s_middle_$i --rehearse-comm --rows $SM --slab-pos middle $C
  b s_last_$i --rehearse-comm --rows $SL --slab-pos last $C
done
echo done
