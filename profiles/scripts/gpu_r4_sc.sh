# Round 4, run SC: one rank's slab of the driver's strong-scaling command at
# N = 2 / 4 / 8 (32768^2 fp64, 20 steps; middle slab, self-exchange rehearsal,
# RCCL and IPC), against the whole grid on the same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4sc
mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/whole.json 2> $O/whole.err || exit 1
for rows in 16384 8192 4096; do
  for t in rccl ipc; do
    timeout -k 10 300 python -u bench.py --rehearse-comm --transport $t --rows $rows --steps 20 --warmup 5 > $O/r${rows}_$t.json 2> $O/r${rows}_$t.err || exit 1
  done
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/whole_2.json 2> $O/whole_2.err || exit 1
python tools/summarize_json.py $O/*.json
