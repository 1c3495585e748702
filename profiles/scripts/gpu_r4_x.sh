# Round 4, run X: XCD-contiguous block numbering (HEAT2D_XCD_REMAP=1) with
# this round's band-major dynamic headline plan, interleaved A/B; fp32 480.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4x
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_def_$i.json 2> $O/b20_def_$i.err || exit 1
  HEAT2D_XCD_REMAP=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20_xcd_$i.json 2> $O/b20_xcd_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_def.json 2> $O/b32_def.err || exit 1
HEAT2D_XCD_REMAP=1 timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_xcd.json 2> $O/b32_xcd.err || exit 1
python tools/summarize_json.py $O/*.json
