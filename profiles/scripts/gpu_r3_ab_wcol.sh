# Headline A/B on one box: fp64 frame-column weight 1.3 (default) vs 1.6, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/abwcol
mkdir -p $O
for i in 1 2 3; do
  for w in 1.3 1.6; do
    HEAT2D_W_COL=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b20_w${w}_$i.json 2> $O/b20_w${w}_$i.err || exit 1
  done
done
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], json.dumps(d['config']['launch_plans']))"; done
