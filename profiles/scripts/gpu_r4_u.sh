# Round 4, run U: long-cycle autotuning borrows a tuned neighbouring depth's
# plan (prepare time of the 240 GB fp32 grid), A/B against --tb 20, and the
# fp32 / fp64 480-step runs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4u
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --dtype fp32 --grid 173056 --steps 64 --warmup 16 > $O/max_new_$i.json 2> $O/max_new_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --dtype fp32 --grid 173056 --steps 64 --warmup 16 --tb 20 > $O/max_tb20_$i.json 2> $O/max_tb20_$i.err || exit 1
done
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/b32_480.json 2> $O/b32_480.err || exit 1
timeout -k 10 300 python -u bench.py --steps 480 --warmup 20 > $O/b64_480.json 2> $O/b64_480.err || exit 1
python tools/summarize_json.py $O/*.json
python -c "
import json,glob
for f in sorted(glob.glob('$O/*.json')):
    d=json.load(open(f)); c=d['config']; print(f.split('/')[-1], d['value'], 'prepare', c['prepare_s'], 'warmup', c.get('warmup_s'), {k: v['origin'] for k, v in c['launch_plans'].items()})
"
