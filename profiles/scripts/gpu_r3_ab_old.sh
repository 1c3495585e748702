# Same-box A/B: session-start tree (build_ab/old, commit a2af7f9) vs the current tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=$GRAFT_REPO_ROOT/gpurun_out/abold
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/new_b20_$i.json 2> $O/new_b20_$i.err || exit 1
  (cd build_ab/old && timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/old_b20_$i.json 2> $O/old_b20_$i.err) || exit 1
  timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/new_s4096_$i.json 2> $O/new_s4096_$i.err || exit 1
  (cd build_ab/old && timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/old_s4096_$i.json 2> $O/old_s4096_$i.err) || exit 1
done
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/new_f32.json 2> $O/new_f32.err || exit 1
(cd build_ab/old && timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/old_f32.json 2> $O/old_f32.err) || exit 1
for f in $O/*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], json.dumps(d['config']['launch_plans'])[:160])"; done
