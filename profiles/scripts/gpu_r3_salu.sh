# Strength-reduced row addressing (SALU per march row 31 -> 12.5): full GPU suite, then benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
O=gpurun_out/salu
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/b20.out 2> $O/b20.err || exit 1
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp32 --steps 1000 --warmup 100 > $O/s4096b.out 2> $O/s4096b.err || exit 1
timeout -k 10 200 python -u bench.py --grid 4096 --dtype fp64 --steps 1000 --warmup 100 > $O/d4096b.out 2> $O/d4096b.err || exit 1
timeout -k 10 300 python -u bench.py --dtype fp32 --steps 480 --warmup 20 > $O/f32_480.out 2> $O/f32_480.err || exit 1
timeout -k 10 300 python -u bench.py --steps 480 --warmup 20 > $O/f64_480.out 2> $O/f64_480.err || exit 1
for f in $O/*.out; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['config']['cycles'], d['config']['prepare_s'], json.dumps(d['config']['launch_plans'])[:300])"; done
export HEAT2D_PLAN_CACHE=off CP_ARITH=jacobi HEAT2D_SPLIT_ORDER=single HEAT2D_SEGMENTS=1007 HEAT2D_TB_RING=6
for pr in 0 1; do HEAT2D_PAIR=$pr timeout -k 10 60 python tools/cycle_probe.py fp32 4096 16 40 1 1 > $O/s4096_k16_p$pr.json || exit 1; done
for f in $O/*.json; do python -c "import json;d=json.load(open('$f'));print('$f', round(d['gpts']), round(d['ms']/d['cycles']*1e3,1),'us/cycle')"; done
