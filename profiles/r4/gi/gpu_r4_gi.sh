# Round 4, run GI: schedule search also tries shallower base depths on tuned
# times (long runs), graph threshold 400 us. Schedule log on stderr
# (HEAT2D_TUNE_LOG=1: sched_log.txt); every run eager or replayed by default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off HEAT2D_TUNE_LOG=1
O=gpurun_out/r4gi
mkdir -p $O
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err
}
run f64_16k_1 --grid 16384 --steps 480 --warmup 20 || exit 1
run f64_16k_2 --grid 16384 --steps 480 --warmup 20 || exit 1
run f64_32k_480 --steps 480 --warmup 20 || exit 1
run f32_32k_480 --dtype fp32 --steps 480 --warmup 20 || exit 1
run f64_8k --grid 8192 --steps 480 --warmup 20 || exit 1
run f32_16k --grid 16384 --dtype fp32 --steps 480 --warmup 20 || exit 1
run small_1 --grid 4096 --dtype fp32 --steps 1000 --warmup 100 || exit 1
run small_2 --grid 4096 --dtype fp32 --steps 1000 --warmup 100 || exit 1
run b20_1 --steps 20 --warmup 5 || exit 1
run b20_2 --steps 20 --warmup 5 || exit 1
python tools/summarize_json.py $O/*.json
grep -h "heat2d sched" $O/*.err > $O/sched_log.txt || true
