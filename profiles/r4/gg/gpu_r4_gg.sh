# Round 4, run GG: where the graph / eager threshold should sit. Mid-size grids
# whose cycles straddle 250 us: --graph off (eager) vs --graph on (replayed),
# interleaved, 2 each; the default's choice is whichever the threshold picks.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r4gg
mkdir -p $O
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err
}
for i in 1 2; do
  run f64_16k_off_$i --grid 16384 --steps 480 --warmup 20 --graph off || exit 1
  run f64_16k_on_$i --grid 16384 --steps 480 --warmup 20 --graph on || exit 1
  run f64_8k_off_$i --grid 8192 --steps 480 --warmup 20 --graph off || exit 1
  run f64_8k_on_$i --grid 8192 --steps 480 --warmup 20 --graph on || exit 1
  run f32_8k_off_$i --grid 8192 --dtype fp32 --steps 1000 --warmup 50 --graph off || exit 1
  run f32_8k_on_$i --grid 8192 --dtype fp32 --steps 1000 --warmup 50 --graph on || exit 1
  run f32_16k_off_$i --grid 16384 --dtype fp32 --steps 480 --warmup 20 --graph off || exit 1
  run f32_16k_on_$i --grid 16384 --dtype fp32 --steps 480 --warmup 20 --graph on || exit 1
  run f64_32k_s100_off_$i --steps 100 --warmup 5 --graph off || exit 1
  run f64_32k_s100_on_$i --steps 100 --warmup 5 --graph on || exit 1
done
python tools/summarize_json.py $O/*.json
