set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 HEAT2D_PLAN_CACHE=off
O=gpurun_out/r3pp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
HEAT2D_PERSIST=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --grid 4096 --dtype fp32 --steps 150 --warmup 15 > $GRAFT_REPO_ROOT/$O/p1.json 2> $GRAFT_REPO_ROOT/$O/p1.err || exit 1
HEAT2D_PERSIST=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/p0 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --grid 4096 --dtype fp32 --steps 150 --warmup 15 > $GRAFT_REPO_ROOT/$O/p0.json 2> $GRAFT_REPO_ROOT/$O/p0.err || exit 1
cd $GRAFT_REPO_ROOT
find $O -name "*kernel_stats.csv" | while read f; do echo "== $f"; head -8 "$f" | cut -c1-300; done
