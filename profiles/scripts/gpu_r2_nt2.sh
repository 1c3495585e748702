#!/bin/bash
# nt vs default row stores: 3 interleaved repetitions of the fp64 benches + FETCH_SIZE per build.
set -o pipefail
O=gpurun_out/nt2
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], {k:(v['order'],v['ring'],v['main_bands']) for k,v in c['launch_plans'].items()})" $1 "$2"; }
for rep in 1 2 3; do
  for v in base nt; do
    if [ $v = base ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$PWD/exp/nt/libheat2d.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b.json || exit 1; show $O/b.json "$v fp64-20"
    timeout -k 10 300 python bench.py --steps 480 --warmup 16 > $O/b.json || exit 1; show $O/b.json "$v fp64-480"
  done
done
unset HEAT2D_LIB
for v in base nt; do
  if [ $v = base ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$PWD/exp/nt/libheat2d.so; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch_$v -- python tools/cycle_probe.py fp32 32768 16 4 > /dev/null || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch64_$v -- python tools/cycle_probe.py fp64 32768 16 4 > /dev/null || exit 1
done
python - <<'PY'
import csv, glob
for tag, es in (("fetch_base", 4), ("fetch_nt", 4), ("fetch64_base", 8), ("fetch64_nt", 8)):
    v = []
    for f in glob.glob(f"gpurun_out/nt2/{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "tb_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                v.append(float(r["Counter_Value"]))
    field = 32768 * 32768 * es
    print(tag, "read per pass (FETCH_SIZE x2) / field:", [round(2 * x * 1024 / field, 3) for x in v[-4:]])
PY
