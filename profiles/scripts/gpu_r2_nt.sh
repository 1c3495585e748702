#!/bin/bash
# nt (aux = 2) vs default row stores (alternative build in exp/nt), interleaved, whole-grid benches.
set -o pipefail
O=gpurun_out/nt
mkdir -p $O
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d['config'];print(sys.argv[2], d['value'], c['cycles'], c.get('hbm_gb_per_s_plan'), {k:(v['order'],v['ring'],v['main_bands'],v['main_waves']) for k,v in c['launch_plans'].items()})" $1 "$2"; }
for rep in 1 2; do
  for v in base nt; do
    if [ $v = base ]; then unset HEAT2D_LIB; else export HEAT2D_LIB=$PWD/exp/nt/libheat2d.so; fi
    timeout -k 10 300 python bench.py --dtype fp32 --steps 480 --warmup 16 > $O/b.json || exit 1; show $O/b.json "$v fp32-480"
    timeout -k 10 300 python bench.py --steps 480 --warmup 16 > $O/b.json || exit 1; show $O/b.json "$v fp64-480"
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b.json || exit 1; show $O/b.json "$v fp64-20"
  done
done
unset HEAT2D_LIB
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace --output-format csv -d $O/fetch_base -- python tools/cycle_probe.py fp32 32768 16 4 > /dev/null || exit 1
HEAT2D_LIB=$PWD/exp/nt/libheat2d.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE --kernel-trace --output-format csv -d $O/fetch_nt -- python tools/cycle_probe.py fp32 32768 16 4 > /dev/null || exit 1
python - <<'PY'
import csv, glob
for tag in ("base", "nt"):
    acc = {}
    for f in glob.glob(f"gpurun_out/nt/fetch_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "tb_kernel" in r["Kernel_Name"]:
                acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    field = 32768 * 32768 * 4
    print(tag, {k: round(2 * (sum(v) / len(v)) * 1024 / field if k == "FETCH_SIZE" else (sum(v) / len(v)) * 1024 / field, 3) for k, v in acc.items()}, "x field per dispatch (FETCH doubled)")
PY
