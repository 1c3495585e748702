set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tile
mkdir -p $O/ctr
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/ctr -o probe -- $R/cuda-hip-mpi-heat-equation-test_amd/_native/tile_probe 32768 > $O/ctr_probe.json 2> $O/ctr_probe.err
rc=$?; echo "counters rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $O/ctr -name "*counter_collection.csv" | head -1); echo "csv: $f"
python3 - "$f" <<'PY' > $O/ctr_summary.json
import csv, json, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    if "strip_kernel" not in k and "tile_kernel" not in k: continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
out = {k: dict(v, dispatches=len(disp[k])) for k, v in agg.items()}
print(json.dumps(out, indent=1))
PY
cat $O/ctr_summary.json
