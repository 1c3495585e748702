#!/bin/bash
# Every BASELINE.json configuration with round-2 code (bench/configs.py), one JSON line each.
set -o pipefail
O=gpurun_out/${CFG_OUT:-configs}
mkdir -p $O
timeout -k 10 900 python -u bench/configs.py > $O/configs.jsonl || { tail -5 $O/configs.jsonl; exit 1; }
python -c "
import json
for l in open('$O/configs.jsonl'):
    d=json.loads(l); print(d['config'], d['n'], d['gpts'], d.get('cycles'), d.get('hbm_gb_per_s_plan'), d.get('prepare_s'), d['field_gb'])"
