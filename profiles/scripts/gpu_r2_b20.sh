#!/bin/bash
# driver command x3 and the 480-step default, after the prepare-ends-warm change
set -o pipefail
mkdir -p gpurun_out/b20
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/b20/b20_$i.json || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b20/b20_$i.json'));print(d['value'],d['ms_per_step'],d['config']['cycles'],d['config']['prepare_s'])"
done
timeout -k 10 300 python bench.py --steps 480 --warmup 5 > gpurun_out/b20/b480.json || exit 1
python -c "import json;d=json.load(open('gpurun_out/b20/b480.json'));print(d['value'],d['ms_per_step'],d['config']['cycles'],d['config']['prepare_s'])"
