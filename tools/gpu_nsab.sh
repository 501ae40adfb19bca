#!/bin/bash
# NS bench A/B over the follow modes (usage: bash tools/gpu_nsab.sh TAG [MODE ...])
set -o pipefail
TAG=${1:-nsab}; shift
MODES=${@:-"all none vit fb"}
mkdir -p gpurun_out
for m in $MODES; do
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 0 --follow $m > gpurun_out/${TAG}_$m.log 2>&1 || { tail -5 gpurun_out/${TAG}_$m.log; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/${TAG}_$m.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$m', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1e3,1), 'us', d.get('op_ms'))
"
done
