#!/bin/bash
# round 4: dense-chain scheduling + layer workloads (c3, random NS)
set -o pipefail
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/r4g_$tag.log 2>&1 || exit 1
  python - gpurun_out/r4g_$tag.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print(sys.argv[1], round(d["value"]/1e6,1), "M", round(d["ms_per_step"],4), d.get("op_ms"), (d.get("roofline") or {}).get("kernel"), (d.get("roofline") or {}).get("avg_launch_ms"))
PY
}
run random --transition random
run c3 --workload c3
run c2 --workload c2
run c5 --workload c5
