#!/bin/bash
# round 4: NeuralHMM -- is the per-step matrix stream bound by each CU or by aggregate HBM?
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python -u bench.py --workload neural --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r4c_$1.log 2>&1 || exit 1
  python - gpurun_out/r4c_$1.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print(sys.argv[1], round(d["ms_per_step"],4), {k: v for k,v in d.items() if k in ("op_ms","kernel_ms")})
PY
}
run both
HMM355_TV_ONLY=fb run fb
HMM355_TV_ONLY=vit run vit
