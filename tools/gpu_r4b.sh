#!/bin/bash
# round 4: fused Viterbi decode -- timing of its parts (HMM355_VIT_TAIL_DIAG bits, timing only)
set -o pipefail
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/r4b_$1.log 2>&1 || exit 1
  python - gpurun_out/r4b_$1.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print(sys.argv[1], round(d["value"]/1e6,1), "M", round(d["ms_per_step"],4), {k: round(v,4) for k,v in d["op_ms"].items()})
PY
}
HMM355_VIT_TAIL=0 run notail
HMM355_VIT_TAIL=1 run full
HMM355_VIT_TAIL=1 HMM355_VIT_TAIL_DIAG=2 run nocompose
HMM355_VIT_TAIL=1 HMM355_VIT_TAIL_DIAG=12 run nowalk_noexpand
HMM355_VIT_TAIL=1 HMM355_VIT_TAIL_DIAG=14 run none
