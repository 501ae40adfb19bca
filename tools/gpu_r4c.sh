#!/bin/bash
# round 4: NeuralHMM -- one log_A stream for alpha + Viterbi (tv_chain_av) vs the split calls
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_neural.py \
  > gpurun_out/r4c_tests.log 2>&1 || { tail -30 gpurun_out/r4c_tests.log; exit 1; }
tail -2 gpurun_out/r4c_tests.log
run() {
  timeout -k 10 200 python -u bench.py --workload neural --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r4c_$1.log 2>&1 || exit 1
  python - gpurun_out/r4c_$1.log <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print(sys.argv[1], round(d["ms_per_step"],4), d.get("roofline",{}).get("kernel"), d.get("roofline",{}).get("avg_launch_ms"))
PY
}
run fused
HMM355_TV_SPLIT=1 run split
HMM355_TV_ONLY=fb run fbonly
HMM355_TV_ONLY=vit run vitonly
