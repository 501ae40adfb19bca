#!/bin/bash
# round 4: fused Viterbi decode -- parity tests, then the NS bench with / without it
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_vit_tail.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py -k "tail or fullsize or north or config3 or gmm" > gpurun_out/r4a_tests.log 2>&1 || { tail -30 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
HMM355_VIT_TAIL=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/r4a_bench_tail.log 2>&1 || exit 1
HMM355_VIT_TAIL=0 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/r4a_bench_notail.log 2>&1 || exit 1
for f in gpurun_out/r4a_bench_tail.log gpurun_out/r4a_bench_notail.log; do
  python - "$f" <<'PY'
import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d=json.loads(l); print(sys.argv[1], round(d["value"]/1e6,1), "M", d["ms_per_step"], d["op_ms"])
PY
done
