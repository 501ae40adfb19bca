#!/bin/bash
# round 4: dense chain after scheduling + branch-free writes -- parity, then benches + traces
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_autograd.py tests/test_gpu_fbpair.py \
  > gpurun_out/r4f_tests.log 2>&1 || { tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -2 gpurun_out/r4f_tests.log
./tools/gpu_r4e.sh || exit 1
bash tools/gpu_prof.sh r4_random --transition random > gpurun_out/r4p_random.log 2>&1 || { tail -5 gpurun_out/r4p_random.log; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/prof_r4_random/summary.json"))
for k,v in d["kernels"].items(): print(k, round(v["avg_us"],1))
PY
bash tools/gpu_prof.sh r4_c3 --workload c3 > gpurun_out/r4p_c3.log 2>&1 || { tail -5 gpurun_out/r4p_c3.log; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/prof_r4_c3/summary.json"))
for k,v in d["kernels"].items(): print(k, round(v["avg_us"],1))
PY
