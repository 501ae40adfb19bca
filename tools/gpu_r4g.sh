#!/bin/bash
# round 4: dense-chain reductions with fewer wait states -- microbench, parity, benches
set -o pipefail
mkdir -p gpurun_out
[ -n "$MB" ] && { timeout -k 10 120 ./tools/mb_dense 32 2000 > gpurun_out/mb_dense6.log 2>&1 || exit 1; }
true
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_trained_layer.py tests/test_gpu_fullsize.py tests/test_gpu_kernels.py tests/test_gpu_autograd.py \
  tests/test_gpu_fbpair.py tests/test_gpu_fullsize_configs.py tests/test_gpu_layers.py -s > gpurun_out/r4g_tests.log 2>&1 || { grep -E "chains|FAIL|Error" gpurun_out/r4g_tests.log | head -20; tail -5 gpurun_out/r4g_tests.log; exit 1; }
grep -E "chains:" gpurun_out/r4g_tests.log | head -3
tail -2 gpurun_out/r4g_tests.log
./tools/gpu_r4e.sh || exit 1
