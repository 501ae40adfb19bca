#!/bin/bash
# round 6: A/B of the NS ops through the raw C ABI (tools/time_follow.py) + kernel traces
# (usage: bash tools/gpu_r6b.sh TAG [LIB:FLAGS ...]; default: this build with and without followers
# and the round-5 library)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r6b}; shift
L=pytorch_hmm_amd/lib/libhmm355.so
SPECS=${@:-"$L:f $L tools/ablate_libs/libhmm355_r5.so"}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_follow.py > gpurun_out/${TAG}_pytest_follow.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest_follow.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest_follow.log
timeout -k 10 200 python -u tools/time_follow.py $SPECS > gpurun_out/${TAG}_time.log 2>&1 || { cat gpurun_out/${TAG}_time.log; exit 1; }
cat gpurun_out/${TAG}_time.log
i=0
for s in $SPECS; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tr$i -o run -- python3 tools/time_follow.py $s > gpurun_out/${TAG}_tr$i.log 2>&1 || exit 1
  echo "== $s"; f=$(find gpurun_out/${TAG}_tr$i -name "*kernel_stats.csv" | head -1); grep hmm355 $f | cut -d, -f1-6 | sed 's/(hmm355[^)]*)//'
done
