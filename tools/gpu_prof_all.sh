#!/bin/bash
# round-end rocprofv3 evidence for every bench workload (usage: bash tools/gpu_prof_all.sh TAG)
set -o pipefail
TAG=${1:-rd6}
bash tools/gpu_prof.sh ${TAG}_ns > gpurun_out/prof_${TAG}_ns.log 2>&1 || exit 1
for w in "random --transition random" "c2 --workload c2" "c3 --workload c3" "c5 --workload c5" "neural --workload neural"; do
  set -- $w
  t=$1; shift
  bash tools/gpu_prof.sh ${TAG}_$t "$@" > gpurun_out/prof_${TAG}_$t.log 2>&1 || { tail -5 gpurun_out/prof_${TAG}_$t.log; exit 1; }
  echo "$t done"
done
