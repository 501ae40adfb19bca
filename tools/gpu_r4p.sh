#!/bin/bash
# round 4 profiles: kernel traces + FETCH/WRITE passes for the NS line, the random-matrix line,
# config 3 and config 5 (tools/gpu_prof.sh), copied to profiles/ by hand afterwards
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_prof.sh r4_ns > gpurun_out/r4p_ns.log 2>&1 || { tail -5 gpurun_out/r4p_ns.log; exit 1; }
bash tools/gpu_prof.sh r4_random --transition random > gpurun_out/r4p_random.log 2>&1 || { tail -5 gpurun_out/r4p_random.log; exit 1; }
bash tools/gpu_prof.sh r4_c3 --workload c3 > gpurun_out/r4p_c3.log 2>&1 || { tail -5 gpurun_out/r4p_c3.log; exit 1; }
bash tools/gpu_prof.sh r4_c5 --workload c5 > gpurun_out/r4p_c5.log 2>&1 || { tail -5 gpurun_out/r4p_c5.log; exit 1; }
bash tools/gpu_prof.sh r4_c2 --workload c2 > gpurun_out/r4p_c2.log 2>&1 || { tail -5 gpurun_out/r4p_c2.log; exit 1; }
for f in ns random c3 c5 c2; do tail -2 gpurun_out/r4p_$f.log | cut -c1-200; done
