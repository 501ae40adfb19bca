# round 3: tests, config-5 bench with both 64-state HSMM geometries, NeuralHMM PMC profile
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3f}
bash tools/gpu_r3.sh $TAG tests "--workload c5" || exit $?
HMM355_HSMM_SUB=8 timeout -k 10 300 python bench.py --workload c5 --cpu-seconds 0 > gpurun_out/${TAG}_c5_sub8.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_c5_sub8.log | cut -c1-400
bash tools/gpu_prof.sh ${TAG}n --workload neural | tail -25
