# round 3: tests + benches + stamp diagnostics of the dense and banded chains
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3d}
bash tools/gpu_r3.sh $TAG tests "--transition random" "--workload c3" || exit $?
timeout -k 10 300 env HMM355_DENSE=1 python tools/stamps.py > gpurun_out/${TAG}_stamps_dense.log 2>&1 || { echo "stamps dense failed"; tail -5 gpurun_out/${TAG}_stamps_dense.log; exit 1; }
timeout -k 10 300 python tools/stamps.py > gpurun_out/${TAG}_stamps_band.log 2>&1 || { echo "stamps band failed"; exit 1; }
head -12 gpurun_out/${TAG}_stamps_dense.log; head -12 gpurun_out/${TAG}_stamps_band.log
