# per-segment stamp diagnostics on the GPU box (usage: bash tools/gpu_stamps.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-st}
timeout -k 10 300 python tools/stamps.py > gpurun_out/${TAG}_stamps.log 2>&1
echo "stamps rc=$?"; cat gpurun_out/${TAG}_stamps.log | tail -30
