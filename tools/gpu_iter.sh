# one GPU iteration: parity tests, ablation timings, bench  (usage: bash tools/gpu_iter.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-it}
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -x > gpurun_out/${TAG}_pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python tools/ablate.py run > gpurun_out/${TAG}_ablate.log 2>&1
echo "ablate rc=$?"; grep ABL gpurun_out/${TAG}_ablate.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/${TAG}_bench.log 2>&1
echo "bench rc=$?"; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-900
