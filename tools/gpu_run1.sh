set -o pipefail
cd $GRAFT_REPO_ROOT
python -c "import torch;print(torch.cuda.get_device_name(0))" > gpurun_out/r1_env.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1
echo "smoke rc=$?"
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider > gpurun_out/r1_pytest.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-seconds 4 > gpurun_out/r1_bench.log 2>&1
echo "bench rc=$?"
