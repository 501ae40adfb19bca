# round-3 final-tree check (usage: bash tools/gpu_r3w.sh TAG): the general HSMM form's tests
# first (short), then every GPU test, smoke() and the NS bench
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-w}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "hsmm_wide" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_wide.log 2>&1
rc=$?; echo "wide rc=$rc"; tail -3 gpurun_out/${TAG}_wide.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -1 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
exit $rc
