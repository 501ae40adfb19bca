# all GPU tests in one process (usage: bash tools/gpu_tests.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-t}
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/${TAG}_pytest.log | tail -30
exit $rc
