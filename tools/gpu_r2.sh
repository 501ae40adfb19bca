# round-2 GPU pass (usage: bash tools/gpu_r2.sh TAG [steps...]); each step has its own time
# limit and the chain stops at the first failure
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r2}; shift
STEPS=${@:-tests bench}
mkdir -p gpurun_out
for s in $STEPS; do
  case $s in
    tests)   timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
             echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/${TAG}_pytest.log | tail -20 ;;
    fullsize) timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1; rc=$?
             echo "fullsize rc=$rc"; tail -5 gpurun_out/${TAG}_full.log ;;
    bench)   timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-900 ;;
    ergodic) timeout -k 10 300 python bench.py --transition ergodic --cpu-seconds 8 > gpurun_out/${TAG}_erg.log 2>&1; rc=$?; echo "ergodic rc=$rc"; tail -1 gpurun_out/${TAG}_erg.log | cut -c1-900 ;;
    random)  timeout -k 10 300 python bench.py --transition random --cpu-seconds 8 > gpurun_out/${TAG}_rand.log 2>&1; rc=$?; echo "random rc=$rc"; tail -1 gpurun_out/${TAG}_rand.log | cut -c1-900 ;;
    stampsd) HMM355_DENSE=1 timeout -k 10 300 python tools/stamps.py > gpurun_out/${TAG}_stampsd.log 2>&1; rc=$?; echo "stamps dense rc=$rc"; tail -22 gpurun_out/${TAG}_stampsd.log ;;
    stampsb) timeout -k 10 300 python tools/stamps.py > gpurun_out/${TAG}_stampsb.log 2>&1; rc=$?; echo "stamps banded rc=$rc"; tail -22 gpurun_out/${TAG}_stampsb.log ;;
    smoke)   timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${TAG}_smoke.log ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  [ $rc -ne 0 ] && exit $rc
done
exit 0
