# quick GPU iteration (usage: bash tools/gpu_quick.sh TAG "pytest files" [bench args ...])
#   runs the named test files, then bench.py with each extra argument string
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; FILES=$2; shift 2
mkdir -p gpurun_out
if [ -n "$FILES" ]; then
  timeout -k 10 600 python -u -m pytest $FILES -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/${TAG}_pytest.log | tail -15
  [ $rc -ne 0 ] && exit $rc
fi
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --cpu-seconds 0 $a > gpurun_out/${TAG}_bench$i.log 2>&1; rc=$?
  echo "bench[$a] rc=$rc"; tail -1 gpurun_out/${TAG}_bench$i.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1),'M/s', d['ms_per_step'], d.get('op_ms'))" || tail -3 gpurun_out/${TAG}_bench$i.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
