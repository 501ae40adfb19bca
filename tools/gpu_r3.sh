# round-3 GPU pass (usage: bash tools/gpu_r3.sh TAG [pytest selection] [extra bench lines...]):
# GPU tests in one process, then the default bench line and the listed extra bench argument
# sets (each quoted, e.g. "--transition random" "--workload c3")
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3}; SEL=${2:-tests}; shift 2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $SEL -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/${TAG}_pytest.log | tail -30
[ $rc -eq 0 ] || exit $rc
i=0
for extra in "" "$@"; do
  timeout -k 10 300 python bench.py --cpu-seconds 0 $extra > gpurun_out/${TAG}_bench$i.log 2>&1
  rc=$?; echo "bench [$extra] rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_bench$i.log; exit $rc; }
  python3 -c "
import json,sys
l=[x for x in open('gpurun_out/${TAG}_bench$i.log') if x.startswith('{')][-1]; d=json.loads(l)
r=d['roofline']; print(round(d['value']/1e6,2),'Mframes/s ms/step',round(d['ms_per_step'],4),'op_ms',d.get('op_ms'),'roof',r.get('kernel'),round(r['frac'],4),round(r.get('avg_launch_ms',0),4))"
  i=$((i+1))
done
