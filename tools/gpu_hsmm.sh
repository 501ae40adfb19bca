# HSMM pass (usage: bash tools/gpu_hsmm.sh TAG): HSMM GPU tests, then the config-5 bench line
# for each group width
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-hs}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_fullsize_configs.py tests/test_gpu_layers.py -k "hsmm or HSMM" -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/${TAG}_pytest.log | tail -20
[ $rc -eq 0 ] || exit $rc
for sub in 4 8 16; do
  HMM355_HSMM_SUB=$sub timeout -k 10 300 python bench.py --workload c5 --cpu-seconds 0 > gpurun_out/${TAG}_c5_sub$sub.log 2>&1
  rc=$?; echo "sub $sub rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/${TAG}_c5_sub$sub.log; exit $rc; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/${TAG}_c5_sub$sub.log') if x.startswith('{')][-1]; d=json.loads(l)
r=d['roofline']; print(round(d['value']/1e6,2),'Mframes/s ms/step',round(d['ms_per_step'],4),'roof',r.get('kernel'),round(r.get('avg_launch_ms',0),4), {k:v.get('avg_launch_ms') for k,v in (d.get('kernels') or {}).items()} if isinstance(d.get('kernels'),dict) else '')"
done
