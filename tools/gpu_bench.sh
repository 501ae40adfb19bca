# bench variants (usage: bash tools/gpu_bench.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-b}
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/${TAG}_bench.log 2>&1 &&
HMM355_DENSE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 0 > gpurun_out/${TAG}_bench_dense.log 2>&1
rc=$?; echo "bench rc=$rc"
for f in gpurun_out/${TAG}_bench.log gpurun_out/${TAG}_bench_dense.log; do python3 -c "
import json,sys
l=[x for x in open('$f') if x.startswith('{')][-1]; d=json.loads(l)
print('$f', round(d['value']/1e6,2),'Mframes/s', 'ms/step', round(d['ms_per_step'],3), 'op_ms', {k:round(v,3) for k,v in d['op_ms'].items()})
"; done
exit $rc
