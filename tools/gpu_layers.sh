# BASELINE configs 1/2/3/5 through the layers (usage: bash tools/gpu_layers.sh TAG [cpu_seconds])
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-ly}; CPU=${2:-10}
export TMPDIR=/tmp
for w in c1 c2 c3 c5; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --cpu-seconds $CPU > gpurun_out/${TAG}_$w.log 2>&1 || { echo "$w failed"; tail -5 gpurun_out/${TAG}_$w.log; exit 1; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/${TAG}_$w.log') if x.startswith('{')][-1]; d=json.loads(l)
r=d['roofline']; c=d.get('cpu_baseline',{})
print('$w', round(d['value']/1e6,3),'Mframes/s', 'ms/step', round(d['ms_per_step'],3), 'roof', r.get('kernel','')[:40], r['bound'], round(r['frac'],4), round(r.get('avg_launch_ms',0),4), 'cpu', round(c.get('value',0)/1e3,1),'kframes/s', 'x', round(c.get('speedup_gpu_over_cpu',0)))
"
done
for w in c2 c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof_$w -o run -- python3 bench.py --workload $w --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/${TAG}_prof_$w.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_prof_$w/run_kernel_stats.csv')):
    if 'hmm355' in r['Name']: print('$w', r['Name'].split('(')[0].replace('void ','')[:40], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
done
