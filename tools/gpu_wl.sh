# one bench workload: bench line + kernel trace (usage: bash tools/gpu_wl.sh TAG WORKLOAD [cpu_seconds])
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-wl}; WL=${2:-ns}; CPU=${3:-8}
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload $WL --steps 10 --warmup 2 --cpu-seconds $CPU > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --workload $WL --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_prof/run_kernel_stats.csv')):
    print(r['Name'].split('(')[0].replace('void ','')[:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
