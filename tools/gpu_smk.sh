# semi-Markov: GPU tests, bench line, kernel trace (usage: bash tools/gpu_smk.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-smk}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_semimarkov.py -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --workload smk --steps 5 --warmup 1 --cpu-seconds 8 > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --workload smk --steps 5 --warmup 1 --cpu-seconds 0 > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_prof/run_kernel_stats.csv')):
    print(r['Name'].split('(')[0].replace('void ','')[:60], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
"
