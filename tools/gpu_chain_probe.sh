# per-kernel durations of tools/chain_probe.py for ablation libs (usage: bash tools/gpu_chain_probe.sh TAG V1 V2 ...)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$v -o run -- python3 tools/chain_probe.py tools/ablate_libs/libhmm355_abl$v.so > gpurun_out/${TAG}_$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_$v/run_kernel_stats.csv')):
    if 'hmm355' in r['Name']: print('abl $v', r['Name'].split('(')[0].replace('void ','')[:34], round(float(r['AverageNs'])/1e3,1),'us')
"
done
