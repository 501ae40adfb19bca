# kernel-trace stats only (usage: bash tools/gpu_trace.sh TAG [bench args])
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-tr}; shift
export TMPDIR=/tmp
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 "$@" > $D/bench_trace.log 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 tools/prof_summary.py $D > $D/summary.json && python3 -c "
import json; d=json.load(open('$D/summary.json'))
for k,v in sorted(d['kernels'].items(), key=lambda x:-x[1]['avg_us']): print(f'{k:40s} {v[\"calls\"]:5d} {v[\"avg_us\"]:10.1f} us')
"
exit $rc
