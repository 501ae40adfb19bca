cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp HMM355_BENCH_NO_KPROF=1
for w in 64 128 192; do
  HMM355_HSMM_WARM=$w timeout -k 10 200 python bench.py --workload c5 --cpu-seconds 0 > gpurun_out/warm_$w.log 2>&1 || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/warm_$w.log') if x.startswith('{')][-1]; d=json.loads(l); print('warm $w', round(d['value']/1e6,2), round(d['ms_per_step'],4))"
done
