# diagnostic timings of the time-varying kernels (usage: bash tools/diag_tv.sh "only batch static N" ...)
cd $GRAFT_REPO_ROOT
for cfg in "$@"; do
  set -- $cfg
  HMM355_TV_ONLY=$1 HMM355_TV_STATIC=$( [ $3 = 1 ] && echo 1 ) timeout -k 10 200 python bench.py --workload neural --steps 5 --warmup 1 --cpu-seconds 0 --batch $2 --N $4 > gpurun_out/diag${TAG}_$1_$2_$3_$4.log 2>&1 || { echo fail $cfg; tail -3 gpurun_out/diag${TAG}_$1_$2_$3_$4.log; exit 1; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/diag${TAG}_$1_$2_$3_$4.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$TAG $cfg', 'ms/step', round(d['ms_per_step'],3))"
done
