# layer workloads c2, c3, c5: the default (one batch at a time) and --overlap-steps lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3o}
for wl in c2 c3 c5; do
  for mode in "" "--overlap-steps"; do
    timeout -k 10 300 python bench.py --workload $wl --cpu-seconds 0 $mode > gpurun_out/${TAG}_${wl}${mode:+_overlap}.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$wl $mode rc=$rc"; tail -20 gpurun_out/${TAG}_${wl}${mode:+_overlap}.log; exit $rc; }
    python3 -c "
import json
l=[x for x in open('gpurun_out/${TAG}_${wl}${mode:+_overlap}.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$wl', '$mode', round(d['value']/1e6,2), 'M frames/s, ms/step', round(d['ms_per_step'],4), 'serial', d.get('ms_per_step_serial'))"
  done
done
