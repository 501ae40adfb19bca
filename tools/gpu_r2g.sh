# round-2 evidence pass: rocprof traces for the ergodic / random NS matrices and large-batch
# bench lines (usage: bash tools/gpu_r2g.sh TAG)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r2g}
mkdir -p gpurun_out
bash tools/gpu_prof.sh ${TAG}e --transition ergodic > gpurun_out/${TAG}_profe.log 2>&1 || { tail -5 gpurun_out/${TAG}_profe.log; exit 1; }
bash tools/gpu_prof.sh ${TAG}r --transition random > gpurun_out/${TAG}_profr.log 2>&1 || { tail -5 gpurun_out/${TAG}_profr.log; exit 1; }
echo "prof ok"
for B in 128 256; do
  timeout -k 10 300 python bench.py --batch $B --cpu-seconds 0 > gpurun_out/${TAG}_b$B.log 2>&1 || { tail -5 gpurun_out/${TAG}_b$B.log; exit 1; }
  HMM355_PAIR=1 timeout -k 10 300 python bench.py --batch $B --cpu-seconds 0 > gpurun_out/${TAG}_b${B}_pair.log 2>&1 || { tail -5 gpurun_out/${TAG}_b${B}_pair.log; exit 1; }
  for f in gpurun_out/${TAG}_b$B.log gpurun_out/${TAG}_b${B}_pair.log; do
    tail -1 $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$f', round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],4), d.get('op_ms'), round(d['roofline']['frac'],4))"
  done
done
