#!/bin/bash
# round 6 GPU pass (usage: bash tools/gpu_r6.sh TAG [quick|full])
#   quick: the follower tests, the full-size parity tests, smoke(), the NS bench with and
#          without the work beside the chains
#   full:  + the whole GPU suite and the other bench workloads
set -o pipefail
TAG=${1:-r6}
MODE=${2:-quick}
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 400 $PYT tests/test_gpu_follow.py tests/test_gpu_fullsize.py tests/test_gpu_band.py \
  > gpurun_out/${TAG}_pytest_follow.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_follow.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_follow.log
if [ "$MODE" = full ]; then
  timeout -k 10 900 $PYT tests > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench_ns.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench_ns.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-follow --cpu-seconds 0 > gpurun_out/${TAG}_bench_ns_nofollow.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench_ns_nofollow.log; exit 1; }
if [ "$MODE" = full ]; then
  for w in "random --transition random" "trained --transition trained" "c2 --workload c2" "c3 --workload c3" "c5 --workload c5" "neural --workload neural"; do
    set -- $w
    tag=$1; shift
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/${TAG}_bench_$tag.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench_$tag.log; exit 1; }
  done
fi
python3 - "$TAG" <<'PY'
import json, glob, sys
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}_bench_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            r = d.get("roofline") or {}
            print(f, round(d["value"] / 1e6, 2), "M", round(d["ms_per_step"], 4), d.get("op_ms"), r.get("kernel"), r.get("frac"))
PY
