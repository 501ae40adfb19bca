#!/bin/bash
# round 4 final pass: the whole GPU suite, smoke(), the NS bench and the other workloads
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r4z_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r4z_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r4z_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4z_smoke.log 2>&1 || { tail -20 gpurun_out/r4z_smoke.log; exit 1; }
tail -1 gpurun_out/r4z_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r4z_bench_ns.log 2>&1 || { tail -5 gpurun_out/r4z_bench_ns.log; exit 1; }
for w in "random --transition random" "trained --transition trained" "c2 --workload c2" "c3 --workload c3" "c5 --workload c5" "neural --workload neural"; do
  set -- $w
  tag=$1; shift
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/r4z_bench_$tag.log 2>&1 || { tail -5 gpurun_out/r4z_bench_$tag.log; exit 1; }
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r4z_bench_*.log")):
    for l in open(f):
        if l.startswith("{"):
            d = json.loads(l)
            r = d.get("roofline") or {}
            print(f, round(d["value"] / 1e6, 2), "M", round(d["ms_per_step"], 4), d.get("op_ms"), r.get("kernel"), r.get("frac"), r.get("traffic_source"))
PY
