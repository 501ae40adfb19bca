cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmc_gmm
mkdir -p $D
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY --output-format csv -d $D/p1 -o run -- python3 bench.py --workload c3 --steps 2 --warmup 1 --cpu-seconds 0 > $D/b1.log 2>&1
rc=$?; echo rc=$rc
python3 - <<'PY'
import csv, glob, collections
fs = glob.glob("gpurun_out/pmc_gmm/p1/**/*counter_collection.csv", recursive=True)
print(fs)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in fs:
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "gmm_score4" not in k and "vit_fwd" not in k: continue
        kk = "gmm" if "gmm" in k else "vit"
        acc[kk][r["Counter_Name"]] += float(r["Counter_Value"])
for kk, d in acc.items():
    print(kk, {c: f"{v:.3e}" for c, v in sorted(d.items())})
PY
exit $rc
