"""Summarise a tools/gpu_prof.sh directory: per-kernel average duration (kernel-trace stats)
and HBM traffic per launch from the PMC passes (FETCH_SIZE x 2 per MI355X_MICROARCH.md's
gfx950 note for wide coalesced reads, + WRITE_SIZE; both in KB in rocprofv3's output)."""
import csv, glob, json, os, re, sys
from collections import defaultdict

D = sys.argv[1]


def short(name):
    m = re.search(r"hmm355::(\w+)(<\d+(?:, *\w+)*>)?", name)
    if not m:  # kernels outside the namespace (viterbi.hip's vit_log_obs_kernel)
        m = re.match(r"(?:void\s+)?(\w+_kernel)(<\d+(?:, *\w+)*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")).replace(" ", "") if m else None


def rows(pattern):
    out = []
    for f in glob.glob(os.path.join(D, "**", pattern), recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


stats = {}
for r in rows("*kernel_stats.csv"):
    k = short(r["Name"])
    if k:
        stats[k] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                    "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3}
counters = defaultdict(lambda: defaultdict(list))
for r in rows("*counter_collection.csv"):
    k = short(r.get("Kernel_Name", ""))
    if k:
        counters[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
traffic = {}
for k, c in counters.items():
    fetch = sum(c.get("FETCH_SIZE", [0])) / max(len(c.get("FETCH_SIZE", [])), 1)
    write = sum(c.get("WRITE_SIZE", [0])) / max(len(c.get("WRITE_SIZE", [])), 1)
    traffic[k] = {"fetch_size_kb": fetch, "write_size_kb": write,
                  "hbm_bytes_per_launch": (2 * fetch + write) * 1024.0}
# band_prep_kernel runs once per transition plan (HMMPyTorch measures its fixed log_P once),
# not per launch of an op, so it is not part of an op's per-launch sum
ops = {"forward_backward": ["fb_recur_kernel", "fb_posterior_kernel"],
       "viterbi": ["vit_log_obs_kernel", "vit_fwd_kernel", "vit_psi_kernel", "vit_backtrace_kernel"]}
op_sum = {}
for op, ks in ops.items():
    sel = [k for k in stats if k.split("<")[0] in ks]
    op_sum[op] = {"kernels": sel, "avg_us_sum": sum(stats[k]["avg_us"] for k in sel),
                  "hbm_bytes_per_launch": sum(traffic.get(k, {}).get("hbm_bytes_per_launch", 0) for k in sel)}
bench = None
for f in glob.glob(os.path.join(D, "bench_trace.log")):
    for line in open(f):
        if line.startswith("{"):
            bench = json.loads(line)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import csrc_sha16  # noqa: E402  (the kernel sources these counters were taken on)
print(json.dumps({"kernels": stats, "traffic": traffic, "ops": op_sum,
                  "bench_config": bench["config"] if bench else None, "csrc_sha16": csrc_sha16()}, indent=1))
