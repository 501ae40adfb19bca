# rocprofv3 evidence for one bench configuration (usage: bash tools/gpu_prof.sh TAG [bench args...])
#   pass 1: --kernel-trace --stats  (per-kernel average durations)
#   pass 2: --pmc FETCH_SIZE        (separate passes: FETCH_SIZE and WRITE_SIZE do not fit one)
#   pass 3: --pmc WRITE_SIZE
# then tools/prof_summary.py -> gpurun_out/prof_TAG/summary.json
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r1}; shift
ARGS="$@"
export TMPDIR=/tmp
# (--no-kernel-profile: no torch.profiler inside the rocprofv3 passes)
D=gpurun_out/prof_$TAG
mkdir -p $D
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-seconds 0 --no-kernel-profile $ARGS > $D/bench_trace.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-kernel-profile $ARGS > $D/bench_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-kernel-profile $ARGS > $D/bench_write.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find $D -name "*.csv" | sort
python3 tools/prof_summary.py $D > $D/summary.json; echo "summary rc=$?"
cat $D/summary.json
tail -1 $D/bench_trace.log | cut -c1-300
exit $rc
