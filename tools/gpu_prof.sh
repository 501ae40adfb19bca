# rocprofv3 kernel-trace + stats of one bench run; writes gpurun_out/prof_<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r1}
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/prof_$TAG/bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
find gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc
