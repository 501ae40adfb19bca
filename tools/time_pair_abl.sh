# time the pair kernel for each ablation library named on the command line (B=32, T=2000)
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  echo "ABL $v"; HMM355_LIB=tools/ablate_libs/libhmm355_abl$v.so timeout -k 10 120 python tools/time_pair.py 2>&1 | grep "^32 2000" || exit 1
done
