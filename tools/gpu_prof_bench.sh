# rocprofv3 kernel stats of the headline bench (ViT-L/14 b512 image window + text window)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py --steps 3 --warmup 1 --text-steps 3 > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"
find gpurun_out/prof_bench -name "*kernel_stats.csv" | head -3
exit $rc
