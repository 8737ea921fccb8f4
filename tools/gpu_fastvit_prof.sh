set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/fastvit_bench.py > gpurun_out/fastvit_bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/fastvit_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fastvit -o run -- python3 tools/fastvit_bench.py --steps 2 --batch 64 > gpurun_out/prof_fastvit.log 2>&1; echo "prof rc=$?"
find gpurun_out/prof_fastvit -name "*kernel_stats.csv"
