# A/B of the hipBLASLt out-proj/fc2 + fused add-LayerNorm block path vs the fused-epilogue MFMA path
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step tests timeout -k 10 300 python -u -m pytest tests/test_clip_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_clip.log 2>&1; tail -3 gpurun_out/pytest_clip.log
grep -q " passed" gpurun_out/pytest_clip.log && ! grep -q " failed" gpurun_out/pytest_clip.log || exit 1
step benchA env LUMEN_BLAS_RESID=0 timeout -k 10 300 python bench.py > gpurun_out/benchA.log 2>&1; grep '^{' gpurun_out/benchA.log | cut -c1-200
step benchB env LUMEN_BLAS_RESID=1 timeout -k 10 300 python bench.py > gpurun_out/benchB.log 2>&1; grep '^{' gpurun_out/benchB.log
step prof timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_blas -o run -- python3 bench.py --steps 3 --warmup 1 --text-steps 3 > gpurun_out/prof_blas.log 2>&1
find gpurun_out/prof_blas -name "*kernel_stats.csv"
exit 0
