set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step tests timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k gemm --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1; tail -3 gpurun_out/pytest_gemm.log
grep -q " passed" gpurun_out/pytest_gemm.log && ! grep -q "failed" gpurun_out/pytest_gemm.log || exit 1
step tl timeout -k 10 120 python tools/gemm_timeline.py > gpurun_out/gemm_timeline.log 2>&1; grep "^M=" gpurun_out/gemm_timeline.log
step gemm timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; grep "^{" gpurun_out/gemm_bench.log
step bench timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; grep '^{' gpurun_out/bench.log
exit 0
