set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step tests timeout -k 10 500 python -m pytest tests/test_kernels_gpu.py tests/test_clip_gpu.py -q -x > gpurun_out/pytest_clip.log 2>&1; tail -2 gpurun_out/pytest_clip.log
grep -q " passed" gpurun_out/pytest_clip.log && ! grep -q "failed" gpurun_out/pytest_clip.log || exit 1
step gemm timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; grep "^{" gpurun_out/gemm_bench.log | cut -c1-200
step attn timeout -k 10 200 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; grep '^{' gpurun_out/attn_bench.log
step bench timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; grep '^{' gpurun_out/bench.log
exit 0
