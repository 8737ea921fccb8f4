# attention/LLM kernel numerics + attention microbench + headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return $rc; }
step tests timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_clip_gpu.py tests/test_llm_ops_gpu.py tests/test_vlm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; tail -3 gpurun_out/pytest_attn.log
grep -q " passed" gpurun_out/pytest_attn.log && ! grep -q "failed" gpurun_out/pytest_attn.log || exit 1
step attn timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attn_bench.log 2>&1; cat gpurun_out/attn_bench.log | grep '^{'
step bench timeout -k 10 200 python bench.py > gpurun_out/bench_attn.log 2>&1; grep '^{' gpurun_out/bench_attn.log
