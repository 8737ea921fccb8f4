# decode-path kernels: numerics tests, then LLaVA-Llama-3-8B decode bench (bf16 + fp8) and a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step tests timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_llm_ops_gpu.py tests/test_kernels_gpu.py tests/test_vlm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dec.log 2>&1; tail -3 gpurun_out/pytest_dec.log
grep -q " passed" gpurun_out/pytest_dec.log && ! grep -q " failed" gpurun_out/pytest_dec.log || exit 1
step v8fp8 timeout -k 10 400 python tools/vlm_bench.py --preset llava-llama3-8b --n 10 --max-new 64 --batch 16 --fp8 > gpurun_out/vlm8b_fp8.log 2>&1; grep '^{' gpurun_out/vlm8b_fp8.log
step v8bf16 timeout -k 10 400 python tools/vlm_bench.py --preset llava-llama3-8b --n 10 --max-new 64 --batch 16 > gpurun_out/vlm8b_bf16.log 2>&1; grep '^{' gpurun_out/vlm8b_bf16.log
step prof timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v8b -o run -- python3 tools/vlm_bench.py --preset llava-llama3-8b --n 3 --warmup 1 --max-new 32 --batch 16 --fp8 > gpurun_out/prof_v8b.log 2>&1
exit 0
