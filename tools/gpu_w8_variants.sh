# decode fp8 GEMM variants (unroll depth, non-temporal weight loads): microbench + 8B decode per variant
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 1 2 3; do
  LUMEN_W8_SKINNY=$v timeout -k 10 120 python tools/w8_decode_bench.py >> gpurun_out/w8_variants.jsonl 2> gpurun_out/w8_err_$v.log || exit 1
done
cat gpurun_out/w8_variants.jsonl
timeout -k 10 120 python -u -m pytest tests/test_fp8_gpu.py tests/test_llm_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_w8.log 2>&1 || { tail -20 gpurun_out/pytest_w8.log; exit 1; }
tail -1 gpurun_out/pytest_w8.log
for v in 1 3; do
  LUMEN_W8_SKINNY=$v timeout -k 10 300 python tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 5 --max-new 64 --batch 16 > gpurun_out/vlm8b_fp8_v$v.log 2>&1 || exit 1
  grep '^{' gpurun_out/vlm8b_fp8_v$v.log
done
