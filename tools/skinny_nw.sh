# A/B of the decode skinny fp8 kernel's waves per workgroup (LUMEN_W8_SKINNY_NW) at M = 1 and 16
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_fp8_gpu.py tests/test_llm_ops_gpu.py -x -q --timeout 60 > gpurun_out/sk_tests.log 2>&1 || { tail -5 gpurun_out/sk_tests.log; exit 1; }
for nw in 4 8 16; do
  for m in 1 16; do
    echo "NW=$nw M=$m"
    LUMEN_W8_SKINNY_NW=$nw timeout -k 10 120 python -u tools/f8_gemm_bench.py --M $m --iters 50 --rounds 3 2>&1 | grep shape || exit 1
  done
done
