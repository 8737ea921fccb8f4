set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2 3 4; do
  LUMEN_F8_VARIANT=$v timeout -k 10 120 python -u -m pytest tests/test_fp8_gpu.py -x -q -k "f8" --timeout 60 > gpurun_out/f8t_$v.log 2>&1 || { echo "test fail v=$v"; tail -5 gpurun_out/f8t_$v.log; exit 1; }
  LUMEN_F8_VARIANT=$v timeout -k 10 200 python -u tools/f8_gemm_bench.py --rounds 3 > gpurun_out/f8b_$v.log 2>&1 || exit 1
  echo "v=$v"; grep shape gpurun_out/f8b_$v.log | python3 -c "import sys,json
for l in sys.stdin:
  d=json.loads(l); print(d['shape'], d['f8f8_us'], d['f8f8_tflops'], 'blas_f8', d.get('blas_f8_us'))"
done
