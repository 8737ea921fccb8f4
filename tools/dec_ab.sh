set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_llm_ops_gpu.py tests/test_vlm_gpu.py tests/test_fp8_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -2 gpurun_out/dec_tests.log
for p in 0 1 2; do
  LUMEN_DECODE_PREFETCH=$p timeout -k 10 300 python tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 30 --batch 16 > gpurun_out/dec_pf$p.log 2>&1 || { tail -20 gpurun_out/dec_pf$p.log; exit 1; }
  echo "pf=$p $(grep '^{' gpurun_out/dec_pf$p.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), round(d["decode_tok_s_single"],1), round(d["batch_decode_tok_s"],1))')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec -o run -- python3 tools/vlm_bench.py --preset llava-llama3-8b --n 3 --warmup 1 --max-new 64 --batch 1 --fp8 > gpurun_out/prof_dec.log 2>&1
echo prof rc=$?
