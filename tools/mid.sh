set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_llm_ops_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/dec_tests2.log 2>&1 || { tail -30 gpurun_out/dec_tests2.log; exit 1; }
tail -1 gpurun_out/dec_tests2.log
timeout -k 10 200 python tools/decode_attn_bench.py --iters 50 > gpurun_out/attn2.log 2>&1; tail -1 gpurun_out/attn2.log
timeout -k 10 300 python tools/mid_gemm_bench.py --tiles=-1,2,1,20000,20002,20003,20005,1609,1001 > gpurun_out/mid577.log 2>&1; tail -1 gpurun_out/mid577.log
timeout -k 10 300 python tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 30 --batch 16 > gpurun_out/vlm8b_r3b.log 2>&1; grep '^{' gpurun_out/vlm8b_r3b.log | cut -c1-400
