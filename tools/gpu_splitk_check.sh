# in-kernel split-K reduction: GPU tests, then the LLaVA-Llama-3-8B (fp8 + bf16) and FastVLM-0.5B benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 10 --max-new 64 --batch 16 > gpurun_out/vlm8b_fp8.log 2>&1 || exit 1
grep '^{' gpurun_out/vlm8b_fp8.log
timeout -k 10 300 python tools/vlm_bench.py --preset llava-llama3-8b --n 10 --max-new 64 --batch 16 > gpurun_out/vlm8b_bf16.log 2>&1 || exit 1
grep '^{' gpurun_out/vlm8b_bf16.log
timeout -k 10 300 python tools/vlm_bench.py --preset fastvlm-0.5b --n 10 --max-new 64 --batch 16 > gpurun_out/vlm05.log 2>&1 || exit 1
grep '^{' gpurun_out/vlm05.log
