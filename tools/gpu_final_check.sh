# full GPU tests, smoke, headline bench and the VLM TTFT benches (8B fp8 / bf16, FastVLM-0.5B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
timeout -k 10 240 python bench.py > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
timeout -k 10 300 python tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 10 --max-new 64 --batch 16 > gpurun_out/vlm8b_fp8.log 2>&1 || exit 1
grep '^{' gpurun_out/vlm8b_fp8.log
timeout -k 10 300 python tools/vlm_bench.py --preset fastvlm-0.5b --n 10 --max-new 64 --batch 16 > gpurun_out/vlm05.log 2>&1 || exit 1
grep '^{' gpurun_out/vlm05.log
