# rocprofv3 kernel trace of Llama-3-8B (LLaVA) single-stream + batched decode, bf16 and fp8 weights
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_v8 -o run -- python3 tools/vlm_bench.py --preset llava-llama3-8b --n 3 --warmup 1 --max-new 32 --batch 16 --fp8 > gpurun_out/prof_v8.log 2>&1
rc=$?; echo "prof rc=$rc"; grep '^{' gpurun_out/prof_v8.log
find gpurun_out/prof_v8 -name "*kernel_stats.csv"
exit $rc
