set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step llmops timeout -k 10 500 python -m pytest tests/test_llm_ops_gpu.py tests/test_kernels_gpu.py -q -x > gpurun_out/pytest_llmops.log 2>&1; tail -5 gpurun_out/pytest_llmops.log
grep -q "passed" gpurun_out/pytest_llmops.log && ! grep -q "failed" gpurun_out/pytest_llmops.log || exit 1
step vlmtest timeout -k 10 400 python -m pytest tests/test_vlm_gpu.py -q -x > gpurun_out/pytest_vlm.log 2>&1; tail -3 gpurun_out/pytest_vlm.log
step vlm05 timeout -k 10 300 python tools/vlm_bench.py --preset fastvlm-0.5b --n 20 --max-new 64 --batch 16 > gpurun_out/vlm_bench_05b.log 2>&1; tail -1 gpurun_out/vlm_bench_05b.log
step vlm8b timeout -k 10 400 python tools/vlm_bench.py --preset llava-llama3-8b --n 10 --max-new 32 --batch 16 > gpurun_out/vlm_bench_8b.log 2>&1; tail -1 gpurun_out/vlm_bench_8b.log
cd /tmp
step profvlm timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vlm05b -o vlm -- python3 $R/tools/vlm_bench.py --preset fastvlm-0.5b --n 5 --max-new 32 --batch 8 > $R/gpurun_out/prof_vlm05b.log 2>&1
exit 0
