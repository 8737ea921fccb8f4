set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step tests timeout -k 10 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fp8.log 2>&1; tail -3 gpurun_out/pytest_fp8.log
grep -q " passed" gpurun_out/pytest_fp8.log && ! grep -q "failed" gpurun_out/pytest_fp8.log || exit 1
step v8bf16 timeout -k 10 400 python tools/vlm_bench.py --preset llava-llama3-8b --n 10 --max-new 64 --batch 16 > gpurun_out/vlm8b_bf16.log 2>&1; grep '^{' gpurun_out/vlm8b_bf16.log
step v8fp8 timeout -k 10 400 python tools/vlm_bench.py --preset llava-llama3-8b --n 10 --max-new 64 --batch 16 --fp8 > gpurun_out/vlm8b_fp8.log 2>&1; grep '^{' gpurun_out/vlm8b_fp8.log
exit 0
