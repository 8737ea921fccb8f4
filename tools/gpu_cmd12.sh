set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_vlm_gpu.py tests/test_llm_ops_gpu.py -q -x > gpurun_out/pytest_vlm.log 2>&1; rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_vlm.log
tail -30 gpurun_out/pytest_vlm.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/vlm_bench.py --preset fastvlm-0.5b --n 20 --max-new 64 --batch 16 > gpurun_out/vlm_bench_05b.log 2>&1; rc=$?
tail -5 gpurun_out/vlm_bench_05b.log
exit $rc
