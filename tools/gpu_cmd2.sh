set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 && cat gpurun_out/gemm_bench.log && \
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1 && cat gpurun_out/bench.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1; echo "prof exit $?"
