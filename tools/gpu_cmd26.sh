set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; echo rc=$?
grep "^{" gpurun_out/gemm_bench.log
GEMM_SHAPES=ksweep timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_ksweep.log 2>&1; echo rc=$?
grep "^{" gpurun_out/gemm_ksweep.log
exit 0
