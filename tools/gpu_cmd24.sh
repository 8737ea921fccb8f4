set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/gemm_timeline.py > gpurun_out/gemm_timeline.log 2>&1; echo rc=$?
cat gpurun_out/gemm_timeline.log | grep -v amdgpu.ids
exit 0
