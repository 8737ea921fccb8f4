set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return $rc; }
step tests timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1; tail -3 gpurun_out/pytest_gpu_all.log
grep -q " passed" gpurun_out/pytest_gpu_all.log && ! grep -q "failed" gpurun_out/pytest_gpu_all.log || exit 1
step bench timeout -k 10 200 python bench.py > gpurun_out/bench_gemmfast.log 2>&1; grep '^{' gpurun_out/bench_gemmfast.log
