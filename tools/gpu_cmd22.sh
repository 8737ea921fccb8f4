set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/blas -o blas --output-format csv -- python tools/blas_names.py > gpurun_out/prof/blas.log 2>&1
echo rc=$?
exit 0
