set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_llm_ops_gpu.py -q -x > gpurun_out/pytest_llm.log 2>&1; rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_llm.log
tail -40 gpurun_out/pytest_llm.log
exit $rc
