set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests/test_face_gpu.py -q -x > gpurun_out/pytest_face.log 2>&1; rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_face.log
tail -40 gpurun_out/pytest_face.log
exit $rc
