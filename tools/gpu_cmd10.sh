set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_postproc_gpu.py tests/test_ocr_gpu.py tests/test_face_gpu.py -q -x > gpurun_out/pytest_ocr.log 2>&1; rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ocr.log
tail -40 gpurun_out/pytest_ocr.log
exit $rc
