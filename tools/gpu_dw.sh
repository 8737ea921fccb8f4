set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py tests/test_fastvit_gpu.py tests/test_face_gpu.py tests/test_ocr_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dw.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_dw.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/dw_bench.py > gpurun_out/dw_bench.log 2>&1; echo "dw rc=$?"; grep '^{' gpurun_out/dw_bench.log
timeout -k 10 300 python tools/fastvit_bench.py > gpurun_out/fastvit_bench2.log 2>&1; echo "fv rc=$?"; grep '^{' gpurun_out/fastvit_bench2.log
