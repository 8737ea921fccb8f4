set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_postproc_gpu.py tests/test_ocr_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/ocr_tests.log 2>&1 || { tail -30 gpurun_out/ocr_tests.log; exit 1; }
tail -1 gpurun_out/ocr_tests.log
timeout -k 10 300 python tools/face_ocr_bench.py --what ocr --predecoded > gpurun_out/ocr_pre2.log 2>&1; grep '^{' gpurun_out/ocr_pre2.log | cut -c1-700
