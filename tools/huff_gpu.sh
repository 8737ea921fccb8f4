set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu_entropy_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/huff_tests.log 2>&1 || { echo tests_failed; tail -30 gpurun_out/huff_tests.log; exit 1; }
tail -2 gpurun_out/huff_tests.log
timeout -k 10 200 python -u tools/jpeg_huff_prof.py --n 10 > gpurun_out/huff_prof.log 2>&1 || { echo prof_failed; tail -20 gpurun_out/huff_prof.log; exit 1; }
timeout -k 10 200 python -u tools/jpeg_huff_prof.py --n 5 --kind noise --lanes 1024,2048 >> gpurun_out/huff_prof.log 2>&1
cat gpurun_out/huff_prof.log
