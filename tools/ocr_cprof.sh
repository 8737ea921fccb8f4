set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m cProfile -o gpurun_out/ocr.pstats tools/face_ocr_bench.py --what ocr --predecoded --iters 5 > gpurun_out/ocr_cprof.log 2>&1; echo rc=$?
python -c "
import pstats; p=pstats.Stats('gpurun_out/ocr.pstats'); p.sort_stats('tottime').print_stats(30)" > gpurun_out/ocr_pstats.txt 2>&1
grep "^{" gpurun_out/ocr_cprof.log | cut -c1-300
