set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/face_ocr_bench.py --what ocr --predecoded > gpurun_out/ocr_pre.log 2>&1; grep '^{' gpurun_out/ocr_pre.log | cut -c1-600
timeout -k 10 300 python tools/face_ocr_bench.py --what ocr --predecoded --image-kind photo > gpurun_out/ocr_pre_photo.log 2>&1; grep '^{' gpurun_out/ocr_pre_photo.log | cut -c1-600
timeout -k 10 300 python tools/face_ocr_bench.py --what face --predecoded --batch 32 > gpurun_out/face_pre.log 2>&1; grep '^{' gpurun_out/face_pre.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ocr -o run -- python3 tools/face_ocr_bench.py --what ocr --iters 3 --predecoded > gpurun_out/prof_ocr.log 2>&1; echo prof_ocr rc=$?
timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM -d gpurun_out/pmc_face_sq -o run -- python3 tools/face_ocr_bench.py --what face --iters 1 --warmup 1 --predecoded > gpurun_out/pmc_face.log 2>&1; echo pmc rc=$?
