set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/face_ocr_bench.py --what ocr --predecoded > gpurun_out/ocr_pre3.log 2>&1; grep '^{' gpurun_out/ocr_pre3.log | cut -c1-700
timeout -k 10 300 python -u tools/serve_bench.py --service clip --model CLIP-ViT-L-14 --device cuda --clients 64 --seconds 15 > gpurun_out/serve_clip2.log 2>&1; grep '^{' gpurun_out/serve_clip2.log
