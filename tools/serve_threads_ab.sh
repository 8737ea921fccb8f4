# Engine batch loops per service (LUMEN_ENGINE_THREADS) A/B on face and CLIP serving (tools/serve_bench.py,
# 10 front ends), alternating on one box; outputs gpurun_out/serve_*_thr*.log
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for t in ${THREADS_AB:-2 3 2 3}; do
  LUMEN_ENGINE_THREADS=$t timeout -k 10 300 python -u tools/serve_bench.py --service face --model antelopev2 --device cuda \
    --clients 128 --frontends 10 --client-procs 12 --seconds 20 > gpurun_out/serve_face_thr$t.$RANDOM.log 2>&1 || exit 1
done
for t in ${THREADS_AB_CLIP:-2 3}; do
  LUMEN_ENGINE_THREADS=$t timeout -k 10 300 python -u tools/serve_bench.py --service clip --model CLIP-ViT-L-14 --device cuda \
    --clients 256 --frontends 10 --client-procs 12 --seconds 20 > gpurun_out/serve_clip_thr$t.log 2>&1 || exit 1
done
