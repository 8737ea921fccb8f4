set -o pipefail
# same-box A/B of the batched face alignment geometry (arm slow: the per-face similarity + inverse loop)
# (the "fast" arm needs the batched geometry that lost this A/B and was reverted: profiles/r6_face_geom_ab_v1.txt)
for arm in slow fast slow fast; do
  timeout -k 10 300 python -c "
import sys, runpy, numpy as np
import lumen_amd.ops.vision as v
if '$arm' == 'slow':
    v.similarity_minv_batch = lambda src, dst=v.ARCFACE_DST: np.stack([v.invert_affine(v.similarity_transform(s, dst)) for s in src])
sys.argv = ['tools/face_ocr_bench.py', '--what', 'face', '--real-dets', '--batch', '32', '--iters', '10']
runpy.run_path('tools/face_ocr_bench.py', run_name='__main__')
" > gpurun_out/fgeom_$arm.log 2>&1 || { echo "arm $arm failed"; tail -5 gpurun_out/fgeom_$arm.log; exit 1; }
  echo "arm=$arm $(grep '^{' gpurun_out/fgeom_$arm.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["value"],1), d.get("host_stage_ms_per_batch"))')"
done
