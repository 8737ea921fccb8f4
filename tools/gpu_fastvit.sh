# FastViT / MobileCLIP2 / FastVLM GPU checks + FastVLM TTFT bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return $rc; }
step tests timeout -k 10 400 python -u -m pytest tests/test_fastvit_gpu.py tests/test_clip_gpu.py tests/test_vlm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_fastvit.log 2>&1; tail -12 gpurun_out/pytest_fastvit.log
grep -q " passed" gpurun_out/pytest_fastvit.log && ! grep -q "failed" gpurun_out/pytest_fastvit.log || exit 1
step vlm timeout -k 10 300 python tools/vlm_bench.py --preset fastvlm-0.5b --n 10 --max-new 64 --batch 16 > gpurun_out/vlm05_fastvit.log 2>&1; grep '^{' gpurun_out/vlm05_fastvit.log
