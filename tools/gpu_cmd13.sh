set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
# run a GPU step; stop the whole script on timeout / abort / segfault (no further GPU work)
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; return 0; }
step vlmtest timeout -k 10 400 python -m pytest tests/test_vlm_gpu.py -q -x > gpurun_out/pytest_vlm.log 2>&1; tail -3 gpurun_out/pytest_vlm.log
step vlm05 timeout -k 10 300 python tools/vlm_bench.py --preset fastvlm-0.5b --n 20 --max-new 64 --batch 16 > gpurun_out/vlm_bench_05b.log 2>&1; tail -1 gpurun_out/vlm_bench_05b.log
step face timeout -k 10 300 python tools/face_ocr_bench.py --what face --batch 32 --faces 4 > gpurun_out/face_bench.log 2>&1; tail -2 gpurun_out/face_bench.log
step ocr timeout -k 10 300 python tools/face_ocr_bench.py --what ocr --batch 16 --crops 20 > gpurun_out/ocr_bench.log 2>&1; tail -2 gpurun_out/ocr_bench.log
step vlm8b timeout -k 10 400 python tools/vlm_bench.py --preset llava-llama3-8b --n 10 --max-new 32 --batch 16 > gpurun_out/vlm_bench_8b.log 2>&1; tail -2 gpurun_out/vlm_bench_8b.log
cd /tmp
step profvlm timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vlm05 -o vlm -- python3 $R/tools/vlm_bench.py --preset fastvlm-0.5b --n 5 --max-new 32 --batch 8 > $R/gpurun_out/prof_vlm05.log 2>&1
step profface timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_face -o face -- python3 $R/tools/face_ocr_bench.py --what face --batch 16 --iters 3 > $R/gpurun_out/prof_face.log 2>&1
exit 0
