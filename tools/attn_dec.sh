set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_attn -o run -- python3 tools/decode_attn_bench.py --iters 100 > gpurun_out/attn_dec.log 2>&1
echo rc=$?; grep '^{' gpurun_out/attn_dec.log
