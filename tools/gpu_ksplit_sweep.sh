# skinny split-K target workgroup count sweep on the Llama-3-8B decode shapes (+ 8B fp8 decode at the best two)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in 256 512 1024 2048; do
  LUMEN_SKINNY_TARGET_WG=$t timeout -k 10 120 python tools/w8_decode_bench.py | sed "s/^{/{\"target_wg\": $t, /" >> gpurun_out/ksplit_sweep.jsonl || exit 1
done
cat gpurun_out/ksplit_sweep.jsonl
