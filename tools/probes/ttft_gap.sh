set -o pipefail
# TTFT with back-to-back requests vs 20 ms idle between them (same box, one model load each)
for gap in 0 20 0 20; do
  timeout -k 10 300 python -u tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 15 --warmup 2 --max-new 16 --batch 0 --gap-ms $gap > gpurun_out/ttft_gap_$gap.log 2>&1 || { echo "gap $gap failed"; tail -5 gpurun_out/ttft_gap_$gap.log; exit 1; }
  echo "gap=$gap $(grep '^{' gpurun_out/ttft_gap_$gap.log | tail -1)"
done
