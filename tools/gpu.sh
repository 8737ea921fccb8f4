# GPU-box task runner (run through gpurun): bash tools/gpu.sh TASK [TASK ...]
#
# Every GPU step runs under its own time limit; the first step that faults, aborts or
# times out ends the script (no retries).  Outputs land in gpurun_out/.
#
#   tests          pytest -m gpu (one process, 120 s per test)
#   tsel           pytest -m gpu on $TESTS only (one process)
#   smoke          __graft_entry__.smoke()
#   bench          headline bench.py (defaults)
#   prof_bench     rocprofv3 kernel stats of the headline bench (3 steps)
#   gemm           tools/gemm_bench_tiles.py on the ViT-L/14 shapes ($GEMM_TILES, $GEMM_EPI)
#   llm_tests      fp8 / LLM-op / VLM GPU tests only
#   cnn_tests      conv / face / OCR / FastViT GPU tests only
#   post_tests     post-processing / image kernels / OCR GPU tests only
#   tp             TP=2 (two ranks sharing the GPU) tests + tools/tp_decode_bench.py (8B fp8)
#   w8bench        tools/w8_decode_bench.py: HBM-cold decode GEMMs ($W8_M rows, default 1,16)
#   vlm8b / vlm05  tools/vlm_bench.py Llama-3-8B fp8 / FastVLM-0.5B (vlm8b_quick: 30 requests)
#   prof_ttft      rocprofv3 kernel trace of 3 single-request TTFTs (8B fp8, 2 new tokens)
#   prof_vlm8b     rocprofv3 kernel stats of the 8B fp8 decode bench (batch 16; prof_vlm8b_b1: single stream)
#   face_ocr       tools/face_ocr_bench.py face + ocr
#   conv           conv_lds variants on the IResNet shapes (tools/conv_bench.py) + LDS-pipeline tests
#   face           face bench pre-decoded (HIP-event stage timers, then host timers) + JPEG-inclusive
#   ocr            OCR bench pre-decoded (HIP-event stage timers) + JPEG-inclusive
#   prof_face / prof_ocr   rocprofv3 kernel stats of the face / OCR bench
#   f8             fp8 tests (tests/test_fp8_gpu.py) + tools/f8_gemm_bench.py ($F8_SHAPES, $F8_M)
#   pmc_face / pmc_ocr   PMC counters (SQ pass + memory pass) of the face / OCR pipelines
#   serve          tools/serve_bench.py: gRPC hub end to end (CLIP ViT-L/14 64 clients, face 32 clients)
#   serve_fe       serving through the engine / front-end topology (CLIP 128 clients, face 64; $SERVE_FE front ends)
#   serve_sweep    CLIP serving through the engine / front ends: 8 / 12 front ends x 128 / 256 clients
#   jpeg           device JPEG tests + tools/jpeg_bench.py
#   mx             MX W8A8 chain tests (tests/test_mx_gpu.py) + fp8 GEMM + LLM-op tests
#   ttft           VLM TTFT only (8B fp8, 30 requests, device JPEG decode)
#   mx_cold        cold-weight timing of the MX chain's GEMMs (full / plain epilogues) vs per-token fp8
#   pp_cold        ping-pong 128x128 pipeline forms vs the aligned ones (fp8 prefill + bf16 vision shapes)
#   f8auto         fp8 tests + cold prefill GEMMs (auto vs codes 1, 2, 16, 17)
#   vlm_tests      VLM / engine GPU tests + GPU entropy JPEG tests
#   acc            full-size fp8 accuracy pins (ViT-L/14-336 W8A8, Llama-3-8B first token)
#   vlm_service    service-level TTFT: gRPC vlm_generate_stream first chunk (tools/vlm_service_ttft.py)
#   vlm_service_fe the same through 2 front ends + 1 GPU engine, 32 streamed tokens
#   vlm_service32  in-process hub, 32 streamed tokens (inter-chunk time, engine counters)
#   attn           tools/attn_bench.py (ViT / text / prefill shapes; split-tail switch A/B)
#   serve128       CLIP serving through 8 front ends, 128 clients from 6 client processes
#   fe_gpu         engine / front-end topology GPU test (tests/test_frontends_gpu.py)
#   face_real      face bench on the detector's real output (detect_and_embed_images; SPMD path under torchrun)
#   shrink         rocpd databases under gpurun_out -> kernel-stats / PMC text, databases > 4 MB removed (64 MiB copy-back cap)
#   pmc_attn       PMC counters (MFMA-busy, LDS, VALU, clock) of tools/attn_bench.py
#   pmc_gemm       PMC counters (MFMA, LDS conflicts, busy) of one ViT-L/14 GEMM shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp

step() {   # step NAME SECONDS CMD...  (stdout+stderr -> gpurun_out/NAME.log)
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  tail -3 "gpurun_out/$name.log"
  case $rc in 0) ;; *) exit $rc ;; esac
}

for task in "$@"; do
  case $task in
    tests) step tests 900 python -u -m pytest tests -m gpu --maxfail=15 -q --timeout 120 --timeout-method thread ;;
    tsel) step tsel 600 python -u -m pytest ${TESTS:-tests/test_comm_gpu.py} -m gpu -x -v --timeout 120 \
        --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 400 python bench.py ;;
    prof_bench)
      step prof_bench 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- \
        python3 bench.py --steps 3 --warmup 1 --text-steps 3 ;;
    gemm)
      step gemm 500 python -u tools/gemm_bench_tiles.py --tiles="${GEMM_TILES:--1}" --epi "${GEMM_EPI:-plain}" \
        --shapes "${GEMM_SHAPES:-vit}" ;;
    f8)
      step f8_tests 300 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread
      step f8_bench 300 python -u tools/f8_gemm_bench.py --M "${F8_M:-624}" --shapes "${F8_SHAPES:-llama8b}" ;;
    llm_tests)
      step llm_tests 400 python -u -m pytest tests/test_fp8_gpu.py tests/test_llm_ops_gpu.py tests/test_vlm_gpu.py \
        -x -q --timeout 120 --timeout-method thread ;;
    w8bench) step w8bench 300 python -u tools/w8_decode_bench.py --m "${W8_M:-1,16}" ;;
    cnn_tests)
      step cnn_tests 400 python -u -m pytest tests/test_cnn_gpu.py tests/test_face_gpu.py tests/test_face_onnx_gpu.py \
        tests/test_ocr_gpu.py tests/test_fastvit_gpu.py -x -q --timeout 120 --timeout-method thread ;;
    post_tests)
      step post_tests 300 python -u -m pytest tests/test_postproc_gpu.py tests/test_kernels_gpu.py tests/test_ocr_gpu.py \
        -x -q --timeout 120 --timeout-method thread ;;
    vlm8b) step vlm8b 600 python tools/vlm_bench.py --preset llava-llama3-8b --fp8 ;;
    vlm8b_quick) step vlm8b_quick 400 python tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 30 ;;
    tp)
      step tp_tests 300 python -u -m pytest tests/test_tp_gpu.py tests/test_comm_gpu.py -x -q --timeout 200 \
        --timeout-method thread
      step tp2_bench 500 python -u tools/tp_decode_bench.py --preset llava-llama3-8b --tp 2 --fp8 --share-gpu ;;
    vlm05) step vlm05 400 python tools/vlm_bench.py --preset fastvlm-0.5b ;;
    prof_vlm8b)
      step prof_vlm8b 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vlm8b -o run -- \
        python3 tools/vlm_bench.py --preset llava-llama3-8b --n 3 --warmup 1 --max-new 32 --batch 16 --fp8 ;;
    prof_vlm8b_b1)
      step prof_vlm8b_b1 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vlm8b_b1 -o run -- \
        python3 tools/vlm_bench.py --preset llava-llama3-8b --n 3 --warmup 1 --max-new 64 --batch 1 --fp8 ;;
    prof_ttft)
      step prof_ttft 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ttft -o run -- \
        python3 tools/vlm_bench.py --preset llava-llama3-8b --n 3 --warmup 2 --max-new 2 --batch 0 --fp8 ;;
    face_ocr)
      step face 400 python tools/face_ocr_bench.py --what face
      step ocr 400 python tools/face_ocr_bench.py --what ocr ;;
    conv)   # conv_lds variants on the IResNet shapes (+ the LDS-pipeline numerics tests)
      step conv_tests 300 python -u -m pytest tests/test_cnn_gpu.py -x -q -k lds_pipeline --timeout 120 \
        --timeout-method thread
      step conv_bench 300 python -u tools/conv_bench.py ${CONV_ARGS:-} ;;
    face)
      step face_pre 300 python tools/face_ocr_bench.py --what face --predecoded --gpu-timers --batch 32
      step face_pre_host 300 python tools/face_ocr_bench.py --what face --predecoded --batch 32
      step face_jpeg 300 python tools/face_ocr_bench.py --what face ;;
    ocr)
      step ocr_pre 300 python tools/face_ocr_bench.py --what ocr --predecoded --gpu-timers
      step ocr_jpeg 300 python tools/face_ocr_bench.py --what ocr ;;
    prof_face)
      step prof_face 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_face -o run -- \
        python3 tools/face_ocr_bench.py --what face --iters 3 --batch 32 --predecoded ;;
    prof_ocr)
      step prof_ocr 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ocr -o run -- \
        python3 tools/face_ocr_bench.py --what ocr --iters 3 ;;
    pmc_face|pmc_ocr)
      w=${task#pmc_}
      step ${task}_sq 120 timeout -s KILL 100 rocprofv3 --kernel-trace \
        --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM \
        -d gpurun_out/${task}_sq -o run -- python3 tools/face_ocr_bench.py --what $w --iters 1 --warmup 1
      step ${task}_mem 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc FETCH_SIZE \
        -d gpurun_out/${task}_mem -o run -- python3 tools/face_ocr_bench.py --what $w --iters 1 --warmup 1 ;;
    pmc_gemm)
      step pmc_gemm 120 timeout -s KILL 100 rocprofv3 --kernel-trace \
        --pmc SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        -d gpurun_out/pmc_gemm -o run -- python3 tools/gemm_bench_tiles.py --tiles=609 --rounds 1 --iters 2 \
        --shapes "${GEMM_SHAPES:-131584x3072x1024}" ;;
    pmc_mfma)   # MFMA-busy / LDS / clock counters of the ViT GEMM tiles ($GEMM_TILES, $GEMM_SHAPES)
      step pmc_mfma 120 timeout -s KILL 100 rocprofv3 --kernel-trace \
        --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        -d gpurun_out/pmc_mfma -o run -- python3 tools/gemm_bench_tiles.py --tiles="${GEMM_TILES:-1839}" --rounds 1 \
        --iters 2 --shapes "${GEMM_SHAPES:-65792x3072x1024,65792x1024x4096}" ;;
    pmc_attn)   # MFMA-busy / LDS / VALU / clock counters of the attention bench kernels
      step pmc_attn 120 timeout -s KILL 100 rocprofv3 --kernel-trace \
        --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU \
        SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
        -d gpurun_out/pmc_attn -o run -- python3 tools/attn_bench.py ;;
    serve)
      step serve_clip 300 python -u tools/serve_bench.py --service clip --model CLIP-ViT-L-14 --device cuda --clients 64 \
        --seconds 20
      step serve_face 300 python -u tools/serve_bench.py --service face --model antelopev2 --device cuda --clients 32 \
        --seconds 20 ;;
    serve_fe)
      step serve_clip_fe 400 python -u tools/serve_bench.py --service clip --model CLIP-ViT-L-14 --device cuda \
        --clients "${SERVE_CLIENTS:-256}" --frontends "${SERVE_FE:-10}" --client-procs 12 --seconds 20
      step serve_face_fe 400 python -u tools/serve_bench.py --service face --model antelopev2 --device cuda \
        --clients "${SERVE_FACE_CLIENTS:-128}" --frontends "${SERVE_FE:-10}" --client-procs 12 --seconds 20 ;;
    serve_sweep)   # CLIP serving through front ends: front-end count x client count
      for fe in 8 12; do for cl in 128 256; do
        step serve_clip_fe${fe}_c${cl} 300 python -u tools/serve_bench.py --service clip --model CLIP-ViT-L-14 \
          --device cuda --clients $cl --frontends $fe --client-procs 6 --seconds 15
      done; done ;;
    serve_linger)   # engine merge window sweep (CLIP, 8 front ends, 256 clients)
      for lg in 2000 5000 10000; do
        step serve_clip_lg${lg} 300 env LUMEN_ENGINE_STATS_S=4 LUMEN_ENGINE_LINGER_US=$lg python -u tools/serve_bench.py \
          --service clip --model CLIP-ViT-L-14 --device cuda --clients 256 --frontends 8 --client-procs 6 --seconds 15
      done ;;
    jpeg)
      step jpeg_tests 200 python -u -m pytest tests/test_jpeg_gpu_entropy_gpu.py tests/test_jpeg_gpu.py tests/test_jpeg_cpu.py -x -q --timeout 120 \
        --timeout-method thread
      step jpeg_bench 300 python -u tools/jpeg_bench.py --n 20 ;;
    mx)
      step mx_tests 400 python -u -m pytest tests/test_mx_gpu.py tests/test_fp8_gpu.py tests/test_llm_ops_gpu.py -q \
        --timeout 120 --timeout-method thread ;;
    mx_cold)   # MX chain GEMMs (cold weights): full epilogues vs plain stores vs the per-token fp8 GEMMs
      step mx_cold_full 300 python -u tools/cold_gemm_bench.py --what mx --epi full --variants=0,1,2,4,10
      step mx_cold_plain 300 python -u tools/cold_gemm_bench.py --what mx --epi plain --variants=0,2
      step f8_cold 300 python -u tools/cold_gemm_bench.py --what prefill --variants=0,2 ;;
    pp_cold)   # ping-pong 128x128 forms (codes 12-15) vs the barrier-aligned ones, cold weights
      step pp_cold_f8 300 python -u tools/cold_gemm_bench.py --what prefill --variants=1,2,12,13,14,15
      step pp_cold_vit 300 python -u tools/cold_gemm_bench.py --what vit --variants=-1,20003,20022,20023,20024,20025 ;;
    f8auto)   # fp8 tests + cold-weight prefill GEMMs: auto selection vs the split-K / 256x256 ping-pong forms
      step f8_tests 400 python -u -m pytest tests/test_fp8_gpu.py -x -q --timeout 120 --timeout-method thread
      step f8_cold 300 python -u tools/cold_gemm_bench.py --what prefill --variants=0,1,2,16,17 ;;
    vlm_tests) step vlm_tests 400 python -u -m pytest tests/test_vlm_gpu.py tests/test_jpeg_gpu_entropy_gpu.py -x -q \
      --timeout 200 --timeout-method thread ;;
    acc) step acc 400 python -u -m pytest tests/test_fp8_accuracy_gpu.py -x -v --timeout 300 --timeout-method thread ;;
    vlm_service) step vlm_service 500 python -u tools/vlm_service_ttft.py --n 30 --max-new 1 ;;
    vlm_service32)   # in-process hub, 32 new tokens streamed (inter-chunk time + engine counters)
      step vlm_service32 500 python -u tools/vlm_service_ttft.py --n 20 --max-new 32 ;;
    attn) step attn 200 python -u tools/attn_bench.py ;;
    vlm_service_fe)   # service TTFT through 2 front ends + 1 engine, 32 new tokens streamed
      step vlm_service_fe 600 python -u tools/vlm_service_ttft.py --n 30 --max-new 32 --frontends 2 ;;
    serve128)   # CLIP through front ends, 128 clients from 6 client processes
      step serve128 400 python -u tools/serve_bench.py --service clip --model CLIP-ViT-L-14 --device cuda \
        --clients 128 --frontends "${SERVE_FE:-8}" --client-procs 6 --seconds 20 ;;
    fe_gpu) step fe_gpu 400 python -u -m pytest tests/test_frontends_gpu.py -x -q --timeout 300 --timeout-method thread ;;
    face_real)   # real detections at batch 32 (GPU stage timers, then host timers)
      step face_real_gpu 300 python -u tools/face_ocr_bench.py --what face --real-dets --batch 32 --iters 5 --gpu-timers
      step face_real 300 python -u tools/face_ocr_bench.py --what face --real-dets --batch 32 --iters 10 ;;
    shrink)   # summarise every rocpd database under gpurun_out (kernel stats, PMC sums), drop the big ones
      for db in $(find gpurun_out -name "*.db" -size +4M); do
        python tools/rocpd_stats.py "$db" "${db%.db}_stats.csv" --top 60 > "${db%.db}_stats.txt" 2>&1 || true
        python tools/rocpd_stats.py "$db" --pmc > "${db%.db}_pmc.txt" 2>&1 || true
        rm -f "$db"
      done
      echo "[shrink] done" ;;
    ttft) step ttft 400 python -u tools/vlm_bench.py --preset llava-llama3-8b --fp8 --n 30 --batch 0 ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
exit 0
