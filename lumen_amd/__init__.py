"""lumen_amd — MI355X-native (gfx950) multi-modal image-understanding stack.

Same capabilities and module API as EdwinZhanCN/Lumen (CLIP / BioCLIP /
SmartCLIP embeddings and zero-shot classification, face detection and
embedding, OCR, vision-language generation behind the ``home_native.v1``
gRPC contract and the lumen-app control plane), re-designed for CDNA4:
hand-written HIP kernels on MFMA registered as ``torch.ops.lumen.*``, one
process per GPU with RCCL (``torch.distributed`` "nccl") over xGMI for data
and tensor parallelism.

Sub-packages:
  ops        compute ops (HIP kernels on GPU, PyTorch reference on CPU)
  models     model families (CLIP ViT/text, BERT, SCRFD, IResNet, DBNet, SVTR, LLM decoder)
  parallel   process groups, DP engine, TP layers, collectives
  runtime    batching, KV-cache manager, schedulers
  resources  config / model_info / result schemas / downloader / synthetic models
  proto      home_native.v1 protobuf messages and gRPC service plumbing
  services   CLIP / BioCLIP / SmartCLIP / face / OCR / VLM gRPC services
  hub        multi-service router + server (`lumen` entry point)
  app        FastAPI control plane (`lumen-webui`)
"""

__version__ = "0.1.0"

from ._native import load_hip, native_status  # noqa: E402,F401
