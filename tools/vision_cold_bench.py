"""LLaVA ViT-L/14-336 vision tower + projector for one 1024x768 image with L2 / MALL flushed before
every call (as in serving, where the 8B decoder streams its weights between requests): GPU ms."""
import copy, json, statistics, sys, time
sys.path.insert(0, ".")
import torch
from lumen_amd._native import load_hip
from lumen_amd.models.llm import LLM_PRESETS
from lumen_amd.models.vlm import VLM, VLM_PRESETS
load_hip(required=True)
cfg = copy.deepcopy(VLM_PRESETS["llava-llama3-8b"]); cfg.llm = LLM_PRESETS["tiny"]; cfg.image_token_id = 259
m = VLM(cfg, device="cuda"); m.random_init(0)
img = torch.randint(0, 256, (768, 1024, 3), dtype=torch.uint8).cuda()
flush = torch.empty(2 << 30, dtype=torch.uint8, device="cuda")
for _ in range(3): m.encode_images([img])
ts = []
for _ in range(20):
    flush.fill_(1)            # evict L2 / MALL (2 GiB write)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); m.encode_images([img]); e1.record(); e1.synchronize()
    ts.append(e0.elapsed_time(e1))
print(json.dumps({"vision_cold_ms": round(statistics.median(ts), 3)}))
