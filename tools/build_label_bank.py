"""Offline label-bank builder (reference packages/lumen-clip/scripts/compute_bioclip_bank.py,
SURVEY C16): encode every label with a model pack's text tower and write the bank in the
on-disk layout the services memory-map:

  <model>/datasets/<name>_labels.json      JSON list (TreeOfLife entries may be
                                           [[taxonomy...], common_name])
  <model>/datasets/<name>_embeddings.npy   float32 [N, D], rows L2-normalised
  model_info.json  datasets.<name> = {labels, embeddings}

Prompts follow the managers: CLIP "a photo of a {label}", BioCLIP "a photo of {name}"
with name = common name or "Genus species".  The text tower runs in batches of 512 on
the MI355X kernels (or the CPU reference with --device cpu).

Multi-GPU: launched with torchrun (one process per GPU), every rank encodes its contiguous
shard of the labels on its own GPU and parallel.DataParallelRunner all-gathers the rows over
RCCL (gloo on the CPU); rank 0 writes the bank.

usage: python tools/build_label_bank.py --cache ~/.lumen --model bioclip-2 --dataset TreeOfLife-10M \
           --labels names.json [--bio] [--device cuda]
       torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/build_label_bank.py ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bio_name(entry) -> str:
    if isinstance(entry, (list, tuple)) and len(entry) == 2 and isinstance(entry[0], (list, tuple)):
        tax, common = entry
        if common:
            return str(common)
        return " ".join(str(t) for t in tax[-2:]) if len(tax) >= 2 else str(tax[-1])
    return str(entry)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cache", required=True)
    ap.add_argument("--model", required=True)
    ap.add_argument("--dataset", required=True)
    ap.add_argument("--labels", required=True, help="JSON list of labels")
    ap.add_argument("--bio", action="store_true", help="BioCLIP prompt / TreeOfLife label format")
    ap.add_argument("--device", default=None)
    ap.add_argument("--runtime", default="torch")
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()

    from lumen_amd.resources.config import ModelConfig, Runtime
    from lumen_amd.services.clip.backend import create_backend
    from lumen_amd.services.clip.resources import ResourceLoader

    labels = json.load(open(a.labels))
    mc = ModelConfig(model=a.model, runtime=Runtime(a.runtime))
    res = ResourceLoader.load_model_resources(a.cache, mc)

    class _S:
        device = a.device
        batch_size = a.batch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    st = None
    if world > 1:
        import torch

        from lumen_amd.parallel.state import init_distributed

        local = int(os.environ.get("LOCAL_RANK", "0"))
        gpu = (a.device or "cuda").startswith("cuda") and torch.cuda.is_available()
        st = init_distributed(tp_size=1, device=torch.device("cuda", local) if gpu else torch.device("cpu"))
        _S.device = f"cuda:{local}" if gpu else "cpu"

    be = create_backend(_S(), res, a.runtime)
    be.initialize()
    prompts = [f"a photo of {bio_name(l)}" if a.bio else f"a photo of a {l}" for l in labels]

    def encode(items):
        embs = []
        for i in range(0, len(items), a.batch):
            embs.append(np.asarray(be.text_batch_to_vectors(items[i:i + a.batch]), np.float32))
            print(f"\r{min(i + a.batch, len(items))}/{len(items)}", end="", flush=True)
        print()
        return np.concatenate(embs) if embs else np.zeros((0, be.cfg.embed_dim), np.float32)

    if st is None:
        emb = encode(prompts)
    else:
        import torch

        from lumen_amd.parallel import Communicator, DataParallelRunner

        comm = Communicator(st.dp_group, st.device, ipc=False)
        run = DataParallelRunner(lambda items: torch.from_numpy(encode(list(items))).to(st.device), comm)
        emb = run.run(prompts).cpu().numpy()
        if st.rank != 0:
            be.close()
            return 0
    emb = emb.astype(np.float32)
    emb /= np.maximum(np.linalg.norm(emb, axis=1, keepdims=True), 1e-12)
    root = Path(res.model_root_path)
    (root / "datasets").mkdir(exist_ok=True)
    lab_rel, emb_rel = f"datasets/{a.dataset}_labels.json", f"datasets/{a.dataset}_embeddings.npy"
    (root / lab_rel).write_text(json.dumps(labels, ensure_ascii=False))
    np.save(root / emb_rel, emb)
    info = json.loads((root / "model_info.json").read_text())
    info.setdefault("datasets", {}) or info.__setitem__("datasets", {})
    if info["datasets"] is None:
        info["datasets"] = {}
    info["datasets"][a.dataset] = {"labels": lab_rel, "embeddings": emb_rel}
    (root / "model_info.json").write_text(json.dumps(info, indent=2))
    print(f"wrote {emb.shape} bank to {root / emb_rel}")
    be.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
