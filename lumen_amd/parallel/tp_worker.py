"""Follower rank of a TP serving group: ``python -m lumen_amd.parallel.tp_worker '<json spec>'``.

Spec (written by :class:`~lumen_amd.parallel.tp.TPServingGroup`): ``cache_dir``,
``model``, ``runtime``, ``precision``, ``device``, ``kv_blocks``, ``max_batch``,
``timeout_s``.  The process joins the group (env RANK / WORLD_SIZE / MASTER_*),
loads its weight shard through the same VLM backend code as the leader, then
replays the leader's engine steps until the stop message.
"""
from __future__ import annotations

import json
import logging
import os
import sys


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    spec = json.loads(argv[0])
    logging.basicConfig(level=os.environ.get("LUMEN_LOG_LEVEL", "WARNING"))
    import torch

    from ..resources.config import ModelConfig, Runtime
    from ..services.common import load_model_resources
    from ..services.vlm.backend import MI355XVLMBackend
    from .state import destroy, env_world, init_distributed

    rank, world, _ = env_world()
    dev = torch.device(spec.get("device") or "cpu")
    st = init_distributed(tp_size=world, rank=rank, world=world, device=dev, timeout_s=float(spec.get("timeout_s", 600)),
                          init_method=f"tcp://{os.environ['MASTER_ADDR']}:{os.environ['MASTER_PORT']}")
    try:
        mc = ModelConfig(model=spec["model"], runtime=Runtime(spec["runtime"]), precision=spec.get("precision"))
        res = load_model_resources(spec["cache_dir"], mc, ("tokenizer_config.json", "lumen_vlm_config.json"))
        be = MI355XVLMBackend(res, device=str(dev), tp=st.tp_info(), kv_blocks=int(spec.get("kv_blocks", 0)),
                              max_batch=int(spec.get("max_batch", 64)))
        be.run_follower()
    finally:
        destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
