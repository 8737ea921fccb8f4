"""How long does staging one face batch take?  32 decoded 1280x720 RGB images -> pinned buffer
(decode-pool memcpy) -> H2D on the uploader's side stream: host time until upload_async returns,
and until its copy completes.  Compare with the face pipeline's ~9.8 ms per batch."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from lumen_amd.utils.image import PinnedUploader  # noqa: E402

dev = torch.device("cuda", 0)
imgs = [np.random.default_rng(i).integers(0, 255, (720, 1280, 3), dtype=np.uint8) for i in range(32)]
up = PinnedUploader(dev)
for _ in range(3):
    up.upload_async(imgs)[2].synchronize()
host, full = [], []
for _ in range(20):
    t = time.perf_counter()
    d, o, ev = up.upload_async(imgs)
    host.append(time.perf_counter() - t)
    ev.synchronize()
    full.append(time.perf_counter() - t)
mb = sum(im.nbytes for im in imgs) / 1e6
print(f"batch {mb:.0f} MB: host staging {np.median(host) * 1e3:.2f} ms, staging + H2D {np.median(full) * 1e3:.2f} ms "
      f"({mb / np.median(full) / 1e3:.1f} GB/s)", flush=True)
