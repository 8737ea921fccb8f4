"""Where a single-image device JPEG decode spends its host time (utils/jpeg.py decode_to_device):
stage-by-stage host timings, back to back and with idle gaps like the TTFT loop's."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from lumen_amd.utils import jpeg

data = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "photo_probe.jpg"), "rb").read()
dev = torch.device("cuda")
for gap in (0.0, 0.015):
    rows = []
    for it in range(40):
        if gap:
            time.sleep(gap)
        t = [time.perf_counter()]
        ji = jpeg.info(data)
        t.append(time.perf_counter())
        n = ji.coef_count
        st = torch.empty(n, dtype=torch.int16).pin_memory() if it == 0 else st
        t.append(time.perf_counter())
        res = jpeg.decode_coefs(data, None, ji, out=st[:n].numpy())
        t.append(time.perf_counter())
        cd = st[:n].to(dev, non_blocking=True)
        t.append(time.perf_counter())
        img = jpeg.decode_image(data, dev)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        if it >= 5:
            rows.append(np.diff(t) * 1e3)
    r = np.median(np.array(rows), 0)
    print(f"gap {gap * 1e3:.0f} ms: info {r[0]:.3f} pin {r[1]:.3f} decode_coefs {r[2]:.3f} h2d {r[3]:.3f} "
          f"full decode_image {r[4]:.3f} ms", flush=True)
