"""Draw face detections (bbox + 5 landmarks + score) on an image
(reference packages/lumen-face/scripts/visualize_detection.py:39-293, PIL instead of cv2).

usage: python tools/visualize_detection.py --config lumen-config.yaml --image in.jpg --out out.jpg
       python tools/visualize_detection.py --json face_v1.json --image in.jpg --out out.jpg
"""
from __future__ import annotations

import argparse
import json
import os
import sys

from PIL import Image, ImageDraw

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COLORS = [(255, 64, 64), (64, 255, 64), (64, 64, 255), (255, 255, 64), (255, 64, 255)]


def draw(img: Image.Image, faces: list[dict]) -> Image.Image:
    out = img.convert("RGB").copy()
    d = ImageDraw.Draw(out)
    for f in faces:
        x1, y1, x2, y2 = f["bbox"]
        d.rectangle([x1, y1, x2, y2], outline=(0, 255, 0), width=2)
        d.text((x1, max(0, y1 - 12)), f"{f.get('confidence', 0):.2f}", fill=(0, 255, 0))
        lm = f.get("landmarks") or []
        for k in range(0, len(lm) - 1, 2):
            x, y = lm[k], lm[k + 1]
            c = COLORS[(k // 2) % len(COLORS)]
            d.ellipse([x - 2, y - 2, x + 2, y + 2], fill=c)
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--image", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--json", help="face_v1 JSON produced by face_detect")
    ap.add_argument("--config", help="lumen config with a face service (runs detection in-process)")
    ap.add_argument("--threshold", type=float, default=0.5)
    a = ap.parse_args()
    img = Image.open(a.image)
    if a.json:
        faces = json.load(open(a.json))["faces"]
    else:
        from lumen_amd.resources.validator import load_and_validate_config
        from lumen_amd.services.face import GeneralFaceService

        cfg = load_and_validate_config(a.config)
        key = next(k for k, s in cfg.services.items() if s.package == "lumen_face")
        svc = GeneralFaceService.from_config(cfg.services[key], cfg.cache_path())
        svc.initialize()
        res, _, _ = svc.handle("face_detect", open(a.image, "rb").read(), "image/jpeg",
                               {"detection_confidence_threshold": str(a.threshold)})
        faces = json.loads(res)["faces"]
        svc.close()
    draw(img, faces).save(a.out)
    print(f"{len(faces)} face(s) -> {a.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
