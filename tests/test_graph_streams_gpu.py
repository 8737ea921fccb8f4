"""hipGraphs replayed at the same time from different threads of one process:
the image-encoder graphs of two VLM models (models/vlm.py VLM._capture) are each captured on a private
stream, so their split-K tickets / workspaces (keyed by stream, csrc/workspace.h) are never shared
with each other or with eager work, and a replay waits on the device for the previous user of its
static buffers (another thread's stream).  An eager micro-batched CLIP tower runs meanwhile on the
shared micro-batch streams.  Every replay equals the eager result of the same input."""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_graphs_replay_concurrently_with_eager_towers():
    from lumen_amd.models.clip import CLIPModel
    from lumen_amd.models.vlm import VLM, VLM_PRESETS

    clip = CLIPModel.random("ViT-B-32", seed=21, dtype=torch.bfloat16, device="cuda")
    vlms = []
    for seed in (4, 5):
        m = VLM(VLM_PRESETS["tiny"], device="cuda")
        m.random_init(seed)
        vlms.append(m)
    g = torch.Generator().manual_seed(22)
    big = torch.randint(0, 256, (384, 224, 224, 3), dtype=torch.uint8, generator=g).cuda()
    v_imgs = [torch.randint(0, 256, (48, 60, 3), dtype=torch.uint8, generator=g).cuda() for _ in range(2)]
    with torch.no_grad():
        big_ref = clip.encode_image_uint8(big).cpu()
        v_refs = [m._encode_tower(m.preprocess(v_imgs), 2).cpu() for m in vlms]

    errors: list = []
    start = threading.Barrier(4)

    def run(fn, ref, n, exact):
        try:
            start.wait(60)
            with torch.no_grad():
                for _ in range(n):
                    out = fn()
                    if exact:
                        assert torch.equal(out, ref)
                    else:
                        assert (out * ref).sum(-1).min().item() > 0.9999
        except BaseException as e:  # noqa: BLE001 - reported by the main thread
            errors.append(e)

    # each thread on a stream of its own; the result is copied to the host on that stream
    def vlm_graph(m):
        def f():
            with torch.cuda.stream(torch.cuda.Stream()):
                return m.encode_images(v_imgs).cpu()
        return f

    def clip_eager_big():        # micro-batched over the shared micro-batch streams
        with torch.cuda.stream(torch.cuda.Stream()):
            return clip.encode_image_uint8(big).cpu()

    ths = [threading.Thread(target=run, args=(vlm_graph(vlms[0]), v_refs[0], 16, True)),
           threading.Thread(target=run, args=(vlm_graph(vlms[0]), v_refs[0], 16, True)),
           threading.Thread(target=run, args=(vlm_graph(vlms[1]), v_refs[1], 16, True)),
           threading.Thread(target=run, args=(clip_eager_big, big_ref, 4, False))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(300)
    torch.cuda.synchronize()
    assert not errors, errors
    for m in vlms:
        assert m._vgraphs and all(v is not False for v in m._vgraphs.values())
    # the two models captured on different private streams
    assert vlms[0]._cap_stream.cuda_stream != vlms[1]._cap_stream.cuda_stream
