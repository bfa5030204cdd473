"""Experiment: the clip bench step with the image batch split over two engine instances on two HIP
streams (+ the text tower on a third), vs the bench's default (text on a side stream)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO]
import torch  # noqa: E402

import clipembed  # noqa: E402
from clipembed import _lib, weights as W  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = clipembed.get_model_config("ViT-L-14-336")
    sd = W.synthetic_state_dict(cfg)
    B = 256
    models = []
    for _ in range(2):
        m = clipembed.CLIP(cfg)
        m.load_state_dict(sd)
        m.to(dev)
        _lib.call("ce_reserve", m.engine.h, B, B)
        models.append(m)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000)).to(dev)
    caps = torch.from_numpy(W.synthetic_captions(B, seed=2000)).to(dev)
    scale = float(models[0].logit_scale.detach().exp())
    s1, s2, s3 = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def step_base():
        main = torch.cuda.current_stream(dev)
        s1.wait_stream(main)
        with torch.cuda.stream(s1):
            ft = models[0].encode_text(caps, normalize=True)
        fi = models[0].encode_image(imgs, normalize=True)
        main.wait_stream(s1)
        return models[0].logits(fi, ft, scale)

    def step_split(nsplit):
        main = torch.cuda.current_stream(dev)
        for st in (s1, s2, s3):
            st.wait_stream(main)
        with torch.cuda.stream(s3):
            ft = models[0].encode_text(caps, normalize=True)
        h = B // nsplit
        parts = []
        with torch.cuda.stream(s1):
            parts.append(models[0].encode_image(imgs[:h], normalize=True))
        with torch.cuda.stream(s2):
            parts.append(models[1].encode_image(imgs[h:], normalize=True))
        for st in (s1, s2, s3):
            main.wait_stream(st)
        fi = torch.cat(parts)
        return models[0].logits(fi, ft, scale)

    def bench(fn, steps=10, warm=3):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        return B * steps / (time.perf_counter() - t)

    ref = step_base()[0]
    out = step_split(2)[0]
    torch.cuda.synchronize()
    print("max |logits diff|", (ref - out).abs().max().item(), flush=True)
    for r in range(3):
        print(f"round {r}: base {bench(step_base):.1f}  split2 {bench(lambda: step_split(2)):.1f} pairs/s", flush=True)


if __name__ == "__main__":
    main()
