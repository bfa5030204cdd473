"""Diagnostic: pooled (packed-row) encode_text vs the oracle for two captions with given EOT positions,
text depth 2 (round 4: the second caption of a 2-caption batch came out wrong)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO]
import clipembed  # noqa: E402
from clipembed import _lib, weights as W  # noqa: E402
from clipembed.config import get_model_config  # noqa: E402
from oracle import clip_oracle as O  # noqa: E402


def cosd(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return (1 - (a * b).sum(-1) / np.linalg.norm(a, axis=-1) / np.linalg.norm(b, axis=-1)).round(6).tolist()


cfg = get_model_config("ViT-L-14-336").with_depth(1, int(os.environ.get("TL", "2")))
sd = W.synthetic_state_dict(cfg)
m = clipembed.CLIP(cfg); m.load_state_dict(sd); m.to("cuda")
rng = np.random.default_rng(5)
L = _lib.lib()
for spec in sys.argv[1:]:
    eots = [int(x) for x in spec.split(",")]
    caps = np.zeros((len(eots), 77), np.int64)
    for i, e in enumerate(eots):
        caps[i, 0] = 49406
        caps[i, 1:e] = rng.integers(1, 49000, e - 1)
        caps[i, e] = 49407
    ref = O.encode_text(sd, caps, cfg)
    out = {}
    for tag, fn in (("default", None), ("no_onetile", lambda: L.ce_set_gemm_variant(8579 & ~8192)),
                    ("attn0", lambda: L.ce_set_attn_variant(0))):
        pg, pa = L.ce_set_gemm_variant(-1), L.ce_set_attn_variant(125)
        L.ce_set_gemm_variant(-1)
        if fn:
            fn()
        r = [cosd(m.encode_text(torch.from_numpy(caps)).cpu().numpy(), ref) for _ in range(2)]
        L.ce_set_gemm_variant(-1); L.ce_set_attn_variant(125)
        out[tag] = r
    print(f"EOTs {eots}: " + "  ".join(f"{k} {v}" for k, v in out.items()), flush=True)
