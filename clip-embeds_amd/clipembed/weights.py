"""Deterministic synthetic weights and inputs (no network: the `openai` checkpoint cannot be
fetched).

Every tensor is produced by a counter-based generator: element i of tensor `name` is
splitmix64(fnv1a64(f"{seed}:{name}") + i) mapped to a uniform on [-1, 1) and scaled so the
tensor's standard deviation matches the open_clip initialisation scale of that parameter
(transformer.py:558-562 and :925-946; PyTorch defaults for the un-initialised vision tower).
The same function regenerates bit-identical tensors anywhere (this container for the golden
fixtures, the GPU box for the parity tests), so no weight file ever has to travel.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

from .config import ModelConfig

_M64 = (1 << 64) - 1
OPENAI_MEAN = (0.48145466, 0.4578275, 0.40821073)   # open_clip/src/open_clip/constants.py:1
OPENAI_STD = (0.26862954, 0.26130258, 0.27577711)   # constants.py:2
SOT, EOT = 49406, 49407


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & _M64
    return h


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(key: str, n: int) -> np.ndarray:
    """n float32 values uniform on [-1, 1), a pure function of (key, index)."""
    base = np.uint64(_fnv1a64(key))
    out = np.empty(n, dtype=np.float32)
    chunk = 1 << 22
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        with np.errstate(over="ignore"):
            idx = np.arange(s, e, dtype=np.uint64) + base
        z = _splitmix64(idx)
        u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / (1 << 24))
        out[s:e] = u * np.float32(2.0) - np.float32(1.0)
    return out


def _tensor(seed: int, name: str, shape, std: float = None, center: float = 0.0, amp: float = None):
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform(f"{seed}:{name}", n)
    a = amp if amp is not None else std * math.sqrt(3.0)
    return (np.float32(center) + u * np.float32(a)).reshape(shape)


def _block(sd, seed, prefix, D, F, layers):
    proj_std = (D ** -0.5) * ((2 * layers) ** -0.5)
    sd[prefix + "ln_1.weight"] = _tensor(seed, prefix + "ln_1.weight", (D,), center=1.0, amp=0.1)
    sd[prefix + "ln_1.bias"] = _tensor(seed, prefix + "ln_1.bias", (D,), amp=0.05)
    sd[prefix + "attn.in_proj_weight"] = _tensor(seed, prefix + "attn.in_proj_weight", (3 * D, D), std=D ** -0.5)
    sd[prefix + "attn.in_proj_bias"] = _tensor(seed, prefix + "attn.in_proj_bias", (3 * D,), amp=0.02)
    sd[prefix + "attn.out_proj.weight"] = _tensor(seed, prefix + "attn.out_proj.weight", (D, D), std=proj_std)
    sd[prefix + "attn.out_proj.bias"] = _tensor(seed, prefix + "attn.out_proj.bias", (D,), amp=0.02)
    sd[prefix + "ln_2.weight"] = _tensor(seed, prefix + "ln_2.weight", (D,), center=1.0, amp=0.1)
    sd[prefix + "ln_2.bias"] = _tensor(seed, prefix + "ln_2.bias", (D,), amp=0.05)
    sd[prefix + "mlp.c_fc.weight"] = _tensor(seed, prefix + "mlp.c_fc.weight", (F, D), std=(2 * D) ** -0.5)
    sd[prefix + "mlp.c_fc.bias"] = _tensor(seed, prefix + "mlp.c_fc.bias", (F,), amp=0.02)
    sd[prefix + "mlp.c_proj.weight"] = _tensor(seed, prefix + "mlp.c_proj.weight", (D, F), std=proj_std)
    sd[prefix + "mlp.c_proj.bias"] = _tensor(seed, prefix + "mlp.c_proj.bias", (D,), amp=0.02)


def synthetic_state_dict(cfg: ModelConfig, seed: int = 7) -> Dict[str, np.ndarray]:
    """open_clip CLIP state dict (float32 numpy) for `cfg`, keys as CLIP.state_dict()."""
    v, t = cfg.vision, cfg.text
    sd: Dict[str, np.ndarray] = {}
    scale = v.width ** -0.5
    sd["visual.class_embedding"] = _tensor(seed, "visual.class_embedding", (v.width,), std=scale)
    sd["visual.positional_embedding"] = _tensor(seed, "visual.positional_embedding", (v.seq_len, v.width), std=scale)
    sd["visual.proj"] = _tensor(seed, "visual.proj", (v.width, cfg.embed_dim), std=scale)
    fan_in = 3 * v.patch_size * v.patch_size
    sd["visual.conv1.weight"] = _tensor(seed, "visual.conv1.weight", (v.width, 3, v.patch_size, v.patch_size),
                                        amp=fan_in ** -0.5)
    for n in ("ln_pre", "ln_post"):
        sd[f"visual.{n}.weight"] = _tensor(seed, f"visual.{n}.weight", (v.width,), center=1.0, amp=0.1)
        sd[f"visual.{n}.bias"] = _tensor(seed, f"visual.{n}.bias", (v.width,), amp=0.05)
    for i in range(v.layers):
        _block(sd, seed, f"visual.transformer.resblocks.{i}.", v.width, v.mlp_width, v.layers)
    sd["token_embedding.weight"] = _tensor(seed, "token_embedding.weight", (t.vocab_size, t.width), std=0.02)
    sd["positional_embedding"] = _tensor(seed, "positional_embedding", (t.context_length, t.width), std=0.01)
    sd["text_projection"] = _tensor(seed, "text_projection", (t.width, cfg.embed_dim), std=t.width ** -0.5)
    sd["ln_final.weight"] = _tensor(seed, "ln_final.weight", (t.width,), center=1.0, amp=0.1)
    sd["ln_final.bias"] = _tensor(seed, "ln_final.bias", (t.width,), amp=0.05)
    for i in range(t.layers):
        _block(sd, seed, f"transformer.resblocks.{i}.", t.width, t.mlp_width, t.layers)
    sd["logit_scale"] = np.array(math.log(1 / 0.07), dtype=np.float32)
    return sd


def synthetic_pacl_heads(cfg: ModelConfig, seed: int = 11) -> Dict[str, np.ndarray]:
    """open_clip_pacl head weights (pacl.py:70-79), keys as open_clip_pacl.state_dict()."""
    Dv, E, Pd = cfg.vision.width, cfg.embed_dim, cfg.pacl_dim or 768
    sd: Dict[str, np.ndarray] = {}

    def lin(name, out_f, in_f):
        sd[name + ".weight"] = _tensor(seed, name + ".weight", (out_f, in_f), amp=in_f ** -0.5)
        sd[name + ".bias"] = _tensor(seed, name + ".bias", (out_f,), amp=in_f ** -0.5)

    sd["visual_projection.0.weight"] = _tensor(seed, "visual_projection.0.weight", (Dv,), center=1.0, amp=0.1)
    sd["visual_projection.0.bias"] = _tensor(seed, "visual_projection.0.bias", (Dv,), amp=0.05)
    lin("visual_projection.2.linear_projection.0", Pd, Dv)
    lin("visual_projection.2.non_linear_projection.0", Pd, Dv)
    lin("visual_projection.2.non_linear_projection.2", Pd, Pd)
    sd["text_projection.0.weight"] = _tensor(seed, "text_projection.0.weight", (E,), center=1.0, amp=0.1)
    sd["text_projection.0.bias"] = _tensor(seed, "text_projection.0.bias", (E,), amp=0.05)
    lin("text_projection.2", Pd, E)
    # Patch_Projection registers one Sequential under two names (pacl.py:39): state_dict has both
    sd["visual_projection.2.text_projection.0.weight"] = sd["visual_projection.2.linear_projection.0.weight"]
    sd["visual_projection.2.text_projection.0.bias"] = sd["visual_projection.2.linear_projection.0.bias"]
    return sd


def synthetic_images_u8(n: int, size: int = 336, seed: int = 1000) -> np.ndarray:
    """uint8 [n, size, size, 3] uniform on [0, 255]."""
    u = uniform(f"images:{seed}", n * size * size * 3)
    return np.clip(np.floor((u + 1.0) * 128.0), 0, 255).astype(np.uint8).reshape(n, size, size, 3)


def normalize_images(u8: np.ndarray, mean=OPENAI_MEAN, std=OPENAI_STD) -> np.ndarray:
    """uint8 NHWC -> float32 NCHW, (x/255 - mean)/std (open_clip transform Normalize)."""
    x = u8.astype(np.float32) / np.float32(255.0)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2))


def synthetic_images(n: int, size: int = 336, seed: int = 1000) -> np.ndarray:
    return normalize_images(synthetic_images_u8(n, size, seed))


def synthetic_captions(n: int, ctx: int = 77, seed: int = 2000, min_len: int = 5, max_len: int = 40) -> np.ndarray:
    """int64 [n, ctx]: SOT, n~U[min_len,max_len] ids in [1, 49405], EOT, zero padding."""
    u = uniform(f"captions:{seed}", n * (ctx + 1))
    u01 = (u + 1.0) * 0.5
    out = np.zeros((n, ctx), dtype=np.int64)
    for i in range(n):
        row = u01[i * (ctx + 1):(i + 1) * (ctx + 1)]
        ln = min_len + int(row[0] * (max_len - min_len + 1))
        ln = min(ln, ctx - 2)
        ids = 1 + np.floor(row[1:1 + ln] * 49405).astype(np.int64)
        out[i, 0] = SOT
        out[i, 1:1 + ln] = np.clip(ids, 1, 49405)
        out[i, 1 + ln] = EOT
    return out
