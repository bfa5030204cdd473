"""Host-side logic: deterministic generator, config registry, state-dict naming vs the
reference's key layout (tests/golden/meta.npz), caption format."""
import os
import json

import numpy as np
import pytest

import clipembed
from clipembed import weights as W
from clipembed.config import get_model_config

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_generator_is_pure_and_scaled():
    a = W.uniform("k", 1000)
    b = W.uniform("k", 1000)
    assert np.array_equal(a, b)
    assert np.array_equal(W.uniform("k", 10), a[:10])
    assert a.min() >= -1 and a.max() < 1 and abs(a.mean()) < 0.1
    assert not np.array_equal(W.uniform("k2", 10), a[:10])


def test_state_dict_keys_match_reference(golden):
    meta = json.loads(str(golden("meta")["json"]))
    ref = meta["clip_state_dict_keys"]
    sd = W.synthetic_state_dict(get_model_config("ViT-L-14-336").with_depth(1, 1))
    assert set(sd) == set(ref)
    for k, shape in ref.items():
        assert list(sd[k].shape) == shape, k
    heads = W.synthetic_pacl_heads(get_model_config("ViT-L-14-336").with_pacl(768))
    assert set(heads) == set(meta["pacl_state_dict_keys"])
    for k, shape in meta["pacl_state_dict_keys"].items():
        assert list(heads[k].shape) == shape, k


def test_captions_format():
    c = W.synthetic_captions(16, seed=3)
    assert c.shape == (16, 77) and c.dtype == np.int64
    for row in c:
        eot = int(np.argmax(row))
        assert row[0] == W.SOT and row[eot] == W.EOT
        assert (row[1:eot] >= 1).all() and (row[1:eot] <= 49405).all() and (row[eot + 1:] == 0).all()


def test_images_normalised():
    x = W.synthetic_images(1, seed=9)
    assert x.shape == (1, 3, 336, 336) and x.dtype == np.float32
    assert -2.0 < x.min() < -1.5 and 2.0 < x.max() < 2.3


def test_registry_geometry():
    cfg = get_model_config("ViT-L-14-336")
    assert (cfg.vision.width, cfg.vision.layers, cfg.vision.heads, cfg.vision.seq_len) == (1024, 24, 16, 577)
    assert (cfg.text.width, cfg.text.layers, cfg.text.heads) == (768, 12, 12)
    assert get_model_config("ViT-L-14-336-quickgelu").quick_gelu
    with pytest.raises(RuntimeError):
        get_model_config("RN50")
    assert cfg.with_depth(2, 1).vision.layers == 2


def test_encoders_refuse_without_device():
    m = clipembed.CLIP(get_model_config("ViT-L-14-336").with_depth(1, 1))
    with pytest.raises(RuntimeError, match="HIP device"):
        m.encode_image(np.zeros((1, 3, 336, 336), np.float32))


def test_gelu_polynomial_error_bound():
    """The GEMM epilogue's packed GELU (csrc/ce_device.h gelu_pair) evaluated in f32 exactly as the
    device does (clamp, t = 0.08 u^2 - 1, Horner, fma(u, p, 0.5), x * phi): error <= 2.5e-6 * max(1, |y|) vs
    the exact-erf GELU of nn.GELU (transformer.py:235-239) over all x."""
    import re
    from scipy.special import erf
    src = open(os.path.join(REPO, "clip-embeds_amd", "csrc", "ce_device.h")).read()
    body = src[src.index("f32x2 gelu_pair"):]
    body = body[:body.index("return x * phi")]
    coefs = [np.float32(re.search(r"p = \(f32x2\)\((-?[0-9.e+-]+)f\)", body).group(1))]
    coefs += [np.float32(c) for c in re.findall(r"fma\(p, t, \(f32x2\)\((-?[0-9.e+-]+)f\)\)", body)]
    assert len(coefs) == 13
    x = np.linspace(-12, 12, 200001).astype(np.float32)
    u = np.clip(x, np.float32(-5), np.float32(5))
    t = (u * u * np.float32(0.08) - np.float32(1)).astype(np.float32)
    p = coefs[0]
    for c in coefs[1:]:
        p = (p * t + c).astype(np.float32)
    g = (x * (u * p + np.float32(0.5))).astype(np.float32)
    ref = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    assert (np.abs(g - ref) / np.maximum(1.0, np.abs(ref))).max() <= 2.5e-6


def test_gelu_sigmoid_error_bound():
    """The four-wave GEMM epilogue's GELU (csrc/ce_device.h gelu_fast4: x / (1 + 2^(u P(u^2))),
    u = clamp(x, +-X), degree-2 P) evaluated in f32 as the device does: error <= 6.5e-5 * max(1, |y|)
    vs the exact-erf GELU of nn.GELU (transformer.py:235-239) over all x (v_exp_f32 / v_rcp_f32
    modelled as correctly rounded; their 1-ulp error is far inside the bound)."""
    import re
    from scipy.special import erf
    src = open(os.path.join(REPO, "clip-embeds_amd", "csrc", "ce_device.h")).read()
    k = {n: np.float32(float(v)) for n, v in re.findall(r"#define CE_GELU_(\w+) (-?[0-9.e+-]+)f", src)}
    x = np.linspace(-20, 20, 400001).astype(np.float32)
    u = np.clip(x, -k["CLAMP"], k["CLAMP"]).astype(np.float32)
    u2 = (u * u).astype(np.float32)
    p = (u2 * k["C2"] + k["C1"]).astype(np.float32)
    p = (p * u2 + k["C0"]).astype(np.float32)
    with np.errstate(over="ignore"):
        e = np.exp2((u * p).astype(np.float64)).astype(np.float32)
    r = (1.0 / (np.float32(1) + e).astype(np.float64)).astype(np.float32)
    g = (x * r).astype(np.float32)
    ref = 0.5 * x.astype(np.float64) * (1 + erf(x.astype(np.float64) / np.sqrt(2)))
    assert (np.abs(g - ref) / np.maximum(1.0, np.abs(ref))).max() <= 6.5e-5


def test_train_transform_ignores_ratio_like_reference():
    """open_clip's non-timm train transform passes only `scale` to RandomResizedCrop and warns
    about any other aug_cfg item (transform.py:334-357): a `ratio` leaves the default (3/4, 4/3)."""
    from clipembed.transforms import DeviceTrainProcessor, image_transform
    with pytest.warns(UserWarning, match="Unused augmentation cfg items"):
        t = image_transform(336, is_train=True, aug_cfg={"scale": (0.5, 1.0), "ratio": (0.5, 2.0)})
    assert isinstance(t, DeviceTrainProcessor)
    assert t.scale == (0.5, 1.0) and t.ratio == (3.0 / 4.0, 4.0 / 3.0)
    with pytest.raises(NotImplementedError):
        image_transform(336, is_train=True, aug_cfg={"color_jitter_prob": 0.5})
    with pytest.raises(NotImplementedError):
        image_transform(336, is_train=True, aug_cfg={"use_timm": True})
