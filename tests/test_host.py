"""Host-side logic: deterministic generator, config registry, state-dict naming vs the
reference's key layout (tests/golden/meta.npz), caption format."""
import json

import numpy as np
import pytest

import clipembed
from clipembed import weights as W
from clipembed.config import get_model_config


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
