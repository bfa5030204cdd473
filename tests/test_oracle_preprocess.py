"""Preprocessing oracle (oracle/preprocess_oracle.py) pinned to the committed fixtures made from
Pillow / torch (tests/golden/make_golden_preprocess.py), and directly to Pillow when importable."""
import hashlib
import importlib.util
import os

import numpy as np
import pytest

from oracle import preprocess_oracle as P

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location("mgp", os.path.join(HERE, "golden", "make_golden_preprocess.py"))
mgp = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mgp)


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(HERE, "golden", "preprocess.npz"))


@pytest.mark.parametrize("i", range(8))
def test_clip_bicubic_bit_exact(gold, i):
    h, w = (int(v) for v in gold["sizes"][i])
    img = mgp.image(i, h, w)
    nh, nw = P.shortest_edge_size(h, w, 336)
    r = img if (nh, nw) == (h, w) else P.pil_resize_bicubic(img, nw, nh)
    top, left = P.center_crop_offsets(nh, nw, 336)
    crop = np.ascontiguousarray(r[top:top + 336, left:left + 336])
    assert hashlib.sha256(crop.tobytes()).digest() == gold[f"clip_sha_{i}"].tobytes()
    out = P.clip_eval_preprocess(img)
    assert np.array_equal(out[:, ::11, ::11], gold[f"clip_sub_{i}"])     # ToTensor/Normalize bit-exact


@pytest.mark.parametrize("i", range(8))
def test_pacl_bilinear_aa(gold, i):
    h, w = (int(v) for v in gold["sizes"][i])
    out = P.pacl_eval_preprocess(mgp.image(i, h, w))
    np.testing.assert_allclose(out[:, ::11, ::11], gold[f"pacl_sub_{i}"], atol=2e-6, rtol=0)


def test_against_pillow_directly():
    Image = pytest.importorskip("PIL.Image")
    rng = np.random.default_rng(5)
    for h, w in [(123, 457), (800, 333)]:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        for ow, oh in [(336, 336), (97, 401), (1000, 50)]:
            ref = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BICUBIC))
            assert np.array_equal(P.pil_resize_bicubic(img, ow, oh), ref)
