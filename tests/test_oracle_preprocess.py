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


def test_train_crop_against_pillow_directly():
    """clip_train_preprocess = Pillow crop + BICUBIC resize to 336 (torchvision F.resized_crop on a PIL
    image) + ToTensor/Normalize, for boxes drawn by clipembed's RandomResizedCrop parameter sampler."""
    Image = pytest.importorskip("PIL.Image")
    import torch
    from clipembed.transforms import random_resized_crop_params
    g = torch.Generator().manual_seed(3)
    for i, (h, w) in enumerate([(480, 640), (336, 336), (200, 150)]):
        img = mgp.image(i, h, w)
        box = random_resized_crop_params(h, w, generator=g)
        top, left, bh, bw = box
        assert 0 <= top and top + bh <= h and 0 <= left and left + bw <= w
        assert 0.9 * h * w * 0.95 <= bh * bw <= h * w          # scale (0.9, 1.0) up to rounding
        ref = np.asarray(Image.fromarray(img).crop((left, top, left + bw, top + bh)).resize((336, 336), Image.BICUBIC))
        x = ref.transpose(2, 0, 1).astype(np.float32) / np.float32(255)
        m = np.asarray(P.OPENAI_MEAN, np.float32)[:, None, None]
        s = np.asarray(P.OPENAI_STD, np.float32)[:, None, None]
        assert np.array_equal(P.clip_train_preprocess(img, box), ((x - m) / s).astype(np.float32))


def test_random_resized_crop_params_rng_stream():
    """Same torch RNG draws as torchvision's RandomResizedCrop.get_params: two uniform_ draws per
    attempt then two randint draws; the fallback (10 rejected attempts) is a central crop."""
    import math
    import torch
    from clipembed.transforms import random_resized_crop_params
    torch.manual_seed(11)
    box = random_resized_crop_params(480, 640)
    torch.manual_seed(11)
    ta = 480 * 640 * torch.empty(1).uniform_(0.9, 1.0).item()
    lr = torch.log(torch.tensor((3 / 4, 4 / 3)))
    ar = torch.exp(torch.empty(1).uniform_(lr[0], lr[1])).item()
    w, h = int(round(math.sqrt(ta * ar))), int(round(math.sqrt(ta / ar)))
    if 0 < w <= 640 and 0 < h <= 480:
        i = torch.randint(0, 480 - h + 1, size=(1,)).item()
        j = torch.randint(0, 640 - w + 1, size=(1,)).item()
        assert box == (i, j, h, w)
    # a 1 x 2000 strip can never host a crop of area >= 0.9 with ratio <= 4/3: central fallback
    assert random_resized_crop_params(1, 2000) == (0, 999, 1, 1)        # h = 1, w = round(1 * 4/3)
