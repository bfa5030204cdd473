"""Device preprocessing (ce_preprocess_images) vs the pinned oracle: the CLIP bicubic path must be
bit-exact (integer Pillow arithmetic + IEEE f32 ToTensor/Normalize), the PACL antialiased
bilinear path within 2e-6 (f32 multiply-add order)."""
import importlib.util
import os

import numpy as np
import pytest
import torch

from oracle import preprocess_oracle as P

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location("mgp", os.path.join(HERE, "golden", "make_golden_preprocess.py"))
mgp = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mgp)


@pytest.fixture(scope="module")
def gold():
    return np.load(os.path.join(HERE, "golden", "preprocess.npz"))


@pytest.fixture(scope="module")
def images(gold):
    return [mgp.image(i, int(h), int(w)) for i, (h, w) in enumerate(gold["sizes"])]


def test_clip_bicubic_batch_bit_exact(images, gold):
    from clipembed import image_transform
    out = image_transform(336)(images).cpu().numpy()          # one launch, mixed sizes
    for i, img in enumerate(images):
        ref = P.clip_eval_preprocess(img)
        assert np.array_equal(out[i], ref), f"image {i} {img.shape}: max |d| {np.abs(out[i] - ref).max()}"
        assert np.array_equal(out[i][:, ::11, ::11], gold[f"clip_sub_{i}"])


def test_pacl_bilinear_aa_batch(images, gold):
    from clipembed import prepare_data
    out = prepare_data("ViT-L-14-336").preprocess_image(images).cpu().numpy()
    for i, img in enumerate(images):
        np.testing.assert_allclose(out[i], P.pacl_eval_preprocess(img), atol=2e-6, rtol=0)
        np.testing.assert_allclose(out[i][:, ::11, ::11], gold[f"pacl_sub_{i}"], atol=2e-6, rtol=0)


def test_single_image_pil_and_bf16(images):
    from PIL import Image
    from clipembed import _lib
    from clipembed.transforms import DeviceImageProcessor
    one = image = images[0]
    y = DeviceImageProcessor(_lib.CE_PRE_CLIP_BICUBIC)(Image.fromarray(one))
    assert tuple(y.shape) == (3, 336, 336)
    ref = torch.from_numpy(P.clip_eval_preprocess(image))
    assert torch.equal(y.cpu(), ref)
    yb = DeviceImageProcessor(_lib.CE_PRE_CLIP_BICUBIC, out_dtype=torch.bfloat16)([one])
    assert torch.equal(yb[0].cpu(), ref.to(torch.bfloat16))


def test_preprocess_feeds_encoder(images):
    """Preprocessed batch straight into encode_image (no host round trip)."""
    import clipembed
    from clipembed import weights as W
    cfg = clipembed.get_model_config("ViT-L-14-336").with_depth(1, 1)
    model = clipembed.CLIP(cfg)
    model.load_state_dict(W.synthetic_state_dict(cfg))
    model.to("cuda")
    _, _, val = clipembed.create_model_and_transforms("ViT-L-14-336")
    f = model.encode_image(val(images[:3]), normalize=True)
    assert f.shape == (3, 768) and torch.isfinite(f).all()


def test_errors():
    from clipembed import ClipEmbedError, _lib
    from clipembed.model import kernel_engine, _ptr, _stream
    e = kernel_engine("cuda")
    buf = torch.zeros(16, dtype=torch.uint8, device="cuda")
    out = torch.empty(1, 3, 336, 336, device="cuda")
    off = np.zeros(1, np.int64)
    hw = np.array([0], np.int32)
    with pytest.raises(ClipEmbedError, match="bad size"):
        _lib.call("ce_preprocess_images", e.h, _stream(e.device), _ptr(buf), off.ctypes.data, hw.ctypes.data,
                  hw.ctypes.data, 1, 0, _lib.CE_F32, _ptr(out))
    one = np.array([4], np.int32)
    with pytest.raises(ClipEmbedError, match="unknown mode"):
        _lib.call("ce_preprocess_images", e.h, _stream(e.device), _ptr(buf), off.ctypes.data, one.ctypes.data,
                  one.ctypes.data, 1, 7, _lib.CE_F32, _ptr(out))


def test_clip_train_crop_bit_exact(images):
    """create_model_and_transforms(...)[1] (eval_clip.py:21-24 feeds it to prepare_data_clip): the
    RandomResizedCrop box from the host torch RNG, the bicubic resample on the device — bit-exact
    against the Pillow-pinned oracle for the same boxes (same seed)."""
    import clipembed
    from clipembed.transforms import DeviceTrainProcessor, random_resized_crop_params
    _, train, val = clipembed.create_model_and_transforms("ViT-L-14-336")
    assert isinstance(train, DeviceTrainProcessor) and not isinstance(val, DeviceTrainProcessor)
    torch.manual_seed(77)
    out = train(images).cpu().numpy()                 # one launch, boxes drawn per image in order
    torch.manual_seed(77)
    for i, img in enumerate(images):
        box = random_resized_crop_params(img.shape[0], img.shape[1])
        ref = P.clip_train_preprocess(img, box)
        assert np.array_equal(out[i], ref), f"image {i} box {box}: max |d| {np.abs(out[i] - ref).max()}"
    from clipembed import ClipEmbedError, _lib
    from clipembed.model import kernel_engine, _ptr, _stream
    e = kernel_engine("cuda")
    buf = torch.zeros(48, dtype=torch.uint8, device="cuda")
    o = torch.empty(1, 3, 336, 336, device="cuda")
    off = np.zeros(1, np.int64)
    hw = np.array([4], np.int32)
    bad = np.array([[0, 2, 4, 3]], np.int32)        # left + width > 4
    with pytest.raises(ClipEmbedError, match="outside"):
        _lib.call("ce_preprocess_images_boxes", e.h, _stream(e.device), _ptr(buf), off.ctypes.data, hw.ctypes.data,
                  hw.ctypes.data, bad.ctypes.data, 1, _lib.CE_F32, _ptr(o))
