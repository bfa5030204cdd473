"""Pins oracle/text_train_torch.py (the f32 autograd restatement of the NegCLIP text-tower step the
C4 GPU test compares against at full size) to the reference's own training step
(tests/golden/train.npz, make_golden_train.py: open_clip CLIP + ClipLoss(local_loss,
gather_with_grad, usehardtext) autograd, 1 vision + 2 text blocks, 4 images, 6 captions).
CPU only."""
import math

import numpy as np
import torch

from clipembed import weights as W
from clipembed.config import get_model_config
from oracle.clip_torch_cpu import TorchCLIP
from oracle.text_train_torch import TorchTextTrainStep


def test_text_train_restatement_matches_reference(golden):
    g = golden("train")
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 2)
    sd = W.synthetic_state_dict(cfg)
    torch.manual_seed(0)
    img = TorchCLIP(sd, cfg).encode_image(torch.from_numpy(W.synthetic_images(4, seed=int(g["images_seed"]))),
                                          normalize=True)
    step = TorchTextTrainStep(sd, cfg)
    loss, grads = step.loss_and_grads(img, g["captions"], math.log(1 / 0.07))
    np.testing.assert_allclose(loss, g["losses"][0], rtol=1e-5)
    for n, gv in grads.items():
        if n == "logit_scale":
            continue
        idx = g[f"gidx:{n}"]
        ours = gv.reshape(-1)[torch.from_numpy(idx)].numpy()
        ref = g[f"grad:{n}"]
        scale = np.abs(ref).max() + 1e-30
        assert np.abs(ours - ref).max() <= 1e-4 * scale, n
        np.testing.assert_allclose(float(gv.double().norm()), float(g[f"gnorm:{n}"]), rtol=1e-4, err_msg=n)


def test_sparc_train_restatement_matches_reference(golden):
    """Pins oracle/sparc_train_torch.py (the f32 autograd restatement of the SPARC head step the GPU tests
    compare the engine against at larger batches) to the reference's own train_sparc.py step
    (tests/golden/sparc_train.npz, make_golden_sparc.py train: sparc_rope(1/576) on 1-block towers,
    SparcLoss(0.1), loss.backward(), dropout off): loss and every head gradient."""
    import hashlib
    from oracle.sparc_train_torch import HEAD_TENSORS, SparcTokens, TorchSparcTrainStep, rope_tokens
    g = golden("sparc_train")
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    imgs = W.synthetic_images(3, seed=1400)
    assert hashlib.sha256(np.ascontiguousarray(imgs).tobytes()).hexdigest() == str(g["images_sha"])
    tok = SparcTokens(W.synthetic_state_dict(cfg), cfg)
    caps = g["captions"]
    pv = rope_tokens(tok.image_tokens(torch.from_numpy(imgs)))
    tt = tok.text_tokens(torch.from_numpy(caps))
    mask = (np.arange(caps.shape[1])[None, :] <= caps.argmax(-1)[:, None]).astype(np.float32)
    np.testing.assert_array_equal(mask, g["mask"])
    step = TorchSparcTrainStep(W.synthetic_pacl_heads(cfg.with_pacl(768)))
    loss, grads, _ = step.loss_and_grads(pv, mask, text_tokens=tt)
    np.testing.assert_allclose(loss, g["loss"], rtol=1e-5)
    rows = [0, 1, 383, 767]
    for n in HEAD_TENSORS:
        gv = grads[n].numpy()
        ref = g[f"grad/{n}"]
        ours = gv if gv.ndim == 1 else gv[rows]
        assert np.abs(ours - ref).max() <= 1e-4 * (np.abs(ref).max() + 1e-30), n
        np.testing.assert_allclose(np.linalg.norm(gv.astype(np.float64)), g[f"grad_norm/{n}"], rtol=1e-4, err_msg=n)


def test_pacl_train_restatement_matches_reference(golden):
    """Pins the PACL step of oracle/sparc_train_torch.py (pacl_loss_and_grads) to the reference's own
    train_pacl.py step (tests/golden/pacl_train.npz, make_golden_sparc.py train_pacl: open_clip_pacl and
    open_clip_pacl_rope on 1-block towers, ClipLoss(0.1), loss.backward(), dropout off)."""
    import hashlib
    from oracle.sparc_train_torch import HEAD_TENSORS, SparcTokens, TorchSparcTrainStep, rope_tokens
    g = golden("pacl_train")
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    imgs = W.synthetic_images(3, seed=1450)
    assert hashlib.sha256(np.ascontiguousarray(imgs).tobytes()).hexdigest() == str(g["images_sha"])
    sd = W.synthetic_state_dict(cfg)
    tok = SparcTokens(sd, cfg)
    caps = g["captions"]
    pt = tok.image_tokens(torch.from_numpy(imgs))
    tt = tok.text_tokens(torch.from_numpy(caps))
    pooled = tt[torch.arange(3), torch.from_numpy(caps).argmax(-1)] @ torch.as_tensor(sd["text_projection"]).float()
    rows = [0, 1, 383, 767]
    for tag, pv in (("pacl", pt), ("pacl_rope", rope_tokens(pt))):
        step = TorchSparcTrainStep(W.synthetic_pacl_heads(cfg.with_pacl(768)))
        loss, grads = step.pacl_loss_and_grads(pv, pooled, p=0.0)
        np.testing.assert_allclose(loss, g[f"{tag}/loss"], rtol=1e-5, err_msg=tag)
        for n in HEAD_TENSORS:
            gv = grads[n].numpy()
            ref = g[f"{tag}/grad/{n}"]
            ours = gv if gv.ndim == 1 else gv[rows]
            assert np.abs(ours - ref).max() <= 1e-4 * (np.abs(ref).max() + 1e-30), (tag, n)
            np.testing.assert_allclose(np.linalg.norm(gv.astype(np.float64)), g[f"{tag}/grad_norm/{n}"], rtol=1e-4,
                                       err_msg=f"{tag} {n}")
