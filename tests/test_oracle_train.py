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
