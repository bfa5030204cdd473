"""TEXT-TOWER TRAINING RESTATEMENT (f32 torch autograd) — test infrastructure only.

The gradient the reference computes for one NegCLIP step of the text tower with a locked image
tower (open_clip_train/train.py:85-112 as launched by train-clip.sh: --lock-image --local-loss
--gather-with-grad --usehardtext), restated with the reference's own ATen calls and autograd on
one rank:
  text forward     CLIP.encode_text (model.py:283-301): token_embedding gather + positional
                   embedding, 12 x ResidualAttentionBlock (transformer.py:257-268; causal mask
                   transformer.py:960-966), ln_final, EOT row (argmax of ids), @ text_projection,
                   F.normalize  (the block itself is oracle/clip_torch_cpu.TorchCLIP._block)
  loss             ClipLoss.get_logits / forward (loss.py:137-193) on one rank: logits_per_image =
                   s I T^T, logits_per_text = s T I^T, labels arange(B) for images and
                   [arange(B), -100 x K] for texts (get_mixed_ground_truth :127-135),
                   (CE_i + CE_t) / 2 with F.cross_entropy's ignore_index -100
  scale            logit_scale.exp() (model.py:435): the gradient is taken w.r.t. logit_scale
It runs on whatever device its tensors live on (the CPU pin against tests/golden/train.npz, the GPU
box at the C4 size).  Imported only by tests/; the product never imports it.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .clip_torch_cpu import TorchCLIP


def text_param_names(cfg):
    """The trainable text-tower tensors (the names clipembed.train.text_tensor_names binds)."""
    names = ["token_embedding.weight", "positional_embedding", "ln_final.weight", "ln_final.bias", "text_projection"]
    for l in range(cfg.text.layers):
        for n in ("ln_1.weight", "ln_1.bias", "attn.in_proj_weight", "attn.in_proj_bias", "attn.out_proj.weight",
                  "attn.out_proj.bias", "ln_2.weight", "ln_2.bias", "mlp.c_fc.weight", "mlp.c_fc.bias",
                  "mlp.c_proj.weight", "mlp.c_proj.bias"):
            names.append(f"transformer.resblocks.{l}.{n}")
    return names


class TorchTextTrainStep(TorchCLIP):
    """Text-tower weights as f32 leaf tensors (requires_grad) on `device`."""

    def __init__(self, sd, cfg, device="cpu"):
        names = text_param_names(cfg)
        sub = {n: sd[n] for n in names}
        super().__init__(sub, cfg)
        self.w = {n: v.to(device).requires_grad_(True) for n, v in self.w.items()}
        self.device = torch.device(device)

    def text_features(self, ids):
        t, w = self.cfg.text, self.w
        ids = torch.as_tensor(ids).long().to(self.device)
        L = ids.shape[1]
        x = w["token_embedding.weight"][ids] + w["positional_embedding"]
        mask = torch.full((L, L), float("-inf"), device=self.device).triu_(1)
        for i in range(t.layers):
            x = self._block(x, f"transformer.resblocks.{i}.", t.heads, mask)
        x = F.layer_norm(x, (t.width,), w["ln_final.weight"], w["ln_final.bias"], 1e-5)
        pooled = x[torch.arange(x.shape[0], device=self.device), ids.argmax(dim=-1)] @ w["text_projection"]
        return F.normalize(pooled, dim=-1)

    def loss_and_grads(self, image_features, ids, logit_scale: float):
        """One step's loss and d loss / d (every text tensor, logit_scale): a dict of f32 tensors on
        the step's device ('logit_scale' included), and the loss as a float."""
        for v in self.w.values():
            v.grad = None
        ls = torch.tensor(float(logit_scale), device=self.device, dtype=torch.float32, requires_grad=True)
        img = torch.as_tensor(image_features).float().to(self.device).clone()   # (may be an inference tensor)
        txt = self.text_features(ids)
        s = ls.exp()
        B, T = img.shape[0], txt.shape[0]
        li = torch.arange(B, device=self.device, dtype=torch.long)
        lt = torch.cat([li, torch.full((T - B,), -100, device=self.device, dtype=torch.long)])
        loss = (F.cross_entropy(s * img @ txt.T, li) + F.cross_entropy(s * txt @ img.T, lt)) / 2
        loss.backward()
        grads: Dict[str, torch.Tensor] = {n: v.grad.detach() for n, v in self.w.items()}
        grads["logit_scale"] = ls.grad.detach().reshape(1)
        return float(loss.detach()), grads
