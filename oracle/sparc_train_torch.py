"""SPARC HEAD TRAINING RESTATEMENT (f32 torch autograd) — test infrastructure only.

One step of Patch-Aligned-Contrastive-Learning/train_sparc.py (train_sparc.py:29-37: forward,
SparcLoss, loss.backward(); the Adam update is torch.optim.Adam's, train_sparc.py:106) restated with
the reference's own ATen calls and autograd, for the trainable SPARC heads on a frozen CLIP:
  visual head      sparc_rope.forward_visual (pacl.py:480-484): apply_rope on the ln_post'd patch
                   tokens, then visual_projection = LayerNorm(1024) -> Dropout(0.1) ->
                   Patch_Projection(1024, 768) (pacl.py:35-48, 397-401): lin(x) + Linear(GELU(Linear(x)))
  text head        sparc.forward_text (pacl.py:431-436): text_projection = LayerNorm(768) ->
                   Dropout(0.1) -> Linear(768, 768) on every ln_final'd token, mask = arange <= EOT
  alignment        sparc.forward (pacl.py:453-478): S = l v^T, min-max over patches, zero below sigma,
                   row-normalised weights, grouped = W v, both L2-normalised
  loss             SparcLoss(temperature) (pacl.py:516-584): 0.5 * CLIP loss of the normalised patch /
                   token means + 1.0 * the mean of the two masked pairwise local losses
Dropout: the reference's model.train() draws torch RNG masks; here the keep-masks are arguments
(None = dropout off, the module in eval mode), so a test can hand in the engine's own masks.
The frozen towers' tokens come in as inputs (SparcTokens below restates them from the CLIP forward).
PACL: pacl_loss_and_grads restates one train_pacl.py step (open_clip_pacl / _rope heads, ClipLoss).
Imported only by tests/; the product never imports it.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from .clip_oracle import apply_rope
from .clip_torch_cpu import TorchCLIP

HEAD_TENSORS = ["visual_projection.0.weight", "visual_projection.0.bias",
                "visual_projection.2.linear_projection.0.weight", "visual_projection.2.linear_projection.0.bias",
                "visual_projection.2.non_linear_projection.0.weight", "visual_projection.2.non_linear_projection.0.bias",
                "visual_projection.2.non_linear_projection.2.weight", "visual_projection.2.non_linear_projection.2.bias",
                "text_projection.0.weight", "text_projection.0.bias", "text_projection.2.weight", "text_projection.2.bias"]


class SparcTokens(TorchCLIP):
    """The frozen towers' token outputs (visual.output_tokens / output_text_tokens, transformer.py:718-741,
    839-855): ln_post of the patch rows, ln_final of every text row."""

    @torch.inference_mode()
    def image_tokens(self, pixels):
        v, w = self.cfg.vision, self.w
        x = F.conv2d(torch.as_tensor(pixels).float(), w["visual.conv1.weight"], stride=v.patch_size)
        x = x.reshape(x.shape[0], x.shape[1], -1).permute(0, 2, 1)
        x = torch.cat([w["visual.class_embedding"].expand(x.shape[0], 1, -1), x], 1) + w["visual.positional_embedding"]
        x = F.layer_norm(x, (v.width,), w["visual.ln_pre.weight"], w["visual.ln_pre.bias"], 1e-5)
        for i in range(v.layers):
            x = self._block(x, f"visual.transformer.resblocks.{i}.", v.heads, None)
        return F.layer_norm(x, (v.width,), w["visual.ln_post.weight"], w["visual.ln_post.bias"], 1e-5)[:, 1:]

    @torch.inference_mode()
    def text_tokens(self, ids):
        t, w = self.cfg.text, self.w
        ids = torch.as_tensor(ids).long()
        L = ids.shape[1]
        x = w["token_embedding.weight"][ids] + w["positional_embedding"]
        mask = torch.full((L, L), float("-inf")).triu_(1)
        for i in range(t.layers):
            x = self._block(x, f"transformer.resblocks.{i}.", t.heads, mask)
        return F.layer_norm(x, (t.width,), w["ln_final.weight"], w["ln_final.bias"], 1e-5)


def rope_tokens(tokens) -> torch.Tensor:
    """apply_rope (pacl.py:147-181) of sparc_rope.forward_visual, through oracle.clip_oracle."""
    return torch.from_numpy(apply_rope(np.asarray(tokens.detach().cpu(), np.float32)))


def sparc_loss(v, l, g, mask, temperature):
    """SparcLoss.forward (pacl.py:522-584) with the reference's ATen calls."""
    scale = 1.0 / temperature
    gi = F.normalize(v.mean(dim=1), dim=-1)
    gt = F.normalize(l.mean(dim=1), dim=-1)
    li = scale * gi @ gt.T
    lt = scale * gt @ gi.T
    labels = torch.arange(li.shape[0], device=v.device)
    global_loss = (F.cross_entropy(li, labels) + F.cross_entropy(lt, labels)) / 2

    def local(a, b):
        B, T, _ = a.shape
        ml = (1.0 - mask) * (-1e8)
        labels2 = torch.eye(T, device=a.device).unsqueeze(0).expand(B, -1, -1).reshape(B * T, -1)
        z = torch.einsum("bmd,bnd->bmn", a, b) * scale + ml.unsqueeze(1)
        ce = F.cross_entropy(z.reshape(B * T, -1), labels2, reduction="none")
        m = mask.reshape(-1)
        return (ce * m).sum() / m.sum()

    return 0.5 * global_loss + 1.0 * (local(g, l) + local(l, g)) / 2


class TorchSparcTrainStep:
    """The SPARC head tensors as f32 leaf tensors (requires_grad) on `device`."""

    def __init__(self, heads_sd, device="cpu"):
        self.device = torch.device(device)
        self.w = {n: torch.as_tensor(np.asarray(heads_sd[n]) if not isinstance(heads_sd[n], torch.Tensor)
                                     else heads_sd[n].detach().cpu()).float().to(self.device).requires_grad_(True)
                  for n in HEAD_TENSORS}

    def _drop(self, x, keep, p):
        return x if keep is None else x * keep.to(x.device, x.dtype) / (1.0 - p)

    def forward(self, patch_tokens, text_tokens=None, l_token_embed=None, sigma=1.0 / 576, p=0.1, keep_v=None,
                keep_t=None):
        w = self.w
        x = torch.as_tensor(patch_tokens).float().to(self.device).clone()     # (inference-mode tokens)
        h = self._drop(F.layer_norm(x, (x.shape[-1],), w["visual_projection.0.weight"], w["visual_projection.0.bias"],
                                    1e-5), keep_v, p)
        v = F.linear(h, w["visual_projection.2.linear_projection.0.weight"],
                     w["visual_projection.2.linear_projection.0.bias"])
        v = v + F.linear(F.gelu(F.linear(h, w["visual_projection.2.non_linear_projection.0.weight"],
                                         w["visual_projection.2.non_linear_projection.0.bias"])),
                         w["visual_projection.2.non_linear_projection.2.weight"],
                         w["visual_projection.2.non_linear_projection.2.bias"])
        if l_token_embed is None:
            t = torch.as_tensor(text_tokens).float().to(self.device).clone()
            ht = self._drop(F.layer_norm(t, (t.shape[-1],), w["text_projection.0.weight"], w["text_projection.0.bias"],
                                         1e-5), keep_t, p)
            l = F.linear(ht, w["text_projection.2.weight"], w["text_projection.2.bias"])
        else:
            l = torch.as_tensor(l_token_embed).float().to(self.device).clone()
        sim = torch.einsum("btd,bpd->btp", l, v)
        mn = sim.min(dim=-1, keepdim=True)[0]
        mx = sim.max(dim=-1, keepdim=True)[0]
        sim = (sim - mn) / (mx - mn + 1e-8)
        sim = torch.where(sim < sigma, 0.0, sim)
        wts = sim / (sim.sum(dim=-1, keepdim=True) + 1e-8)
        g = F.normalize(torch.einsum("btp,bpd->btd", wts, v), p=2, dim=-1)
        return v, F.normalize(l, p=2, dim=-1), g

    def pacl_loss_and_grads(self, patch_tokens, pooled_text, temperature=0.1, p=0.1, keep_v=None, keep_t=None):
        """One train_pacl.py step's loss and head gradients (train_pacl.py:34-39 on open_clip_pacl /
        open_clip_pacl_rope, pacl.py:112-145,184-197): the visual head on the (RoPE'd) patch tokens, the
        ones-weighted patch sum, the text head on the pooled text embedding [B, 768], both
        L2-normalised, ClipLoss(temperature) (pacl.py:489-514).  keep_t: [B, 768] (or [B, 1, 768])."""
        for t in self.w.values():
            t.grad = None
        w = self.w
        x = torch.as_tensor(patch_tokens).float().to(self.device).clone()
        h = self._drop(F.layer_norm(x, (x.shape[-1],), w["visual_projection.0.weight"], w["visual_projection.0.bias"],
                                    1e-5), keep_v, p)
        v = F.linear(h, w["visual_projection.2.linear_projection.0.weight"],
                     w["visual_projection.2.linear_projection.0.bias"])
        v = v + F.linear(F.gelu(F.linear(h, w["visual_projection.2.non_linear_projection.0.weight"],
                                         w["visual_projection.2.non_linear_projection.0.bias"])),
                         w["visual_projection.2.non_linear_projection.2.weight"],
                         w["visual_projection.2.non_linear_projection.2.bias"])
        t = torch.as_tensor(pooled_text).float().to(self.device).clone()
        if keep_t is not None:
            keep_t = torch.as_tensor(keep_t).reshape(t.shape)
        ht = self._drop(F.layer_norm(t, (t.shape[-1],), w["text_projection.0.weight"], w["text_projection.0.bias"],
                                     1e-5), keep_t, p)
        tp = F.linear(ht, w["text_projection.2.weight"], w["text_projection.2.bias"])
        img = F.normalize(v.sum(dim=1), dim=-1)
        txt = F.normalize(tp, dim=-1)
        li = img @ txt.T / temperature
        labels = torch.arange(li.shape[0], device=li.device)
        loss = (F.cross_entropy(li, labels) + F.cross_entropy(li.T, labels)) / 2
        loss.backward()
        grads = {n: (t_.grad.detach().clone() if t_.grad is not None else None) for n, t_ in self.w.items()}
        return float(loss.detach()), grads

    def loss_and_grads(self, patch_tokens, mask, text_tokens=None, l_token_embed=None, sigma=1.0 / 576,
                       temperature=0.1, p=0.1, keep_v=None, keep_t=None):
        for t in self.w.values():
            t.grad = None
        v, l, g = self.forward(patch_tokens, text_tokens, l_token_embed, sigma, p, keep_v, keep_t)
        loss = sparc_loss(v, l, g, torch.as_tensor(mask).float().to(self.device), temperature)
        loss.backward()
        grads: Dict[str, Optional[torch.Tensor]] = {n: (t.grad.detach().clone() if t.grad is not None else None)
                                                    for n, t in self.w.items()}
        return float(loss), grads, (v.detach(), l.detach(), g.detach())
