"""CPU BASELINE RESTATEMENT — test/benchmark infrastructure only.

The reference's CPU forward of CLIP ViT-L/14-336 (open_clip, float32) restated with the same ATen
calls the reference makes, so that bench.py's `cpu_baseline` leg times what a user of the reference
runs on the host, not a NumPy port:
  conv1            nn.Conv2d(3, 1024, 14, 14, bias=False)         transformer.py:549-555  -> F.conv2d
  cls / pos / LN   VisionTransformer._embeds                      transformer.py:701-716  -> F.layer_norm
  block            ResidualAttentionBlock.forward                 transformer.py:257-268
  attention        nn.MultiheadAttention(batch_first) in eval     transformer.py:228,242-255
                                                                  -> F.multi_head_attention_forward
  MLP              c_fc -> GELU(erf) / QuickGELU -> c_proj         transformer.py:235-239  -> F.linear, F.gelu
  pool + proj      _pool('tok') / EOT argmax, @ proj              transformer.py:718-741,839-855
  encode_*         CLIP.encode_image / encode_text                model.py:279-301
  logits           normalize, exp(logit_scale) I T^T               model.py:303-310
It is imported only by tests/ (pinned against tests/golden like oracle/clip_oracle.py) and by
bench.py's cpu_baseline leg.  The product package never imports it.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _t(sd, name):
    v = sd[name]
    return v if isinstance(v, torch.Tensor) else torch.from_numpy(v)


class TorchCLIP:
    """Weights as f32 CPU tensors (converted once), forward under torch.inference_mode()."""

    def __init__(self, sd, cfg):
        self.cfg = cfg
        self.w = {k: _t(sd, k).float().contiguous() for k in sd}
        self.act = (lambda x: x * torch.sigmoid(1.702 * x)) if cfg.quick_gelu else F.gelu

    def _block(self, x, p, heads, mask):
        w = self.w
        h = F.layer_norm(x, (x.shape[-1],), w[p + "ln_1.weight"], w[p + "ln_1.bias"], 1e-5)
        # nn.MultiheadAttention(batch_first=True): (L, B, D) internally
        hq = h.transpose(0, 1)
        a, _ = F.multi_head_attention_forward(
            hq, hq, hq, x.shape[-1], heads, w[p + "attn.in_proj_weight"], w[p + "attn.in_proj_bias"], None, None,
            False, 0.0, w[p + "attn.out_proj.weight"], w[p + "attn.out_proj.bias"], training=False,
            need_weights=False, attn_mask=mask)
        x = x + a.transpose(0, 1)
        h = F.layer_norm(x, (x.shape[-1],), w[p + "ln_2.weight"], w[p + "ln_2.bias"], 1e-5)
        h = self.act(F.linear(h, w[p + "mlp.c_fc.weight"], w[p + "mlp.c_fc.bias"]))
        return x + F.linear(h, w[p + "mlp.c_proj.weight"], w[p + "mlp.c_proj.bias"])

    @torch.inference_mode()
    def encode_image(self, pixels, normalize=False):
        v, w = self.cfg.vision, self.w
        x = torch.as_tensor(pixels).float()
        x = F.conv2d(x, w["visual.conv1.weight"], stride=v.patch_size)          # [B, D, G, G]
        x = x.reshape(x.shape[0], x.shape[1], -1).permute(0, 2, 1)
        cls = w["visual.class_embedding"].expand(x.shape[0], 1, -1)
        x = torch.cat([cls, x], 1) + w["visual.positional_embedding"]
        x = F.layer_norm(x, (v.width,), w["visual.ln_pre.weight"], w["visual.ln_pre.bias"], 1e-5)
        for i in range(v.layers):
            x = self._block(x, f"visual.transformer.resblocks.{i}.", v.heads, None)
        x = F.layer_norm(x, (v.width,), w["visual.ln_post.weight"], w["visual.ln_post.bias"], 1e-5)
        pooled = x[:, 0] @ w["visual.proj"]
        return F.normalize(pooled, dim=-1) if normalize else pooled

    @torch.inference_mode()
    def encode_text(self, ids, normalize=False):
        t, w = self.cfg.text, self.w
        ids = torch.as_tensor(ids).long()
        L = ids.shape[1]
        x = w["token_embedding.weight"][ids] + w["positional_embedding"]
        mask = torch.full((L, L), float("-inf")).triu_(1)
        for i in range(t.layers):
            x = self._block(x, f"transformer.resblocks.{i}.", t.heads, mask)
        x = F.layer_norm(x, (t.width,), w["ln_final.weight"], w["ln_final.bias"], 1e-5)
        pooled = x[torch.arange(x.shape[0]), ids.argmax(dim=-1)] @ w["text_projection"]
        return F.normalize(pooled, dim=-1) if normalize else pooled

    @torch.inference_mode()
    def get_logits(self, fi, ft, scale):
        li = scale * fi @ ft.T
        return li, li.T
