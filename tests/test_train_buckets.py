"""CPU: the NegCLIP trainer's gradient buckets (clipembed.train.TextTowerTrainer._make_buckets) partition
the flat gradient buffer exactly, in the order the backward finishes them (head + logit_scale, blocks
top-down, embeddings), for the flat layout the trainer builds ([decay | no-decay | logit_scale],
main.py:335-349).  No engine: the layout is rebuilt here over CPU zeros."""
from types import SimpleNamespace

import pytest
import torch

from clipembed.config import get_model_config
from clipembed.train import TextTowerTrainer, _excluded, text_tensor_names


def _fake_trainer(layers):
    cfg = get_model_config("ViT-L-14-336").with_depth(1, layers)
    model = SimpleNamespace(cfg=cfg)
    t, D, F = cfg.text, cfg.text.width, cfg.text.width * 4
    shapes = {"token_embedding.weight": (64, D), "positional_embedding": (77, D),
              "ln_final.weight": (D,), "ln_final.bias": (D,), "text_projection": (D, cfg.embed_dim)}
    for l in range(t.layers):
        p = f"transformer.resblocks.{l}."
        shapes.update({p + "ln_1.weight": (D,), p + "ln_1.bias": (D,), p + "attn.in_proj_weight": (3 * D, D),
                       p + "attn.in_proj_bias": (3 * D,), p + "attn.out_proj.weight": (D, D),
                       p + "attn.out_proj.bias": (D,), p + "ln_2.weight": (D,), p + "ln_2.bias": (D,),
                       p + "mlp.c_fc.weight": (F, D), p + "mlp.c_fc.bias": (F,), p + "mlp.c_proj.weight": (D, F),
                       p + "mlp.c_proj.bias": (D,)})
    names = text_tensor_names(model)
    assert sorted(names) == sorted(shapes)
    decay = [n for n in names if not _excluded(n, torch.empty(shapes[n], device="meta"))]
    order = decay + [n for n in names if n not in decay]
    tr = TextTowerTrainer.__new__(TextTowerTrainer)
    tr.model = model
    tr.n_total = sum(torch.Size(shapes[n]).numel() for n in order) + 1
    tr.grad = torch.zeros(tr.n_total)
    tr.gviews, off = {}, 0
    for n in order:
        k = torch.Size(shapes[n]).numel()
        tr.gviews[n] = tr.grad[off:off + k].view(shapes[n])
        off += k
    return tr


@pytest.mark.parametrize("layers,per", [(12, 1), (12, 2), (12, 5), (2, 1), (1, 3)])
def test_buckets_partition_flat_buffer(layers, per):
    tr = _fake_trainer(layers)
    buckets = tr._make_buckets(per)
    # the head first (event 0), then one bucket per `per` blocks top-down, the embeddings last
    assert buckets[0][0] == 0 and buckets[-1][0] is None
    evs = [e for e, _ in buckets[1:-1]]
    assert evs == sorted(evs) and evs[-1] == layers and len(evs) == -(-layers // per)
    mark = torch.zeros(tr.n_total, dtype=torch.int32)
    for _, runs in buckets:
        for lo, hi in runs:
            mark[lo:hi] += 1
    assert bool((mark == 1).all())
    # logit_scale (the last element) travels with the head bucket
    assert any(lo <= tr.n_total - 1 < hi for lo, hi in buckets[0][1])
    # every tensor of block b sits in the bucket whose event follows block b's backward
    for e, runs in buckets[1:-1]:
        lowest = layers - e
        for n, v in tr.gviews.items():
            if n.startswith(f"transformer.resblocks.{lowest}."):
                o = v.storage_offset()
                assert any(lo <= o < hi for lo, hi in runs), n
