"""Deterministic per-rank inputs of the sharded-loss fixtures (sparc_dist.npz): a pure function of
(rank, sizes) through clipembed.weights.uniform, so the fixture script (build container, reference
run) and the tests (CPU gloo ranks, GPU ranks) build identical tensors without shipping them."""
import numpy as np

from clipembed import weights as W

EOTS = [[0, 76, 9, 30], [1, 55, 17, 5]]   # per rank: EOT at 0 (one live token) and 76 (all live)


def _l2(x):
    return (x / np.maximum(np.linalg.norm(x, axis=-1, keepdims=True), 1e-12)).astype(np.float32)


def sparc_shard(rank, B=4, P=576, T=77, D=768):
    """v [B,P,D] unnormalised patch embeddings, l / g [B,T,D] L2-normalised token / grouped
    embeddings (g correlated with l, as grouping makes them), mask [B,T] (1 up to the EOT)."""
    v = 0.5 * W.uniform(f"sparc-dist-v-{rank}", B * P * D).reshape(B, P, D)
    l = _l2(W.uniform(f"sparc-dist-l-{rank}", B * T * D).reshape(B, T, D))
    g = _l2(l + 0.7 * W.uniform(f"sparc-dist-g-{rank}", B * T * D).reshape(B, T, D) / np.sqrt(D))
    eot = np.array(EOTS[rank][:B])
    mask = (np.arange(T)[None, :] <= eot[:, None]).astype(np.float32)
    return v.astype(np.float32), l, g, mask


def pacl_shard(rank, B=4, D=768):
    """L2-normalised pooled image / text features [B,D] (the PACL forward's outputs)."""
    img = _l2(W.uniform(f"pacl-dist-i-{rank}", B * D).reshape(B, D))
    txt = _l2(img + 0.3 * W.uniform(f"pacl-dist-t-{rank}", B * D).reshape(B, D))
    return img, txt
