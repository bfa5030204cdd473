"""The CPU oracle (oracle/clip_oracle.py) against golden vectors produced by the reference
itself (tests/golden/make_golden.py).  This is what pins the oracle; the GPU parity tests then
compare the HIP engine against the oracle and against these same fixtures."""
import hashlib

import numpy as np
import pytest

from clipembed import weights as W
from clipembed.config import get_model_config
from oracle import clip_oracle as O

ROWS_V = [0, 1, 23, 24, 287, 300, 551, 575]
ROWS_T = [0, 1, 5, 20, 40, 76]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rel(a, b):
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def clip_case(golden, tag, cfg, n_img):
    g = golden(tag)
    imgs = W.synthetic_images(n_img, seed=1000)
    assert sha(imgs) == str(g["images_sha"]), "image generator drifted from the golden inputs"
    sd = W.synthetic_state_dict(cfg)
    np.testing.assert_array_equal(sd["visual.conv1.weight"].ravel()[:8], g["weights_probe"][0])
    np.testing.assert_array_equal(sd["token_embedding.weight"].ravel()[:8], g["weights_probe"][1])
    pi, ti = O.encode_image(sd, imgs, cfg, output_tokens=True)
    pt, tt = O.encode_text(sd, g["captions"], cfg, output_tokens=True)
    return g, sd, imgs, pi, ti, pt, tt


@pytest.mark.parametrize("tag,name,layers", [("clip_v2t2", "ViT-L-14-336", (2, 2)),
                                             ("clip_quickgelu_v1t1", "ViT-L-14-336-quickgelu", (1, 1))])
def test_clip_reduced_depth(golden, tag, name, layers):
    cfg = get_model_config(name).with_depth(*layers)
    g, sd, imgs, pi, ti, pt, tt = clip_case(golden, tag, cfg, 2)
    assert rel(pi, g["image_pooled"]) < 2e-5
    assert rel(pt, g["text_pooled"]) < 2e-5
    assert rel(ti[:, ROWS_V], g["image_tokens_rows"]) < 2e-5
    assert rel(tt[:, ROWS_T], g["text_tokens_rows"]) < 2e-5
    np.testing.assert_allclose(ti.sum((1, 2)), g["image_tokens_sum"], rtol=1e-3, atol=0.5)
    il, tl = O.get_logits(O.l2normalize(pi), O.l2normalize(pt), float(g["logit_scale_exp"]))
    np.testing.assert_allclose(il, g["image_logits"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(tl, g["text_logits"], rtol=1e-5, atol=1e-4)


@pytest.mark.slow
def test_clip_full_depth(golden):
    cfg = get_model_config("ViT-L-14-336")
    g, sd, imgs, pi, ti, pt, tt = clip_case(golden, "clip_full", cfg, 2)
    assert rel(pi, g["image_pooled"]) < 1e-4
    assert rel(pt, g["text_pooled"]) < 1e-4
    assert rel(ti[:, ROWS_V], g["image_tokens_rows"]) < 1e-4
    il, _ = O.get_logits(O.l2normalize(pi), O.l2normalize(pt), float(g["logit_scale_exp"]))
    np.testing.assert_allclose(il, g["image_logits"], rtol=1e-4, atol=1e-3)
    assert (il.argmax(1) == g["image_logits"].argmax(1)).all()


def test_pacl_variants(golden):
    cfg = get_model_config("ViT-L-14-336").with_depth(2, 2)
    g = golden("pacl")
    imgs = W.synthetic_images(2, seed=1100)
    assert sha(imgs) == str(g["images_sha"])
    sd = W.synthetic_state_dict(cfg)
    heads = W.synthetic_pacl_heads(cfg.with_pacl(768))
    caps = g["captions"]
    _, tokens = O.encode_image(sd, imgs, cfg, output_tokens=True)
    vp = O.pacl_visual_head(heads, tokens)
    tp = O.pacl_text_head(heads, O.encode_text(sd, caps, cfg))
    assert rel(vp[:, ROWS_V[1:]], g["visual_proj_rows"]) < 2e-5
    assert rel(tp, g["text_proj"]) < 2e-5
    for tag, weights, rope in (("pacl", "ones", "none"), ("pacl_rope", "ones", "before"),
                               ("pacl_rope_after", "sigmoid", "after")):
        a, b = O.pacl_forward(sd, heads, imgs, caps, cfg, weights=weights, rope=rope)
        assert rel(a, g[f"{tag}_img"]) < 5e-5, tag
        assert rel(b, g[f"{tag}_txt"]) < 5e-5, tag
        a1, b1 = O.pacl_forward(sd, heads, imgs[:1], caps, cfg, weights=weights, rope=rope)
        assert a1.shape == g[f"{tag}_bcast_img"].shape == (2, 768)
        assert rel(a1, g[f"{tag}_bcast_img"]) < 5e-5, tag
    a, _ = O.pacl_pool(vp, tp, weights="sigmoid")
    assert rel(a, g["pacl_sigmoid_img"]) < 5e-5


def test_apply_rope(golden):
    x = W.uniform("rope-input", 2 * 576 * 128).reshape(2, 576, 128)
    y = O.apply_rope(x)
    # f32 pow differs from torch's by <= 1 ulp on a few inv_freq entries; angles up to 575 rad
    # amplify that to ~3e-5 absolute in sin/cos (see oracle.apply_rope)
    assert rel(y, golden("rope")["y"]) < 1e-4


def test_sparc(golden):
    g = golden("sparc")
    v = W.uniform("sparc-v", 2 * 576 * 64).reshape(2, 576, 64)
    l = W.uniform("sparc-l", 2 * 77 * 64).reshape(2, 77, 64)
    for name, sigma in (("s576", 1.0 / 576), ("s625", 1.0 / 625)):
        grouped, lnorm, _ = O.sparc_forward(v, l, sigma)
        assert rel(grouped, g[f"{name}_grouped"]) < 1e-5
        assert rel(lnorm, g[f"{name}_l_norm"]) < 1e-6
        gl = O.l2normalize(grouped.mean(1)) @ O.l2normalize(lnorm.mean(1)).T
        np.testing.assert_allclose(gl, g[f"{name}_score_local"], rtol=1e-5, atol=1e-6)
        mask = (np.arange(77)[None, :] <= np.array([[20], [76]])).astype(np.float32)
        loss = O.sparc_loss(v, g[f"{name}_l_norm"], g[f"{name}_grouped"], mask, 0.1)
        np.testing.assert_allclose(loss, g[f"{name}_sparc_loss"], rtol=1e-5)


def test_losses(golden):
    g = golden("loss")
    a = O.l2normalize(W.uniform("loss-a", 8 * 768).reshape(8, 768))
    b = O.l2normalize(W.uniform("loss-b", 8 * 768).reshape(8, 768))
    np.testing.assert_allclose(O.pacl_clip_loss(a, b, 0.1), g["pacl_clip_loss"], rtol=1e-5)
    s = 14.2857
    lab = np.arange(8)
    single = (O.cross_entropy(s * a @ b.T, lab) + O.cross_entropy(s * b @ a.T, lab)) / 2
    np.testing.assert_allclose(single, g["openclip_single"], rtol=1e-5)


def test_negclip_two_ranks(golden):
    g = golden("negclip")
    B, D = 4, 768
    imgs = [O.l2normalize(W.uniform(f"neg-img-{r}", B * D).reshape(B, D)) for r in range(2)]
    txts = [O.l2normalize(W.uniform(f"neg-txt-{r}", (B + K) * D).reshape(B + K, D)) for r, K in enumerate([2, 3])]
    for r in range(2):
        got = O.negclip_local_loss(imgs, txts, B, r, 14.2857)
        np.testing.assert_allclose(got, g[f"hard_r{r}"], rtol=1e-5)
        plain = O.negclip_local_loss(imgs, [t[:B] for t in txts], B, r, 14.2857)
        np.testing.assert_allclose(plain, g[f"plain_local_r{r}"], rtol=1e-5)


@pytest.mark.parametrize("tag,name,layers", [("clip_v2t2", "ViT-L-14-336", (2, 2)),
                                             ("clip_quickgelu_v1t1", "ViT-L-14-336-quickgelu", (1, 1))])
def test_torch_cpu_baseline_vs_golden(golden, tag, name, layers):
    """The torch f32 CPU restatement bench.py times as the reference's CPU path
    (oracle/clip_torch_cpu.py: the reference's own ATen calls) is pinned to the same goldens."""
    from oracle.clip_torch_cpu import TorchCLIP
    cfg = get_model_config(name).with_depth(*layers)
    g = golden(tag)
    sd = W.synthetic_state_dict(cfg)
    m = TorchCLIP(sd, cfg)
    pi = m.encode_image(W.synthetic_images(2, seed=1000)).numpy()
    pt = m.encode_text(g["captions"]).numpy()
    assert rel(pi, g["image_pooled"]) < 2e-5
    assert rel(pt, g["text_pooled"]) < 2e-5
    fi = m.encode_image(W.synthetic_images(2, seed=1000), normalize=True)
    ft = m.encode_text(g["captions"], normalize=True)
    il, _ = m.get_logits(fi, ft, float(g["logit_scale_exp"]))
    np.testing.assert_allclose(il.numpy(), g["image_logits"], rtol=1e-5, atol=1e-4)
