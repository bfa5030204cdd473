"""End-to-end parity of the HIP engine (through the C ABI) against the reference's golden vectors
(tests/golden, produced by running open_clip / pacl.py) and the pinned CPU oracle.

Tolerance (north_star): the engine computes in bf16 (MFMA, f32 accumulate, f32 residual stream,
f32 LayerNorm statistics); pooled embeddings must be within 1e-3 cosine distance of the f32
reference and produce identical top-1 retrieval indices."""
import numpy as np
import pytest
import torch

import clipembed
from clipembed import ClipEmbedError, weights as W
from clipembed.config import get_model_config
from clipembed.pacl import (apply_rope, open_clip_pacl, open_clip_pacl_rope, open_clip_pacl_rope_after,
                            open_clip_pacl_sigmoid)
from oracle import clip_oracle as O

pytestmark = pytest.mark.gpu

ROWS_V = [0, 1, 23, 24, 287, 300, 551, 575]
ROWS_T = [0, 1, 5, 20, 40, 76]
COS_TOL = 1e-3


def cos_dist(a, b):
    a = np.asarray(a, np.float64).reshape(-1, a.shape[-1])
    b = np.asarray(b, np.float64).reshape(-1, b.shape[-1])
    c = (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
    return float((1 - c).max())


def make_model(cfg):
    m = clipembed.CLIP(cfg)
    m.load_state_dict(W.synthetic_state_dict(cfg))
    return m.to("cuda")


@pytest.fixture(scope="module")
def small():
    return make_model(get_model_config("ViT-L-14-336").with_depth(2, 2))


def test_reduced_depth_vs_golden(small, golden):
    g = golden("clip_v2t2")
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1000))
    caps = torch.from_numpy(g["captions"])
    small.visual.output_tokens = True
    small.output_text_tokens = True
    try:
        pi, ti = small.encode_image(imgs)
        pt, tt = small.encode_text(caps)
    finally:
        small.visual.output_tokens = False
        small.output_text_tokens = False
    pi, ti, pt, tt = (x.cpu().numpy() for x in (pi, ti, pt, tt))
    assert cos_dist(pi, g["image_pooled"]) < COS_TOL
    assert cos_dist(pt, g["text_pooled"]) < COS_TOL
    assert cos_dist(ti[:, ROWS_V], g["image_tokens_rows"]) < COS_TOL
    assert cos_dist(tt[:, ROWS_T], g["text_tokens_rows"]) < COS_TOL
    il, tl = small.get_logits(imgs, caps)
    # logits = scale * cosine: hold them to the features' bar (rows as vectors within 1e-3 cosine
    # distance of the reference rows) and each cosine within 2e-3 absolute
    il_n = il.cpu().numpy()
    assert cos_dist(il_n, g["image_logits"]) < COS_TOL
    s_ref = float(g["logit_scale_exp"])
    np.testing.assert_allclose(il_n / s_ref, g["image_logits"] / s_ref, atol=2e-3)
    assert np.array_equal(tl.cpu().numpy(), il.cpu().numpy().T)
    fi, ft, ls = small(imgs, caps)
    assert cos_dist(fi.cpu().numpy(), g["image_features"]) < COS_TOL
    np.testing.assert_allclose(np.linalg.norm(fi.cpu().numpy(), axis=-1), 1.0, rtol=1e-5)
    np.testing.assert_allclose(float(ls), float(g["logit_scale_exp"]), rtol=1e-6)


def test_reduced_depth_vs_oracle_batch(small):
    """Batch of 5 images / 7 texts (ragged tiles) against the oracle on the same inputs."""
    cfg = small.cfg
    sd = W.synthetic_state_dict(cfg)
    imgs = W.synthetic_images(5, seed=1234)
    caps = W.synthetic_captions(7, seed=4321)
    pi = small.encode_image(torch.from_numpy(imgs)).cpu().numpy()
    pt = small.encode_text(torch.from_numpy(caps)).cpu().numpy()
    assert cos_dist(pi, O.encode_image(sd, imgs, cfg)) < COS_TOL
    assert cos_dist(pt, O.encode_text(sd, caps, cfg)) < COS_TOL


def test_pooled_prune_vs_oracle_ragged(small):
    """Pooled-only calls run each tower's last block for the pooled rows only (CLS / EOT,
    ce_set_pooled_prune, default on): against the oracle on 3 images and 5 captions whose EOT sits
    at positions 1, 76 and in between, and against the unpruned path (prune off, and the tokens
    call, which never prunes) within 2e-5 cosine."""
    cfg = small.cfg
    sd = W.synthetic_state_dict(cfg)
    imgs = torch.from_numpy(W.synthetic_images(3, seed=77))
    caps = W.synthetic_captions(5, seed=78)
    rng = np.random.default_rng(79)
    caps[0] = 0
    caps[0, :2] = [49406, 49407]                                  # empty caption: EOT at 1
    caps[1] = rng.integers(1, 49000, 77)
    caps[1, 0], caps[1, 76] = 49406, 49407                        # EOT at the last position
    ct = torch.from_numpy(caps)
    pi, pt = small.encode_image(imgs), small.encode_text(ct)
    prev = small.engine.set_pooled_prune(False)
    try:
        assert prev
        qi, qt = small.encode_image(imgs), small.encode_text(ct)
    finally:
        small.engine.set_pooled_prune(prev)
    small.visual.output_tokens = True
    small.output_text_tokens = True
    try:
        ri, _ = small.encode_image(imgs)
        rt, _ = small.encode_text(ct)
    finally:
        small.visual.output_tokens = False
        small.output_text_tokens = False
    pi, pt, qi, qt, ri, rt = (x.cpu().numpy() for x in (pi, pt, qi, qt, ri, rt))
    assert cos_dist(pi, qi) < 2e-5 and cos_dist(pt, qt) < 2e-5
    assert np.array_equal(qi, ri) and np.array_equal(qt, rt)
    assert cos_dist(pi, O.encode_image(sd, imgs.numpy(), cfg)) < COS_TOL
    assert cos_dist(pt, O.encode_text(sd, caps, cfg)) < COS_TOL


@pytest.mark.parametrize("eots", [(13, 33), (40, 5, 60), (2, 2)])
def test_pooled_text_packed_rows_every_caption(small, eots):
    """Packed text rows (pooled-only encode_text): every caption of the batch, not only the first (whose
    packed and unpacked rows coincide), matches the unpruned tokens call and the oracle; also with the
    per-kernel profile pass on, which reads the packed offsets back (round-4 regression: that readback
    displaced the pooled-row selection)."""
    cfg = small.cfg
    sd = W.synthetic_state_dict(cfg)
    rng = np.random.default_rng(sum(eots))
    caps = np.zeros((len(eots), 77), np.int64)
    for i, e in enumerate(eots):
        caps[i, 0], caps[i, e] = 49406, 49407
        caps[i, 1:e] = rng.integers(1, 49000, e - 1)
    ct = torch.from_numpy(caps)
    ref = O.encode_text(sd, caps, cfg)
    pt = small.encode_text(ct).cpu().numpy()
    small.engine.set_timing(True)
    try:
        pt2 = small.encode_text(ct).cpu().numpy()
    finally:
        small.engine.set_timing(False)
    small.output_text_tokens = True
    try:
        rt, _ = small.encode_text(ct)
    finally:
        small.output_text_tokens = False
    rt = rt.cpu().numpy()
    assert cos_dist(pt, rt) < 2e-5 and cos_dist(pt2, rt) < 2e-5
    assert cos_dist(pt, ref) < COS_TOL


def test_text_width_outside_the_fold_kernel():
    """A text width the LN-fold entry kernel does not cover (1536: D % 64 == 0 but not one of its
    256/512/768/1024/1280 instantiations) runs the unfolded text tower instead of failing
    (round-3 advisor finding), within 1e-3 cosine of the oracle."""
    import dataclasses
    base = get_model_config("ViT-L-14-336").with_depth(1, 1)
    cfg = dataclasses.replace(base, name="text-1536", text=dataclasses.replace(base.text, width=1536, heads=24,
                                                                                mlp_width=6144))
    sd = W.synthetic_state_dict(cfg)
    m = clipembed.CLIP(cfg)
    m.load_state_dict(sd)
    m.to("cuda")
    caps = W.synthetic_captions(3, seed=91)
    got = m.encode_text(torch.from_numpy(caps)).cpu().numpy()
    assert cos_dist(got, O.encode_text(sd, caps, cfg)) < COS_TOL


def test_bf16_pixels(small):
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1000))
    a = small.encode_image(imgs)
    b = small.encode_image(imgs.to(torch.bfloat16))
    assert cos_dist(a.cpu().numpy(), b.cpu().numpy()) < 1e-3


def test_quickgelu_vs_golden(golden):
    cfg = get_model_config("ViT-L-14-336-quickgelu").with_depth(1, 1)
    m = make_model(cfg)
    g = golden("clip_quickgelu_v1t1")
    pi = m.encode_image(torch.from_numpy(W.synthetic_images(2, seed=1000))).cpu().numpy()
    pt = m.encode_text(torch.from_numpy(g["captions"])).cpu().numpy()
    assert cos_dist(pi, g["image_pooled"]) < COS_TOL
    assert cos_dist(pt, g["text_pooled"]) < COS_TOL


def test_full_depth_vs_golden(golden):
    """ViT-L/14-336 at full depth (24 + 12 blocks) vs the reference f32 CPU forward."""
    cfg = get_model_config("ViT-L-14-336")
    m = make_model(cfg)
    g = golden("clip_full")
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1000))
    caps = torch.from_numpy(g["captions"])
    m.visual.output_tokens = True
    pi, ti = m.encode_image(imgs)
    m.visual.output_tokens = False
    pt = m.encode_text(caps)
    assert cos_dist(pi.cpu().numpy(), g["image_pooled"]) < COS_TOL
    assert cos_dist(pt.cpu().numpy(), g["text_pooled"]) < COS_TOL
    assert cos_dist(ti.cpu().numpy()[:, ROWS_V], g["image_tokens_rows"]) < COS_TOL
    il, _ = m.get_logits(imgs, caps)
    assert (il.cpu().numpy().argmax(1) == g["image_logits"].argmax(1)).all()
    assert (il.cpu().numpy().argmax(0) == g["image_logits"].argmax(0)).all()


def test_full_depth_retrieval_top1_vs_oracle():
    """Top-1 retrieval indices over 6 x 6 synthetic pairs identical to the f32 oracle."""
    cfg = get_model_config("ViT-L-14-336")
    m = make_model(cfg)
    sd = W.synthetic_state_dict(cfg)
    imgs = W.synthetic_images(6, seed=777)
    caps = W.synthetic_captions(6, seed=888)
    il, _ = m.get_logits(torch.from_numpy(imgs), torch.from_numpy(caps))
    oi = O.encode_image(sd, imgs, cfg, normalize=True)
    ot = O.encode_text(sd, caps, cfg, normalize=True)
    ref, _ = O.get_logits(oi, ot, float(np.exp(np.log(1 / 0.07))))
    got = il.cpu().numpy()
    assert cos_dist(got, ref) < COS_TOL
    assert (got.argmax(1) == ref.argmax(1)).all() and (got.argmax(0) == ref.argmax(0)).all()


def _ran_folded(m, fn):
    """Run fn() with kernel timing on; True when the folded LayerNorm path ran (its stats launches)."""
    e = m._engine
    e.set_timing(True)
    try:
        out = fn()
        torch.cuda.synchronize()
        names = {k["name"] for k in e.kernel_stats()}
    finally:
        e.set_timing(False)
    return out, "ln_stats_v" in names


def test_resid_hl_matches_f32_stream():
    """The folded image tower with its residual stream as hi/lo bf16 planes (default) vs the f32
    stream + bf16 copy, full depth: pooled and token outputs within 1e-5 cosine of each other
    (|x - (hi + lo)| <= 2^-16 |x| per residual GEMM) and within 1e-3 of the golden."""
    cfg = get_model_config("ViT-L-14-336")
    m = make_model(cfg)
    imgs = torch.from_numpy(W.synthetic_images(3, seed=98))
    m.visual.output_tokens = True
    try:
        ph, th = m.encode_image(imgs)
        prev = m._engine.set_resid_hl(False)
        assert prev
        try:
            pf, tf = m.encode_image(imgs)
        finally:
            m._engine.set_resid_hl(True)
        assert cos_dist(ph.cpu().numpy(), pf.cpu().numpy()) < 1e-5
        assert cos_dist(th.cpu().numpy()[:, ROWS_V], tf.cpu().numpy()[:, ROWS_V]) < 1e-5
        o = O.encode_image(W.synthetic_state_dict(cfg), imgs.numpy(), cfg)
        assert cos_dist(ph.cpu().numpy(), o) < COS_TOL
    finally:
        m.visual.output_tokens = False


def test_ln_fold_matches_unfolded():
    """Image tower with ln_1/ln_2 folded into in_proj/c_fc (default) vs the LayerNorm path, at full
    depth: pooled and token outputs within 2e-4 cosine of each other and both within 1e-3 of the
    golden.  A partial reload of one LN weight invalidates that fold (the unfolded
    path runs, with the new weight); a whole-block reload restores it."""
    cfg = get_model_config("ViT-L-14-336")
    m = make_model(cfg)
    imgs = torch.from_numpy(W.synthetic_images(3, seed=99))
    m.visual.output_tokens = True
    try:
        (pf, tf), folded = _ran_folded(m, lambda: m.encode_image(imgs))
        assert folded
        prev = m._engine.set_ln_fold(False)
        assert prev
        (pu, tu), folded = _ran_folded(m, lambda: m.encode_image(imgs))
        assert not folded
        m._engine.set_ln_fold(True)
        assert cos_dist(pf.cpu().numpy(), pu.cpu().numpy()) < 2e-4
        assert cos_dist(tf.cpu().numpy()[:, ROWS_V], tu.cpu().numpy()[:, ROWS_V]) < 2e-4
        sd = W.synthetic_state_dict(cfg)
        o = O.encode_image(sd, imgs.numpy(), cfg)
        assert cos_dist(pf.cpu().numpy(), o) < COS_TOL
        # partial reload: one LN weight alone -> fold of that block is stale -> unfolded path
        k = "visual.transformer.resblocks.3.ln_2.weight"
        w2 = torch.from_numpy(sd[k] * 1.5)
        m.load_state_dict({k: w2})
        (p2, _), folded = _ran_folded(m, lambda: m.encode_image(imgs))
        assert not folded
        sd2 = dict(sd)
        sd2[k] = w2.numpy()
        assert cos_dist(p2.cpu().numpy(), O.encode_image(sd2, imgs.numpy(), cfg)) < COS_TOL
        # whole block reload refolds it
        pfx = "visual.transformer.resblocks.3."
        m.load_state_dict({n: torch.from_numpy(np.asarray(v)) for n, v in sd2.items() if n.startswith(pfx)})
        (p3, _), folded = _ran_folded(m, lambda: m.encode_image(imgs))
        assert folded
        assert cos_dist(p3.cpu().numpy(), p2.cpu().numpy()) < 2e-4
    finally:
        m.visual.output_tokens = False


def _ran_text_folded(m, fn):
    e = m._engine
    e.set_timing(True)
    try:
        out = fn()
        torch.cuda.synchronize()
        names = {k["name"] for k in e.kernel_stats()}
    finally:
        e.set_timing(False)
    return out, "ln_stats_t" in names and "ln_t" not in names


def test_text_ln_fold_matches_unfolded():
    """Text tower with ln_1/ln_2 folded into in_proj/c_fc and its residual stream as hi/lo planes
    (default, as the image tower) vs the LayerNorm path, full depth, causal blocks: pooled and
    token outputs within 2e-4 cosine of each other and within 1e-3 of the golden reference; the
    f32-stream fold agrees to 1e-5; a partial reload of one LN weight runs the unfolded text blocks
    with the new weight."""
    cfg = get_model_config("ViT-L-14-336")
    m = make_model(cfg)
    caps = torch.from_numpy(W.synthetic_captions(5, seed=77))
    m.output_text_tokens = True
    try:
        (pf, tf), folded = _ran_text_folded(m, lambda: m.encode_text(caps))
        assert folded
        prev = m._engine.set_resid_hl(False)
        try:
            (ph, th), folded = _ran_text_folded(m, lambda: m.encode_text(caps))
            assert folded
        finally:
            m._engine.set_resid_hl(prev)
        # 12 random-init causal blocks amplify the rare 1-ulp bf16 flips of the GEMM operand that the
        # two streams' residuals (f32 vs hi + lo, |x - (hi + lo)| <= 2^-16 |x|) cause; one block shows
        # the per-block agreement (test_text_resid_hl_one_block)
        assert cos_dist(pf.cpu().numpy(), ph.cpu().numpy()) < 3e-5
        m._engine.set_ln_fold(False)
        try:
            (pu, tu), folded = _ran_text_folded(m, lambda: m.encode_text(caps))
            assert not folded
        finally:
            m._engine.set_ln_fold(True)
        assert cos_dist(pf.cpu().numpy(), pu.cpu().numpy()) < 2e-4
        assert cos_dist(tf.cpu().numpy().reshape(-1, 768), tu.cpu().numpy().reshape(-1, 768)) < 2e-4
        sd = W.synthetic_state_dict(cfg)
        o = O.encode_text(sd, caps.numpy(), cfg)
        assert cos_dist(pf.cpu().numpy(), o) < COS_TOL
        k = "transformer.resblocks.5.ln_1.bias"
        b2 = torch.from_numpy(sd[k] + 0.5)
        m.load_state_dict({k: b2})
        (p2, _), folded = _ran_text_folded(m, lambda: m.encode_text(caps))
        assert not folded
        sd2 = dict(sd)
        sd2[k] = b2.numpy()
        assert cos_dist(p2.cpu().numpy(), O.encode_text(sd2, caps.numpy(), cfg)) < COS_TOL
        m.load_state_dict({k: torch.from_numpy(sd[k])})
    finally:
        m.output_text_tokens = False


def test_text_resid_hl_one_block():
    """One folded text block: the hi/lo residual planes (written by the embedding kernel, updated
    by the out-proj GEMM) vs the f32 stream.  The text residual stream is small (token + positional
    embeddings, std ~0.02), so the LN fold's rstd (~50) magnifies the rare 1-ulp flips of bf16(x)
    that the two representations cause: measured 7.0e-7 token cosine distance between them vs
    2.7e-5 for either against the f32 oracle (the unfolded LayerNorm path: 2.4e-5;
    tools/diag_text_fold.py)."""
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    m = make_model(cfg)
    caps = torch.from_numpy(W.synthetic_captions(8, seed=78))
    m.output_text_tokens = True
    try:
        ph, th = m.encode_text(caps)
        prev = m._engine.set_resid_hl(False)
        try:
            pf, tf = m.encode_text(caps)
        finally:
            m._engine.set_resid_hl(prev)
        assert cos_dist(th.cpu().numpy().reshape(-1, 768), tf.cpu().numpy().reshape(-1, 768)) < 5e-6
        assert cos_dist(ph.cpu().numpy(), pf.cpu().numpy()) < 5e-6
        o, ot = O.encode_text(W.synthetic_state_dict(cfg), caps.numpy(), cfg, output_tokens=True)
        assert cos_dist(ph.cpu().numpy(), o) < COS_TOL
        assert cos_dist(th.cpu().numpy(), ot) < 1e-4
    finally:
        m.output_text_tokens = False


@pytest.fixture(scope="module")
def pacl_models():
    cfg = get_model_config("ViT-L-14-336").with_depth(2, 2)
    sd = W.synthetic_state_dict(cfg)
    heads = W.synthetic_pacl_heads(cfg.with_pacl(768))
    out = {}
    for tag, cls in (("pacl", open_clip_pacl), ("pacl_rope", open_clip_pacl_rope),
                     ("pacl_rope_after", open_clip_pacl_rope_after), ("pacl_sigmoid", open_clip_pacl_sigmoid)):
        mod = cls(cfg=cfg, clip_state_dict=sd)
        mod.load_state_dict(heads)
        mod.to("cuda")
        out[tag] = mod
    return out


@pytest.mark.parametrize("tag", ["pacl", "pacl_rope", "pacl_rope_after"])
def test_pacl_forward_vs_golden(pacl_models, golden, tag):
    g = golden("pacl")
    mod = pacl_models[tag]
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1100))
    caps = torch.from_numpy(g["captions"])
    a, b = mod(imgs, caps)
    assert cos_dist(a.cpu().numpy(), g[f"{tag}_img"]) < COS_TOL
    assert cos_dist(b.cpu().numpy(), g[f"{tag}_txt"]) < COS_TOL
    a1, b1 = mod(imgs[:1], caps)                      # Q6: 1 image x 2 texts -> [2, 768]
    assert tuple(a1.shape) == g[f"{tag}_bcast_img"].shape == (2, 768)
    assert cos_dist(a1.cpu().numpy(), g[f"{tag}_bcast_img"]) < COS_TOL


def test_pacl_heads_and_sigmoid_pool(pacl_models, golden):
    g = golden("pacl")
    mod = pacl_models["pacl_sigmoid"]
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1100))
    caps = torch.from_numpy(g["captions"])
    vp = mod.forward_visual(imgs)
    tp = mod.forward_text(caps)
    assert cos_dist(vp.cpu().numpy()[:, ROWS_V[1:]], g["visual_proj_rows"]) < COS_TOL
    assert cos_dist(tp.cpu().numpy(), g["text_proj"]) < COS_TOL
    a, _ = mod.pool(vp, tp)
    assert cos_dist(a.cpu().numpy(), g["pacl_sigmoid_img"]) < COS_TOL
    a2, _ = mod(imgs, caps)
    assert cos_dist(a2.cpu().numpy(), g["pacl_sigmoid_img"]) < COS_TOL


def test_pacl_pool_exact_vs_oracle(pacl_models):
    """Pooling kernel alone on f32 inputs (no bf16 upstream): tight tolerance, all broadcast shapes."""
    mod = pacl_models["pacl_sigmoid"]
    rng = np.random.default_rng(0)
    vp = rng.standard_normal((3, 576, 768)).astype(np.float32)
    tp = rng.standard_normal((3, 768)).astype(np.float32)
    for bi, bt in ((3, 3), (1, 3), (3, 1), (1, 1)):
        for weights, cls in (("ones", open_clip_pacl), ("sigmoid", open_clip_pacl_sigmoid),
                             ("sigmoid_rope", open_clip_pacl_rope_after)):
            m = mod
            m.weight_mode, m.rope = cls.weight_mode, cls.rope
            a, b = m.pool(torch.from_numpy(vp[:bi]).cuda(), torch.from_numpy(tp[:bt]).cuda())
            ra, rb = O.pacl_pool(vp[:bi], tp[:bt], weights="ones" if weights == "ones" else "sigmoid",
                                 rope_after=weights == "sigmoid_rope")
            np.testing.assert_allclose(a.cpu().numpy(), ra, atol=2e-5)
            np.testing.assert_allclose(b.cpu().numpy(), rb, atol=2e-6)
    mod.weight_mode, mod.rope = open_clip_pacl_sigmoid.weight_mode, open_clip_pacl_sigmoid.rope


@pytest.mark.parametrize("B,P,D,bf16", [(64, 576, 768, True), (5, 40, 1024, False), (2, 17, 128, True),
                                         (512, 576, 768, True)])
def test_pacl_pool_splits_vs_oracle(pacl_models, B, P, D, bf16):
    """The two-pass pooling (pacl.py:120-145) at shapes that exercise its patch splits: many
    splits per row (B = 64: 36 splits of 16 patches), ragged splits (P = 40, 17), D = 1024 and
    D = 128 (partial 16-B chunk rounds), f32 and bf16 inputs, the C3 batch (B = 512, 8 splits),
    and the Q6 broadcasts; vs the oracle on the same (bf16-rounded) values."""
    mod = pacl_models["pacl_sigmoid"]
    rng = np.random.default_rng(B + P + D)
    vp = torch.from_numpy(rng.standard_normal((B, P, D)).astype(np.float32))
    if bf16:
        vp = vp.to(torch.bfloat16)
    vpf = vp.float().numpy()
    tp = rng.standard_normal((B, D)).astype(np.float32)
    modes = [("ones", open_clip_pacl), ("sigmoid", open_clip_pacl_sigmoid)]
    if P == 576 and D == 768:
        modes.append(("sigmoid_rope", open_clip_pacl_rope_after))
    try:
        for bi, bt in ((B, B), (1, B), (B, 1)) if B <= 64 else ((B, B),):
            for weights, cls in modes:
                mod.weight_mode, mod.rope = cls.weight_mode, cls.rope
                a, b = mod.pool(vp[:bi].cuda(), torch.from_numpy(tp[:bt]).cuda())
                ra, rb = O.pacl_pool(vpf[:bi], tp[:bt], weights="ones" if weights == "ones" else "sigmoid",
                                     rope_after=weights == "sigmoid_rope")
                np.testing.assert_allclose(a.cpu().numpy(), ra, atol=2e-5, err_msg=f"{weights} {bi}x{bt}")
                np.testing.assert_allclose(b.cpu().numpy(), rb, atol=2e-6)
    finally:
        mod.weight_mode, mod.rope = open_clip_pacl_sigmoid.weight_mode, open_clip_pacl_sigmoid.rope


def test_apply_rope_vs_golden(pacl_models, golden):
    eng = pacl_models["pacl"].engine
    x = W.uniform("rope-input", 2 * 576 * 128).reshape(2, 576, 128)
    # the engine's tables cover D = 1024 (vision) and 768 (PACL); compare at D = 1024 vs the oracle
    x1024 = W.uniform("rope-1024", 576 * 1024).reshape(1, 576, 1024)
    y = apply_rope(torch.from_numpy(x1024).cuda(), engine=eng).cpu().numpy()
    np.testing.assert_allclose(y, O.apply_rope(x1024), atol=1e-4)
    assert O.apply_rope(x).shape == golden("rope")["y"].shape


@pytest.mark.parametrize("name,sigma", [("s576", 1.0 / 576), ("s625", 1.0 / 625)])
def test_sparc_vs_golden(pacl_models, golden, name, sigma):
    g = golden("sparc")
    eng = pacl_models["pacl"].engine
    v = torch.from_numpy(W.uniform("sparc-v", 2 * 576 * 64).reshape(2, 576, 64)).cuda()
    l = torch.from_numpy(W.uniform("sparc-l", 2 * 77 * 64).reshape(2, 77, 64)).cuda()
    grouped = torch.empty(2, 77, 64, device="cuda")
    lnorm = torch.empty_like(grouped)
    sim = torch.empty(2, 77, 576, device="cuda")
    from clipembed import _lib
    from clipembed.model import _ptr, _stream
    _lib.call("ce_sparc_forward", eng.h, _stream(eng.device), _ptr(v), _ptr(l), 2, 576, 77, 64, sigma,
              _ptr(grouped), _ptr(lnorm), _ptr(sim))
    np.testing.assert_allclose(grouped.cpu().numpy(), g[f"{name}_grouped"], atol=2e-5)
    np.testing.assert_allclose(lnorm.cpu().numpy(), g[f"{name}_l_norm"], atol=2e-6)
    np.testing.assert_allclose(sim.cpu().numpy(), np.einsum("btd,bpd->btp", l.cpu().numpy(), v.cpu().numpy()),
                               atol=1e-4)


@pytest.mark.parametrize("name,sigma", [("s576", 1.0 / 576), ("s625", 1.0 / 625)])
def test_sparc_loss_vs_golden(golden, name, sigma):
    """SparcLoss (pacl.py:516-584) through ce_sparc_loss on the reference's own (v, l_norm,
    grouped) fixture, mask = tokens <= EOT at 20 and 76; rtol 1e-5 (f32 sums of 2x77 rows)."""
    from clipembed.pacl import SparcLoss
    g = golden("sparc")
    v = torch.from_numpy(W.uniform("sparc-v", 2 * 576 * 64).reshape(2, 576, 64)).cuda()
    lt = torch.from_numpy(g[f"{name}_l_norm"]).cuda()
    gr = torch.from_numpy(g[f"{name}_grouped"]).cuda()
    mask = torch.from_numpy((np.arange(77)[None, :] <= np.array([[20], [76]])).astype(np.float32)).cuda()
    loss = SparcLoss(0.1)(v, lt, gr, mask)
    np.testing.assert_allclose(float(loss), float(g[f"{name}_sparc_loss"]), rtol=1e-5)


def test_sparc_loss_vs_oracle_ragged():
    """Larger batch with ragged masks (one sample with only SOT+EOT valid) and non-default
    weights/temperature vs the oracle restatement."""
    from clipembed.pacl import SparcLoss
    B, P, T, D = 6, 576, 77, 96
    v = W.uniform("sl-v", B * P * D).reshape(B, P, D)
    lt = O.l2normalize(W.uniform("sl-l", B * T * D).reshape(B, T, D))
    gr = O.l2normalize(W.uniform("sl-g", B * T * D).reshape(B, T, D))
    eot = np.array([1, 5, 20, 40, 76, 33])
    mask = (np.arange(T)[None, :] <= eot[:, None]).astype(np.float32)
    fn = SparcLoss(0.07)
    fn.global_weight, fn.local_weight = 0.3, 0.7
    got = float(fn(*(torch.from_numpy(x).cuda() for x in (v, lt, gr, mask))))
    s = 1.0 / 0.07
    gi, gt = O.l2normalize(v.mean(1)), O.l2normalize(lt.mean(1))
    lab = np.arange(B)
    glob = (O.cross_entropy(s * gi @ gt.T, lab) + O.cross_entropy(s * gt @ gi.T, lab)) / 2
    local = (O.sparc_masked_pairwise_loss(gr, lt, mask, s) + O.sparc_masked_pairwise_loss(lt, gr, mask, s)) / 2
    np.testing.assert_allclose(got, 0.3 * glob + 0.7 * local, rtol=2e-5)


def test_pacl_clip_loss_mirror(golden):
    """pacl.py ClipLoss(temperature) mirror on a weightless kernel handle."""
    from clipembed.pacl import ClipLoss as PaclClipLoss
    g = golden("loss")
    a = torch.from_numpy(O.l2normalize(W.uniform("loss-a", 8 * 768).reshape(8, 768))).cuda()
    b = torch.from_numpy(O.l2normalize(W.uniform("loss-b", 8 * 768).reshape(8, 768))).cuda()
    np.testing.assert_allclose(float(PaclClipLoss(0.1)(a, b)), float(g["pacl_clip_loss"]), rtol=1e-5)


def test_logits_and_cross_entropy(small, golden):
    from clipembed.loss import ClipLoss
    g = golden("loss")
    a = torch.from_numpy(O.l2normalize(W.uniform("loss-a", 8 * 768).reshape(8, 768))).cuda()
    b = torch.from_numpy(O.l2normalize(W.uniform("loss-b", 8 * 768).reshape(8, 768))).cuda()
    fn = ClipLoss(engine=small.engine)
    np.testing.assert_allclose(float(fn(a, b, 10.0)), float(g["pacl_clip_loss"]), rtol=1e-5)
    np.testing.assert_allclose(float(fn(a, b, 14.2857)), float(g["openclip_single"]), rtol=1e-5)
    il, tl = small.logits(a, b, 100.0)
    ref = 100.0 * a.cpu().numpy() @ b.cpu().numpy().T
    np.testing.assert_allclose(il.cpu().numpy(), ref, atol=1e-4)
    np.testing.assert_allclose(tl.cpu().numpy(), ref.T, atol=1e-4)
    # labels: -100 is ignored; a label outside [0, C) (F.cross_entropy raises) poisons the loss
    logits = il.contiguous()
    lab = torch.arange(8, device="cuda")
    lab[3] = -100
    ref_ce = torch.nn.functional.cross_entropy(logits.cpu(), lab.cpu(), ignore_index=-100)
    np.testing.assert_allclose(float(fn._ce(logits, lab)), float(ref_ce), rtol=1e-5)
    for bad in (8, 1 << 40, -1):
        lab2 = torch.arange(8, device="cuda")
        lab2[5] = bad
        assert np.isnan(float(fn._ce(logits, lab2)))


def test_error_behaviour(small):
    with pytest.raises(ClipEmbedError, match="context length"):
        from clipembed import _lib
        from clipembed.model import _ptr, _stream
        ids = torch.zeros(2, 76, dtype=torch.int64, device="cuda")
        out = torch.empty(2, 768, device="cuda")
        _lib.call("ce_encode_text", small.engine.h, _stream(small.engine.device), _ptr(ids), 2, 76, 0, _ptr(out),
                  None, 0)
    with pytest.raises(RuntimeError, match="encode_image expects"):
        small.encode_image(torch.zeros(1, 3, 224, 224))
    empty = clipembed.CLIP(small.cfg).to("cuda")
    with pytest.raises(ClipEmbedError, match="has not been loaded"):
        empty.encode_image(torch.zeros(1, 3, 336, 336))
