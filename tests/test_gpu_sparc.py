"""SPARC at real dimensions (D = 768, T = 77, P = 576) through clipembed.pacl.sparc / sparc_rope
(pacl.py:380-484) against the reference's own outputs (tests/golden/sparc_full.npz, made by
tests/golden/make_golden_sparc.py with 1-block towers), plus the precomputed-text-embedding path
(sparc.align, the train_sparc.py input) and SparcLoss at the C5 batch.

Tolerances: the towers run in bf16 (1e-3 cosine distance on embeddings, north_star); the SPARC
arithmetic after them runs in f32 on the matrix cores (exact f32 products) — checked separately
against the f32 oracle on identical inputs (1e-4 on the grouped rows, 1e-6 on the
normalised tokens)."""
import numpy as np
import pytest
import torch

from clipembed import weights as W
from clipembed.config import get_model_config
from clipembed.pacl import SparcLoss, sparc, sparc_rope
from oracle import clip_oracle as O

pytestmark = pytest.mark.gpu
ROWS_T = [0, 1, 5, 9, 20, 40, 76]
ROWS_P = [0, 1, 23, 24, 287, 300, 550, 575]
COS_TOL = 1e-3


def cos_dist(a, b):
    a = np.asarray(a, np.float64).reshape(-1, a.shape[-1])
    b = np.asarray(b, np.float64).reshape(-1, b.shape[-1])
    c = (a * b).sum(-1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
    return float((1 - c).max())


@pytest.fixture(scope="module")
def models():
    cfg = get_model_config("ViT-L-14-336").with_depth(1, 1)
    sd = W.synthetic_state_dict(cfg)
    heads = W.synthetic_pacl_heads(cfg.with_pacl(768))
    out = {}
    for tag, cls in (("sparc", sparc), ("sparc_rope", sparc_rope)):
        m = cls(sigma=1.0 / 576, cfg=cfg, clip_state_dict=sd)
        m.load_state_dict(heads)
        m.to("cuda")
        out[tag] = m
    return out


@pytest.mark.parametrize("tag", ["sparc", "sparc_rope"])
def test_sparc_forward_scoring_vs_reference(models, golden, tag):
    g = golden("sparc_full")
    m = models[tag]
    imgs = torch.from_numpy(W.synthetic_images(2, seed=1300)).cuda()
    caps = torch.from_numpy(g["captions"]).cuda()
    v, l, gr, mask = m(imgs, caps)
    v, l, gr = v.cpu().numpy(), l.cpu().numpy(), gr.cpu().numpy()
    assert cos_dist(v[:, ROWS_P], g[f"{tag}_v_rows"]) < COS_TOL
    assert cos_dist(l[:, ROWS_T], g[f"{tag}_l_rows"]) < COS_TOL
    assert cos_dist(gr[:, ROWS_T], g[f"{tag}_g_rows"]) < COS_TOL
    np.testing.assert_array_equal(mask.cpu().numpy(), g[f"{tag}_mask"])
    for mode in ("local", "global"):
        s = m.scoring(imgs, caps, local=mode == "local").cpu().numpy()
        np.testing.assert_allclose(s, g[f"{tag}_score_{mode}"], atol=2e-3)
        assert (s.argmax(1) == g[f"{tag}_score_{mode}"].argmax(1)).all()
    sb = m.scoring(imgs[:1], caps, local=True).cpu().numpy()        # 1 image x 2 captions
    np.testing.assert_allclose(sb, g[f"{tag}_score_bcast"], atol=2e-3)
    loss = SparcLoss(0.07, engine=m.engine)(torch.from_numpy(v).cuda(), torch.from_numpy(l).cuda(),
                                            torch.from_numpy(gr).cuda(), mask)
    np.testing.assert_allclose(float(loss), float(g[f"{tag}_loss"]), rtol=2e-3)


def test_sparc_align_precomputed_embeddings_vs_oracle(models):
    """sparc.align (similarity -> min-max -> threshold -> weights -> grouping -> L2; pacl.py:455-476)
    on given f32 embeddings at the C5 shape per sample, B = 64: f32 matrix-core GEMMs vs the f32
    oracle; SparcLoss on them vs the oracle."""
    m = models["sparc"]
    rng = np.random.default_rng(4)
    B, T, P, D = 64, 77, 576, 768
    v = (rng.standard_normal((B, P, D)) * 0.5).astype(np.float32)
    l = (rng.standard_normal((B, T, D)) * 0.5).astype(np.float32)
    gr, ln = m.align(torch.from_numpy(v).cuda(), torch.from_numpy(l).cuda())
    rg, rl, _ = O.sparc_forward(v, l, 1.0 / 576)
    # (a similarity within an f32 rounding of the threshold may land on the other side: 1e-4)
    np.testing.assert_allclose(gr.cpu().numpy(), rg, atol=1e-4)
    np.testing.assert_allclose(ln.cpu().numpy(), rl, atol=1e-6)
    eot = rng.integers(6, 42, B)
    mask = (np.arange(T)[None, :] <= eot[:, None]).astype(np.float32)
    loss = SparcLoss(0.07, engine=m.engine)(torch.from_numpy(v).cuda(), ln, gr, torch.from_numpy(mask).cuda())
    np.testing.assert_allclose(float(loss), O.sparc_loss(v, rl, rg, mask, 0.07), rtol=1e-4)


@pytest.mark.parametrize("B,T,P,D", [(64, 77, 576, 768), (3, 5, 40, 128), (2, 77, 576, 1024)])
def test_fgemm_variants_agree(models, B, T, P, D):
    """The register-blocked 96 x 128 f32 GEMM (the default for SPARC's similarity and grouping
    einsums, pacl.py:460,472) and the selectable short-M 80 x 192 kernel (v_mfma_f32_16x16x4_f32,
    ce_set_fgemm_variant(2), measured slower: DESIGN §6.11) vs the 64 x 64 kernel, on the same inputs,
    and vs the oracle; ragged M / N / K tiles and D = 1024."""
    from clipembed import _lib
    m = models["sparc"]
    rng = np.random.default_rng(B * 7 + D)
    v = torch.from_numpy((rng.standard_normal((B, P, D)) * 0.5).astype(np.float32)).cuda()
    l = torch.from_numpy((rng.standard_normal((B, T, D)) * 0.5).astype(np.float32)).cuda()
    res = {}
    for var in (2, 1, 0):
        prev = _lib.lib().ce_set_fgemm_variant(var)
        try:
            gr, ln = m.align(v, l)
            torch.cuda.synchronize()
        finally:
            _lib.lib().ce_set_fgemm_variant(prev)
        res[var] = (gr.cpu().numpy(), ln.cpu().numpy())
    # (a similarity within an f32 rounding of the threshold may land on the other side: 1e-4)
    for var in (2, 1):
        np.testing.assert_allclose(res[var][0], res[0][0], atol=1e-4)
        np.testing.assert_allclose(res[var][1], res[0][1], atol=1e-7)
    rg, rl, _ = O.sparc_forward(v.cpu().numpy(), l.cpu().numpy(), 1.0 / 576)
    for var in (2, 1):
        np.testing.assert_allclose(res[var][0], rg, atol=1e-4)
