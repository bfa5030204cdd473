"""The NegCLIP text-tower step at the C4 per-GPU workload (BASELINE configs[3]; exactly what
`bench.py --workload negclip` times): full-depth ViT-L-14-336, 1,024 images + 512 hard-negative
captions per GPU, so the text tower runs M = 1,536 x 77 = 118,272 rows through 12 blocks.

At that size the GEMM policy picks paths the toy-size test (tests/test_gpu_train.py, M = 462)
never reaches: the four-wave persistent kernel for the forward QKV / c_fc GEMMs and every dX GEMM,
and the MN-major weight-gradient GEMM (gemm_tn.hip: dW_* over K = 118,272 token rows, split-K over
9-36 tiles) in place of transposed copies + the forward GEMM.  The test asserts those paths fired
(ce_gemm_path_counts) and checks the step against
  * the same step on the plain path (ce_set_gemm_auto(0) + ce_set_gemm_splitk(0) +
    ce_set_train_dw_tn(0): the 4-phase kernel only, no split-K, dW on transposed copies): loss and
    every gradient tensor, cosine >= 0.9999;
  * the reference's f32 autograd of the same step (oracle/text_train_torch.py, pinned to the
    reference's own training step in tests/test_oracle_train.py), run here in f32 on the GPU:
    every gradient tensor cosine >= 0.995 and norm within 3 %, loss within 5e-3 (the engine's
    GEMMs are bf16 with f32 accumulation, standing in for the reference's --precision amp).
Reference: open_clip_train/train.py:85-112, open_clip/src/open_clip/loss.py:67-193."""
import ctypes
import math

import numpy as np
import pytest
import torch

import clipembed
from clipembed import _lib, weights as W
from clipembed.config import get_model_config
from clipembed.train import TextTowerTrainer

pytestmark = pytest.mark.gpu

B_IMG, K_HARD = 1024, 512
# ce_gemm_path_counts indices (include/clipembed.h): path + epilogue (0 = plain)
W4PP, NT, FIXUP = 0, 3, 6


def path_counts(reset=True):
    c = (ctypes.c_int64 * 13)()
    _lib.call("ce_gemm_path_counts", c, 13, 1 if reset else 0)
    return list(c)


def _cos(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return float((a * b).sum() / (a.norm() * b.norm() + 1e-30))


@pytest.fixture(scope="module")
def c4():
    cfg = get_model_config("ViT-L-14-336")
    m = clipembed.CLIP(cfg)
    m.load_state_dict(W.synthetic_state_dict(cfg))
    m.to("cuda")
    tr = TextTowerTrainer(m, lr=5e-6, usehardtext=True)
    imgs = torch.from_numpy(W.synthetic_images(B_IMG, seed=1000)).cuda()
    caps = torch.from_numpy(W.synthetic_captions(B_IMG + K_HARD, seed=2000)).cuda()
    img = m.encode_image(imgs, normalize=True)
    del imgs
    torch.cuda.synchronize()

    def run():
        tr.grad.fill_(float("nan"))           # every gradient slot must be written by the step
        loss = float(tr.compute_grads_from_features(img, caps))
        torch.cuda.synchronize()
        return loss, tr.grad.clone()

    path_counts()
    loss_big, g_big = run()
    cnt_big = path_counts()
    L = _lib.lib()
    pa, ps, pt = L.ce_set_gemm_auto(0), L.ce_set_gemm_splitk(0), L.ce_set_train_dw_tn(0)
    try:
        path_counts()
        loss_plain, g_plain = run()
        cnt_plain = path_counts()
    finally:
        L.ce_set_gemm_auto(pa)
        L.ce_set_gemm_splitk(ps)
        L.ce_set_train_dw_tn(pt)
    pf = L.ce_set_train_act_bwd_fuse(0)
    try:
        loss_unfused, g_unfused = run()
    finally:
        L.ce_set_train_act_bwd_fuse(pf)
    return dict(m=m, tr=tr, img=img, caps=caps, loss_big=loss_big, g_big=g_big, cnt_big=cnt_big,
                loss_plain=loss_plain, g_plain=g_plain, cnt_plain=cnt_plain, loss_unfused=loss_unfused,
                g_unfused=g_unfused)


def _views(tr, flat):
    out = {}
    for n, v in tr.gviews.items():
        off = (v.data_ptr() - tr.grad.data_ptr()) // 4
        out[n] = flat[off:off + v.numel()].view(v.shape)
    out["logit_scale"] = flat[-1:]
    return out


def test_big_grid_paths_fire(c4):
    """Per text block: QKV, c_fc and the four dX GEMMs on the four-wave persistent kernel;
    out-proj / c_proj (residual epilogue) on the 4-phase kernel; the four dW GEMMs on the MN-major
    kernel (not counted by ce_gemm_path_counts).  The plain run uses neither the persistent kernel
    nor split-K, and its dW GEMMs run on the 4-phase kernel over transposed copies."""
    nl = 12
    cnt = c4["cnt_big"]
    assert cnt[W4PP] == 6 * nl, cnt
    assert cnt[FIXUP] == 0, cnt
    assert cnt[NT] == 2 * nl, cnt
    assert sum(cnt) == 8 * nl, cnt
    cp = c4["cnt_plain"]
    assert cp[W4PP] == 0 and cp[FIXUP] == 0 and cp[NT] == 12 * nl and sum(cp) == 12 * nl, cp


def test_gradients_finite_and_paths_agree(c4):
    """Big-grid paths vs the plain path: the same step up to f32 summation order (and the bf16
    rounding of intermediate gradients that order can flip)."""
    assert math.isfinite(c4["loss_big"])
    assert abs(c4["loss_big"] - c4["loss_plain"]) <= 1e-4 * abs(c4["loss_plain"])
    assert torch.isfinite(c4["g_big"]).all() and torch.isfinite(c4["g_plain"]).all()
    vb, vp = _views(c4["tr"], c4["g_big"]), _views(c4["tr"], c4["g_plain"])
    bad = []
    for n in vb:
        if vp[n].abs().max() == 0:
            assert vb[n].abs().max() == 0, n
            continue
        c = _cos(vb[n], vp[n])
        if c < 0.9999:
            bad.append((n, round(c, 6)))
    assert not bad, bad


def test_matches_f32_autograd_restatement(c4):
    """The engine's gradients at the C4 size vs the reference's f32 autograd of the same step."""
    from oracle.text_train_torch import TorchTextTrainStep
    m, tr = c4["m"], c4["tr"]
    ref_step = TorchTextTrainStep(m._sd, m.cfg, device="cuda")
    loss_ref, g_ref = ref_step.loss_and_grads(c4["img"], c4["caps"], float(tr.logit_scale))
    del ref_step
    np.testing.assert_allclose(c4["loss_big"], loss_ref, rtol=5e-3)
    ours = _views(tr, c4["g_big"])
    bad = []
    for n, r in g_ref.items():
        o = ours[n].reshape(r.shape)
        c = _cos(o, r)
        nr = float(o.double().norm() / (r.double().norm() + 1e-30))
        if not (c >= 0.995 and abs(nr - 1) < 0.03):
            bad.append((n, round(c, 5), round(nr, 4)))
    assert not bad, bad


def test_act_backward_fused_matches_separate_kernel(c4):
    """The activation backward in the dX_proj GEMM's epilogue (launch_gemm_act_bwd) vs the GEMM then
    launch_act_bwd_colsum: the same bf16 dpre values, so every gradient but the c_fc biases is
    bitwise identical; the c_fc bias sums (per 128-row block + DPP reduce-scatter vs per row chunk)
    differ in f32 summation order only."""
    assert c4["loss_big"] == c4["loss_unfused"]
    vb, vu = _views(c4["tr"], c4["g_big"]), _views(c4["tr"], c4["g_unfused"])
    for n in vb:
        if n.endswith("mlp.c_fc.bias"):
            d = (vb[n] - vu[n]).abs().max().item()
            assert d <= 1e-5 * max(vu[n].abs().max().item(), 1e-12), (n, d)
        else:
            assert torch.equal(vb[n], vu[n]), n



@pytest.mark.parametrize("model", ["ViT-L-14-336", "ViT-L-14-336-quickgelu"])
def test_act_backward_fused_ragged_rows(model):
    """The fused activation backward (ACT_GELU_BWD / ACT_QGELU_BWD epilogue) at M = 1,000 x 77 = 77,000
    text rows: M % 128 = 72, so the last 128-row block of the bias column sums is partial (rows >= M
    read as zeros and must add nothing), with both activations (the C4 test above covers GELU
    at M % 256 == 0 only).  Fused vs the GEMM + launch_act_bwd_colsum path on the same step: every
    gradient but the c_fc biases bitwise equal (same bf16 dpre values), the c_fc biases within 1e-5 of
    their magnitude (f32 summation order), and the fused path actually taken (the engine's per-kernel
    tags: dX_proj_act when fused, dX_proj + t_act_bwd otherwise)."""
    cfg = get_model_config(model).with_depth(1, 2)
    m = clipembed.CLIP(cfg)
    m.load_state_dict(W.synthetic_state_dict(cfg))
    m.to("cuda")
    tr = TextTowerTrainer(m, lr=5e-6, usehardtext=True)
    g = torch.Generator(device="cpu").manual_seed(7)
    img = torch.nn.functional.normalize(torch.randn(600, cfg.embed_dim, generator=g), dim=-1).cuda()
    caps = torch.from_numpy(W.synthetic_captions(1000, seed=2100)).cuda()
    L = _lib.lib()
    outs = []
    for fuse in (1, 0):
        prev = L.ce_set_train_act_bwd_fuse(fuse)
        try:
            tr.grad.fill_(float("nan"))
            m.engine.set_timing(True)
            loss = float(tr.compute_grads_from_features(img, caps))
            torch.cuda.synchronize()
            tags = {s["name"]: s["launches"] for s in m.engine.kernel_stats()}
        finally:
            m.engine.set_timing(False)
            L.ce_set_train_act_bwd_fuse(prev)
        outs.append((loss, tr.grad.clone(), tags))
    (lf, gf, tf), (lu, gu, tu) = outs
    assert tf.get("dX_proj_act") == 2 and "dX_proj" not in tf, tf      # both blocks fused
    assert tu.get("dX_proj") == 2 and "dX_proj_act" not in tu, tu
    assert lf == lu and torch.isfinite(gf).all()
    vf, vu = _views(tr, gf), _views(tr, gu)
    for n in vf:
        if n.endswith("mlp.c_fc.bias"):
            d = (vf[n] - vu[n]).abs().max().item()
            assert d <= 1e-5 * max(vu[n].abs().max().item(), 1e-12), (n, d)
        else:
            assert torch.equal(vf[n], vu[n]), n
