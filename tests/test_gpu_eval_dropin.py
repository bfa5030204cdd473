"""The evaluation drivers' scoring flow through clipembed with ONE import swapped (BASELINE
configs[0], C1): eval_clip.py:21-24 takes create_model_and_transforms(...)[1] (the training
RandomResizedCrop transform) into prepare_data_clip and scores What'sUp items (:49-65) and MMVP
pairs (:296-331); eval_pacl.py:49-57 scores the PACL head with prepare_data.  Decisions are checked
against the reference's own f32 CPU run on the same items (tests/golden/eval_decisions.npz, made
by tests/golden/make_golden_eval.py).

Decision margins (logit units: 100 x cosine difference, or log-odds) are reported.  A decision
must match the reference unless the reference margin is inside the numerical tie band TIE, and
every margin must agree with the reference's within MARGIN_TOL (the bf16 engine vs the f32
reference: features within 1e-3 cosine distance move a 100-scaled logit by well under this).
40 items (20 MMVP pairs = 40 MMVP decisions): at least MIN_ASSERTED decisions of every kind lie
outside the tie band and are asserted identical.

The tie band is derived from the measured margin error: TIE = max(TIE_FLOOR, 3 x max |engine margin -
reference margin|) over that kind's decisions (capped at 2 x MARGIN_TOL).  With random-init weights two
gradient test images embed almost alike, so most MMVP margins of the gradient pairs are below 0.2; the
`mmvp2` pairs (a gradient image against a single-colour one, make_golden_eval.py) give margins of
0.1-5.6, and at least MIN_ASSERTED_MMVP2 of their 40 decisions must be asserted identical."""
import importlib.util
import os

import numpy as np
import pytest
import torch

import clipembed
from clipembed import weights as W

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location("mgp", os.path.join(HERE, "golden", "make_golden_preprocess.py"))
mgp = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mgp)
_spec2 = importlib.util.spec_from_file_location("mge", os.path.join(HERE, "golden", "make_golden_eval.py"))

MARGIN_TOL = 0.1
TIE_FLOOR = 0.02
MIN_ASSERTED = 8
MIN_ASSERTED_MMVP2 = 30


def _items():
    # the item table of the generator (parsed without importing it: its imports need the reference)
    src = open(os.path.join(HERE, "golden", "make_golden_eval.py")).read()
    start = src.index("ITEMS = [")
    end = src.index("]\n", start) + 1
    ns = {}
    exec(src[start:end], ns)
    return ns["ITEMS"]


ITEMS = _items()


def pil(k):
    from PIL import Image
    i, h, w = ITEMS[k][:3]
    return Image.fromarray(mgp.image(i, h, w))


@pytest.fixture(scope="module")
def drop_in():
    """`model, image_processor, _ = oc.create_model_and_transforms(...)` with oc = clipembed."""
    cfg = clipembed.get_model_config("ViT-L-14-336")
    model, image_processor, _ = clipembed.create_model_and_transforms("ViT-L-14-336")
    model.load_state_dict(W.synthetic_state_dict(cfg))
    model.to(torch.device("cuda:0"))
    model.eval()
    return model, image_processor


def _check(name, got_margin, ref_margin, got_dec, ref_dec, min_asserted=MIN_ASSERTED):
    got_margin, ref_margin = np.asarray(got_margin, np.float64), np.asarray(ref_margin, np.float64)
    d = np.abs(got_margin - ref_margin)
    tie = min(2 * MARGIN_TOL, max(TIE_FLOOR, 3.0 * float(d.max())))
    ties = np.abs(ref_margin) < tie
    print(f"{name}: ref margins {np.round(ref_margin, 3).tolist()}, engine {np.round(got_margin, 3).tolist()}, "
          f"max |diff| {d.max():.4f}, tie band {tie:.4f}, ties {int(ties.sum())}")
    assert d.max() < MARGIN_TOL, f"{name}: margin differs by {d.max()}"
    got_dec, ref_dec = np.asarray(got_dec), np.asarray(ref_dec)
    assert int((~ties).sum()) >= min_asserted, f"{name}: only {int((~ties).sum())} decisions outside the tie band"
    assert np.array_equal(got_dec[~ties], ref_dec[~ties]), f"{name}: decisions {got_dec} vs {ref_dec}"
    print(f"{name}: {int((~ties).sum())} decisions asserted identical, "
          f"{int((got_dec == ref_dec).sum())}/{got_dec.size} identical overall")
    return int((got_dec == ref_dec).sum()), got_dec.size


def test_eval_clip_whatsup_and_mmvp(drop_in, golden):
    g = golden("eval_decisions")
    model, image_processor = drop_in
    process = clipembed.prepare_data_clip(image_processor)          # eval_clip.py:24
    device = torch.device("cuda:0")
    # What'sUp (eval_clip.py:49-65)
    torch.manual_seed(1234)
    margins, correct = [], []
    for k in range(len(ITEMS)):
        input_pixels = process.preprocess_image(pil(k)).unsqueeze(0).to(device)
        assert np.array_equal(image_processor.last_boxes[0], g["whatsup_boxes"][k])
        tokenized_text = torch.from_numpy(g["ids"][k]).to(device)
        with torch.no_grad():
            image_features = model.encode_image(input_pixels)
            text_features = model.encode_text(tokenized_text)
            image_features /= image_features.norm(dim=-1, keepdim=True)
            text_features /= text_features.norm(dim=-1, keepdim=True)
            text_probs = (100.0 * image_features @ text_features.T).softmax(dim=-1)
        correct.append(1 if text_probs[0][0] > text_probs[0][1] else 0)
        margins.append(float(torch.log(text_probs[0][0] / text_probs[0][1])))
    p = g["whatsup_probs"]
    same, n = _check("whatsup", margins, np.log(p[:, 0] / p[:, 1]), correct, g["whatsup_correct"])
    # MMVP t2i (eval_clip.py:296-331)
    torch.manual_seed(4321)
    margins, preds = [], []
    for j in range(len(ITEMS) // 2):
        texts = torch.from_numpy(g["mmvp_ids"][j]).to(device)
        img1 = process.preprocess_image(pil(2 * j)).unsqueeze(0).to(device)
        img2 = process.preprocess_image(pil(2 * j + 1)).unsqueeze(0).to(device)
        imgs = torch.cat((img1, img2), dim=0)
        with torch.no_grad():
            image_features = model.encode_image(imgs)
            text_features = model.encode_text(texts)
            image_features /= image_features.norm(dim=-1, keepdim=True)
            text_features /= text_features.norm(dim=-1, keepdim=True)
            text_probs = (100.0 * text_features @ image_features.T).softmax(dim=-1)
        probs1, probs2 = text_probs[0].cpu().numpy(), text_probs[1].cpu().numpy()
        preds.append([int(probs1[0] > 0.5), int(probs2[0] > 0.5)])
        margins.append([float(np.log(probs1[0] / probs1[1])), float(np.log(probs2[0] / probs2[1]))])
    m = g["mmvp_probs"]
    s2, n2 = _check("mmvp", np.ravel(margins), np.ravel(np.log(m[:, :, 0] / m[:, :, 1])), np.ravel(preds),
                    np.ravel(g["mmvp_pred_img1"]))
    # MMVP on contrasting image pairs (make_golden_eval.py mmvp2): same flow, larger margins
    torch.manual_seed(4322)
    margins, preds = [], []
    for j in range(len(ITEMS) // 2):
        texts = torch.from_numpy(g["mmvp2_ids"][j]).to(device)
        (i0, h0, w0), (i1, h1, w1) = ITEMS[2 * j][:3], ITEMS[2 * j + 1][:3]
        from PIL import Image
        a, b = (mgp.image(i0, h0, w0), mgp.solid_image(i1, h1, w1)) if j % 2 == 0 else \
               (mgp.solid_image(i0, h0, w0), mgp.image(i1, h1, w1))
        img1 = process.preprocess_image(Image.fromarray(a)).unsqueeze(0).to(device)
        assert np.array_equal(image_processor.last_boxes[0], g["mmvp2_boxes"][2 * j])
        img2 = process.preprocess_image(Image.fromarray(b)).unsqueeze(0).to(device)
        assert np.array_equal(image_processor.last_boxes[0], g["mmvp2_boxes"][2 * j + 1])
        imgs = torch.cat((img1, img2), dim=0)
        with torch.no_grad():
            image_features = model.encode_image(imgs)
            text_features = model.encode_text(texts)
            image_features /= image_features.norm(dim=-1, keepdim=True)
            text_features /= text_features.norm(dim=-1, keepdim=True)
            text_probs = (100.0 * text_features @ image_features.T).softmax(dim=-1)
        probs1, probs2 = text_probs[0].cpu().numpy(), text_probs[1].cpu().numpy()
        preds.append([int(probs1[0] > 0.5), int(probs2[0] > 0.5)])
        margins.append([float(np.log(probs1[0] / probs1[1])), float(np.log(probs2[0] / probs2[1]))])
    m2 = g["mmvp2_probs"]
    s3, n3 = _check("mmvp2", np.ravel(margins), np.ravel(np.log(m2[:, :, 0] / m2[:, :, 1])), np.ravel(preds),
                    np.ravel(g["mmvp2_pred_img1"]), MIN_ASSERTED_MMVP2)
    print(f"identical decisions: whatsup {same}/{n}, mmvp {s2}/{n2}, mmvp2 {s3}/{n3}")


def test_eval_pacl_whatsup(golden):
    from clipembed.pacl import open_clip_pacl
    g = golden("eval_decisions")
    cfg = clipembed.get_model_config("ViT-L-14-336")
    model = open_clip_pacl("ViT-L-14-336", clip_state_dict=W.synthetic_state_dict(cfg))
    model.load_state_dict(W.synthetic_pacl_heads(cfg.with_pacl(768)))
    device = torch.device("cuda:0")
    model.to(device)
    process = clipembed.prepare_data(base_model="ViT-L-14-336")     # eval_pacl.py:19
    margins, correct = [], []
    for k in range(len(ITEMS)):
        input_pixels = process.preprocess_image(pil(k)).unsqueeze(0).to(device)
        tokenized_text = torch.from_numpy(g["ids"][k]).to(device)
        with torch.no_grad():
            image_features, text_features = model(input_pixels, tokenized_text)
            text_probs = 100.0 * image_features @ text_features.T
            correct.append(1 if text_probs[0][0] > text_probs[1][1] else 0)
        margins.append(float(text_probs[0][0] - text_probs[1][1]))
    s = g["pacl_scores"]
    same, n = _check("pacl", margins, s[:, 0, 0] - s[:, 1, 1], correct, g["pacl_correct"])
    print(f"identical decisions: pacl {same}/{n}")


@pytest.mark.parametrize("tag", ["sparc", "sparc_rope"])
def test_eval_sparc_whatsup(golden, tag):
    """eval_sparc.py:26-56: prepare_data's PACL transform, model.scoring(1 image, 2 captions, local) for
    local False and True, correct = s[0][0] > s[1][1]; against the reference's full-depth f32 run
    (tests/golden/eval_sparc_decisions.npz, make_golden_eval.py sparc).  Margins in 100 x cosine units."""
    from clipembed.pacl import sparc, sparc_rope
    g = golden("eval_sparc_decisions")
    cfg = clipembed.get_model_config("ViT-L-14-336")
    cls = sparc_rope if tag == "sparc_rope" else sparc
    model = cls(sigma=1.0 / 576, cfg=cfg, clip_state_dict=W.synthetic_state_dict(cfg))
    model.load_state_dict(W.synthetic_pacl_heads(cfg.with_pacl(768)))
    device = torch.device("cuda:0")
    model.to(device)
    process = clipembed.prepare_data(base_model="ViT-L-14-336")
    for local in (False, True):
        margins, correct = [], []
        for k in range(len(ITEMS)):
            input_pixels = process.preprocess_image(pil(k)).unsqueeze(0).to(device)
            tokenized_text = torch.from_numpy(g["ids"][k]).to(device)
            with torch.no_grad():
                s = model.scoring(input_pixels, tokenized_text, local=local)
            correct.append(1 if s[0][0] > s[1][1] else 0)
            margins.append(100.0 * float(s[0][0] - s[1][1]))
        key = f"{tag}_{'local' if local else 'global'}"
        ref = g[f"{key}_scores"]
        same, n = _check(key, margins, 100.0 * (ref[:, 0, 0] - ref[:, 1, 1]), correct, g[f"{key}_correct"])
        print(f"identical decisions: {key} {same}/{n}")


@pytest.mark.parametrize("tag", ["pacl_rope", "pacl_rope_after"])
def test_eval_pacl_variants_whatsup(golden, tag):
    """eval_pacl.py:49-57 with the RoPE variants its model path selects (eval_pacl.py:372-377), against
    the reference's full-depth run (tests/golden/eval_pacl_variants.npz, make_golden_eval.py pacl)."""
    from clipembed.pacl import open_clip_pacl_rope, open_clip_pacl_rope_after
    g = golden("eval_pacl_variants")
    cfg = clipembed.get_model_config("ViT-L-14-336")
    cls = open_clip_pacl_rope if tag == "pacl_rope" else open_clip_pacl_rope_after
    model = cls("ViT-L-14-336", clip_state_dict=W.synthetic_state_dict(cfg))
    model.load_state_dict(W.synthetic_pacl_heads(cfg.with_pacl(768)))
    device = torch.device("cuda:0")
    model.to(device)
    process = clipembed.prepare_data(base_model="ViT-L-14-336")
    margins, correct = [], []
    for k in range(len(ITEMS)):
        input_pixels = process.preprocess_image(pil(k)).unsqueeze(0).to(device)
        tokenized_text = torch.from_numpy(g["ids"][k]).to(device)
        with torch.no_grad():
            image_features, text_features = model(input_pixels, tokenized_text)
            text_probs = 100.0 * image_features @ text_features.T
        correct.append(1 if text_probs[0][0] > text_probs[1][1] else 0)
        margins.append(float(text_probs[0][0] - text_probs[1][1]))
    s = g[f"{tag}_scores"]
    same, n = _check(tag, margins, s[:, 0, 0] - s[:, 1, 1], correct, g[f"{tag}_correct"])
    print(f"identical decisions: {tag} {same}/{n}")
