"""Host-side logic of bench.py (no GPU): the FLOP accounting of the pooled-only row skipping that
the bench line reports as step_mfma_frac / model_flops_frac, and the command-line contract."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "clip-embeds_amd")]

import bench  # noqa: E402
from clipembed.config import get_model_config  # noqa: E402


def test_pooled_prune_flops_image_and_text():
    cfg = get_model_config("ViT-L-14-336")
    assert bench.pooled_prune_flops(cfg, on=False) == (0.0, 0.0)
    img, txt = bench.pooled_prune_flops(cfg, on=True)
    # last image block: 576 non-CLS rows of out-proj (2 D^2) + c_fc / c_proj (4 D F) + their
    # attention queries (4 D L per row): 12.2 GFLOP per image, 3.2 % of the 381.9 GFLOP forward
    D, F, L = 1024, 4096, 577
    assert img == 576 * (2.0 * D * D + 4.0 * D * F) + 4.0 * D * L * 576
    assert 12.0e9 < img < 12.5e9 and txt == 0.0
    # text: captions filling the context skip only the last block's non-EOT rows; shorter captions
    # skip more, never more than the whole text forward
    _, full = bench.pooled_prune_flops(cfg, True, np.full(8, 76))
    _, short = bench.pooled_prune_flops(cfg, True, np.full(8, 10))
    assert 0.0 < full < bench.TEXT_FLOPS / 12
    assert full < short < bench.TEXT_FLOPS


def test_bench_cli_contract():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    for flag in ("--gpus", "--steps", "--warmup", "--workload", "--no-pooled-prune", "--no-every-row"):
        assert flag in r.stdout
