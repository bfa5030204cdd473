"""Diagnostic: which q-blocks the dynamic persistent attention (variant 4989) leaves unwritten or wrong."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO, os.path.join(REPO, "tests")]
import torch  # noqa: E402
from clipembed import _lib  # noqa: E402
from test_gpu_kernels import attn_ref  # noqa: E402

for (B, L, H) in ((32, 577, 16), (3, 577, 4)):
    g = torch.Generator(device="cpu").manual_seed(1)
    qkv = torch.randn(B * L, 3 * H * 64, generator=g).to(torch.bfloat16).cuda()
    ref = attn_ref(qkv, B, L, H, False)
    lib = _lib.lib()
    prev = lib.ce_set_attn_variant(4989)
    for rep in range(3):
        out = torch.full((B * L, H * 64), float("nan"), device="cuda", dtype=torch.bfloat16)
        _lib.call("ce_kernel_attention", ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                  ctypes.c_void_p(qkv.data_ptr()), ctypes.c_void_p(out.data_ptr()), B, L, H, 0)
        torch.cuda.synchronize()
        o = out.float().view(B, L, H, 64)
        r = ref.view(B, L, H, 64)
        nan_rows = torch.isnan(o).any(-1)             # [B, L, H]
        bad = ((o - r).abs().amax(-1) > 0.05) & ~nan_rows
        nqb = (L + 127) // 128
        blk_nan = nan_rows.view(B, L, H).permute(0, 2, 1)    # [B, H, L]
        nb = []
        for qb in range(nqb):
            nb.append(int(blk_nan[:, :, qb * 128:(qb + 1) * 128].any(-1).sum()))
        print(f"B={B} L={L} H={H} rep {rep}: unwritten rows {int(nan_rows.sum())}, wrong rows {int(bad.sum())}, "
              f"blocks with unwritten rows per qb {nb}")
    lib.ce_set_attn_variant(prev)
