"""Throughput of the NegCLIP training step (BASELINE configs[3] per GPU: 1024 image-text pairs +
hard-negative captions, locked image tower, text tower trained with AdamW), one process per GPU.

    python tools/bench_train.py [--batch 1024] [--hard 512] [--steps 3] [--warmup 1]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_train.py

Prints one JSON line (rank 0): pairs/s over all ranks, ms/step, and the per-kernel breakdown of
one profiled step (engine HIP-event timing) on stderr.  Synthetic inputs, random-init weights.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "clip-embeds_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--hard", type=int, default=512, help="hard-negative captions per GPU")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    import clipembed
    from clipembed import weights as W
    cfg = clipembed.get_model_config("ViT-L-14-336")
    m = clipembed.CLIP(cfg)
    m.load_state_dict(W.synthetic_state_dict(cfg))
    m.to(dev)
    tr = clipembed.TextTowerTrainer(m, lr=5e-6, usehardtext=args.hard > 0, rank=rank, world_size=world)
    B = args.batch
    imgs = torch.from_numpy(W.synthetic_images(B, seed=1000 + rank)).to(dev)
    caps = torch.from_numpy(W.synthetic_captions(B + args.hard, seed=2000 + rank)).to(dev)
    for _ in range(args.warmup):
        tr.step(imgs, caps)
    torch.cuda.synchronize()
    m.engine.set_timing(True)
    tr.step(imgs, caps)
    torch.cuda.synchronize()
    prof = sorted(m.engine.kernel_stats(), key=lambda s: -s["ms"])
    m.engine.set_timing(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = [tr.step(imgs, caps) for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t)
    if rank == 0:
        tot = sum(s["ms"] for s in prof)
        for s in prof[:25]:
            print(f"  {s['name']:<16} {s['ms']:9.3f} ms  {100 * s['ms'] / tot:5.1f}%  {s['launches']:4d} launches  "
                  f"{(s['flops'] / max(s['ms'], 1e-9)) / 1e9:8.1f} TFLOP/s", file=sys.stderr)
        print(json.dumps({"metric": "NegCLIP training step (locked image tower), image-text pairs/s",
                          "value": round(world * B * args.steps / el, 2), "unit": "pairs/s", "n_gpus": world,
                          "ms_per_step": round(1000 * el / args.steps, 2), "batch_per_gpu": B,
                          "hard_negatives_per_gpu": args.hard, "losses": [round(x, 5) for x in losses],
                          "dtype": "bf16 GEMMs, f32 master weights", "data": "synthetic"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
