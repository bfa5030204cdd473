"""bench.py's N > 1 code path on the one-GPU box: two ranks launched as the driver launches them
(torch.distributed.run via bench.py --gpus 2), both on cuda:0 over gloo (RCCL runs one rank per
device).  Exercises what a multi-GPU run executes besides the collectives' transport: the rank
setup, the barrier + max-over-ranks timing, the embedding all-gather and local logits (clip), the
global-batch SparcLoss / PACL ClipLoss exchange (sparc, pacl), the NegCLIP trainer's all-gathers of
features and sizes, reduce-scatter of their gradient and DDP all-reduce with the engine's text-tower
backward (negclip, BASELINE configs[3]), rank 0's single JSON line.  Not a
scaling measurement (the two ranks share one GPU)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("workload,batch", [("clip", 16), ("sparc", 8), ("pacl", 8), ("negclip", 16)])
def test_bench_two_ranks_shared_device(workload, batch):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--share-device", "--dist-backend", "gloo",
           "--workload", workload, "--batch", str(batch), "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
           "--no-every-row", "--no-timing"]
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["global_batch"] == 2 * batch
    assert "all_gather" in d["config"]["exchange"] and "gloo" in d["config"]["dist_backend"]
