"""`python bench.py --gpus 2` starts its own two ranks (bench.launch_ranks) and reports
n_gpus 2 with the same CMC/mAP as one GPU.  On a one-GPU box the two ranks share cuda:0 over
gloo (`--backend gloo`: host collectives; RCCL needs one GPU per rank), so this runs the whole
multi-rank bench path — self-launch, world-size check, sharded embed, gallery all-gather,
per-rank eval rows gathered and reduced in query order, the per-rank timing record — that the
driver's 8-GPU run takes with torchrun and nccl."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUICK = ["--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-rerank", "--no-msmt17", "--no-text",
         "--no-jpeg", "--no-backend", "--no-preprocess", "--no-files"]


def _bench(*args):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args, *QUICK], capture_output=True,
                       text=True, timeout=240, cwd=REPO,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_self_launched_equal_one(gpu):
    one = _bench("--gpus", "1")
    two = _bench("--gpus", "2", "--backend", "gloo")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["parallelism"].startswith("dp2")
    assert two["mAP"] == one["mAP"] and two["rank1"] == one["rank1"]
    rk = two["ranks"]
    assert len(rk["embed_s"]) == 2 and len(rk["allgather_s"]) == 2
    # the gathered gallery: 15913 rows x (768 + 512) fp32
    assert rk["allgather_bytes"] == 15913 * 1280 * 4


def test_bench_world_size_must_match_gpus(gpu):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", *QUICK], capture_output=True,
                       text=True, timeout=120, cwd=REPO, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=1 but --gpus 2" in r.stderr
