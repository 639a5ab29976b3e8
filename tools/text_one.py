"""The text leg of bench.py on its own (for rocprofv3 --kernel-trace --stats): N token rows of
30-50 tokens through the CLIP text tower (random-init weights), REPS times.

    python tools/text_one.py [N (default 42000)] [REPS (default 3)] [--full-ctx]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import reidmi_boot  # noqa: E402

reidmi_boot.load()
from multimodal_reid_amd import synthetic as syn  # noqa: E402
from multimodal_reid_amd.model import TextTransformer  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 42000
    reps = int(args[1]) if len(args) > 1 else 3
    tm = TextTransformer(syn.text_state_dict(seed=0), device=torch.device("cuda"))
    tm.trim_context = "--full-ctx" not in sys.argv
    tokens = torch.from_numpy(syn.token_ids(n, seed=5, min_len=30, max_len=50)).cuda()
    tm.encode_text(tokens)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        tm.encode_text(tokens)
    torch.cuda.synchronize()
    s = (time.perf_counter() - t) / reps
    print(f"text tower {n} rows, ctx_used {tm.ctx_used(tokens)}: {s * 1e3:.1f} ms  {n / s:.0f} rows/s")


if __name__ == "__main__":
    main()
