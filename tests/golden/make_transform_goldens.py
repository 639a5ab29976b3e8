"""Golden vectors for the test-time transform (data_prepare.py:257-261), made with the
third-party code the reference relies on for it: Pillow (PIL.Image.resize(BILINEAR), what
torchvision's Resize does to a PIL image) + ToTensor/Normalize restated in torch exactly
as torchvision computes them (uint8 -> float32 / 255, then (x - mean) / std).  torchvision
itself is absent here.  Runs only in the build container; writes tests/golden/transforms.npz.

Inputs are regenerated from (h, w, seed) by `source_image` (also used by the tests); the
fixture stores, per case, the SHA-256 of the resized uint8 image and of the normalised
float32 tensor, and the full resized images of the first few cases.

    python tests/golden/make_transform_goldens.py
"""
import hashlib
import os

import numpy as np
import PIL
import torch
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))


def source_image(h, w, seed):
    """Deterministic RGB test image: smooth gradients + noise (exercises rounding and clipping)."""
    r = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy) * 7) % 256], -1)
    noise = r.integers(-40, 41, (h, w, 3))
    return np.clip(base + noise, 0, 255).astype(np.uint8)


def cases():
    """(h, w, oh, ow, seed): Market crops (128x64), upscale / downscale / identity per axis,
    odd sizes, tall narrow sources (Pillow's vertical-first order), tiny images."""
    c = [(128, 64, 256, 128, 1), (256, 128, 256, 128, 2), (400, 200, 256, 128, 3), (255, 127, 256, 128, 4),
         (257, 129, 256, 128, 5), (37, 19, 256, 128, 6), (604, 2, 256, 128, 7), (402, 4, 256, 128, 8),
         (3000, 20, 256, 128, 9), (1, 1, 256, 128, 10), (256, 300, 256, 128, 11), (100, 128, 256, 128, 12),
         (700, 350, 256, 128, 13), (128, 64, 224, 224, 14), (333, 97, 384, 192, 15)]
    r = np.random.default_rng(2024)
    for i in range(48):
        c.append((int(r.integers(16, 800)), int(r.integers(8, 400)), 256, 128, 100 + i))
    return c


def to_tensor_normalize(img_u8, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5)):
    t = torch.from_numpy(np.array(img_u8, copy=True)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    m = torch.as_tensor(mean, dtype=torch.float32).view(-1, 1, 1)
    s = torch.as_tensor(std, dtype=torch.float32).view(-1, 1, 1)
    return t.sub_(m).div_(s).numpy()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    cs = cases()
    res_sha, norm_sha, full = [], [], []
    for k, (h, w, oh, ow, seed) in enumerate(cs):
        img = source_image(h, w, seed)
        out = np.asarray(Image.fromarray(img, "RGB").resize((ow, oh), Image.BILINEAR))
        res_sha.append(sha(out))
        norm_sha.append(sha(to_tensor_normalize(out)))
        if k < 6:
            full.append(out)
    np.savez_compressed(os.path.join(HERE, "transforms.npz"), cases=np.array(cs, np.int64),
                        resized_sha=np.array(res_sha), normalized_sha=np.array(norm_sha),
                        resized_first=np.stack(full), pillow_version=np.array(PIL.__version__))
    print(f"{len(cs)} cases, Pillow {PIL.__version__}")


if __name__ == "__main__":
    main()
