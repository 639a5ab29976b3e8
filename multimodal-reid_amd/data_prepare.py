"""Test-time image transforms of the reference's loaders, on the GPU.

data_prepare.py:257-270 builds, per image (reidDataset.__getitem__, data_prepare.py:87-92):

    transform_test           = Resize((h, w)) -> ToTensor() -> Normalize(mean, std)
    transform_test_augmented = Resize((h, w)) -> RandomHorizontalFlip(1.0) -> Pad((10, 5))
                               -> RandomCrop((h, w)) -> ToTensor() -> Normalize(mean, std)

with mean = std = 0.5 for the ViT (ImageNet statistics for the ResNet).  Here the decoded
RGB images of a whole batch go to the device as one packed uint8 buffer and
`reidmi_preprocess_u8` produces the normalised [B, 3, h, w] tensor, bit-exact with
PIL.Image.resize(BILINEAR) + ToTensor + Normalize (oracle/transforms_oracle.c pins the
arithmetic against Pillow).  The augmented view's flip / pad / crop commute with ToTensor
and Normalize, so they are not materialised: the encoder's im2col applies them from per-image
crop offsets (`tta_offsets`, `zero_shot_learning.embed_pair(tta=...)`).

The JPEG files themselves (data_prepare.py:89 `Image.open(path).convert("RGB")`) decode on the
device too: `decode_jpeg` parses the headers on the host (`reidmi_jpeg_plan`), ships the file
bytes and the plan to the GPU once, and `reidmi_jpeg_decode` produces the same packed HWC
batch `preprocess` builds from PIL images — bit-exact with Pillow's decoder.
"""
import ctypes
import os
import sys
import warnings

import numpy as np
import torch

from . import _lib

VIT_MEAN = (0.5, 0.5, 0.5)
VIT_STD = (0.5, 0.5, 0.5)
CNN_MEAN = (0.485, 0.456, 0.406)
CNN_STD = (0.229, 0.224, 0.225)


def norm_stats(model_type):
    """data_prepare.py:260,268: ViT statistics for model_type == "vit", ImageNet otherwise."""
    return (VIT_MEAN, VIT_STD) if model_type == "vit" else (CNN_MEAN, CNN_STD)


def _as_hwc_u8(img):
    if isinstance(img, np.ndarray):
        a = img
    else:  # PIL image: data_prepare.py:88 converts to RGB
        a = np.asarray(img.convert("RGB"))
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        raise ValueError(f"expected an RGB image (PIL or HxWx3 uint8 array), got {a.dtype} {a.shape}")
    return np.ascontiguousarray(a)


def pack_images(images):
    """Concatenate HWC uint8 images: (flat uint8 buffer, meta int64 [B][3] = (offset, h, w),
    max_h, max_w)."""
    arrs = [_as_hwc_u8(im) for im in images]
    meta = np.zeros((len(arrs), 3), np.int64)
    off = 0
    for i, a in enumerate(arrs):
        meta[i] = (off, a.shape[0], a.shape[1])
        off += a.size
    buf = np.concatenate([a.reshape(-1) for a in arrs]) if arrs else np.zeros(0, np.uint8)
    max_h = int(meta[:, 1].max()) if arrs else 1
    max_w = int(meta[:, 2].max()) if arrs else 1
    return buf, meta, max_h, max_w


def preprocess(images, height=256, width=128, model_type="vit", dtype=torch.float16, device=None, out=None):
    """Resize((height, width)) -> ToTensor -> Normalize of a batch of decoded RGB images
    (PIL images or HxWx3 uint8 arrays of any sizes) -> device tensor [B, 3, height, width]
    of `dtype` (torch.float32 = exactly the reference's tensor; torch.float16 = that tensor
    rounded to nearest-even, the encoder's input)."""
    if dtype not in (torch.float32, torch.float16):
        raise ValueError("dtype must be torch.float32 or torch.float16")
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    buf, meta, max_h, max_w = pack_images(images)
    B = meta.shape[0]
    if out is None:
        out = torch.empty((B, 3, height, width), dtype=dtype, device=device)
    elif tuple(out.shape) != (B, 3, height, width) or out.dtype != dtype or not out.is_contiguous():
        raise ValueError("out must be a contiguous [B, 3, height, width] tensor of `dtype`")
    if B == 0:
        return out
    _lib.require_cuda(out)
    pix = torch.from_numpy(buf).pin_memory().to(device, non_blocking=True)
    dmeta = torch.from_numpy(meta).pin_memory().to(device, non_blocking=True)
    mean, std = norm_stats(model_type)
    mean_c = (ctypes.c_float * 3)(*mean)
    std_c = (ctypes.c_float * 3)(*std)
    _lib.call("reidmi_preprocess_u8", _lib.ptr(pix), _lib.ptr(dmeta), B, max_h, max_w, height, width, mean_c, std_c,
              0 if dtype == torch.float32 else 1, _lib.ptr(out), _lib.stream(device))
    # no sync: the pinned staging buffers are recorded against the copy by torch's host
    # caching allocator, and pix/dmeta are freed stream-ordered on this stream
    return out


class EvalTransform:
    """Callable stand-in for data_prepare.get_loader's `transform_test` over a whole batch."""

    def __init__(self, image_height=256, image_width=128, model_type="vit", dtype=torch.float16):
        self.h, self.w, self.model_type, self.dtype = image_height, image_width, model_type, dtype

    def __call__(self, images, device=None):
        return preprocess(images, self.h, self.w, self.model_type, self.dtype, device)


# CPython lays a bytes object's data (NUL-terminated) right after its header: the first byte
# sits at id(b) + sys.getsizeof(b"") - 1.  Reading 19k pointers that way costs ~1 ms where a
# ctypes array of c_char_p costs ~5-10 ms; `_bytes_pointers` checks the layout on the batch's
# first object and uses the ctypes route where it does not hold.
_BYTES_DATA = sys.getsizeof(b"") - 1


def _bytes_pointers(blobs):
    n = len(blobs)
    p = np.fromiter(map(id, blobs), np.int64, n) + _BYTES_DATA
    if n and ctypes.cast(ctypes.c_char_p(blobs[0]), ctypes.c_void_p).value != int(p[0]):
        arr = (ctypes.c_char_p * n)(*blobs)
        p = np.frombuffer(ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64 * n)).contents, np.int64).copy()
        return p, arr
    return p, blobs


def read_files(files, out=None, nthreads=0):
    """Gather a batch of JPEG files (paths, or in-memory bytes-like objects) into ONE host
    buffer: (uint8 array, int64 offsets [B+1]).  Paths are read by reidmi_files_read, bytes
    copied by reidmi_bytes_gather — both on up to 16 host threads (`nthreads`, 0 = default),
    the file side of data_prepare.py:89's `Image.open(path)` in 4 DataLoader workers.  `out`:
    a preallocated uint8 array (e.g. a pinned tensor's numpy view), used when large enough.
    A path that cannot be read raises OSError (as open() would)."""
    files = list(files)
    n = len(files)
    kinds = {isinstance(f, (bytes, bytearray, memoryview)) for f in files}
    if len(kinds) > 1:  # mixed batch: read the paths here, then gather everything as bytes
        files = [f if isinstance(f, (bytes, bytearray, memoryview)) else open(os.fspath(f), "rb").read()
                 for f in files]
        kinds = {True}
    offsets = np.zeros(n + 1, np.int64)
    vp = ctypes.c_void_p
    if kinds == {True}:
        blobs = [f if type(f) is bytes else bytes(f) for f in files]  # exact bytes: the layout _bytes_pointers reads
        offsets[1:] = np.cumsum(np.fromiter(map(len, blobs), np.int64, n))
        total = int(offsets[-1])
        buf = out[:total] if out is not None and out.size >= total else np.empty(total, np.uint8)
        ptrs, keep = _bytes_pointers(blobs)
        _lib.call("reidmi_bytes_gather", ptrs.ctypes.data_as(vp), n, offsets.ctypes.data_as(vp),
                  buf.ctypes.data_as(vp), int(nthreads))
        del keep
        return buf, offsets
    paths = [os.fsencode(os.fspath(f)) for f in files]
    ptrs, keep = _bytes_pointers(paths)
    sizes = np.empty(n, np.int64)
    _lib.call("reidmi_files_size", ptrs.ctypes.data_as(vp), n, sizes.ctypes.data_as(vp), int(nthreads))
    if n and (sizes < 0).any():
        i = int(np.argmax(sizes < 0))
        raise FileNotFoundError(f"cannot open {os.fsdecode(paths[i])} ({int((sizes < 0).sum())} of {n} files)")
    offsets[1:] = np.cumsum(sizes)
    total = int(offsets[-1])
    buf = out[:total] if out is not None and out.size >= total else np.empty(total, np.uint8)
    status = np.zeros(n, np.int32)
    _lib.call("reidmi_files_read", ptrs.ctypes.data_as(vp), n, offsets.ctypes.data_as(vp), buf.ctypes.data_as(vp),
              status.ctypes.data_as(vp), int(nthreads))
    del keep
    if status.any():
        i = int(np.argmax(status != 0))
        raise OSError(f"reading {os.fsdecode(paths[i])} failed ({'changed size' if status[i] == 2 else 'read error'})")
    return buf, offsets


def _to_device(a, device):
    """Host numpy array -> device tensor; read-only buffers are only read by the copy."""
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        return torch.from_numpy(a).to(device)


JPEG_STATUS = {1: "not a JPEG or truncated", 2: "progressive / lossless / arithmetic-coded / 12-bit / multi-scan",
               3: "component layout other than grayscale or 3 x {4:4:4, 4:2:2, 4:2:0}",
               4: "missing or malformed quantisation / Huffman tables", 5: "entropy-coded data does not decode",
               6: "image file is truncated (libjpeg's input would run out before the last MCU)"}


class JpegBatch:
    """Host side of a JPEG batch: the file bytes, the decode plan (reidmi_jpeg_plan) and the
    per-image status / (offset, h, w) of the decoded layout.  Host only: needs no GPU."""

    def __init__(self, files, buffer=None, plan_out=None):
        # buffer: (uint8 bytes, int64 offsets [B+1]) already joined by read_files (files unused);
        # plan_out: a uint8 array the plan is written into when it fits (the loader's pinned slot)
        self.buf, self.offsets = read_files(files) if buffer is None else buffer
        B = len(self.offsets) - 1
        self.B = B
        self.meta = np.zeros((B, 3), np.int64)
        self.status = np.zeros(B, np.int32)
        self.info = np.zeros(10, np.int64)
        args = (self.buf.ctypes.data_as(ctypes.c_void_p), self.offsets.ctypes.data_as(ctypes.c_void_p), B)
        out = (self.meta.ctypes.data_as(ctypes.c_void_p), self.status.ctypes.data_as(ctypes.c_void_p),
               self.info.ctypes.data_as(ctypes.c_void_p))
        # one parse when the tables fit the first guess (a dataset has a handful of distinct ones)
        cap = 4096 + B * 256 + 64 * 1536
        if plan_out is not None and plan_out.size >= cap:
            cap = plan_out.size
            self.plan = plan_out
        else:
            self.plan = np.zeros(cap, np.uint8)
        _lib.call("reidmi_jpeg_plan", *args, self.plan.ctypes.data_as(ctypes.c_void_p), cap, *out)
        if int(self.info[0]) > cap:
            self.plan = np.zeros(int(self.info[0]), np.uint8)
            _lib.call("reidmi_jpeg_plan", *args, self.plan.ctypes.data_as(ctypes.c_void_p), int(self.info[0]), *out)
        self.plan = self.plan[:int(self.info[0])]
        self.ws_bytes, self.out_bytes = int(self.info[1]), int(self.info[2])
        self.max_h, self.max_w = max(int(self.info[3]), 1), max(int(self.info[4]), 1)

    def raise_for_status(self, status=None):
        st = self.status if status is None else status
        bad = np.nonzero(st)[0]
        if bad.size:
            i = int(bad[0])
            raise ValueError(f"{bad.size} of {self.B} JPEG files cannot be decoded on the device; file {i}: "
                             f"{JPEG_STATUS.get(int(st[i]), int(st[i]))}")


def decode_jpeg(files, device=None, check=True, return_status=False):
    """Image.open(f).convert("RGB") of every file (data_prepare.py:89), on the GPU.
    Returns (pix uint8 device tensor of the packed HWC images, meta int64 device tensor [B][3]
    = (offset, h, w), JpegBatch) — the input reidmi_preprocess_u8 takes — and, with
    return_status, the per-file device status (JPEG_STATUS codes).  With check=True an
    unsupported or undecodable file raises (there is no host fallback)."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    jb = files if isinstance(files, JpegBatch) else JpegBatch(files)
    if check:
        jb.raise_for_status()
    dev_files = _to_device(jb.buf, device) if jb.buf.size else torch.zeros(1, dtype=torch.uint8, device=device)
    dplan = _to_device(jb.plan, device)
    ws = torch.empty(max(jb.ws_bytes, 1), dtype=torch.uint8, device=device)
    pix = torch.empty(max(jb.out_bytes, 1), dtype=torch.uint8, device=device)
    err = torch.empty(max(jb.B, 1), dtype=torch.int32, device=device)
    _lib.require_cuda(pix)
    info = jb.info.copy()
    _lib.call("reidmi_jpeg_decode", _lib.ptr(dev_files), _lib.ptr(dplan), info.ctypes.data_as(ctypes.c_void_p), jb.B,
              _lib.ptr(ws), ws.numel(), _lib.ptr(pix), _lib.ptr(err), _lib.stream(device))
    if check and jb.B:
        jb.raise_for_status(err[:jb.B].cpu().numpy())
    meta = torch.from_numpy(jb.meta).to(device, non_blocking=True)
    return (pix, meta, jb, err[:jb.B]) if return_status else (pix, meta, jb)


def preprocess_jpeg(files, height=256, width=128, model_type="vit", dtype=torch.float16, device=None, out=None):
    """reidDataset.__getitem__ + transform_test for a batch of JPEG files, all on the GPU:
    decode_jpeg -> Resize -> ToTensor -> Normalize -> [B, 3, height, width]."""
    if dtype not in (torch.float32, torch.float16):
        raise ValueError("dtype must be torch.float32 or torch.float16")
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    pix, meta, jb = decode_jpeg(files, device)
    B = jb.B
    if out is None:
        out = torch.empty((B, 3, height, width), dtype=dtype, device=device)
    elif tuple(out.shape) != (B, 3, height, width) or out.dtype != dtype or not out.is_contiguous():
        raise ValueError("out must be a contiguous [B, 3, height, width] tensor of `dtype`")
    if B == 0:
        return out
    mean, std = norm_stats(model_type)
    mean_c = (ctypes.c_float * 3)(*mean)
    std_c = (ctypes.c_float * 3)(*std)
    _lib.call("reidmi_preprocess_u8", _lib.ptr(pix), _lib.ptr(meta), B, jb.max_h, jb.max_w, height, width, mean_c,
              std_c, 0 if dtype == torch.float32 else 1, _lib.ptr(out), _lib.stream(device))
    return out


def get_loader(dataset, batch_size, image_height, image_width, model_type, **kw):
    """data_prepare.py:256-284 on the device for an already-listed dataset (loader.get_loader):
    (loader_gallery, loader_query, loader_gallery_augmented, loader_query_augmented)."""
    from .loader import get_loader as _get_loader
    return _get_loader(dataset, batch_size, image_height, image_width, model_type, **kw)


def tta_offsets(n, generator=None):
    """RandomCrop((h, w)) offsets after Pad((10, 5)) for the augmented view (data_prepare.py:
    266-267): int32 [n][2] = (top i in [0, 10], left j in [0, 20]), as the encoder's TTA
    im2col takes them (the reference draws them unseeded inside DataLoader workers)."""
    g = generator if isinstance(generator, np.random.Generator) else np.random.default_rng(generator)
    return np.stack([g.integers(0, 11, n), g.integers(0, 21, n)], 1).astype(np.int32)
