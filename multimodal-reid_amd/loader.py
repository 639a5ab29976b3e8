"""Device-side eval loaders: the caller surface of the reference's `get_loader`
(data_prepare.py:256-284) feeding `inference()` (zero_shot_learning.py:61-134).

The reference builds four DataLoaders (gallery / query x plain / augmented view), each running
`reidDataset.__getitem__` (data_prepare.py:87-96: `Image.open(path).convert("RGB")` + the
transform) in 4 worker processes, then `images.cuda()` per batch.  Here one batch of files is

  host   read into one pinned buffer by native threads (reidmi_files_read / reidmi_bytes_gather)
         and header-parsed (reidmi_jpeg_plan) on a background thread, depth batches ahead;
  device copied to HBM, decoded (reidmi_jpeg_decode) and resized / normalised
         (reidmi_preprocess_u8) on a side HIP stream, one batch ahead of the consumer — so the
         encoder of batch k (on the caller's stream) runs while batch k+1 decodes;

and yielded as `(images, target, cams, seqs, indices)` exactly like the reference's loaders
(images a device fp16 [B, 3, H, W] tensor, the labels int64 CPU tensors).  The augmented
loader's images are a `TtaView`: the plain view's device tensor plus the RandomCrop offsets —
transform_test_augmented's flip / Pad((10, 5)) / crop commute with ToTensor / Normalize, and the
encoder's im2col applies them (zero_shot_learning.embed_pair(tta=...)), so the view is never
materialised.  The two loaders of a pair share the decode: iterated in lockstep (the zip of
`inference`), every batch is decoded once.

Out of scope: the dataset directory walks (`get_dataset`, datasets/*.py).  The
loaders take the dataset's item lists — `dataset.query` / `dataset.gallery`, tuples
(path or bytes, pid, camid, seqid, idx) as datasets/dataset_market.py:79 builds them.
"""
import concurrent.futures
import ctypes

import numpy as np
import torch

from . import _lib
from .data_prepare import JpegBatch, read_files, norm_stats, tta_offsets


class TtaView:
    """One batch of transform_test_augmented (data_prepare.py:262-270) kept implicit: `images`
    (the plain view, device [B, 3, H, W]) + `offsets` (device int32 [B, 2] = RandomCrop's (top,
    left) after Pad((10, 5)), data_prepare.tta_offsets)."""
    __slots__ = ("images", "offsets")

    def __init__(self, images, offsets):
        self.images, self.offsets = images, offsets

    @property
    def shape(self):
        return self.images.shape

    def size(self, dim=None):
        return self.images.size() if dim is None else self.images.size(dim)

    def __len__(self):
        return self.images.shape[0]


def _items(items):
    """(files, pids, camids, seqids, idxs) from the reference's dataset tuples (path, pid, camid,
    seqid, idx); 3- and 4-tuples get seqid 0 / idx = position."""
    files, cols = [], [[], [], [], []]
    for k, it in enumerate(items):
        files.append(it[0])
        cols[0].append(int(it[1]))
        cols[1].append(int(it[2]))
        cols[2].append(int(it[3]) if len(it) > 3 else 0)
        cols[3].append(int(it[4]) if len(it) > 4 else k)
    return files, [np.asarray(c, np.int64) for c in cols]


def _shard_items(items, tta_seed, shard):
    """(items, RandomCrop offsets) of this rank's contiguous shard (distributed.shard) of the
    list, or of all of it (shard None).  The offsets are drawn once for the whole list (the
    reference draws them unseeded in the workers, data_prepare.py:266-267), so a shard's items
    get the offsets they get in one process."""
    items = list(items)
    tta = tta_offsets(len(items), tta_seed)
    if shard is not None:
        from .distributed import shard as _shard
        lo, hi = _shard(len(items), *shard)
        items, tta = items[lo:hi], tta[lo:hi]
    return items, tta


class _Slot:
    """Pinned host staging of one batch in flight: file bytes, plan, meta, device status."""

    def __init__(self):
        self.files = torch.empty(0, dtype=torch.uint8).pin_memory()
        self.plan = torch.empty(0, dtype=torch.uint8).pin_memory()
        self.meta = torch.zeros(0, dtype=torch.int64).pin_memory()
        self.err = torch.zeros(0, dtype=torch.int32).pin_memory()
        self.free = None   # event after the last device read of this slot's buffers

    def reserve(self, files_bytes, plan_bytes, n):
        if self.free is not None:
            self.free.synchronize()   # the previous batch's H2D copies / status read-back are done
        if self.files.numel() < files_bytes:
            self.files = torch.empty(int(files_bytes * 1.25) + 4096, dtype=torch.uint8).pin_memory()
        if self.plan.numel() < plan_bytes:
            self.plan = torch.empty(int(plan_bytes * 1.25) + 4096, dtype=torch.uint8).pin_memory()
        if self.err.numel() < n:
            self.err = torch.zeros(int(n * 1.25) + 64, dtype=torch.int32).pin_memory()
            self.meta = torch.zeros(3 * self.err.numel(), dtype=torch.int64).pin_memory()


class _Pipeline:
    """The shared source of a plain / augmented loader pair (see the module docstring)."""

    def __init__(self, items, batch_size, image_height, image_width, model_type, dtype, device, host_threads,
                 depth, tta_seed, shard=None):
        if dtype not in (torch.float32, torch.float16):
            raise ValueError("dtype must be torch.float32 or torch.float16")
        items, tta = _shard_items(items, tta_seed, shard)
        self.files, (self.pids, self.cams, self.seqs, self.idxs) = _items(items)
        self.N = len(self.files)
        self.bs = int(batch_size)
        if self.bs <= 0:
            raise ValueError("batch_size must be positive")
        self.nb = (self.N + self.bs - 1) // self.bs
        self.h, self.w, self.dtype = int(image_height), int(image_width), dtype
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        mean, std = norm_stats(model_type)
        self.mean_c, self.std_c = (ctypes.c_float * 3)(*mean), (ctypes.c_float * 3)(*std)
        self.host_threads = int(host_threads)
        self.depth = max(1, int(depth))
        self.slots = [_Slot() for _ in range(self.depth + 2)]
        self.pool = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="reidmi-loader")
        self.side = torch.cuda.Stream(self.device)
        self.host = {}      # batch -> future of the host stage
        self.ready = {}     # batch -> [images, event, slot, jpeg batch, status checked] on the side stream
                            # (or the exception its host stage raised)
        self.tta = torch.from_numpy(np.ascontiguousarray(tta)).to(self.device)  # for the encoder's im2col

    def rows(self, k):
        return k * self.bs, min(self.N, (k + 1) * self.bs)

    # host stage (background thread; the native calls release the GIL)
    def _host_stage(self, k):
        a, b = self.rows(k)
        slot = self.slots[k % len(self.slots)]
        files = self.files[a:b]
        # size first (in-memory bytes: their lengths; paths: read_files sizes them natively)
        nbytes = sum(map(len, files)) if all(isinstance(f, (bytes, bytearray, memoryview)) for f in files) else 0
        slot.reserve(nbytes, 4096 + (b - a) * 256 + 64 * 1536, b - a)
        buf, off = read_files(files, out=slot.files.numpy(), nthreads=self.host_threads)
        if buf.ctypes.data != slot.files.data_ptr():   # paths larger than the slot: stage a pinned copy
            slot.reserve(buf.size, 0, 0)
            slot.files.numpy()[:buf.size] = buf
        jb = JpegBatch(None, buffer=(slot.files.numpy()[:buf.size], off), plan_out=slot.plan.numpy())
        jb.raise_for_status()
        slot.meta.numpy()[:3 * jb.B] = jb.meta.reshape(-1)
        return jb, slot

    def _submit_host(self, k):
        if 0 <= k < self.nb and k not in self.host and k not in self.ready:
            self.host[k] = self.pool.submit(self._host_stage, k)

    # device stage (side stream)
    def _launch(self, k):
        if k in self.ready or not 0 <= k < self.nb:
            return
        self._submit_host(k)
        try:
            jb, slot = self.host.pop(k).result()
        except Exception as e:   # surfaces when batch k itself is asked for, not at its prefetch
            self.ready[k] = e
            return
        a, b = self.rows(k)
        B = b - a
        dev = self.device
        with torch.cuda.stream(self.side):
            st = _lib.stream(dev)
            nf = int(jb.buf.size)
            dfiles = torch.empty(max(nf, 1), dtype=torch.uint8, device=dev)
            if nf:
                dfiles[:nf].copy_(slot.files[:nf], non_blocking=True)
            np_plan = int(jb.plan.size)
            dplan = torch.empty(max(np_plan, 1), dtype=torch.uint8, device=dev)
            if np_plan:
                if jb.plan.ctypes.data == slot.plan.data_ptr():
                    dplan[:np_plan].copy_(slot.plan[:np_plan], non_blocking=True)
                else:   # the plan outgrew the slot's first guess (many distinct tables): pin it
                    dplan[:np_plan].copy_(torch.from_numpy(jb.plan).pin_memory(), non_blocking=True)
            dmeta = torch.empty((max(B, 1), 3), dtype=torch.int64, device=dev)
            if B:
                dmeta.view(-1)[:3 * B].copy_(slot.meta[:3 * B], non_blocking=True)
            ws = torch.empty(max(jb.ws_bytes, 1), dtype=torch.uint8, device=dev)
            pix = torch.empty(max(jb.out_bytes, 1), dtype=torch.uint8, device=dev)
            err = torch.empty(max(B, 1), dtype=torch.int32, device=dev)
            images = torch.empty((B, 3, self.h, self.w), dtype=self.dtype, device=dev)
            info = jb.info.copy()
            _lib.call("reidmi_jpeg_decode", _lib.ptr(dfiles), _lib.ptr(dplan), info.ctypes.data_as(ctypes.c_void_p),
                      B, _lib.ptr(ws), ws.numel(), _lib.ptr(pix), _lib.ptr(err), st)
            _lib.call("reidmi_preprocess_u8", _lib.ptr(pix), _lib.ptr(dmeta), B, jb.max_h, jb.max_w, self.h, self.w,
                      self.mean_c, self.std_c, 0 if self.dtype == torch.float32 else 1, _lib.ptr(images), st)
            slot.err[:B].copy_(err[:B], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.side)
            slot.free = ev
        self.ready[k] = [images, ev, slot, jb, False]

    def get(self, k):
        """Batch k's device images, ready on the caller's stream; prefetches the next ones."""
        self._launch(k)
        for j in range(k + 1, k + 1 + self.depth):
            self._submit_host(j)
        self._launch(k + 1)   # batch k+1 decodes while the caller's work on batch k runs
        entry = self.ready[k]
        if isinstance(entry, Exception):
            del self.ready[k]
            raise entry
        images, ev, slot, jb, checked = entry
        ev.synchronize()      # waits for the side stream only (decode of batch k)
        B = images.shape[0]
        if B and not checked:   # the device status, read back into the slot (once: slots are reused)
            try:
                jb.raise_for_status(slot.err[:B].numpy().copy())
            except ValueError:
                del self.ready[k]
                raise
            entry[4] = True
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        images.record_stream(cur)
        for old in [j for j in self.ready if j < k - 1]:   # the pair's partner may still ask for k-1
            del self.ready[old]
        return images

    def labels(self, k):
        a, b = self.rows(k)
        return (torch.from_numpy(self.pids[a:b]), torch.from_numpy(self.cams[a:b]), torch.from_numpy(self.seqs[a:b]),
                torch.from_numpy(self.idxs[a:b]))

    def close(self):
        self.pool.shutdown(wait=True)
        self.host.clear()
        self.ready.clear()


class DeviceLoader:
    """One of get_loader's four loaders: iterates (images, target, cams, seqs, indices) batches
    in item order (shuffle=False, data_prepare.py:275-283).  `augmented` loaders yield TtaView
    images (transform_test_augmented); plain ones a device tensor (transform_test)."""

    def __init__(self, pipeline, augmented):
        self.pipe, self.augmented = pipeline, augmented
        self.batch_size = pipeline.bs
        self.dataset = pipeline.files

    def __len__(self):
        return self.pipe.nb

    def __iter__(self):
        p = self.pipe
        for k in range(p.nb):
            images = p.get(k)
            if self.augmented:
                a, b = p.rows(k)
                images = TtaView(images, p.tta[a:b])
            yield (images,) + p.labels(k)


def loader_pair(items, batch_size, image_height=256, image_width=128, model_type="vit", dtype=torch.float16,
                device=None, host_threads=0, depth=2, tta_seed=0, shard=None):
    """(plain loader, augmented loader) over one item list, sharing one decode pipeline."""
    p = _Pipeline(items, batch_size, image_height, image_width, model_type, dtype, device, host_threads, depth,
                  tta_seed, shard)
    return DeviceLoader(p, False), DeviceLoader(p, True)


def get_loader(dataset, batch_size, image_height, image_width, model_type, dtype=torch.float16, device=None,
               host_threads=0, depth=2, tta_seed=0, shard=None):
    """data_prepare.py:256-284 for an already-listed dataset (`dataset.query`, `dataset.gallery`):
    returns (loader_gallery, loader_query, loader_gallery_augmented, loader_query_augmented),
    the reference's order.  `tta_seed` seeds the augmented views' RandomCrop offsets (gallery
    and query draw from seeds tta_seed and tta_seed + 1).  `shard=(rank, world)`: each loader
    walks this rank's contiguous shard of its list (one process per GPU; the items keep the
    offsets they have in one process) — feed the shards to get_cmc_map(..., sharded=True)."""
    if model_type != "vit":
        raise NotImplementedError("libreidmi implements the ViT tower (north-star path) only")
    g, ga = loader_pair(dataset.gallery, batch_size, image_height, image_width, model_type, dtype, device,
                        host_threads, depth, tta_seed, shard)
    q, qa = loader_pair(dataset.query, batch_size, image_height, image_width, model_type, dtype, device,
                        host_threads, depth, None if tta_seed is None else tta_seed + 1, shard)
    return g, q, ga, qa
