"""The device loaders (loader.get_loader, the caller surface of data_prepare.py:256-284) feeding
inference() (zero_shot_learning.py:61-134): what they yield equals the per-call path
decode_jpeg -> preprocess_jpeg -> embed_pair(tta=...) bit for bit (itself pinned to Pillow +
the reference's transforms in test_jpeg.py / test_transforms.py), for files given as paths or as
in-memory bytes, with a ragged last batch; labels pass through in item order."""
import types

import numpy as np
import pytest
import torch

from multimodal_reid_amd import synthetic as syn

pytestmark = pytest.mark.gpu


def _items(n, seed, tmp_path=None):
    files = syn.jpeg_files(n - 2, 128, 64, seed=seed, quality=90)
    files += [syn.jpeg_files(1, 150, 61, seed=seed + 1, subsampling=1)[0],   # another size, 4:2:2
              syn.jpeg_files(1, 97, 50, seed=seed + 2, subsampling=0)[0]]    # 4:4:4
    r = np.random.default_rng(seed)
    pids = r.integers(-1, 40, n)
    cams = r.integers(0, 6, n)
    seqs = r.integers(0, 9, n)
    if tmp_path is not None:
        paths = []
        for k, b in enumerate(files):
            p = tmp_path / f"{k:04d}_c{cams[k]}.jpg"
            p.write_bytes(b)
            paths.append(str(p))
        srcs = paths
    else:
        srcs = files
    return [(srcs[k], int(pids[k]), int(cams[k]), int(seqs[k]), k) for k in range(n)], files


@pytest.fixture(scope="module")
def vit(gpu):
    from multimodal_reid_amd import model
    return model.VisionTransformer(syn.vit_state_dict("ViT-B/16", seed=3))  # resblocks[:12] run: 12 layers


@pytest.mark.parametrize("source", ["bytes", "paths"])
def test_loader_batches_equal_per_call_path(gpu, source, tmp_path):
    from multimodal_reid_amd import data_prepare, loader
    items, files = _items(300, 5, tmp_path if source == "paths" else None)
    plain, aug = loader.loader_pair(items, 128, tta_seed=11)
    assert len(plain) == len(aug) == 3
    offs = data_prepare.tta_offsets(300, 11)
    seen = 0
    for (im, t, c, s, i), (va, ta, *_r) in zip(plain, aug):
        B = im.shape[0]
        ref = data_prepare.preprocess_jpeg(files[seen:seen + B])
        assert im.dtype == torch.float16 and torch.equal(im.view(torch.int16), ref.view(torch.int16))
        assert isinstance(va, loader.TtaView) and va.images is im   # one decode for the pair
        assert np.array_equal(va.offsets.cpu().numpy(), offs[seen:seen + B])
        for col, k in ((t, 1), (c, 2), (s, 3), (i, 4), (ta, 1)):
            assert col.dtype == torch.int64 and col.tolist() == [it[k] for it in items[seen:seen + B]]
        seen += B
    assert seen == 300
    # iterated on their own (not in lockstep), the augmented loader decodes again: same bits
    for k, (va, *_r) in enumerate(aug):
        ref = data_prepare.preprocess_jpeg(files[k * 128:(k + 1) * 128])
        assert torch.equal(va.images.view(torch.int16), ref.view(torch.int16))


def test_get_loader_inference_equals_embed_pair(gpu, vit, tmp_path):
    """get_loader(dataset) -> inference(): embeddings, targets, cams, seqs equal the per-call
    path (decode -> preprocess -> embed_pair with the same RandomCrop offsets) bit for bit."""
    from multimodal_reid_amd import data_prepare, loader
    from multimodal_reid_amd import zero_shot_learning as zsl
    q_items, q_files = _items(70, 21, tmp_path)
    g_items, g_files = _items(230, 22)
    ds = types.SimpleNamespace(query=q_items, gallery=g_items)
    lg, lq, lga, lqa = loader.get_loader(ds, 96, 256, 128, "vit", tta_seed=7)
    assert data_prepare.get_loader is not None
    for lp, la, items, files, seed in ((lg, lga, g_items, g_files, 7), (lq, lqa, q_items, q_files, 8)):
        emb, tgt, cams, seqs = zsl.inference(vit, None, None, None, lp, la, False, "vit")
        imgs = data_prepare.preprocess_jpeg(files)
        ref = zsl.embed_pair(vit, imgs, tta=data_prepare.tta_offsets(len(files), seed))
        assert emb.shape == ref.shape == (len(files), vit.width + vit.out_dim)
        assert torch.equal(emb.view(torch.int32), ref.view(torch.int32))
        assert tgt.tolist() == [it[1] for it in items] and cams.tolist() == [it[2] for it in items]
        assert seqs.tolist() == [it[3] for it in items]


def test_loader_raises_on_undecodable_file(gpu):
    """No host fallback: a file the device cannot decode raises while iterating (as the
    reference's loader raises from PIL inside its workers)."""
    from multimodal_reid_amd import loader
    items, files = _items(40, 31)
    bad = bytearray(files[25])
    bad = bytes(bad[:len(bad) // 2])   # truncated inside the scan
    items[25] = (bad,) + items[25][1:]
    plain, _ = loader.loader_pair(items, 16)
    it = iter(plain)
    next(it)
    with pytest.raises(ValueError, match="truncated|cannot be decoded"):
        for _ in it:
            pass
