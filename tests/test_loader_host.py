"""Host side of the device loaders (CPU, no GPU): the native threaded file gather
(reidmi_files_size / reidmi_files_read / reidmi_bytes_gather through data_prepare.read_files) and
the item-list parsing of loader.get_loader (datasets/dataset_market.py:79 tuples)."""

import numpy as np
import pytest

from multimodal_reid_amd import data_prepare, loader


def _blobs(n, seed):
    r = np.random.default_rng(seed)
    return [bytes(r.integers(0, 256, int(r.integers(0, 9000)), dtype=np.uint8)) for _ in range(n)]


@pytest.mark.parametrize("nthreads", [0, 1, 3, 16])
def test_read_files_bytes_and_paths(tmp_path, nthreads):
    blobs = _blobs(700, nthreads) + [b""]  # an empty file too
    want = b"".join(blobs)
    buf, off = data_prepare.read_files(blobs, nthreads=nthreads)
    assert buf.tobytes() == want and off[0] == 0 and np.array_equal(np.diff(off), [len(b) for b in blobs])
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"{i}.jpg"
        p.write_bytes(b)
        paths.append(p if i % 2 else str(p))  # PathLike and str
    buf2, off2 = data_prepare.read_files(paths, nthreads=nthreads)
    assert buf2.tobytes() == want and np.array_equal(off2, off)
    # bytearray / memoryview / bytes subclasses / a mixed batch: the same bytes
    class B(bytes):
        pass
    mixed = [bytearray(blobs[0]), memoryview(blobs[1]), B(blobs[2]), paths[3], blobs[4]]
    buf3, _ = data_prepare.read_files(mixed, nthreads=nthreads)
    assert buf3.tobytes() == b"".join(blobs[:5])


def test_read_files_into_preallocated_buffer_and_errors(tmp_path):
    blobs = _blobs(50, 9)
    total = sum(map(len, blobs))
    out = np.full(total + 100, 7, np.uint8)
    buf, _ = data_prepare.read_files(blobs, out=out)
    assert buf.ctypes.data == out.ctypes.data and buf.tobytes() == b"".join(blobs) and out[total] == 7
    small = np.zeros(max(total - 1, 0), np.uint8)  # too small: a fresh array, the caller's untouched
    buf, _ = data_prepare.read_files(blobs, out=small)
    assert buf.ctypes.data != small.ctypes.data and not small.any()
    (tmp_path / "a.jpg").write_bytes(b"x")
    with pytest.raises(FileNotFoundError, match="missing.jpg"):
        data_prepare.read_files([tmp_path / "a.jpg", tmp_path / "missing.jpg"])
    with pytest.raises(FileNotFoundError):
        data_prepare.read_files([tmp_path])  # a directory is not a file
    buf, off = data_prepare.read_files([])
    assert buf.size == 0 and off.tolist() == [0]


def test_loader_item_lists():
    files, (p, c, s, i) = loader._items([("a", 3, 1, 7, 70), ("b", -1, 2, 8, 71), ("c", 0, 5)])
    assert files == ["a", "b", "c"]
    assert p.tolist() == [3, -1, 0] and c.tolist() == [1, 2, 5] and s.tolist() == [7, 8, 0] and i.tolist() == [70, 71, 2]
    assert all(a.dtype == np.int64 for a in (p, c, s, i))


def test_shard_items_keep_one_process_offsets():
    """get_loader(..., shard=(rank, world)): the ranks' contiguous shards cover the list in
    order, and every item keeps the RandomCrop offsets it has in one process."""
    from multimodal_reid_amd import data_prepare, loader
    items = [(b"x%d" % k, k % 7, k % 3, 0, k) for k in range(103)]
    full, off = loader._shard_items(items, 9, None)
    assert full == items and np.array_equal(off, data_prepare.tta_offsets(103, 9))
    for world in (2, 3, 8):
        got_items, got_off = [], []
        for rank in range(world):
            it, o = loader._shard_items(items, 9, (rank, world))
            assert len(it) == len(o)
            got_items += it
            got_off.append(o)
        assert got_items == items and np.array_equal(np.concatenate(got_off), off)
