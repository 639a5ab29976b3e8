"""CLIP byte-level BPE tokenizer (host side).  PARITY UNPINNED: CLIP's vocabulary file is not
available offline, so the algorithm is checked on a synthetic merges file: byte symbols,
</w> word ends, merge ranks, special tokens, the row layout of clip.tokenize and truncation."""
import numpy as np
import pytest

from multimodal_reid_amd import tokenizer as tk


@pytest.fixture()
def tok(tmp_path):
    merges = ["#version: synthetic", "p h", "ph o", "t o</w>", "pho to</w>", "o f</w>"]
    p = tmp_path / "merges.txt"
    p.write_text("\n".join(merges) + "\n")
    return tk.SimpleTokenizer(str(p))


def test_vocab_layout(tok):
    b2u = tk.bytes_to_unicode()
    assert len(b2u) == 256 and len(set(b2u.values())) == 256
    assert tok.encoder["!"] == 0 and tok.encoder["a</w>"] == 256 + list(b2u).index(ord("a"))
    assert list(b2u)[:94] == list(range(ord("!"), ord("~") + 1)) and b2u[0] == chr(256)
    assert tok.encoder["ph"] == 512 and tok.encoder["photo</w>"] == 515
    assert tok.encoder[tk.SOT] == 517 and tok.encoder[tk.EOT] == 518


def test_bpe_merges_and_cleaning(tok):
    ids = tok.encode("  A  &amp;amp; photo of\\n")
    words = [tok.decoder[i] for i in ids]
    assert words == ["a</w>", "&</w>", "photo</w>", "of</w>", "\\</w>", "n</w>"]  # HTML unescaped twice
    assert tok.decode(tok.encode("a photo of")) == "a photo of "


def test_tokenize_rows(tok):
    t = tk.tokenize(["a photo of", "photo"], context_length=8, tokenizer=tok)
    assert t.dtype == np.int64 and t.shape == (2, 8)
    assert list(t[0][:5]) == [517, tok.encoder["a</w>"], 515, tok.encoder["of</w>"], 518] and not t[0][5:].any()
    assert (t.argmax(-1) == np.array([4, 2])).all()  # EOT is the row maximum (text_encoder.py:23)
    with pytest.raises(RuntimeError):
        tk.tokenize("a photo of a photo of a photo", context_length=5, tokenizer=tok)
    tr = tk.tokenize("a photo of a photo of a photo", context_length=5, truncate=True, tokenizer=tok)
    assert tr[0, -1] == 518
    with pytest.raises(NotImplementedError):
        tk.tokenize("a photo")
