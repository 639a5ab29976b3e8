"""CLIP's byte-level BPE tokenizer (host side, §8f-3): what zero_shot_learning.py:43,52 and
the prompt learners (coop.py:76, maple.py:36) call as ``clip.tokenize``.

    SimpleTokenizer(bpe_path).encode(text) -> [token ids]
    tokenize(texts, context_length=77, truncate=False, tokenizer=None) -> int64 [N, 77]

The algorithm is OpenAI CLIP's published one (the ``clip`` package, not vendored in the
reference): text cleaned (HTML unescaped twice, whitespace collapsed, lower-cased), split by
CLIP's regex, each piece's UTF-8 bytes mapped to printable unicode and merged by the BPE ranks
of the merges file (49152 - 256 - 2 merges), ids = the 256 byte symbols, their ``</w>``
forms, the merges, then ``<|startoftext|>`` / ``<|endoftext|>``.  Rows are
[SOT, ids..., EOT, 0...]; EOT is the largest id, which the text tower's argmax relies on.

PARITY UNPINNED: the vocabulary file (bpe_simple_vocab_16e6.txt.gz) is not available
offline, so ids cannot be checked against the reference's; tests/test_tokenizer.py checks the
algorithm on a synthetic merges file.  ftfy.fix_text (a dependency of clip's basic_clean) is
not installed either and is skipped (a no-op on clean ASCII text such as the templates).
"""
import gzip
import html
from functools import lru_cache

import numpy as np
import regex as re

SOT, EOT = "<|startoftext|>", "<|endoftext|>"


@lru_cache()
def bytes_to_unicode():
    """Reversible byte -> printable-unicode map (printable Latin-1 bytes map to themselves,
    the rest to code points from 256 up)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = list(bs)
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))  # iteration order = vocabulary order


def _pairs(word):
    return {(word[i], word[i + 1]) for i in range(len(word) - 1)}


def _clean(text):
    text = html.unescape(html.unescape(text)).strip()
    return re.sub(r"\s+", " ", text).strip()


class SimpleTokenizer:
    def __init__(self, bpe_path, n_merges=49152 - 256 - 2):
        opener = gzip.open if str(bpe_path).endswith(".gz") else open
        with opener(bpe_path, "rt", encoding="utf-8") as f:
            lines = f.read().split("\n")
        merges = [tuple(m.split()) for m in lines[1:n_merges + 1] if m.strip()]
        b2u = bytes_to_unicode()
        vocab = list(b2u.values())
        vocab += [v + "</w>" for v in vocab]
        vocab += ["".join(m) for m in merges]
        vocab += [SOT, EOT]
        self.byte_encoder = b2u
        self.byte_decoder = {v: k for k, v in b2u.items()}
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.decoder = {i: v for v, i in self.encoder.items()}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {SOT: SOT, EOT: EOT}
        self.pat = re.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|"""
                              r"""[^\s\p{L}\p{N}]+""", re.IGNORECASE)

    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        pairs = _pairs(word)
        if not pairs:
            return token + "</w>"
        while True:
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if best not in self.bpe_ranks:
                break
            a, b = best
            merged, i = [], 0
            while i < len(word):
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    merged.append(a + b)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = tuple(merged)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        out = " ".join(word)
        self.cache[token] = out
        return out

    def encode(self, text):
        ids = []
        for piece in re.findall(self.pat, _clean(text).lower()):
            piece = "".join(self.byte_encoder[b] for b in piece.encode("utf-8"))
            ids.extend(self.encoder[t] for t in self.bpe(piece).split(" "))
        return ids

    def decode(self, ids):
        text = "".join(self.decoder[i] for i in ids)
        return bytearray(self.byte_decoder[c] for c in text).decode("utf-8", errors="replace").replace("</w>", " ")


def tokenize(texts, context_length=77, truncate=False, tokenizer=None):
    """clip.tokenize: int64 [N, context_length] rows [SOT, ids..., EOT, 0...]; a text longer
    than the context raises unless ``truncate`` (then the last kept id becomes EOT)."""
    if tokenizer is None:
        raise NotImplementedError("a SimpleTokenizer over CLIP's BPE vocabulary file is required "
                                  "(bpe_simple_vocab_16e6.txt.gz is not available offline)")
    if isinstance(texts, str):
        texts = [texts]
    sot, eot = tokenizer.encoder[SOT], tokenizer.encoder[EOT]
    out = np.zeros((len(texts), context_length), np.int64)
    for i, t in enumerate(texts):
        ids = [sot] + tokenizer.encode(t) + [eot]
        if len(ids) > context_length:
            if not truncate:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
            ids = ids[:context_length]
            ids[-1] = eot
        out[i, :len(ids)] = ids
    return out
