"""open_clip.tokenize mirror (open_clip/tokenizer.py:159-189, SimpleTokenizer): CLIP's byte-level
BPE (Radford et al. 2021), host-side like the reference.

The merge table is the vocabulary file open_clip ships (`bpe_simple_vocab_16e6.txt.gz`); it
is data, not bundled here -- pass its path, or set DACLIP_BPE_VOCAB. Algorithm:
  * text: html-unescape (twice), collapse whitespace, lower-case (ftfy.fix_text is applied
    when ftfy is importable; it is a no-op for plain ASCII);
  * pre-tokenise with the CLIP regex (specials, contractions, letter runs, single digits,
    other non-space runs);
  * map each piece's UTF-8 bytes to printable unicode (the 188 printable latin-1 bytes
    map to themselves, the other 68 to U+0100..; vocabulary order: printable first),
    mark the last symbol with '</w>' and apply merges greedily by rank;
  * ids: 256 byte symbols, their '</w>' forms, one id per merge, then <start_of_text> and
    <end_of_text> (49406, 49407 for the released vocabulary);
  * tokenize(): [sot] + ids + [eot], cut to context_length (the last slot stays eot), zero
    padded -> int64 [N, context_length].
"""
from __future__ import annotations

import gzip
import html
import os
from functools import lru_cache
from typing import Dict, List, Optional, Sequence, Tuple, Union

import regex
import torch

SOT, EOT = "<start_of_text>", "<end_of_text>"


def _byte_symbols() -> Dict[int, str]:
    """byte -> symbol, ordered as the vocabulary enumerates them: the printable bytes first
    (in byte order), then the remapped ones."""
    printable = (list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) +
                 list(range(ord("®"), ord("ÿ") + 1)))
    table = {b: chr(b) for b in printable}
    extra = 0
    for b in range(256):
        if b not in table:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def _clean(text: str) -> str:
    try:
        import ftfy  # optional, as in the reference
        text = ftfy.fix_text(text)
    except Exception:
        pass
    text = html.unescape(html.unescape(text)).strip()
    return regex.sub(r"\s+", " ", text).strip().lower()


class BPETokenizer:
    PATTERN = regex.compile(
        r"<start_of_text>|<end_of_text>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+",
        regex.IGNORECASE)

    def __init__(self, vocab_path: Optional[str] = None):
        path = vocab_path or os.environ.get("DACLIP_BPE_VOCAB")
        if not path or not os.path.exists(path):
            raise FileNotFoundError("BPE vocabulary not found: pass vocab_path or set DACLIP_BPE_VOCAB to "
                                    "open_clip's bpe_simple_vocab_16e6.txt.gz")
        with gzip.open(path, "rt", encoding="utf-8") as f:
            lines = f.read().split("\n")
        n_merges = 49152 - 256 - 2
        merges = [tuple(l.split()) for l in lines[1:1 + n_merges]]
        self.bytes = _byte_symbols()
        symbols = list(self.bytes.values())
        symbols = symbols + [s + "</w>" for s in symbols] + ["".join(m) for m in merges] + [SOT, EOT]
        self.encoder = {s: i for i, s in enumerate(symbols)}
        self.rank = {m: i for i, m in enumerate(merges)}
        self.sot, self.eot = self.encoder[SOT], self.encoder[EOT]

    def _bpe(self, piece: str) -> List[str]:
        return list(self._bpe_cached(piece))

    @lru_cache(maxsize=65536)
    def _bpe_cached(self, piece: str) -> Tuple[str, ...]:
        if piece in (SOT, EOT):
            return (piece,)
        word = list(piece[:-1]) + [piece[-1] + "</w>"]
        while len(word) > 1:
            best, bi = None, -1
            for i in range(len(word) - 1):
                r = self.rank.get((word[i], word[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if best is None:
                break
            a, b = word[bi], word[bi + 1]
            merged, i = [], 0
            while i < len(word):           # merge every occurrence of the best pair
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    merged.append(a + b)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = merged
        return tuple(word)

    def encode(self, text: str) -> List[int]:
        ids = []
        for tok in self.PATTERN.findall(_clean(text)):
            piece = "".join(self.bytes[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[s] for s in self._bpe(piece))
        return ids

    def __call__(self, texts: Union[str, Sequence[str]], context_length: int = 77) -> torch.Tensor:
        if isinstance(texts, str):
            texts = [texts]
        out = torch.zeros(len(texts), context_length, dtype=torch.long)
        for i, t in enumerate(texts):
            ids = [self.sot] + self.encode(t) + [self.eot]
            if len(ids) > context_length:
                ids = ids[:context_length]
                ids[-1] = self.eot
            out[i, :len(ids)] = torch.tensor(ids, dtype=torch.long)
        return out


_default: Optional[BPETokenizer] = None


def tokenize(texts: Union[str, Sequence[str]], context_length: int = 77,
             vocab_path: Optional[str] = None) -> torch.LongTensor:
    """open_clip.tokenize(texts, context_length) -> int64 [N, context_length]."""
    global _default
    if vocab_path is not None:
        return BPETokenizer(vocab_path)(texts, context_length)
    if _default is None:
        _default = BPETokenizer()
    return _default(texts, context_length)


def get_tokenizer(model_name: str = "daclip_ViT-B-32"):
    """open_clip.get_tokenizer: every DA-CLIP config uses the CLIP BPE at context 77."""
    return lambda texts, context_length=77: tokenize(texts, context_length)
