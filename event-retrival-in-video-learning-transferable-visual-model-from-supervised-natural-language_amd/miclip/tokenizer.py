"""``clip.tokenize`` — CLIP's byte-level BPE (openai/CLIP ``simple_tokenizer``
algorithm, restated) over a LOCAL vocabulary file.

Call sites: ``embedding_service.py:169`` (``clip.tokenize([q])``) and
``compare_models.py:1202`` (``truncate=True``).  The BPE merges file
(``bpe_simple_vocab_16e6.txt.gz``) is not in the container, so
it is read from ``$CLIP_BPE_PATH`` or an explicit path; without it tokenize
raises and callers pass token ids directly (the bench and the parity tests do).
Tokenizer parity against openai/CLIP is therefore **unpinned** here.
"""
from __future__ import annotations

import functools
import gzip
import html
import os

import regex as re

SOT = "<|startoftext|>"
EOT = "<|endoftext|>"


@functools.lru_cache()
def bytes_to_unicode():
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def _pairs(word):
    return {(a, b) for a, b in zip(word[:-1], word[1:])}


# ftfy.fix_text (openai/CLIP basic_clean's first step; ftfy 6 default
# TextFixerConfig) is not installed here.  Restated: the deterministic fixers
# that apply to well-formed Unicode input, in ftfy's order — terminal escapes,
# mojibake repair (the common case, below), Latin ligatures, character width,
# curly quotes, line breaks, control characters, NFC.  Of ftfy's fix_encoding
# only the whole-string case is restated: UTF-8 bytes that were decoded as
# Windows-1252 / Latin-1 ("cafÃ©", "âœ”", doubly "Ã¢â‚¬â„¢"), recognised by a
# UTF-8 lead byte followed by a continuation byte as those codecs render them,
# undone while the string re-encodes in (sloppy) Windows-1252 and the bytes
# decode as UTF-8.  A string with any character outside Windows-1252 (Vietnamese
# ư / ơ / ạ, CJK, emoji) never re-encodes, so well-formed text is left alone.
# ftfy's badness heuristics for partial and mixed mojibake
# (decode_inconsistent_utf8, restore_byte_a0, replace_lossy_sequences) are not
# restated: parity with ftfy itself is unpinned.
_ANSI = re.compile(r"\x1b\[[\d;]*[@-~]")
_LIGATURES = {"\u0132": "IJ", "\u0133": "ij", "\u01f1": "DZ", "\u01f2": "Dz", "\u01f3": "dz", "\u01c4": "DŽ",
              "\u01c5": "Dž", "\u01c6": "dž", "\u01c7": "LJ", "\u01c8": "Lj", "\u01c9": "lj", "\u01ca": "NJ",
              "\u01cb": "Nj", "\u01cc": "nj", "\ufb00": "ff", "\ufb01": "fi", "\ufb02": "fl", "\ufb03": "ffi",
              "\ufb04": "ffl", "\ufb05": "ſt", "\ufb06": "st"}
# ftfy uncurl_quotes: SINGLE_QUOTE_RE [\u02bc\u2018-\u201b] -> ', DOUBLE_QUOTE_RE [\u201c-\u201f] -> "
# (primes U+2032 / U+2033 are left alone)
_QUOTES = {"\u02bc": "'", "\u2018": "'", "\u2019": "'", "\u201a": "'", "\u201b": "'", "\u201c": '"',
           "\u201d": '"', "\u201e": '"', "\u201f": '"'}
# ftfy chardata CONTROL_CHARS: U+0000-0008, 000B, 000E-001F, 007F, 206A-206F, FEFF, FFF9-FFFC,
# 1D173-1D17A (musical formatting), E0000-E007F (tags)
_CONTROL = re.compile(r"[\x00-\x08\x0b\x0e-\x1f\x7f\u206a-\u206f\ufff9-\ufffc\ufeff"
                      r"\U0001d173-\U0001d17a\U000e0000-\U000e007f]")


# cp1252 renders bytes 0x80-0x9F as these characters (the five bytes it leaves undefined,
# 0x81 0x8D 0x8F 0x90 0x9D, pass through as U+0081 ... in ftfy's "sloppy-windows-1252")
_CP1252_HIGH = "€\x81‚ƒ„…†‡ˆ‰Š‹Œ\x8dŽ\x8f\x90‘’“”•–—˜™š›œ\x9džŸ"
_SLOPPY_1252 = {c: 0x80 + i for i, c in enumerate(_CP1252_HIGH)}
_SLOPPY_1252.update({chr(b): b for b in range(0xA0, 0x100)})
# a UTF-8 lead byte (0xC2-0xF4) followed by a continuation byte (0x80-0xBF), as cp1252 shows them
_MOJIBAKE = re.compile("[\u00c2-\u00f4][" + re.escape(_CP1252_HIGH) + "\u00a0-\u00bf]")


def _sloppy_1252_bytes(text):
    out = bytearray()
    for c in text:
        o = ord(c)
        if o < 0x80:
            out.append(o)
        elif c in _SLOPPY_1252:
            out.append(_SLOPPY_1252[c])
        else:
            return None
    return bytes(out)


def fix_encoding_subset(text):
    """ftfy fix_encoding, whole-string case: re-decode text that is UTF-8 read as cp1252."""
    for _ in range(4):               # doubly (or triply) encoded text unwinds one layer a pass
        if not _MOJIBAKE.search(text):
            break
        b = _sloppy_1252_bytes(text)
        if b is None:
            break
        try:
            fixed = b.decode("utf-8")
        except UnicodeDecodeError:
            break
        if fixed == text:
            break
        text = fixed
    return text


def fix_text_subset(text):
    import unicodedata
    text = _ANSI.sub("", text)
    text = fix_encoding_subset(text)
    text = "".join(_LIGATURES.get(c, c) for c in text)
    # fix_character_width: fullwidth / halfwidth forms and the ideographic space, by NFKC of those characters
    text = "".join(unicodedata.normalize("NFKC", c) if ("\uff01" <= c <= "\uffee" or c == "\u3000") else c
                   for c in text)
    text = "".join(_QUOTES.get(c, c) for c in text)
    text = text.replace("\r\n", "\n").replace("\r", "\n")
    for c in ("\u2028", "\u2029", "\u0085"):
        text = text.replace(c, "\n")
    text = _CONTROL.sub("", text)
    return unicodedata.normalize("NFC", text)


def _clean(text):
    """basic_clean + whitespace_clean of openai/CLIP simple_tokenizer."""
    text = fix_text_subset(text)
    text = html.unescape(html.unescape(text))
    return re.sub(r"\s+", " ", text.strip()).strip()


class SimpleTokenizer:
    def __init__(self, bpe_path: str, n_merges: int = 49152 - 256 - 2):
        opener = gzip.open if bpe_path.endswith(".gz") else open
        with opener(bpe_path, "rb") as f:
            lines = f.read().decode("utf-8").split("\n")
        merges = [tuple(m.split()) for m in lines[1:n_merges + 1] if m.strip()]
        self.byte_encoder = bytes_to_unicode()
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab]
        vocab += ["".join(m) for m in merges]
        vocab += [SOT, EOT]
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.decoder = {i: v for v, i in self.encoder.items()}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {SOT: SOT, EOT: EOT}
        self.pat = re.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""",
                              re.IGNORECASE)

    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        pairs = _pairs(word)
        if not pairs:
            return token + "</w>"
        while True:
            bigram = min(pairs, key=lambda p: self.bpe_ranks.get(p, float("inf")))
            if bigram not in self.bpe_ranks:
                break
            first, second = bigram
            new_word = []
            i = 0
            while i < len(word):
                try:
                    j = word.index(first, i)
                except ValueError:
                    new_word.extend(word[i:])
                    break
                new_word.extend(word[i:j])
                i = j
                if word[i] == first and i < len(word) - 1 and word[i + 1] == second:
                    new_word.append(first + second)
                    i += 2
                else:
                    new_word.append(word[i])
                    i += 1
            word = tuple(new_word)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        out = " ".join(word)
        self.cache[token] = out
        return out

    def encode(self, text):
        ids = []
        text = _clean(text).lower()
        for tok in re.findall(self.pat, text):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[t] for t in self.bpe(tok).split(" "))
        return ids


@functools.lru_cache(maxsize=4)
def _tokenizer(path):
    return SimpleTokenizer(path)


def tokenize(texts, context_length: int = 77, truncate: bool = False, bpe_path: str | None = None):
    """Same contract as openai/CLIP ``clip.tokenize``: IntTensor [len(texts), context_length]."""
    import torch
    path = bpe_path or os.environ.get("CLIP_BPE_PATH")
    if not path or not os.path.isfile(path):
        raise RuntimeError("clip.tokenize needs the CLIP BPE vocabulary (bpe_simple_vocab_16e6.txt.gz); set "
                           "CLIP_BPE_PATH to a local copy or pass token ids to encode_text directly")
    tok = _tokenizer(path)
    if isinstance(texts, str):
        texts = [texts]
    sot, eot = tok.encoder[SOT], tok.encoder[EOT]
    result = torch.zeros(len(texts), context_length, dtype=torch.int)
    for i, t in enumerate(texts):
        ids = [sot] + tok.encode(t) + [eot]
        if len(ids) > context_length:
            if truncate:
                ids = ids[:context_length]
                ids[-1] = eot
            else:
                raise RuntimeError(f"Input {t} is too long for context length {context_length}")
        result[i, :len(ids)] = torch.tensor(ids, dtype=torch.int)
    return result
