"""Host side of the GPU JPEG path (miclip/jpeg.py): marker parsing of the
reference's frames and of Pillow-written files, and the Huffman decode tables
in libjpeg's derived form (checked by decoding every code of every table)."""
import glob
import io
import os

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))


def test_parse_reference_frames():
    from miclip import jpeg
    for f in sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg"))):
        h = jpeg.parse(open(f, "rb").read())
        assert h.supported and (h.width, h.height, h.ncomp) == (1280, 720, 3)
        assert h.samp == [(2, 2), (1, 1), (1, 1)] and h.ri == 0


def _codes(bits):
    code, out = 0, []
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            out.append((code, ln))
            code += 1
        code <<= 1
    return out


def test_huff_tables_decode_every_code():
    """For every (code, length) of every table in the reference frames and a
    Pillow file with optimised tables: the 9-bit look-ahead (short codes) or the
    maxcode / valoff walk (long codes) returns the code's symbol."""
    from PIL import Image
    from miclip import jpeg
    bufs = [open(f, "rb").read() for f in sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[:2]]
    b = io.BytesIO()
    Image.fromarray((np.random.default_rng(1).random((40, 40, 3)) * 255).astype(np.uint8)).save(
        b, "JPEG", quality=60, optimize=True)
    bufs.append(b.getvalue())
    n, n2 = 0, [0]
    for buf in bufs:
        for (bits, vals) in jpeg.parse(buf).huff.values():
            t = jpeg.build_huff(bits, vals)
            for k, (code, ln) in enumerate(_codes(bits)):
                if ln <= 9:
                    for tail in (0, (1 << (9 - ln)) - 1):
                        lk = int(t["look"][(code << (9 - ln)) | tail])
                        assert lk >> 8 == ln and lk & 0xFF == vals[k]
                else:
                    peek9 = code >> (ln - 9)
                    assert t["look"][peek9] == 0
                    l, c = 10, code >> (ln - 10)
                    while c > t["maxcode"][l]:
                        l += 1
                        c = code >> (ln - l) if l <= ln else code << (l - ln)
                    assert l == ln and t["vals"][(c + t["valoff"][l]) & 0xFF] == vals[k]
                    if t["l2n"]:   # second-level table: every 16-bit window under this code
                        lo = (code << (16 - ln)) - int(t["l2base"])
                        for tail in (0, (1 << (16 - ln)) - 1):
                            assert 0 <= lo + tail < t["l2n"]
                            assert int(t["look2"][lo + tail]) == (ln << 8) | vals[k]
                        n2[0] += 1
                n += 1
    assert n > 300 and n2[0] > 100


def test_unsupported_kinds_are_flagged():
    from PIL import Image
    from miclip import jpeg
    im = Image.fromarray((np.random.default_rng(2).random((20, 24, 3)) * 255).astype(np.uint8))
    b = io.BytesIO()
    im.save(b, "JPEG", progressive=True)
    assert not jpeg.parse(b.getvalue()).supported
    b = io.BytesIO()
    im.convert("CMYK").save(b, "JPEG")
    assert not jpeg.parse(b.getvalue()).supported
    assert not jpeg.parse(b"\x89PNG....").supported
