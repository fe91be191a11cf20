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


def _segments_of(buf):
    """(marker, start, end) of the marker segments before the scan data."""
    out, i = [], 2
    while i + 4 <= len(buf):
        m = buf[i + 1]
        ln = (buf[i + 2] << 8) | buf[i + 3]
        out.append((m, i, i + 2 + ln))
        if m == 0xDA:
            break
        i += 2 + ln
    return out


def test_colour_space_guess_without_jfif():
    """libjpeg (Pillow) guesses the colour space of a 3-component file with no
    JFIF / Adobe marker from its component ids ('R','G','B' = no YCbCr
    transform): such files go to the host decoder; JFIF files and ids 1, 2, 3
    stay on the GPU path."""
    from PIL import Image
    from miclip import jpeg
    b = io.BytesIO()
    Image.fromarray((np.random.default_rng(3).random((16, 24, 3)) * 255).astype(np.uint8)).save(b, "JPEG")
    buf = bytearray(b.getvalue())
    assert jpeg._parse(bytes(buf)).supported
    app0 = [(s, e) for m, s, e in _segments_of(buf) if m == 0xE0]
    assert app0
    s0, e0 = app0[0]
    nojfif = buf[:s0] + buf[e0:]
    assert jpeg._parse(bytes(nojfif)).supported                   # ids 1, 2, 3: YCbCr either way

    def with_ids(b0, ids):
        b0 = bytearray(b0)
        for m, s, e in _segments_of(b0):
            if m == 0xC0:
                for c in range(3):
                    b0[s + 4 + 6 + 3 * c] = ids[c]
            if m == 0xDA:
                for c in range(3):
                    b0[s + 4 + 1 + 2 * c] = ids[c]
        return bytes(b0)

    rgb_ids = [ord("R"), ord("G"), ord("B")]
    h = jpeg._parse(with_ids(nojfif, rgb_ids))
    assert not h.supported and "JFIF" in h.why
    assert jpeg._parse(with_ids(buf, rgb_ids)).supported           # JFIF marker: YCbCr regardless of ids


def test_decode_budget_slices():
    """Decode launches bounded by device bytes (4K frames would not fit 8192 at a time)."""
    from miclip import jpeg
    from miclip.preprocess import _budget_slices
    assert list(_budget_slices([5, 5, 5, 5], 10)) == [(0, 2), (2, 4)]
    assert list(_budget_slices([30, 5, 5], 10)) == [(0, 1), (1, 3)]          # an oversized item goes alone
    assert list(_budget_slices([], 10)) == []
    h = jpeg.parse(open(sorted(glob.glob(os.path.join(ROOT, "golden", "ref_frames", "*.jpg")))[0], "rb").read())
    # 1280x720 4:2:0: RGB 2.76 MB + (14400 + 2 * 3600) blocks * 192 B
    assert jpeg.decoded_bytes(h) == 3 * 1280 * 720 + 192 * 21600
