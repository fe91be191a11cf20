"""Baseline JPEG decode on the GPU (``mi_jpeg_decode``, ``csrc/jpeg.hip``),
bit-identical to Pillow's ``Image.open(p).convert("RGB")`` — the decode step
of the reference's frame ingest (``Backend/services/embedding_service.py:472-480``,
``Backend/embedding.py:46``).

The host reads each file's markers (DQT, SOF0/SOF1, DHT, DRI, SOS), builds the
Huffman decode tables in libjpeg's derived form (9-bit look-ahead + maxcode /
value offsets per code length), de-zigzags the quantisation tables, locates
restart markers, and hands one batch per geometry to the device with the
Huffman tables deduplicated into sets (a video's frames share one): the entropy
decode runs one lane per frame (or per restart interval) with the sets in LDS,
the IDCT one thread per block, the upsampling + colour conversion one thread
per pixel.

Files the device path does not cover (progressive or arithmetic coding,
12-bit samples, CMYK / Adobe-transform or 4-component images, sampling other
than chroma 1x1 with luma 1x1 / 2x1 / 2x2, more than two Huffman tables of a
class, EXIF orientation is NOT applied by either path) are decoded by Pillow
on the host, so every frame gets the reference's pixels.
"""
from __future__ import annotations

import struct
import threading

import numpy as np

from . import _native as N

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                   13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59,
                   52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], dtype=np.int64)
HUFF_BYTES = 3480
L2_MAX = 1024
_HUFF_DT = np.dtype([("look", "<u2", 512), ("maxcode", "<i4", 18), ("valoff", "<i4", 18), ("vals", "u1", 256),
                     ("l2base", "<i4"), ("l2n", "<i4"), ("look2", "<u2", L2_MAX)])
assert _HUFF_DT.itemsize == HUFF_BYTES


_HUFF_CACHE = {}


def _huff_cached(bits, vals):
    key = (bytes(bits), bytes(vals))
    t = _HUFF_CACHE.get(key)
    if t is None:
        if len(_HUFF_CACHE) > 4096:
            _HUFF_CACHE.clear()
        t = _HUFF_CACHE[key] = build_huff(bits, vals)
    return key, t


def build_huff(bits, vals):
    """libjpeg jpeg_make_d_derived_tbl: canonical codes from the 16 length
    counts; 9-bit look-ahead entries (length << 8) | symbol; maxcode / value
    offsets for the longer codes.  Codes of 10-16 bits are canonical-last, so
    they and the invalid tail fill the 16-bit window range [l2base, 65536):
    when that range has <= L2_MAX values, look2 maps each to (length << 8) |
    symbol (0: corrupt), one LDS lookup instead of libjpeg's per-length walk."""
    t = np.zeros((), dtype=_HUFF_DT)
    t["maxcode"][:] = -1
    t["maxcode"][17] = 0x7FFFFFFF
    vals = list(vals)
    t["vals"][:len(vals)] = vals
    code, p = 0, 0
    for ln in range(1, 17):
        n = bits[ln - 1]
        if n:
            t["valoff"][ln] = p - code
            for _ in range(n):
                if ln <= 9:
                    lo = code << (9 - ln)
                    t["look"][lo:lo + (1 << (9 - ln))] = (ln << 8) | vals[p]
                code += 1
                p += 1
            t["maxcode"][ln] = code - 1
        code <<= 1
    code, p, first = 0, 0, None
    longs = []
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            if ln >= 10:
                if first is None:
                    first = code << (16 - ln)
                longs.append((code << (16 - ln), 1 << (16 - ln), (ln << 8) | vals[p]))
            code += 1
            p += 1
        code <<= 1
    if first is not None and 65536 - first <= L2_MAX:
        t["l2base"], t["l2n"] = first, 65536 - first
        for lo, n, e in longs:
            t["look2"][lo - first:lo - first + n] = e
    return t


class JpegHeader:
    __slots__ = ("width", "height", "ncomp", "samp", "qsel", "dcsel", "acsel", "ri", "qt", "huff", "scan_start",
                 "supported", "why")


_HEAD_CACHE = {}


def _scan_start(buf):
    """Byte offset just past the first SOS segment (a bare marker walk), or None."""
    n = len(buf)
    if n < 4 or buf[0] != 0xFF or buf[1] != 0xD8:
        return None
    i = 2
    while i + 4 <= n:
        if buf[i] != 0xFF:
            return None
        m = buf[i + 1]
        if m == 0xFF:
            i += 1
            continue
        if m in (0xD8, 0x01) or 0xD0 <= m <= 0xD7:
            i += 2
            continue
        if m == 0xD9:
            return None
        ln = (buf[i + 2] << 8) | buf[i + 3]
        if m == 0xDA:
            return i + 2 + ln
        i += 2 + ln
    return None


_HEAD_MRU = []   # (header bytes, parsed header) of the most recently seen encoders


def parse(buf: bytes) -> JpegHeader:
    """Marker walk up to the first SOS; sets ``supported`` False (with ``why``)
    for anything the device decoder does not restate.  Frames of one encoder
    share their header bytes, so the parsed header is cached by those bytes
    (everything before the entropy-coded data); only the end-of-image check is
    per file.  A buffer that starts with a recently seen header's bytes IS that
    header (the bytes end at the scan start), so the marker walk -- 7 us of
    Python per frame, most of a batch's host time before the first launch -- is
    skipped for it."""
    h = None
    for key, hh in _HEAD_MRU:
        if buf.startswith(key):
            h = hh
            break
    if h is None:
        ss = _scan_start(buf)
        if ss is None:
            return _parse(buf)
        key = bytes(buf[:ss])
        h = _HEAD_CACHE.get(key)
        if h is None:
            if len(_HEAD_CACHE) > 1024:
                _HEAD_CACHE.clear()
            h = _HEAD_CACHE[key] = _parse(buf, check_eoi=False)
        _HEAD_MRU.insert(0, (key, h))
        del _HEAD_MRU[8:]
    if h.supported and buf.rfind(b"\xff\xd9") <= h.scan_start:   # truncated: Pillow raises; let it
        t = JpegHeader()
        for f in JpegHeader.__slots__:
            setattr(t, f, getattr(h, f))
        t.supported, t.why = False, "no EOI after the scan"
        return t
    return h


def _parse(buf, check_eoi=True) -> JpegHeader:
    h = JpegHeader()
    h.supported, h.why = False, ""
    h.qt, h.huff, h.ri = {}, {}, 0
    h.width = h.height = h.ncomp = 0
    comps = []
    if len(buf) < 4 or buf[0] != 0xFF or buf[1] != 0xD8:
        h.why = "not a JPEG"
        return h
    i = 2
    adobe_transform = None
    jfif = False
    while i + 4 <= len(buf):
        if buf[i] != 0xFF:
            h.why = "bad marker"
            return h
        m = buf[i + 1]
        if m == 0xFF:          # fill byte
            i += 1
            continue
        if m in (0xD8, 0x01) or 0xD0 <= m <= 0xD7:
            i += 2
            continue
        ln = struct.unpack(">H", buf[i + 2:i + 4])[0]
        seg = buf[i + 4:i + 2 + ln]
        if m == 0xDB:                                     # DQT
            j = 0
            while j < len(seg):
                pq, tq = seg[j] >> 4, seg[j] & 15
                if pq:
                    q = np.frombuffer(seg[j + 1:j + 129], dtype=">u2").astype(np.uint16)
                    j += 129
                else:
                    q = np.frombuffer(seg[j + 1:j + 65], dtype=np.uint8).astype(np.uint16)
                    j += 65
                nat = np.zeros(64, np.uint16)
                nat[ZIGZAG] = q
                h.qt[tq] = nat
        elif m in (0xC0, 0xC1):                           # baseline / extended sequential, Huffman
            if seg[0] != 8:
                h.why = "sample precision != 8"
                return h
            h.height, h.width = struct.unpack(">HH", seg[1:5])
            h.ncomp = seg[5]
            for c in range(h.ncomp):
                cid, hv, tq = seg[6 + 3 * c], seg[7 + 3 * c], seg[8 + 3 * c]
                comps.append((cid, hv >> 4, hv & 15, tq))
        elif 0xC2 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            h.why = f"SOF{m - 0xC0} (progressive / lossless / arithmetic)"
            return h
        elif m == 0xC4:                                   # DHT
            j = 0
            while j < len(seg):
                tc, th = seg[j] >> 4, seg[j] & 15
                bits = list(seg[j + 1:j + 17])
                n = sum(bits)
                h.huff[(tc, th)] = (bits, bytes(seg[j + 17:j + 17 + n]))
                j += 17 + n
        elif m == 0xDD:                                   # DRI
            h.ri = struct.unpack(">H", seg[:2])[0]
        elif m == 0xE0 and seg[:5] == b"JFIF\x00":
            jfif = True
        elif m == 0xEE and seg[:5] == b"Adobe" and len(seg) >= 12:
            adobe_transform = seg[11]
        elif m == 0xDA:                                   # SOS
            ns = seg[0]
            scomp = [(seg[1 + 2 * k], seg[2 + 2 * k] >> 4, seg[2 + 2 * k] & 15) for k in range(ns)]
            ss, se, ahal = seg[1 + 2 * ns], seg[2 + 2 * ns], seg[3 + 2 * ns]
            h.scan_start = i + 2 + ln
            if not comps:
                h.why = "SOS before SOF"
                return h
            if ns != h.ncomp or ss != 0 or se != 63 or ahal != 0:
                h.why = "not a single interleaved sequential scan"
                return h
            byid = {cid: (hs, vs, tq) for cid, hs, vs, tq in comps}
            try:
                h.samp = [(byid[cid][0], byid[cid][1]) for cid, _, _ in scomp]
                h.qsel = [byid[cid][2] for cid, _, _ in scomp]
            except KeyError:
                h.why = "scan names an unknown component"
                return h
            h.dcsel = [td for _, td, _ in scomp]
            h.acsel = [ta for _, _, ta in scomp]
            if h.ncomp == 3:
                if adobe_transform == 0:
                    h.why = "Adobe RGB (no YCbCr transform)"
                    return h
                # libjpeg default_decompress_parms guesses the colour space from the component ids
                # when there is neither a JFIF nor an Adobe marker ('R','G','B' -> no transform)
                if not jfif and adobe_transform is None and tuple(c[0] for c in comps) != (1, 2, 3):
                    h.why = "no JFIF / Adobe marker and component ids other than 1, 2, 3"
                    return h
                if h.samp[1] != (1, 1) or h.samp[2] != (1, 1) or h.samp[0] not in ((1, 1), (2, 1), (2, 2)):
                    h.why = f"sampling {h.samp}"
                    return h
            elif h.ncomp != 1:
                h.why = f"{h.ncomp} components"
                return h
            if any(t > 1 for t in h.dcsel + h.acsel):
                h.why = "Huffman table id > 1"
                return h
            if any(q not in h.qt for q in h.qsel) or any((0, t) not in h.huff for t in h.dcsel) or \
                    any((1, t) not in h.huff for t in h.acsel):
                h.why = "missing table"
                return h
            if any(max(h.huff[(0, t)][1], default=0) > 15 for t in h.dcsel):
                h.why = "DC table symbol > 15"     # libjpeg rejects the table (JERR_BAD_HUFF_TABLE)
                return h
            if any(q > 3 for q in h.qsel) or h.width < 1 or h.height < 1:
                h.why = "bad frame header"
                return h
            if check_eoi and buf.rfind(b"\xff\xd9") <= h.scan_start:   # truncated: Pillow raises; let it
                h.why = "no EOI after the scan"
                return h
            h.supported = True
            return h
        elif m == 0xD9:
            break
        i += 2 + ln
    h.why = h.why or "no scan"
    return h


def decoded_bytes(h) -> int:
    """Device bytes one frame holds while ``mi_jpeg_decode`` runs: the RGB
    output plus the coefficient workspace (int16 + 1 byte per sample of every
    component block, ``jpeg_workspace_bytes``); host-decoded frames hold their
    RGB only."""
    W, H = max(h.width, 1), max(h.height, 1)
    if not h.supported:
        return 3 * W * H
    hs = [s[0] for s in h.samp] if h.ncomp == 3 else [1]
    vs = [s[1] for s in h.samp] if h.ncomp == 3 else [1]
    mcux, mcuy = -(-W // (8 * max(hs))), -(-H // (8 * max(vs)))
    blocks = sum(mcux * a * mcuy * b for a, b in zip(hs, vs))
    return 3 * W * H + 192 * blocks


def _geom_key(h):
    return (h.width, h.height, h.ncomp, tuple(h.samp), h.ri)


def _segments(buf, h):
    """Entropy-coded byte ranges of the restart segments (one without DRI)."""
    start = h.scan_start
    if not h.ri:
        return [(start, len(buf))]
    segs, j, n = [], start, len(buf)
    s0 = start
    while j + 1 < n:
        if buf[j] == 0xFF:
            c = buf[j + 1]
            if 0xD0 <= c <= 0xD7:
                segs.append((s0, j))
                j += 2
                s0 = j
                continue
            if c == 0xD9:
                break
            j += 2 if c == 0x00 else 1
            continue
        j += 1
    segs.append((s0, n))
    return segs


_STAGE = [None, None]            # two pinned staging buffers (double-buffered uploads)
_STAGE_EVT = [None, None]        # the last H2D copy out of each
_STAGE_LOCK = threading.Lock()
_PAD = np.frombuffer(b"\xff\xd9" * 16, np.uint8)


def _bytes_data_off():
    import ctypes
    b = bytes(b"jpeg-probe")
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p).value - id(b)


_BYTES_DATA_OFF = _bytes_data_off()
SUB_FRAMES = 2048                # frames per decode launch: the host gathers launch j + 1 while the GPU decodes j
FIRST_SUB = 512                  # the first launch of a group: the pipeline's unhidden head


_COPY_STREAMS = {}


def _copy_stream(dev):
    """A side stream per device for the frames' H2D copies, so the copy of launch
    j + 1 overlaps the decode kernels of launch j on the compute stream."""
    import torch
    cs = _COPY_STREAMS.get(dev)
    if cs is None:
        cs = _COPY_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return cs


def _upload(bufs, keep, segl, starts, total, dev, slot=0):
    """Entropy-coded bytes of the kept frames gathered straight into pinned
    staging buffer `slot` by 16 native threads (mi_host_gather, no GIL), then
    an asynchronous DMA to the device on the copy stream, which the current
    (compute) stream waits for; 32 bytes of EOI markers as padding.  The buffer
    is reused only after its previous copy has completed (event), so a caller
    alternating slots overlaps the next gather and copy with the kernels that
    consume this one."""
    import ctypes
    import torch
    with _STAGE_LOCK:
        if _STAGE_EVT[slot] is not None:
            _STAGE_EVT[slot].synchronize()
        st = _STAGE[slot]
        if st is None or st.numel() < total + 32:
            st = torch.empty(max(total + 32, 1 << 26), dtype=torch.uint8, pin_memory=True)
            _STAGE[slot] = st
        n = len(keep)
        # a bytes object's data sits at a fixed offset from its address (CPython), measured once;
        # any other object type takes the ctypes path
        ptrs = np.fromiter((id(bufs[i]) + _BYTES_DATA_OFF + sg[0][0] if type(bufs[i]) is bytes
                            else ctypes.cast(ctypes.c_char_p(bufs[i]), ctypes.c_void_p).value + sg[0][0]
                            for i, sg in zip(keep, segl)), np.uint64, n)
        lens = np.diff(np.asarray(starts, np.int64))
        keepalive = [bufs[i] for i in keep]
        N.check(N.lib().mi_host_gather(st.data_ptr(), ptrs.ctypes.data, lens.ctypes.data, n, 16), "mi_host_gather")
        del keepalive
        st.numpy()[total:total + 32] = _PAD
        cur = torch.cuda.current_stream(dev)
        cs = _copy_stream(dev)
        # allocated on the copy stream's pool (the caching allocator reuses a block freed after its
        # record_stream(cur) only once the compute stream's work on it is done): no wait on the
        # compute stream, so this copy overlaps the previous launch's kernels
        with torch.cuda.stream(cs):
            d = torch.empty(total + 32, dtype=torch.uint8, device=dev)
            d.copy_(st[:total + 32], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cs)
        _STAGE_EVT[slot] = ev
        cur.wait_event(ev)
        d.record_stream(cur)
        return d


def launch_args(bufs, heads, keep, segl, key, dedupe=True):
    """mi_jpeg_decode's arguments for the frames ``keep`` of one geometry group
    ``key`` (their entropy-coded segments ``segl`` concatenated in order):
    (geom int32[20], huff [nsets, 4] tables, huff_idx int32[B], qtab uint16[B, 4, 64],
    seg_off / seg_end int64[B * nseg] into the concatenation, starts int64[B + 1]
    (frame r's bytes at [starts[r], starts[r + 1])), nsets), or None when the
    frames' table selectors differ."""
    W, H, nc, samp, ri = key
    h0 = heads[keep[0]]
    B = len(keep)
    lens = np.array([sg[-1][1] - sg[0][0] for sg in segl], np.int64)
    starts = np.zeros(B + 1, np.int64)
    np.cumsum(lens, out=starts[1:])
    if ri:
        offs = [int(starts[r]) + a - sg[0][0] for r, sg in enumerate(segl) for a, _ in sg]
        ends = [int(starts[r]) + b - sg[0][0] for r, sg in enumerate(segl) for _, b in sg]
    else:
        offs, ends = starts[:-1], starts[1:]
    # table sets deduplicated: frames of one encoder share one set (and one
    # cached header object), which the entropy kernel stages in LDS
    # (per distinct header object, then mapped to the frames: a per-frame Python loop over numpy
    # scalars cost ~1.4 us a frame before the first launch)
    hobj = [heads[i] for i in keep]
    uniq = {}
    for h in hobj:
        uniq.setdefault(id(h), h)
    first_of = list(uniq.values())
    index_of = {k: u for u, k in enumerate(uniq)}
    hid = np.fromiter((index_of[id(h)] for h in hobj), np.int64, B)
    per_head, qts = [], []
    for h in first_of:
        slots, tabs = [None] * 4, [None] * 4
        for (tc, th), (bits, vals) in h.huff.items():
            if th <= 1:
                slots[th * 2 + tc], tabs[th * 2 + tc] = _huff_cached(bits, vals)
        q4 = np.zeros((4, 64), np.uint16)
        for tq, q in h.qt.items():
            if tq <= 3:
                q4[tq] = q
        qts.append(q4)
        per_head.append((tuple(slots), tabs))
    sets, set_of = [], {}
    if dedupe:
        hset = np.zeros(len(per_head), np.int32)
        for u, (slots, tabs) in enumerate(per_head):
            if slots not in set_of:
                set_of[slots] = len(sets)
                sets.append(tabs)
            hset[u] = set_of[slots]
        hidx = hset[hid]
    else:
        sets = [per_head[u][1] for u in hid]
        hidx = np.arange(B, dtype=np.int32)
    qt = np.ascontiguousarray(np.stack(qts)[hid])
    nseg = len(segl[0])
    geom = np.zeros(20, np.int32)
    geom[:5] = (W, H, nc, ri, nseg)
    for c in range(nc):
        geom[5 + 2 * c], geom[6 + 2 * c] = (samp[c] if nc == 3 else (1, 1))
        geom[11 + c], geom[14 + c], geom[17 + c] = h0.qsel[c], h0.dcsel[c], h0.acsel[c]
    # per-frame table selectors must agree within the group (they come from the SOS / SOF)
    if not all(h.qsel == h0.qsel and h.dcsel == h0.dcsel and h.acsel == h0.acsel for h in first_of):
        return None
    huff = np.zeros((len(sets), 4), dtype=_HUFF_DT)
    for u, tabs in enumerate(sets):
        for j, t in enumerate(tabs):
            if t is not None:
                huff[u, j] = t
    return (geom, huff, hidx, qt, np.asarray(offs, np.int64), np.asarray(ends, np.int64), starts, len(sets))


def decode_batch(bufs, device="cuda", dedupe=True):
    """Decode JPEG byte strings on the GPU where the geometry allows, Pillow
    otherwise.  Returns a list of uint8 [H, W, 3] device tensors (None for a
    file neither path can read) in input order; frames of one geometry are
    decoded in one launch.  ``dedupe=False`` passes one table set per frame
    (no index array: the kernel's global-memory table path)."""
    out = [None] * len(bufs)
    for idx, rgb in decode_groups(bufs, device, dedupe=dedupe):
        if rgb is not None:
            for r, i in enumerate(idx):
                out[i] = rgb[r]
    return out


def decode_groups(bufs, device="cuda", dedupe=True, heads=None, transform=None):
    """``decode_batch`` by launch: yields (indices, uint8 [len(indices), H, W, 3]
    device tensor) per geometry group in one buffer (frames the host decodes
    come one per group; (indices, None) for a file neither path can read), so a
    consumer can take each group's frames without restacking them.

    ``transform=(n, squash, out_dtype)``: yield the preprocessed frames
    [len(indices), 3, n, n] instead (openai/CLIP ``_transform(n)``, or the
    squash resize of compare_models.py:387-391), through the fused
    ``mi_jpeg_decode_transform`` (no RGB frames in HBM; bit-identical to decoding
    and then ``preprocess.preprocess_frames``); host-decoded frames and sources
    the fused kernel does not take are decoded and then preprocessed."""
    import torch
    L = N.lib()
    if heads is None:
        heads = [parse(b) for b in bufs]

    def host(i):
        idx, rgb = _host_group(bufs, i, device)
        if transform is None or rgb is None:
            return idx, rgb
        from .preprocess import preprocess_frames
        return idx, preprocess_frames(rgb, transform[0], squash=transform[1], out_dtype=transform[2])

    groups, gkey = {}, {}
    for i, h in enumerate(heads):
        if h.supported:
            k = gkey.get(id(h))
            if k is None:
                k = gkey[id(h)] = _geom_key(h)
            groups.setdefault(k, []).append(i)
        else:
            yield host(i)
    dev = torch.device(device)
    for key, idx in groups.items():
        W, H, nc, samp, ri = key
        mcux = -(-W // (8 * (max(s[0] for s in samp) if nc == 3 else 1)))
        mcuy = -(-H // (8 * (max(s[1] for s in samp) if nc == 3 else 1)))
        nseg = -(-(mcux * mcuy) // ri) if ri else 1
        keep, segl = [], []
        for i in idx:
            h = heads[i]
            if ri:
                segs = _segments(bufs[i], h)
                if len(segs) != nseg:     # restart markers not where DRI says: leave it to the host decoder
                    yield host(i)
                    continue
            else:
                segs = ((h.scan_start, len(bufs[i])),)
            keep.append(i)
            segl.append(segs)
        if not keep:
            continue
        B = len(keep)
        args = launch_args(bufs, heads, keep, segl, key, dedupe)
        if args is None:     # per-frame table selectors differ within the group: the host decoder
            for i in keep:
                yield host(i)
            continue
        geom, huff, hidx, qt, offs, ends, starts, nsets = args
        gp = geom.ctypes.data
        # launches of SUB_FRAMES frames: the host gathers (and the copy stream uploads) launch
        # j + 1 while the GPU decodes launch j; the per-frame arrays go up once for the group,
        # each launch's segment offsets relative to its own data
        # the first launch is short (FIRST_SUB frames), so the GPU starts after a short gather +
        # copy instead of a whole launch's worth (the rest of the pipeline hides the host side)
        step = max(1, min(B, SUB_FRAMES))
        first = FIRST_SUB if B > 2 * FIRST_SUB else step
        subs = [(0, min(B, first))] + [(j0, min(B, j0 + step)) for j0 in range(min(B, first), B, step)]
        rel = offs.copy(), ends.copy()
        for j0, j1 in subs:
            rel[0][j0 * nseg:j1 * nseg] -= starts[j0]
            rel[1][j0 * nseg:j1 * nseg] -= starts[j0]
        d_huff = torch.from_numpy(huff.view(np.uint8).reshape(-1)).to(dev)
        d_off = torch.from_numpy(rel[0]).to(dev)
        d_end = torch.from_numpy(rel[1]).to(dev)
        d_hidx = torch.from_numpy(np.ascontiguousarray(hidx)).to(dev)
        d_qt = torch.from_numpy(np.ascontiguousarray(qt)).to(dev)
        fused = transform is not None
        if fused:
            n, squash, odt = transform
            out = torch.empty(B, 3, n, n, dtype=odt, device=dev)
            mode = N.MI_PREP_SQUASH if squash else N.MI_PREP_CLIP
        else:
            out = torch.empty(B, H, W, 3, dtype=torch.uint8, device=dev)
        nb = max(L.mi_jpeg_workspace_bytes(gp, j1 - j0, int(starts[j1] - starts[j0])) for j0, j1 in subs)
        ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
        for u, (j0, j1) in enumerate(subs):
            base, sub_total = int(starts[j0]), int(starts[j1] - starts[j0])
            d_data = _upload(bufs, keep[j0:j1], segl[j0:j1], starts[j0:j1 + 1] - base, sub_total, dev, slot=u & 1)
            # without dedupe frame f uses set f: this launch's frames start at set j0
            hp = d_huff.data_ptr() + (0 if dedupe else j0 * 4 * HUFF_BYTES)
            a = (d_data.data_ptr(), sub_total, d_off.data_ptr() + j0 * nseg * 8, d_end.data_ptr() + j0 * nseg * 8, hp,
                 d_hidx.data_ptr() + j0 * 4 if dedupe else None, nsets, d_qt.data_ptr() + j0 * 4 * 64 * 2, gp, j1 - j0)
            if fused:
                rc = L.mi_jpeg_decode_transform(*a, n, mode, out[j0:j1].data_ptr(), N.dtype_code(odt), ws.data_ptr(),
                                                nb, N.stream_ptr(dev))
                if rc == -3:     # MI_ERR_UNSUPPORTED: too large for the fused kernel's LDS bands
                    from .preprocess import preprocess_frames
                    rgb = torch.empty(j1 - j0, H, W, 3, dtype=torch.uint8, device=dev)
                    N.check(L.mi_jpeg_decode(*a, rgb.data_ptr(), ws.data_ptr(), nb, N.stream_ptr(dev)),
                            "mi_jpeg_decode")
                    out[j0:j1] = preprocess_frames(rgb, n, squash=squash, out_dtype=odt)
                else:
                    N.check(rc, "mi_jpeg_decode_transform")
            else:
                N.check(L.mi_jpeg_decode(*a, out[j0:j1].data_ptr(), ws.data_ptr(), nb, N.stream_ptr(dev)),
                        "mi_jpeg_decode")
            del d_data
        del ws
        yield keep, out


def _host_group(bufs, i, device):
    t = _host_decode(bufs[i], device)
    return [i], (t.unsqueeze(0) if t is not None else None)


def _host_decode(buf, device):
    import io

    import torch
    from PIL import Image
    try:
        with Image.open(io.BytesIO(buf)) as im:
            return torch.from_numpy(np.asarray(im.convert("RGB"), dtype=np.uint8).copy()).to(device)
    except Exception:
        return None


def decode_files(paths, device="cuda"):
    """``decode_batch`` over files (read on the host, decoded on the GPU)."""
    bufs = []
    for p in paths:
        try:
            with open(p, "rb") as f:
                bufs.append(f.read())
        except OSError:
            bufs.append(b"")
    return decode_batch(bufs, device)
