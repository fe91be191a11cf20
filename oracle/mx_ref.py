"""ORACLE (test infrastructure only) — MX-style fp8 (OCP e4m3 elements, one
e8m0 scale per 64 consecutive elements of a row: the block the gfx950
16x16x128 block-scaled MFMA applies) reference arithmetic for the
"fp8 MFMA weights" configuration (BASELINE.json configs[4]).  The reference
has no fp8 path of its own (openai/CLIP runs fp16 on GPU / fp32 on CPU), so
this fixes the quantisation the HIP path must implement exactly:

  X = floor(log2(max |v| over a 64-block)) - 8    (8 = e4m3's largest exponent)
  q = RNE_e4m3(clamp(v * 2^-X, -448, 448)),  scale byte = X + 127 (X >= -127)

and the GEMM it feeds: sum_k (q_a * 2^Xa) (q_w * 2^Xw) in float64.
"""
from __future__ import annotations

import numpy as np


def e4m3_table():
    """float values of the 256 OCP e4m3fn codes (0x7f / 0xff are NaN)."""
    v = np.zeros(256, np.float64)
    for c in range(256):
        s, e, m = c >> 7, (c >> 3) & 15, c & 7
        if e == 15 and m == 7:
            v[c] = np.nan
            continue
        mag = (1 + m / 8.0) * 2.0 ** (e - 7) if e else (m / 8.0) * 2.0 ** -6
        v[c] = -mag if s else mag
    return v


E4M3 = e4m3_table()


def block_exponents(x, block=64):
    a = np.abs(np.asarray(x, np.float64)).reshape(x.shape[0], -1, block).max(-1)
    with np.errstate(divide="ignore"):
        X = np.where(a > 0, np.floor(np.log2(np.where(a > 0, a, 1.0))) - 8, -127)
    return np.clip(X, -127, 127).astype(np.int32)


def quantize(x, block=64):
    """x [rows, K] -> (codes uint8 [rows, K], scale bytes uint8 [rows, K/64]) with RNE."""
    x = np.asarray(x, np.float64)
    X = block_exponents(x, block)
    y = np.clip(x.reshape(x.shape[0], -1, block) * 2.0 ** -X[..., None], -448, 448).reshape(x.shape)
    finite = np.where(np.isnan(E4M3), np.inf, E4M3)
    order = np.argsort(finite[:254 + 2])  # codes sorted by value (NaNs last)
    vals = finite[order]
    idx = np.clip(np.searchsorted(vals, y), 1, len(vals) - 1)
    lo, hi = vals[idx - 1], vals[idx]
    pick_hi = (hi - y) < (y - lo)
    tie = (hi - y) == (y - lo)
    # ties: even mantissa (code LSB 0)
    hi_code, lo_code = order[idx], order[idx - 1]
    pick_hi |= tie & ((hi_code & 1) == 0)
    codes = np.where(pick_hi, hi_code, lo_code).astype(np.uint8)
    # +0 / -0: keep the sign of zero irrelevant (both decode to 0)
    return codes, (X + 127).astype(np.uint8)


def dequantize(codes, scales, block=64):
    v = E4M3[codes].reshape(codes.shape[0], -1, block)
    return (v * 2.0 ** (scales.astype(np.float64) - 127)[..., None]).reshape(codes.shape)


def gemm(qa, sa, qw, sw):
    """float64 out[M, N] = dequant(A) . dequant(W)^T."""
    return dequantize(qa, sa) @ dequantize(qw, sw).T


def to_stage_major(scales):
    """[rows, K/64] -> the kernels' stage-major layout [K/128, rows_pad, 2] (flattened)."""
    rows, nb = scales.shape
    rp = rows + (rows & 1)
    out = np.zeros((nb // 2, rp, 2), np.uint8)
    out[:, :rows, :] = scales.reshape(rows, nb // 2, 2).transpose(1, 0, 2)
    return out.reshape(-1)


def from_stage_major(buf, rows, K):
    rp = rows + (rows & 1)
    return np.asarray(buf, np.uint8).reshape(K // 128, rp, 2)[:, :rows, :].transpose(1, 0, 2).reshape(rows, K // 64)
