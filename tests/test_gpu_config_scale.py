"""configs[2] and configs[4] at the pass size bench.py runs them.

bench.py (`chunk`: up to ~500 000 token rows per pass) embeds
  * configs[2], ViT-L/14 bf16, 100k frames: 52 passes of 1924 frames
    (M = 494 468 rows, W = 1024, S = 257, 1932 M-tiles), and
  * configs[4], ViT-L/14@336px MX-fp8, one 125k-frame shard: 145 passes of 863
    frames (M = 497 951 rows, S = 577, 1946 M-tiles).
Both passes take the CLS-row last block (api.cpp last_block_cls / run_tower_mx:
the default at >= 256 frames per chunk), the persistent GEMMs' XCD-ranged tile
walk, and byte offsets past 2^31 in `mlp` / `qkv`.  Reference call site:
Backend/services/embedding_service.py:461-495 (a folder's frames encoded as
batch stacks by model.encode_image).

For ONE such pass through the product library, sampled frames are checked
against
  * the float64 oracle (oracle/clip_ref.py): 1 - cos <= 1e-3 (the north star's
    bound; the MX-fp8 tower's FP8_COS is the same number), plus the deviation
    cosine of test_gpu_encode (0.99 for bf16; a regression floor for MX-fp8);
  * an 8-frame-chunk encode of the same pixels (the full last block, two M
    tiles): bit-identical -- every kernel's per-row arithmetic is independent of
    M, of the tile walk and of the CLS-row gather;
  * the A/B build with MICLIP_CLS_LAST=0 (the full last block at the same pass
    size): bit-identical.

Sampled frames: the first tile (0-2; frame 0 spans rows 0-256 and crosses the
first M-tile boundary), the end of XCD 0's m-range of the N = 3W / N = W GEMMs
(m-major, ntiles / 8 tiles per XCD), the middle, the 2^31-byte crossings of
the bf16 `mlp` ([M, 4W]) and `qkv` ([M, 3W]) buffers, and the last, partial
M-tile.  ADVICE r5: the S > 64 attention paths under the CLS-row last block
(ViT-B/16, S = 197, bf16 / fp8 / fp32 towers) are checked bit for bit against
the full block by test_cls_last_bit_identical_s197."""
import numpy as np
import pytest

from conftest import state_dict

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3


def bench_chunk(frames, tokens):
    """bench.py's pass size: up to ~500k token rows, equal-size passes."""
    cap = max(8, 500_000 // tokens)
    return -(-frames // -(-frames // cap))


def sample_frames(chunk, S, W):
    """Frames at the tile / XCD-range / 2^31-offset boundaries of a chunk-frame pass."""
    M = chunk * S
    tiles_m = -(-M // 256)
    out = {0, 1, 2, chunk // 2, chunk - 2, chunk - 1}
    for n_tiles in (3 * W // 256, W // 256):          # in_proj, out_proj / c_proj (m-major walk)
        per_xcd = tiles_m * n_tiles // 8
        mb = (per_xcd - 1) // n_tiles                  # the last m-block of XCD 0's range
        out |= {(mb * 256) // S, min(chunk - 1, (mb * 256 + 255) // S)}
    for cols in (4 * W, 3 * W):                        # bf16 mlp / qkv: the row holding byte 2^31
        row = (1 << 31) // (cols * 2)
        if row < M:
            out |= {row // S, min(chunk - 1, row // S + 1)}
    out |= {((tiles_m - 1) * 256) // S}                # the last, partial M-tile
    return sorted(f for f in out if 0 <= f < chunk)


def _model(name, gpu, **kw):
    from miclip import config, model as M
    return M.CLIP(config.get_config(name), state_dict(name), device=gpu, **kw)


def _run_config(gpu, monkeypatch, name, frames, wts):
    import torch
    from miclip import _native, config
    from oracle import clip_ref
    from oracle.clip_ref import cosine
    cfg = config.get_config(name)
    S, W = cfg.vision_tokens, cfg.vision_width
    chunk = bench_chunk(frames, S)
    big = _model(name, gpu, image_chunk=chunk, weights=wts)
    assert big._chunks[0] == chunk
    g = torch.Generator(device=gpu).manual_seed(1234)   # bench.py's generator (rank 0)
    R = cfg.image_resolution
    pixels = torch.randn(chunk, 3, R, R, device=gpu, generator=g, dtype=torch.float32).bfloat16()
    emb = big.encode_image(pixels, out_dtype=torch.float32).cpu().numpy()
    assert emb.shape == (chunk, cfg.embed_dim) and np.isfinite(emb).all()
    del big
    torch.cuda.empty_cache()

    sample = sample_frames(chunk, S, W)
    idx = torch.tensor(sample, device=gpu)
    got = emb[sample]

    # the same pixels in 8-frame chunks (the full last block, M = 8 S rows)
    small = _model(name, gpu, image_chunk=8, weights=wts)
    got8 = small.encode_image(pixels[idx], out_dtype=torch.float32).cpu().numpy()
    del small
    c8 = cosine(got, got8)

    # the full last block at the same pass size (A/B build)
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_CLS_LAST", "0")
    full_m = _model(name, gpu, image_chunk=chunk, weights=wts)
    full = full_m.encode_image(pixels, out_dtype=torch.float32).cpu().numpy()
    del full_m
    monkeypatch.undo()
    torch.cuda.empty_cache()

    # float64 truth of the sampled frames (the bf16 pixels' exact values, as the GPU reads them)
    px = pixels[idx].float().cpu().numpy()
    ref = clip_ref.encode_image(px, state_dict(name), cfg, np.float64)
    cos = cosine(got, ref)
    print(f"{name} {wts}: chunk {chunk} (M = {chunk * S}), frames {sample}; 1 - cos vs fp64 max "
          f"{1 - cos.min():.3e}; vs 8-frame chunks max {1 - c8.min():.3e}; "
          f"full last block max |diff| {np.abs(emb - full).max():.3e}")
    assert np.all(cos > 1 - COS_TOL), dict(zip(sample, (1 - cos).tolist()))
    dg, dr = got - got.mean(0), ref - ref.mean(0)
    dcos = cosine(dg, dr).min()
    print(f"{name} {wts}: deviation cosine (frame-to-frame differences) min {dcos:.4f}")
    # bf16: the deviations themselves within 0.99 (test_gpu_encode's bound).  MX-fp8 (e4m3: 3
    # mantissa bits for weights and activations) keeps the north star's 1 - cos <= 1e-3 on the
    # embeddings (6.5e-4 here) but not on the small frame-to-frame differences of random pixels
    # under random weights: 0.88 measured (r6a); the floor guards against a regression only
    assert dcos > (0.99 if wts == "bf16" else 0.85)
    assert np.array_equal(got.view(np.int32), got8.view(np.int32)), dict(zip(sample, (1 - c8).tolist()))
    assert np.array_equal(emb.view(np.int32), full.view(np.int32))


def test_configs2_l14_bf16_bench_pass(gpu, monkeypatch):
    """BASELINE configs[2]: ViT-L/14 bf16, 100k frames -> 1924-frame passes."""
    _run_config(gpu, monkeypatch, "ViT-L/14", 100_000, "bf16")


def test_configs4_l14_336_fp8_bench_pass(gpu, monkeypatch):
    """BASELINE configs[4]: ViT-L/14@336px MX-fp8, a 125k-frame shard -> 863-frame passes."""
    _run_config(gpu, monkeypatch, "ViT-L/14@336px", 125_000, "fp8")


@pytest.mark.parametrize("wts", ["bf16", "fp8", "fp32"])
def test_cls_last_bit_identical_s197(gpu, monkeypatch, wts):
    """the CLS-row last block with S > 64 (ViT-B/16, 197 tokens: the
    resident-K/V attention kernel for bf16 / fp8, the scalar f32 kernel for the
    fp32 tower, on stale non-CLS Q rows) equals the full block bit for bit at
    260 frames (>= 256: the CLS-row path), and 8-frame chunks give the same rows."""
    import torch
    from miclip import _native, config, weights
    name, n = "ViT-B/16", 260
    cfg = config.get_config(name)
    px = torch.from_numpy(weights.synthetic_pixels(n, cfg.image_resolution, seed=197)).to(gpu).bfloat16()
    got = _model(name, gpu, image_chunk=n, weights=wts).encode_image(px).cpu().numpy()
    assert np.isfinite(got).all()
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_CLS_LAST", "0")
    full = _model(name, gpu, image_chunk=n, weights=wts).encode_image(px).cpu().numpy()
    monkeypatch.undo()
    assert np.array_equal(got.view(np.int32), full.view(np.int32)), np.abs(got - full).max()
    pick = torch.tensor([0, 1, 129, 258, 259], device=gpu)
    small = _model(name, gpu, image_chunk=8, weights=wts).encode_image(px[pick]).cpu().numpy()
    assert np.array_equal(got[pick.cpu().numpy()].view(np.int32), small.view(np.int32))
