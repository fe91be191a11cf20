"""The configuration bench.py times, checked.

bench.py's step at BASELINE configs[1] embeds 10 000 ViT-B/32 frames as ONE
500 000-row pass (image_chunk = 10000, bench.py `chunk`), encodes 32 token
rows and ranks top-10 (reference call sites: Backend/services/
embedding_service.py:461-495 encodes a whole folder's frames as one batch
stack, :314-320 ranks).  At that size the pass runs 1954 M-tiles per GEMM,
the persistent kernels' grouped / XCD-ranged tile walk, the fused-residual
epilogues, and byte offsets into `mlp` / `qkv` past 2^31.  This test runs
that pass through the product library and checks:

  * sampled frames against the float64 oracle (oracle/clip_ref.py, 1 - cos <=
    1e-3, the north star's bound, plus the deviation cosine of test_gpu_encode);
  * the same frames against an encode of the same pixels in 8-frame chunks
    (400 rows: two M-tiles, no offset above 2^27): bit-identical, since every
    kernel's per-row arithmetic is independent of M and of the tile walk
    (measured: max difference 0, profiles/r05_a_pytest_bench_config.log);
  * the 10k x 32 top-10 against float64 scores of the same rows
    (rank_ref.assert_topk_equivalent: identical except float64 near-ties).

Sampled frames (S = 50 rows each, 256-row M-tiles): the first tile (0, 1),
the first tile boundary (5 spans rows 250-299), the qkv GEMM's first XCD
range end (m-block 244, frame 1250), c_fc's first XCD range end (m-block 488
split over two XCDs, frames 2499-2503), the middle, the 2^31-byte crossing of
`mlp` ([M, 3072] bf16: row 349525, frame 6990) and of `qkv` ([M, 2304] bf16:
row 466033, frame 9320), and the last, partial M-tile (frames 9998, 9999:
tile 1953 holds rows 499968-499999 of 500000)."""
import numpy as np
import pytest

from conftest import state_dict

pytestmark = pytest.mark.gpu

COS_TOL = 1e-3
FRAMES, QUERIES, K = 10_000, 32, 10
SAMPLE = [0, 1, 5, 6, 1249, 1250, 2499, 2500, 4999, 6990, 6991, 7777, 9320, 9321, 9998, 9999]


def test_bench_configs1_single_pass_vs_oracle(gpu):
    import torch
    from miclip import config, model as M, retrieval, weights
    from oracle import clip_ref, rank_ref
    from oracle.clip_ref import cosine
    name = "ViT-B/32"
    cfg = config.get_config(name)
    sd = state_dict(name)
    big = M.CLIP(cfg, sd, device=gpu, image_chunk=FRAMES)
    assert big._chunks[0] == FRAMES                    # one 500k-row pass, as bench.py runs it
    g = torch.Generator(device=gpu).manual_seed(1234)  # bench.py's generator (rank 0)
    R = cfg.image_resolution
    pixels = torch.randn(FRAMES, 3, R, R, device=gpu, generator=g, dtype=torch.float32).bfloat16()
    tokens = torch.from_numpy(weights.synthetic_tokens(QUERIES, cfg.context_length, cfg.vocab_size)).to(gpu)

    emb = big.encode_image(pixels, out_dtype=torch.float32)
    txt = big.encode_text(tokens, normalize=True, out_dtype=torch.float32)
    top_s, top_i = retrieval.rank_topk(emb, txt, K)
    torch.cuda.synchronize()
    emb_h = emb.cpu().numpy()
    assert emb_h.shape == (FRAMES, cfg.embed_dim) and np.isfinite(emb_h).all()

    # sampled frames vs float64 truth (the bf16 pixels' exact values, as the GPU reads them)
    idx = torch.tensor(SAMPLE, device=gpu)
    px = pixels[idx].float().cpu().numpy()
    ref = clip_ref.encode_image(px, sd, cfg, np.float64)
    got = emb_h[SAMPLE]
    cos = cosine(got, ref)
    assert np.all(cos > 1 - COS_TOL), dict(zip(SAMPLE, (1 - cos).tolist()))
    dg, dr = got - got.mean(0), ref - ref.mean(0)
    assert cosine(dg, dr).min() > 0.99

    # the same pixels in 8-frame chunks (two 400-row passes)
    del big
    torch.cuda.empty_cache()
    small = M.CLIP(cfg, sd, device=gpu, image_chunk=8)
    got8 = small.encode_image(pixels[idx], out_dtype=torch.float32).cpu().numpy()
    c8 = cosine(got, got8)
    rel = np.abs(got - got8).max() / np.abs(got8).max()
    print(f"single pass vs 8-frame chunks: 1 - cos max {1 - c8.min():.3e}, max rel diff {rel:.3e}; "
          f"vs fp64 1 - cos max {1 - cos.min():.3e}")
    assert np.array_equal(got, got8), (1 - c8).tolist()

    # the timed step's ranking against float64 scores of the same rows
    S = rank_ref.scores_ref(emb_h, txt.cpu().numpy())
    ts, ti = top_s.cpu().numpy(), top_i.cpu().numpy()
    swaps = sum(rank_ref.assert_topk_equivalent(ts[q], ti[q], S[q], K) for q in range(QUERIES))
    assert swaps <= 2
