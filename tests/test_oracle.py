"""CPU: the oracle against the golden vectors (HF-pinned encoders, the
reference's committed corpus for ranking) — pins the checker before any GPU
result is judged against it."""
import numpy as np
import pytest

from conftest import golden, state_dict


@pytest.mark.parametrize("name,fname", [("test-tiny", "test_tiny.npz"), ("test-small", "test_small.npz"),
                                        ("ViT-B/32", "vit_b32.npz")])
def test_encoder_oracle_matches_hf_golden(name, fname):
    from miclip import config, weights
    from oracle import clip_ref
    cfg = config.get_config(name)
    g = golden(fname)
    sd = state_dict(name)
    px = weights.synthetic_pixels(int(g["n_images"]), cfg.image_resolution)
    img = clip_ref.encode_image(px, sd, cfg, np.float32)
    txt = clip_ref.encode_text(g["tokens"], sd, cfg, np.float32)
    np.testing.assert_allclose(img, g["image"], rtol=0, atol=2e-5 * np.abs(g["image"]).max())
    np.testing.assert_allclose(txt, g["text"], rtol=0, atol=2e-5 * np.abs(g["text"]).max())
    assert 1 - clip_ref.cosine(img, g["image"]).min() < 1e-9


@pytest.mark.slow
def test_l14_oracle_matches_hf_golden():
    from miclip import config, weights
    from oracle import clip_ref
    cfg = config.get_config("ViT-L/14")
    g = golden("vit_l14.npz")
    sd = weights.make_state_dict(cfg)
    px = weights.synthetic_pixels(int(g["n_images"]), cfg.image_resolution)
    img = clip_ref.encode_image(px, sd, cfg, np.float32)
    assert 1 - clip_ref.cosine(img, g["image"]).min() < 1e-9


def test_tokens_regenerate_bit_exactly():
    from miclip import weights
    g = golden("vit_b32.npz")
    assert np.array_equal(weights.synthetic_tokens(4), g["tokens"])


def test_weight_generator_is_pinned():
    """Counter-based generator: fixed values regardless of host (exact integer
    arithmetic + correctly rounded IEEE ops)."""
    from miclip import weights
    x = weights.normal(2, "visual.proj", (4,), 0.036)
    assert x.dtype == np.float32
    y = weights.normal(2, "visual.proj", (4,), 0.036)
    assert np.array_equal(x, y)
    z = weights.normal(2, "visual.proj", ((1 << 22) + 5,), 1.0)
    assert abs(float(z.mean())) < 2e-3 and abs(float(z.std()) - 1) < 2e-3
    assert np.array_equal(z[:4], weights.normal(2, "visual.proj", (4,), 1.0))
    assert np.array_equal(z[-3:], weights.normal(2, "visual.proj", ((1 << 22) + 5,), 1.0)[-3:])


def test_search_top_frames_restatement_on_reference_corpus():
    """Literal search_top_frames (argsort[::-1] + stable re-sort) == the
    deterministic (score desc, index asc) rule on the reference's corpus."""
    from oracle import rank_ref
    g = golden("rank_video_test_4.npz")
    corpus, q, k = g["corpus"], g["queries"], int(g["k"])
    s, i = rank_ref.topk_ref(corpus, q, k)
    assert np.array_equal(i, g["top_index"])
    frames = [f"{j}.jpg" for j in range(corpus.shape[0])]
    for r in range(q.shape[0]):
        names, _ = rank_ref.search_top_frames_ref(corpus, q[r:r + 1], k, frames)
        assert names == [frames[j] for j in g["top_index"][r]]


def test_rk_restatement():
    from oracle import rank_ref
    g = golden("rk_flow.npz")
    ref = rank_ref.retrieval_metrics_ref(g["image_features"], g["text_features"], list(g["caption_image_ids"]),
                                         list(g["image_ids"]))
    assert np.array_equal(ref["t2i_ranks"], g["t2i_ranks"])
    assert np.array_equal(ref["i2t_ranks"], g["i2t_ranks"])
    # the stable count-greater rule equals argsort(-s) on tie-free fixtures
    S = g["image_features"].astype(np.float64) @ g["text_features"].T.astype(np.float64)
    for t in range(0, 500, 37):
        assert rank_ref.rank_of_target_ref(S[:, t], g["caption_image_ids"][t]) == g["t2i_ranks"][t]


def test_topk_ref_edge_cases():
    from oracle import rank_ref
    rng = np.random.default_rng(3)
    C = rng.standard_normal((20, 32))
    C[4] = 0
    q = rng.standard_normal((1, 32))
    s, i = rank_ref.topk_ref(C, q, 5, nan_policy="first")
    assert i[0, 0] == 4 and np.isnan(s[0, 0])
    s, i = rank_ref.topk_ref(C, q, 25, nan_policy="last")
    assert i.shape == (1, 20) and i[0, -1] == 4
    s, i = rank_ref.topk_ref(C, q, 3, index_base=100)
    assert (i >= 100).all()


@pytest.mark.parametrize("name,fname", [("test-small", "test_small.npz"), ("ViT-B/32", "vit_b32.npz")])
def test_torch_cpu_restatement_matches_golden(name, fname):
    """oracle/clip_torch.py (the torch-CPU fp32 form the CPU baseline times,
    BASELINE.md) against the same HF-pinned goldens."""
    from miclip import config, weights
    from oracle import clip_ref, clip_torch
    cfg = config.get_config(name)
    g = golden(fname)
    m = clip_torch.TorchCLIP(state_dict(name), cfg)
    px = weights.synthetic_pixels(int(g["n_images"]), cfg.image_resolution)
    img = np.concatenate([m.encode_image(px[i:i + 1]) for i in range(px.shape[0])])   # batch 1, embedding.py:46-50
    txt = m.encode_text(g["tokens"])
    np.testing.assert_allclose(img, g["image"], rtol=0, atol=5e-5 * np.abs(g["image"]).max())
    np.testing.assert_allclose(txt, g["text"], rtol=0, atol=5e-5 * np.abs(g["text"]).max())
    assert 1 - clip_ref.cosine(img, g["image"]).min() < 1e-8


def _f16_rows(rng, R, D):
    X = (rng.standard_normal((R, D)) * np.exp(rng.uniform(-7, 2.5, (R, D)))).astype(np.float16)
    X[0] = 0                                         # zero row -> NaN (0/0)
    X[1, :] = np.float16(6e-8)                        # f16 subnormal squares -> 0
    X[2, 0] = np.float16(200.0)                       # square overflows f16 -> inf norm -> 0 / NaN
    X[3, min(5, D - 1)] = np.float16(np.nan)
    if R > 8:
        X[8:, 0] = rng.uniform(31, 45, R - 8).astype(np.float16)   # one dominant square: exercises the tree order
    return X


@pytest.mark.parametrize("D", [1, 7, 8, 32, 96, 130, 512, 544, 768, 992, 1024])
def test_f16_norm_plan_matches_numpy(D):
    """The float16 row normalisation csrc/corpus.hip replays (oracle
    rank_ref.normalize_rows_f16) is NumPy's own float16 evaluation of
    embedding_service.py:209-210, bit for bit (NaN positions included)."""
    from oracle import rank_ref
    rng = np.random.default_rng(D)
    X = _f16_rows(rng, 4000 if D <= 544 else 1500, D)
    with np.errstate(all="ignore"):
        ref = X / np.linalg.norm(X, axis=-1, keepdims=True)
    got = rank_ref.normalize_rows_f16(X)
    assert ref.dtype == np.float16 and got.dtype == np.float16
    nan = np.isnan(ref)
    assert np.array_equal(nan, np.isnan(got))
    assert np.array_equal(ref.view(np.uint16)[~nan], got.view(np.uint16)[~nan])
    leaves, _ = rank_ref.pairwise_plan(D)
    assert len(leaves) <= 8                           # one lane per strided accumulator in the kernel


def test_f16_plan_initial_value_is_identity():
    """The half add-reduce starts from the identity 0 and sums all D squares
    pairwise (not x_0 + pairwise(x_1..)): rows built so that the two differ."""
    from oracle import rank_ref
    rng = np.random.default_rng(1)
    X = (rng.standard_normal((200000, 512)) * 0.03).astype(np.float16)
    X[:, 0] = rng.uniform(31, 45, X.shape[0]).astype(np.float16)
    with np.errstate(all="ignore"):
        ref = X / np.linalg.norm(X, axis=-1, keepdims=True)
    assert np.array_equal(ref.view(np.uint16), rank_ref.normalize_rows_f16(X).view(np.uint16))


def test_fp16_reference_corpus_fixture():
    """tests/golden/rank_video_test_3.npz (the reference's float16 default
    corpus, video_test_3 == image_embeddings.npy byte for byte): the stored
    normalised rows are NumPy's, the frame lists are the literal
    search_top_frames restatement, and that literal answer equals the
    (score desc, index asc) order of the exact scores of those float16 rows."""
    from oracle import rank_ref
    g = golden("rank_video_test_3.npz")
    raw, q = g["corpus"], g["queries"]
    assert raw.dtype == np.float16 and bool(g["image_embeddings_identical"])
    E16 = rank_ref.normalize_rows(raw)
    assert np.array_equal(E16.view(np.uint16), g["normalized"].view(np.uint16))
    assert np.array_equal(rank_ref.normalize_rows_f16(raw).view(np.uint16), g["normalized"].view(np.uint16))
    frames = [f"{i}.jpg" for i in range(raw.shape[0])]
    for r in range(0, q.shape[0], 23):
        _, idx = rank_ref.search_top_frames_ref(raw, q[r:r + 1], 60, frames)
        assert np.array_equal(np.asarray(idx[:60]), g["top_index_60"][r])
    _, exact = rank_ref.topk_ref(E16.astype(np.float64), q, 60, norm="none")
    assert np.array_equal(exact, g["top_index_60"])
    assert np.array_equal(exact[:, :10], g["top_index_10"])
