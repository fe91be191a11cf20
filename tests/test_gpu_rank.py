"""Fused normalise + cosine + top-k kernel, merge, score matrix and
rank-of-target vs the NumPy restatement of the reference ranking
(embedding_service.py:314-320, compare_models.py:994-1090)."""
import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _t(a, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


@pytest.mark.parametrize("N,D,Q,k", [(1, 512, 1, 10), (9, 512, 3, 10), (49, 512, 1, 60), (1000, 512, 32, 10),
                                     (10000, 512, 32, 10), (4097, 768, 33, 16), (20000, 128, 5, 64),
                                     (300, 1024, 70, 1)])
def test_topk_matches_oracle(gpu, N, D, Q, k):
    from miclip import retrieval, weights
    from oracle import rank_ref
    corpus = weights.normal(11, f"c{N}", (N, D))          # un-normalised rows
    q = weights.synthetic_corpus(Q, D, seed=12)
    s, i = retrieval.rank_topk(_t(corpus, gpu), _t(q, gpu), k)
    S = rank_ref.scores_ref(corpus, q)
    assert s.shape == (Q, min(k, N))
    for r in range(Q):
        rank_ref.assert_topk_equivalent(s[r].cpu().numpy(), i[r].cpu().numpy(), S[r], k)


@pytest.mark.parametrize("dtype", ["bf16", "f16"])
def test_topk_half_corpus(gpu, dtype):
    """bf16/fp16 corpus rows are ranked on their exact f32 values."""
    import torch
    from miclip import retrieval, weights
    from oracle import rank_ref
    corpus = weights.normal(13, "half", (3000, 512))
    tdt = torch.bfloat16 if dtype == "bf16" else torch.float16
    c = torch.from_numpy(corpus).to(tdt)
    q = weights.synthetic_corpus(8, 512, seed=14)
    s, i = retrieval.rank_topk(c.to(gpu), _t(q, gpu), 10)
    S = rank_ref.scores_ref(c.float().numpy(), q)
    for r in range(8):
        rank_ref.assert_topk_equivalent(s[r].cpu().numpy(), i[r].cpu().numpy(), S[r], 10)


@pytest.mark.parametrize("D", [1, 7, 32, 96, 130, 512, 544, 768, 992, 1024])
def test_normalize_rows_f16_bit_identical_to_numpy(gpu, D):
    """mi_normalize_rows_f16 == NumPy's float16 `E / np.linalg.norm(E, axis=-1,
    keepdims=True)` (embedding_service.py:209-210) bit for bit, NaN rows
    included, out of place and in place."""
    import torch
    from miclip import retrieval
    from test_oracle import _f16_rows
    X = _f16_rows(np.random.default_rng(100 + D), 3001, D)
    with np.errstate(all="ignore"):
        ref = X / np.linalg.norm(X, axis=-1, keepdims=True)
    t = _t(X, gpu)
    got = retrieval.normalize_rows_f16(t).cpu().numpy()
    nan = np.isnan(ref)
    assert np.array_equal(nan, np.isnan(got))
    assert np.array_equal(ref.view(np.uint16)[~nan], got.view(np.uint16)[~nan])
    retrieval.normalize_rows_f16(t, out=t)
    assert np.array_equal(np.isnan(t.cpu().numpy()), nan)
    assert np.array_equal(t.cpu().numpy().view(np.uint16)[~nan], ref.view(np.uint16)[~nan])
    e = torch.zeros(0, D, dtype=torch.float16, device=gpu)
    assert retrieval.normalize_rows_f16(e).shape == (0, D)


def test_reference_fp16_corpus_fixture(gpu):
    """The app's default corpus, the reference's float16 file
    Backend/embedding/video_test_3_embeddings.npy (== image_embeddings.npy):
    rows normalised on the device in NumPy's float16 arithmetic (bit-identical
    to the fixture's NumPy rows), ranked as stored against f32 text vectors:
    identical frame lists to the literal search_top_frames restatement for
    all 200 queries at k = 10 and k = 60 (fixture: make_golden.py --fp16-rank).
    A query whose literal answer hinges on a float64 gap < 2e-7 between
    consecutive top scores (the host BLAS's summation order decides those) may
    swap exactly those two rows; none may differ otherwise."""
    import torch
    from miclip import retrieval
    from oracle import rank_ref
    g = golden("rank_video_test_3.npz")
    raw, q = g["corpus"], g["queries"]
    E = retrieval.normalize_rows_f16(_t(raw, gpu))
    assert E.dtype == torch.float16
    assert np.array_equal(E.cpu().numpy().view(np.uint16), g["normalized"].view(np.uint16))
    S = q.astype(np.float64) @ g["normalized"].astype(np.float64).T
    swaps = 0
    for k in (10, 60):
        s, i = retrieval.rank_topk(E, _t(q, gpu), k, norm="none")
        i = i.cpu().numpy()
        ref = g[f"top_index_{k}"]
        for r in range(q.shape[0]):
            if np.array_equal(i[r], ref[r]):
                continue
            assert g[f"gap_{k}"][r] < 2e-7, (k, r, i[r], ref[r])
            swaps += rank_ref.assert_topk_equivalent(s[r].cpu().numpy(), i[r], S[r], k, tol=2e-7)
        exp = np.take_along_axis(S, i, 1)
        assert np.allclose(s.cpu().numpy(), exp, rtol=0, atol=2e-6)
    assert swaps <= 2


def test_topk_nan_rows_and_ties(gpu):
    from miclip import retrieval
    from oracle import rank_ref
    rng = np.random.default_rng(0)
    corpus = rng.standard_normal((500, 512)).astype(np.float32)
    corpus[[3, 77, 400]] = 0.0                 # zero rows -> NaN scores
    corpus[10] = corpus[20]                    # exact duplicate rows -> exact tie
    q = rng.standard_normal((2, 512)).astype(np.float32)
    q[1] = corpus[20] / np.linalg.norm(corpus[20])
    for pol in ("first", "last"):
        s, i = retrieval.rank_topk(_t(corpus, gpu), _t(q, gpu), 12, nan_policy=pol)
        rs, ri = rank_ref.topk_ref(corpus, q, 12, nan_policy=pol)
        s, i = s.cpu().numpy(), i.cpu().numpy()
        if pol == "first":
            assert list(i[0, :3]) == [3, 77, 400] and np.isnan(s[0, :3]).all()
        assert list(i[1, :2] if pol == "last" else i[1, 3:5]) == [10, 20]   # tie -> index asc
        for r in range(2):
            rank_ref.assert_topk_equivalent(s[r], i[r], rank_ref.scores_ref(corpus, q)[r], 12, nan_policy=pol)


def test_topk_index_base_and_empty(gpu):
    import torch
    from miclip import retrieval, weights
    corpus = weights.synthetic_corpus(100, 512)
    q = corpus[5:7]
    s, i = retrieval.rank_topk(_t(corpus, gpu), _t(q, gpu), 3, index_base=1_000_000)
    assert i[0, 0].item() == 1_000_005 and i[1, 0].item() == 1_000_006
    e = torch.zeros(0, 512, device=gpu)
    s, i = retrieval.rank_topk(e, _t(q, gpu), 5)
    assert s.shape == (2, 0)


def test_merge_matches_oracle(gpu):
    from miclip import retrieval
    from oracle import rank_ref
    rng = np.random.default_rng(1)
    Q, C, k = 7, 8 * 10, 10
    cs = rng.standard_normal((Q, C)).astype(np.float32)
    ci = rng.permutation(10_000)[:Q * C].reshape(Q, C).astype(np.int64)
    ci[0, :5] = -1
    cs[1, 3] = np.nan
    for pol in ("first", "last"):
        s, i = retrieval.merge_topk(_t(cs, gpu), _t(ci, gpu), k, nan_policy=pol)
        rs, ri = rank_ref.merge_ref(cs, ci, k, nan_policy=pol)
        assert np.array_equal(i.cpu().numpy(), ri)
        assert np.allclose(s.cpu().numpy(), rs, equal_nan=True)


def test_score_matrix_and_ranks(gpu):
    from miclip import evaluate, retrieval, weights
    from oracle import rank_ref
    img = weights.synthetic_corpus(200, 512, seed=21)
    txt = weights.synthetic_corpus(1000, 512, seed=22)
    S = retrieval.score_matrix(_t(img, gpu), _t(txt, gpu)).cpu().numpy()     # [T, I]
    assert np.allclose(S, (txt.astype(np.float64) @ img.T.astype(np.float64)), atol=2e-6)
    cap_ids = [j // 5 for j in range(1000)]
    res = evaluate.retrieval_metrics(_t(img, gpu), _t(txt, gpu), cap_ids, list(range(200)))
    ref = rank_ref.retrieval_metrics_ref(img, txt, cap_ids, list(range(200)))
    assert np.array_equal(res["t2i_ranks"], ref["t2i_ranks"])
    assert np.array_equal(res["i2t_ranks"], ref["i2t_ranks"])
    for d in ("t2i", "i2t", "mean"):
        for m, v in ref[d].items():
            assert res[d][m] == pytest.approx(v, abs=0), (d, m)


def test_reference_corpus_fixture(gpu):
    """The reference's own committed encode_image outputs
    (Backend/embedding/video_test_4_embeddings.npy, fp32 un-normalised) ranked
    for synthetic text vectors: identical frame lists to the literal
    search_top_frames restatement (fixture generated by make_golden.py)."""
    from miclip import retrieval
    g = golden("rank_video_test_4.npz")
    corpus, queries = g["corpus"], g["queries"]
    s, i = retrieval.rank_topk(_t(corpus, gpu), _t(queries, gpu), int(g["k"]))
    assert np.array_equal(i.cpu().numpy(), g["top_index"])
    assert np.allclose(s.cpu().numpy(), g["top_score"], atol=2e-6)


def test_reference_flow_rk_fixture(gpu):
    """R@K flow on the reference's committed embeddings (frames as 'images',
    noisy copies as 'captions'): ranks and R@1/5/10 identical to the literal
    compare_models.py restatement."""
    from miclip import evaluate
    g = golden("rk_flow.npz")
    res = evaluate.retrieval_metrics(_t(g["image_features"], gpu), _t(g["text_features"], gpu),
                                     list(g["caption_image_ids"]), list(g["image_ids"]))
    assert np.array_equal(res["t2i_ranks"], g["t2i_ranks"])
    assert np.array_equal(res["i2t_ranks"], g["i2t_ranks"])
    for d, arr in (("t2i", g["t2i_r"]), ("i2t", g["i2t_r"])):
        assert [res[d]["R@1"], res[d]["R@5"], res[d]["R@10"]] == list(arr)


@pytest.mark.parametrize("N,D,Q,k,dt", [(20000, 512, 32, 10, "f32"), (4097, 768, 7, 8, "f32"), (4097, 768, 7, 16, "f32"),
                                        (500, 512, 3, 60, "f32"),
                                        (3, 512, 2, 10, "f32"), (33, 768, 40, 1, "f32"), (70001, 512, 5, 16, "f16"),
                                        (9000, 768, 33, 10, "bf16"), (1000, 256, 4, 10, "f32")])
def test_mirrored_corpus_matches_exact(gpu, N, D, Q, k, dt):
    """fp16 mirror + exact re-score == the exact pass over the master, bit for
    bit (§8(f) item 2): certified queries from the mirror, the rest (and
    k > 12, D outside {512, 768}) from the exact pass."""
    import torch
    from miclip import retrieval, weights
    tdt = {"f32": torch.float32, "f16": torch.float16, "bf16": torch.bfloat16}[dt]
    corpus = _t(weights.normal(21, f"m{N}", (N, D)), gpu).to(tdt)
    q = _t(weights.synthetic_corpus(Q, D, seed=22), gpu)
    mc = retrieval.MirroredCorpus(corpus)
    s, i = mc.topk(q, k)
    s0, i0 = retrieval.rank_topk(corpus, q, k)
    assert s.shape == s0.shape
    assert (i.cpu() == i0.cpu()).all()
    assert (s.cpu() == s0.cpu()).all()
    if k <= retrieval.MirroredCorpus.MAX_K and D in (512, 768):
        assert mc.certified >= Q - 1      # random corpora: the certificate holds


def test_mirrored_corpus_edge_cases(gpu):
    """index_base, NaN rows (zero rows: NaN first -> uncertified -> exact pass;
    NaN last -> certified past them), nan_policy, mirror of the real corpus."""
    import torch
    from miclip import retrieval, weights
    g = golden("rank_video_test_4.npz")
    rows = np.array(g["corpus"], dtype=np.float32)
    q = _t(weights.synthetic_corpus(6, rows.shape[1], seed=25), gpu)
    for zero in (False, True):
        c = rows.copy()
        if zero:
            c[[3, 100]] = 0.0
        corpus = _t(c, gpu)
        for pol in ("first", "last"):
            mc = retrieval.MirroredCorpus(corpus)
            s, i = mc.topk(q, 10, nan_policy=pol, index_base=1000)
            s0, i0 = retrieval.rank_topk(corpus, q, 10, index_base=1000, nan_policy=pol)
            assert (i.cpu() == i0.cpu()).all() and torch.equal(s.cpu().view(torch.int32), s0.cpu().view(torch.int32)), (zero, pol)
            if zero and pol == "first":
                assert mc.fallbacks == 6


def test_mirrored_corpus_near_ties_fall_back(gpu):
    """Rows that tie in fp16 across the candidate edge fail the certificate and
    take the exact path; the answer is still the f32 one."""
    import torch
    from miclip import retrieval, weights
    base = weights.normal(23, "tie", (1, 512))
    rows = np.repeat(base, 400, axis=0) + weights.normal(24, "eps", (400, 512)) * 1e-4   # near-duplicates
    corpus = _t(rows, gpu)
    q = torch.from_numpy(base / np.linalg.norm(base)).to(gpu)
    mc = retrieval.MirroredCorpus(corpus)
    s, i = mc.topk(q, 10)
    s0, i0 = retrieval.rank_topk(corpus, q, 10)
    assert (i.cpu() == i0.cpu()).all() and (s.cpu() == s0.cpu()).all()
    assert mc.fallbacks == 1


@pytest.mark.parametrize("N,k,pol", [(3000, 65, "first"), (3000, 3000, "last"), (20000, 1000, "first"),
                                     (20000, 8192, "last"), (20000, 9000, "first"), (20000, 20000, "first"),
                                     (20000, 25000, "last"), (1, 100, "first")])
def test_topk_large_k_select_path(gpu, N, k, pol):
    """k > 64: exact scores + radix select + bitonic chunks + merge-path passes
    (rank.hip).  Zero rows (NaN), groups of duplicated rows (exact ties at
    every position, index ascending) and k >= N (a full sort, the reference's
    argsort(s)[::-1] when top_k >= N, embedding_service.py:317-318)."""
    from miclip import retrieval, weights
    from oracle import rank_ref
    corpus = weights.normal(21, f"large{N}", (N, 256))
    if N > 10:
        corpus[[5, N // 2, N - 1]] = 0.0
        for a in range(0, N - 20, max(1, N // 37)):
            corpus[a + 7] = corpus[a]                      # exact ties
    q = weights.synthetic_corpus(3, 256, seed=22)
    s, i = retrieval.rank_topk(_t(corpus, gpu), _t(q, gpu), k, nan_policy=pol)
    kk = min(k, N)
    assert s.shape == (3, kk)
    S = rank_ref.scores_ref(corpus, q)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    for r in range(3):
        rank_ref.assert_topk_equivalent(s[r], i[r], S[r], kk, nan_policy=pol)
        # ties and NaNs: where float64 scores are EQUAL the order is index ascending, exactly
        for p in range(kk - 1):
            a, b = S[r][i[r][p]], S[r][i[r][p + 1]]
            if a == b or (np.isnan(a) and np.isnan(b)):
                assert i[r][p] < i[r][p + 1]


def test_topk_large_k_matches_fused_path_prefix(gpu):
    """The select path and the fused single pass agree on the first 64."""
    from miclip import retrieval, weights
    corpus = _t(weights.normal(23, "pref", (50000, 512)), gpu)
    q = _t(weights.synthetic_corpus(32, 512, seed=24), gpu)
    s1, i1 = retrieval.rank_topk(corpus, q, 64)
    s2, i2 = retrieval.rank_topk(corpus, q, 500)
    assert np.array_equal(i1.cpu().numpy(), i2[:, :64].cpu().numpy())
    assert np.array_equal(s1.cpu().numpy(), s2[:, :64].cpu().numpy())


def test_mirror_large_corpus_ties_nan(gpu):
    """300k rows: the mirror path == the exact pass, including exact ties
    between rows and later duplicates (index ascending) and a NaN row, for
    both NaN policies."""
    import torch
    from miclip import retrieval, weights
    c = weights.normal(31, "seed", (300_000, 512))
    c[200_000:200_100] = c[0:100]                   # later duplicates: ties, index ascending
    c[250_000] = 0.0                                # a NaN row
    corpus = _t(c, gpu)
    q = _t(np.concatenate([weights.synthetic_corpus(30, 512, seed=32), c[[5, 77]]]), gpu)
    mc = retrieval.MirroredCorpus(corpus)
    for pol in ("first", "last"):
        s1, i1 = mc.topk(q, 10, nan_policy=pol)
        s0, i0 = retrieval.rank_topk(corpus, q, 10, nan_policy=pol)
        assert torch.equal(i1, i0)
        assert torch.equal(s1.view(torch.int32), s0.view(torch.int32))
    assert mc.certified >= 30   # NaN-last: certified; NaN-first: the NaN row is a candidate -> exact pass


@pytest.mark.parametrize("N,Q", [(1, 1), (9, 3), (1000, 32), (10000, 33), (100003, 32)])
def test_rank_reg_nine_slot_ring_bit_identical(gpu, monkeypatch, N, Q):
    """rank_reg's 9-slot / 7-in-flight ring (A/B build, MICLIP_RANK_NB=9), with its LDS
    allocation sized from the same rank_reg_lds_bytes(NB) as the kernel's ring
    (round 2's attempt allocated 8 slots' worth: the norms sat past the end of
    the LDS, read as zeros, and every test failed): bit-identical to the
    default 8-slot ring, including N = 1."""
    import torch
    from miclip import _native, retrieval, weights
    corpus = _t(weights.normal(21, f"nb{N}", (N, 512)), gpu)
    q = _t(weights.synthetic_corpus(Q, 512, seed=22), gpu)
    s8, i8 = retrieval.rank_topk(corpus, q, 10)                    # product library: the 8-slot ring
    monkeypatch.setattr(_native, "lib", _native.lib_ab)             # the A/B build, whose MICLIP_RANK_NB=9 ...
    monkeypatch.setenv("MICLIP_RANK_NB", "9")                       # ... selects rank_reg<512, 9, 7>
    s9, i9 = retrieval.rank_topk(corpus, q, 10)
    torch.cuda.synchronize()
    assert torch.equal(i8, i9) and torch.equal(s8, s9)


@pytest.mark.parametrize("dt", ["bf16", "f16"])
@pytest.mark.parametrize("N,Q", [(1, 1), (77, 3), (4099, 32), (100003, 33)])
def test_rank_reg_half_corpus_bit_identical(gpu, monkeypatch, dt, N, Q):
    """16-bit corpora at D = 512 run rank_reg (64-k ring chunks of bf16 / fp16
    rows, converted exactly to f32 after the fragment read): candidates bit for
    bit those of rank_stream (A/B build, MICLIP_RANK_REG=0), which converts in
    its loads; and the top-k of the oracle's f32 scores of the same values."""
    import torch
    from miclip import _native, retrieval, weights
    from oracle import rank_ref
    tdt = torch.bfloat16 if dt == "bf16" else torch.float16
    c32 = weights.normal(31, f"h{N}", (N, 512))
    c32[N // 2] = 0.0                                                # a zero row: inv_norm's guard
    c = torch.from_numpy(c32).to(tdt).to(gpu)
    q = _t(weights.synthetic_corpus(Q, 512, seed=32), gpu)
    s0, i0 = retrieval.rank_topk(c, q, 10)
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_RANK_REG", "0")
    s1, i1 = retrieval.rank_topk(c, q, 10)
    torch.cuda.synchronize()
    assert torch.equal(i0, i1) and torch.equal(s0.view(torch.int32), s1.view(torch.int32))
    if N <= 5000:
        S = rank_ref.scores_ref(c.float().cpu().numpy(), q.cpu().numpy())
        for r in range(Q):
            rank_ref.assert_topk_equivalent(s0[r].cpu().numpy(), i0[r].cpu().numpy(), S[r], 10)


@pytest.mark.parametrize("D", [512, 768])
@pytest.mark.parametrize("k", [1, 10, 16])
def test_in_launch_merge_mass_ties(gpu, D, k):
    """The in-launch merge (last workgroup of each query block reduces every
    workgroup's top-k above the global k-th-key threshold) under exact ties in
    every workgroup: 200003 rows drawn from 5 distinct vectors and a zero row
    (NaN score), 33 queries (two query blocks).  Identical rows score bit for
    bit alike, so the top-k is the best vector's lowest row indices (NaN rows
    first under nan_policy="first")."""
    from miclip import retrieval
    rng = np.random.default_rng(D + k)
    base = rng.standard_normal((6, D)).astype(np.float32)
    base[5] = 0.0
    N = 200_003
    pick = rng.integers(0, 6, N)
    corpus = base[pick]
    q = rng.standard_normal((33, D)).astype(np.float32)
    sb = (base[:5].astype(np.float64) / np.linalg.norm(base[:5], axis=1, keepdims=True)) @ q.T.astype(np.float64)
    for pol in ("first", "last"):
        s, i = retrieval.rank_topk(_t(corpus, gpu), _t(q, gpu), k, nan_policy=pol)
        i = i.cpu().numpy()
        for r in range(33):
            order = np.argsort(-sb[:, r], kind="stable")
            ranked = [np.flatnonzero(pick == 5)] if pol == "first" else []
            ranked += [np.flatnonzero(pick == v) for v in order]
            want = np.concatenate(ranked)[:k]
            np.testing.assert_array_equal(i[r], want, err_msg=f"query {r} {pol}")


@pytest.mark.parametrize("D", [512, 768])
def test_split_merge_static_frames_no_cliff(gpu, D):
    """a corpus of identical rows (a static video: every frame embeds alike) ties every
    workgroup's whole top-k on one key.  The split merge (rank.hip fold_merge_kernel) cuts on the
    packed (key, ~index) entry, so it appends ~k^2 entries instead of all nlines x k and its
    quadratic rank-by-counting stays small: the call is bit-exact (the k lowest indices, one score)
    and costs no more than ranking a random corpus of the same size, beyond noise.  D = 512 takes
    rank_reg (256 workgroups), D = 768 rank_stream (up to 512)."""
    import torch
    from miclip import retrieval, weights
    N, Q, k = 200_000, 32, 10
    row = weights.normal(61, "static", (1, D))
    same = _t(np.repeat(row, N, axis=0), gpu)
    rand = _t(weights.normal(62, "random", (N, D)), gpu)
    q = _t(weights.synthetic_corpus(Q, D, seed=63), gpu)
    s, i = retrieval.rank_topk(same, q, k)
    torch.cuda.synchronize()
    assert (i.cpu().numpy() == np.arange(k)[None, :]).all()
    sc = s.cpu().numpy()
    assert (sc == sc[:, :1]).all()

    def timed(c, n=20):
        retrieval.rank_topk(c, q, k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            retrieval.rank_topk(c, q, k)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / n
    t_same, t_rand = timed(same), timed(rand)
    print(f"D {D}: identical rows {t_same:.1f} us, random rows {t_rand:.1f} us per call")
    assert t_same < 1.5 * t_rand + 30.0, (t_same, t_rand)


def _ranked_both_ways(monkeypatch, c, q, k, **kw):
    """mi_rank_topk through the A/B build with the certified pass forced on for
    every eligible call (MICLIP_RANK_CERT=2) and switched off (0)."""
    import torch
    from miclip import _native, retrieval
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_RANK_CERT", "2")
    s1, i1 = retrieval.rank_topk(c, q, k, **kw)
    monkeypatch.setenv("MICLIP_RANK_CERT", "0")
    s0, i0 = retrieval.rank_topk(c, q, k, **kw)
    torch.cuda.synchronize()
    return (s1, i1), (s0, i0)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
@pytest.mark.parametrize("N,Q,k", [(1, 1, 1), (15, 3, 10), (16, 2, 12), (17, 5, 12), (1000, 32, 10),
                                   (40003, 33, 1), (100003, 70, 10)])
def test_certified_pass_bit_identical(gpu, monkeypatch, dt, N, Q, k):
    """rank_cert.hip (bf16-MFMA pass over f32 / bf16 rows with q = q1 + q2 and, f32 rows,
    c = c_hi + c_lo; exact re-score of its top-16; certificates; the exact pass gated by
    them) gives the exact pass's results bit for bit: L2 and guarded-L2 norms, NaN
    first / last, fewer rows than candidates, one and three query blocks."""
    import torch
    from miclip import weights
    c32 = weights.normal(41, f"c{N}", (N, 512))
    c = _t(c32, gpu) if dt == "f32" else torch.from_numpy(c32).to(torch.bfloat16).to(gpu)
    q = _t(weights.synthetic_corpus(Q, 512, seed=42), gpu)
    for norm, pol in (("l2", "first"), ("l2_guard", "last")):
        (s1, i1), (s0, i0) = _ranked_both_ways(monkeypatch, c, q, k, norm=norm, nan_policy=pol)
        assert torch.equal(i1, i0), (norm, pol)
        assert torch.equal(s1.view(torch.int32), s0.view(torch.int32)), (norm, pol)


@pytest.mark.parametrize("dt", ["f32", "bf16"])
def test_certified_pass_ties_and_unsafe_rows_fall_back(gpu, monkeypatch, dt):
    """Rows the certificate cannot separate or its bound does not cover go to the exact
    pass: exact duplicates of the best rows (ties across the candidate edge), a row of
    tiny values (sum of squares below 1e-15) and a zero row (NaN score under L2)."""
    import torch
    from miclip import weights
    N, Q = 50_000, 40
    c32 = weights.normal(43, "ties", (N, 512))
    q32 = weights.synthetic_corpus(Q, 512, seed=44)
    c32[100:140] = c32[7]                       # 41 identical rows: ties at every k
    c32[-5:] = q32[:5] * 3.0                     # rows parallel to queries 0..4
    for extra in ("none", "tiny", "zero"):
        cc = c32.copy()
        if extra == "tiny":
            cc[1234] = 1e-9
        elif extra == "zero":
            cc[1234] = 0.0
        c = _t(cc, gpu) if dt == "f32" else torch.from_numpy(cc).to(torch.bfloat16).to(gpu)
        for pol in ("first", "last"):
            (s1, i1), (s0, i0) = _ranked_both_ways(monkeypatch, c, _t(q32, gpu), 12, nan_policy=pol)
            assert torch.equal(i1, i0), (extra, pol)
            assert torch.equal(s1.view(torch.int32), s0.view(torch.int32)), (extra, pol)


def test_certified_pass_product_default_large_corpus(gpu, monkeypatch):
    """The product library routes f32 / bf16 corpora of >= 262144 rows (D = 512, k <= 12)
    through the certified pass: identical to the A/B build's exact pass."""
    import torch
    from miclip import _native, retrieval, weights
    c = _t(weights.normal(45, "big", (300_001, 512)), gpu)
    q = _t(weights.synthetic_corpus(32, 512, seed=46), gpu)
    for cc in (c, c.bfloat16()):
        s1, i1 = retrieval.rank_topk(cc, q, 10)
        monkeypatch.setattr(_native, "lib", _native.lib_ab)
        monkeypatch.setenv("MICLIP_RANK_CERT", "0")
        s0, i0 = retrieval.rank_topk(cc, q, 10)
        monkeypatch.undo()
        torch.cuda.synchronize()
        assert torch.equal(i1, i0) and torch.equal(s1.view(torch.int32), s0.view(torch.int32))


@pytest.mark.parametrize("N,Q,k,dt", [(1, 1, 1, "f32"), (9, 3, 10, "f32"), (4099, 33, 16, "bf16"),
                                      (125_000, 32, 10, "f32"), (300_001, 40, 10, "f32"),
                                      (300_001, 33, 12, "bf16"), (1_000_003, 32, 10, "f32")])
def test_split_merge_bit_identical_to_in_launch_merge(gpu, monkeypatch, N, Q, k, dt):
    """The split merge (the pass writes every lane's sorted list, fold_merge_kernel reduces
    each query's lines; the product default of rank_reg, the certified pass and the mirror)
    gives the round-4 in-launch merge's results bit for bit (A/B build, MICLIP_RANK_FOLD=1):
    one and two query blocks, 1 .. 256 workgroups, the exact and the certified routes, with
    a block of duplicated rows (ties across workgroups) and a zero row (NaN)."""
    import torch
    from miclip import _native, retrieval, weights
    c32 = weights.normal(51, f"sm{N}", (N, 512))
    if N > 1000:
        c32[N // 3: N // 3 + 40] = c32[N // 2]      # 41 equal rows in different workgroups
        c32[N // 4] = 0.0
    c = _t(c32, gpu) if dt == "f32" else torch.from_numpy(c32).to(torch.bfloat16).to(gpu)
    q = _t(weights.synthetic_corpus(Q, 512, seed=52), gpu)
    q[0] = torch.from_numpy(c32[N // 2]).to(gpu)       # a query whose best rows tie
    for pol in ("first", "last"):
        s1, i1 = retrieval.rank_topk(c, q, k, nan_policy=pol)
        monkeypatch.setattr(_native, "lib", _native.lib_ab)
        monkeypatch.setenv("MICLIP_RANK_FOLD", "1")
        s0, i0 = retrieval.rank_topk(c, q, k, nan_policy=pol)
        monkeypatch.undo()
        torch.cuda.synchronize()
        assert torch.equal(i1, i0), pol
        assert torch.equal(s1.view(torch.int32), s0.view(torch.int32)), pol
    if N >= 262_144 and dt == "f32":   # the mirror's pass merges the same way
        mc = retrieval.MirroredCorpus(c)
        s1, i1 = mc.topk(q, k)
        monkeypatch.setattr(_native, "lib", _native.lib_ab)
        monkeypatch.setenv("MICLIP_RANK_FOLD", "1")
        mc0 = retrieval.MirroredCorpus(c)
        s0, i0 = mc0.topk(q, k)
        monkeypatch.undo()
        torch.cuda.synchronize()
        assert torch.equal(i1, i0) and torch.equal(s1.view(torch.int32), s0.view(torch.int32))
