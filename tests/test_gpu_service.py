"""EmbeddingService mirror end to end on the GPU:
folder ingest (host decode + GPU preprocessing + encode_image + L2) -> .npy,
then search_top_frames / extract_query_confidence / search_top_frames_by_image
over the HBM-resident corpus, against the oracle restatement of
Backend/services/embedding_service.py:151-392 on the same rows.

The injected services are minimal in-memory stand-ins with the reference's
method names (cache_service.py, path_service.py, data_service.py:24-55 —
frame list = sorted file names).  clip.tokenize needs a BPE vocabulary that is
not in this image (tokenizer parity unpinned), so the query -> token ids step
is replaced by the deterministic synthetic tokenizer of miclip.weights."""
import json
import os
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class Cache:
    def __init__(self):
        self.d = {}

    def _get(self, *k):
        return self.d.get(k)

    def _set(self, v, *k):
        self.d[k] = v

    def get_text_features(self, key, video):
        return self._get("t", key, video)

    def set_text_features(self, key, video, v):
        self._set(v, "t", key, video)

    def get_embeddings(self, path):
        return self._get("e", path)

    def set_embeddings(self, path, v):
        self._set(v, "e", path)

    def get_frames_list(self, path):
        return self._get("f", path)

    def set_frames_list(self, path, v):
        self._set(v, "f", path)

    def get_search_results(self, key, video):
        return self._get("s", key, video)

    def set_search_results(self, key, video, v):
        self._set(v, "s", key, video)


class Paths:
    def __init__(self, root):
        self.root = root

    def get_embeddings_path(self, video):
        return os.path.join(self.root, "embedding", f"{video}_embeddings.npy")

    def get_metadata_path(self, video):
        return os.path.join(self.root, "metadata", f"{video}_metadata.json")


class Data:
    def __init__(self, paths, frame_dir):
        self.paths, self.frame_dir = paths, frame_dir

    def load_frames_from_json(self, video):
        with open(self.paths.get_metadata_path(video)) as f:
            return [item["frame"] for item in json.load(f)]


def _frames(tmp_path, n=24):
    from PIL import Image
    d = tmp_path / "frames"
    d.mkdir()
    rng = np.random.default_rng(5)
    names = []
    for i in range(n):
        h, w = (90, 160) if i % 3 else (120, 120)    # two frame sizes -> two upload groups
        yy, xx = np.mgrid[0:h, 0:w]
        base = (127 + 100 * np.sin(xx / (3.0 + i) + yy / (5.0 + i)))[..., None] * np.array([1.0, 0.8, 0.5])
        img = np.clip(base + rng.normal(0, 30, (h, w, 3)), 0, 255).astype(np.uint8)
        names.append(f"{i:04d}.png")
        Image.fromarray(img).save(d / names[-1])
    (d / "broken.png").write_bytes(b"not an image")   # unreadable frame -> zero row (embedding_service.py:476-480)
    names.append("broken.png")
    return d, sorted(names)


def _tokens(q, cfg):
    from miclip import weights
    seed = zlib.crc32(q.encode()) % 1000
    return weights.synthetic_tokens(1, cfg.context_length, cfg.vocab_size, seed=seed)


@pytest.fixture()
def service(gpu, tmp_path, monkeypatch):
    import torch
    from miclip import api, service as S
    root = tmp_path / "state"
    (root / "metadata").mkdir(parents=True)
    frame_dir, names = _frames(tmp_path)
    with open(root / "metadata" / "vid_metadata.json", "w") as f:
        json.dump([{"frame": n} for n in names], f)
    paths = Paths(str(root))
    svc = S.EmbeddingService(Cache(), paths, Data(paths, frame_dir), device="cuda", model_name="test-small")
    cfg = svc.original_model.cfg
    monkeypatch.setattr(api, "tokenize", lambda texts, *a, **k: torch.from_numpy(
        np.concatenate([_tokens(t, cfg) for t in texts])))
    return svc, frame_dir, names, paths


def test_ingest_rows_match_host_preprocessing(service):
    import torch
    from PIL import Image
    svc, frame_dir, names, paths = service
    out = svc.extract_and_save_embeddings_from_folder(str(frame_dir), video_name="vid", batch_size=10)
    rows = np.load(out)
    assert rows.shape == (len(names), svc.original_model.cfg.embed_dim)
    tf = svc.preprocess
    for i, name in enumerate(names):
        if name == "broken.png":
            x = torch.zeros(1, 3, tf.n_px, tf.n_px)
        else:
            x = tf(Image.open(frame_dir / name).convert("RGB")).unsqueeze(0)
        ref = svc.original_model.encode_image(x, normalize=True, out_dtype=torch.float32).cpu().numpy()[0]
        np.testing.assert_allclose(rows[i], ref, rtol=0, atol=2e-6)
    np.testing.assert_allclose(np.linalg.norm(rows, axis=1), 1.0, atol=1e-5)


def test_search_confidence_and_image_query_match_oracle(service):
    from oracle import rank_ref
    svc, frame_dir, names, paths = service
    svc.extract_and_save_embeddings_from_folder(str(frame_dir), video_name="vid")
    rows = np.load(paths.get_embeddings_path("vid"))
    for q in ("a red car at night", "people walking"):
        k = 7
        got = svc.search_top_frames(q, k, "vid")
        t = svc.get_text_features(q, "vid")
        ref_frames, _ = rank_ref.search_top_frames_ref(rows, t, k, names)
        assert got == ref_frames[:k]
        assert svc.search_top_frames(q, k, "vid") == got          # cached path
        conf = svc.extract_query_confidence(got[0], q, "vid")
        i = names.index(got[0])
        e = rows / np.linalg.norm(rows, axis=1, keepdims=True)
        assert abs(conf - float(e[i] @ t[0])) < 1e-5
    img_q = rows[3]
    got = svc.search_top_frames_by_image(img_q, 5, "vid")
    ref_frames, _ = rank_ref.search_top_frames_ref(rows, img_q[None], 5, names)
    assert got == ref_frames[:5] and got[0] == names[3]


def test_error_semantics(service):
    svc, frame_dir, names, paths = service
    assert svc.search_top_frames("anything", 5, "missing_video") == []      # embedding_service.py:342-344
    assert svc.extract_query_confidence("nope.png", "x", "missing_video") == 0.0  # :280-282
    svc.extract_and_save_embeddings_from_folder(str(frame_dir), video_name="vid")
    assert svc.extract_query_confidence("not_a_frame.png", "x", "vid") == 0.0


def _ref_search_by_image(svc, image_path, thr, top_k, data, fmt, video_name):
    """search_service.py:611-706 restated literally (local-path branch): encode
    the query, top_k * 3 candidates, then re-encode EVERY candidate frame
    (extract_image_embedding) for its cosine, threshold, sort, [:top_k]."""
    import torch
    from pathlib import Path
    from PIL import Image
    image = svc.preprocess(Image.open(image_path).convert("RGB")).unsqueeze(0)
    f = svc.original_model.encode_image(image, out_dtype=torch.float32).float()
    feats = (f / f.norm(dim=-1, keepdim=True)).cpu().numpy()
    results = []
    for frame_name in svc.search_top_frames_by_image(feats, top_k * 3, video_name):
        try:
            frame_idx = int(Path(frame_name).stem)
            frame_data = next((item for item in data if item.get("frameidx") == frame_idx), None)
            if frame_data:
                emb = svc.extract_image_embedding(frame_name)
                if emb is not None:
                    sim = np.dot(emb, feats.T)[0][0]
                    if sim >= thr:
                        fd = frame_data.copy()
                        fd["clip_similarity"] = float(sim)
                        ev = fmt(fd)
                        ev["clip_similarity"] = float(sim)
                        ev["confidence"] = float(sim)
                        results.append(ev)
        except Exception as e:
            print(f"Error processing frame {frame_name}: {e}")
    results.sort(key=lambda x: x.get("clip_similarity", 0), reverse=True)
    return results[:top_k]


class _SearchData:
    def __init__(self, data):
        self.data = data

    def load_json_data(self, video_name):
        return self.data

    def format_event_for_frontend(self, fd):
        return {"frame": fd["frame"], "frameidx": fd["frameidx"]}


@pytest.mark.parametrize("reencode", [False, True])
def test_search_by_image_matches_reference_flow(service, monkeypatch, reencode):
    """miclip.search.search_by_image against the literal restatement: same
    events in the same order, similarities within 1e-5 (the stored rows are the
    encoder's own output; the reference recomputes them by re-encoding); the
    query frame itself ranks first at cosine ~1; an unreadable candidate frame
    (zero row / failed re-encode) never appears; the data:image branch returns
    [] as the reference's does (it hands undecoded base64 to PIL)."""
    from miclip import search
    svc, frame_dir, names, paths = service
    svc.extract_and_save_embeddings_from_folder(str(frame_dir), video_name="vid")
    monkeypatch.chdir(frame_dir)           # frame names are paths relative to the working directory, as there
    data = [{"frame": n, "frameidx": int(n.split(".")[0])} for n in names if n != "broken.png"]
    data.insert(3, {"frame": "dup", "frameidx": data[5]["frameidx"]})   # duplicate frameidx: the first wins
    ds = _SearchData(data)
    for qi, thr, k in ((4, 0.0, 5), (9, 0.5, 8), (17, -1.0, 10)):
        q = str(frame_dir / names[qi])
        ref = _ref_search_by_image(svc, q, thr, k, data, ds.format_event_for_frontend, "vid")
        got = search.search_by_image(svc, ds, q, thr, k, "vid", reencode=reencode)
        assert [e["frame"] for e in got] == [e["frame"] for e in ref]
        for a, b in zip(got, ref):
            assert abs(a["clip_similarity"] - b["clip_similarity"]) < 1e-5 and a["confidence"] == a["clip_similarity"]
        assert got and got[0]["frame"] in (names[qi], "dup") and got[0]["clip_similarity"] > 0.999
        assert all(e["frame"] != "broken.png" for e in got)
    import base64
    png = (frame_dir / names[2]).read_bytes()
    assert search.search_by_image(svc, ds, "data:image/png;base64," + base64.b64encode(png).decode(), 0.0, 5,
                                  "vid") == []


def test_large_corpus_ranks_through_mirror(service):
    """A corpus of >= MIRROR_MIN_ROWS rows gets the fp16 ranking mirror
    (retrieval.MirroredCorpus); search_top_frames_by_image (top_k <= 12) then
    ranks through it and returns exactly the exact pass's frames, the order of
    embedding_service.py:365-372 (argsort(s)[::-1][:k] on normalised rows)."""
    import torch
    from miclip import retrieval, service as S, weights
    svc, frame_dir, names, paths = service
    n = S.MIRROR_MIN_ROWS + 1000
    rows = weights.normal(41, "svc", (n, 512))
    os.makedirs(os.path.dirname(paths.get_embeddings_path("big")), exist_ok=True)
    np.save(paths.get_embeddings_path("big"), rows)
    big = [f"f{i:07d}.jpg" for i in range(n)]
    with open(paths.get_metadata_path("big"), "w") as f:
        json.dump([{"frame": x} for x in big], f)
    q = weights.synthetic_corpus(1, 512, seed=42)[0]
    got = svc.search_top_frames_by_image(q, 10, "big")
    assert len(svc._mirrors) == 1
    mc = next(iter(svc._mirrors.values()))
    assert mc.certified == 1 and mc.fallbacks == 0
    s, i = retrieval.rank_topk(torch.from_numpy(rows).cuda(), torch.from_numpy(q[None]).cuda(), 10)
    assert got == [big[j] for j in i[0].cpu().numpy()]
    got40 = svc.search_top_frames_by_image(q, 40, "big")          # k > 12: the exact pass
    assert got40[:10] == got and mc.certified == 1


def test_fp16_corpus_file_matches_reference(service, monkeypatch):
    """search_top_frames / extract_query_confidence / search_top_frames_by_image
    over the reference's float16 corpus file (video_test_3_embeddings.npy, the
    app's default corpus; fixture rank_video_test_3.npz): the frame lists equal
    the literal restatement (get_embeddings normalises in float16,
    embedding_service.py:209-210, then :314-336), and the confidences the
    reference's per-frame path computes from get_embeddings' rows
    (:219-282) agree with the ranking: each returned frame's confidence is its
    rank score, in non-increasing order."""
    from conftest import golden
    svc, frame_dir, names, paths = service
    g = golden("rank_video_test_3.npz")
    raw, q = g["corpus"], g["queries"]
    os.makedirs(os.path.dirname(paths.get_embeddings_path("v3")), exist_ok=True)
    np.save(paths.get_embeddings_path("v3"), raw)
    frames = [f"{i}.jpg" for i in range(raw.shape[0])]
    with open(paths.get_metadata_path("v3"), "w") as f:
        json.dump([{"frame": x} for x in frames], f)
    feats = {f"query {r}": q[r:r + 1] for r in range(0, q.shape[0], 7)}
    monkeypatch.setattr(svc, "get_text_features", lambda query, video_name=None: feats[query])
    E = svc.get_embeddings("v3")
    assert E.dtype == np.float16 and np.array_equal(E.view(np.uint16), g["normalized"].view(np.uint16))
    for text, t in feats.items():
        r = int(text.split()[1])
        for k in (10, 60):
            got = svc.search_top_frames(text, k, "v3")
            assert got == [frames[j] for j in g[f"top_index_{k}"][r]], (r, k)
        conf = [svc.extract_query_confidence(fr, text, "v3") for fr in got]
        assert all(a >= b - 2e-7 for a, b in zip(conf, conf[1:]))
        exact = [float(E[int(fr.split(".")[0])].astype(np.float64) @ t[0].astype(np.float64)) for fr in got]
        assert np.allclose(conf, exact, rtol=0, atol=1e-6)
    got = svc.search_top_frames_by_image(q[3], 10, "v3")
    assert got == [frames[j] for j in g["top_index_10"][3]]
