"""``EmbeddingService`` with the reference's interface, ranking on the GPU.

Mirror of ``Backend/services/embedding_service.py:69-536`` — same constructor
(injected cache/path/data services), same method names, arguments, return
types and swallow-to-``[]``/``0.0`` error semantics (:280-282, :342-344), so
``Backend/app.py`` and ``Backend/query_strategies.py`` (which receive
``search_top_frames`` / ``extract_query_confidence`` as callables,
app.py:157-174) work unchanged.  What moves to the device:

  get_text_features      clip.tokenize -> encode_text (+L2 in the kernel)      :151-184
  search_top_frames      np.dot + np.argsort(s)[::-1][:k] -> one fused kernel  :284-344
                         over the HBM-resident corpus (file rows, normalised
                         as get_embeddings does at load :209-210: f32 files
                         in the rank kernel; float16 files -- the reference's
                         default video_test_3 / image_embeddings.npy -- by
                         mi_normalize_rows_f16 in NumPy's float16 arithmetic,
                         then ranked as stored)
  search_top_frames_by_image                                                    :346-392
  extract_and_save_embeddings_from_folder  batches -> encode_image (+L2)      :425-536

The frame list (row order) still comes from ``data_service.load_frames_from_json``
(data_service.py:48), and ``get_embeddings`` keeps returning the normalised
numpy array other callers (visualization_service) expect.
"""
from __future__ import annotations

import json
import os

import numpy as np

from . import api
from .preprocess import decode_chunk, load_frames
from .retrieval import MirroredCorpus, normalize_rows_f16, rank_topk

# corpora from this many rows on also get an fp16 ranking mirror (scripts/mirror_micro.py:
# 1M rows 1.6-1.9x faster than the exact pass, 125k rows slower: fixed merge/re-score cost)
MIRROR_MIN_ROWS = 262_144
from .weights import load_classifier, load_state_dict


def gemm_f32(a, w, bias=None, relu=False):
    """f32 [M,K] . [N,K]^T (+bias) (+ReLU) through ``mi_op_gemm_f32`` (the fp32
    tower's exact-f32 MFMA GEMM); K is zero-padded to a multiple of 32."""
    import torch
    from . import _native as N
    a = a.float().contiguous()
    w = w.float().contiguous()
    M, K = a.shape
    Nn = w.shape[0]
    if K % 32:
        pad = 32 - K % 32
        a = torch.nn.functional.pad(a, (0, pad))
        w = torch.nn.functional.pad(w, (0, pad))
        K += pad
    out = torch.empty(M, Nn, dtype=torch.float32, device=a.device)
    if M == 0:
        return out
    b = bias.float().contiguous() if bias is not None else None
    with torch.cuda.device(a.device):
        N.check(N.lib().mi_op_gemm_f32(a.data_ptr(), w.data_ptr(), b.data_ptr() if b is not None else None,
                                       out.data_ptr(), M, Nn, K, 3 if relu else 0, N.stream_ptr(a.device)),
                "mi_op_gemm_f32")
    return out


class FinetunedCLIP:
    """``CLIPWithClassifier`` (embedding_service.py:16-67) on the device:
    ``clip_model.float()`` (:22, the fp32 tower), ``model(images)`` = L2-normalised
    image features (:36-49); with texts, the CLIP logits (logit_scale.exp() *
    I . T^T) and the 3-class head Linear(D, 512) -> ReLU -> Dropout (identity at
    inference) -> Linear(512, 3) on the checkpoint's ``classifier.*`` weights
    (:51-67)."""

    def __init__(self, clip_model, classifier=None):
        import torch
        self.clip_model = clip_model.float()
        self.logit_scale = clip_model.logit_scale
        self.classifier = None
        if classifier is not None:
            dev = self.clip_model.device
            self.classifier = {k: torch.from_numpy(v).to(dev) for k, v in classifier.items()}

    def __call__(self, images, texts=None, get_embeddings=False):
        import torch
        if texts is not None and self.classifier is None:
            # checked before any encode: the reference's CLIPWithClassifier always has the head
            raise ValueError("this checkpoint has no classifier.* weights: class logits are unavailable")
        image_features = self.clip_model.encode_image(images, normalize=True, out_dtype=torch.float32)
        if texts is None:
            return image_features
        text_features = self.clip_model.encode_text(texts, normalize=True, out_dtype=torch.float32)
        from .retrieval import score_matrix
        scale = float(np.exp(np.float32(self.logit_scale.item())))
        # (logit_scale * image_features) @ text_features.t()  (:57-58)
        logits_per_image = score_matrix(text_features, image_features * scale, norm="none")
        logits_per_text = logits_per_image.t()
        c = self.classifier
        hidden = gemm_f32(image_features, c["0.weight"], c["0.bias"], relu=True)
        class_logits = gemm_f32(hidden, c["3.weight"], c["3.bias"])
        if get_embeddings:
            return image_features, text_features, logits_per_image, logits_per_text, class_logits
        return logits_per_image, logits_per_text, class_logits

    def eval(self):
        return self

    def to(self, device):
        self.clip_model.to(device)
        return self


class EmbeddingService:
    def __init__(self, cache_service, path_service, data_service, device="cuda", model_name="ViT-B/32",
                 checkpoint_path=None):
        self.cache_service = cache_service
        self.path_service = path_service
        self.data_service = data_service
        self.device = device
        self.model_name = model_name
        self.original_model, self.preprocess = api.load(model_name, device=device)
        self.finetuned_model = None
        self.active_model = "original"
        self.checkpoint_path = checkpoint_path or os.environ.get("CLIP_FINETUNED_CHECKPOINT", "")
        self._device_corpus = {}
        self._mirrors = {}          # id(device corpus) -> MirroredCorpus (large corpora)
        self._lookup = {}
        if self.checkpoint_path and os.path.exists(self.checkpoint_path):
            try:
                self._load_finetuned_model(self.checkpoint_path)
            except Exception as e:  # reference: print and continue (:98-99)
                print(f"Error loading finetuned model: {e}")

    # ----------------------------------------------------------- model state
    def _load_finetuned_model(self, checkpoint_path):
        sd = load_state_dict(checkpoint_path)       # unwraps model_state_dict / clip_model.*
        model, _ = api.load(self.model_name, device=self.device)
        model.load_state_dict(sd)
        self.finetuned_model = FinetunedCLIP(model, load_classifier(checkpoint_path))

    def set_active_model(self, model_name):
        if model_name == "original":
            self.active_model = "original"
            return True
        if model_name == "finetuned":
            if self.finetuned_model is not None:
                self.active_model = "finetuned"
                return True
            return False
        return False

    def get_active_model_name(self):
        return self.active_model

    def _clip(self):
        if self.active_model == "finetuned" and self.finetuned_model is not None:
            return self.finetuned_model.clip_model
        return self.original_model

    # ------------------------------------------------------------- features
    def get_text_features(self, query, video_name=None):
        cache_key = f"{self.active_model}_{query}_{video_name or 'default'}"
        features = self.cache_service.get_text_features(cache_key, video_name)
        if features is not None:
            return features
        tokens = api.tokenize([query])
        feats = self._clip().encode_text(tokens, normalize=True, out_dtype=__import__("torch").float32)
        features = feats.cpu().numpy()
        self.cache_service.set_text_features(cache_key, video_name, features)
        return features

    def get_embeddings(self, video_name=None):
        embeddings_path = self.path_service.get_embeddings_path(video_name)
        embeddings = self.cache_service.get_embeddings(embeddings_path)
        if embeddings is not None:
            return embeddings
        if not os.path.exists(embeddings_path):
            print(f"Warning: Embeddings file not found: {embeddings_path}")
            return None
        try:
            embeddings = np.load(embeddings_path)
            embeddings = embeddings / np.linalg.norm(embeddings, axis=-1, keepdims=True)
            self.cache_service.set_embeddings(embeddings_path, embeddings)
            return embeddings
        except Exception as e:
            print(f"Error loading embeddings: {e}")
            return None

    def _corpus_on_device(self, video_name):
        """(rows, norm) resident in HBM for the rank kernel, normalised as
        get_embeddings normalises the file (embedding_service.py:209-210):
        f32 rows stay raw and the rank kernel normalises each row in the same
        pass (norm "l2"); float16 rows -- NumPy normalises those in float16 --
        are normalised once on the device bit for bit as NumPy does it
        (``normalize_rows_f16``) and ranked as they are (norm "none"), so
        search_top_frames ranks exactly the rows extract_query_confidence
        reads from get_embeddings."""
        import torch
        path = self.path_service.get_embeddings_path(video_name)
        if not os.path.exists(path):
            return None
        mtime = os.path.getmtime(path)
        hit = self._device_corpus.get(path)
        if hit is not None and hit[0] == mtime:
            return hit[1]
        if hit is not None:
            self._mirrors.pop(id(hit[1][0]), None)   # the file changed: drop the old rows' mirror
        raw = np.load(path)
        if raw.dtype not in (np.float32, np.float16):
            raw = raw.astype(np.float32)
        t = torch.from_numpy(np.ascontiguousarray(raw)).to(self.original_model.device)
        if t.dtype == torch.float16:
            entry = (normalize_rows_f16(t, out=t), "none")
        else:
            entry = (t, "l2")
            if t.shape[0] >= MIRROR_MIN_ROWS and t.shape[1] in (512, 768):
                self._mirrors[id(t)] = MirroredCorpus(t)
        self._device_corpus[path] = (mtime, entry)
        return entry

    def _frames(self, video_name):
        json_path = self.path_service.get_metadata_path(video_name)
        frames = self.cache_service.get_frames_list(json_path)
        if frames is None:
            frames = self.data_service.load_frames_from_json(video_name)
            self.cache_service.set_frames_list(json_path, frames)
        return frames

    def _rank(self, entry, query_vec, top_k):
        """Top-k (score desc, index asc; NaN first as argsort(s)[::-1]); any
        k up to the corpus size (a full sort when top_k >= N, as the reference's
        np.argsort(s)[::-1] at embedding_service.py:317-318).  ``entry`` is
        ``_corpus_on_device``'s (rows, norm)."""
        import torch
        corpus, norm = entry
        k = min(int(top_k), corpus.shape[0])
        if k <= 0:
            return np.zeros(0, np.float32), np.zeros(0, np.int64)
        q = torch.as_tensor(np.asarray(query_vec, dtype=np.float32).reshape(1, -1), device=corpus.device)
        mc = self._mirrors.get(id(corpus))
        if mc is not None and mc.master is corpus and norm == "l2" and k <= MirroredCorpus.MAX_K:
            s, i = mc.topk(q, k, norm="l2", nan_policy="first")   # certified == the exact pass, bit for bit
        else:
            s, i = rank_topk(corpus, q, k, norm=norm, nan_policy="first")
        return s[0].cpu().numpy(), i[0].cpu().numpy()

    # --------------------------------------------------------------- search
    def extract_query_confidence(self, frame_path, query, video_name=None):
        try:
            text_features = self.get_text_features(query, video_name)
            embeddings = self.get_embeddings(video_name)
            if embeddings is None:
                return 0.0
            frames = self._frames(video_name)
            cached = self._lookup.get(id(frames))
            if cached is None or cached[0] is not frames:
                # first occurrence wins, as list.index (embedding_service.py:264-271)
                by_path = {f: i for i, f in reversed(list(enumerate(frames)))}
                by_name = {os.path.basename(f): i for i, f in reversed(list(enumerate(frames)))}
                cached = (frames, by_path, by_name)
                self._lookup[id(frames)] = cached
            index = cached[1].get(frame_path)
            if index is None:
                index = cached[2].get(os.path.basename(frame_path))
                if index is None:
                    return 0.0
            return float(np.dot(embeddings[index:index + 1], text_features.T)[0][0])
        except Exception as e:
            print(f"Error extracting query confidence: {e}")
            return 0.0

    def search_top_frames(self, query, top_k, video_name=None):
        try:
            cache_key = f"search_{self.active_model}_{query}_{top_k}"
            cached = self.cache_service.get_search_results(cache_key, video_name)
            if cached is not None:
                return cached
            text_features = self.get_text_features(query, video_name)
            corpus = self._corpus_on_device(video_name)
            if corpus is None:
                return []
            _, idx = self._rank(corpus, text_features, top_k)
            frames = self._frames(video_name)
            top_frames = [frames[i] for i in idx]
            self.cache_service.set_search_results(cache_key, video_name, top_frames)
            return top_frames
        except Exception as e:
            print(f"Error in search_top_frames: {e}")
            return []

    def search_top_frames_by_image(self, image_features, top_k, video_name=None):
        try:
            corpus = self._corpus_on_device(video_name)
            if corpus is None:
                return []
            _, idx = self._rank(corpus, np.asarray(image_features, dtype=np.float32).reshape(-1), top_k)
            frames = self._frames(video_name)
            return [frames[i] for i in idx]
        except Exception as e:
            print(f"Error in search_top_frames_by_image: {e}")
            return []

    # --------------------------------------------------------------- ingest
    def extract_image_embedding(self, image_path):
        try:
            from PIL import Image
            import torch
            image = self.preprocess(Image.open(image_path)).unsqueeze(0)
            if self.active_model == "finetuned" and self.finetuned_model is not None:
                feats = self.finetuned_model(image)
            else:
                feats = self.original_model.encode_image(image, normalize=True, out_dtype=torch.float32)
            return feats.float().cpu().numpy()
        except Exception as e:
            print(f"Error extracting embedding from {image_path}: {e}")
            return None

    def extract_and_save_embeddings_from_folder(self, folder_path, model_name=None, video_name=None,
                                                batch_size=256):
        import torch

        current = self.active_model
        if model_name:
            if model_name == "finetuned" and self.finetuned_model is None:
                model_name = "original"
            self.set_active_model(model_name)
        embeddings_path = self.path_service.get_embeddings_path(video_name)
        os.makedirs(os.path.dirname(embeddings_path) or ".", exist_ok=True)
        frame_files = sorted(f for f in os.listdir(folder_path) if f.endswith((".jpg", ".jpeg", ".png")))
        if not frame_files:
            self.set_active_model(current)
            return None
        model = self._clip()
        R = model.cfg.image_resolution
        out = []
        step = decode_chunk(batch_size)
        for j in range(0, len(frame_files), step):
            # GPU JPEG decode + resize/crop/normalise (Pillow-exact, miclip.preprocess.load_frames) over a
            # large chunk (the decode runs one lane per frame), then the reference's encode batches
            frames, _ = load_frames([os.path.join(folder_path, f) for f in frame_files[j:j + step]], R,
                                    device=model.device)
            for i in range(0, frames.shape[0], batch_size):
                out.append(model.encode_image(frames[i:i + batch_size], normalize=True,
                                              out_dtype=torch.float32).cpu().numpy())
        embeddings = np.vstack(out)
        np.save(embeddings_path, embeddings)
        metadata_path = self.path_service.get_metadata_path(video_name)
        if os.path.exists(metadata_path):
            try:
                with open(metadata_path, "r", encoding="utf-8") as f:
                    metadata = json.load(f)
                if isinstance(metadata, list):
                    for item in metadata:
                        item["embedding_model"] = self.active_model
                elif isinstance(metadata, dict):
                    metadata["embedding_model"] = self.active_model
                with open(metadata_path, "w", encoding="utf-8") as f:
                    json.dump(metadata, f, ensure_ascii=False, indent=2)
            except Exception as e:
                print(f"Error updating metadata with model info: {e}")
        self.set_active_model(current)
        return embeddings_path
