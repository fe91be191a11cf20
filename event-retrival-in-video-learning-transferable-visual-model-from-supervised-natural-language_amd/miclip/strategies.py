"""The two CLIP query strategies of ``Backend/query_strategies.py`` with the
reference's signatures and results, minus its per-candidate linear scans
(SURVEY.md §8(f) item 4).

  query_by_text_clip                     query_strategies.py:36-119
  query_by_text_with_adaptive_threshold  query_strategies.py:121-186

Both take the injected callables the Flask app passes (``search_top_frames``,
``extract_query_confidence``, ``format_event_for_frontend``, app.py:157-174)
and behave as the reference does: ``top_k * 3`` candidates from
``search_top_frames``, the metadata row whose ``frameidx`` equals the
candidate file's stem (FIRST such row, as ``next(...)`` finds it), a confidence
per candidate, the threshold (adaptive variant), a stable sort by
``clip_similarity`` descending, ``[:top_k]``; any error returns ``[]``.

What changes: the reference scans the whole metadata list for every candidate
(``next(item for item in data if ...)``, :95 and :160, O(K*N)); here the
``frameidx`` -> row map is built once per metadata list (O(N + K)), and
``EmbeddingService.extract_query_confidence`` is an O(1) lookup.  The
Vietnamese preprocessing + network translation step
(``word_processing.py:68-75``) is out of scope: pass
``text_processor`` (any object with ``preprocess_and_translate``) to keep it;
by default the query is used as given.  ``data`` may be passed directly instead
of being read from the metadata JSON the reference resolves
(``get_video_metadata_path``, :17-34).
"""
from __future__ import annotations

import json
import os
from pathlib import Path

_index_cache = {}


def get_video_metadata_path(video_name=None, video_data_mapping=None, metadata_dir="metadata"):
    """query_strategies.py:17-34 (default file ``output_samples.json``)."""
    if video_name and video_data_mapping and video_name in video_data_mapping:
        return os.path.normpath(video_data_mapping[video_name]["metadata_file"])
    return os.path.join(metadata_dir, "output_samples.json")


def _frameidx_index(data):
    """frameidx -> first metadata row with it (``next(...)`` semantics)."""
    hit = _index_cache.get(id(data))
    if hit is not None and hit[0] is data and hit[1] == len(data):
        return hit[2]
    index = {}
    for item in data:
        key = item.get("frameidx") if isinstance(item, dict) else None
        if key is not None and key not in index:
            index[key] = item
    _index_cache.clear()          # one live metadata list at a time
    _index_cache[id(data)] = (data, len(data), index)
    return index


def _load_data(video_name, video_data_mapping, data):
    if data is not None:
        return data
    with open(get_video_metadata_path(video_name, video_data_mapping), "r", encoding="utf-8") as f:
        return json.load(f)


def _text(query, text_processor):
    return text_processor.preprocess_and_translate(query) if text_processor is not None else query


def _stem_index(frame_name):
    try:
        return int(Path(frame_name).stem)
    except Exception:
        return None


def query_by_text_clip(query, top_k, search_top_frames, extract_query_confidence, format_event_for_frontend,
                       video_name=None, video_data_mapping=None, data=None, text_processor=None):
    try:
        processed_text = _text(query, text_processor)
        query_frames = search_top_frames(processed_text, top_k * 3, video_name)
        index = _frameidx_index(_load_data(video_name, video_data_mapping, data))
        results, seen = [], set()
        for frame_name in query_frames:
            if frame_name in seen:
                continue
            seen.add(frame_name)
            try:
                frame_idx = _stem_index(frame_name)
                if frame_idx is None:
                    continue
                frame_data = index.get(frame_idx)
                if not frame_data:
                    continue
                confidence = extract_query_confidence(frame_name, processed_text, video_name)
                fd = frame_data.copy()
                fd["clip_similarity"] = confidence
                event = format_event_for_frontend(fd)
                event["clip_similarity"] = confidence
                results.append(event)
            except Exception as e:
                print(f"Error processing frame {frame_name}: {e}")
        results.sort(key=lambda x: x.get("clip_similarity", 0), reverse=True)
        return results[:top_k]
    except Exception as e:
        print(f"Error in text clip query: {e}")
        return []


def query_by_text_with_adaptive_threshold(query, adaptive_threshold, top_k, search_top_frames,
                                          extract_query_confidence, format_event_for_frontend, video_name=None,
                                          video_data_mapping=None, data=None, text_processor=None):
    try:
        processed_text = _text(query, text_processor)
        query_frames = search_top_frames(processed_text, top_k * 3, video_name)
        index = _frameidx_index(_load_data(video_name, video_data_mapping, data))
        semantic_results = []
        for frame_name in query_frames:
            try:
                frame_idx = int(Path(frame_name).stem)
                frame_data = index.get(frame_idx)
                if frame_data:
                    confidence = extract_query_confidence(frame_name, processed_text, video_name)
                    if confidence >= adaptive_threshold:
                        fd = frame_data.copy()
                        fd["clip_similarity"] = confidence
                        event = format_event_for_frontend(fd)
                        event["clip_similarity"] = confidence
                        semantic_results.append(event)
            except Exception as e:
                print(f"Error processing frame {frame_name}: {e}")
        semantic_results.sort(key=lambda x: x.get("clip_similarity", 0), reverse=True)
        return semantic_results[:top_k]
    except Exception as e:
        print(f"Error in query_by_text_with_adaptive_threshold: {e}")
        return []
