"""CPU: host-side logic around the kernels (config inference, weight packing,
tokenizer, preprocessing, sharding, service/ranking glue with fakes)."""
import gzip
import os

import numpy as np
import pytest

from conftest import state_dict


def test_config_inference_from_state_dict():
    from miclip import config
    for name in ("test-tiny", "test-small", "ViT-B/32"):
        cfg = config.from_state_dict(state_dict(name))
        assert cfg == config.get_config(name)
    assert "ViT-B/32" in config.available_models() and "test-tiny" not in config.available_models()


def test_flops_match_survey():
    from miclip import config
    b32 = config.get_config("ViT-B/32")
    assert abs(b32.image_flops() / 1e9 - 8.818) < 0.01
    assert abs(config.get_config("ViT-L/14").image_flops() / 1e9 - 162.03) < 0.1
    assert abs(config.get_config("ViT-L/14@336px").image_flops() / 1e9 - 381.92) < 0.1


def test_executed_flops_of_the_cls_row_last_block():
    """image_flops_executed: the last block's out_proj / c_fc / c_proj skipped for S - 1 of S rows
    (api.cpp last_block_cls) -- what bench.py's end-to-end MFMA fraction counts."""
    from miclip import config
    b32 = config.get_config("ViT-B/32")
    W, S = b32.vision_width, b32.vision_tokens
    assert b32.image_flops_executed(False) == b32.image_flops()
    assert b32.image_flops() - b32.image_flops_executed() == 2.0 * (S - 1) * W * 9 * W
    assert 0.93 < b32.image_flops_executed() / b32.image_flops() < 0.95
    # the last in_proj's Q for the CLS rows only, and its attention for the CLS query's 16-row tile
    assert b32.image_flops_executed() - b32.image_flops_executed(True, True) == 2.0 * (S - 1) * W * W
    assert (b32.image_flops_executed(True, True) - b32.image_flops_executed(True, True, 16)
            == 4.0 * (S - 16) * S * W)
    assert b32.image_attention_flops() == 4.0 * S * S * W * b32.vision_layers


def test_bench_step_work_and_mfma_fraction():
    """bench.py's end-to-end MFMA fraction: executed work per engine at its dense peak (ADVICE r5:
    the MX-fp8 tower's CLS-row last block counted; VERDICT r5: the fp32 parity mode no longer
    reports f32-equivalent flops over the f32 peak, a fraction above 1)."""
    import bench
    from miclip import config
    b32, l336 = config.get_config("ViT-B/32"), config.get_config("ViT-L/14@336px")
    w = bench.step_work(b32, "bf16", 10_000, True)
    assert w["cls_last"] and w["image"] == b32.image_flops_executed(True, True, 16)
    assert not bench.step_work(b32, "bf16", 200, True)["cls_last"]        # < 256 frames per chunk
    w8 = bench.step_work(l336, "fp8", 863, False)
    assert w8["cls_last"] and w8["image"] == l336.image_flops_executed(True)   # MX: no Q / attention skip
    w32 = bench.step_work(b32, "fp32", 10_000, False)
    assert w32["image"] == b32.image_flops_executed(True, True, 32)
    t16 = bench.mfma_time_at_peak(w, "bf16", 10_000, 32, 512)
    t32 = bench.mfma_time_at_peak(w32, "fp32", 10_000, 32, 512)
    assert 0.03 < t16 < 0.04            # ~35 ms of bf16 MFMA work at 2.5 PF for 10k B/32 frames
    assert 3 * t16 < t32 < 5 * t16      # 3x the products on the f16 MFMA + exact-f32 attention


def test_pack_order_covers_state_dict():
    from miclip import _native, config
    cfg = config.get_config("test-small")
    sd = state_dict("test-small")
    order = _native.weight_order(cfg)
    assert sorted(order) == sorted(sd)
    blob = _native.pack_weights(sd, cfg)
    assert blob[0] == sd["visual.conv1.weight"].reshape(-1)[0] and blob[-1] == sd["logit_scale"]


def _toy_bpe(tmp_path):
    lines = ["#version: 0.2", "h e", "l l", "he ll", "hell o</w>", "w o", "r l", "wo rl", "worl d</w>"]
    p = tmp_path / "toy_bpe.txt.gz"
    with gzip.open(p, "wb") as f:
        f.write("\n".join(lines).encode())
    return str(p)


def test_tokenizer_contract(tmp_path):
    from miclip.tokenizer import tokenize, _tokenizer
    path = _toy_bpe(tmp_path)
    tok = _tokenizer(path)
    t = tokenize(["Hello   world", "hello"], bpe_path=path)
    assert t.shape == (2, 77) and str(t.dtype) == "torch.int32"
    sot, eot = tok.encoder["<|startoftext|>"], tok.encoder["<|endoftext|>"]
    assert t[0, 0] == sot and t[0, 3] == eot and (t[0, 4:] == 0).all()
    assert tok.decoder[int(t[0, 1])] == "hello</w>" and tok.decoder[int(t[0, 2])] == "world</w>"
    assert int(t[1].argmax()) == 2            # EOT is the row argmax (pooling rule)
    long = " ".join(["hello"] * 100)
    with pytest.raises(RuntimeError):
        tokenize([long], bpe_path=path)
    tt = tokenize([long], truncate=True, bpe_path=path)
    assert tt[0, -1] == eot


def test_tokenize_without_vocab_raises(monkeypatch):
    from miclip.tokenizer import tokenize
    monkeypatch.delenv("CLIP_BPE_PATH", raising=False)
    with pytest.raises(RuntimeError, match="CLIP_BPE_PATH"):
        tokenize(["a photo"])


def test_preprocess_matches_torchvision_semantics():
    from PIL import Image
    from miclip.preprocess import Transform, MEAN, STD
    img = Image.fromarray((np.arange(720 * 1280 * 3) % 251).astype(np.uint8).reshape(720, 1280, 3))
    x = Transform(224)(img)
    assert tuple(x.shape) == (3, 224, 224)
    # resize short side 720 -> 224: long side int(224*1280/720) = 398, crop left round(87.0)
    r = img.resize((398, 224), Image.BICUBIC).crop((87, 0, 311, 224))
    ref = (np.asarray(r, np.float32) / 255 - MEAN) / STD
    np.testing.assert_allclose(x.numpy().transpose(1, 2, 0), ref, atol=1e-6)
    y = Transform(224, squash=True)(img)
    assert tuple(y.shape) == (3, 224, 224)


def test_shard_range_partitions():
    from miclip.distributed import shard_range
    for n, w in ((10, 3), (1_000_000, 8), (5, 8), (0, 2)):
        spans = [shard_range(n, w, r) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert max(e - s for s, e in spans) - min(e - s for s, e in spans) <= 1


def test_synthetic_tokens_format():
    from miclip import weights
    t = weights.synthetic_tokens(50)
    for row in t:
        L = int(np.argmax(row))
        assert row[0] == 49406 and row[L] == 49407 and 6 <= L <= 31 and (row[L + 1:] == 0).all()
        assert (row[1:L] >= 256).all() and (row[1:L] < 49406).all()


def test_tokenizer_clean_restates_ftfy_subset():
    """basic_clean's ftfy.fix_text step (ftfy is not installed: restated subset,
    miclip/tokenizer.py), then the double html.unescape and whitespace_clean of
    openai/CLIP simple_tokenizer.  Expected strings follow ftfy 6's documented
    fixers (ligatures, character width, curly quotes, line breaks, control
    characters, terminal escapes, NFC); parity against ftfy itself is unpinned."""
    import unicodedata
    from miclip.tokenizer import _clean
    assert _clean("ﬁsh “quoted”") == 'fish "quoted"'
    assert _clean("ＡＢＣ　１２３") == "ABC 123"
    assert _clean("école") == unicodedata.normalize("NFC", "école")
    assert _clean("line\r\nbreak x") == "line break x"
    assert _clean("\x1b[31mred\x1b[0m") == "red"
    assert _clean("tab\x00ctl") == "tabctl"
    assert _clean("a &amp;amp; b") == "a & b"
    assert _clean("  plain   query  ") == "plain query"
    # ftfy uncurl_quotes tables: U+02BC and U+2018-201B -> ', U+201C-201F -> ", primes untouched
    assert _clean("it\u02bcs \u201bx\u201f") == "it's 'x\""
    assert _clean("5\u2032 10\u2033") == "5\u2032 10\u2033"
    # ftfy CONTROL_CHARS includes musical formatting U+1D173-1D17A and tags U+E0000-E007F
    assert _clean("a\U0001d173b\U000e0041c\U000e007fd") == "abcd"


def test_tokenizer_mojibake_repair_subset():
    """ftfy fix_encoding's whole-string case (restated in miclip/tokenizer.py): UTF-8 read as
    Windows-1252, once or twice, is decoded back; text with any character outside
    Windows-1252 (the reference's Vietnamese queries), legitimate Latin-1 text and lone
    lead characters are left alone.  Examples follow ftfy's documentation; parity against
    ftfy itself is unpinned (not installed)."""
    from miclip.tokenizer import _clean, fix_encoding_subset

    def as_cp1252(t):   # UTF-8 bytes shown through sloppy Windows-1252
        hi = "€\x81‚ƒ„…†‡ˆ‰Š‹Œ\x8dŽ\x8f\x90‘’“”•–—˜™š›œ\x9džŸ"
        return "".join(chr(b) if b < 0x80 or b >= 0xA0 else hi[b - 0x80] for b in t.encode("utf-8"))

    assert fix_encoding_subset("cafÃ©") == "café"
    assert fix_encoding_subset("âœ” No problems") == "✔ No problems"
    assert fix_encoding_subset("schÃ¶n Ã‰cole Â£100") == "schön École £100"
    # doubly encoded, then uncurl_quotes
    assert _clean("The Mona Lisa doesnÃ¢â‚¬â„¢t have eyebrows.") == "The Mona Lisa doesn't have eyebrows."
    for t in ["người đi xe đạp trên đường", "cảnh hoàng hôn trên biển", "naïve café", "日本語 🚀", "Ã", "plain"]:
        assert fix_encoding_subset(t) == t, t                  # well-formed: untouched
        if any(ord(c) > 0x7F for c in t) and len(t) > 1:
            assert fix_encoding_subset(as_cp1252(t)) == t, t    # its mojibake: repaired
            assert fix_encoding_subset(as_cp1252(as_cp1252(t))) == t, t
