"""The north star's R@K claim end to end: compare_models.py's CLIP evaluation
flow (ModelComparison.evaluate_model, :908-1100) with this package's encoders
in the loop — images -> encode_image -> guarded L2 (:1102-1173), captions ->
encode_text -> guarded L2 (:1190-1261), S = I . T^T (:999), t2i / i2t ranks
(:1004-1062), R@1/5/10 (:1020-1073) — against the same flow on the float64
oracle encoders (fixture ``tests/golden/rk_e2e_b32.npz``, make_golden.py
``rk_e2e_golden``: 100 ViT-B/32 frames x 500 captions, captions assigned so
that every decisive score comparison differs by > 1e-5, ~100x the f32 tower's
score error).

* weights="fp32" (the reference's CPU / model.float() arithmetic): every
  t2i / i2t rank and every metric identical.
* weights="bf16" (the throughput mode): ranks that flip are counted and
  reported, not asserted equal.
"""
import numpy as np
import pytest

from conftest import golden, state_dict

pytestmark = pytest.mark.gpu

METRICS = ("R@1", "R@5", "R@10", "MRR", "Median_Rank", "Mean_Rank")


def _flow(gpu, weights_mode):
    import torch
    from miclip import config, evaluate, model as M, weights
    g = golden("rk_e2e_b32.npz")
    cfg = config.get_config("ViT-B/32")
    m = M.CLIP(cfg, state_dict("ViT-B/32"), device=gpu, weights=weights_mode, image_chunk=64)
    px = torch.from_numpy(weights.synthetic_pixels(int(g["n_img"]), cfg.image_resolution, seed=int(g["pixel_seed"])))
    pool = weights.synthetic_tokens(int(g["n_pool"]), cfg.context_length, cfg.vocab_size, seed=int(g["token_seed"]))
    tokens = torch.from_numpy(pool[g["caption_index"]])
    res = evaluate.evaluate_model(m, px, tokens, g["caption_image_ids"].tolist(), list(range(int(g["n_img"]))))
    return g, res


def test_rk_flow_fp32_identical(gpu):
    g, res = _flow(gpu, "fp32")
    img = res["image_features"].cpu().numpy().astype(np.float64)
    txt = res["text_features"].cpu().numpy().astype(np.float64)
    S = img @ txt.T
    S_ref = g["image_features"].astype(np.float64) @ g["text_features"].astype(np.float64).T
    err = np.abs(S - S_ref).max()
    print(f"fp32 flow: max |S - S_ref| {err:.3e} (decisive gaps >= {float(g['min_gap']):.3e})")
    assert err < float(g["gap"]) / 10, err          # the premise of bit-identical ranks
    np.testing.assert_array_equal(res["t2i_ranks"], g["t2i_ranks"])
    np.testing.assert_array_equal(res["i2t_ranks"], g["i2t_ranks"])
    for d in ("t2i", "i2t"):
        assert [res[d][k] for k in METRICS] == g[d].tolist(), d
    t, i = [float(v) for v in g["t2i"][:3]], [float(v) for v in g["i2t"][:3]]
    assert res["mean"]["rsum"] == t[0] + t[1] + t[2] + i[0] + i[1] + i[2]      # compare_models.py:1087-1088 order


def test_rk_flow_bf16_flips_reported(gpu):
    """The bf16 tower keeps 1 - cos <= 1e-3 but its score error (~1e-3) is far
    above the fixture's 1e-5 gaps: flips are expected and counted."""
    g, res = _flow(gpu, "bf16")
    t2i = int((res["t2i_ranks"] != g["t2i_ranks"]).sum())
    i2t = int((res["i2t_ranks"] != g["i2t_ranks"]).sum())
    dr = {d: [res[d][k] - v for k, v in zip(METRICS[:3], g[d][:3])] for d in ("t2i", "i2t")}
    print(f"bf16 flow: t2i ranks changed {t2i}/{len(g['t2i_ranks'])}, i2t {i2t}/{len(g['i2t_ranks'])}, "
          f"R@1/5/10 deltas {dr}")
    from oracle.clip_ref import cosine
    img = res["image_features"].cpu().numpy()
    assert cosine(img, g["image_features"]).min() > 1 - 1e-3


def test_model_float_switches_to_fp32_tower(gpu):
    """openai/CLIP's model.float() (CLIPWithClassifier, embedding_service.py:22)
    makes the model fp32: here the context is rebuilt on the fp32 tower, and its
    outputs equal a weights="fp32" model's bit for bit."""
    import torch
    from miclip import config, model as M, weights
    cfg = config.get_config("test-small")
    px = torch.from_numpy(weights.synthetic_pixels(5, cfg.image_resolution))
    tk = torch.from_numpy(weights.synthetic_tokens(4, cfg.context_length, cfg.vocab_size))
    a = M.CLIP(cfg, state_dict("test-small"), device=gpu)
    assert a.weights == "bf16"
    a.float()
    assert a.weights == "fp32"
    b = M.CLIP(cfg, state_dict("test-small"), device=gpu, weights="fp32")
    assert torch.equal(a.encode_image(px), b.encode_image(px))
    assert torch.equal(a.encode_text(tk), b.encode_text(tk))


@pytest.mark.parametrize("name", ["test-tiny", "test-small", "ViT-B/32"])
def test_fp32_tower_vs_oracle(gpu, name):
    """The fp32 tower within f32 rounding of the float64 oracle (the bf16 tower's
    bound is 1 - cos <= 1e-3; here 1e-9), batches that cross the context's
    chunk, guarded normalisation."""
    import torch
    from miclip import config, model as M, weights
    from oracle import clip_ref
    cfg = config.get_config(name)
    sd = state_dict(name)
    m = M.CLIP(cfg, sd, device=gpu, weights="fp32", image_chunk=3, text_chunk=2)
    px = weights.synthetic_pixels(5, cfg.image_resolution)
    tk = weights.synthetic_tokens(5, cfg.context_length, cfg.vocab_size)
    img = m.encode_image(torch.from_numpy(px)).cpu().numpy()
    txt = m.encode_text(torch.from_numpy(tk)).cpu().numpy()
    ri = clip_ref.encode_image(px, sd, cfg, np.float64)
    rt = clip_ref.encode_text(tk, sd, cfg, np.float64)
    for got, ref, what in ((img, ri, "image"), (txt, rt, "text")):
        rel = np.abs(got - ref).max() / np.abs(ref).max()
        print(f"{name} fp32 {what}: max rel err {rel:.2e}, 1-cos {1 - clip_ref.cosine(got, ref).min():.2e}")
        assert rel < 2e-5, (what, rel)
        assert clip_ref.cosine(got, ref).min() > 1 - 1e-9
    g = m.encode_image(torch.from_numpy(px), normalize="guarded").cpu().numpy()
    np.testing.assert_allclose(g, img / np.linalg.norm(img, axis=1, keepdims=True), rtol=0, atol=1e-6)


@pytest.mark.parametrize("name,n", [("ViT-B/32", 8), ("ViT-B/32", 13), ("test-small", 40), ("ViT-B/32", 300)])
def test_fp32_tower_8phase_bit_identical(gpu, monkeypatch, name, n):
    """The fp32 tower's split-f16 GEMMs on the 8-phase kernel (in_proj EPI_F32, out_proj / c_proj
    EPI_RESID_F32, c_fc EPI_SPLIT_GELU writing c_proj's operand; the default for >= 256 rows),
    with the activations' split stored once and (>= 256 frames) the CLS-row last block, against
    the ping-pong kernel over the full layout and the full last block (A/B build, MICLIP_F32_8Q=0,
    MICLIP_CLS_LAST=0): image and text embeddings finite and bit for bit (whole and partial
    256-row tiles), and within f32 rounding of the float64 oracle."""
    import torch
    from miclip import _native, config, model as M, weights
    from oracle import clip_ref
    cfg = config.get_config(name)
    sd = state_dict(name)
    px = torch.from_numpy(weights.synthetic_pixels(n, cfg.image_resolution, seed=n))
    tk = torch.from_numpy(weights.synthetic_tokens(n, cfg.context_length, cfg.vocab_size, seed=n))
    m = M.CLIP(cfg, sd, device=gpu, weights="fp32", image_chunk=n, text_chunk=n)
    img, txt = m.encode_image(px).cpu().numpy(), m.encode_text(tk).cpu().numpy()
    # (300 frames: 15000 rows, several tiles per workgroup, so the epilogues run inside the tile loop;
    # also the CLS-row last block and the stored-once split operands against the full pass)
    assert np.isfinite(img).all() and np.isfinite(txt).all()
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_F32_8Q", "0")
    monkeypatch.setenv("MICLIP_CLS_LAST", "0")
    m0 = M.CLIP(cfg, sd, device=gpu, weights="fp32", image_chunk=n, text_chunk=n)
    img0, txt0 = m0.encode_image(px).cpu().numpy(), m0.encode_text(tk).cpu().numpy()
    del m0
    monkeypatch.undo()
    assert np.array_equal(img.view(np.int32), img0.view(np.int32))
    assert np.array_equal(txt.view(np.int32), txt0.view(np.int32))
    ri = clip_ref.encode_image(px.numpy(), sd, cfg, np.float64)
    assert np.abs(img - ri).max() / np.abs(ri).max() < 2e-5
    assert clip_ref.cosine(img, ri).min() > 1 - 1e-9


@pytest.mark.parametrize("pix", ["f32", "bf16"])
def test_fp32_conv1_split_from_pixels_bit_identical(gpu, monkeypatch, pix):
    """conv1's split operand built straight from the pixels (precise.hip im2col_split2h, the
    default for P % 4 == 0) against im2col_f32 + split2h_rows (A/B build, MICLIP_IM2COL_SPLIT=0):
    image embeddings bit for bit, f32 and bf16 pixel inputs."""
    import torch
    from miclip import _native, config, model as M, weights
    cfg = config.get_config("ViT-B/32")
    sd = state_dict("ViT-B/32")
    px = torch.from_numpy(weights.synthetic_pixels(12, cfg.image_resolution, seed=9)).to(gpu)
    if pix == "bf16":
        px = px.bfloat16()
    got = M.CLIP(cfg, sd, device=gpu, weights="fp32", image_chunk=12).encode_image(px).cpu().numpy()
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_IM2COL_SPLIT", "0")
    ref = M.CLIP(cfg, sd, device=gpu, weights="fp32", image_chunk=12).encode_image(px).cpu().numpy()
    monkeypatch.undo()
    assert np.isfinite(got).all()
    assert np.array_equal(got.view(np.int32), ref.view(np.int32))


def test_fp32_tower_last_block_on_cls_rows_bit_identical(gpu, monkeypatch):
    """The fp32 tower's last block after attention on the gathered CLS rows only (the default
    for >= 256 frames per chunk, as the bf16 tower's last_block_cls): image embeddings equal the
    full block's (A/B build, MICLIP_CLS_LAST=0) bit for bit."""
    import torch
    from miclip import _native, config, model as M, weights
    cfg = config.get_config("ViT-B/32")
    sd = state_dict("ViT-B/32")
    px = torch.from_numpy(weights.synthetic_pixels(300, cfg.image_resolution, seed=3))
    got = M.CLIP(cfg, sd, device=gpu, weights="fp32", image_chunk=300).encode_image(px).cpu().numpy()
    monkeypatch.setattr(_native, "lib", _native.lib_ab)
    monkeypatch.setenv("MICLIP_CLS_LAST", "0")
    full = M.CLIP(cfg, sd, device=gpu, weights="fp32", image_chunk=300).encode_image(px).cpu().numpy()
    monkeypatch.undo()
    assert np.array_equal(got.view(np.int32), full.view(np.int32))


@pytest.mark.parametrize("name,fname", [("ViT-L/14", "vit_l14.npz"), ("ViT-L/14@336px", "vit_l14_336px.npz")])
def test_fp32_tower_l14_golden(gpu, name, fname):
    """L/14 (257 tokens) and L/14@336px (577 tokens: the 256-thread attention
    path) on the fp32 tower against the HF-pinned fixtures (HF fp32 outputs)."""
    import torch
    from miclip import config, model as M, weights
    from oracle.clip_ref import cosine
    cfg = config.get_config(name)
    g = golden(fname)
    m = M.CLIP(cfg, state_dict(name), device=gpu, weights="fp32", image_chunk=2, text_chunk=2)
    px = weights.synthetic_pixels(int(g["n_images"]), cfg.image_resolution)
    img = m.encode_image(torch.from_numpy(px)).cpu().numpy()
    txt = m.encode_text(torch.from_numpy(g["tokens"])).cpu().numpy()
    for got, ref, what in ((img, g["image"], "image"), (txt, g["text"], "text")):
        c = cosine(got, ref).min()
        print(f"{name} fp32 {what}: 1-cos {1 - c:.2e}")
        assert c > 1 - 1e-8, (what, c)
