"""Per-kernel parity: HIP GEMM / LayerNorm / attention vs a
plain torch fp32 reference on the same bf16 operands."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _lib():
    from miclip import _native
    return _native


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (100, 128, 64), (513, 384, 768), (3200, 2304, 768),
                                   (777, 768, 3072)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm(gpu, M, N, K, epi):
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K + epi)
    A = (torch.randn(M, K, generator=g) * 0.5).bfloat16().to(gpu)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16().to(gpu)
    bias = torch.randn(N, generator=g).float().to(gpu)
    ref = A.float() @ W.float().t() + bias
    if epi in (0, 1):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    else:
        out = torch.randn(M, N, generator=g).float().to(gpu) if epi == 2 else torch.empty(M, N, device=gpu)
        base = out.clone()
    N_.check(N_.lib().mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), out.data_ptr(), M, N, K, epi,
                                 _stream()), "gemm")
    torch.cuda.synchronize()
    if epi == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    if epi == 2:
        ref = ref + base
    got = out.float()
    err = (got - ref).abs().max().item()
    tol = (2e-2 if epi in (0, 1) else 2e-4) * max(1.0, ref.abs().max().item())
    assert err < tol, f"max err {err} (tol {tol})"


@pytest.mark.parametrize("M,N,K,epi", [(20000, 3072, 768, 1), (5000, 2304, 768, 0), (3000, 768, 3072, 0),
                                       (777, 768, 128, 1), (256, 256, 256, 0), (70001, 768, 768, 0)])
def test_gemm_8phase_schedules_bit_identical(gpu, M, N, K, epi):
    """The 8-phase kernels (gemm_8p v98, gemm_8q v110 block epilogue / v113 flat DMAs; gemm_8r v120 256 x 128 deferred epilogue
    DMAs) run the same MFMA order and epilogue arithmetic, so their outputs
    must match bit for bit, over multi-tile persistent walks, partial last
    M-tiles and one-pair K; v98 is also checked against torch fp32.  The
    variants live in the A/B build (scripts/ab); the product library's default
    path must equal them too."""
    import torch
    N_ = _lib()
    AB = N_.lib_ab()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = (torch.rand(M, K, generator=g) * 2 - 1).bfloat16().to(gpu)
    W = ((torch.rand(N, K, generator=g) * 2 - 1) * K ** -0.5).bfloat16().to(gpu)
    bias = torch.randn(N, generator=g).float().to(gpu)
    outs = {}
    for v in (98, 110, 113, 120, 0):
        out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
        L = N_.lib() if v == 0 else AB            # v = 0: the product library's default dispatch
        rc = L.mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), out.data_ptr(), M, N, K, epi | (v << 8),
                          _stream())
        if rc:
            raise N_.MiClipError(f"gemm v{v}: {L.mi_last_error()}")
        outs[v] = out
    torch.cuda.synchronize()
    ref = A.float() @ W.float().t() + bias
    if epi == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    err = (outs[98].float() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err
    for v in (110, 113, 120):
        assert torch.equal(outs[v], outs[98]), f"v{v} differs from v98"
    # the product default is gemm_8q wherever it applies (K >= 256); below that the ping-pong kernel
    if K >= 256:
        assert torch.equal(outs[0], outs[110]), "product default differs from v110"
    else:
        assert (outs[0].float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())
    # the product library has no schedule overrides: they fail loudly instead of falling back
    rc = N_.lib().mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), outs[0].data_ptr(), M, N, K,
                             epi | (98 << 8), _stream())
    assert rc == -3 and b"A/B build" in N_.lib().mi_last_error()      # MI_ERR_UNSUPPORTED


def test_gemm_asymmetric_identity(gpu):
    """A = I with an asymmetric W catches a transposed C write (guide §3)."""
    import torch
    N_ = _lib()
    M, N, K = 128, 128, 128
    A = torch.eye(M, K, dtype=torch.bfloat16, device=gpu)
    W = (torch.arange(N * K, device=gpu).reshape(N, K) % 251).bfloat16()
    out = torch.empty(M, N, device=gpu)
    N_.check(N_.lib().mi_op_gemm(A.data_ptr(), W.data_ptr(), None, out.data_ptr(), M, N, K, 3, _stream()), "gemm")
    torch.cuda.synchronize()
    assert torch.equal(out, W.float().t().contiguous())


@pytest.mark.parametrize("rows,W", [(1, 128), (77, 512), (1000, 768), (50, 1024)])
def test_layernorm(gpu, rows, W):
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(rows + W)
    x = (torch.randn(rows, W, generator=g) * 3 + 1).to(gpu)
    gamma = (1 + 0.1 * torch.randn(W, generator=g)).to(gpu)
    beta = (0.1 * torch.randn(W, generator=g)).to(gpu)
    out = torch.empty(rows, W, dtype=torch.bfloat16, device=gpu)
    N_.check(N_.lib().mi_op_layernorm(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), out.data_ptr(), rows, W,
                                      _stream()), "layernorm")
    torch.cuda.synchronize()
    ref = torch.nn.functional.layer_norm(x.double(), (W,), gamma.double(), beta.double(), 1e-5)
    err = (out.double() - ref).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("rows,W", [(1, 128), (1000, 768), (50, 1024), (33, 512)])
@pytest.mark.parametrize("xmode", [0, 1, 2])
def test_residual_ln(gpu, rows, W, xmode):
    """x += delta; out = LN(x) for the three residual storage modes (f32, f32 -> fp16, fp16 half-row).
    The written-back residual is bit-exact: the f32 sum x + bf16(delta), rounded to fp16 when stored as fp16."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(rows * 3 + W + xmode)
    x32 = torch.randn(rows, W, generator=g) * 3 + 1
    delta = torch.randn(rows, W, generator=g).bfloat16()
    gamma = (1 + 0.1 * torch.randn(W, generator=g))
    beta = 0.1 * torch.randn(W, generator=g)
    slot = torch.zeros(rows, W, dtype=torch.float32)  # f32 row slots; fp16 modes use their first halves
    if xmode == 2:
        x32 = x32.half().float()  # the fp16 stream holds fp16 values
        slot.view(torch.float16).view(rows, 2 * W)[:, :W] = x32.half()
    else:
        slot.copy_(x32)
    xd = slot.to(gpu)
    out = torch.empty(rows, W, dtype=torch.bfloat16, device=gpu)
    dd, gd, bd = delta.to(gpu), gamma.to(gpu), beta.to(gpu)  # held: a freed temporary's block is reused
    N_.check(N_.lib().mi_op_residual_ln(xd.data_ptr(), dd.data_ptr(), gd.data_ptr(), bd.data_ptr(), out.data_ptr(),
                                        rows, W, xmode, _stream()), "residual_ln")
    torch.cuda.synchronize()
    s = x32 + delta.float()  # f32 add, as the kernel
    if xmode == 0:
        assert torch.equal(xd.cpu(), s)
    else:
        got = xd.cpu().view(torch.float16).view(rows, 2 * W)[:, :W]
        assert torch.equal(got, s.half())
    ref = torch.nn.functional.layer_norm(s.double(), (W,), gamma.double(), beta.double(), 1e-5)
    err = (out.cpu().double() - ref).abs().max().item()
    assert err < 2e-2, err


def _half_slots(x16):
    """fp16 rows [rows, W] in the vision tower's half-slot layout: f32 slots [rows, W]
    whose first halves hold the row (row stride 2W fp16 elements)."""
    import torch
    rows, W = x16.shape
    slot = torch.zeros(rows, W, dtype=torch.float32)
    slot.view(torch.float16).view(rows, 2 * W)[:, :W] = x16
    return slot


@pytest.mark.parametrize("rows,W", [(1, 128), (1000, 768), (50, 1024), (33, 512)])
def test_residual_stats(gpu, rows, W):
    """mi_op_residual_stats: the fp16 residual add is bit-exact (f32 x + bf16 delta rounded to
    fp16), and rs holds (rstd, rstd * mean) of the STORED fp16 row (LayerNorm eps 1e-5)."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(rows * 5 + W)
    x16 = (torch.randn(rows, W, generator=g) * 3 + 1).half()
    delta = torch.randn(rows, W, generator=g).bfloat16()
    xd, dd = _half_slots(x16).to(gpu), delta.to(gpu)
    rs = torch.full((rows, 2), float("nan"), device=gpu)
    N_.check(N_.lib().mi_op_residual_stats(xd.data_ptr(), dd.data_ptr(), rs.data_ptr(), rows, W, _stream()),
             "residual_stats")
    torch.cuda.synchronize()
    s = (x16.float() + delta.float()).half()
    assert torch.equal(xd.cpu().view(torch.float16).view(rows, 2 * W)[:, :W], s)
    sd = s.double()
    mean = sd.mean(1)
    rstd = 1 / torch.sqrt(((sd - mean[:, None]) ** 2).mean(1) + 1e-5)
    np.testing.assert_allclose(rs[:, 0].cpu().double(), rstd, rtol=2e-6)
    np.testing.assert_allclose(rs[:, 1].cpu().double(), rstd * mean, rtol=2e-6, atol=2e-6)


@pytest.mark.parametrize("M,N,K,gelu,half_slot", [(256, 256, 256, 0, True), (1000, 2304, 768, 0, True),
                                                  (20000, 3072, 768, 1, True), (777, 4096, 1024, 1, True),
                                                  (513, 768, 768, 0, False), (300, 3072, 768, 1, False)])
def test_gemm_ln(gpu, M, N, K, gelu, half_slot):
    """mi_op_gemm_ln (LayerNorm folded into the GEMM: the bf16 vision tower's in_proj after ln_1
    and c_fc + QuickGELU after ln_2) against float64 LN(x) W^T + b with the UNFOLDED weights:
    the fold itself (W' = fp16(W * gamma), colsum, colc) is part of what is checked.  Tolerance
    as the bf16 GEMMs above (2e-2 of max(1, |ref|)); partial last M-tiles, the half-slot
    operand stride 2K and plain rows."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + gelu)
    x16 = (torch.randn(M, K, generator=g) * 2 + 0.5).half()
    W = torch.randn(N, K, generator=g) * K ** -0.5
    gamma = 1 + 0.2 * torch.randn(K, generator=g)
    beta = 0.1 * torch.randn(K, generator=g)
    bias = 0.1 * torch.randn(N, generator=g)
    Wf = (W.double() * gamma.double()).half()
    colsum = Wf.double().sum(1).float()
    colc = (bias.double() + W.double() @ beta.double()).float()
    xd = _half_slots(x16).to(gpu) if half_slot else x16.to(gpu)
    lda = 2 * K if half_slot else K
    xs = x16.double()
    mean = xs.mean(1)
    rstd = 1 / torch.sqrt(((xs - mean[:, None]) ** 2).mean(1) + 1e-5)
    rs = torch.zeros(M + 256, 2)                  # readable for M + 256 rows (the header's contract)
    rs[:M, 0], rs[:M, 1] = rstd.float(), (rstd * mean).float()
    rs, Wd, sd, cd = rs.to(gpu), Wf.to(gpu), colsum.to(gpu), colc.to(gpu)
    out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
    N_.check(N_.lib().mi_op_gemm_ln(xd.data_ptr(), lda, rs.data_ptr(), Wd.data_ptr(), sd.data_ptr(), cd.data_ptr(),
                                    out.data_ptr(), M, N, K, gelu, _stream()), "gemm_ln")
    torch.cuda.synchronize()
    ln = torch.nn.functional.layer_norm(xs, (K,), gamma.double(), beta.double(), 1e-5)
    ref = ln @ W.double().t() + bias.double()
    if gelu:
        ref = ref * torch.sigmoid(1.702 * ref)
    got = out.cpu().double()
    assert torch.isfinite(got).all()
    err = (got - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err


@pytest.mark.parametrize("M,W,K,half_slot", [(256, 256, 256, True), (1000, 768, 768, True), (777, 768, 3072, True),
                                             (20000, 768, 768, True), (300, 1024, 4096, False),
                                             (513, 512, 1024, False)])
def test_gemm_residual(gpu, M, W, K, half_slot):
    """mi_op_gemm_residual (out_proj / c_proj with the residual add fused into the epilogue)
    against the unfused pair it replaces: mi_op_gemm (bf16 out) then mi_op_residual_stats.
    The stored fp16 residual stream must be bit-identical; rs (combined from per-64-column
    partials) within 2e-6 relative of the float64 statistics of the stored rows, as
    test_residual_stats.  Partial last M-tiles, multi-tile persistent walks, K = 4W."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + 3 * W + K)
    x16 = (torch.randn(M, W, generator=g) * 3 + 1).half()
    A = (torch.randn(M, K, generator=g) * 0.5).bfloat16()
    Wt = (torch.randn(W, K, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(W, generator=g).float()
    Ad, Wd, bd = A.to(gpu), Wt.to(gpu), bias.to(gpu)
    delta = torch.empty(M, W, dtype=torch.bfloat16, device=gpu)
    N_.check(N_.lib().mi_op_gemm(Ad.data_ptr(), Wd.data_ptr(), bd.data_ptr(), delta.data_ptr(), M, W, K, 0,
                                 _stream()), "gemm")
    xd = _half_slots(x16).to(gpu) if half_slot else x16.to(gpu)
    ldx = 2 * W if half_slot else W
    ps = torch.full((M, W // 64, 2), float("nan"), device=gpu)
    rs = torch.full((M, 2), float("nan"), device=gpu)
    N_.check(N_.lib().mi_op_gemm_residual(xd.data_ptr(), ldx, Ad.data_ptr(), K, Wd.data_ptr(), bd.data_ptr(),
                                          ps.data_ptr(), rs.data_ptr(), M, W, K, _stream()), "gemm_residual")
    torch.cuda.synchronize()
    s = (x16.float() + delta.cpu().float()).half()
    got = xd.cpu().view(torch.float16).view(M, 2 * W)[:, :W] if half_slot else xd.cpu()
    assert torch.equal(got, s)
    sd = s.double()
    mean = sd.mean(1)
    rstd = 1 / torch.sqrt(((sd - mean[:, None]) ** 2).mean(1) + 1e-5)
    np.testing.assert_allclose(rs[:, 0].cpu().double(), rstd, rtol=2e-6)
    np.testing.assert_allclose(rs[:, 1].cpu().double(), rstd * mean, rtol=2e-6, atol=2e-6)
    # the partials themselves: per 64 columns, the sum and the squared deviations from its mean
    blk = sd.view(M, W // 64, 64)
    psum = blk.sum(2)
    pm2 = ((blk - psum[..., None] / 64) ** 2).sum(2)
    np.testing.assert_allclose(ps[..., 0].cpu().double(), psum, rtol=1e-5, atol=1e-3)
    np.testing.assert_allclose(ps[..., 1].cpu().double(), pm2, rtol=1e-5, atol=1e-3)


def test_gemm_residual_rejects_unsupported_shapes(gpu):
    import torch
    N_ = _lib()
    t = torch.zeros(4096, device=gpu)
    p = t.data_ptr()
    # W not a multiple of 256, K not a multiple of 128, M < 256, lda < K, ldx < W, W > 1024
    for M, W, K, lda, ldx in [(256, 200, 256, 256, 200), (256, 256, 192, 192, 256), (100, 256, 256, 256, 256),
                              (256, 256, 256, 128, 256), (256, 256, 256, 256, 128), (256, 1280, 256, 256, 1280)]:
        assert N_.lib().mi_op_gemm_residual(p, ldx, p, lda, p, p, p, p, M, W, K, _stream()) == -3
    assert N_.lib().mi_op_gemm_residual(0, 256, p, 256, p, p, p, p, 256, 256, 256, _stream()) == -1


def test_gemm_ln_rejects_unsupported_shapes(gpu):
    import torch
    N_ = _lib()
    t = torch.zeros(4096, device=gpu)
    p = t.data_ptr()
    for M, N, K, lda in [(256, 200, 256, 256), (256, 256, 192, 192), (100, 256, 256, 256), (256, 256, 256, 128)]:
        assert N_.lib().mi_op_gemm_ln(p, lda, p, p, p, p, p, M, N, K, 0, _stream()) == -3    # MI_ERR_UNSUPPORTED
    assert N_.lib().mi_op_gemm_ln(p, 256, p, p, p, p, p, 256, 256, 256, 2, _stream()) == -1  # MI_ERR_ARG (gelu)


@pytest.mark.parametrize("B,S,W,causal", [(1, 50, 768, 0), (7, 50, 768, 0), (3, 77, 512, 1), (2, 17, 128, 0),
                                          (2, 10, 256, 1), (1, 257, 1024, 0), (4, 197, 768, 0),
                                          # long-sequence (flash) kernel: L/14@336 = 577 tokens, ragged tails,
                                          # causal, chunk boundaries
                                          (2, 577, 1024, 0), (1, 300, 256, 1), (3, 130, 128, 0), (1, 640, 128, 1),
                                          (2, 97, 256, 0), (1, 128, 192, 1), (2, 385, 128, 0)])
# default (S > 64 non-causal: K/V resident in LDS; else the flash kernel) / one-wave kernel (S <= 96) /
# chunk-streaming flash kernel (S > 64)
@pytest.mark.parametrize("flash", [0, 0x100, 0x200])
def test_attention(gpu, B, S, W, causal, flash):
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(B * S + W + causal)
    qkv = (torch.randn(B * S, 3 * W, generator=g) * 1.5).bfloat16().to(gpu)
    out = torch.empty(B * S, W, dtype=torch.bfloat16, device=gpu)
    L = N_.lib_ab() if flash == 0x100 else N_.lib()   # the one-wave kernel is in the A/B build
    rc = L.mi_op_attention(qkv.data_ptr(), out.data_ptr(), B, S, W, causal | flash, _stream())
    if rc:
        raise N_.MiClipError(f"attention: {L.mi_last_error()}")
    torch.cuda.synchronize()
    H = W // 64
    x = qkv.double().reshape(B, S, 3, H, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = q @ k.transpose(-1, -2) * 0.125
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device=gpu), 1), float("-inf"))
    ref = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B * S, W)
    err = (out.double() - ref).abs().max().item()
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err


def test_errors_are_raised(gpu):
    import torch
    N_ = _lib()
    A = torch.zeros(8, 64, dtype=torch.bfloat16, device=gpu)
    rc = N_.lib().mi_op_gemm(A.data_ptr(), A.data_ptr(), None, A.data_ptr(), 8, 100, 64, 0, _stream())
    assert rc != 0 and b"N" in N_.lib().mi_last_error()
    with pytest.raises(N_.MiClipError):
        N_.check(rc, "gemm")


@pytest.mark.parametrize("S", [577, 257, 130])
@pytest.mark.parametrize("mode", [0, 0x200])
def test_attention_growing_max(gpu, S, mode):
    """Scores whose row max keeps growing along the keys: every 64-key chunk
    moves the running max by more than the lazy-rescale threshold (2^8), so
    the rescale branch runs on each chunk (attention_res_kernel by default,
    attention_flash_kernel with bit 9)."""
    import torch
    N_ = _lib()
    B, W = 2, 256
    g = torch.Generator(device="cpu").manual_seed(S)
    qkv = torch.randn(B, S, 3, W // 64, 64, generator=g)
    qkv[:, :, 0] = qkv[:, :, 0].abs() * 0.5 + 0.5                      # q > 0
    ramp = torch.linspace(0.05, 4.0, S).reshape(1, S, 1, 1)
    qkv[:, :, 1] = qkv[:, :, 1].abs() * ramp                           # k grows with the key index
    qkv = qkv.reshape(B * S, 3 * W).bfloat16().to(gpu)
    out = torch.empty(B * S, W, dtype=torch.bfloat16, device=gpu)
    N_.check(N_.lib().mi_op_attention(qkv.data_ptr(), out.data_ptr(), B, S, W, mode, _stream()), "attention")
    torch.cuda.synchronize()
    H = W // 64
    x = qkv.double().reshape(B, S, 3, H, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    ref = (torch.softmax(q @ k.transpose(-1, -2) * 0.125, -1) @ v).transpose(1, 2).reshape(B * S, W)
    err = (out.double() - ref).abs().max().item()
    assert err < 3e-2, err


@pytest.mark.parametrize("B,S,W", [(2, 577, 1024), (3, 257, 768), (2, 130, 128), (1, 97, 256), (2, 385, 128),
                                   (1, 640, 192)])
@pytest.mark.parametrize("var", ["2", "3"])
def test_attention_res_variants_bit_identical(gpu, monkeypatch, B, S, W, var):
    """attention_res_kernel's variants (A/B build, MICLIP_ATTN_VAR): 11 (= 1) = 8 waves,
    one query tile at a time, every tile whole (the product default for S <= 320);
    2 = 8 waves, two tiles at a time (shared K / V^T
    fragment reads, an odd last tile alone); 3 = 16 waves.  Per tile the arithmetic
    is the same, so every variant equals variant 11 bit for bit — tile counts
    37 / 17 / 9 / 7 / 25 / 40 cover odd and even pairs.  (Variant 12 splits a
    nearly empty last tile across the waves: test_attention_split_last_tile.)"""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(S + W)
    qkv = (torch.randn(B * S, 3 * W, generator=g) * 1.5).bfloat16().to(gpu)
    a = torch.empty(B * S, W, dtype=torch.bfloat16, device=gpu)
    b = torch.empty_like(a)
    La = N_.lib_ab()
    monkeypatch.setenv("MICLIP_ATTN_VAR", "11")
    assert La.mi_op_attention(qkv.data_ptr(), a.data_ptr(), B, S, W, 0, _stream()) == 0, La.mi_last_error()
    monkeypatch.setenv("MICLIP_ATTN_VAR", var)
    assert La.mi_op_attention(qkv.data_ptr(), b.data_ptr(), B, S, W, 0, _stream()) == 0, La.mi_last_error()
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("B,S,W", [(2, 577, 1024), (3, 257, 768), (2, 130, 128), (1, 97, 256), (2, 385, 128),
                                   (1, 640, 192), (2, 100, 128)])
@pytest.mark.parametrize("grow", [False, True])
@pytest.mark.parametrize("var", ["4", "5", "6", "10"])
def test_attention_r32_kernel(gpu, monkeypatch, B, S, W, grow, var):
    """attention_r32_kernel (32x32x16 MFMAs, P kept in the lane as the PV B
    operand, V^T by transposed reads; MICLIP_ATTN_VAR=4 (8 waves, two blocks at
    a time), 5 (12 waves, one block), 6 (12 waves, staggered start), 10 (12 waves,
    two-phase K/V load) in the A/B build)
    against float64, on random rows and on rows whose max grows along the keys
    (the lazy-rescale branch on every chunk).  Query-block counts 19 / 9 / 5 /
    4 / 13 / 20 / 4 cover pairs, singles and a last block of one row."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(S + W + grow)
    if grow:
        qkv = torch.randn(B, S, 3, W // 64, 64, generator=g)
        qkv[:, :, 0] = qkv[:, :, 0].abs() * 0.5 + 0.5
        qkv[:, :, 1] = qkv[:, :, 1].abs() * torch.linspace(0.05, 4.0, S).reshape(1, S, 1, 1)
        qkv = qkv.reshape(B * S, 3 * W).bfloat16().to(gpu)
    else:
        qkv = (torch.randn(B * S, 3 * W, generator=g) * 1.5).bfloat16().to(gpu)
    out = torch.empty(B * S, W, dtype=torch.bfloat16, device=gpu)
    monkeypatch.setenv("MICLIP_ATTN_VAR", var)
    La = N_.lib_ab()
    assert La.mi_op_attention(qkv.data_ptr(), out.data_ptr(), B, S, W, 0, _stream()) == 0, La.mi_last_error()
    torch.cuda.synchronize()
    H = W // 64
    x = qkv.double().reshape(B, S, 3, H, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    ref = (torch.softmax(q @ k.transpose(-1, -2) * 0.125, -1) @ v).transpose(1, 2).reshape(B * S, W)
    err = (out.double() - ref).abs().max().item()
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err
    if var == "10":   # the two-phase K/V load changes no arithmetic: bit-identical to variant 5
        d = torch.empty_like(out)
        monkeypatch.setenv("MICLIP_ATTN_VAR", "5")
        assert La.mi_op_attention(qkv.data_ptr(), d.data_ptr(), B, S, W, 0, _stream()) == 0, La.mi_last_error()
        torch.cuda.synchronize()
        assert torch.equal(d, out)
    if var == "5" and S > 320:   # the product default for S > 320 is this kernel
        d = torch.empty_like(out)
        N_.check(N_.lib().mi_op_attention(qkv.data_ptr(), d.data_ptr(), B, S, W, 0, _stream()), "attention")
        torch.cuda.synchronize()
        assert torch.equal(d, out)


@pytest.mark.parametrize("B,S,W", [(3, 257, 1024), (2, 257, 768), (2, 130, 256), (1, 97, 128), (2, 193, 128),
                                   (1, 260, 64)])
def test_attention_split_last_tile(gpu, monkeypatch, B, S, W):
    """attention_res_kernel SPLIT (A/B variant 12, measured and not the default: for
    64 < S <= 320 with S % 16 in 1..4, e.g. ViT-L/14's 257 tokens): the nearly empty
    last query tile is shared out over the 8 waves' key tiles and its partial softmax
    states merged in LDS.  Rows of the full tiles are bit-identical to the default
    kernel (variant 11); the last tile's rows are within the float64 tolerance of
    test_attention."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(3 * S + W)
    qkv = (torch.randn(B * S, 3 * W, generator=g) * 1.5).bfloat16().to(gpu)
    a = torch.empty(B * S, W, dtype=torch.bfloat16, device=gpu)
    b = torch.empty_like(a)
    La = N_.lib_ab()
    monkeypatch.setenv("MICLIP_ATTN_VAR", "12")
    assert La.mi_op_attention(qkv.data_ptr(), a.data_ptr(), B, S, W, 0, _stream()) == 0, La.mi_last_error()
    monkeypatch.setenv("MICLIP_ATTN_VAR", "11")
    assert La.mi_op_attention(qkv.data_ptr(), b.data_ptr(), B, S, W, 0, _stream()) == 0, La.mi_last_error()
    torch.cuda.synchronize()
    last = 16 * ((S + 15) // 16 - 1)
    full = torch.arange(B * S, device=gpu) % S < last
    assert torch.equal(a[full], b[full])
    H = W // 64
    x = qkv.double().reshape(B, S, 3, H, 64)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    ref = (torch.softmax(q @ k.transpose(-1, -2) * 0.125, -1) @ v).transpose(1, 2).reshape(B * S, W)
    err = (a.double() - ref).abs().max().item()
    assert err < 3e-2 * max(1.0, ref.abs().max().item()), err
    err_b = (b.double() - ref)[~full].abs().max().item()
    assert (a.double() - ref)[~full].abs().max().item() <= 2 * err_b + 2e-3


@pytest.mark.parametrize("M,N,K,epi", [(1, 64, 32, 0), (100, 128, 64, 1), (513, 384, 768, 2), (3000, 3072, 768, 1),
                                       (777, 768, 3072, 2), (50, 512, 768, 3), (20000, 2304, 768, 0)])
def test_gemm_f32(gpu, M, N, K, epi):
    """mi_op_gemm_f32 (the fp32 tower's exact-f32 MFMA GEMM) against float64, within f32
    rounding (1e-5 of max(1, |ref|)); epilogues 0 store, 1 QuickGELU, 2 +=, 3 ReLU."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M * 3 + N + K + epi)
    A = (torch.randn(M, K, generator=g) * 0.5).to(gpu)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    base = torch.randn(M, N, generator=g).to(gpu)
    out = base.clone() if epi == 2 else torch.full((M, N), float("nan"), device=gpu)
    N_.check(N_.lib().mi_op_gemm_f32(A.data_ptr(), W.data_ptr(), bias.data_ptr(), out.data_ptr(), M, N, K, epi,
                                     _stream()), "gemm_f32")
    torch.cuda.synchronize()
    ref = A.double() @ W.double().t() + bias.double()
    if epi == 1:
        ref = ref * torch.sigmoid(1.702 * ref)
    elif epi == 2:
        ref = ref + base.double()
    elif epi == 3:
        ref = ref.clamp_min(0)
    err = (out.double() - ref).abs().max().item()
    assert err < 1e-5 * max(1.0, ref.abs().max().item()), err


def _bf16_rne(x):
    """float32 -> bf16 bits, round to nearest even (NaN stays NaN), as the kernels' f2bf."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return np.where(nan, ((u >> 16) | 0x40).astype(np.uint16), r)


def _split6_ref(x, role, gelu):
    x = np.asarray(x, np.float32)
    if gelu:
        x = (x * (np.float32(1) / (np.float32(1) + np.exp(np.float32(-1.702) * x)))).astype(np.float32)
    b2f = lambda h: (h.astype(np.uint32) << 16).view(np.float32)
    x1 = _bf16_rne(x)
    fin = np.isfinite(x)
    x1 = np.where(fin & ((x1 & 0x7FFF) == 0x7F80), (x1 & 0x8000) | 0x7F7F, x1).astype(np.uint16)
    with np.errstate(invalid="ignore"):
        r1 = (x - b2f(x1)).astype(np.float32)
        x2 = np.where(fin, _bf16_rne(r1), 0).astype(np.uint16)
        x3 = np.where(fin, _bf16_rne((r1 - b2f(x2)).astype(np.float32)), 0).astype(np.uint16)
    t = (x1, x2, x3)
    order = (0, 0, 0, 1, 1, 2) if role else (0, 1, 2, 0, 1, 0)
    return np.concatenate([t[o] for o in order], axis=1)


@pytest.mark.parametrize("role,gelu", [(0, 0), (1, 0), (0, 1)])
def test_split6_bit_exact(gpu, role, gelu):
    """mi_op_split6 (the fp32 tower's split-bf16 operands) against its numpy restatement, bit
    for bit, with inf / NaN / subnormal / zero / past-bf16-range (3.4e38) entries; and x1 + x2 + x3 = x to 2^-24 relative
    (2^-133 absolute below the normal range).
    (gelu: only the finite-row comparison -- expf and numpy's exp may differ in the last bit.)"""
    import torch
    N_ = _lib()
    rng = np.random.default_rng(7 + role + 2 * gelu)
    rows, K = 300, 768
    x = (rng.standard_normal((rows, K)) * np.exp(rng.uniform(-20, 20, (rows, K)))).astype(np.float32)
    if not gelu:
        x[0, :8] = [np.inf, -np.inf, np.nan, 0.0, -0.0, 1e-40, -3e-39, 3.4e38]
    xd = torch.from_numpy(x).to(gpu)
    out = torch.zeros(rows, 6 * K, dtype=torch.int16, device=gpu)
    N_.check(N_.lib().mi_op_split6(xd.data_ptr(), K, rows, K, role, gelu, out.data_ptr(), _stream()), "split6")
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    if gelu:
        xg = torch.from_numpy(x).to(gpu)
        xg = (xg * (1.0 / (1.0 + torch.exp(-1.702 * xg)))).cpu().numpy()   # the device's value, then split
        ref = _split6_ref(xg, role, 0)
        ok = np.isfinite(xg).all(axis=1)
        close = (got[ok] == ref[ok]).mean()
        assert close > 0.999, close
        return
    ref = _split6_ref(x, role, 0)
    assert np.array_equal(got, ref)
    b2f = lambda h: (h.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    t = [got[:, j * K:(j + 1) * K] for j in range(6)]
    x1, x2, x3 = (t[0], t[1], t[2]) if role == 0 else (t[0], t[3], t[5])
    fin = np.isfinite(x)
    s = b2f(x1) + b2f(x2) + b2f(x3)
    err = np.abs(s[fin] - x[fin].astype(np.float64))
    # relative 2^-24, and the bf16 terms' subnormal spacing (2^-133) for f32-subnormal inputs
    assert (err <= 2.0 ** -24 * np.abs(x[fin].astype(np.float64)) + 2.0 ** -133).all()


@pytest.mark.parametrize("M,N,K,epi", [(513, 384, 768, 3), (3000, 768, 3072, 2), (20000, 2304, 768, 3)])
def test_split6_gemm_f32_grade(gpu, M, N, K, epi):
    """The fp32 tower's GEMM as run since round 4: split-bf16 operands (mi_op_split6) and one
    bf16 GEMM over K' = 6K with an f32 epilogue (mi_op_gemm 3 = store, 2 = +=), against float64
    within f32-GEMM error (1e-5 of max(1, |ref|), as test_gemm_f32)."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    A = (torch.randn(M, K, generator=g) * 0.5).to(gpu)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    base = torch.randn(M, N, generator=g).to(gpu)
    A6 = torch.empty(M, 6 * K, dtype=torch.int16, device=gpu)
    W6 = torch.empty(N, 6 * K, dtype=torch.int16, device=gpu)
    L = N_.lib()
    N_.check(L.mi_op_split6(A.data_ptr(), K, M, K, 0, 0, A6.data_ptr(), _stream()), "split6 A")
    N_.check(L.mi_op_split6(W.data_ptr(), K, N, K, 1, 0, W6.data_ptr(), _stream()), "split6 W")
    out = base.clone() if epi == 2 else torch.full((M, N), float("nan"), device=gpu)
    N_.check(L.mi_op_gemm(A6.data_ptr(), W6.data_ptr(), bias.data_ptr(), out.data_ptr(), M, N, 6 * K, epi, _stream()),
             "gemm")
    torch.cuda.synchronize()
    ref = A.double() @ W.double().t() + bias.double()
    if epi == 2:
        ref = ref + base.double()
    err = (out.double() - ref).abs().max().item()
    assert err < 1e-5 * max(1.0, ref.abs().max().item()), err


# ---------------------------------------------------------------- split-f16 operands (round 5)
def _split2h_ref(x, role, gelu):
    """numpy restatement of split2h_rows (precise.hip): per-row power-of-two scale with the row's
    max |x s| in [2^13, 2^14), x1 = f16(x s), x2 = f16(x s - x1) (0 where x1 is not finite),
    activations [x1 x1 x2] / weights [x1 x2 x1], scale = 1 / s."""
    x = np.asarray(x, np.float32)
    if gelu:
        x = (x * (np.float32(1) / (np.float32(1) + np.exp(np.float32(-1.702) * x)))).astype(np.float32)
    with np.errstate(invalid="ignore", over="ignore"):
        mx = np.nanmax(np.where(np.isnan(x), 0, np.abs(x)), axis=1)
        ok = (mx > 0) & np.isfinite(mx)
        _, ex = np.frexp(np.where(ok, mx, 1).astype(np.float32))
        e = np.clip(np.where(ok, 14 - ex, 0), -126, 126).astype(np.int32)
        xs = np.ldexp(x, e[:, None]).astype(np.float32)
        x1 = xs.astype(np.float16)
        r = (xs - x1.astype(np.float32)).astype(np.float32)
        x2 = np.where(np.isfinite(x1), r.astype(np.float16), np.float16(0))
    t = (x1.view(np.uint16), x2.view(np.uint16))
    order = (0, 1, 0) if role else (0, 0, 1)
    return np.concatenate([t[o] for o in order], axis=1), np.ldexp(np.float32(1), -e).astype(np.float32)


@pytest.mark.parametrize("role,gelu,K", [(0, 0, 768), (1, 0, 768), (0, 0, 3072), (0, 1, 3072), (1, 0, 128)])
def test_split2h_bit_exact(gpu, role, gelu, K):
    """mi_op_split2h (the fp32 tower's split-f16 operands) against its numpy restatement, bit for
    bit, rows of magnitudes 1e-30 .. 1e30 with inf / NaN / zero / subnormal entries and an
    all-zero row; and (x1 + x2) / s = x to 2^-22 of the row's largest value."""
    import torch
    N_ = _lib()
    rng = np.random.default_rng(11 + role + 2 * gelu + K)
    rows = 300
    x = (rng.standard_normal((rows, K)) * np.exp(rng.uniform(-5, 5, (rows, K)))
         * np.exp(rng.uniform(-60, 60, (rows, 1)))).astype(np.float32)
    if gelu:
        x = (rng.standard_normal((rows, K)) * 3).astype(np.float32)
    else:
        x[0, :8] = [np.inf, -np.inf, np.nan, 0.0, -0.0, 1e-40, -3e-39, 3.4e38]
        x[1, :4] = [1e-40, -2e-39, 0.0, 5e-45]
        x[2] = 0.0
        x[3, :3] = [np.nan, 1.0, -2.0]
    xd = torch.from_numpy(x).to(gpu)
    out = torch.zeros(rows, 3 * K, dtype=torch.int16, device=gpu)
    sc = torch.zeros(rows, device=gpu)
    N_.check(N_.lib().mi_op_split2h(xd.data_ptr(), K, rows, K, role, gelu, out.data_ptr(), sc.data_ptr(), _stream()),
             "split2h")
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    gsc = sc.cpu().numpy()
    if gelu:   # the device's QuickGELU values (expf vs numpy's exp may differ in the last bit), then split
        xg = (xd * (1.0 / (1.0 + torch.exp(-1.702 * xd)))).cpu().numpy()
        ref, rsc = _split2h_ref(xg, role, 0)
        assert (got == ref).mean() > 0.999 and (gsc == rsc).mean() > 0.99
        return
    ref, rsc = _split2h_ref(x, role, 0)
    assert np.array_equal(gsc, rsc)
    assert np.array_equal(got, ref), np.argwhere(got != ref)[:5]
    h = lambda u: u.view(np.float16).astype(np.float64)
    x1, x2 = h(got[:, :K]), h(got[:, 2 * K:] if role == 0 else got[:, K:2 * K])
    fin = np.isfinite(x).all(axis=1)
    back = (x1 + x2) * gsc[:, None].astype(np.float64)
    bound = 2.0 ** -22 * np.abs(x.astype(np.float64)).max(axis=1, keepdims=True) + 2.0 ** -149
    assert (np.abs(back - x.astype(np.float64))[fin] <= bound[fin]).all()


@pytest.mark.parametrize("M,N,K,epi", [(513, 384, 768, 3), (3000, 768, 3072, 2), (20000, 2304, 768, 3),
                                       (1000, 256, 608, 3)])
def test_split2h_gemm_f32_grade(gpu, M, N, K, epi):
    """The fp32 tower's GEMM since round 5: split-f16 operands (mi_op_split2h) and one f16 GEMM
    over K' = 3K with the row / column scales in its f32 epilogue (mi_op_gemm_split2h 3 = store,
    2 = +=), against float64 within f32-GEMM error (1e-5 of max(1, |ref|), as test_gemm_f32);
    rows and weight rows of magnitudes spread over 1e-8 .. 1e8 (the scales keep every row's
    precision) -- checked row-relative."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    A = (torch.randn(M, K, generator=g) * 0.5 * torch.exp(torch.empty(M, 1).uniform_(-18, 18, generator=g))).to(gpu)
    W = (torch.randn(N, K, generator=g) * K ** -0.5 * torch.exp(torch.empty(N, 1).uniform_(-2, 2, generator=g))).to(gpu)
    bias = torch.randn(N, generator=g).to(gpu) * 0
    base = torch.randn(M, N, generator=g).to(gpu)
    A3 = torch.empty(M, 3 * K, dtype=torch.int16, device=gpu)
    W3 = torch.empty(N, 3 * K, dtype=torch.int16, device=gpu)
    sa, sw = torch.empty(M, device=gpu), torch.empty(N, device=gpu)
    L = N_.lib()
    N_.check(L.mi_op_split2h(A.data_ptr(), K, M, K, 0, 0, A3.data_ptr(), sa.data_ptr(), _stream()), "split2h A")
    N_.check(L.mi_op_split2h(W.data_ptr(), K, N, K, 1, 0, W3.data_ptr(), sw.data_ptr(), _stream()), "split2h W")
    out = base.clone() if epi == 2 else torch.full((M, N), float("nan"), device=gpu)
    N_.check(L.mi_op_gemm_split2h(A3.data_ptr(), W3.data_ptr(), sa.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                  out.data_ptr(), M, N, 3 * K, epi, _stream()), "gemm_split2h")
    torch.cuda.synchronize()
    ref = A.double() @ W.double().t() + bias.double() + (base.double() if epi == 2 else 0)
    # row-relative: the row's |A| |W| scale (the f32 GEMM's own error bound is relative to it);
    # the += path also rounds base + product to f32 (half an ulp of the result)
    rowscale = (A.double().abs() @ W.double().abs().t()).max(dim=1, keepdim=True).values
    err = (out.double() - ref).abs() - (2.0 ** -24 * ref.abs() if epi == 2 else 0)
    err = (err / rowscale.clamp_min(1e-300)).max().item()
    assert err < 1e-6, err


@pytest.mark.parametrize("M,N,K,epi", [(3000, 768, 3072, 2), (20000, 2304, 768, 3), (257, 256, 256, 3),
                                       (777, 512, 1024, 2), (256, 1024, 512, 3), (512, 768, 768, 2),
                                       (1023, 2304, 768, 3)])
def test_split2h_gemm_8phase_bit_identical(gpu, monkeypatch, M, N, K, epi):
    """The split-f16 GEMM on the 8-phase kernel (gemm_8q.hip's SPL epilogues, the default where
    it applies: N % 256 == 0, K' % 128 == 0, M >= 256) gives the ping-pong kernel's results bit
    for bit (A/B build, MICLIP_F32_8Q=0): store and += forms, with a bias, partial last m-tiles,
    rows of widely spread magnitudes; and it stays within the f32 grade of float64."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(7 * M + N + K + epi)
    A = (torch.randn(M, K, generator=g) * torch.exp(torch.empty(M, 1).uniform_(-9, 9, generator=g))).to(gpu)
    W = (torch.randn(N, K, generator=g) * K ** -0.5 * torch.exp(torch.empty(N, 1).uniform_(-2, 2, generator=g))).to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    base = torch.randn(M, N, generator=g).to(gpu)
    A3 = torch.empty(M, 3 * K, dtype=torch.int16, device=gpu)
    W3 = torch.empty(N, 3 * K, dtype=torch.int16, device=gpu)
    sa, sw = torch.empty(M, device=gpu), torch.empty(N, device=gpu)
    L = N_.lib()
    N_.check(L.mi_op_split2h(A.data_ptr(), K, M, K, 0, 0, A3.data_ptr(), sa.data_ptr(), _stream()), "split2h A")
    N_.check(L.mi_op_split2h(W.data_ptr(), K, N, K, 1, 0, W3.data_ptr(), sw.data_ptr(), _stream()), "split2h W")
    outs = []
    for lib, flag in ((L, None), (N_.lib_ab(), "0")):
        if flag is None:
            monkeypatch.delenv("MICLIP_F32_8Q", raising=False)
        else:
            monkeypatch.setenv("MICLIP_F32_8Q", flag)
        out = base.clone() if epi == 2 else torch.full((M, N), float("nan"), device=gpu)
        N_.check(lib.mi_op_gemm_split2h(A3.data_ptr(), W3.data_ptr(), sa.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                        out.data_ptr(), M, N, 3 * K, epi, _stream()), "gemm_split2h")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))
    ref = A.double() @ W.double().t() + bias.double() + (base.double() if epi == 2 else 0)
    rowscale = (A.double().abs() @ W.double().abs().t()).max(dim=1, keepdim=True).values + bias.double().abs().max()
    err = (outs[0].double() - ref).abs() - (2.0 ** -24 * ref.abs() if epi == 2 else 0)
    assert (err / rowscale).max().item() < 1e-6


@pytest.mark.parametrize("B,S,W,causal", [(37, 50, 768, 0), (5, 77, 512, 1), (3, 1, 128, 0), (4, 33, 128, 1),
                                          (6, 96, 256, 0), (2, 128, 128, 1), (9, 64, 192, 0)])
def test_attention_f32_descriptor_form_bit_identical(gpu, monkeypatch, B, S, W, causal):
    """The exact-f32 MFMA attention with its loads and stores through range-limited buffer
    descriptors (padding rows read zeros, their stores drop, no branches; the A/B build's
    MICLIP_ATTN_F32_V=4 at S <= 64, the product kernel at 64 < S <= 128) against the
    conditional-load form (MICLIP_ATTN_F32_V=1), bit for bit."""
    import torch
    N_ = _lib()
    rng = np.random.default_rng(B * 7 + S + W + causal)
    d = torch.from_numpy((rng.standard_normal((B * S, 3 * W)) * 2).astype(np.float32)).to(gpu)
    outs = []
    for lib, v in ((N_.lib_ab(), "4"), (N_.lib_ab(), "1")):
        monkeypatch.setenv("MICLIP_ATTN_F32_V", v)
        out = torch.full((B * S + 64, W), float("nan"), device=gpu)   # rows past B * S stay untouched
        N_.check(lib.mi_op_attention_f32(d.data_ptr(), out.data_ptr(), B, S, W, causal, _stream()), "attn f32")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][:B * S].view(torch.int32), outs[1][:B * S].view(torch.int32))
    assert torch.isnan(outs[0][B * S:]).all()


@pytest.mark.parametrize("M,N,K,epi", [(3000, 768, 3072, 2), (1023, 2304, 768, 3), (256, 256, 512, 3),
                                       (30000, 768, 768, 2), (30000, 3072, 768, 3)])
def test_split2h_dedup_layout_bit_identical(gpu, M, N, K, epi):
    """The activations' split stored once (mi_op_split2h role 2, [x1 x2]) and read by the
    8-phase GEMM as [x1 x1 x2] (mi_op_gemm_split2h epi | 0x100) give the full layout's results
    bit for bit; the role-2 rows are the role-0 rows without the repeated x1 block."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N + K)
    A = (torch.randn(M, K, generator=g) * torch.exp(torch.empty(M, 1).uniform_(-9, 9, generator=g))).to(gpu)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).to(gpu)
    bias = torch.randn(N, generator=g).to(gpu)
    base = torch.randn(M, N, generator=g).to(gpu)
    L = N_.lib()
    A3 = torch.empty(M, 3 * K, dtype=torch.int16, device=gpu)
    A2 = torch.empty(M, 2 * K, dtype=torch.int16, device=gpu)
    W3 = torch.empty(N, 3 * K, dtype=torch.int16, device=gpu)
    sa, sa2, sw = torch.empty(M, device=gpu), torch.empty(M, device=gpu), torch.empty(N, device=gpu)
    N_.check(L.mi_op_split2h(A.data_ptr(), K, M, K, 0, 0, A3.data_ptr(), sa.data_ptr(), _stream()), "split2h A")
    N_.check(L.mi_op_split2h(A.data_ptr(), K, M, K, 2, 0, A2.data_ptr(), sa2.data_ptr(), _stream()), "split2h A dedup")
    N_.check(L.mi_op_split2h(W.data_ptr(), K, N, K, 1, 0, W3.data_ptr(), sw.data_ptr(), _stream()), "split2h W")
    torch.cuda.synchronize()
    assert torch.equal(A2[:, :K], A3[:, :K]) and torch.equal(A2[:, K:], A3[:, 2 * K:]) and torch.equal(sa, sa2)
    outs = []
    for a, flag in ((A3, 0), (A2, 0x100)):
        out = base.clone() if epi == 2 else torch.full((M, N), float("nan"), device=gpu)
        N_.check(L.mi_op_gemm_split2h(a.data_ptr(), W3.data_ptr(), sa.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                      out.data_ptr(), M, N, 3 * K, epi | flag, _stream()), "gemm_split2h")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.int32), outs[1].view(torch.int32))


def _attn_ref(qkv, B, S, W, causal):
    H = W // 64
    x = qkv.reshape(B, S, 3, H, 64).astype(np.float64)
    q, k, v = x[:, :, 0], x[:, :, 1], x[:, :, 2]
    s = np.einsum("bqhd,bkhd->bhqk", q, k) / 8.0
    if causal:
        s = s + np.triu(np.full((S, S), -np.inf), 1)
    s = np.exp(s - s.max(-1, keepdims=True))
    p = s / s.sum(-1, keepdims=True)
    return np.einsum("bhqk,bkhd->bqhd", p, v).reshape(B * S, W)


@pytest.mark.parametrize("B,S,W,causal", [(37, 50, 768, 0), (5, 77, 512, 1), (3, 1, 128, 0), (4, 33, 128, 1),
                                          (6, 96, 256, 0), (2, 128, 128, 1), (2, 257, 128, 0)])
def test_attention_f32_vs_float64(gpu, B, S, W, causal):
    """mi_op_attention_f32 (the fp32 tower's MHA core: the exact-f32 MFMA kernel for S <= 128,
    the per-row kernel above) against float64 within f32 rounding."""
    import torch
    N_ = _lib()
    rng = np.random.default_rng(B * 1000 + S + W + causal)
    qkv = (rng.standard_normal((B * S, 3 * W)) * 2).astype(np.float32)
    d = torch.from_numpy(qkv).to(gpu)
    out = torch.full((B * S, W), float("nan"), device=gpu)
    N_.check(N_.lib().mi_op_attention_f32(d.data_ptr(), out.data_ptr(), B, S, W, causal, _stream()), "attn f32")
    torch.cuda.synchronize()
    ref = _attn_ref(qkv, B, S, W, causal)
    got = out.cpu().numpy().astype(np.float64)
    assert np.isfinite(got).all()
    err = np.abs(got - ref).max()
    assert err < 2e-6 * max(1.0, np.abs(ref).max()), err


@pytest.mark.parametrize("M,W,K", [(3000, 768, 768), (2049, 768, 3072), (70001, 768, 768)])
def test_gemm_residual_lagging_group_early_epilogue_bit_identical(gpu, monkeypatch, M, W, K):
    """The fused residual GEMM with the lagging M-group's epilogue beside the leading one's
    (gemm_8q F_BEARLY; A/B build, MICLIP_RES_ABL=14) against the product kernel: the stored fp16
    stream, the row statistics and the partials bit for bit (the same arithmetic, another place
    in the schedule); partial last tiles and multi-tile persistent walks."""
    import torch
    from miclip import _native
    g = torch.Generator(device="cpu").manual_seed(M + W + K)
    x16 = _half_slots((torch.randn(M, W, generator=g) * 3 + 1).half()).to(gpu)
    A = (torch.randn(M, K, generator=g) * 0.5).bfloat16().to(gpu)
    Wt = (torch.randn(W, K, generator=g) * K ** -0.5).bfloat16().to(gpu)
    bias = torch.randn(W, generator=g).float().to(gpu)
    outs = []
    for lib, env in ((_native.lib(), None), (_native.lib_ab(), "14")):
        if env:
            monkeypatch.setenv("MICLIP_RES_ABL", env)
        x = x16.clone()
        ps = torch.full((M, W // 64, 2), float("nan"), device=gpu)
        rs = torch.full((M, 2), float("nan"), device=gpu)
        _native.check(lib.mi_op_gemm_residual(x.data_ptr(), 2 * W, A.data_ptr(), K, Wt.data_ptr(), bias.data_ptr(),
                                              ps.data_ptr(), rs.data_ptr(), M, W, K, _stream()), "gemm_residual")
        torch.cuda.synchronize()
        outs.append((x.cpu(), ps.cpu(), rs.cpu()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B,S,W,causal", [(7, 50, 768, 0), (5, 33, 256, 1), (3, 64, 128, 0), (4, 17, 512, 1),
                                          (300, 50, 768, 0), (9, 1, 768, 0)])
def test_attention_f32_batched_bit_identical(gpu, monkeypatch, B, S, W, causal):
    """The exact-f32 MFMA forms of the fp32 tower's S <= 64 attention (A/B build): the batched-load
    kernel (attn_f32_mfma_b_kernel, MICLIP_ATTN_F32_V=4: each query block's loads issued together,
    K and V once per (sequence, head)), the kernel that loads next to each first use (=2, the
    round-5 default) and the one-wave-per-SIMD form with every load ahead of the first MFMA
    (attn_f32_mfma_pre_kernel, =3): the same MFMAs in the same order, so the outputs are
    bit-identical -- one and two key tiles, causal, 300 sequences, S = 1.  The product kernel
    (split-f16 operands) is checked against float64 by test_attention_f32_vs_float64 and against
    these by test_attention_f32_split_vs_exact."""
    import torch
    from miclip import _native
    rng = np.random.default_rng(B * 1000 + S + W + causal)
    qkv = torch.from_numpy((rng.standard_normal((B * S, 3 * W)) * 2).astype(np.float32)).to(gpu)
    outs = []
    for lib, env in ((_native.lib_ab(), "4"), (_native.lib_ab(), "2"), (_native.lib_ab(), "3")):
        monkeypatch.setenv("MICLIP_ATTN_F32_V", env)
        out = torch.full((B * S, W), float("nan"), device=gpu)
        _native.check(lib.mi_op_attention_f32(qkv.data_ptr(), out.data_ptr(), B, S, W, causal, _stream()), "attn f32")
        torch.cuda.synchronize()
        outs.append(out)
    assert torch.isfinite(outs[0]).all()
    for o in outs[1:]:
        assert torch.equal(outs[0].view(torch.int32), o.view(torch.int32))


@pytest.mark.parametrize("B,S,W,causal,scale", [(7, 50, 768, 0, 2.0), (5, 33, 256, 1, 2.0), (3, 64, 128, 0, 2.0),
                                                (300, 50, 768, 0, 2.0), (9, 1, 768, 0, 2.0), (6, 50, 512, 0, 30.0),
                                                (6, 50, 512, 0, 1e-3)])
def test_attention_f32_split_vs_exact(gpu, monkeypatch, B, S, W, causal, scale):
    """The product S <= 64 attention of the fp32 tower (attn_f32s_kernel: split-f16 operands on the
    f16 MFMA, the tower GEMMs' arithmetic) against the exact-f32 MFMA kernel (A/B build,
    MICLIP_ATTN_F32_V=4) and float64, with rows of any magnitude (each token's q / k / v scaled by
    10^[-3, 3]): scores then reach ~10^6, where any f32 rounding of a score moves the softmax, so
    the bound is the exact-f32 kernel's own error against float64 (the same grade: at most twice
    it, measured 0.2-1.3x) -- per (row, head), relative to the head's largest |V|."""
    import torch
    from miclip import _native
    rng = np.random.default_rng(B * 1000 + S + W + causal + int(scale * 7))
    qkv = (rng.standard_normal((B * S, 3 * W)) * scale).astype(np.float32)
    qkv *= (10.0 ** rng.uniform(-3, 3, size=(B * S, 1))).astype(np.float32)   # rows of any magnitude
    d = torch.from_numpy(qkv).to(gpu)
    outs = []
    for lib, env in ((_native.lib(), None), (_native.lib_ab(), "4")):
        if env:
            monkeypatch.setenv("MICLIP_ATTN_F32_V", env)
        out = torch.full((B * S, W), float("nan"), device=gpu)
        _native.check(lib.mi_op_attention_f32(d.data_ptr(), out.data_ptr(), B, S, W, causal, _stream()), "attn f32")
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy().astype(np.float64))
    ref = _attn_ref(qkv, B, S, W, causal)
    got, exact = outs
    assert np.isfinite(got).all()
    H = W // 64
    # per (row, head): error against the head's output scale (max |V| of the sequence's head)
    vmax = np.abs(qkv[:, 2 * W:].astype(np.float64)).reshape(B, S, H, 64).max(axis=(1, 3))   # [B, H]
    scl = np.repeat(vmax, S, axis=0)[:, :, None]                                                 # [B S, H, 1]
    e_split = (np.abs(got - ref).reshape(B * S, H, 64) / scl).max()
    e_exact = (np.abs(exact - ref).reshape(B * S, H, 64) / scl).max()
    print(f"split-f16 {e_split:.3e}  exact-f32 {e_exact:.3e}  (relative to the head's max |V|)")
    assert e_split <= 2 * e_exact + 2e-7, (e_split, e_exact)


@pytest.mark.parametrize("B,S,W,causal", [(7, 50, 768, 0), (5, 33, 256, 1), (300, 50, 768, 0), (4, 64, 128, 0),
                                          (3, 1, 512, 0)])
def test_attention_f32_split_output_bit_exact(gpu, B, S, W, causal):
    """mi_op_attention_f32_split (the fp32 tower's attention writing out_proj's split operand,
    round 6) against its restatement on the f32-output kernel's values: the sequence's scale from
    the bound (max over its rows of rmax * bw + bb) * (1 + 2^-8) -- here rmax = the row's max |v|,
    bw = 1, bb = 0, a valid bound since each output is a convex combination of V rows -- then
    split2h's x1 = f16(o s), x2 = f16(o s - x1), bit for bit, in both layouts (role 2 [x1 x2], the
    tower's default, and role 0 [x1 x1 x2])."""
    import torch
    from miclip import _native
    N_ = _lib()
    rng = np.random.default_rng(B * 31 + S + W + causal)
    qkv = (rng.standard_normal((B * S, 3 * W)) * 2).astype(np.float32)
    qkv *= (10.0 ** rng.uniform(-2, 2, size=(B, 1, 1))).astype(np.float32).repeat(S, axis=1).reshape(B * S, 1)
    rmax = np.abs(qkv[:, 2 * W:]).max(axis=1).astype(np.float32)
    d = torch.from_numpy(qkv).to(gpu)
    rm = torch.from_numpy(rmax).to(gpu)
    o = torch.full((B * S, W), float("nan"), device=gpu)
    N_.check(N_.lib().mi_op_attention_f32(d.data_ptr(), o.data_ptr(), B, S, W, causal, _stream()), "attn f32")
    torch.cuda.synchronize()
    o = o.cpu().numpy()
    # the sequence's scale: split_exp of the f32 bound
    bound = (rmax.reshape(B, S).max(axis=1).astype(np.float32) * np.float32(1.0)) * np.float32(1.0 + 1.0 / 256.0)
    _, ex = np.frexp(bound.astype(np.float32))
    e = np.clip(14 - ex, -126, 126)
    e[~(bound > 0)] = 0
    s = np.ldexp(np.float32(1.0), e).astype(np.float32).repeat(S)[:, None]
    x = (o * s).astype(np.float32)
    x1 = x.astype(np.float16)
    x2 = (x - x1.astype(np.float32)).astype(np.float16)
    for role, blocks in ((2, (x1, x2)), (0, (x1, x1, x2))):
        a3 = torch.zeros((B * S, len(blocks) * W), dtype=torch.float16, device=gpu)
        sc = torch.full((B * S,), float("nan"), device=gpu)
        _native.check(N_.lib().mi_op_attention_f32_split(d.data_ptr(), rm.data_ptr(), 1.0, 0.0, a3.data_ptr(), role,
                                                         sc.data_ptr(), B, S, W, causal, _stream()), "attn f32 split")
        torch.cuda.synchronize()
        assert np.array_equal(sc.cpu().numpy(), (1.0 / s[:, 0]).astype(np.float32))
        want = np.concatenate(blocks, axis=1)
        got = a3.cpu().numpy()
        assert np.array_equal(got.view(np.uint16), want.view(np.uint16)), np.argwhere(got.view(np.uint16) != want.view(np.uint16))[:5]


@pytest.mark.parametrize("M,N,K", [(2464, 1536, 512), (2464, 512, 512), (2464, 512, 2048), (400, 2304, 768),
                                   (65, 128, 64), (1000, 768, 3072)])
def test_gemm_small_tiles_bit_identical(gpu, monkeypatch, M, N, K):
    """The smallest bf16 GEMMs (fewer 128 x 128 tiles than CUs: the text tower at 32 queries, small
    image batches) on 64 x 64 tiles (round 6) against 128 x 128 tiles (A/B MICLIP_SMALL64=0) and the
    256 x 256 path (MICLIP_SMALLM=0): the same k order per output, bit for bit; ragged M."""
    import torch
    from miclip import _native
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N + K)
    A = (torch.randn(M, K, generator=g) * 0.5).bfloat16().to(gpu)
    W = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16().to(gpu)
    bias = torch.randn(N, generator=g).float().to(gpu)
    outs = []
    for lib, env in ((_native.lib(), {}), (_native.lib_ab(), {"MICLIP_SMALL64": "0"}),
                     (_native.lib_ab(), {"MICLIP_SMALLM": "0"})):
        for k in ("MICLIP_SMALL64", "MICLIP_SMALLM"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=gpu)
        _native.check(lib.mi_op_gemm(A.data_ptr(), W.data_ptr(), bias.data_ptr(), out.data_ptr(), M, N, K, 0,
                                     _stream()), "gemm")
        torch.cuda.synchronize()
        outs.append(out)
    ref = A.float() @ W.float().t() + bias
    assert (outs[0].float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())
    for o in outs[1:]:
        assert torch.equal(outs[0].view(torch.int16), o.view(torch.int16))
