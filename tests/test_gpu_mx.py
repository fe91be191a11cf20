"""MX-fp8 operators (configs[4] "fp8 MFMA weights"): the bf16 -> MX quantiser
and the block-scaled MFMA GEMM against oracle/mx_ref.py (float64)."""
import numpy as np
import pytest

from oracle import mx_ref

pytestmark = pytest.mark.gpu


def _lib():
    from miclip import _native
    return _native


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


def _quant_gpu(x_bf16):
    import torch
    N_ = _lib()
    rows, K = x_bf16.shape
    q = torch.empty(rows, K, dtype=torch.uint8, device=x_bf16.device)
    s = torch.zeros((K // 128) * (rows + (rows & 1)) * 2, dtype=torch.uint8, device=x_bf16.device)
    N_.check(N_.lib().mi_op_quantize_mx(x_bf16.data_ptr(), q.data_ptr(), s.data_ptr(), rows, K, _stream()), "quant")
    return q, s


def test_quantize_matches_oracle(gpu):
    import torch
    g = torch.Generator(device="cpu").manual_seed(3)
    x = (torch.randn(97, 256, generator=g) * torch.logspace(-3, 3, 256)).bfloat16()
    x[5, :64] = 0                                 # all-zero block -> scale 2^-127, codes 0
    x[7, 40] = 1e4                                # one large outlier in a block
    q, s = _quant_gpu(x.to(gpu))
    torch.cuda.synchronize()
    rq, rs = mx_ref.quantize(x.float().numpy())
    assert np.array_equal(mx_ref.from_stage_major(s.cpu().numpy(), 97, 256), rs)
    got = mx_ref.E4M3[q.cpu().numpy()]
    ref = mx_ref.E4M3[rq]
    assert np.array_equal(got, ref)               # same values (+0 / -0 codes may differ)


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (301, 512, 1024), (1000, 768, 256), (4096, 1024, 4096)])
@pytest.mark.parametrize("epi", [3, 0, 1])
def test_gemm_mx_matches_oracle(gpu, M, N, K, epi):
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    a = (torch.randn(M, K, generator=g) * 2).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, generator=g)
    qa, sa = _quant_gpu(a.to(gpu))
    qw, sw = _quant_gpu(w.to(gpu))
    out = torch.empty(M, N, dtype=torch.float32 if epi == 3 else torch.bfloat16, device=gpu)
    bd = bias.to(gpu)
    N_.check(N_.lib().mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bd.data_ptr(),
                                    out.data_ptr(), M, N, K, epi, _stream()), "gemm_mx")
    torch.cuda.synchronize()
    sa_, sw_ = (mx_ref.from_stage_major(x.cpu().numpy(), r, K) for x, r in ((sa, M), (sw, N)))
    ref = mx_ref.gemm(qa.cpu().numpy(), sa_, qw.cpu().numpy(), sw_) + bias.double().numpy()
    if epi == 1:
        ref = ref / (1 + np.exp(-1.702 * ref))
    got = out.double().cpu().numpy()
    scale = np.abs(ref).max()
    tol = (1e-4 if epi == 3 else 1e-2) * scale
    assert np.abs(got - ref).max() < tol, (np.abs(got - ref).max(), tol)


def test_gemm_mx_asymmetric_identity(gpu):
    """A = I (exact in e4m3) with an asymmetric W catches a transposed C write."""
    import torch
    N_ = _lib()
    M = N = 256
    K = 256
    a = torch.eye(M, K).bfloat16()
    w = ((torch.arange(N * K).reshape(N, K) % 7) - 3).float().bfloat16()
    qa, sa = _quant_gpu(a.to(gpu))
    qw, sw = _quant_gpu(w.to(gpu))
    out = torch.empty(M, N, device=gpu)
    N_.check(N_.lib().mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), None,
                                    out.data_ptr(), M, N, K, 3, _stream()), "gemm_mx")
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), w.float().t().contiguous())


@pytest.mark.parametrize("M,N,K", [(300, 256, 512), (517, 768, 1024)])
def test_gemm_mx_block_scales(gpu, M, N, K):
    """Magnitudes spanning 2^-12..2^12 across rows AND 64-k blocks: every
    (row, k-block) scale byte must reach the MFMA lane that owns it."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + K)
    rs = 2.0 ** torch.randint(-6, 7, (M, 1), generator=g).float()
    ks = 2.0 ** torch.randint(-6, 7, (1, K // 64), generator=g).float().repeat_interleave(64, 1)
    a = (torch.randn(M, K, generator=g) * rs * ks).bfloat16()
    ws = 2.0 ** torch.randint(-6, 7, (N, K // 64), generator=g).float().repeat_interleave(64, 1)
    w = (torch.randn(N, K, generator=g) * ws * K ** -0.5).bfloat16()
    qa, sa = _quant_gpu(a.to(gpu))
    qw, sw = _quant_gpu(w.to(gpu))
    out = torch.empty(M, N, device=gpu)
    N_.check(N_.lib().mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), None,
                                    out.data_ptr(), M, N, K, 3, _stream()), "gemm_mx")
    torch.cuda.synchronize()
    sa_, sw_ = (mx_ref.from_stage_major(x.cpu().numpy(), r, K) for x, r in ((sa, M), (sw, N)))
    ref = mx_ref.gemm(qa.cpu().numpy(), sa_, qw.cpu().numpy(), sw_)
    got = out.double().cpu().numpy()
    # per-row tolerance: rows differ by 2^12 in scale
    err = np.abs(got - ref).max(1) / np.maximum(np.abs(ref).max(1), 1e-30)
    assert err.max() < 1e-4, err.max()


@pytest.mark.parametrize("M,N,K", [(256, 256, 512), (1000, 1024, 1024), (4099, 768, 4096), (40000, 1024, 1024)])
@pytest.mark.parametrize("epi", [0, 1, 4])
def test_gemm_mx8q_matches_16x16x128_kernel(gpu, M, N, K, epi):
    """The 8-phase persistent MX kernel (gemm_mx8q.hip, variant 8) runs the same
    v_mfma_scale_f32_16x16x128_f8f6f4 in the same k order as the
    double-buffered kernel (variant 1): bit-identical bf16 / GELU / MX-fp8
    outputs (e4m3 bytes and their scales), with row tails past M, several
    tiles per workgroup (40000 rows) and K up to 4096."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + K + epi)
    a = (torch.randn(M, K, generator=g) * 2).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, generator=g).to(gpu)
    qa, sa = _quant_gpu(a.to(gpu))
    qw, sw = _quant_gpu(w.to(gpu))
    outs = []
    for variant in (8, 1):
        if epi == 4:
            mp = M + (M & 1)
            out = torch.zeros((M * N + 255) // 256 * 256 + (N // 128) * mp * 2, dtype=torch.uint8, device=gpu)
        else:
            out = torch.zeros(M, N, dtype=torch.bfloat16, device=gpu)
        AB = N_.lib_ab()          # kernel overrides: the A/B build (scripts/ab)
        rc = AB.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                              out.data_ptr(), M, N, K, epi | (variant << 8), _stream())
        if rc:
            raise N_.MiClipError(f"gemm_mx v{variant}: {AB.mi_last_error()}")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.uint8), outs[1].view(torch.uint8))
    if epi == 4:   # and the fp8 output decodes to the oracle's GELU within e4m3 rounding
        q = outs[0][:M * N].cpu().numpy().reshape(M, N)
        s = outs[0][(M * N + 255) // 256 * 256:].cpu().numpy()
        got = mx_ref.E4M3[q] * 2.0 ** (mx_ref.from_stage_major(s, M, N).repeat(64, 1).astype(np.float64) - 127)
        sa_, sw_ = (mx_ref.from_stage_major(x.cpu().numpy(), r, K) for x, r in ((sa, M), (sw, N)))
        ref = mx_ref.gemm(qa.cpu().numpy(), sa_, qw.cpu().numpy(), sw_) + bias.double().cpu().numpy()
        ref = ref / (1 + np.exp(-1.702 * ref))
        # e4m3 keeps 3 mantissa bits (half an ulp = 2^-4 of the value); block values scaled into
        # [448, 512) saturate at 448 (up to 1/8); plus the block's subnormal floor
        assert np.all(np.abs(got - ref) <= 0.125 * np.abs(ref) + 0.01 * np.abs(ref).max())


@pytest.mark.parametrize("M,N,K", [(256, 256, 512), (1001, 1024, 1024), (40000, 4096, 1024)])
def test_gemm_mx_default_fp8_output_rows(gpu, M, N, K):
    """The product MX kernel's (ping-pong 32x32x64) QuickGELU -> MX-fp8 epilogue, whose 16-byte
    row stores take each lane's four e4m3 dwords through a half swap: every e4m3 byte and scale
    lands where the consumer reads it -- decoded, the output matches the oracle's GELU within e4m3
    rounding (row tails past M, odd M, 40000 rows)."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + K + 7)
    a = (torch.randn(M, K, generator=g) * 2).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, generator=g).to(gpu)
    qa, sa = _quant_gpu(a.to(gpu))
    qw, sw = _quant_gpu(w.to(gpu))
    mp = M + (M & 1)
    out = torch.zeros((M * N + 255) // 256 * 256 + (N // 128) * mp * 2, dtype=torch.uint8, device=gpu)
    N_.check(N_.lib().mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                    out.data_ptr(), M, N, K, 4, _stream()), "gemm_mx")
    torch.cuda.synchronize()
    rows = np.arange(M) if M <= 2000 else np.r_[0:300, M // 2:M // 2 + 300, M - 300:M]
    q = out[:M * N].cpu().numpy().reshape(M, N)[rows]
    s = out[(M * N + 255) // 256 * 256:].cpu().numpy()
    got = mx_ref.E4M3[q] * 2.0 ** (mx_ref.from_stage_major(s, M, N)[rows].repeat(64, 1).astype(np.float64) - 127)
    sa_ = mx_ref.from_stage_major(sa.cpu().numpy(), M, K)[rows]
    sw_ = mx_ref.from_stage_major(sw.cpu().numpy(), N, K)
    ref = mx_ref.gemm(qa.cpu().numpy()[rows], sa_, qw.cpu().numpy(), sw_) + bias.double().cpu().numpy()
    ref = ref / (1 + np.exp(-1.702 * ref))
    assert np.all(np.abs(got - ref) <= 0.125 * np.abs(ref) + 0.01 * np.abs(ref).max())


@pytest.mark.parametrize("M,N,K", [(40000, 1024, 1024), (70001, 4096, 1024), (100003, 1024, 4096)])
@pytest.mark.parametrize("epi", [0, 1, 3, 4])
def test_gemm_mx_persistent_bit_identical(gpu, monkeypatch, M, N, K, epi):
    """The persistent MX ping-pong (gemm_mxppp_kernel: one workgroup per CU, the next tile's first
    stages and bias streamed in under this tile's last stages, counted waits across the tile
    boundary; and its lean stage loop, MICLIP_MX_PERSIST=4) against
    one workgroup per tile (gemm_mxpp_kernel, MICLIP_MX_PERSIST=0, A/B build):
    the same MFMAs in the same k order and the same epilogue arithmetic, so bf16 / GELU / f32 /
    MX-fp8 outputs (e4m3 bytes and their scales) are byte-identical -- several tiles per CU, odd M
    and a partial last m-tile (its stores drain with vmcnt(0)), K = 1024 and 4096."""
    import torch
    N_ = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    a = (torch.randn(M, K, generator=g) * 2).bfloat16()
    w = (torch.randn(N, K, generator=g) * K ** -0.5).bfloat16()
    bias = torch.randn(N, generator=g).to(gpu)
    qa, sa = _quant_gpu(a.to(gpu))
    qw, sw = _quant_gpu(w.to(gpu))
    outs = []
    for lib, persist in ((N_.lib(), None), (N_.lib_ab(), "1"), (N_.lib_ab(), "0"), (N_.lib_ab(), "4")):
        if persist is not None:
            monkeypatch.setenv("MICLIP_MX_PERSIST", persist)
        if epi == 4:
            mp = M + (M & 1)
            out = torch.zeros((M * N + 255) // 256 * 256 + (N // 128) * mp * 2, dtype=torch.uint8, device=gpu)
        else:
            out = torch.zeros(M, N, dtype=torch.float32 if epi == 3 else torch.bfloat16, device=gpu)
        rc = lib.mi_op_gemm_mx(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                               out.data_ptr(), M, N, K, epi, _stream())
        if rc:
            raise N_.MiClipError(f"gemm_mx: {lib.mi_last_error()}")
        outs.append(out)
    torch.cuda.synchronize()
    assert torch.equal(outs[0].view(torch.uint8), outs[1].view(torch.uint8))   # product = A/B persistent
    assert torch.equal(outs[1].view(torch.uint8), outs[2].view(torch.uint8))   # persistent = per tile
    assert torch.equal(outs[1].view(torch.uint8), outs[3].view(torch.uint8))   # the lean stage loop (A/B)
