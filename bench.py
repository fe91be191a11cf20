"""Benchmark: frames/sec embedded + ranked (BASELINE.json metric) on MI355X.

One step = the reference's hot path over one batch of synthetic input, all on
the GPU, inputs resident in HBM before the timed region:
  encode_image of the rank's frame shard (ViT-B/32, bf16 MFMA)   -> corpus [N,512] f32 in HBM
  encode_text of Q synthetic token rows (+L2 in the kernel)       -> queries [Q,512]
  fused normalise + cosine + top-k over the corpus                -> [Q,k]
  (N>1) RCCL all-gather of the per-shard top-k + merge kernel
Workload at N=1 is BASELINE.json configs[1] (ViT-B/32 bf16, 10k frames x 32
queries, top-10); with --gpus N each rank embeds its own 10k-frame shard
(weak scaling), or with --global-frames G one G-frame corpus is split into N
contiguous shards (strong scaling; configs[3] = --global-frames 1000000 on 8).

Launch: python bench.py [--gpus N --steps K --warmup W].  With N > 1 and no
WORLD_SIZE in the environment this process starts torch.distributed.run with
N workers (one per GPU, RCCL backend "nccl") as a child, before touching the
GPU; under torch.distributed.run directly it is one of the N ranks.  Rank 0
prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "event-retrival-in-video-learning-transferable-visual-model-from-supervised-natural-language_amd")
for _p in (PKG, ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md (spec)
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA (spec, no sparsity)
FP8_PEAK_TFLOPS = 5000.0       # dense fp8 / MX-fp8 MFMA (spec, no sparsity)
F32_MFMA_PEAK_TFLOPS = 157.3


def _progress(msg):
    """A progress line on stderr (stdout carries only the JSON result)."""
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="ViT-B/32")
    ap.add_argument("--frames", type=int, default=10_000, help="frames per GPU (weak scaling: each rank's shard)")
    ap.add_argument("--global-frames", type=int, default=None,
                    help="strong scaling: one corpus of this many frames split into contiguous shards "
                         "(configs[3]: 1000000 over 8 GPUs = 125k per rank)")
    ap.add_argument("--queries", type=int, default=32)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--image-chunk", type=int, default=None)
    ap.add_argument("--weights", choices=["bf16", "fp8", "fp32"], default="bf16",
                    help="fp8: vision GEMMs on the MX-fp8 block-scaled MFMA (BASELINE configs[4]); "
                         "fp32: the parity mode (model.float(): f32 activations and residual stream, every "
                         "tower GEMM at f32-GEMM accuracy through split operands on the 16-bit MFMA; the "
                         "exact-f32 MFMA GEMM is the A/B alternative, MICLIP_F32_SPLIT=0)")
    ap.add_argument("--no-parity-mode", action="store_true",
                    help="skip the fp32-tower (R@K parity mode) measurement beside the bf16 line")
    ap.add_argument("--parity-steps", type=int, default=3)
    ap.add_argument("--cpu-frames", type=int, default=256,
                    help="CPU baseline sample: frames encoded at batch 64 (secondary figure)")
    ap.add_argument("--cpu-frames-b1", type=int, default=64,
                    help="CPU baseline sample: frames encoded one per call (Backend/embedding.py; configs[0]'s 64)")
    ap.add_argument("--no-rank-roofline", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher rehearsal on CPU/gloo: rendezvous + all-gather, no GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="the N > 1 process group: nccl (RCCL over xGMI, the measured path) or gloo (a rehearsal "
                         "of the multi-rank step on fewer GPUs than ranks: rank r uses GPU r %% device_count)")
    return ap.parse_args()


def lnfold_active(model, cfg):
    """The bf16 vision tower runs LayerNorm folded into in_proj / c_fc when its width is a
    multiple of 256 and at most 1024 (api.cpp lnfold / mi_clip_encode_image `fold`; the product
    library has no switch)."""
    return getattr(model, "weights", "bf16") == "bf16" and cfg.vision_width % 256 == 0 and cfg.vision_width <= 1024


def step_work(cfg, weights, chunk, lnfold):
    """The MFMA work one step executes, per frame and per query, split by the engine it runs on
    (api.cpp: at >= 256 frames per chunk the last block's out_proj / c_fc / c_proj run on the CLS
    rows only -- in the LN-folded bf16, the MX-fp8 and the fp32 towers; the bf16 and fp32 towers
    also compute the last in_proj's Q for the CLS rows only and the last attention for the CLS
    query's tile: 16 rows in the S <= 64 flash kernel, 32 in the f32 MFMA kernel (S <= 128))."""
    S = cfg.vision_tokens
    cls_last = chunk >= 256 and ((weights == "bf16" and lnfold) or weights == "fp32"
                                 or (weights == "fp8" and cfg.vision_width % 128 == 0))
    q_cls = cls_last and weights in ("bf16", "fp32")
    rows = None
    if cls_last and weights == "bf16" and S <= 64:
        rows = 16
    elif cls_last and weights == "fp32" and S <= 128:
        rows = 32
    return {"cls_last": cls_last, "image": cfg.image_flops_executed(cls_last, q_cls, rows),
            "image_attn": cfg.image_attention_flops(rows), "text": cfg.text_flops(),
            "text_attn": cfg.text_attention_flops()}


def mfma_time_at_peak(w, weights, frames, queries, dim):
    """Seconds the step's executed MFMA work needs at each engine's dense peak: bf16 towers on the
    bf16/f16 MFMA (2.5 PF); MX-fp8 runs' vision GEMMs on the fp8 MFMA (5 PF), their attention and
    text tower bf16; fp32 runs' GEMMs as split-f16 (3x the products on the f16 MFMA) and their
    attention on the exact-f32 MFMA; the rank pass's 2 N Q D on the exact-f32 MFMA.  Divided by the
    step time this is the end-to-end MFMA fraction (<= 1 by construction)."""
    img_gemm, img_attn = frames * (w["image"] - w["image_attn"]), frames * w["image_attn"]
    txt_gemm, txt_attn = queries * (w["text"] - w["text_attn"]), queries * w["text_attn"]
    rank = 2.0 * frames * queries * dim
    bf, f8, f32 = BF16_PEAK_TFLOPS * 1e12, FP8_PEAK_TFLOPS * 1e12, F32_MFMA_PEAK_TFLOPS * 1e12
    if weights == "fp32":
        return 3 * (img_gemm + txt_gemm) / bf + (img_attn + txt_attn + rank) / f32
    if weights == "fp8":
        return img_gemm / f8 + (img_attn + txt_gemm + txt_attn) / bf + rank / f32
    return (img_gemm + img_attn + txt_gemm + txt_attn) / bf + rank / f32


def kernel_timing(model, cfg, chunk, reps=20):
    """Average duration of each encoder kernel at the bench's chunk shape, timed
    with HIP events on the stream the kernels are launched on."""
    import torch
    from miclip import _native as N

    L = N.lib()
    dev = model.device
    W, S = cfg.vision_width, cfg.vision_tokens
    M = chunk * S
    g = torch.Generator(device=dev).manual_seed(0)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    A = (torch.randn(M, 4 * W, device=dev, generator=g) * 0.5).bfloat16()
    Wt = (torch.randn(4 * W, 4 * W, device=dev, generator=g) * 0.02).bfloat16()
    bias = torch.zeros(4 * W, device=dev)
    outb = torch.empty(M, 4 * W, dtype=torch.bfloat16, device=dev)
    outf = torch.zeros(M, W, device=dev)
    res = {}

    def timed(name, fn, flops=None, nbytes=None):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) * 1e3 / reps
        d = {"us": round(us, 2)}
        if flops:
            d["tflops"] = round(flops / us / 1e6, 1)
        if nbytes:
            d["gbs"] = round(nbytes / us / 1e3, 1)
        res[name] = d

    gemms = [("gemm_qkv", 3 * W, W, 0, outb), ("gemm_out", W, W, 0, outb), ("gemm_fc", 4 * W, W, 1, outb),
             ("gemm_proj", W, 4 * W, 0, outb)]
    if getattr(model, "weights", "bf16") == "fp32":
        # the parity mode's GEMMs since round 5: split-f16 operands (mi_op_split2h: a power-of-two
        # row scale, 2 fp16 terms per f32 value; the weights' copies built at load) and one f16 GEMM
        # over K' = 3K with the row / column scales in its f32 epilogue (api.cpp run_tower_f32);
        # "tflops" counts the f32 GEMM's useful flops, "f16_tflops" the MFMA work executed (3x);
        # "<gemm>_split" times a split pass over that GEMM's input (in the tower none runs: ln_1 / ln_2
        # write their splits directly, c_fc's epilogue writes c_proj's and, since round 6, attention
        # writes out_proj's), "attention" the S <= 64 attention on split-f16 operands with f32
        # output, "attention_split" the same writing out_proj's split operand (the tower's launch)
        del A, outb
        Af = torch.randn(M, 4 * W, device=dev, generator=g) * 0.5
        Wf = torch.randn(4 * W, 4 * W, device=dev, generator=g) * 0.02
        outF = torch.zeros(M, 4 * W, device=dev)
        A3 = torch.empty(M, 3 * 4 * W, dtype=torch.int16, device=dev)
        sa, sw = torch.empty(M, device=dev), torch.empty(4 * W, device=dev)
        for name, Nn, K, epi, _ in gemms:
            W3 = torch.empty(Nn, 3 * K, dtype=torch.int16, device=dev)
            N.check(L.mi_op_split2h(Wf.data_ptr(), 4 * W, Nn, K, 1, 0, W3.data_ptr(), sw.data_ptr(), sp), "split2h W")
            gelu = 1 if name == "gemm_proj" else 0   # c_proj's input: QuickGELU applied in the split
            timed(name + "_split", lambda K=K, gelu=gelu: N.check(
                L.mi_op_split2h(Af.data_ptr(), 4 * W, M, K, 0, gelu, A3.data_ptr(), sa.data_ptr(), sp), "split2h A"),
                  nbytes=M * K * 4 + M * 3 * K * 2)
            ep = 2 if name in ("gemm_out", "gemm_proj") else 3   # += into the residual / f32 store
            timed(name, lambda Nn=Nn, K=K, ep=ep, W3=W3: N.check(
                L.mi_op_gemm_split2h(A3.data_ptr(), W3.data_ptr(), sa.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                     outF.data_ptr(), M, Nn, 3 * K, ep, sp), "gemm split-f16"), flops=2.0 * M * Nn * K)
            res[name]["f16_tflops"] = round(res[name]["tflops"] * 3, 1)
            del W3
        del Wf, A3
        qkv32 = Af[:, :3 * W].contiguous()
        del Af
        att32 = outF[:, :W].contiguous()
        timed("attention", lambda: N.check(L.mi_op_attention_f32(qkv32.data_ptr(), att32.data_ptr(), chunk, S, W, 0, sp),
                                           "attn f32"), flops=4.0 * chunk * S * S * W, nbytes=M * 4 * W * 4)
        if S <= 64:
            rmax = qkv32[:, 2 * W:].abs().amax(dim=1).contiguous()   # a valid bound: bw = 1, bb = 0
            a3o = torch.empty(M, 2 * W, dtype=torch.int16, device=dev)
            rso = torch.empty(M, device=dev)
            timed("attention_split", lambda: N.check(L.mi_op_attention_f32_split(
                qkv32.data_ptr(), rmax.data_ptr(), 1.0, 0.0, a3o.data_ptr(), 2, rso.data_ptr(), chunk, S, W, 0, sp),
                "attn f32 split"), flops=4.0 * chunk * S * S * W, nbytes=M * 4 * W * 4)
            del rmax, a3o, rso
        del outF, qkv32, att32
        return res
    if getattr(model, "weights", "bf16") == "fp8":
        # MX-fp8 operands: e4m3 codes + stage-major e8m0 scales (mi_op_quantize_mx)
        def mx(t):
            rows, K = t.shape
            q = torch.empty(rows, K, dtype=torch.uint8, device=dev)
            sc = torch.empty((K // 128) * ((rows + 1) & ~1) * 2, dtype=torch.uint8, device=dev)
            N.check(L.mi_op_quantize_mx(t.data_ptr(), q.data_ptr(), sc.data_ptr(), rows, K, sp), "quantize_mx")
            return q, sc
        for name, Nn, K, epi, out in gemms:
            Aq, As = mx(A[:, :K].contiguous())
            Wq, Ws = mx(Wt[:Nn, :K].contiguous())
            if name == "gemm_fc":   # the tower's c_fc: QuickGELU -> MX-fp8 codes + scales (EPI_GELU_MX)
                epi = 4
                out = torch.empty((M * Nn + 255) // 256 * 256 + (Nn // 128) * ((M + 1) & ~1) * 2,
                                  dtype=torch.uint8, device=dev)
            timed(name, lambda Nn=Nn, K=K, epi=epi, out=out, Aq=Aq, As=As, Wq=Wq, Ws=Ws: N.check(
                L.mi_op_gemm_mx(Aq.data_ptr(), As.data_ptr(), Wq.data_ptr(), Ws.data_ptr(), bias.data_ptr(),
                                out.data_ptr(), M, Nn, K, epi, sp), "gemm_mx"), flops=2.0 * M * Nn * K)
    elif lnfold_active(model, cfg):
        # the product bf16 tower (W % 256 == 0): in_proj / c_fc are the LayerNorm-folded GEMMs
        # (gemm_8q_kernel<EPI_LN_*>, fp16 operands of the half-slot residual stream, lda = 2W),
        # out_proj / c_proj add into that stream in their epilogues and store row partial
        # statistics, then residual_finalize (mi_op_gemm_residual; api.cpp run_tower_fold)
        x16 = (torch.rand(M, 2 * W, device=dev, generator=g) * 2 - 1).half()
        x16r = x16.clone()            # the fused GEMMs' in-place stream (keeps x16's values bounded)
        Wh = (torch.randn(4 * W, W, device=dev, generator=g) * 0.02).half()
        colsum = Wh.float().sum(1)
        rs = torch.rand(M + 256, 2, device=dev, generator=g) + 0.5
        rs2 = torch.empty(M, 2, device=dev)
        ps = torch.empty(M, W // 64, 2, device=dev)
        for name, Nn, K, epi, out in gemms:
            if name in ("gemm_qkv", "gemm_fc"):
                timed(name, lambda Nn=Nn, epi=epi, out=out: N.check(
                    L.mi_op_gemm_ln(x16.data_ptr(), 2 * W, rs.data_ptr(), Wh.data_ptr(), colsum.data_ptr(),
                                    bias.data_ptr(), out.data_ptr(), M, Nn, W, epi, sp), "gemm_ln"),
                      flops=2.0 * M * Nn * W)
            else:   # the residual add fused: x16 read + written, partials, then residual_finalize
                timed(name, lambda K=K: N.check(
                    L.mi_op_gemm_residual(x16r.data_ptr(), 2 * W, A.data_ptr(), K, Wt.data_ptr(), bias.data_ptr(),
                                          ps.data_ptr(), rs2.data_ptr(), M, W, K, sp), "gemm_residual"),
                      flops=2.0 * M * W * K)
        del x16, x16r, Wh, colsum, rs, rs2, ps
    else:
        for name, Nn, K, epi, out in gemms:
            timed(name, lambda Nn=Nn, K=K, epi=epi, out=out: N.check(
                L.mi_op_gemm(A.data_ptr(), Wt.data_ptr(), bias.data_ptr(), out.data_ptr(), M, Nn, K, epi, sp),
                "gemm"), flops=2.0 * M * Nn * K)
    qkv = torch.randn(M, 3 * W, device=dev, generator=g).bfloat16()
    att = torch.empty(M, W, dtype=torch.bfloat16, device=dev)
    timed("attention", lambda: N.check(L.mi_op_attention(qkv.data_ptr(), att.data_ptr(), chunk, S, W, 0, sp),
                                       "attn"), flops=4.0 * chunk * S * S * W,
          nbytes=M * 4 * W * 2)
    x = torch.randn(M, W, device=dev, generator=g)
    gam = torch.ones(W, device=dev)
    timed("layernorm", lambda: N.check(L.mi_op_layernorm(x.data_ptr(), gam.data_ptr(), gam.data_ptr(),
                                                         att.data_ptr(), M, W, sp), "ln"), nbytes=M * W * 6)
    return res


def pmc_traffic(shape, fp8=False, epilogue=None):
    """HBM bytes per launch of the GEMM at `shape` [M, N, K] from the newest
    committed PMC summary (profiles/*_gemm_traffic.json, made by
    scripts/gpu_traffic.sh + scripts/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE,
    the gfx950 corrections of MI355X_MICROARCH.md "HBM"; MX-fp8:
    profiles/*_fp8_gemm_traffic.json from scripts/gpu_fp8_traffic.sh), with the
    MFMA-busy fraction of the same summary's GRBM/SQ pass.  `epilogue` (gemm_micro's
    code, 7 = the LayerNorm-folded c_fc) selects the kernel measured.  None if absent."""
    import glob
    pat = "*_fp8_gemm_traffic.json" if fp8 else "*_gemm_traffic.json"
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", pat)), reverse=True):
        if not fp8 and f.endswith("_fp8_gemm_traffic.json"):
            continue
        try:
            d = json.load(open(f))
            for v in ([d] if fp8 else d.values()):
                if list(v["shape"]) == list(shape) and (epilogue is None or v.get("epilogue") == epilogue):
                    return v["traffic_bytes"], os.path.relpath(f, ROOT), v.get("mfma_busy")
        except (OSError, ValueError, KeyError, AttributeError):
            continue
    return None, None, None


def preprocess_timing(dev, n_px, B=256, H=720, W=1280, reps=10):
    """GPU frame preprocessing (mi_preprocess_frames)
    of B decoded 1280x720 uint8 frames -> [B,3,n,n] bf16, HIP events on the
    launch stream.  Not part of the timed step (the metric starts from
    preprocessed 224^2 tensors, as the reference's synthetic tests do)."""
    import torch
    from miclip.preprocess import preprocess_frames
    g = torch.Generator(device=dev).manual_seed(5)
    frames = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    preprocess_frames(frames, n_px, out_dtype=torch.bfloat16)
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        preprocess_frames(frames, n_px, out_dtype=torch.bfloat16)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    us = e0.elapsed_time(e1) * 1e3 / reps
    return {"us": round(us, 2), "frames_per_s": round(B / us * 1e6, 1),
            "gbs": round(B * H * W * 3 / us / 1e3, 1), "shape": [B, H, W, 3]}


def jpeg_ingest_timing(dev, n_px, B=8192, threads=16, pil_frames=1024):
    """Frame ingest from JPEG bytes in host memory to preprocessed [B,3,n,n]
    bf16 tensors: the reference's 16 real 1280x720
    frames (tests/golden/ref_frames) repeated to B.  GPU path: header parse +
    table build on the host, mi_jpeg_decode_transform on the device (entropy
    decode + IDCT, then colour conversion, both resample passes and Normalize
    fused; bit-identical to Pillow + torchvision, tests/test_gpu_jpeg.py), and
    the pre-r04 two-step path (decode to RGB + mi_preprocess_frames); host path: Pillow
    decode on `threads` host threads, as the reference decodes, + the same GPU
    preprocessing, timed on the first `pil_frames` frames.  The GPU entropy
    decode runs one lane per 1-KB chunk of a frame's scan (jpeg.hip, chunked
    speculative decode).  Wall-clock, synchronised; not part of the timed step."""
    import glob
    import io
    import time
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    import torch
    from PIL import Image
    from miclip import jpeg
    from miclip.preprocess import preprocess_frames
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "ref_frames", "*.jpg")))
    if not files:
        return None
    raw = [open(f, "rb").read() for f in files]
    bufs = [raw[i % len(raw)] for i in range(B)]

    def gpu():   # fused decode + colour + resample + normalise (mi_jpeg_decode_transform), per geometry group
        return [x for _, x in jpeg.decode_groups(bufs, dev, transform=(n_px, False, torch.bfloat16))]

    def gpu_two_step():   # decode to RGB, then mi_preprocess_frames (the pre-r04 path)
        return [preprocess_frames(rgb, n_px, out_dtype=torch.bfloat16) for _, rgb in jpeg.decode_groups(bufs, dev)]

    def pil_one(b):
        with Image.open(io.BytesIO(b)) as im:
            return np.asarray(im.convert("RGB"), dtype=np.uint8)

    def host():
        with ThreadPoolExecutor(threads) as ex:
            arrs = list(ex.map(pil_one, bufs[:pil_frames]))
        return preprocess_frames(torch.from_numpy(np.stack(arrs)).to(dev), n_px, out_dtype=torch.bfloat16)

    res = {"frames": B, "pil_frames": pil_frames,
           "source": "tests/golden/ref_frames (16 reference frames, 1280x720 4:2:0)", "host_threads": threads}
    for name, fn, n in (("gpu_decode", gpu, B), ("gpu_decode_two_step", gpu_two_step, B),
                        ("pil_decode", host, pil_frames)):
        out = fn()
        torch.cuda.synchronize(dev)
        best = 1e9
        for _ in range(2):
            out = None
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize(dev)
            best = min(best, time.perf_counter() - t0)
        res[name + "_frames_per_s"] = round(n / best, 1)
        del out
    torch.cuda.empty_cache()
    return res


def rank_timing(corpus, txt, k, reps=50):
    import torch
    from miclip import retrieval
    retrieval.rank_topk(corpus, txt, k)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        retrieval.rank_topk(corpus, txt, k)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    nbytes = corpus.numel() * corpus.element_size()
    return {"us": round(us, 2), "gbs": round(nbytes / us / 1e3, 1),
            "tflops_f32": round(2.0 * corpus.shape[0] * txt.shape[0] * corpus.shape[1] / us / 1e6, 2)}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _usable_cores():
    """Host cores this process may run on: BASELINE.md's plan is
    torch.set_num_threads(os.cpu_count()), but on the GPU box os.cpu_count()
    reports the whole host (256) while the process's share is a cgroup CPU quota
    (16); threads beyond the share only contend.  min(affinity, quota)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_baseline(cfg, n_frames_metric, Q, k, b1_frames, b64_frames, check=None):
    """The reference CPU path timed on this box's host cores (BASELINE.md
    CPU-baseline plan): the torch-CPU fp32 restatement of openai/CLIP
    (oracle/clip_torch.py) run as Backend/embedding.py does on a CPU host,
    one image per call (embedding.py:39-52, `b1_frames` frames = configs[0]'s
    64) and, secondarily, at batch 64 (`b64_frames` frames); one encode_text;
    np.dot + np.argsort(s)[::-1][:k] over an N-row corpus
    (embedding_service.py:314-320).  Extrapolated to the metric's workload
    (N frames embedded + Q queries ranked).  The numpy restatement
    (oracle/clip_ref.py) at batch 64 is reported beside it."""
    import numpy as np
    import torch
    from miclip import weights
    from oracle import clip_ref, clip_torch, rank_ref
    # threads: $OMP_NUM_THREADS when set (16 on the GPU box), else the process's usable cores;
    # BASELINE.md's literal torch.set_num_threads(os.cpu_count()) is timed beside it
    env_threads = os.environ.get("OMP_NUM_THREADS", "")
    threads = int(env_threads) if env_threads.isdigit() and int(env_threads) > 0 else _usable_cores()
    torch.set_num_threads(threads)
    sd = weights.make_state_dict(cfg)
    m = clip_torch.TorchCLIP(sd, cfg)
    n_px = max(b1_frames, b64_frames, 64)
    px = weights.synthetic_pixels(n_px, cfg.image_resolution)
    tk = weights.synthetic_tokens(1, cfg.context_length, cfg.vocab_size)
    m.encode_image(px[:1])                                  # warm-up (allocator, thread pool)
    t0 = time.perf_counter()
    emb = np.concatenate([m.encode_image(px[i:i + 1]) for i in range(b1_frames)])
    t_b1 = (time.perf_counter() - t0) / b1_frames
    t0 = time.perf_counter()
    for i in range(0, b64_frames, 64):
        m.encode_image(px[i:i + 64])
    t_b64 = (time.perf_counter() - t0) / b64_frames
    t0 = time.perf_counter()
    np.concatenate([clip_ref.encode_image(px[i:i + 64], sd, cfg) for i in range(0, 64, 64)])
    t_np = (time.perf_counter() - t0) / 64
    t0 = time.perf_counter()
    txt = m.encode_text(tk)
    t_txt = time.perf_counter() - t0
    corpus = np.tile(emb, (n_frames_metric // emb.shape[0] + 1, 1))[:n_frames_metric]
    frames = list(range(n_frames_metric))
    t0 = time.perf_counter()
    rank_ref.search_top_frames_ref(corpus, txt, k, frames)
    t_rank = time.perf_counter() - t0

    def rate(t_img):
        return n_frames_metric / (n_frames_metric * t_img + Q * t_txt + Q * t_rank)

    check_cos = None
    if check is not None:   # the GPU's timed-pass rows of these frames against the fp32 CPU model
        cpx, crows = check
        ref = m.encode_image(cpx)
        check_cos = float(clip_ref.cosine(crows, ref).min())

    return {"value": round(rate(t_b1), 2), "unit": "frames/s", "cores": int(threads), "kind": "port",
            "check_min_cosine": check_cos,
            "nproc": os.cpu_count(), "cores_available": _usable_cores(), "cpu_model": _cpu_model(),
            "batch64_value": round(rate(t_b64), 2), "numpy_batch64_value": round(rate(t_np), 2),
            "threads_policy": "OMP_NUM_THREADS" if env_threads.isdigit() and int(env_threads) > 0
                              else "min(affinity, cgroup quota)",

            "sample": f"torch-CPU fp32 restatement of openai/CLIP (oracle/clip_torch.py), {threads} threads: "
                      f"{b1_frames} frames one per call as Backend/embedding.py:39-52 ({t_b1 * 1e3:.1f} ms/frame; "
                      f"batch 64 over {b64_frames} frames: {t_b64 * 1e3:.1f} ms/frame; numpy oracle batch 64: "
                      f"{t_np * 1e3:.1f} ms/frame) + 1 encode_text ({t_txt * 1e3:.1f} ms) + np.dot/argsort over "
                      f"{n_frames_metric} rows ({t_rank * 1e3:.2f} ms/query); extrapolated to {n_frames_metric} "
                      f"frames x {Q} queries"}


def rank_roofline(dev, reps=20):
    """The fused normalise + cosine + top-k kernel (mi_rank_topk) at sizes where
    it is HBM-bound (N*D*elt bytes per launch against the HBM
    roofline), HIP events on the launch stream: configs[3]'s 125k-row shard
    and a 1M-row corpus, D = 512 / 768, Q = 32 / 1000, f32 and bf16 rows."""
    import torch
    from miclip import retrieval
    out = {}
    g = torch.Generator(device=dev).manual_seed(3)
    for (N, D, Q, dt) in [(125_000, 512, 32, torch.float32), (1_000_000, 512, 32, torch.float32),
                          (1_000_000, 512, 32, torch.bfloat16), (1_000_000, 768, 32, torch.float32),
                          (1_000_000, 768, 1000, torch.float32)]:
        corpus = torch.randn(N, D, device=dev, generator=g).to(dt)
        q = torch.nn.functional.normalize(torch.randn(Q, D, device=dev, generator=g), dim=1)
        retrieval.rank_topk(corpus, q, 10)
        torch.cuda.synchronize(dev)
        stream = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = reps if Q <= 32 else 3
        e0.record(stream)
        for _ in range(n):
            retrieval.rank_topk(corpus, q, 10)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        us = e0.elapsed_time(e1) * 1e3 / n
        nbytes = corpus.numel() * corpus.element_size()
        name = f"N{N // 1000}k_D{D}_Q{Q}_{'f32' if dt == torch.float32 else 'bf16'}"
        out[name] = {"us": round(us, 1), "gbs": round(nbytes / us / 1e3, 1),
                     "hbm_frac": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
                     "tflops_f32_mfma": round(2.0 * N * Q * D / us / 1e6, 2)}
        if dt == torch.float32 and N >= 1_000_000:
            out[name.replace("_f32", "_mirror")] = mirror_timing(corpus, q, reps if Q <= 32 else 3, us)
        del corpus
    return out


def mirror_timing(corpus, q, n, exact_us):
    """The same ranking through the fp16 mirror (retrieval.MirroredCorpus,
    csrc/rank_mirror.hip): mirror pass + merge + exact re-score of 16
    candidates per query, certificate read back, exact pass for uncertified
    queries — the whole MirroredCorpus.topk, results checked identical to the
    exact pass.  bytes = the fp16 mirror's N*D*2."""
    import torch
    from miclip import retrieval
    mc = retrieval.MirroredCorpus(corpus)
    s, i = mc.topk(q, 10)
    s0, i0 = retrieval.rank_topk(corpus, q, 10)
    identical = bool(torch.equal(i, i0) and torch.equal(s, s0))
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(n):
        mc.topk(q, 10)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    nbytes = mc.mirror.numel() * 2
    return {"us": round(us, 1), "gbs": round(nbytes / us / 1e3, 1),
            "hbm_frac": round(nbytes / us / 1e3 / HBM_PEAK_GBS, 4),
            "speedup_vs_exact": round(exact_us / us, 2), "identical_to_exact": identical,
            "certified": f"{mc.certified}/{mc.certified + mc.fallbacks}"}


def parity_mode(args, dev, pixels, tokens, Q, k, base, chunk):
    """The R@K parity mode: the same step on the
    fp32 tower (`weights="fp32"`, openai/CLIP's fp32 arithmetic: f32 activations
    and residual stream, each tower GEMM as ONE 16-bit MFMA GEMM over split
    operands with f32 accumulation, at f32-GEMM accuracy; the exact-f32 MFMA GEMM
    is the A/B alternative), timed like the headline over --parity-steps steps,
    with the roofline of its c_fc GEMM against the 16-bit MFMA peak it runs on."""
    import torch
    from miclip import api, retrieval
    model, _ = api.load(args.model, device=dev, image_chunk=chunk, weights="fp32")
    cfg = model.cfg

    def step():
        emb = model.encode_image(pixels, out_dtype=torch.float32)
        txt = model.encode_text(tokens, normalize=True, out_dtype=torch.float32)
        return retrieval.rank_topk(emb, txt, k, index_base=base)

    step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.parity_steps):
        step()
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / args.parity_steps * 1e3
    kern = kernel_timing(model, cfg, chunk, reps=5)
    M = chunk * cfg.vision_tokens
    fl = 2.0 * M * 4 * cfg.vision_width * cfg.vision_width
    fc = kern["gemm_fc"]["us"]
    w = step_work(cfg, "fp32", chunk, False)
    t_peak = mfma_time_at_peak(w, "fp32", pixels.shape[0], Q, cfg.embed_dim)
    out = {"weights": "fp32", "value": round(pixels.shape[0] / (ms / 1e3), 1), "unit": "frames/s",
           "ms_per_step": round(ms, 3), "steps": args.parity_steps,
           "note": "fp32 tower (split-f16 GEMMs, f32-grade; exact-f32 MFMA attention): the mode whose R@1/5/10 "
                   "equal the float64 oracle flow (tests/test_gpu_rk_flow.py)",
           "roofline": {"bound": "mfma",
                        "kernel": "gemm_8q_kernel<EPI_F32> over split-f16 operands, K' = 3K, at mlp.c_fc's shape "
                                  "(mi_op_gemm_split2h; the tower's own c_fc launch adds QuickGELU and c_proj's "
                                  "operand split in the epilogue, EPI_SPLIT_GELU)",
                        "achieved": round(3 * fl / (fc * 1e-6) / 1e12, 1), "peak": BF16_PEAK_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(3 * fl / (fc * 1e-6) / 1e12 / BF16_PEAK_TFLOPS, 4),
                        "f32_equivalent_tflops": round(fl / (fc * 1e-6) / 1e12, 1),
                        "f32_mfma_peak": F32_MFMA_PEAK_TFLOPS,
                        "traffic": None, "launch_shape": [M, 4 * cfg.vision_width, 3 * cfg.vision_width],
                        "avg_launch_us": fc},
           # the executed work at its engines' peaks (split-f16 GEMMs: 3x the products on the f16 MFMA;
           # attention and rank on the exact-f32 MFMA) over the step time
           "mfma_frac_end_to_end": round(t_peak / (ms / 1e3), 4),
           "kernels": kern}
    del model
    torch.cuda.empty_cache()
    return out


def launch_workers(args):
    """`bench.py --gpus N` without torch.distributed.run: start N worker
    processes (one per GPU) through torch.distributed.run as a CHILD process,
    before this process touches the GPU, and return its exit code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def dry_run(args, world, rank):
    """Launcher rehearsal on CPU (gloo): the same rendezvous, barrier,
    max-over-ranks timing and top-k all-gather + merge shape as the GPU run,
    with no GPU and no kernels (tests/test_bench_launcher.py)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    Q, k = args.queries, args.k
    t0 = time.perf_counter()
    s = torch.full((Q, k), float(rank))
    i = torch.arange(Q * k, dtype=torch.int64).reshape(Q, k) + rank * 1_000_000
    if world > 1:
        gs = [torch.empty_like(s) for _ in range(world)]
        gi = [torch.empty_like(i) for _ in range(world)]
        dist.all_gather(gs, s)
        dist.all_gather(gi, i)
        ok = all(bool((gs[r] == r).all()) and bool((gi[r] // 1_000_000 == r).all()) for r in range(world))
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        seen = dist.get_world_size()
    else:
        ok, seen = True, 1
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": args.gpus, "world_size_seen": seen, "gather_ok": ok}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "0"))
    if world_env == 0 and args.gpus > 1:
        sys.exit(launch_workers(args))         # the parent never touches the GPU
    world = world_env or 1
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with `python -m torch.distributed.run "
              f"--nnodes=1 --nproc-per-node {args.gpus} --master-addr 127.0.0.1 --master-port P bench.py --gpus "
              f"{args.gpus} ...` or plain `python bench.py --gpus {args.gpus}`", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        return dry_run(args, world, rank)

    import numpy as np
    import torch
    import torch.distributed as dist

    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    os.environ.setdefault("MICLIP_SYNTHETIC_WEIGHTS", "1")     # random-init weights of the architecture (data: synthetic)
    if world > 1:
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:   # rehearsal: ranks may share a GPU (RCCL refuses two ranks on one device)
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from miclip import api, distributed, retrieval, weights

    strong = args.global_frames is not None
    if strong:     # configs[3]/[4]: a fixed corpus split into contiguous shards
        lo, hi = distributed.shard_range(args.global_frames, world, rank)
        Nf, base = hi - lo, lo
    else:          # weak scaling: every rank embeds its own --frames shard
        Nf, base = args.frames, rank * args.frames
    chunk = args.image_chunk
    if chunk is None:  # equal-size passes (so every GEMM launch has one shape)
        from miclip.config import get_config
        # up to ~500k token rows per pass: B/32's 10k frames in one pass (one
        # tile round fewer on the N = 768 / qkv GEMMs than two 5000-frame
        # passes; +0.4 % measured, scripts/gpu_ab_args.sh)
        cap = max(8, 500_000 // get_config(args.model).vision_tokens)
        chunk = -(-Nf // -(-Nf // cap))
    model, _ = api.load(args.model, device=dev, image_chunk=chunk, weights=args.weights)
    cfg = model.cfg
    chunk = model._chunks[0]
    Q, k = args.queries, args.k
    R = cfg.image_resolution
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    pixels = torch.randn(Nf, 3, R, R, device=dev, generator=g, dtype=torch.float32).bfloat16()
    tokens = torch.from_numpy(weights.synthetic_tokens(Q, cfg.context_length, cfg.vocab_size)).to(dev)

    def step():
        emb = model.encode_image(pixels, out_dtype=torch.float32)
        txt = model.encode_text(tokens, normalize=True, out_dtype=torch.float32)
        if world > 1:
            return emb, distributed.sharded_topk(emb, txt, k, base)
        return emb, retrieval.rank_topk(emb, txt, k, index_base=base)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    from miclip import _native as _N
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        emb, (top_s, top_i) = step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    # the roofline kernel (mlp.c_fc of the LayerNorm-folded bf16 tower) timed live: HIP events on the
    # launch stream around each of its launches (mi_clip_kernel_events) in `ev_steps` further steps of
    # the same workload run AFTER the timed loop, so the timed steps carry no event records
    ev_steps = min(args.steps, 5)
    n_fc = min(ev_steps * cfg.vision_layers * (-(-Nf // chunk)), 1 << 16)   # the library's event capacity
    fc_us = None
    if lnfold_active(model, cfg) and not args.no_kernel_timing:
        import ctypes
        _N.check(_N.lib().mi_clip_kernel_events(model._ctx, 1, n_fc), "mi_clip_kernel_events")
        for _ in range(ev_steps):
            step()
        torch.cuda.synchronize(dev)
        buf = (ctypes.c_float * n_fc)()
        got = _N.lib().mi_clip_kernel_times(model._ctx, buf, n_fc)
        _N.check(0 if got >= 0 else got, "mi_clip_kernel_times")
        _N.check(_N.lib().mi_clip_kernel_events(model._ctx, 0, 0), "mi_clip_kernel_events off")
        fc_us = [buf[i] for i in range(got)]
    seen = 1
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        seen = dist.get_world_size()
    assert torch.isfinite(top_s[:, 0]).all() and (top_i[:, 0] >= 0).all()
    # outside the timed region: the timed pass's rows at tile / XCD-range / 2^31-offset / last-tile
    # frames (tests/test_gpu_bench_config.py) re-encoded as one small chunk must be bit-identical
    # (every kernel's per-row arithmetic is independent of the pass size); the CPU baseline leg
    # checks the same rows against the torch-CPU fp32 restatement
    # (at least 8 frames, so that the re-encode's B * S rows fill the 256-row tiles the LayerNorm-folded
    # GEMMs need, as the timed pass does: 5 B/32 frames = 250 rows take the unfolded tower, whose
    # products round differently -- seen with --frames 4000)
    vidx = sorted({f for f in (0, 5, 1250, 2500, 4999, 6990, 9320, Nf - 1) if f < Nf})
    for f in range(Nf):
        if len(vidx) >= 8:
            break
        if f not in vidx:
            vidx.append(f)
    vidx = sorted(vidx)
    vt = torch.tensor(vidx, device=dev)
    emb_v = emb[vt].cpu()
    again = model.encode_image(pixels[vt], out_dtype=torch.float32).cpu()
    verify = {"frames": vidx, "single_pass_equals_small_chunk": bool(torch.equal(emb_v, again))}
    assert verify["single_pass_equals_small_chunk"], "timed pass rows differ from a small-chunk re-encode"

    ms = elapsed / args.steps * 1e3
    total_frames = (args.global_frames if strong else Nf * world) * args.steps
    value = total_frames / elapsed
    result = None
    if rank == 0:
        _progress(f"timed {args.steps} steps: {ms:.2f} ms/step; kernel timings")
        kern = {} if args.no_kernel_timing else kernel_timing(model, cfg, chunk)
        txt = model.encode_text(tokens, normalize=True, out_dtype=torch.float32)
        kern["rank_topk"] = rank_timing(emb, txt, k)
        kern["preprocess_720p"] = preprocess_timing(dev, cfg.image_resolution)
        ingest = jpeg_ingest_timing(dev, cfg.image_resolution)
        if ingest:
            kern["jpeg_ingest_720p"] = ingest
        _progress("rank roofline")
        rank_roof = None if args.no_rank_roofline else rank_roofline(dev)
        # executed work (step_work: the CLS-row last block of the bf16, MX-fp8 and fp32 towers at >= 256
        # frames per chunk) at its engines' dense peaks over the step time, per rank
        work = step_work(cfg, args.weights, chunk, lnfold_active(model, cfg))
        cls_last = work["cls_last"]
        mfma_frac = mfma_time_at_peak(work, args.weights, Nf, Q, cfg.embed_dim) / (ms / 1e3)
        dom = kern.get("gemm_fc")
        if dom and fc_us:   # the launches of the timed steps (events), not the micro loop
            dom = {"us": round(sum(fc_us) / len(fc_us), 2), "launches": len(fc_us),
                   "min_us": round(min(fc_us), 2), "max_us": round(max(fc_us), 2),
                   "micro_us": kern["gemm_fc"]["us"]}
        M = chunk * cfg.vision_tokens
        roof = None
        if dom:
            fl = 2.0 * M * 4 * cfg.vision_width * cfg.vision_width
            fp8 = args.weights == "fp8"
            f32 = args.weights == "fp32"
            if f32:   # the MFMA work the split-f16 GEMM executes: K' = 3K on the f16 MFMA
                fl *= 3
            ach = fl / (dom["us"] * 1e-6) / 1e12
            shape = [M, 4 * cfg.vision_width, cfg.vision_width]
            lnf = lnfold_active(model, cfg)
            traffic, tsrc, busy = (None, None, None) if f32 else pmc_traffic(shape, fp8, 7 if lnf else None)
            peak = FP8_PEAK_TFLOPS if fp8 else BF16_PEAK_TFLOPS
            eb = 1 if fp8 else 2   # operand element bytes (fp8 adds 1/64 B of scales per element; fp32: 3 fp16 terms)
            roof = {"bound": "mfma",
                    "kernel": ("gemm_mxppp_kernel<EPI_GELU_MX> (mlp.c_fc + QuickGELU -> MX-fp8, MX-fp8 operands; "
                               "persistent ping-pong)" if fp8
                               else "gemm_8q_kernel<EPI_F32> (split-f16 operands, K' = 3K, at mlp.c_fc's shape)" if f32
                               else "gemm_8q_kernel<EPI_LN_GELU_BF16> (8-phase interleaved persistent, 256x256x64, descriptor DMAs; "
                               "ln_2 folded into the epilogue, fp16 operands on the f16 MFMA; mlp.c_fc + QuickGELU)" if lnf
                               else "gemm_8q_kernel<EPI_GELU_BF16> (8-phase interleaved persistent, 256x256x64, descriptor DMAs; mlp.c_fc + QuickGELU)"),
                    "achieved": round(ach, 1), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4), "traffic": traffic,
                    "traffic_source": tsrc,
                    "mfma_busy_pmc": busy,
                    "algorithmic_bytes": int(eb * (1 + fp8 / 64) * (3 if f32 else 1) * (M * cfg.vision_width + 4 * cfg.vision_width ** 2)
                                             + ((1 + 1 / 64) if fp8 else 4 if f32 else 2) * M * 4 * cfg.vision_width
                                             + (8 * M + 8 * 4 * cfg.vision_width if lnf else 0)),
                    "flops_per_launch": fl, "launch_shape": [M, 4 * cfg.vision_width, cfg.vision_width],
                    "avg_launch_us": dom["us"],
                    "timing": (f"HIP events around each c_fc launch of {ev_steps} steps run after the timed loop "
                               f"(mi_clip_kernel_events; the timed steps are not instrumented): "
                               f"{dom['launches']} launches, {dom['min_us']}-{dom['max_us']} us; the random-operand "
                               f"micro loop (kernels.gemm_fc) {dom['micro_us']} us") if "launches" in dom
                              else "HIP events around the kernel_timing micro loop (random operands)"}
        parity = None
        _progress("parity mode / cpu baseline")
        if not args.no_parity_mode and world == 1 and args.weights == "bf16":
            parity = parity_mode(args, dev, pixels, tokens, Q, k, base, chunk)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(cfg, Nf, Q, k, args.cpu_frames_b1, args.cpu_frames,
                               check=(pixels[vt].float().cpu().numpy(), emb_v.numpy()))
            verify["gpu_rows_vs_cpu_fp32_min_cosine"] = cpu.pop("check_min_cosine", None)
        workload = f"{cfg.name} {args.weights}, "
        if strong:
            workload += f"{args.global_frames} frames over {world} shards x {Q} text queries, top-{k}"
        else:
            workload += f"{Nf} frames/GPU x {Q} text queries, top-{k}"
        if world > 1:
            workload += (" (RCCL all-gather top-k)" if args.dist_backend == "nccl"
                         else " (gloo all-gather top-k: a rehearsal, ranks sharing GPUs)")
        elif (cfg.name, Nf, Q, k) == ("ViT-B/32", 10_000, 32, 10):
            workload += " (BASELINE configs[1])"
        result = {
            "metric": "frames/sec embedded+ranked, ViT-B/32 224², 1/2/4/8 MI355X; R@1/5/10 parity",
            "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "world_size_seen": seen, "build_id": _N.lib().mi_build_id().decode(),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None,
            "dtype": {"bf16": "bf16", "fp32": "f32"}.get(args.weights, "fp8-e4m3(MX) vision GEMMs, bf16 rest"),
            "data": "synthetic (random pixels/tokens, deterministic random-init weights of the real architecture)",
            "config": {"workload": workload, "frames_per_gpu": Nf,
                       "global_frames": args.global_frames if strong else Nf * world, "queries": Q, "k": k,
                       "image_chunk": chunk, "parallelism": f"dp{world}"},
            "roofline": roof,
            "rank_roofline": rank_roof,
            "mfma_frac_end_to_end": round(mfma_frac, 4),
            "mfma_frac_flops": ("executed work at each engine's dense peak over the step time: the last block's "
                                "out_proj / c_fc / c_proj on the CLS rows only (their other rows are never read)"
                                + ("; its Q projection and attention for the CLS queries only" if cls_last and args.weights != "fp8" else "")
                                if cls_last else "the full model at each engine's dense peak over the step time"),
            "parity_mode": parity,
            "verify": verify,
            "kernels": kern,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
