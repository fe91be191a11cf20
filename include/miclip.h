/*
 * miclip.h — C-ABI of the MI355X-native CLIP frame-embedding + text->frame
 * retrieval path (gfx950 HIP kernels in libmiclip.so).
 *
 * The reference has no native code: its GPU work is the
 * third-party openai/CLIP package driven from Python, and its ranking is host
 * NumPy.  Each entry point below replaces one reference interface; the
 * replaced interface is cited next to it.  Plain pointers and sizes only: the
 * Python host (`miclip/_native.py`, ctypes) passes torch tensors' data_ptr()
 * and the current HIP stream.
 *
 * Conventions
 *   - Return 0 (MI_OK) on success, a negative MI_ERR_* code on error; the
 *     message is in mi_last_error() (thread-local).  The Python shim raises.
 *   - Callers own every input/output buffer (device pointers unless noted);
 *     an mi_clip context owns weights and activation workspace.
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  No entry point
 *     allocates or synchronises after mi_clip_reserve(), so encode/rank calls
 *     can be captured in a hipGraph.
 *   - Context entry points are serialised by a per-context mutex (the Flask
 *     dev server shares one EmbeddingService across request threads,
 *     Backend/app.py:969).
 *   - Ranking order: score descending, then global index ascending.  NaN
 *     scores (zero-norm rows) sort first under MI_NAN_FIRST
 *     (np.argsort(s)[::-1], embedding_service.py:317-320) or last under
 *     MI_NAN_LAST (np.argsort(-s), compare_models.py:1014).
 */
#ifndef MICLIP_H
#define MICLIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MICLIP_ABI_VERSION 7   /* 2: mi_jpeg_workspace_bytes / mi_jpeg_decode take the data size;
                                  3: mi_normalize_rows_f16, mi_jpeg_decode_transform;
                                  4: mi_op_split2h, mi_op_gemm_split2h, mi_op_attention_f32;
                                  5: mi_clip_kernel_events, mi_clip_kernel_times;
                                  6: mi_build_id, mi_build_sources;
                                  7: mi_op_attention_f32_split */

enum mi_dtype { MI_F32 = 0, MI_BF16 = 1, MI_F16 = 2, MI_FP8 = 3 /* weights only: MX-fp8 vision GEMMs */ };
enum mi_status { MI_OK = 0, MI_ERR_ARG = -1, MI_ERR_HIP = -2, MI_ERR_UNSUPPORTED = -3, MI_ERR_STATE = -4 };
enum mi_nan_policy { MI_NAN_FIRST = 0, MI_NAN_LAST = 1 };
/* corpus row normalisation inside the rank/score kernels */
enum mi_norm_mode {
  MI_NORM_L2 = 0,       /* e/||e|| ; zero row -> NaN   (embedding_service.py:210)           */
  MI_NORM_L2_GUARD = 1, /* e/||e|| if ||e||>1e-8 else e (compare_models.py:1168-1171)       */
  MI_NORM_NONE = 2      /* raw dot products (features already normalised, compare_models:999) */
};

/* image preprocessing (mi_preprocess_frames) */
enum mi_prep_mode {
  MI_PREP_CLIP = 0,   /* openai/CLIP _transform: Resize(n, bicubic) short side + CenterCrop(n) + ToTensor + Normalize */
  MI_PREP_SQUASH = 1  /* compare_models.py:387-391: Resize((n, n)) (bilinear) + ToTensor + Normalize            */
};
enum mi_resample_filter { MI_RESAMPLE_BICUBIC = 0, MI_RESAMPLE_BILINEAR = 1 };

/* Architecture of a ViT CLIP (openai/CLIP build_model inference; miclip/config.py). */
typedef struct mi_clip_arch {
  int32_t embed_dim;         /* D: 512 (B/32), 768 (L/14)      */
  int32_t image_resolution;  /* 224 / 336                      */
  int32_t vision_layers;
  int32_t vision_width;      /* multiple of 64; heads = width/64 */
  int32_t vision_patch_size;
  int32_t context_length;    /* 77                             */
  int32_t vocab_size;        /* 49408                          */
  int32_t text_width;        /* multiple of 64                 */
  int32_t text_heads;        /* text_width / 64                */
  int32_t text_layers;
} mi_clip_arch;

typedef struct mi_clip mi_clip;

int mi_abi_version(void);
/* The library's source fingerprint: the first 16 hex digits of the sha256 of the concatenated
   sources it was compiled from (mi_build_sources: their names, relative to csrc/, in order).
   miclip._native recomputes it from the sources next to the library and refuses a mismatch. */
const char* mi_build_id(void);
const char* mi_build_sources(void);
const char* mi_last_error(void);

/* Number of float32 elements of the canonical weight blob for `arch`
 * (OpenAI state-dict tensors concatenated in the order documented in
 * DESIGN.md "Weight blob"; packer: miclip/_native.py pack_weights). */
int64_t mi_clip_weights_numel(const mi_clip_arch* arch);

/* Replaces openai/CLIP `clip.load(name, device, jit=False)` model construction
 * (call sites Backend/embedding.py:22, Backend/services/embedding_service.py:86,106,
 * compare_models.py:316).  `weights` is a HOST float32 blob of
 * mi_clip_weights_numel(arch) elements; weights are converted to `weight_dtype`
 * and uploaded to `device`:
 *   MI_BF16  bf16 MFMA GEMMs, fp16 vision residual stream (throughput mode; the
 *            reference's GPU path is fp16, openai/CLIP convert_weights);
 *   MI_F32   every GEMM on the exact-f32 MFMA, every activation and the residual
 *            stream f32 — the reference's CPU / `model.float()` arithmetic
 *            (Backend/embedding.py:21-22 on a CPU, CLIPWithClassifier
 *            embedding_service.py:22): the parity mode of the R@K flow;
 *   MI_FP8   the vision tower's four GEMMs per block on the block-scaled fp8 MFMA
 *            with MX-fp8 weights (e4m3 + e8m0 per 64 k) and MX-fp8 activations
 *            produced by the LayerNorm / attention / QuickGELU kernels
 *            (BASELINE.json configs[4]). */
int mi_clip_create(const mi_clip_arch* arch, const float* weights, int64_t numel,
                   int device, int weight_dtype, mi_clip** out);
int mi_clip_destroy(mi_clip* ctx);

/* Allocate activation workspace for up to `image_chunk` frames / `text_chunk`
 * queries per internal pass (larger batches are processed chunk by chunk).
 * The only allocating call besides create. */
int mi_clip_reserve(mi_clip* ctx, int64_t image_chunk, int64_t text_chunk);

/* Replaces `model.encode_image(x)` (VisionTransformer.forward; call sites
 * Backend/embedding.py:49, embedding_service.py:490, compare_models.py:1118)
 * and, with l2_normalize=1, the normalisation that follows it
 * (embedding_service.py:502, CLIPWithClassifier.forward :45); l2_normalize=2 is
 * compare_models.py's guarded form (f/||f|| if ||f|| > 1e-8 else f, :1166-1171).
 * pixels: device [B,3,R,R] in `in_dtype` (MI_F32 / MI_BF16);
 * out: device [B,embed_dim] in `out_dtype` (MI_F32 / MI_BF16 / MI_F16). */
int mi_clip_encode_image(mi_clip* ctx, const void* pixels, int64_t B, int in_dtype,
                         void* out, int out_dtype, int l2_normalize, void* stream);

/* Replaces `model.encode_text(tokens)` (embedding_service.py:174,177;
 * compare_models.py:1204).  tokens: device int32 [Q,context_length] in
 * clip.tokenize format; pooling at the row argmax (EOT). */
int mi_clip_encode_text(mi_clip* ctx, const int32_t* tokens, int64_t Q,
                        void* out, int out_dtype, int l2_normalize, void* stream);

/* Workspace bytes mi_rank_topk needs for (N, Q, k). */
size_t mi_rank_workspace_bytes(int64_t N, int64_t Q, int32_t k);

/* Replaces the ranking of EmbeddingService.search_top_frames
 * (embedding_service.py:314-320: np.dot(E_normalised, t.T) + np.argsort(s)[::-1][:k])
 * and search_top_frames_by_image (:365-372).  One fused pass: per corpus row
 * L2 norm (norm_mode) + fp32-exact dot with every query + top-k.
 * corpus: device [N,D] (MI_F32/MI_BF16/MI_F16, row stride D); queries: device
 * f32 [Q,D]; out_scores f32 [Q,k], out_index int64 [Q,k] (global index =
 * index_base + row; slots past N are index -1, score -inf).  32 <= D <= 1024,
 * D % 32 == 0 (32 queries x D f32 are staged in LDS).  1 <= k <= 2^24:
 * k <= 64 is the single fused pass (register top-k lists); larger k (the
 * reference's top_k*3 candidates for UI requests above 21, query_strategies.py:55,
 * and full sorts, embedding_service.py:317-318) runs the exact score matrix +
 * radix select + sort kernels over the same scores, with the workspace
 * mi_rank_workspace_bytes reports for that k (it includes Q*N f32 scores). */
int mi_rank_topk(const void* corpus, int64_t N, int64_t D, int corpus_dtype,
                 const float* queries, int64_t Q, int32_t k, int64_t index_base,
                 int norm_mode, int nan_policy, float* out_scores, int64_t* out_index,
                 void* workspace, size_t workspace_bytes, void* stream);

/* Ranking mirror of a corpus for mi_rank_mirror (an
 * HBM-resident half-width mirror beside the f32 master of
 * EmbeddingService.get_embeddings, embedding_service.py:186-217).
 * mirror: device fp16 [N,D] = c / ||c|| per row, with the reciprocal norm of
 * mi_rank_topk's MI_NORM_L2 (a zero row becomes NaN, as E/||E|| does at
 * embedding_service.py:210).  D = 512 or 768. */
int mi_mirror_build(const void* corpus, int64_t N, int64_t D, int corpus_dtype, void* mirror_f16, void* stream);

/* Replaces get_embeddings' row normalisation of a float16 `.npy` corpus
 * (Backend/services/embedding_service.py:209-210,
 * `embeddings / np.linalg.norm(embeddings, axis=-1, keepdims=True)` evaluated by
 * NumPy in float16 — the reference's default corpus files video_test_3 /
 * image_embeddings.npy are float16) bit for bit: f16 squares, NumPy's pairwise
 * f32 summation of them rounded to f16, f16 sqrt, f16 quotients (csrc/corpus.hip).
 * A zero row becomes NaN as in the reference.  rows / out: device fp16 [N,D]
 * (out == rows allowed); 1 <= D <= 1024.  search_top_frames' ranking of such a
 * file is then mi_rank_topk(out, ..., MI_F16, MI_NORM_NONE, ...) with the f32
 * query (embedding_service.py:314-320). */
int mi_normalize_rows_f16(const void* rows, int64_t N, int64_t D, void* out, void* stream);

/* Workspace bytes mi_rank_mirror needs for (N, Q). */
size_t mi_rank_mirror_workspace_bytes(int64_t N, int64_t Q);

/* search_top_frames' ranking (embedding_service.py:314-320, MI_NORM_L2) through
 * the mirror: one fp16 MFMA pass over the mirror (half the f32 bytes) for the
 * top 16 mirror candidates per query, then the exact f32 scores of those
 * candidates from the master with mi_rank_topk's arithmetic and a per-query
 * certificate.  out_certified[q] = 1: out_scores/out_index [Q,k] are
 * bit-identical to mi_rank_topk(master, ..., MI_NORM_L2, nan_policy); 0: a
 * near-tie across the candidate edge or a non-finite score: rank that query
 * with mi_rank_topk.  1 <= k <= 16. */
int mi_rank_mirror(const void* mirror_f16, const void* master, int64_t N, int64_t D, int master_dtype,
                   const float* queries, int64_t Q, int32_t k, int64_t index_base, int nan_policy,
                   float* out_scores, int64_t* out_index, int32_t* out_certified,
                   void* workspace, size_t workspace_bytes, void* stream);

/* Merge per-query candidate lists (e.g. the RCCL all-gather of per-shard
 * top-k) into the global top-k with the same order rule.
 * cand_scores f32 [Q,C], cand_index int64 [Q,C] (index -1 = empty slot); 1 <= k <= 64. */
int mi_rank_merge(const float* cand_scores, const int64_t* cand_index, int64_t Q, int64_t C,
                  int32_t k, int nan_policy, float* out_scores, int64_t* out_index, void* stream);

/* Full similarity matrix for the R@K evaluation flow
 * (compare_models.py:999 `image_features @ text_features.T`):
 * out[q][n] = <queries[q], corpus[n]/norm(n)>  (f32, fp32-exact products). */
int mi_score_matrix(const void* corpus, int64_t N, int64_t D, int corpus_dtype,
                    const float* queries, int64_t Q, int norm_mode, float* out, void* stream);

/* Rank of a target column per query row (compare_models.py:1013-1015,
 * 1057-1061: position of the ground truth in argsort(-s), 1-based):
 * rank[t] = 1 + #{n : s[q][n] > s[q][g]} + #{n < g : s[q][n] == s[q][g]},
 * q = pair_query[t], g = pair_target[t]; NaN sorts last (argsort(-s)). */
int mi_rank_of_targets(const float* scores, int64_t Q, int64_t N, const int64_t* pair_query,
                       const int64_t* pair_target, int64_t T, int64_t* out_rank, void* stream);

/* Pillow ImagingResample coefficients (host only, no GPU): the resize of
 * in_size -> out_size over the source box [in0, in1) with `filter`, exactly as
 * Pillow computes them (libImaging/Resample.c precompute_coeffs +
 * normalize_coeffs_8bpc; restated in oracle/preprocess_ref.py).  Writes
 * kk [out_size][ksize] int32 (22 fractional bits) and bounds [out_size][2] =
 * (first tap, tap count); returns ksize (> 0) or a negative MI_ERR_*.
 * Exposed so the host side of the preprocessing can be checked on a CPU. */
int mi_resample_coeffs(int32_t in_size, double in0, double in1, int32_t out_size, int filter, int32_t* kk,
                       int64_t kk_cap, int32_t* bounds);

/* Workspace bytes mi_preprocess_frames needs. */
size_t mi_preprocess_workspace_bytes(int64_t B, int32_t H, int32_t W, int32_t n, int mode);

/* Replaces the per-frame host preprocessing before encode_image
 * (openai/CLIP `preprocess(Image.open(p))`: Backend/embedding.py:46,
 * Backend/services/embedding_service.py:406,475; and the squash transform of
 * compare_models.py:387-391) for a batch of decoded frames of one size.
 * frames: device uint8 [B,H,W,3] (RGB, row-major HWC); out: device [B,3,n,n]
 * in MI_F32 / MI_BF16.  Resampling is Pillow-exact (the uint8 image before
 * ToTensor is bit-identical to PIL.Image.resize), ToTensor/Normalize are f32
 * as torchvision computes them. */
int mi_preprocess_frames(const uint8_t* frames, int64_t B, int32_t H, int32_t W, int32_t n, int mode, void* out,
                         int out_dtype, void* workspace, size_t workspace_bytes, void* stream);

/* ---- baseline JPEG decode ----
 * Replaces the host decode of the reference's frame ingest,
 * `Image.open(p).convert("RGB")` (Backend/services/embedding_service.py:472-480,
 * Backend/embedding.py:46), for a batch of baseline-Huffman JPEGs of ONE geometry;
 * output bit-identical to Pillow (libjpeg ISLOW IDCT, fancy upsampling, JCS_RGB).
 * The caller (miclip/jpeg.py) parses headers and builds the tables; all pointers
 * are device memory:
 *   data      concatenated entropy-coded segments of all frames (bytes after SOS),
 *             readable for 16 bytes past the last segment end (aligned 16-byte reads);
 *             data_bytes = its size (the segments lie in [0, data_bytes))
 *   seg_off / seg_end  [B * nseg] byte offsets of each restart segment (nseg = 1
 *             without restart markers); a segment ends at its RSTn / EOI marker.
 *             Contract: frames' segments are disjoint, in frame order and inside
 *             [0, data_bytes) (miclip/jpeg.py concatenates the frames' scans).  Offsets
 *             are clipped to [0, data_bytes) on the device; with nseg = 1 a frame whose
 *             segment starts before an earlier frame's end (a repeated or out-of-order
 *             frame) is left out of the chunked decode and decoded by the serial
 *             kernel, so no input layout writes outside the workspace
 *   huff      [nsets][4] decode tables {dc0, ac0, dc1, ac1}, MI_JPEG_HUFF_BYTES each
 *   huff_idx  [B] int32 table set of each frame, in [0, nsets) (frames of one
 *             encoder share a set; up to 11 sets are staged in LDS), or NULL:
 *             frame f uses set f (nsets ignored)
 *   qtab      [B][4][64] uint16 quantisation tables in natural order
 *   geom      host int32[20]: W, H, ncomp (1 or 3), restart interval (MCUs),
 *             nseg, (h, v) sampling per component, quant / dc / ac table
 *             selector per component
 *   out_rgb   [B, H, W, 3] uint8
 * Supported: 8-bit, 1 component, or 3 components with chroma 1x1 and luma
 * 1x1 / 2x1 / 2x2.  Scans without restart markers (nseg = 1) are entropy-decoded
 * by 1-KB chunks in parallel (speculative decode + consistency rounds, jpeg.hip),
 * scans with restart intervals one lane per interval; the workspace holds the
 * coefficients, the component planes and, for nseg = 1, the chunk state and an
 * unstuffed copy of the data. */
#define MI_JPEG_HUFF_BYTES 3480
size_t mi_jpeg_workspace_bytes(const int32_t* geom, int32_t B, int64_t data_bytes);
int mi_jpeg_decode(const uint8_t* data, int64_t data_bytes, const int64_t* seg_off, const int64_t* seg_end, const void* huff,
                   const int32_t* huff_idx, int32_t nsets, const uint16_t* qtab, const int32_t* geom, int32_t B,
                   uint8_t* out_rgb, void* workspace, size_t workspace_bytes, void* stream);

/* mi_jpeg_decode fused with mi_preprocess_frames: the same arguments and workspace
 * (mi_jpeg_workspace_bytes), and out = device [B,3,n,n] (MI_F32 / MI_BF16) =
 * mi_preprocess_frames(decoded RGB, n, mode) bit for bit — Pillow decode +
 * openai/CLIP _transform (mode MI_PREP_CLIP) or compare_models.py's squash
 * (MI_PREP_SQUASH), i.e. the reference's `preprocess(Image.open(p))`
 * (Backend/services/embedding_service.py:472-480, Backend/embedding.py:46) — without
 * the RGB frames: colour conversion, both resample passes and Normalize run in one
 * kernel over the component planes (csrc/jpeg.hip jpeg_transform_kernel).
 * MI_ERR_UNSUPPORTED when the source does not fit its LDS bands (then decode +
 * preprocess separately). */
int mi_jpeg_decode_transform(const uint8_t* data, int64_t data_bytes, const int64_t* seg_off, const int64_t* seg_end,
                             const void* huff, const int32_t* huff_idx, int32_t nsets, const uint16_t* qtab,
                             const int32_t* geom, int32_t B, int32_t n, int mode, void* out, int out_dtype,
                             void* workspace, size_t workspace_bytes, void* stream);

/* Host-side gather of the frames' entropy-coded bytes into one (pinned) staging
 * buffer before the upload: n pieces src[i] of len[i] bytes concatenated into
 * dst on `threads` host threads (plain memcpy; the Python caller's bytes
 * objects stay where they are).  Replaces the reference's per-file host decode
 * inputs (embedding_service.py:472-480) on the way to mi_jpeg_decode. */
int mi_host_gather(void* dst, const void* const* src, const int64_t* len, int64_t n, int32_t threads);

/* ---- operator-level entry points (per-kernel parity tests) ----
 * mi_op_gemm: out = A[M,K] . W[N,K]^T (+bias) with epilogue
 *   0: bf16 out; 1: bf16 QuickGELU out; 2: f32 out += (residual); 3: f32 out.
 *   (nn.Linear of attn.in_proj / out_proj / mlp.c_fc / c_proj, conv1 as GEMM)
 * mi_op_layernorm: bf16 out = LN(x f32 [rows,W]) (openai/CLIP LayerNorm, fp32)
 * mi_op_attention: bf16 [B*S, W] = MHA core over packed qkv bf16 [B*S, 3W]
 *   (nn.MultiheadAttention softmax(qk^T/8)v per 64-wide head; causal for text).
 *   causal bit 0: causal mask; bits 8 / 9 select the alternative kernels for
 *   A/B and parity tests (one-wave S <= 96 / chunk-streaming flash S > 64) */
int mi_op_gemm(const void* A, const void* W, const float* bias, void* out, int32_t M, int32_t N, int32_t K,
               int32_t epilogue, void* stream);
/* mi_op_gemm_f32: f32 out[M,N] = A[M,K] . W[N,K]^T (+bias) on the exact-f32 MFMA (the
 *   MI_F32 tower's GEMM, precise.hip); epilogue 0 store, 1 QuickGELU, 2 out += (residual),
 *   3 ReLU (CLIPWithClassifier's classifier head, embedding_service.py:26-31).  K % 32 == 0,
 *   any M, N; rows of A / W contiguous (lda = ldw = K, ldo = N). */
int mi_op_gemm_f32(const float* A, const float* W, const float* bias, float* out, int32_t M, int32_t N, int32_t K,
                   int32_t epilogue, void* stream);
int mi_op_layernorm(const float* x, const float* gamma, const float* beta, void* out, int32_t rows, int32_t W,
                    void* stream);
int mi_op_attention(const void* qkv, void* out, int32_t B, int32_t S, int32_t W, int32_t causal, void* stream);
/* mi_op_residual_ln: x += delta (bf16 [rows,W]); out bf16 = LN(x) — the residual add +
 *   ln_2 / next ln_1 of openai/CLIP ResidualAttentionBlock (x = x + attn(ln_1(x));
 *   x = x + mlp(ln_2(x))).  xmode 0: x f32 [rows,W]; 1: x read f32, written back fp16
 *   into the first half of each f32 row slot; 2: x fp16 in that half-row layout
 *   (the vision tower's residual stream after its first add). */
int mi_op_residual_ln(void* x, const void* delta, const float* gamma, const float* beta, void* out, int32_t rows,
                      int32_t W, int32_t xmode, void* stream);
/* The LayerNorm-folded pair of the bf16 vision tower, the same
 * ResidualAttentionBlock arithmetic with ln_1 / ln_2 moved into the GEMM epilogue:
 * mi_op_residual_stats: x (fp16 half-slot layout, xmode 2 above) += delta (bf16 [rows,W]);
 *   rs [rows][2] f32 = (rstd, rstd * mean) of each stored row (LayerNorm eps 1e-5).
 * mi_op_gemm_ln: out bf16 [M,N] = LN(x) . W^T + b computed as
 *   rstd * (x . Wf^T) - rstd * mean * colsum + colc, QuickGELU applied when gelu == 1
 *   (attn.in_proj after ln_1: gelu 0; mlp.c_fc after ln_2: gelu 1).  x16: fp16 rows of
 *   stride lda elements; rs: as above, READABLE for M + 256 rows (the kernel stages
 *   whole 256-row tiles; the extra rows are never used); Wf [N,K] fp16 = W * gamma
 *   (column-scaled nn.Linear weight); colsum [N] = sum_k Wf[n,k];
 *   colc [N] = b_n + sum_k beta_k W[n,k].  N % 256 == 0, K % 128 == 0, K >= 256,
 *   M >= 256, lda >= K, lda % 8 == 0. */
int mi_op_residual_stats(void* x, const void* delta, float* rs, int32_t rows, int32_t W, void* stream);
/* mi_op_split6: the split-bf16 operands of the fp32 tower's GEMMs (weight_dtype MI_F32,
 *   DESIGN.md §4.7).  Each f32 value x = x1 + x2 + x3 + O(2^-24 |x|), x1 = bf16(x),
 *   x2 = bf16(x - x1), x3 = bf16(x - x1 - x2) (round to nearest even; inf / NaN: x2 = x3 = 0;
 *   a finite x that rounds past bf16's range takes x1 = the largest bf16 of its sign);
 *   row r of x [rows][K] (stride ldx floats) becomes out[r] = 6K bf16 in six K-blocks:
 *   role 0 (activations) [x1 x2 x3 x1 x2 x1], role 1 (weights, [N][K]) [x1 x1 x1 x2 x2 x3].
 *   mi_op_gemm (epilogue 2 or 3) over K' = 6K then sums a1w1 + a2w1 + a3w1 + a1w2 + a2w2 +
 *   a1w3 in f32.  gelu 1 applies QuickGELU (x * 1 / (1 + exp(-1.702 x))) first. */
int mi_op_split6(const float* x, int64_t ldx, int64_t rows, int32_t K, int32_t role, int32_t gelu, void* out,
                 void* stream);
/* mi_op_split2h: the split-f16 operands of the fp32 tower's GEMMs (weight_dtype MI_F32, the
 *   default since ABI 4).  Row r of x [rows][K] (stride ldx floats) is scaled
 *   by a power of two s_r with max_k |x[r][k] s_r| in [2^13, 2^14) (s_r = 1 for an all-zero or
 *   non-finite row; the exponent clamped to [-126, 126]) and split as x s = x1 + x2 + O(2^-22
 *   |x s|), x1 = f16(x s), x2 = f16(x s - x1) (round to nearest even; x2 = 0 where x1 is not
 *   finite); out[r] = 3K fp16 in three K-blocks, role 0 (activations) [x1 x1 x2], role 1
 *   (weights [N][K]) [x1 x2 x1]; role 2 (activations stored once, 2K fp16 per row) [x1 x2];
 *   scale[r] = 1 / s_r.  gelu 1 applies QuickGELU first (as mi_op_split6).  K % 4 == 0,
 *   4 <= K <= 4096, ldx % 4 == 0.
 * mi_op_gemm_split2h: out f32 [M,N] (epi 3) or out += (epi 2) of
 *   (A3 . W3^T) * a_scale[m] * w_scale[n] + bias[n], with A3 [M][K3] / W3 [N][K3] the fp16
 *   operands above (K3 = 3K) on the f16 MFMA with f32 accumulation: a1 w1 + a1 w2 + a2 w1, an
 *   f32-grade product.  N % 128 == 0, K3 % 32 == 0.  epi | 0x100: A3 is the role-2 layout
 *   [M][2K] (the 8-phase kernel reads it as [x1 x1 x2]; needs a bias, M >= 256,
 *   N % 256 == 0, K % 64 == 0).
 * mi_op_attention_f32: f32 MHA core of the fp32 tower: qkv f32 [B*S, 3W] (q | k | v, head dim
 *   64) -> out f32 [B*S, W], softmax(q k^T / 8 (+ causal mask)) v per (sequence, head); S <= 64
 *   on split-f16 operands on the f16 MFMA (f32-GEMM grade, as mi_op_gemm_split2h), S <= 128 on the
 *   exact-f32 MFMA, longer sequences on a per-row f32 kernel.
 * mi_op_attention_f32_split (S <= 64): the same output as out_proj's split operand (role 0
 *   [x1 x1 x2] / role 2 [x1 x2] fp16 rows, as mi_op_split2h) with ONE scale per sequence,
 *   scale[row] = 1 / s: s is the power of two with B_seq s in [2^13, 2^14) for the bound
 *   B_seq = (max over the sequence's rows of rmax[row] * bw + bb) * (1 + 2^-8) -- rmax the row max
 *   |h| of the LayerNorm output that produced V = h W_v^T + b_v, bw = max_d sum_k |W_v[d][k]|,
 *   bb = max |b_v| -- so every head of a row shares it; x1 = f16(o s), x2 = f16(o s - x1). */
int mi_op_split2h(const float* x, int64_t ldx, int64_t rows, int32_t K, int32_t role, int32_t gelu, void* out,
                  float* scale, void* stream);
/* Kernel timing of the product path (measurement only; bench.py's roofline): after
 * mi_clip_kernel_events(ctx, MI_KERNEL_C_FC, capacity) the next `capacity` launches of the
 * vision tower's mlp.c_fc GEMM (the LayerNorm-folded bf16 tower) are bracketed by HIP events on
 * the caller's stream; mi_clip_kernel_times(ctx, us, n) waits for them and writes the first
 * min(n, recorded) durations in microseconds, returning that count.  capacity 0 (or kind
 * MI_KERNEL_NONE) switches the recording off. */
enum mi_kernel_kind { MI_KERNEL_NONE = 0, MI_KERNEL_C_FC = 1 };
int mi_clip_kernel_events(mi_clip* ctx, int32_t kind, int32_t capacity);
int mi_clip_kernel_times(mi_clip* ctx, float* us, int32_t n);
int mi_op_gemm_split2h(const void* A3, const void* W3, const float* a_scale, const float* w_scale, const float* bias,
                       float* out, int32_t M, int32_t N, int32_t K3, int32_t epi, void* stream);
int mi_op_attention_f32(const float* qkv, float* out, int32_t B, int32_t S, int32_t W, int32_t causal, void* stream);
int mi_op_attention_f32_split(const float* qkv, const float* rmax, float bw, float bb, void* out, int32_t role,
                              float* scale, int32_t B, int32_t S, int32_t W, int32_t causal, void* stream);
int mi_op_gemm_ln(const void* x16, int64_t lda, const float* rs, const void* Wf, const float* colsum,
                  const float* colc, void* out, int32_t M, int32_t N, int32_t K, int32_t gelu, void* stream);
/* mi_op_gemm_residual: attn.out_proj / mlp.c_proj with the residual add fused (replaces
 *   mi_gemm + mi_op_residual_stats in the folded tower):
 *   x16 [M][W] fp16 (row stride ldx elements) = f16(x16 + bf16(A . W^T + bias)) — exactly
 *   mi_op_residual_stats' stored values — and rs [M][2] = (rstd, rstd * mean) of the stored
 *   rows, combined from per-64-column partials (sum, sum of squared deviations) that the GEMM
 *   epilogue writes to ps [M][W / 64][2] f32 (scratch).  A [M][K] bf16 (stride lda), W [W][K]
 *   bf16, bias [W] f32 or NULL.  W % 256 == 0, W <= 1024, K % 128 == 0, K >= 256, M >= 256,
 *   lda >= K, ldx >= W, both multiples of 8, x16 16-byte aligned.  Replaces
 *   openai/CLIP model.py ResidualAttentionBlock's "x = x + attn(...)" / "x = x + mlp(...)". */
int mi_op_gemm_residual(void* x16, int64_t ldx, const void* A, int64_t lda, const void* W, const float* bias,
                        float* ps, float* rs, int32_t M, int32_t Wd, int32_t K, void* stream);

/* MX-fp8 operator entry points (the "fp8 MFMA weights" configuration,
 * BASELINE.json configs[4]; OCP e4m3 elements with one e8m0 scale per 64
 * consecutive k of a row — the block the gfx950 16x16x128 block-scaled MFMA
 * applies, probed in scripts/probes/mx_scale_map.hip):
 * mi_op_quantize_mx: bf16 [rows][K] -> e4m3 q [rows][K] + e8m0 scales, stage-major
 *   [K/128][rows_pad][2] (rows_pad = rows rounded up to even; byte kb & 1 of
 *   row r in stage kb >> 1 scales k-block kb); K % 128 == 0
 * mi_op_gemm_mx: out = (A * 2^sA) . (W * 2^sW)^T (+bias) on the block-scaled MFMA,
 *   A [M][K] / W [N][K] e4m3 with their scales; epilogue 0 bf16, 1 bf16 QuickGELU, 3 f32,
 *   4 QuickGELU -> MX-fp8 (the c_fc -> c_proj hand-off: out holds the e4m3 [M][N] bytes and,
 *   from byte offset M*N rounded up to 256, their stage-major scales [N/128][M_pad][2]).
 *   Bits 8+ of epi select a kernel for A/B (0 default: the ping-pong 32x32x64 kernel; 1 the
 *   double-buffered 16x16x128 kernel; 8 the 8-phase persistent kernel, bit-identical to 1).
 *   K % 128 == 0, N % 256 == 0. */
int mi_op_quantize_mx(const void* in, void* q, void* scales, int32_t rows, int32_t K, void* stream);
int mi_op_gemm_mx(const void* A, const void* a_scale, const void* W, const void* w_scale, const float* bias, void* out,
                  int32_t M, int32_t N, int32_t K, int32_t epi, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MICLIP_H */
