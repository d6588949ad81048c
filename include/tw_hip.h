/*
 * tw_hip.h — C-ABI of libtw_hip.so, the MI355X (gfx950) kernels behind the taiwan-whisper
 * distillation hot path.
 *
 * The reference has no native plugin API: its hot path calls HF
 * Transformers / ATen / cuBLAS / SDPA / NCCL implicitly.  Each entry point below replaces
 * one of those implicit kernels and cites the reference line that triggers it.  The
 * Python host package (taiwan-whisper_amd/tw) binds these with ctypes; INTEGRATION.md shows
 * the binding a maintainer would add on the reference side.
 *
 * Conventions
 *   - plain device pointers, int64 leading dimensions in ELEMENTS, row-major;
 *   - dtype codes: 0 = fp32, 1 = bf16, 2 = fp16;
 *   - every call is stream-ordered on `stream` (a hipStream_t), never synchronises,
 *     never allocates; workspaces are caller-provided;
 *   - return 0 on success, 1 = invalid argument/shape, 2 = unsupported, 3 = HIP launch error;
 *   - the library holds no global mutable state; calls are reentrant.
 */
#ifndef TW_HIP_H
#define TW_HIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef void* tw_stream_t; /* hipStream_t */

/* GEMM flags */
#define TW_GEMM_BIAS 1
#define TW_GEMM_ROUND 2
#define TW_GEMM_GELU 4
#define TW_GEMM_RES 8
#define TW_GEMM_ACCUM 16
#define TW_GEMM_AUX_OUT 32
#define TW_GEMM_DGELU 64
#define TW_GEMM_TILE128 256   /* force the 128x128 tile (A/B benchmarking) */
#define TW_GEMM_TILE256 512   /* force the 256x256 tile */
#define TW_GEMM_TILE256x128 1024  /* force the 256x128 tile with the 3-stage LDS ring */
#define TW_GEMM_TILE256PP 2048    /* force the 256x256 ping-pong kernel (a_trans = b_trans = 0 only) */


/* bf16 MFMA GEMM  C[b] = epi(alpha * A[b] . B[b]^T), A [M][K] (a_trans: [K][M]), B [N][K] (b_trans: [K][N]).
 * Replaces every nn.Linear / Conv1d (as GEMM) / tied proj_out matmul of the step, forward and
 * backward: HF modeling_whisper.py:279-345 (q/k/v/out_proj), :618-619 (conv1/conv2), :400-410 and
 * :495-505 (fc1 + GELU + fc2), :1080 (proj_out); run_distillation.py:1528,1534,1665 (fwd, teacher fwd, backward).
 * Epilogue order: +bias[n] (bf16) -> ROUND to bf16 -> DGELU (x gelu'(aux)) -> GELU (aux <- pre-act)
 *   -> +res[m % res_mod][n] -> +C_old (ACCUM) -> store as c_dtype.  K % 8 == 0 unless both operands are MN-major; a_trans needs M % 8 == 0,
 *   b_trans needs N % 8 == 0; lda, ldb % 8 == 0; A, B 16-byte aligned. */
int tw_gemm_bf16(const void* A, int64_t lda, int a_trans, const void* B, int64_t ldb, int b_trans, void* C,
                 int64_t ldc, int c_dtype, int M, int N, int K, int batch, int64_t sA, int64_t sB, int64_t sC,
                 float alpha, const void* bias, const void* res, int64_t ldr, int64_t sR, int res_dtype, int res_mod,
                 void* aux, int64_t ldaux, int64_t sAux, int flags, tw_stream_t stream);

/* Decode-step Linear for up to 4 rows (batch-1 long-form): C = epi(A . W^T), one output column per wave.
 * A = x [M][K] bf16, or LayerNorm(x) when ln_w != NULL (fp32 gamma ln_w / beta ln_b, eps; K % 256 == 0;
 * A is bit-identical to tw_layernorm_fwd's bf16 output, so an LN launch + GEMM pair becomes one launch).
 * Replaces, per decode step, HF WhisperDecoderLayer's LayerNorm + nn.Linear pairs and the plain Linears
 * (modeling_whisper.py:448-506) for a batch of <= 4.  W [N][K] bf16; flags / bias / res / aux as
 * tw_gemm_bf16 (F_BIAS, F_ROUND, F_GELU, F_RES, F_AUX_OUT, F_ACCUM); C fp32 or bf16.  kv_cache != NULL fuses
 * tw_kv_append: columns n >= kv_col0 are also stored at kv_cache[m*kv_sb + (*t_dev)*kv_ld + n - kv_col0]
 * (the self-attention K/V row of the step, the fused QKV projection's k | v part). */
int tw_gemv_bf16(const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps, const void* W,
                 int64_t ldw, void* C, int64_t ldc, int c_dtype, int M, int N, int K, const void* bias,
                 const void* res, int64_t ldr, int res_dtype, void* aux, int64_t ldaux, int flags,
                 void* kv_cache, int64_t kv_sb, int64_t kv_ld, int kv_col0, const int* t_dev, tw_stream_t stream);

/* LayerNorm fp32-statistics forward / backward (D % 64 == 0, D <= 1280).
 * Replaces nn.LayerNorm at HF modeling_whisper.py:392,402,470,485,498,642,790 (autocast fp32 op). */
int tw_layernorm_fwd(const void* x, int x_dtype, const float* w, const float* b, void* y, int y_dtype,
                     float* mean_out, float* rstd_out, int rows, int D, float eps, tw_stream_t stream);
/* Residual add fused into the LayerNorm that follows it (D % 256 == 0, 16-B aligned rows): x_out = x + r
 * (r = the preceding Linear's bf16 output: the HF residual `hidden_states = residual + hidden_states` at
 * modeling_whisper.py:399,412 / 479,495,506; fp32 stream x_dtype 0 under autocast, bf16 stream x_dtype 1
 * rounded once), y = bf16 LayerNorm(x_out).  x_out may alias x.  Bit-identical to tw_gemm_bf16's residual
 * epilogue followed by tw_layernorm_fwd. */
int tw_add_layernorm_fwd(const void* x, int x_dtype, const void* r, void* x_out, const float* w, const float* b,
                         void* y, float* mean_out, float* rstd_out, int rows, int D, float eps, tw_stream_t stream);
int tw_layernorm_bwd(const void* x, int x_dtype, const float* w, const float* mean, const float* rstd, const void* dy,
                     int dy_dtype, float* dx, int dx_accum, float* dw_out, float* db_out, int rows, int D,
                     float* workspace, int64_t workspace_floats, tw_stream_t stream);
/* tw_layernorm_bwd_ex: tw_layernorm_bwd that also writes g16 = the bf16 (g_dtype 1) / fp16 (2) rounding of the final dx
 * (the autocast cast of the stream gradient the preceding block's GEMMs read; g16 may be NULL). */
int tw_layernorm_bwd_ex(const void* x, int x_dtype, const float* w, const float* mean, const float* rstd, const void* dy,
                        int dy_dtype, float* dx, int dx_accum, float* dw_out, float* db_out, int rows, int D,
                        float* workspace, int64_t workspace_floats, void* g16, int g_dtype, tw_stream_t stream);

/* Flash attention, head_dim 64, bf16 (replaces SDPA at HF modeling_whisper.py:337-350 for encoder
 * self-attn, decoder causal self-attn and cross-attn).  lse: [B][H][Tq] fp32 (natural log). */
int tw_attn_fwd(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv, void* O,
                int64_t ldo, float* lse, int B, int H, int Tq, int Tk, int head_dim, int causal, float scale,
                tw_stream_t stream);
int tw_attn_bwd(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv, const void* O,
                int64_t ldo, const void* dO, int64_t lddo, const float* lse, void* dQ, int64_t lddq, void* dK,
                int64_t lddk, void* dV, int64_t lddv, int B, int H, int Tq, int Tk, int head_dim, int causal,
                float scale, float* workspace /* B*H*Tq floats */, tw_stream_t stream);

/* Fused CE + temperature KL loss and its logits gradient (replaces run_distillation.py:1507-1516,
 * :1539-1549 and HF CE :1082-1087).  out3 = [loss, ce, kl*T^2]; dlogits (same dtype as the logits:
 * bf16 under autocast, fp32 on the fp32 path) may be NULL, or s_logits itself (the gradient written in place). */
int tw_kl_ce(const void* s_logits, const void* t_logits, int64_t ld, int logits_dtype, const int64_t* labels,
             int64_t rows, int V, float T, float ce_w, float kl_w, const int* n_valid, float grad_scale, float* row_out,
             float* out3, void* dlogits, tw_stream_t stream);

/* Whisper log-mel (replaces WhisperFeatureExtractor at run_distillation.py:1217).
 * wav [B][480000] fp32 -> mel_out [B][80][3000] fp32 and optional conv1 input [B][3002][80] bf16. */
int tw_logmel(const float* wav, int B, const float* basis, const int* mel_start, const float* mel_w, float* mel_out,
              void* conv_in, void* workspace /* B uint32 */, tw_stream_t stream);
/* Same front end over clips of any length (long-form inputs: HF __call__(truncation=False,
 * padding="longest"), run_eval.py:572-581): wav [B][n_samples] fp32 (shorter clips zero-padded to the
 * longest, as HF pads) -> mel_out [B][80][n_samples/160], conv_in [B][n_samples/160 + 2][80] bf16.
 * n_samples must exceed 200 (the reflect pad).  tw_logmel == tw_logmel_len(n_samples = 480000). */
int tw_logmel_len(const float* wav, int B, int64_t n_samples, const float* basis, const int* mel_start,
                  const float* mel_w, float* mel_out, void* conv_in, void* workspace, tw_stream_t stream);
int tw_mel_to_conv_input(const float* mel, void* xt, int B, int nmel, int T, tw_stream_t stream);

/* Decoder token + learned position embedding (HF modeling_whisper.py:736,754-761) and its
 * backward into the tied embedding gradient: deterministic (rows of one id summed in position order,
 * one writer per id); positions whose id == padding_idx add nothing (nn.Embedding's padding_idx,
 * = config.pad_token_id in HF WhisperDecoder; -1: none).  Scratch: the per-device block. */
int tw_embed_fwd(const int64_t* ids, const void* tok, int tok_dtype, const void* pos, int pos_dtype, void* out,
                 int out_dtype, int rows, int T, int pos_offset, int D, tw_stream_t stream);
int tw_embed_bwd(const int64_t* ids, const float* dh, float* dE, int rows, int D, int64_t padding_idx,
                 tw_stream_t stream);

/* dst[c][r] = src[r][c], bf16 [rows][cols] (row stride ld_src) -> [cols][rows] (ld_dst): the tied
 * embedding as the K-major operand of the LM-head input gradient (dh = dlogits . E, K = vocabulary). */
int tw_transpose_bf16(const void* src, int64_t ld_src, int rows, int cols, void* dst, int64_t ld_dst,
                      tw_stream_t stream);
/* autocast weight cast fp32 -> bf16 (ACC:accelerator.py autocast of every Linear weight). */
int tw_cast_f32_bf16(const float* src, void* dst, int64_t n, tw_stream_t stream);
/* bias gradient: out[c] (+)= [round](sum_r x[r][c]) (round_bf16: 0 none, 1 to bf16, 2 to fp16; x fp32 / bf16 / fp16);
 * deterministic two-pass, workspace >= ceil(rows/64)*cols. */
int tw_colsum(const void* x, int x_dtype, int64_t ldx, int rows, int cols, float* out, int accum, int round_bf16,
              float* workspace, int64_t workspace_floats, tw_stream_t stream);

/* clip_grad_norm_ + AdamW (run_distillation.py:1450-1455,1666-1668). */
int tw_l2norm(const float* x, int64_t n, float* norm_out, float* workspace /* 1024 floats */, tw_stream_t stream);
int tw_adamw(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float b1, float b2,
             float eps, float wd, int step, const float* norm, float max_norm, tw_stream_t stream);
int tw_clip_scale(float* x, int64_t n, const float* norm, float max_norm, tw_stream_t stream);

/* conv-stem backward helpers (HF modeling_whisper.py:618-619). */
int tw_im2col3(const void* src, int64_t src_rows, void* dst, int B, int T_out, int stride, int C,
               tw_stream_t stream);
int tw_col2im_s2(const float* dA, float* dX, int B, int T_in, int T_out, int C, tw_stream_t stream);
/* GELU backward on a bf16 activation: out = bf16(bf16(g) * gelu'(pre)). */
int tw_gelu_bwd(const void* g, int g_dtype, const void* pre, void* out, int64_t n, tw_stream_t stream);

/* teacher decoder input = shift_tokens_right(labels) (run_distillation.py:1534, HF modeling_whisper.py:68-81);
 * number of labels >= 0 (kl_divergence normaliser, run_distillation.py:1512-1515). */
int tw_shift_tokens_right(const int64_t* labels, int64_t* out, int B, int T, int64_t pad, int64_t start,
                          tw_stream_t stream);
int tw_count_valid(const int64_t* labels, int64_t n, int* out, tw_stream_t stream);

/* Greedy decoding with a KV cache (generate_step run_distillation.py:1580-1584,
 * run_pseudo_labelling.py:917-922; HF generation_whisper.py greedy loop, per-step attention of
 * modeling_whisper.py:265-350 with past_key_values).
 * Position-independent steps (for graph capture): the step index t lives in device memory
 * (t_dev) and is read by the kernels that depend on it; tw_step_advance adds `by` to it.
 * tw_decode_attn: one query row per (batch b, head h): O[b][h*64..] = softmax(scale * q.K^T) V over
 * the first Tk key rows (Tk += *tk_dev when tk_dev != NULL); q at q + b*sqb + h*64, key j at
 * k + b*skb + j*ldk + h*64 (v alike), output at o + b*sob + h*64 (bf16).  head_dim 64, Tk <= 2048.
 * tw_greedy_select: HF SuppressTokens / SuppressTokensAtBegin (logits_process.py) + argmax
 * (lowest id on ties) over the first V logits of each bf16 row; suppress_bits / begin_bits are
 * V-bit masks; rows with done[b] != 0 emit eos; the token is written to ids[b*ld_ids + col] and
 * next_ids[b], and done[b] |= (token == eos).  With t_dev != NULL: col += *t_dev and the begin mask
 * applies when col == begin_col (apply_begin is ignored).
 * tw_embed_step: out[b] = tok[ids[b]] + pos[*t_dev] (decoder input embedding of one step).
 * tw_kv_append: cache[b*sb + (*t_dev)*ld_row + 0..n) = src[b*ld_src + 0..n) (16-B vectors: bf16 n % 8 == 0,
 * fp32 n % 4 == 0).
 * dtype / logits_dtype (0 = fp32, 1 = bf16) select the element type of q/K/V/O and of the logits rows:
 * bf16 under autocast, fp32 on the fp32 path (mixed_precision "no"). */
int tw_decode_attn(const void* q, int64_t sqb, const void* k, int64_t ldk, int64_t skb, const void* v, int64_t ldv,
                   int64_t svb, void* o, int64_t sob, int B, int H, int Tk, const int* tk_dev, int head_dim,
                   float scale, int dtype, tw_stream_t stream);
/* tw_decode_attn_hs: tw_decode_attn with head strides for K and V -- key j of head h at k + b*skb + h*hsk + j*ldk
 * (v alike; tw_decode_attn is hsk = hsv = 64).  The head-major cross-attention K/V ([H][Tk][64] per clip:
 * hsk = Tk*64, ldk = 64) of ONE clip serve every row of a batch with skb = svb = 0 (the temperature-fallback batch
 * of one window: HF generate_with_fallback, generation_whisper.py; each row reads exactly the K/V of its batch-1
 * decode). */
int tw_decode_attn_hs(const void* q, int64_t sqb, const void* k, int64_t ldk, int64_t skb, int64_t hsk,
                      const void* v, int64_t ldv, int64_t svb, int64_t hsv, void* o, int64_t sob, int B, int H, int Tk,
                      const int* tk_dev, int head_dim, float scale, int dtype, tw_stream_t stream);
int tw_greedy_select(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                     const uint32_t* begin_bits, int apply_begin, int64_t eos, uint8_t* done, int64_t* ids,
                     int64_t ld_ids, int col, int64_t* next_ids, const int* t_dev, int begin_col, tw_stream_t stream);
/* tw_greedy_select_ts: as tw_greedy_select plus HF WhisperTimeStampLogitsProcessor (applied after the
 * suppress masks): <|notimestamps|> (no_ts) masked, pair / monotonicity rules from the previous two
 * generated tokens (columns >= begin_col of ids) and last_ts[b] (the row's last emitted timestamp,
 * -1 = none; updated here), the window's first step limited to timestamps <= ts_begin + max_initial
 * (max_initial < 0: no limit), and timestamps forced when logsumexp over them exceeds the best text
 * logit.  col += *t_dev when t_dev != NULL. */
int tw_greedy_select_ts(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                        const uint32_t* begin_bits, int64_t eos, uint8_t* done, int64_t* ids, int64_t ld_ids, int col,
                        int64_t* next_ids, const int* t_dev, int begin_col, int ts_begin, int no_ts, int max_initial,
                        int* last_ts, tw_stream_t stream);
/* Temperature fallback (HF generate_with_fallback, generation_whisper.py:970-1090; _need_fallback :1243-1290;
 * _retrieve_avg_logprobs :1958-1975; WhisperNoSpeechDetection logits_process.py:2050-2112).
 * tw_select_sample[_ts]: tw_greedy_select[_ts] with ctl = device int32[3] {bits of 1/T, seed lo, seed hi}
 * (1/T == 0: argmax; else Gumbel-max sampling over the processed row, i.e. multinomial(softmax(x/T)) with
 * a counter-based hash RNG keyed by (seed, b, col, id) -- not torch's RNG stream) and, when sum_logp !=
 * NULL, sum_logp[b] += log_softmax(processed row)[chosen] for rows not yet finished (the eos step
 * included).  B, V < 2^21.
 * tw_token_logprob: out[b] = log_softmax(logits[b*ld + 0..V))[token] (the no-speech probability is
 * exp(out) at the <|startoftranscript|> position). */
int tw_select_sample(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                     const uint32_t* begin_bits, int apply_begin, int64_t eos, uint8_t* done, int64_t* ids,
                     int64_t ld_ids, int col, int64_t* next_ids, const int* t_dev, int begin_col, const uint32_t* ctl,
                     float* sum_logp, tw_stream_t stream);
int tw_select_sample_ts(const void* logits, int64_t ld, int logits_dtype, int B, int V, const uint32_t* suppress_bits,
                        const uint32_t* begin_bits, int64_t eos, uint8_t* done, int64_t* ids, int64_t ld_ids, int col,
                        int64_t* next_ids, const int* t_dev, int begin_col, int ts_begin, int no_ts, int max_initial,
                        int* last_ts, const uint32_t* ctl, float* sum_logp, tw_stream_t stream);
int tw_token_logprob(const void* logits, int64_t ld, int logits_dtype, int B, int V, int token, float* out,
                     tw_stream_t stream);
int tw_embed_step(const int64_t* ids, const void* tok, int tok_dtype, const void* pos, int pos_dtype, void* out,
                  int out_dtype, int B, int D, const int* t_dev, tw_stream_t stream);
/* tw_kv_head_major: the cross-attention K/V as the KV projection writes it (rows b*Tk + t of [B*Tk][ld], k at
 * columns 0..64H, v at 64H..128H) -> dst = K [B][H][Tk][64] followed by V [B][H][Tk][64], so tw_decode_attn reads
 * each (clip, head) as two contiguous runs (called as B*H one-head clips: ldk = 64, skb = Tk*64).  Replaces the
 * layout of HF's cross-attention past_key_values ([B][H][Tk][64], modeling_whisper.py WhisperAttention).  dtype bf16
 * or f32; ld a multiple of 16 B. */
int tw_kv_head_major(const void* src, int64_t ld, void* dst, int B, int Tk, int H, int dtype, tw_stream_t stream);
int tw_kv_append(const void* src, int64_t ld_src, void* cache, int64_t ld_row, int64_t sb, int B, int n, int dtype,
                 const int* t_dev, tw_stream_t stream);
int tw_step_advance(int* t_dev, int by, tw_stream_t stream);

/* ---- fp32 arithmetic path (mixed_precision = "no", run_distillation.py:815-823: the reference's default
 * --dtype float32; the fp32 greedy decode pinned token-for-token to HF fp32 generate).  Exact-fp32 MFMA
 * (v_mfma_f32_16x16x4_f32), nothing rounded to bf16.
 * tw_gemm_f32: C[b] = epi(alpha * op(A[b]) op(B[b])^T) with the tw_gemm_bf16 operand conventions
 *   (A [M][K], a_trans: [K][M]; B [N][K], b_trans: [K][N]) and flags BIAS / GELU (+AUX_OUT) / DGELU / RES /
 *   ACCUM (ROUND and the tile flags are ignored); bias / res / aux fp32; two batch levels: batch entries
 *   bz = bo * batch_inner + bi at offsets bo*s? + bi*s?_in.  lda, ldb % 4 == 0, A and B 16-B aligned.
 * tw_attn_fwd_f32 / tw_attn_bwd_f32: SDPA over (B, H) with head_dim 64 and the tw_attn_* layouts, composed
 *   from tw_gemm_f32 products and exact row softmax kernels over a caller workspace (fwd >= Tq*round4(Tk)
 *   floats, bwd twice that; larger workspaces take more (b, h) pairs per pass).  lse [B][H][Tq] (natural log).
 * tw_mel_to_conv_input_f32 / tw_im2col3_f32 / tw_gelu_bwd_f32: the conv-stem helpers in fp32. */
int tw_gemm_f32(const float* A, int64_t lda, int a_trans, const float* B, int64_t ldb, int b_trans, float* C,
                int64_t ldc, int M, int N, int K, int batch, int64_t sA, int64_t sB, int64_t sC, int batch_inner,
                int64_t sA_in, int64_t sB_in, int64_t sC_in, float alpha, const float* bias, const float* res,
                int64_t ldr, int64_t sR, int res_mod, float* aux, int64_t ldaux, int64_t sAux, int flags,
                tw_stream_t stream);
int tw_attn_fwd_f32(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv, float* O,
                    int64_t ldo, float* lse, int B, int H, int Tq, int Tk, int head_dim, int causal, float scale,
                    float* workspace, int64_t workspace_floats, tw_stream_t stream);
int tw_attn_bwd_f32(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv,
                    const float* O, int64_t ldo, const float* dO, int64_t lddo, const float* lse, float* dQ,
                    int64_t lddq, float* dK, int64_t lddk, float* dV, int64_t lddv, int B, int H, int Tq, int Tk,
                    int head_dim, int causal, float scale, float* workspace, int64_t workspace_floats,
                    tw_stream_t stream);
int tw_mel_to_conv_input_f32(const float* mel, float* xt, int B, int nmel, int T, tw_stream_t stream);
int tw_im2col3_f32(const float* src, int64_t src_rows, float* dst, int B, int T_out, int stride, int C,
                   tw_stream_t stream);
int tw_gelu_bwd_f32(const float* g, const float* pre, float* out, int64_t n, tw_stream_t stream);

/* ---- fp16 arithmetic path: a torch_dtype=float16 model without autocast, the arithmetic of the reference's fp16
 * decode call sites (training/run_eval.py:99 `--dtype float16` default, :500-509 `model.to(dtype)`, :589
 * `input_features.to(dtype)`; training/run_pseudo_labelling.py:461-463 under run-pseudo-labelling.sh:30):
 * v_mfma_f32_16x16x32_f16 with fp32 accumulation, every 16-bit operand / output IEEE fp16 (RNE).
 * tw_gemm_f16: tw_gemm_bf16 for fp16 operands (the decode path uses the forward products only);
 *   A, B, bias, aux fp16; C and res fp16 (code 2) or fp32; epilogue order as tw_gemm_bf16 with the rounding
 *   to fp16, plus TW_GEMM_CLAMP16: after the residual add, clamp to +-(65504 - 1000) (HF WhisperEncoderLayer,
 *   modeling_whisper.py:409-411, the fp16 encoder stream).
 * tw_gemv_f16: tw_gemv_bf16 for fp16 x / W / bias / C (LayerNorm fused as there, fp16 output of the LN).
 * tw_attn_fwd_f16: tw_attn_fwd for fp16 Q/K/V/O (P rounded to fp16 for the PV product, fp32 row sums).
 * tw_mel_to_conv_input_f16: log-mel [B][80][T] fp32 -> fp16 conv1 input [B][T+2][80] (the .to(float16) cast).
 * fp16-AUTOCAST TRAINING (run_distillation.py:815-817 --dtype float16: mixed_precision="fp16", fp16 teacher,
 * GradScaler; round 6) uses the same entries plus:
 *   tw_gemm_f16 with a_trans / b_trans (the dX and dW products; split-K dW rounds its fp32 chunk sum to fp16);
 *   tw_attn_bwd_f16: tw_attn_bwd for fp16 tensors; tw_gelu_bwd_f16: tw_gelu_bwd for an fp16 activation;
 *   tw_cast_f32_f16: autocast's fp32 -> fp16 weight cast; tw_colsum with round_bf16 = 2;
 *   tw_adamw_ex: tw_adamw with the 16-bit weight copy in p16_dtype (1 bf16, 2 fp16) and GradScaler.unscale_
 *   folded in: g and norm are the loss-scaled gradient and its norm, inv_scale = 1 / scale (a power of two,
 *   so g * inv_scale is exact); tw_adamw(...) == tw_adamw_ex(..., TW bf16, ..., inv_scale = 1).
 * The dtype-coded entries above (tw_layernorm_fwd, tw_embed_fwd / tw_embed_step, tw_decode_attn, the selection
 * kernels, tw_token_logprob, tw_kv_append, tw_kv_head_major, tw_kl_ce) take code 2 for fp16 rows. */
#define TW_GEMM_CLAMP16 128
int tw_gemm_f16(const void* A, int64_t lda, int a_trans, const void* B, int64_t ldb, int b_trans, void* C,
                int64_t ldc, int c_dtype, int M, int N, int K, int batch, int64_t sA, int64_t sB, int64_t sC,
                float alpha, const void* bias, const void* res, int64_t ldr, int64_t sR, int res_dtype, int res_mod,
                void* aux, int64_t ldaux, int64_t sAux, int flags, tw_stream_t stream);
int tw_gemv_f16(const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps, const void* W,
                int64_t ldw, void* C, int64_t ldc, int c_dtype, int M, int N, int K, const void* bias,
                const void* res, int64_t ldr, int res_dtype, void* aux, int64_t ldaux, int flags,
                void* kv_cache, int64_t kv_sb, int64_t kv_ld, int kv_col0, const int* t_dev, tw_stream_t stream);
int tw_attn_fwd_f16(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv, void* O,
                    int64_t ldo, float* lse, int B, int H, int Tq, int Tk, int head_dim, int causal, float scale,
                    tw_stream_t stream);
int tw_mel_to_conv_input_f16(const float* mel, void* xt, int B, int nmel, int T, tw_stream_t stream);
int tw_attn_bwd_f16(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv, const void* O,
                    int64_t ldo, const void* dO, int64_t lddo, const float* lse, void* dQ, int64_t lddq, void* dK,
                    int64_t lddk, void* dV, int64_t lddv, int B, int H, int Tq, int Tk, int head_dim, int causal,
                    float scale, float* workspace, tw_stream_t stream);
int tw_gelu_bwd_f16(const void* g, int g_dtype, const void* pre, void* out, int64_t n, tw_stream_t stream);
int tw_cast_f32_f16(const float* src, void* dst, int64_t n, tw_stream_t stream);
/* tw_add_layernorm_fwd_f16: tw_add_layernorm_fwd on the fp32 stream of fp16 autocast: r and y fp16 (x fp32 only) */
int tw_add_layernorm_fwd_f16(const void* x, int x_dtype, const void* r, void* x_out, const float* w, const float* b,
                             void* y, float* mean_out, float* rstd_out, int rows, int D, float eps, tw_stream_t stream);
int tw_adamw_ex(float* p, const float* g, float* m, float* v, void* p16, int p16_dtype, int64_t n, float lr, float b1,
                float b2, float eps, float wd, int step, const float* norm, float max_norm, float inv_scale,
                tw_stream_t stream);

/* ---- host code: FLAC decoding for the data feed (replaces soundfile / libsndfile's sf.read of the
 * reference corpus, dataset/cool_dataset.py:55).  `data` is the whole file in host memory.
 * tw_flac_info: info[4] = {channels, sample_rate, bits_per_sample, total samples per channel (0 = unknown)}.
 * tw_flac_decode: interleaved int32 samples into out[cap] (out == NULL: count only), *frames = samples per
 * channel; every frame's CRC-8 header and CRC-16 footer is checked (1 = malformed stream). */
int tw_flac_info(const uint8_t* data, int64_t n, int64_t* info);
int tw_flac_decode(const uint8_t* data, int64_t n, int32_t* out, int64_t cap, int64_t* frames);

#ifdef __cplusplus
}
#endif
#endif /* TW_HIP_H */
