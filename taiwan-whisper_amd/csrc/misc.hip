// HBM-bound helper kernels of the distillation step:
//   embedding gather (+learned positions) and its scatter-add backward (K7),
//   fp32->bf16 weight casts (autocast's per-forward weight cast), bias-grad column sums,
//   global grad L2 norm + fused clip/AdamW update (K11/K12, run_distillation.py:1666-1668),
//   conv-stem im2col / col2im for the conv backward (K2), teacher decoder-input shift
//   (HF shift_tokens_right, run_distillation.py:1534) and valid-label count.
#include "common.h"

namespace {

__global__ void embed_fwd_kernel(const int64_t* __restrict__ ids, const void* __restrict__ tok, int tok_dtype,
                                 const void* __restrict__ pos, int pos_dtype, void* __restrict__ out, int out_dtype,
                                 int rows, int T, int pos_offset, int D) {
  const int row = blockIdx.x;
  if (row >= rows) return;
  const int64_t id = ids[row];
  const int t = row % T + pos_offset;
  for (int e = threadIdx.x; e < D; e += blockDim.x) {
    const float a = ld_as_f32(tok, tok_dtype, id * D + e);
    const float b = ld_as_f32(pos, pos_dtype, (int64_t)t * D + e);
    const float s = a + b;
    st_from_f32(out, out_dtype, (int64_t)row * D + e, s);
  }
}

// H: fp16 words (fp16 autocast's weight cast), else bf16
template <bool H>
__global__ void cast_f32_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ dst, int64_t n) {
  int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (; i + 3 < n; i += stride) {
    f32x4 v = *(const f32x4*)(src + i);
    *(bf16x4*)(dst + i) = bf16x4{f2e<H>(v[0]), f2e<H>(v[1]), f2e<H>(v[2]), f2e<H>(v[3])};
  }
  for (; i < n; ++i) dst[i] = f2e<H>(src[i]);
}

// Column sums over rows (bias gradient of an autocast Linear, computed in bf16 then added to the
// fp32 grad).  Pass 1: block (CS_ROWS x 512 columns) -> partial[chunk][cols] with 8 columns per
// lane (16-B bf16 / 2x16-B fp32 loads); pass 2: deterministic sum over chunks (+round, +accumulate).
// 64-row chunks (round 6; were 256): c2's decoder bias gradients (14 304 rows x 768) ran on 112 blocks at 0.8 TB/s
// and the encoder's (48 000 rows) on 376 at 1.9 TB/s -- too few loads in flight for HBM.
constexpr int CS_COLS = 512, CS_ROWS = 64;
__global__ __launch_bounds__(256) void colsum_partial_kernel(const void* __restrict__ x, int x_dtype, int64_t ldx,
                                                             int rows, int cols, float* __restrict__ partial) {
  __shared__ float red[4][CS_COLS];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = blockIdx.x * CS_COLS + lane * 8;
  const int r0 = blockIdx.y * CS_ROWS;
  const int r1 = min(rows, r0 + CS_ROWS);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool vec = (c0 + 7 < cols) && ((ldx & 7) == 0);
#pragma unroll 4
  for (int r = r0 + wv; r < r1; r += 4) {
    const int64_t o = (int64_t)r * ldx + c0;
    if (vec) {
      if (x_dtype == TW_BF16) {
        const bf16x8 v = *(const bf16x8*)((const bf16*)x + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
      } else if (x_dtype == TW_F16) {
        float t[8];
        load8((const f16*)x + o, t);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += t[j];
      } else {
        const f32x4 a = *(const f32x4*)((const float*)x + o);
        const f32x4 b = *(const f32x4*)((const float*)x + o + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[j] += a[j]; acc[4 + j] += b[j]; }
      }
    } else {
      for (int j = 0; j < 8; ++j)
        if (c0 + j < cols) acc[j] += ld_as_f32(x, x_dtype, o + j);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[wv][lane * 8 + j] = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < CS_COLS; c += 256) {
    const int gc = blockIdx.x * CS_COLS + c;
    if (gc < cols) partial[(int64_t)blockIdx.y * cols + gc] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  }
}

// out[c] = [out[c] +] round?(sum_k partial[k][c]) (round 1: to bf16, 2: to fp16): 16 columns per block, 64 thread
// rows each summing every 64th chunk, fixed-order combine in LDS (deterministic)
__global__ __launch_bounds__(1024) void colsum_final_kernel(const float* __restrict__ partial, int nchunk, int cols,
                                                            float* __restrict__ out, int accum, int round_bf16) {
  __shared__ float st[64][16];
  const int cl = threadIdx.x & 15, j = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float t = 0.f;
  if (c < cols)
#pragma unroll 4
    for (int k = j; k < nchunk; k += 64) t += partial[(int64_t)k * cols + c];
  st[j][cl] = t;
  __syncthreads();
  if (j == 0 && c < cols) {
    for (int k = 1; k < 64; ++k) t += st[k][cl];
    if (round_bf16 == 2) t = rnd<true>(t);
    else if (round_bf16) t = rbf(t);
    out[c] = accum ? out[c] + t : t;
  }
}

// sum of squares of a fp32 vector -> partial[blockIdx.x]
__global__ void sumsq_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ partial) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    s += v * v;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ void finalize_norm_kernel(const float* __restrict__ partial, int nb, float* __restrict__ norm_out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 64) s += partial[i];
  s = wave_sum(s);
  if (threadIdx.x == 0) norm_out[0] = sqrtf(s);
}

// torch.optim.AdamW (foreach=False, non-capturable) with the clip_grad_norm_ factor fused:
//   g *= min(1, max_norm / (norm + 1e-6)); p *= 1 - lr*wd; m = lerp(m, g, 1-b1);
//   v = b2 v + (1-b2) g^2; p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps);  optional 16-bit copy of p (H: fp16).
// inv_scale (fp16 autocast's GradScaler.unscale_, a power of two): g and norm are the loss-scaled gradient and its
// norm; g * inv_scale is the unscaled gradient exactly, and so is norm * inv_scale its norm (1.0 otherwise).
template <bool H>
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, bf16* __restrict__ p_bf16, int64_t n, float lr, float b1, float b2,
                             float eps, float wd, float bc1, float bc2_sqrt, const float* __restrict__ norm,
                             float max_norm, float inv_scale) {
  float coef = 1.f;
  if (norm != nullptr && max_norm > 0.f) {
    coef = max_norm / (norm[0] * inv_scale + 1e-6f);
    coef = coef < 1.f ? coef : 1.f;
  }
  const float step_size = lr / bc1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = (g[i] * inv_scale) * coef;
    float pi = p[i];
    pi = pi * (1.f - lr * wd);
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);
    float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi; m[i] = mi; v[i] = vi;
    if (p_bf16) p_bf16[i] = f2e<H>(pi);
  }
}

__global__ void scale_kernel(float* __restrict__ x, int64_t n, const float* __restrict__ norm, float max_norm) {
  float coef = max_norm / (norm[0] + 1e-6f);
  if (coef >= 1.f) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] *= coef;
}

// dst[b*T_out + t][k*C + c] = src[b][t*stride + k][c]    (src rows per batch = src_rows)
__global__ void im2col_kernel(const bf16* __restrict__ src, int64_t src_rows, bf16* __restrict__ dst, int B, int T_out,
                              int stride, int C) {
  const int64_t row = blockIdx.x;    // b*T_out + t
  if (row >= (int64_t)B * T_out) return;
  const int b = row / T_out, t = row % T_out;
  for (int j = threadIdx.x; j < 3 * C; j += blockDim.x) {
    const int k = j / C, c = j % C;
    dst[row * 3 * C + j] = src[((int64_t)b * src_rows + (int64_t)t * stride + k) * C + c];
  }
}

// conv2 (k3, s2, p1) input-gradient: dX[b][s][c] = sum over (t,k) with 2t+k-1 = s of dA[b*T_out+t][k*C+c]
__global__ void col2im_s2_kernel(const float* __restrict__ dA, float* __restrict__ dX, int B, int T_in, int T_out,
                                 int C) {
  const int64_t row = blockIdx.x;    // b*T_in + s
  if (row >= (int64_t)B * T_in) return;
  const int b = row / T_in, s = row % T_in;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float acc = 0.f;
    if ((s & 1) == 0) {
      const int t = s / 2;
      acc = dA[((int64_t)b * T_out + t) * 3 * C + 1 * C + c];
    } else {
      const int t0 = (s + 1) / 2, t2 = (s - 1) / 2;
      if (t0 < T_out) acc += dA[((int64_t)b * T_out + t0) * 3 * C + 0 * C + c];
      acc += dA[((int64_t)b * T_out + t2) * 3 * C + 2 * C + c];
    }
    dX[row * C + c] = acc;
  }
}

// HF shift_tokens_right on device: out[b][0] = start; out[b][t] = labels[b][t-1] (-100 -> pad)
__global__ void shift_right_kernel(const int64_t* __restrict__ labels, int64_t* __restrict__ out, int B, int T,
                                   int64_t pad, int64_t start) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)B * T) return;
  const int t = i % T;
  int64_t v = t == 0 ? start : labels[i - 1];
  out[i] = v == -100 ? pad : v;
}

__global__ void count_valid_kernel(const int64_t* __restrict__ labels, int64_t n, int* __restrict__ out) {
  int c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    c += labels[i] >= 0 ? 1 : 0;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// mel [B][80][3000] f32 -> time-major 16-bit conv1 input [B][3002][80] with zero rows 0 and 3001 (E = bf16:
// the autocast cast of the Conv1d input; E = f16: run_eval.py:589 input_features.to(float16))
template <typename E>
__global__ void mel_to_conv_input_kernel(const float* __restrict__ mel, E* __restrict__ xt, int B, int nmel,
                                         int T) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)B * (T + 2) * nmel;
  if (i >= n) return;
  const int c = i % nmel;
  const int64_t r = i / nmel;
  const int b = r / (T + 2), tt = r % (T + 2);
  float v = 0.f;
  if (tt >= 1 && tt <= T) v = mel[((int64_t)b * nmel + c) * T + (tt - 1)];
  from_f32(xt[i], v);
}

// out = e( e(g) * gelu'(pre) )  — GELU backward on an autocast 16-bit activation (e = bf16, or fp16 for H)
template <bool H>
__global__ void gelu_bwd_kernel(const void* __restrict__ g, int g_dtype, const bf16* __restrict__ pre,
                                bf16* __restrict__ out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gv = rnd<H>(ld_as_f32(g, g_dtype, i));
    out[i] = f2e<H>(gv * gelu_grad_of<H>(e2f<H>(pre[i])));
  }
}

inline int nblocks(int64_t n, int bs, int cap = 4096) {
  int64_t b = (n + bs - 1) / bs;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" int tw_embed_fwd(const int64_t* ids, const void* tok, int tok_dtype, const void* pos, int pos_dtype,
                            void* out, int out_dtype, int rows, int T, int pos_offset, int D, hipStream_t stream) {
  if (rows <= 0) return TW_OK;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(rows), dim3(256), 0, stream, ids, tok, tok_dtype, pos, pos_dtype, out,
                     out_dtype, rows, T, pos_offset, D);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

namespace {

// dst[c][r] = src[r][c] for a [rows][cols] bf16 matrix: 64x64 tiles through LDS (16-B row reads, 2-B column
// writes coalesced per row of the tile; +2 pad per LDS row keeps the transposed reads conflict-light)
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ src, int64_t lds_, int rows,
                                                             int cols, bf16* __restrict__ dst, int64_t ldd, int vec) {
  __shared__ bf16 t[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tr = threadIdx.x >> 3, tc = (threadIdx.x & 7) * 8;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = tr + 32 * i;
    if (r0 + r < rows) {
      if (vec && c0 + tc + 8 <= cols) {
        const bf16x8 v = *(const bf16x8*)(src + (int64_t)(r0 + r) * lds_ + c0 + tc);
#pragma unroll
        for (int q = 0; q < 8; ++q) t[r][tc + q] = v[q];
      } else {
        for (int q = 0; q < 8; ++q)
          if (c0 + tc + q < cols) t[r][tc + q] = src[(int64_t)(r0 + r) * lds_ + c0 + tc + q];
      }
    }
  }
  __syncthreads();
  const int oc = threadIdx.x & 63, orow = threadIdx.x >> 6;
  for (int j = orow; j < 64; j += 4) {           // output row c0 + j holds source column c0 + j
    if (c0 + j < cols && r0 + oc < rows) dst[(int64_t)(c0 + j) * ldd + r0 + oc] = t[oc][j];
  }
}

}  // namespace

extern "C" int tw_transpose_bf16(const void* src, int64_t ld_src, int rows, int cols, void* dst, int64_t ld_dst,
                                 hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return TW_OK;
  const int vec = !(ld_src & 7) && !((uintptr_t)src & 15);     // 16-B row reads when aligned
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((cols + 63) / 64, (rows + 63) / 64), dim3(256), 0, stream,
                     (const bf16*)src, ld_src, rows, cols, (bf16*)dst, ld_dst, vec);
  TW_CHECK_LAUNCH();
  return TW_OK;
}


extern "C" int tw_cast_f32_bf16(const float* src, void* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(cast_f32_bf16_kernel<false>, dim3(nblocks(n / 4 + 1, 256)), dim3(256), 0, stream, src, (bf16*)dst,
                     n);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_cast_f32_f16(const float* src, void* dst, int64_t n, hipStream_t stream) {
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(cast_f32_bf16_kernel<true>, dim3(nblocks(n / 4 + 1, 256)), dim3(256), 0, stream, src, (bf16*)dst,
                     n);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// workspace >= ceil(rows/64) * cols floats
extern "C" int tw_colsum(const void* x, int x_dtype, int64_t ldx, int rows, int cols, float* out, int accum,
                         int round_bf16, float* workspace, int64_t workspace_floats, hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return TW_OK;
  const int nchunk = (rows + CS_ROWS - 1) / CS_ROWS;
  if (workspace_floats < (int64_t)nchunk * cols) return TW_EINVAL;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((cols + CS_COLS - 1) / CS_COLS, nchunk), dim3(256), 0, stream, x,
                     x_dtype, ldx, rows, cols, workspace);
  hipLaunchKernelGGL(colsum_final_kernel, dim3((cols + 15) / 16), dim3(1024), 0, stream, workspace, nchunk, cols, out,
                     accum, round_bf16);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// norm_out[0] = ||x||_2 ; workspace >= 1024 floats
extern "C" int tw_l2norm(const float* x, int64_t n, float* norm_out, float* workspace, hipStream_t stream) {
  const int nb = nblocks(n, 256, 1024);
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(256), 0, stream, x, n, workspace);
  hipLaunchKernelGGL(finalize_norm_kernel, dim3(1), dim3(64), 0, stream, workspace, nb, norm_out);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_adamw_ex(float* p, const float* g, float* m, float* v, void* p16, int p16_dtype, int64_t n, float lr,
                           float b1, float b2, float eps, float wd, int step, const float* norm, float max_norm,
                           float inv_scale, hipStream_t stream) {
  if (n <= 0) return TW_OK;
  if (step < 1 || !(inv_scale > 0.f)) return TW_EINVAL;
  if (p16 && p16_dtype != TW_BF16 && p16_dtype != TW_F16) return TW_EINVAL;
  const float bc1 = 1.f - powf(b1, (float)step);
  const float bc2 = 1.f - powf(b2, (float)step);
  if (p16 && p16_dtype == TW_F16)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(nblocks(n, 256, 8192)), dim3(256), 0, stream, p, g, m, v, (bf16*)p16, n,
                       lr, b1, b2, eps, wd, bc1, sqrtf(bc2), norm, max_norm, inv_scale);
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3(nblocks(n, 256, 8192)), dim3(256), 0, stream, p, g, m, v, (bf16*)p16,
                       n, lr, b1, b2, eps, wd, bc1, sqrtf(bc2), norm, max_norm, inv_scale);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_adamw(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float b1,
                        float b2, float eps, float wd, int step, const float* norm, float max_norm,
                        hipStream_t stream) {
  return tw_adamw_ex(p, g, m, v, p_bf16, TW_BF16, n, lr, b1, b2, eps, wd, step, norm, max_norm, 1.0f, stream);
}

extern "C" int tw_clip_scale(float* x, int64_t n, const float* norm, float max_norm, hipStream_t stream) {
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(scale_kernel, dim3(nblocks(n, 256, 8192)), dim3(256), 0, stream, x, n, norm, max_norm);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_im2col3(const void* src, int64_t src_rows, void* dst, int B, int T_out, int stride, int C,
                          hipStream_t stream) {
  if (B <= 0 || T_out <= 0) return TW_OK;
  hipLaunchKernelGGL(im2col_kernel, dim3((int64_t)B * T_out), dim3(256), 0, stream, (const bf16*)src, src_rows,
                     (bf16*)dst, B, T_out, stride, C);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_col2im_s2(const float* dA, float* dX, int B, int T_in, int T_out, int C, hipStream_t stream) {
  if (B <= 0) return TW_OK;
  hipLaunchKernelGGL(col2im_s2_kernel, dim3((int64_t)B * T_in), dim3(256), 0, stream, dA, dX, B, T_in, T_out, C);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_shift_tokens_right(const int64_t* labels, int64_t* out, int B, int T, int64_t pad, int64_t start,
                                     hipStream_t stream) {
  const int64_t n = (int64_t)B * T;
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(shift_right_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, labels, out, B, T, pad, start);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_count_valid(const int64_t* labels, int64_t n, int* out, hipStream_t stream) {
  if (hipMemsetAsync(out, 0, sizeof(int), stream) != hipSuccess) return TW_EHIP;
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(count_valid_kernel, dim3(nblocks(n, 256, 1024)), dim3(256), 0, stream, labels, n, out);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_mel_to_conv_input(const float* mel, void* xt, int B, int nmel, int T, hipStream_t stream) {
  const int64_t n = (int64_t)B * (T + 2) * nmel;
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(mel_to_conv_input_kernel<bf16>, dim3((n + 255) / 256), dim3(256), 0, stream, mel, (bf16*)xt, B,
                     nmel, T);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_mel_to_conv_input_f16(const float* mel, void* xt, int B, int nmel, int T, hipStream_t stream) {
  const int64_t n = (int64_t)B * (T + 2) * nmel;
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(mel_to_conv_input_kernel<f16>, dim3((n + 255) / 256), dim3(256), 0, stream, mel, (f16*)xt, B,
                     nmel, T);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_gelu_bwd(const void* g, int g_dtype, const void* pre, void* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(gelu_bwd_kernel<false>, dim3(nblocks(n, 256, 8192)), dim3(256), 0, stream, g, g_dtype,
                     (const bf16*)pre, (bf16*)out, n);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_gelu_bwd_f16(const void* g, int g_dtype, const void* pre, void* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(gelu_bwd_kernel<true>, dim3(nblocks(n, 256, 8192)), dim3(256), 0, stream, g, g_dtype,
                     (const bf16*)pre, (bf16*)out, n);
  TW_CHECK_LAUNCH();
  return TW_OK;
}
