// LayerNorm forward/backward.  Rows of D elements, one wave per row,
// fp32 statistics (autocast runs layer_norm in fp32: HF modeling_whisper.py:392,402,470,
// 485,498,642,790).  Input fp32 (student residual stream) or bf16 (teacher stream);
// output bf16 (feeds the next bf16 GEMM) or fp32.
#include "common.h"

#include <algorithm>

namespace {

constexpr int WPB = 4;   // waves (rows) per block

// ADD (fp32 x, VEC 4 only): the residual update of the preceding Linear fused in front of the
// statistics -- x_out = x + r (r = the Linear's bf16 output, the same fp32 add the GEMM's residual
// epilogue performs, so x_out is bit-identical), then the LayerNorm of x_out.  This moves the fp32
// residual read + write out of the GEMM epilogue, where every CU of the persistent kernel issues it
// at once between two tiles, into this streaming pass.
// RH: r holds fp16 words (the fp16-autocast Linear output), else bf16
template <int VEC, int MAXJ, bool ADD = false, bool RH = false>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const void* __restrict__ x, int x_dtype,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     void* __restrict__ y, int y_dtype, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int rows, int D, float eps,
                                                     const bf16* __restrict__ r = nullptr, float* x_out = nullptr) {
  const int lane = lane_id();
  const int row = blockIdx.x * WPB + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int J = D / (64 * VEC);
  const int64_t base = (int64_t)row * D;
  float v[MAXJ][VEC];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (j < J) {
      const int e = (j * 64 + lane) * VEC;
      if constexpr (ADD) {
        const f32x4 t = *(const f32x4*)((const float*)x + base + e);
        const bf16x4 u = *(const bf16x4*)(r + base + e);
        const f32x4 o = f32x4{t[0] + e2f<RH>(u[0]), t[1] + e2f<RH>(u[1]), t[2] + e2f<RH>(u[2]), t[3] + e2f<RH>(u[3])};
        *(f32x4*)(x_out + base + e) = o;
        v[j][0] = o[0]; v[j][1] = o[1]; v[j][2] = o[2]; v[j][3] = o[3];
      } else if (VEC == 4) {
        if (x_dtype == TW_F32) {
          f32x4 t = *(const f32x4*)((const float*)x + base + e);
          v[j][0] = t[0]; v[j][1] = t[1]; v[j][2] = t[2]; v[j][3] = t[3];
        } else if (x_dtype == TW_BF16) {
          bf16x4 t = *(const bf16x4*)((const bf16*)x + base + e);
          v[j][0] = bf2f(t[0]); v[j][1] = bf2f(t[1]); v[j][2] = bf2f(t[2]); v[j][3] = bf2f(t[3]);
        } else {
          f16x4 t = *(const f16x4*)((const f16*)x + base + e);
          v[j][0] = (float)t[0]; v[j][1] = (float)t[1]; v[j][2] = (float)t[2]; v[j][3] = (float)t[3];
        }
      } else {
        v[j][0] = ld_as_f32(x, x_dtype, base + e);
      }
#pragma unroll
      for (int q = 0; q < VEC; ++q) s += v[j][q];
    }
  }
  const float mean = wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
    if (j < J)
#pragma unroll
      for (int q = 0; q < VEC; ++q) { const float d = v[j][q] - mean; ss += d * d; }
  const float rstd = rsqrtf(wave_sum(ss) / D + eps);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    if (j < J) {
      const int e = (j * 64 + lane) * VEC;
      float o[VEC];
#pragma unroll
      for (int q = 0; q < VEC; ++q) o[q] = (v[j][q] - mean) * rstd * w[e + q] + b[e + q];
      if (y_dtype == TW_BF16) {
        if (VEC == 4) *(bf16x4*)((bf16*)y + base + e) = bf16x4{f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
        else ((bf16*)y)[base + e] = f2bf(o[0]);
      } else if (y_dtype == TW_F16) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) ((f16*)y)[base + e + q] = (_Float16)o[q];
      } else {
        if (VEC == 4) *(f32x4*)((float*)y + base + e) = f32x4{o[0], o[1], o[2], o[3]};
        else ((float*)y)[base + e] = o[0];
      }
    }
  }
}

// bf16 -> bf16 rows with D % 256 == 0 (the teacher's bf16 residual stream): a half-wave per row
// (8 rows per 256-thread block), NCH chunks of 8 bf16 per lane as 16-B loads / stores, statistics
// reduced over the 32 lanes of the half (same two-pass mean / variance as ln_fwd_kernel).
// ADD: x_out = bf16(x + r) first (the bf16 stream's residual update, the same fp32 add + one round as the
// GEMM's residual epilogue), then the LayerNorm of x_out.
// H: the rows hold fp16 words (the fp16 stream of a torch_dtype=float16 model), else bf16
template <int NCH, bool ADD = false, bool H = false>
__global__ __launch_bounds__(256) void ln_fwd_bf16_kernel(const bf16* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, bf16* __restrict__ y,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                          int rows, int D, float eps, const bf16* __restrict__ r = nullptr,
                                                          bf16* x_out = nullptr) {
  // gamma / beta staged once per block in LDS (8 rows share them), so the output pass has no global loads
  __shared__ f32x4 sw[NCH * 64], sb[NCH * 64];
  const int lane = lane_id(), hl = lane & 31;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool ok = row < rows;
  // a tail half-wave reads the last row (in range) unconditionally and stores nothing: every load of the
  // row is issued before the first wait (no per-chunk branch + vmcnt(0) round trip)
  const int64_t base = (int64_t)(ok ? row : rows - 1) * D;
  constexpr int KS = (NCH * 64 + 255) / 256;
  int ix[KS];
  f32x4 gw[KS], gb[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {  // gamma / beta loads first: waiting on them does not wait on the rows
    ix[k] = min((int)threadIdx.x + k * 256, NCH * 64 - 1);
    gw[k] = ((const f32x4*)w)[ix[k]];
    gb[k] = ((const f32x4*)b)[ix[k]];
  }
  bf16x8 t[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) t[c] = *(const bf16x8*)(x + base + (c * 32 + hl) * 8);
  if constexpr (ADD) {
    bf16x8 u[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) u[c] = *(const bf16x8*)(r + base + (c * 32 + hl) * 8);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
      for (int q = 0; q < 8; ++q) t[c][q] = f2e<H>(e2f<H>(t[c][q]) + e2f<H>(u[c][q]));
  }
#pragma unroll
  for (int k = 0; k < KS; ++k) {  // stage (the loads were issued first; a clamped index rewrites the same value)
    sw[ix[k]] = gw[k];
    sb[ix[k]] = gb[k];
  }
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int q = 0; q < 8; ++q) s += e2f<H>(t[c][q]);
  s = half_sum_dpp(s);          // xor 16, 8, 4, 2, 1: the __shfl_xor butterfly's order on permlane / DPP
  const float mean = s / D;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int q = 0; q < 8; ++q) { const float d = e2f<H>(t[c][q]) - mean; ss += d * d; }
  ss = half_sum_dpp(ss);
  const float rstd = rsqrtf(ss / D + eps);
  __syncthreads();
  if (!ok) return;
  if (hl == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int e = (c * 32 + hl) * 8;
    if constexpr (ADD) *(bf16x8*)(x_out + base + e) = t[c];
    const f32x4 w0 = sw[e / 4], w1 = sw[e / 4 + 1], b0 = sb[e / 4], b1 = sb[e / 4 + 1];
    bf16x8 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      o[q] = f2e<H>((e2f<H>(t[c][q]) - mean) * rstd * w0[q] + b0[q]);
      o[q + 4] = f2e<H>((e2f<H>(t[c][q + 4]) - mean) * rstd * w1[q] + b1[q]);
    }
    *(bf16x8*)(y + base + e) = o;
  }
}

// 4 consecutive elements of a fp32 / bf16 / fp16 row as fp32 (one 16-B or 8-B load; i a multiple of 4, the base 16-B
// aligned)
__device__ __forceinline__ f32x4 ld4_as_f32(const void* p, int dtype, int64_t i) {
  if (dtype == TW_F32) return *(const f32x4*)((const float*)p + i);
  if (dtype == TW_BF16) {
    const bf16x4 t = *(const bf16x4*)((const bf16*)p + i);
    return f32x4{bf2f(t[0]), bf2f(t[1]), bf2f(t[2]), bf2f(t[3])};
  }
  const f16x4 t = *(const f16x4*)((const f16*)p + i);
  return f32x4{(float)t[0], (float)t[1], (float)t[2], (float)t[3]};
}

// dx = rstd * (w*dy - mean(w*dy) - xhat * mean(w*dy*xhat)); dx accumulated into dx_out (fp32).
// Per-block partial dw/db written to partial[blockIdx.x][2][D] for a column reduction.
// g16 (optional): the 16-bit copy of the final dx (g_dtype 1 bf16, 2 fp16) -- the autocast rounding of the stream
// gradient that the preceding block's first GEMM consumes, fused here instead of a separate cast pass.
template <int VEC, int MAXJ>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const void* __restrict__ x, int x_dtype,
                                                     const float* __restrict__ w, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const void* __restrict__ dy,
                                                     int dy_dtype, float* __restrict__ dx, int dx_accum,
                                                     float* __restrict__ partial, int rows, int D,
                                                     void* __restrict__ g16 = nullptr, int g_dtype = TW_BF16) {
  __shared__ float red[WPB][2][1280];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const int J = D / (64 * VEC);
  float dw[MAXJ][VEC], db[MAXJ][VEC];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
#pragma unroll
    for (int q = 0; q < VEC; ++q) { dw[j][q] = 0.f; db[j][q] = 0.f; }
  for (int row = blockIdx.x * WPB + wv; row < rows; row += gridDim.x * WPB) {
    const int64_t base = (int64_t)row * D;
    const float mu = mean_in[row], rs = rstd_in[row];
    float xh[MAXJ][VEC], g[MAXJ][VEC];
    float s1 = 0.f, s2 = 0.f;
    // VEC 4: each lane's 4 consecutive x / dy values as one 16-B (fp32) or 8-B (16-bit) load, every load of the row
    // issued before the arithmetic (the host checks the 16-B alignment); else one element per lane and load
    float xs[MAXJ][VEC], ds[MAXJ][VEC];
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      if (j < J) {
        if constexpr (VEC == 4) {
          const int64_t e = base + (j * 64 + lane) * 4;
          const f32x4 a = ld4_as_f32(x, x_dtype, e), c = ld4_as_f32(dy, dy_dtype, e);
#pragma unroll
          for (int q = 0; q < 4; ++q) { xs[j][q] = a[q]; ds[j][q] = c[q]; }
        } else {
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            const int e = (j * 64 + lane) * VEC + q;
            xs[j][q] = ld_as_f32(x, x_dtype, base + e);
            ds[j][q] = ld_as_f32(dy, dy_dtype, base + e);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      if (j < J) {
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          const int e = (j * 64 + lane) * VEC + q;
          const float xv = xs[j][q];
          const float dv = ds[j][q];
          xh[j][q] = (xv - mu) * rs;
          g[j][q] = dv * w[e];
          s1 += g[j][q];
          s2 += g[j][q] * xh[j][q];
          dw[j][q] += dv * xh[j][q];
          db[j][q] += dv;
        }
      }
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      if (j < J) {
        if constexpr (VEC == 4) {
          float* d = dx + base + (j * 64 + lane) * 4;
          f32x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[q] = rs * (g[j][q] - s1 - xh[j][q] * s2);
          if (dx_accum) o += *(const f32x4*)d;
          *(f32x4*)d = o;
          if (g16) {
            const int64_t e = base + (j * 64 + lane) * 4;
            if (g_dtype == TW_F16)
              *(f16x4*)((f16*)g16 + e) = f16x4{(_Float16)o[0], (_Float16)o[1], (_Float16)o[2], (_Float16)o[3]};
            else
              *(bf16x4*)((bf16*)g16 + e) = bf16x4{f2bf(o[0]), f2bf(o[1]), f2bf(o[2]), f2bf(o[3])};
          }
        } else {
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            const int e = (j * 64 + lane) * VEC + q;
            const float o = rs * (g[j][q] - s1 - xh[j][q] * s2);
            const float f = dx_accum ? dx[base + e] + o : o;
            dx[base + e] = f;
            if (g16) st_from_f32(g16, g_dtype, base + e, f);
          }
        }
      }
    }
  }
  // block reduction of dw/db over the 4 waves
#pragma unroll
  for (int j = 0; j < MAXJ; ++j)
    if (j < J)
#pragma unroll
      for (int q = 0; q < VEC; ++q) {
        const int e = (j * 64 + lane) * VEC + q;
        red[wv][0][e] = dw[j][q];
        red[wv][1][e] = db[j][q];
      }
  __syncthreads();
  for (int e = threadIdx.x; e < D; e += blockDim.x) {
    float a = 0.f, c = 0.f;
#pragma unroll
    for (int k = 0; k < WPB; ++k) { a += red[k][0][e]; c += red[k][1][e]; }
    partial[(int64_t)blockIdx.x * 2 * D + e] = a;
    partial[(int64_t)blockIdx.x * 2 * D + D + e] = c;
  }
}

// dw_out[c] += sum_b partial[b][0][c]; db_out[c] += sum_b partial[b][1][c].  64 columns per
// block; 16 thread rows each sum every 16th partial (coalesced 256-B rows, many loads in flight),
// then a fixed-order combine in LDS (deterministic)
__global__ __launch_bounds__(1024) void ln_param_reduce_kernel(const float* __restrict__ partial, int nb, int D,
                                                               float* __restrict__ dw_out, float* __restrict__ db_out) {
  __shared__ float sa[16][64], sb[16][64];
  const int cl = threadIdx.x & 63, j = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float a = 0.f, s = 0.f;
  if (c < D)
    for (int b = j; b < nb; b += 16) {
      a += partial[(int64_t)b * 2 * D + c];
      s += partial[(int64_t)b * 2 * D + D + c];
    }
  sa[j][cl] = a;
  sb[j][cl] = s;
  __syncthreads();
  if (j == 0 && c < D) {
    for (int k = 1; k < 16; ++k) {
      a += sa[k][cl];
      s += sb[k][cl];
    }
    if (dw_out) dw_out[c] += a;
    if (db_out) db_out[c] += s;
  }
}

}  // namespace

extern "C" int tw_layernorm_fwd(const void* x, int x_dtype, const float* w, const float* b, void* y, int y_dtype,
                                float* mean_out, float* rstd_out, int rows, int D, float eps, hipStream_t stream) {
  if (rows <= 0) return TW_OK;
  if (D % 64 || D > 1280) return TW_EUNSUPPORTED;
  dim3 grid((rows + WPB - 1) / WPB), block(64 * WPB);
  const bool a16 = (((uintptr_t)x | (uintptr_t)y | (uintptr_t)w | (uintptr_t)b) & 15) == 0;
  if (x_dtype == TW_F16 && y_dtype == TW_F16 && D % 256 == 0 && a16) {
    const dim3 g2((rows + 2 * WPB - 1) / (2 * WPB));
    const bf16* xb = (const bf16*)x;
    bf16* yb = (bf16*)y;
    switch (D / 256) {
      case 1: hipLaunchKernelGGL((ln_fwd_bf16_kernel<1, false, true>), g2, block, 0, stream, xb, w, b, yb, mean_out,
                                 rstd_out, rows, D, eps); break;
      case 2: hipLaunchKernelGGL((ln_fwd_bf16_kernel<2, false, true>), g2, block, 0, stream, xb, w, b, yb, mean_out,
                                 rstd_out, rows, D, eps); break;
      case 3: hipLaunchKernelGGL((ln_fwd_bf16_kernel<3, false, true>), g2, block, 0, stream, xb, w, b, yb, mean_out,
                                 rstd_out, rows, D, eps); break;
      case 4: hipLaunchKernelGGL((ln_fwd_bf16_kernel<4, false, true>), g2, block, 0, stream, xb, w, b, yb, mean_out,
                                 rstd_out, rows, D, eps); break;
      default: hipLaunchKernelGGL((ln_fwd_bf16_kernel<5, false, true>), g2, block, 0, stream, xb, w, b, yb, mean_out,
                                  rstd_out, rows, D, eps); break;
    }
  } else if (x_dtype == TW_BF16 && y_dtype == TW_BF16 && D % 256 == 0 && a16) {
    const dim3 g2((rows + 2 * WPB - 1) / (2 * WPB));
    switch (D / 256) {
      case 1: hipLaunchKernelGGL(ln_fwd_bf16_kernel<1>, g2, block, 0, stream, (const bf16*)x, w, b, (bf16*)y, mean_out,
                                 rstd_out, rows, D, eps); break;
      case 2: hipLaunchKernelGGL(ln_fwd_bf16_kernel<2>, g2, block, 0, stream, (const bf16*)x, w, b, (bf16*)y, mean_out,
                                 rstd_out, rows, D, eps); break;
      case 3: hipLaunchKernelGGL(ln_fwd_bf16_kernel<3>, g2, block, 0, stream, (const bf16*)x, w, b, (bf16*)y, mean_out,
                                 rstd_out, rows, D, eps); break;
      case 4: hipLaunchKernelGGL(ln_fwd_bf16_kernel<4>, g2, block, 0, stream, (const bf16*)x, w, b, (bf16*)y, mean_out,
                                 rstd_out, rows, D, eps); break;
      default: hipLaunchKernelGGL(ln_fwd_bf16_kernel<5>, g2, block, 0, stream, (const bf16*)x, w, b, (bf16*)y, mean_out,
                                  rstd_out, rows, D, eps); break;
    }
  } else if (D % 256 == 0)
    hipLaunchKernelGGL((ln_fwd_kernel<4, 5>), grid, block, 0, stream, x, x_dtype, w, b, y, y_dtype, mean_out,
                       rstd_out, rows, D, eps);
  else
    hipLaunchKernelGGL((ln_fwd_kernel<1, 20>), grid, block, 0, stream, x, x_dtype, w, b, y, y_dtype, mean_out,
                       rstd_out, rows, D, eps);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_add_layernorm_fwd(const void* x, int x_dtype, const void* r, void* x_out, const float* w,
                                    const float* b, void* y, float* mean_out, float* rstd_out, int rows, int D,
                                    float eps, hipStream_t stream) {
  if (rows <= 0) return TW_OK;
  if (D % 256 || D > 1280) return TW_EUNSUPPORTED;
  if ((((uintptr_t)x | (uintptr_t)r | (uintptr_t)x_out | (uintptr_t)y | (uintptr_t)w | (uintptr_t)b) & 15) != 0)
    return TW_EINVAL;
  if (x_dtype == TW_F32) {
    hipLaunchKernelGGL((ln_fwd_kernel<4, 5, true>), dim3((rows + WPB - 1) / WPB), dim3(64 * WPB), 0, stream, x,
                       (int)TW_F32, w, b, y, (int)TW_BF16, mean_out, rstd_out, rows, D, eps, (const bf16*)r,
                       (float*)x_out);
  } else {
    const dim3 g2((rows + 2 * WPB - 1) / (2 * WPB)), block(64 * WPB);
    const bf16 *xb = (const bf16*)x, *rb = (const bf16*)r;
    bf16 *yb = (bf16*)y, *xo = (bf16*)x_out;
    switch (D / 256) {
      case 1: hipLaunchKernelGGL((ln_fwd_bf16_kernel<1, true>), g2, block, 0, stream, xb, w, b, yb, mean_out, rstd_out,
                                 rows, D, eps, rb, xo); break;
      case 2: hipLaunchKernelGGL((ln_fwd_bf16_kernel<2, true>), g2, block, 0, stream, xb, w, b, yb, mean_out, rstd_out,
                                 rows, D, eps, rb, xo); break;
      case 3: hipLaunchKernelGGL((ln_fwd_bf16_kernel<3, true>), g2, block, 0, stream, xb, w, b, yb, mean_out, rstd_out,
                                 rows, D, eps, rb, xo); break;
      case 4: hipLaunchKernelGGL((ln_fwd_bf16_kernel<4, true>), g2, block, 0, stream, xb, w, b, yb, mean_out, rstd_out,
                                 rows, D, eps, rb, xo); break;
      default: hipLaunchKernelGGL((ln_fwd_bf16_kernel<5, true>), g2, block, 0, stream, xb, w, b, yb, mean_out, rstd_out,
                                  rows, D, eps, rb, xo); break;
    }
  }
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// fp16 autocast (round 6): x_out = x + r over the fp32 stream with r the fp16 Linear output, y = fp16 LN(x_out)
extern "C" int tw_add_layernorm_fwd_f16(const void* x, int x_dtype, const void* r, void* x_out, const float* w,
                                        const float* b, void* y, float* mean_out, float* rstd_out, int rows, int D,
                                        float eps, hipStream_t stream) {
  if (rows <= 0) return TW_OK;
  if (D % 256 || D > 1280) return TW_EUNSUPPORTED;
  if (x_dtype != TW_F32) return TW_EUNSUPPORTED;
  if ((((uintptr_t)x | (uintptr_t)r | (uintptr_t)x_out | (uintptr_t)y | (uintptr_t)w | (uintptr_t)b) & 15) != 0)
    return TW_EINVAL;
  hipLaunchKernelGGL((ln_fwd_kernel<4, 5, true, true>), dim3((rows + WPB - 1) / WPB), dim3(64 * WPB), 0, stream, x,
                     (int)TW_F32, w, b, y, (int)TW_F16, mean_out, rstd_out, rows, D, eps, (const bf16*)r,
                     (float*)x_out);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// workspace: >= nblk*2*D floats where nblk = min(1024, ceil(rows/4)); dw/db accumulated into dw_out/db_out;
// g16 (may be NULL): also the bf16 (g_dtype 1) / fp16 (2) rounding of the final dx
extern "C" int tw_layernorm_bwd_ex(const void* x, int x_dtype, const float* w, const float* mean, const float* rstd,
                                   const void* dy, int dy_dtype, float* dx, int dx_accum, float* dw_out,
                                   float* db_out, int rows, int D, float* workspace, int64_t workspace_floats,
                                   void* g16, int g_dtype, hipStream_t stream) {
  if (rows <= 0) return TW_OK;
  if (g16 && g_dtype != TW_BF16 && g_dtype != TW_F16) return TW_EINVAL;
  if (D % 64 || D > 1280) return TW_EUNSUPPORTED;
  int nblk = (rows + WPB - 1) / WPB;
  if (nblk > 1024) nblk = 1024;
  if (workspace_floats < (int64_t)nblk * 2 * D) return TW_EINVAL;
  // VEC 4 with the exact number of 256-column chunks as MAXJ: the per-lane arrays (x, dy, xhat, g, dw, db) sized
  // for the row, not for D = 1280 (D = 768: fewer registers, more waves per SIMD)
  const bool v4 = D % 256 == 0 && (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)dx | (uintptr_t)w | (uintptr_t)g16) & 15) == 0;
#define TW_LN_BWD(J)                                                                                          \
  hipLaunchKernelGGL((ln_bwd_kernel<4, J>), dim3(nblk), dim3(256), 0, stream, x, x_dtype, w, mean, rstd, dy, dy_dtype, \
                     dx, dx_accum, workspace, rows, D, g16, g_dtype)
  // D = 1280 holds 162 VGPRs = 3 waves per SIMD: one block per resident slot (768 on a 256-CU MI355X: all resident
  // at once) instead of a 1024-block grid whose last quarter would run as a second, mostly idle round.  The cap is
  // the occupancy query x the device's CU count (cached), not a constant of one part.
  if (v4 && D > 1024) {
    static const int cap = [] {
      int dev = 0, cus = 0, per = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)ln_bwd_kernel<4, 5>, 256, 0);
      return std::max(1, cus) * std::max(1, per);
    }();
    if (nblk > cap) nblk = cap;
  }
  if (v4 && D == 256) TW_LN_BWD(1);
  else if (v4 && D == 512) TW_LN_BWD(2);
  else if (v4 && D == 768) TW_LN_BWD(3);
  else if (v4 && D == 1024) TW_LN_BWD(4);
  else if (v4) TW_LN_BWD(5);
#undef TW_LN_BWD
  else
    hipLaunchKernelGGL((ln_bwd_kernel<1, 20>), dim3(nblk), dim3(256), 0, stream, x, x_dtype, w, mean, rstd, dy,
                       dy_dtype, dx, dx_accum, workspace, rows, D, g16, g_dtype);
  TW_CHECK_LAUNCH();
  hipLaunchKernelGGL(ln_param_reduce_kernel, dim3((D + 63) / 64), dim3(1024), 0, stream, workspace, nblk, D, dw_out,
                     db_out);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_layernorm_bwd(const void* x, int x_dtype, const float* w, const float* mean, const float* rstd,
                                const void* dy, int dy_dtype, float* dx, int dx_accum, float* dw_out, float* db_out,
                                int rows, int D, float* workspace, int64_t workspace_floats, hipStream_t stream) {
  return tw_layernorm_bwd_ex(x, x_dtype, w, mean, rstd, dy, dy_dtype, dx, dx_accum, dw_out, db_out, rows, D, workspace,
                             workspace_floats, nullptr, TW_BF16, stream);
}
