// The GEMM epilogue value (also the skinny / split-K reduce kernels' per-element epilogue) and the batch <= 8
// GEMV body of gemv_kernel (gemm.hip, one launch per LN + Linear of the decode step).
#pragma once
#include "gemm_impl.h"

namespace twg {

// the epilogue value of C[m][n] (writes the GELU pre-activation to aux on the way), before the store
template <bool H>
__device__ __forceinline__ float epi_value(const GemmP& p, int m, int n, float v) {
  const int flags = p.flags;
  v *= p.alpha;
  if (flags & F_BIAS) v += e2f<H>(p.bias[n]);
  if (flags & F_ROUND) v = rnd<H>(v);
  if (flags & F_DGELU) v = rnd<H>(v * gelu_erf_grad(e2f<H>(p.aux[(int64_t)m * p.ldaux + n])));
  if (flags & F_GELU) {
    if (flags & F_AUX_OUT) p.aux[(int64_t)m * p.ldaux + n] = f2e<H>(v);
    v = rnd<H>(gelu_of<H>(v));
  }
  if (flags & F_RES) {
    const int mr = p.res_mod > 0 ? (m % p.res_mod) : m;
    const int64_t ri = (int64_t)mr * p.ldr + n;
    v += ld16_as_f32<H>(p.res, p.res_dtype, ri);
  }
  if (flags & F_ACCUM) v += ld16_as_f32<H>(p.C, p.c_dtype, (int64_t)m * p.ldc + n);
  if (flags & F_CLAMP16) v = clamp_f16_stream(rnd<H>(v));
  return v;
}

// ---------------------------------------------------------------------------------------------
// GEMV for the batch <= 8 decode step: CPW output columns per wave.  The A rows go to LDS first -- as
// given, or through the LayerNorm in front of the Linear (ln_w != nullptr: the pre-LN residual stream x in,
// the same half-wave statistics, order and 16-bit output as ln_fwd_bf16_kernel, so A is bit-identical to
// tw_layernorm_fwd's output) -- then each wave streams its W rows (16 B per lane; the first PRE pieces per
// lane are loaded before the A rows are staged, so their HBM latency hides behind the LayerNorm / LDS
// prologue) against the LDS rows, fp32 FMAs in k order per lane, one butterfly sum, and lane 0 applies the
// full epilogue.  Fusing the LN removes one launch per LN'd Linear, which is most of a batch-1 step's cost.
// PRE is sized to K (3 pieces cover K = 1280, 10 cover 5120): more registers would cut the waves per SIMD.
// ---------------------------------------------------------------------------------------------
// Optional KV-cache append fused into the epilogue (the decode step's QKV projection): output columns
// n >= kv.col0 are also stored at kv.cache[m * kv.sb + (*kv.t) * kv.ld + n - kv.col0] -- what tw_kv_append
// copies, one launch fewer per decoder layer.
struct GemvKV {
  void* cache;
  int64_t sb, ld;
  int col0;
  const int* t;
};

// the first PRE 16-B pieces per lane of W rows n0 .. n0 + CPW - 1 (rows past N read row 0, never stored)
template <bool H, int CPW, int PRE>
__device__ __forceinline__ void gemv_preload(const GemmP& p, int n0, int lane, bf16x8 (&wpre)[CPW][PRE]) {
  const int npre = min(PRE, (p.K - lane * 8 + 511) / 512);
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    const int n = n0 + c;
    const bf16* wr = p.B + (int64_t)(n < p.N ? n : 0) * p.ldb;
#pragma unroll
    for (int u = 0; u < PRE; ++u) wpre[c][u] = (u < npre) ? *(const bf16x8*)(wr + lane * 8 + u * 512) : bf16x8{};
  }
}

// A rows -> xs [MR][K] (16-bit), LayerNorm'd when lnw is given; wave w of nw stages rows w, w + nw, ...
template <bool H, int MR>
__device__ __forceinline__ void gemv_stage_rows(const GemmP& p, const float* __restrict__ lnw,
                                                const float* __restrict__ lnb, float eps, bf16* xs, int wave, int nw,
                                                int lane) {
  const int K = p.K;
  for (int row = wave; row < MR; row += nw) {
    bf16* dst = xs + (int64_t)row * K;
    if (row >= p.M) {
      for (int e = lane * 8; e < K; e += 512) *(bf16x8*)(dst + e) = bf16x8{};
    } else if (lnw) {
      const bf16* xr = p.A + (int64_t)row * p.lda;
      const int hl = lane & 31, nch = K / 256;
      float s = 0.f;
      for (int c = 0; c < nch; ++c) {
        const bf16x8 t = *(const bf16x8*)(xr + (c * 32 + hl) * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) s += e2f<H>(t[q]);
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const float mean = s / K;
      float ss = 0.f;
      for (int c = 0; c < nch; ++c) {
        const bf16x8 t = *(const bf16x8*)(xr + (c * 32 + hl) * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) { const float d = e2f<H>(t[q]) - mean; ss += d * d; }
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) ss += __shfl_xor(ss, o, 64);
      const float rstd = rsqrtf(ss / K + eps);
      if (lane < 32) {
        for (int c = 0; c < nch; ++c) {
          const int e = (c * 32 + hl) * 8;
          const bf16x8 t = *(const bf16x8*)(xr + e);
          const f32x4 w0 = *(const f32x4*)(lnw + e), w1 = *(const f32x4*)(lnw + e + 4);
          const f32x4 b0 = *(const f32x4*)(lnb + e), b1 = *(const f32x4*)(lnb + e + 4);
          float v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = e2f<H>(t[q]);
          bf16x8 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o[q] = f2e<H>((v[q] - mean) * rstd * w0[q] + b0[q]);
            o[q + 4] = f2e<H>((v[q + 4] - mean) * rstd * w1[q] + b1[q]);
          }
          *(bf16x8*)(dst + e) = o;
        }
      }
    } else {
      const bf16* xr = p.A + (int64_t)row * p.lda;
      for (int e = lane * 8; e < K; e += 512) *(bf16x8*)(dst + e) = *(const bf16x8*)(xr + e);
    }
  }
}

// columns n0 .. n0 + CPW - 1 against the staged rows (xs visible to this wave), then the epilogue by lane 0
template <bool H, int MR, int CPW, int PRE>
__device__ __forceinline__ void gemv_finish(const GemmP& p, const GemvKV& kv, const bf16* xs, int n0, int lane,
                                            const bf16x8 (&wpre)[CPW][PRE]) {
  const int K = p.K;
  const int npre = min(PRE, (K - lane * 8 + 511) / 512);
  float acc[CPW][MR];
#pragma unroll
  for (int c = 0; c < CPW; ++c)
#pragma unroll
    for (int r = 0; r < MR; ++r) acc[c][r] = 0.f;
  // k order per lane: pieces u = 0, 1, ... at k = lane*8 + 512u (the preloaded ones first, the rest streamed)
#pragma unroll
  for (int u = 0; u < PRE; ++u) {
    if (u < npre) {
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const bf16x8 a8 = *(const bf16x8*)(xs + (int64_t)r * K + lane * 8 + u * 512);
#pragma unroll
        for (int c = 0; c < CPW; ++c)
#pragma unroll
          for (int q = 0; q < 8; ++q) acc[c][r] = fmaf(e2f<H>(wpre[c][u][q]), e2f<H>(a8[q]), acc[c][r]);
      }
    }
  }
  for (int k0 = lane * 8 + PRE * 512; k0 < K; k0 += 512) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int n = n0 + c;
      const bf16x8 w8 = *(const bf16x8*)(p.B + (int64_t)(n < p.N ? n : 0) * p.ldb + k0);
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const bf16x8 a8 = *(const bf16x8*)(xs + (int64_t)r * K + k0);
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[c][r] = fmaf(e2f<H>(w8[q]), e2f<H>(a8[q]), acc[c][r]);
      }
    }
  }
#pragma unroll
  for (int c = 0; c < CPW; ++c)
#pragma unroll
    for (int r = 0; r < MR; ++r) acc[c][r] = wave_sum(acc[c][r]);
  if (lane == 0) {
    const int64_t t = kv.cache ? (int64_t)*kv.t : 0;
#pragma unroll
    for (int c = 0; c < CPW; ++c)
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const int n = n0 + c;
        if (r < p.M && n < p.N) {
          const float v = epi_value<H>(p, r, n, acc[c][r]);
          const int64_t co = (int64_t)r * p.ldc + n;
          if (p.c_dtype == TW_BF16) ((bf16*)p.C)[co] = f2e<H>(v);
          else ((float*)p.C)[co] = v;
          if (kv.cache && n >= kv.col0) {
            const int64_t ko = r * kv.sb + t * kv.ld + (n - kv.col0);
            if (p.c_dtype == TW_BF16) ((bf16*)kv.cache)[ko] = f2e<H>(v);
            else ((float*)kv.cache)[ko] = v;
          }
        }
      }
  }
}

}  // namespace twg
