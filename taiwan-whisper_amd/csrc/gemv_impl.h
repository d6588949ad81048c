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
  if (flags & F_DGELU) v = rnd<H>(v * gelu_grad_of<H>(e2f<H>(p.aux[(int64_t)m * p.ldaux + n])));
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

// one 16-B piece of a weight row, a non-temporal load: the decode step streams each weight once per step (1.5 GB per
// large-v2 step, far past the 256 MiB Infinity Cache), so nothing is gained by keeping it; the nt policy cut the
// batch-1 large-v2 fp16 step from 2.18 to 2.01 ms (tools/bench_step.py, profiles/r05_j_gemv_variants_ab.log)
__device__ __forceinline__ bf16x8 ldw8(const bf16* q) { return __builtin_nontemporal_load((const bf16x8*)q); }

// the first PRE 16-B pieces per lane of W rows n0 .. n0 + CPW - 1 (rows past N read row 0, never stored)
template <bool H, int CPW, int PRE>
__device__ __forceinline__ void gemv_preload(const GemmP& p, int n0, int lane, bf16x8 (&wpre)[CPW][PRE]) {
  const int npre = min(PRE, (p.K - lane * 8 + 511) / 512);
#pragma unroll
  for (int c = 0; c < CPW; ++c) {
    const int n = n0 + c;
    const bf16* wr = p.B + (int64_t)(n < p.N ? n : 0) * p.ldb;
#pragma unroll
    for (int u = 0; u < PRE; ++u) wpre[c][u] = (u < npre) ? ldw8(wr + lane * 8 + u * 512) : bf16x8{};
  }
}

// A rows -> xs [MR][K] (16-bit), LayerNorm'd when lnw is given; wave w of nw stages rows w, w + nw, ...
template <bool H, int MR>
__device__ __forceinline__ void gemv_stage_rows(const GemmP& p, const float* __restrict__ lnw,
                                                const float* __restrict__ lnb, float eps, bf16* xs, int wave, int nw,
                                                int lane, const float* lnp = nullptr) {
  const int K = p.K;
  if (lnp) {
    // one global pass: every row of this wave (rows wave, wave + nw, ...) loaded to registers at once while the LN
    // parameters arrive in LDS (lnp: w then b, the kernel's LDS-DMA at entry), then the same half-wave statistics
    // in the same order as below (bit-identical A); one round trip to memory instead of two or three
    constexpr int RPW = (MR + 3) / 4;
    const int hl = lane & 31, nch = K / 256;
    bf16x8 t[RPW][5];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = wave + j * nw;
      const bf16* xr = p.A + (int64_t)(row < p.M ? row : 0) * p.lda;
#pragma unroll
      for (int c = 0; c < 5; ++c) t[j][c] = c < nch ? *(const bf16x8*)(xr + (c * 32 + hl) * 8) : bf16x8{};
    }
    // the statistics of the wave's rows in lockstep: their butterflies interleave instead of running one after the
    // other (each row's own sums keep the order below, so A stays bit-identical)
    float s[RPW], mean[RPW], rstd[RPW];
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      s[j] = 0.f;
#pragma unroll
      for (int c = 0; c < 5; ++c)
        if (c < nch)
#pragma unroll
          for (int q = 0; q < 8; ++q) s[j] += e2f<H>(t[j][c][q]);
    }
    // xor 16, 8, 4, 2, 1 within each 32-lane half on permlane / DPP (half_sum_dpp: the order of the __shfl_xor
    // butterfly it replaces, bit-identical, without the ds_bpermute round trips)
#pragma unroll
    for (int j = 0; j < RPW; ++j) s[j] = half_sum_dpp(s[j]);
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      mean[j] = s[j] / K;
      s[j] = 0.f;
#pragma unroll
      for (int c = 0; c < 5; ++c)
        if (c < nch)
#pragma unroll
          for (int q = 0; q < 8; ++q) { const float d = e2f<H>(t[j][c][q]) - mean[j]; s[j] += d * d; }
    }
    // xor 16, 8, 4, 2, 1 within each 32-lane half on permlane / DPP (half_sum_dpp: the order of the __shfl_xor
    // butterfly it replaces, bit-identical, without the ds_bpermute round trips)
#pragma unroll
    for (int j = 0; j < RPW; ++j) s[j] = half_sum_dpp(s[j]);
#pragma unroll
    for (int j = 0; j < RPW; ++j) rstd[j] = rsqrtf(s[j] / K + eps);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pieces of the LN parameters have landed
    __syncthreads();                                    // ... and every other wave's
#pragma unroll
    for (int j = 0; j < RPW; ++j) {
      const int row = wave + j * nw;
      if (row >= MR) break;
      bf16* dst = xs + (int64_t)row * K;
      if (row >= p.M) {
        for (int e = lane * 8; e < K; e += 512) *(bf16x8*)(dst + e) = bf16x8{};
        continue;
      }
      if (lane < 32) {
#pragma unroll
        for (int c = 0; c < 5; ++c) {
          if (c < nch) {
            // LN parameters from LDS, read per chunk (held for every chunk they would cost ~80 VGPRs: at MR = 8 that
            // cut the waves per SIMD below what the wide Linears need)
            const int e = (c * 32 + hl) * 8;
            const f32x4 w0 = *(const f32x4*)(lnp + e), w1 = *(const f32x4*)(lnp + e + 4);
            const f32x4 b0 = *(const f32x4*)(lnp + K + e), b1 = *(const f32x4*)(lnp + K + e + 4);
            bf16x8 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              o[q] = f2e<H>((e2f<H>(t[j][c][q]) - mean[j]) * rstd[j] * w0[q] + b0[q]);
              o[q + 4] = f2e<H>((e2f<H>(t[j][c][q + 4]) - mean[j]) * rstd[j] * w1[q] + b1[q]);
            }
            *(bf16x8*)(dst + (c * 32 + hl) * 8) = o;
          }
        }
      }
    }
    return;
  }
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
      s = half_sum_dpp(s);
      const float mean = s / K;
      float ss = 0.f;
      for (int c = 0; c < nch; ++c) {
        const bf16x8 t = *(const bf16x8*)(xr + (c * 32 + hl) * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) { const float d = e2f<H>(t[q]) - mean; ss += d * d; }
      }
      ss = half_sum_dpp(ss);
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
      // up to 5 pieces per lane loaded before any is stored: one memory round trip per 2560 columns instead of one
      // per piece (the rows were just written by the previous launch and come from L2)
      const bf16* xr = p.A + (int64_t)row * p.lda;
      for (int e0 = lane * 8; e0 < K; e0 += 5 * 512) {
        bf16x8 t[5];
#pragma unroll
        for (int c = 0; c < 5; ++c)
          if (e0 + c * 512 < K) t[c] = *(const bf16x8*)(xr + e0 + c * 512);
#pragma unroll
        for (int c = 0; c < 5; ++c)
          if (e0 + c * 512 < K) *(bf16x8*)(dst + e0 + c * 512) = t[c];
      }
    }
  }
}

// columns n0 .. n0 + CPW - 1 against the staged rows (xs visible to this wave), then the epilogue by lane 0
// acc = fma(w[q], a[q], acc) for q = 0..7 in order, the 16-bit operands widened exactly to fp32.  fp16: one
// v_fma_mix_f32 per element (the f16 -> f32 widening inside the FMA: the same single rounding as fmaf on the widened
// operands, without the 16 v_cvt_f32_f16 per 8 elements the compiler otherwise emits beside each row)
typedef __attribute__((ext_vector_type(4))) unsigned int gv_u32x4;

template <bool H>
__device__ __forceinline__ void fma8(float& acc, const bf16x8& w, const bf16x8& a) {
  if constexpr (H) {
    const gv_u32x4 wu = __builtin_bit_cast(gv_u32x4, w), au = __builtin_bit_cast(gv_u32x4, a);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(wu[i]), "v"(au[i]));
      asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(wu[i]), "v"(au[i]));
    }
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = fmaf(e2f<H>(w[q]), e2f<H>(a[q]), acc);
  }
}

// NV values per lane -> lane l returns the wave total of value `idx` (idx = -1: this lane holds none).  Stage xor 32:
// v_permlane32_swap(vdst = y, vsrc = x) leaves lanes 0..31 y_l + y_(l+32) and lanes 32..63 x_(l-32) + x_l -- the
// operands of swap32_sum in the same order -- so pairing value j with j + NV/2 halves the values per lane; stage
// xor 16 does the same within each 32-lane half (v_permlane16_swap: even 16-lane rows keep the second value of a
// pair); the rest (xor 8, 4, 2, 1) run on the remaining values as in wave_sum_dpp.
template <int NV>
__device__ __forceinline__ float wave_reduce_scatter(const float (&v)[NV], int lane, int& idx) {
  const bool hiA = lane >= 32, hiB = (lane & 16) != 0;
  if constexpr (NV == 1) {
    idx = lane == 0 ? 0 : -1;
    return wave_sum_dpp(v[0]);
  } else {
    constexpr int NA = NV / 2;
    float w[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[j + NA]), __float_as_uint(v[j]), false, false);
      w[j] = __uint_as_float(a[0]) + __uint_as_float(a[1]);      // lanes < 32: value j + NA; lanes >= 32: value j
    }
    if constexpr (NA == 1) {
      float t = swap16_sum(w[0]);
      t += TW_DPP(t, TW_ROW_ROR(8));
      t += TW_DPP(t, TW_ROW_ROR(4));
      t += TW_DPP(t, TW_ROW_ROR(2));
      t += TW_DPP(t, TW_ROW_ROR(1));
      idx = (lane & 31) == 0 ? (hiA ? 0 : 1) : -1;
      return t;
    } else {
      constexpr int NB = NA / 2;
      float u[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(w[j + NB]), __float_as_uint(w[j]), false, false);
        u[j] = __uint_as_float(a[0]) + __uint_as_float(a[1]);    // even rows: w[j + NB]; odd rows: w[j]
      }
      float mine = 0.f;
      const int jl = lane & 15;
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        float t = u[j];
        t += TW_DPP(t, TW_ROW_ROR(8));
        t += TW_DPP(t, TW_ROW_ROR(4));
        t += TW_DPP(t, TW_ROW_ROR(2));
        t += TW_DPP(t, TW_ROW_ROR(1));
        if (jl == j) mine = t;
      }
      idx = jl < NB ? jl + (hiB ? 0 : NB) + (hiA ? 0 : NA) : -1;
      return mine;
    }
  }
}

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
        for (int c = 0; c < CPW; ++c) fma8<H>(acc[c][r], wpre[c][u], a8);
      }
    }
  }
  for (int k0 = lane * 8 + PRE * 512; k0 < K; k0 += 512) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int n = n0 + c;
      const bf16x8 w8 = ldw8(p.B + (int64_t)(n < p.N ? n : 0) * p.ldb + k0);
#pragma unroll
      for (int r = 0; r < MR; ++r) {
        const bf16x8 a8 = *(const bf16x8*)(xs + (int64_t)r * K + k0);
        fma8<H>(acc[c][r], w8, a8);
      }
    }
  }
  // the wave's CPW x MR totals, each the xor 32, 16, 8, 4, 2, 1 butterfly of wave_sum_dpp (the same additions in the
  // same order: bit-identical to summing each value alone), as a reduce-scatter: a v_permlane32/16_swap exchanges two
  // values at once, so the first two stages move half, then a quarter of the values; one lane per value then runs
  // its epilogue (the same per-element arithmetic as a single lane running them in turn)
  static_assert(CPW * MR <= 64, "one output per lane");
  float vals[CPW * MR];
#pragma unroll
  for (int c = 0; c < CPW; ++c)
#pragma unroll
    for (int r = 0; r < MR; ++r) vals[c * MR + r] = acc[c][r];
  int idx;
  const float mine = wave_reduce_scatter<CPW * MR>(vals, lane, idx);
  const int c = idx / MR, r = idx % MR;
  const int n = n0 + c;
  if (idx >= 0 && r < p.M && n < p.N) {
    const float v = epi_value<H>(p, r, n, mine);
    const int64_t co = (int64_t)r * p.ldc + n;
    if (p.c_dtype == TW_BF16) ((bf16*)p.C)[co] = f2e<H>(v);
    else ((float*)p.C)[co] = v;
    if (kv.cache && n >= kv.col0) {
      const int64_t t = (int64_t)*kv.t;
      const int64_t ko = r * kv.sb + t * kv.ld + (n - kv.col0);
      if (p.c_dtype == TW_BF16) ((bf16*)kv.cache)[ko] = f2e<H>(v);
      else ((float*)kv.cache)[ko] = v;
    }
  }
}

}  // namespace twg
