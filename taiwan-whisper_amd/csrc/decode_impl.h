// Decode attention bodies (one query row per (clip, head) over a KV cache) of the kernels in decode.hip.
#pragma once
#include "common.h"

namespace twd {

constexpr int DA_THREADS = 256;
constexpr int DA_MAX_TK = 2048;
constexpr int DA_SPLIT = 128;   // keys per workgroup of the split (flash-decoding) variant
constexpr int DA_U = 4;           // key sub-steps per wave iteration (loads in flight per lane)
constexpr int DA_BIG = 4096;      // (clip, head) pairs from which the one-workgroup-per-pair kernel takes DA_U = 2

struct DecP {
  const void* q; int64_t sqb;
  const void* k; int64_t ldk, skb;
  const void* v; int64_t ldv, svb;
  void* o; int64_t sob;
  int64_t hsk, hsv;   // head strides of K and V (64: heads side by side in a row; Tk*64: head-major blocks)
  int H, Tk;
  const int* tk_dev;  // nullable: effective Tk = *tk_dev + Tk (graph-captured decode steps)
  float c;        // scale * log2(e)
};

// K / V rows of the one-workgroup-per-pair kernel are read once per decode step: NT streams them past the caches
// (nontemporal loads, 16-bit forms; the fp32 path reads plainly)
template <bool NT>
__device__ __forceinline__ void load8_kv(const bf16* p, float* o) {
  if constexpr (NT) {
    const bf16x8 v = __builtin_nontemporal_load((const bf16x8*)p);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
  } else {
    load8(p, o);
  }
}
template <bool NT>
__device__ __forceinline__ void load8_kv(const f16* p, float* o) {
  if constexpr (NT) {
    const f16x8 v = __builtin_nontemporal_load((const f16x8*)p);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (float)v[j];
  } else {
    load8(p, o);
  }
}
template <bool NT>
__device__ __forceinline__ void load8_kv(const float* p, float* o) { load8(p, o); }

// lane = (key slot ks = lane >> 3, 8-element chunk ch = lane & 7); a wave covers 8 keys per step.
// E = bf16 (autocast path) or float (fp32 path: exact expf, no rounding of the output).
// The body attends keys [lo, hi).  part == nullptr: normalise and store O.  Otherwise (split over keys,
// flash-decoding) store the chunk's unnormalised o[64], its max m (log2 domain) and sum l to part[0..65]
// for decode_attn_combine_kernel.
template <typename E, int DA_U = twd::DA_U, bool NT = false>
__device__ __forceinline__ void decode_attn_body(const DecP& p, int b, int h, int lo, int hi, float* part) {
  __shared__ float sc[DA_MAX_TK];
  __shared__ float red[DA_THREADS / 64][64];
  __shared__ float red_l[DA_THREADS / 64];
  __shared__ float red_m[DA_THREADS / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ks = lane >> 3, ch = lane & 7;
  constexpr bool F32 = sizeof(E) == 4;
  const E* qb = (const E*)p.q + b * p.sqb + h * 64 + ch * 8;
  const E* kb = (const E*)p.k + b * p.skb + h * p.hsk + ch * 8;
  const E* vb = (const E*)p.v + b * p.svb + h * p.hsv + ch * 8;
  float qv[8];
  load8(qb, qv);
  // pass 1: scores (log2 domain) -> LDS, running max.  A wave takes 8 keys x DA_U sub-steps per iteration
  // (keys k0 + 8u + ks): DA_U independent 16-B loads per lane in flight before the reductions.
  float mx = -INFINITY;
  for (int k0 = lo + wave * 8 * DA_U; k0 < hi; k0 += DA_THREADS / 8 * DA_U) {
    float t[DA_U][8];
#pragma unroll
    for (int u = 0; u < DA_U; ++u) {
      const int key = k0 + 8 * u + ks;
      if (key < hi) load8_kv<NT>(kb + (int64_t)key * p.ldk, t[u]);
    }
#pragma unroll
    for (int u = 0; u < DA_U; ++u) {
      const int key = k0 + 8 * u + ks;
      float sv = 0.f;
      if (key < hi) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sv = fmaf(qv[j], t[u][j], sv);
      }
      sv = oct_sum_dpp(sv);          // xor 1, 2, 4 on the VALU (bit-identical to the shuffles: common.h)
      if (key < hi) {
        sv *= p.c;
        if (ch == 0) sc[key - lo] = sv;
        mx = fmaxf(mx, sv);
      }
    }
  }
  mx = wave_max_dpp(mx);
  if (lane == 0) red_m[wave] = mx;
  __syncthreads();
  float m = red_m[0];
#pragma unroll
  for (int w = 1; w < DA_THREADS / 64; ++w) m = fmaxf(m, red_m[w]);
  // pass 2: p = exp2(s - m), l = sum p, o = sum p * V (same key order within each lane slot)
  float o[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float l = 0.f;
  for (int k0 = lo + wave * 8 * DA_U; k0 < hi; k0 += DA_THREADS / 8 * DA_U) {
    float t[DA_U][8];
#pragma unroll
    for (int u = 0; u < DA_U; ++u) {
      const int key = k0 + 8 * u + ks;
      if (key < hi) load8_kv<NT>(vb + (int64_t)key * p.ldv, t[u]);
    }
#pragma unroll
    for (int u = 0; u < DA_U; ++u) {
      const int key = k0 + 8 * u + ks;
      if (key < hi) {
        const float pe = F32 ? exp2f(sc[key - lo] - m) : __builtin_amdgcn_exp2f(sc[key - lo] - m);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = fmaf(pe, t[u][j], o[j]);
        if (ch == 0) l += pe;
      }
    }
  }
  // reduce over the 8 key slots of the wave (lanes ch, ch+8, ..., ch+56), then over waves
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = stride8_sum_dpp(o[j]);    // xor 8, 16, 32
  l = wave_sum_dpp(l);
  if (ks == 0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wave][ch * 8 + j] = o[j];
  }
  if (lane == 0) red_l[wave] = l;
  __syncthreads();
  if (tid < 64) {
    float acc = 0.f, lt = 0.f;
#pragma unroll
    for (int w = 0; w < DA_THREADS / 64; ++w) {
      acc += red[w][tid];
      lt += red_l[w];
    }
    if (part) {
      part[tid] = acc;
      if (tid == 0) {
        part[64] = m;
        part[65] = lt;
      }
    } else {
      ((E*)p.o)[b * p.sob + h * 64 + tid] = e_from_f32<E>(acc / lt);
    }
  }
}

// O = sum_c 2^(m_c - M) o_c / sum_c 2^(m_c - M) l_c over the chunks of one (clip, head), in chunk order,
// by the 64 lanes of one wave (lane = output dimension).  Lane c loads chunk c's (m, l) and every lane its
// column of all chunks up front (independent loads instead of a dependent chain), weights by shuffles.
constexpr int DA_MAX_CHUNK = 16;
template <typename E>
__device__ __forceinline__ void combine_row(const DecP& p, int bh, int nchunk, const float* part) {
  const int lane = threadIdx.x & 63;
  const int b = bh / p.H, h = bh % p.H;
  const float mc = lane < nchunk ? part[lane * 66 + 64] : -INFINITY;
  const float lc = lane < nchunk ? part[lane * 66 + 65] : 0.f;
  float oc[DA_MAX_CHUNK];
#pragma unroll
  for (int c = 0; c < DA_MAX_CHUNK; ++c) oc[c] = c < nchunk ? part[c * 66 + lane] : 0.f;
  const float M = wave_max_dpp(mc);
  const float wc = mc == -INFINITY ? 0.f : (sizeof(E) == 4 ? exp2f(mc - M) : __builtin_amdgcn_exp2f(mc - M));
  float acc = 0.f, lt = 0.f;
#pragma unroll
  for (int c = 0; c < DA_MAX_CHUNK; ++c) {
    if (c < nchunk) {
      const float w = readlane_f(wc, c), l = readlane_f(lc, c);
      if (readlane_f(mc, c) != -INFINITY) {
        acc = fmaf(w, oc[c], acc);
        lt = fmaf(w, l, lt);
      }
    }
  }
  ((E*)p.o)[b * p.sob + h * 64 + lane] = e_from_f32<E>(acc / lt);
}


}  // namespace twd
