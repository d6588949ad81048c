// Shared pieces of the bf16 MFMA GEMMs (gemm.hip): the kernel parameter block,
// LDS staging / fragment helpers, the persistent tile walk and the fused epilogues.
#pragma once
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace twg {


constexpr int BK = 64;

enum {
  F_BIAS = 1,      // v += bias[n]            (bias bf16, autocast casts it)
  F_ROUND = 2,     // v = bf16(v)             (autocast Linear output)
  F_GELU = 4,      // [aux = v]; v = bf16(gelu(v))
  F_RES = 8,       // v = res[m % res_mod][n] + v
  F_ACCUM = 16,    // v += C_old
  F_AUX_OUT = 32,  // store pre-activation to aux (with F_GELU)
  F_DGELU = 64,    // v = bf16(v * gelu'(aux[m][n]))  (gelu backward, aux = pre-activation)
  F_CLAMP16 = 128, // after the residual add: clamp to +-(fp16 max - 1000) (HF fp16 encoder layer, fp16 GEMMs only)
};

// Inside the kernels a 16-bit C / residual / aux (c_dtype, res_dtype == TW_BF16) holds the operand type of
// the instantiation (template flag H: bf16 words, or fp16 words for the H = true instantiations); the host
// entry points map TW_F16 to that code for the fp16 GEMMs.
template <bool H>
__device__ __forceinline__ float ld16_as_f32(const void* p, int dtype, int64_t i) {
  return dtype == TW_BF16 ? e2f<H>(((const bf16*)p)[i]) : ((const float*)p)[i];
}

struct GemmP {
  const bf16* A; const bf16* B; void* C;
  int64_t lda, ldb, ldc;
  int M, N, K;
  int64_t sA, sB, sC;
  float alpha;
  const bf16* bias;
  const void* res; int64_t ldr; int64_t sR; int res_dtype; int res_mod;
  bf16* aux; int64_t ldaux; int64_t sAux;
  int c_dtype; int flags;
  int tiles_n, tiles_mn, group_m, tiles_total;
  int epi;         // fast epilogue kind chosen on the host (EPI_*), EPI_GENERIC otherwise
  float* ws;       // skinny split-K: fp32 partials [gridDim.y][M][N] (nullptr: epilogue in place)
};

__device__ __forceinline__ int xr_mn(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

// K-major tile [R rows][64 k] -> LDS, 128-B rows, 16-B chunk c of row r at c ^ (r & 7).
// R/8 pieces of 1 KiB (8 rows each), NW waves.
template <int R, int NW>
__device__ __forceinline__ void stage_k(const bf16* base, int64_t ld, int rows_left, int k_left, char* lds, int wave,
                                        int lane) {
  const auto rs = make_rsrc(base);
#pragma unroll
  for (int i = 0; i < R / 8 / NW; ++i) {
    const int pce = wave + NW * i;
    const int r = pce * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const bool ok = (r < rows_left) && (c * 8 < k_left);
    const uint32_t off = ok ? (uint32_t)(((int64_t)r * ld + c * 8) * 2) : TW_OOB;
    buf_load_lds16(rs, lds + pce * 1024, off);
  }
}

// MN-major tile [64 k-rows][R cols] -> LDS, 2R-byte k-rows, 32-B slot s of k-row r at s ^ xr_mn(r).
template <int R, int NW>
__device__ __forceinline__ void stage_mn(const bf16* base, int64_t ld, int cols_left, int k_left, char* lds, int wave,
                                         int lane) {
  const auto rs = make_rsrc(base);
  constexpr int LPR = R / 8;          // lanes (16-B chunks) per k-row
  constexpr int RPP = 64 / LPR;       // k-rows per 1-KiB piece
#pragma unroll
  for (int i = 0; i < R / 8 / NW; ++i) {
    const int pce = wave + NW * i;
    const int kr = pce * RPP + lane / LPR;
    const int pc = lane % LPR;
    const int s = (pc >> 1) ^ xr_mn(kr);
    const int col = s * 16 + (pc & 1) * 8;
    const bool ok = (kr < k_left) && (col < cols_left);
    const uint32_t off = ok ? (uint32_t)(((int64_t)kr * ld + col) * 2) : TW_OOB;
    buf_load_lds16(rs, lds + pce * 1024, off);
  }
}

__device__ __forceinline__ bf16x8 frag_k(const char* tile, int rbase, int kk, int lane) {
  const int r = rbase + (lane & 15);
  const int c = kk * 4 + (lane >> 4);
  return *(const bf16x8*)(tile + r * 128 + ((c ^ (r & 7)) << 4));
}

template <int R>
__device__ __forceinline__ bf16x8 frag_mn(const char* tile, int cbase, int kk, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = cbase + 4 * (i & 3);
  const int slot = col >> 4, inoff = (col & 15) * 2;
  const int kr0 = kk * 32 + 8 * g + (i >> 2);
  const int kr1 = kr0 + 4;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const char* a0 = tile + kr0 * (2 * R) + ((slot ^ xr_mn(kr0)) << 5) + inoff;
  const char* a1 = tile + kr1 * (2 * R) + ((slot ^ xr_mn(kr1)) << 5) + inoff;
  s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(uint32_t)(uintptr_t)a0);
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(uint32_t)(uintptr_t)a1);
  s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// Block tile BMxBN, waves WMxWN (each (BM/WM)x(BN/WN)), two LDS stages, one barrier per K-step.
// blockIdx.x enumerates (m-tile, n-tile) pairs remapped so that consecutive tiles of one m-row
// share an XCD (L2 reuse of the A panel; blocks b and b+8 share an XCD).
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0() {   // s_waitcnt vmcnt(N) lgkmcnt(0), N compile-time
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
  else if constexpr (N == 16) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
  else static_assert(N < 0, "add the vmcnt immediate");
}

// Linear tile id -> (m-tile, n-tile), grouped: runs of group_m m-tiles are walked n-tile by
// n-tile, so the ~32 tiles one XCD holds at a time share group_m A panels and 32/group_m B
// panels in its L2 (group_m = 1: plain row-major).
__device__ __forceinline__ void tile_coords(int tid, const GemmP& p, int& mt, int& nt) {
  const int tiles_m = p.tiles_mn / p.tiles_n;
  const int per_group = p.group_m * p.tiles_n;
  const int g = tid / per_group, first = g * p.group_m;
  const int gm = min(p.group_m, tiles_m - first);
  const int r = tid - g * per_group;
  mt = first + r % gm;
  nt = r / gm;
}

// Generic epilogue (any flag combination, ragged edges): lane holds C[m][n..n+3] of each 16x16
// fragment (swapped-operand MFMA layout).
// MI0 .. MI1 (MI1 < 0: all): the fragment rows written (the persistent kernel splits a tile's epilogue
// over several load segments).
// RAGGED: only ever called for tiles past an edge (no full-tile vector path compiled in).
template <bool H, int BM, int BN, int WM, int WN, int MI0 = 0, int MI1 = -1, bool RAGGED = false>
__device__ __forceinline__ void epilogue_generic(const GemmP& p, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                         int n0, int wm, int wn, int lane, int bz) {
  constexpr int FN = BN / WN / 16;
  constexpr int FM = MI1 < 0 ? BM / WM / 16 : MI1;
  const int g = lane >> 4, li = lane & 15;
  const int flags = p.flags;
  char* C = (char*)p.C;
  const bool full_tile = !RAGGED && (m0 + BM <= p.M) && (n0 + BN <= p.N) && ((p.ldc & 3) == 0) &&
                         (!(flags & F_RES) || ((p.ldr & 3) == 0 && p.res_mod == 0)) &&
                         (!(flags & (F_AUX_OUT | F_DGELU)) || (p.ldaux & 3) == 0);
  if (full_tile) {
    // fast path: no bounds checks, vector loads/stores, bias hoisted, loads of one fragment
    // row issued before any of its stores (C may alias res for in-place residual updates)
    float bv[FN][4];
#pragma unroll
    for (int ni = 0; ni < FN; ++ni) {
      if (flags & F_BIAS) {
        const bf16x4 t = *(const bf16x4*)(p.bias + n0 + wn * (BN / WN) + ni * 16 + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[ni][r] = e2f<H>(t[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[ni][r] = 0.f;
      }
    }
#pragma unroll
    for (int mi = MI0; mi < FM; ++mi) {
      const int m = m0 + wm * (BM / WM) + mi * 16 + li;
      const int nb = n0 + wn * (BN / WN) + 4 * g;
      float ex[FN][4];     // residual / old-C / aux operand, loaded up front
      if (flags & (F_RES | F_ACCUM | F_DGELU)) {
#pragma unroll
        for (int ni = 0; ni < FN; ++ni) {
          const int n = nb + ni * 16;
          if (flags & F_DGELU) {
            const bf16x4 t = *(const bf16x4*)(p.aux + bz * p.sAux + (int64_t)m * p.ldaux + n);
#pragma unroll
            for (int r = 0; r < 4; ++r) ex[ni][r] = e2f<H>(t[r]);
          } else {
            const bool res = flags & F_RES;
            const void* src = res ? p.res : (const void*)C;
            const int dt = res ? p.res_dtype : p.c_dtype;
            const int64_t o = res ? bz * p.sR + (int64_t)m * p.ldr + n : bz * p.sC + (int64_t)m * p.ldc + n;
            if (dt == TW_BF16) {
              const bf16x4 t = *(const bf16x4*)((const bf16*)src + o);
#pragma unroll
              for (int r = 0; r < 4; ++r) ex[ni][r] = e2f<H>(t[r]);
            } else {
              const f32x4 t = *(const f32x4*)((const float*)src + o);
#pragma unroll
              for (int r = 0; r < 4; ++r) ex[ni][r] = t[r];
            }
          }
        }
      }
#pragma unroll
      for (int ni = 0; ni < FN; ++ni) {
        const int n = nb + ni * 16;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = p.alpha * acc[mi][ni][r] + bv[ni][r];
          if (flags & F_ROUND) v[r] = rnd<H>(v[r]);
          if (flags & F_DGELU) v[r] = rnd<H>(v[r] * gelu_grad_of<H>(ex[ni][r]));
        }
        if (flags & F_GELU) {
          if (flags & F_AUX_OUT)
            *(bf16x4*)(p.aux + bz * p.sAux + (int64_t)m * p.ldaux + n) =
                bf16x4{f2e<H>(v[0]), f2e<H>(v[1]), f2e<H>(v[2]), f2e<H>(v[3])};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = rnd<H>(gelu_of<H>(v[r]));
        }
        if (flags & (F_RES | F_ACCUM)) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += ex[ni][r];
        }
        if (flags & F_CLAMP16) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = clamp_f16_stream(rnd<H>(v[r]));
        }
        const int64_t co = bz * p.sC + (int64_t)m * p.ldc + n;
        if (p.c_dtype == TW_BF16) *(bf16x4*)((bf16*)C + co) = bf16x4{f2e<H>(v[0]), f2e<H>(v[1]), f2e<H>(v[2]), f2e<H>(v[3])};
        else *(f32x4*)((float*)C + co) = f32x4{v[0], v[1], v[2], v[3]};
      }
    }
    return;
  }
#pragma unroll
  for (int mi = MI0; mi < FM; ++mi) {
    const int m = m0 + wm * (BM / WM) + mi * 16 + li;
    if (m >= p.M) continue;
#pragma unroll
    for (int ni = 0; ni < FN; ++ni) {
      const int n = n0 + wn * (BN / WN) + ni * 16 + 4 * g;
      if (n >= p.N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = p.alpha * acc[mi][ni][r];
      const bool full = (n + 3 < p.N);
      const int nv = full ? 4 : (p.N - n);
      if (flags & F_BIAS) {
        for (int r = 0; r < nv; ++r) v[r] += e2f<H>(p.bias[n + r]);
      }
      if (flags & F_ROUND) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = rnd<H>(v[r]);
      }
      if (flags & F_DGELU) {
        const bf16* ax = p.aux + bz * p.sAux + (int64_t)m * p.ldaux + n;
        for (int r = 0; r < nv; ++r) v[r] = rnd<H>(v[r] * gelu_grad_of<H>(e2f<H>(ax[r])));
      }
      if (flags & F_GELU) {
        if (flags & F_AUX_OUT) {
          bf16* ax = p.aux + bz * p.sAux + (int64_t)m * p.ldaux + n;
          for (int r = 0; r < nv; ++r) ax[r] = f2e<H>(v[r]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = rnd<H>(gelu_of<H>(v[r]));
      }
      if (flags & F_RES) {
        const int mr = p.res_mod > 0 ? (m % p.res_mod) : m;
        const int64_t ro = bz * p.sR + (int64_t)mr * p.ldr + n;
        for (int r = 0; r < nv; ++r) v[r] += ld16_as_f32<H>(p.res, p.res_dtype, ro + r);
      }
      const int64_t co = bz * p.sC + (int64_t)m * p.ldc + n;
      if (flags & F_ACCUM) {
        for (int r = 0; r < nv; ++r) v[r] += ld16_as_f32<H>(C, p.c_dtype, co + r);
      }
      if (flags & F_CLAMP16) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = clamp_f16_stream(rnd<H>(v[r]));
      }
      if (p.c_dtype == TW_BF16) {
        bf16* cp = (bf16*)C + co;
        if (full && ((co & 3) == 0)) {
          *(bf16x4*)cp = bf16x4{f2e<H>(v[0]), f2e<H>(v[1]), f2e<H>(v[2]), f2e<H>(v[3])};
        } else {
          for (int r = 0; r < nv; ++r) cp[r] = f2e<H>(v[r]);
        }
      } else {
        float* cp = (float*)C + co;
        if (full && ((co & 3) == 0)) {
          *(f32x4*)cp = f32x4{v[0], v[1], v[2], v[3]};
        } else {
          for (int r = 0; r < nv; ++r) cp[r] = v[r];
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Specialised full-tile epilogues for the step's hot flag combinations (chosen on the host, so
// the per-element code carries no flag branches).  bf16 tiles are written 16 B per lane: the
// fragments (ni, ni+1) of one row block are exchanged with v_permlane16_swap, after which lane
// (li, g) holds 8 consecutive columns at  16*ni + (g&1)*16 + (g>>1)*8  (64 contiguous bytes per
// row per store instruction instead of 32).  The same exchange maps a 16-B residual load back
// to fragment order (the swap is an involution), so each lane reads and writes the same bytes
// (in-place residual updates stay race-free).
// ---------------------------------------------------------------------------------------------
// EPI_DGELU (round 6): the GELU backward of the dX products, v = e(e(acc) * gelu'(aux)) on 16-bit C and aux
enum { EPI_GENERIC = 0, EPI_STORE_BF16, EPI_STORE_F32, EPI_GELU, EPI_GELU_AUX, EPI_RES_BF16, EPI_RES_F32, EPI_DGELU };

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool H>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  if constexpr (H) {
    // fp16: one v_cvt_pk_f16_f32 (gfx950, RNE) on the two fp32 values, opaque to the compiler, so it cannot fold
    // the fp32 epilogue arithmetic into a single-rounding v_fma_mixlo_f16 (f2e's reason for its asm barrier)
    uint32_t r;
    asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
  } else {
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    return __builtin_bit_cast(uint32_t, bf16x2{f2e<H>(a), f2e<H>(b)});
  }
}
template <bool H>
__device__ __forceinline__ float lo_e(uint32_t u) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu));
  else return __builtin_bit_cast(float, u << 16);
}
template <bool H>
__device__ __forceinline__ float hi_e(uint32_t u) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16));
  else return __builtin_bit_cast(float, u & 0xffff0000u);
}

// packed fragments X (ni) and Y (ni+1), 2 words each -> this lane's 16 B of the pair (swapped layout)
__device__ __forceinline__ u32x4 swap_u4(uint32_t x0, uint32_t x1, uint32_t y0, uint32_t y1) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  return u32x4{s0[0], s1[0], s0[1], s1[1]};
}
// fragments X (ni) and Y (ni+1), 4 floats each -> this lane's 16 B of the pair (swapped layout)
template <bool H>
__device__ __forceinline__ u32x4 pair_to_u4(const float (&x)[4], const float (&y)[4]) {
  return swap_u4(pack2<H>(x[0], x[1]), pack2<H>(x[2], x[3]), pack2<H>(y[0], y[1]), pack2<H>(y[2], y[3]));
}
// inverse: this lane's 16 B of the pair (swapped layout) -> fragments X, Y as floats
template <bool H>
__device__ __forceinline__ void u4_to_pair(u32x4 r, float (&x)[4], float (&y)[4]) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(r[0], r[2], false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(r[1], r[3], false, false);
  x[0] = lo_e<H>(s0[0]); x[1] = hi_e<H>(s0[0]); x[2] = lo_e<H>(s1[0]); x[3] = hi_e<H>(s1[0]);
  y[0] = lo_e<H>(s0[1]); y[1] = hi_e<H>(s0[1]); y[2] = lo_e<H>(s1[1]); y[3] = hi_e<H>(s1[1]);
}

// PB: the tile's bias was staged in LDS (`braw` = its first column, see gemm_pp_kernel) -- a global load
// inside the epilogue would wait for every LDS-DMA still in flight (loads retire in order).  Without bias,
// -0.0 is added (the neutral element: x + -0.0 == x for every x, signed zeros included).
template <bool H, int BM, int BN, int WM, int WN, int KIND, int MI0 = 0, int MI1 = -1, bool PB = false>
__device__ __forceinline__ void epilogue_fast(const GemmP& p, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                              int n0, int wm, int wn, int lane, int bz,
                                              const bf16* braw = nullptr) {
  constexpr int FN = BN / WN / 16;
  constexpr int FM = MI1 < 0 ? BM / WM / 16 : MI1;
  static_assert(FN % 2 == 0, "fragment pairs");
  const int g = lane >> 4, li = lane & 15;
  const int cw = n0 + wn * (BN / WN);                 // wave's first column
  const int sw = (g & 1) * 16 + (g >> 1) * 8;        // this lane's column in a swapped pair
  const bool rd = p.flags & F_ROUND;
  float bv[FN][4];
  if constexpr (PB) {
    const bool hb = p.flags & F_BIAS;
#pragma unroll
    for (int ni = 0; ni < FN; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[ni][r] = -0.f;
    if (hb) {
#pragma unroll
      for (int ni = 0; ni < FN; ++ni) {
        const bf16x4 t = *(const bf16x4*)(braw + wn * (BN / WN) + ni * 16 + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[ni][r] = e2f<H>(t[r]);
      }
    }
  } else {
#pragma unroll
    for (int ni = 0; ni < FN; ++ni) {
      if (p.flags & F_BIAS) {
        const bf16x4 t = *(const bf16x4*)(p.bias + cw + ni * 16 + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[ni][r] = e2f<H>(t[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[ni][r] = 0.f;
      }
    }
  }
  // Residual operands are loaded a batch of row blocks at a time, before any store of those rows (in-place
  // updates): one memory round trip per batch instead of one per row block (each load waits for everything issued
  // before it, LDS-DMA and the previous batch's stores included).  bf16: 4 row blocks (32 VGPRs, two round trips per
  // tile; round 4: encoder-shape out_proj 352 -> 332 us, fc1-shaped 1240 -> 1204 us, profiles/r04_l_res_epilogue_ab.log;
  // 8 spill); fp32: 2 (32 VGPRs).
  // (EPI_DGELU: the 16-bit pre-activation rows loaded the same way as a bf16 residual)
  constexpr bool R16 = KIND == EPI_RES_BF16 || KIND == EPI_DGELU;
  constexpr int RB = R16 ? 4 : (KIND == EPI_RES_F32 ? 2 : 1);
#pragma unroll
  for (int mb = MI0; mb < FM; mb += RB) {
  u32x4 rball[R16 ? RB : 1][FN / 2];
  f32x4 rfall[KIND == EPI_RES_F32 ? RB : 1][FN];
#pragma unroll
  for (int q = 0; q < RB && mb + q < FM; ++q) {
    const int64_t m = m0 + wm * (BM / WM) + (mb + q) * 16 + li;
    if constexpr (KIND == EPI_RES_BF16) {
      const bf16* rrow = (const bf16*)p.res + bz * p.sR + m * p.ldr + cw;
#pragma unroll
      for (int np = 0; np < FN / 2; ++np)
        rball[q][np] = *(const u32x4*)(rrow + np * 32 + sw);
    }
    if constexpr (KIND == EPI_DGELU) {
      const bf16* arow = p.aux + bz * p.sAux + m * p.ldaux + cw;
#pragma unroll
      for (int np = 0; np < FN / 2; ++np)
        rball[q][np] = *(const u32x4*)(arow + np * 32 + sw);
    }
    if constexpr (KIND == EPI_RES_F32) {
      const float* rrow = (const float*)p.res + bz * p.sR + m * p.ldr + cw;
#pragma unroll
      for (int ni = 0; ni < FN; ++ni)
        rfall[q][ni] = *(const f32x4*)(rrow + ni * 16 + 4 * g);
    }
  }
#pragma unroll
  for (int q = 0; q < RB && mb + q < FM; ++q) {
    const int mi = mb + q;
    const int64_t m = m0 + wm * (BM / WM) + mi * 16 + li;
    const auto& rb = rball[R16 ? q : 0];
    const auto& rf = rfall[KIND == EPI_RES_F32 ? q : 0];
#pragma unroll
    for (int np = 0; np < FN / 2; ++np) {
      float v[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[h][r] = p.alpha * acc[mi][2 * np + h][r] + bv[2 * np + h][r];
      if constexpr (KIND == EPI_STORE_BF16) {
        bf16* crow = (bf16*)p.C + bz * p.sC + m * p.ldc + cw;
        *(u32x4*)(crow + np * 32 + sw) = pair_to_u4<H>(v[0], v[1]);
      } else if constexpr (KIND == EPI_STORE_F32) {
        float* crow = (float*)p.C + bz * p.sC + m * p.ldc + cw;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = rd ? rnd<H>(v[h][r]) : v[h][r];
          *(f32x4*)(crow + (2 * np + h) * 16 + 4 * g) = o;
        }
      } else if constexpr (KIND == EPI_GELU || KIND == EPI_GELU_AUX) {
        // autocast: the Linear output is bf16.  GELU only: one v_cvt_pk per two values, unpacked (rnd<H> of each
        // value, bit for bit; 2102 vs 2250 instructions per tile and wave, 56 vs 141 s_nop).  With the aux output
        // the per-value rounding stays: swapping the freshly packed words for the aux store serialised the GELU
        // chains (2783 vs 2563 instructions, 623 vs 275 s_nop).
        if constexpr (KIND == EPI_GELU) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t w0 = pack2<H>(v[h][0], v[h][1]), w1 = pack2<H>(v[h][2], v[h][3]);
            v[h][0] = lo_e<H>(w0);
            v[h][1] = hi_e<H>(w0);
            v[h][2] = lo_e<H>(w1);
            v[h][3] = hi_e<H>(w1);
          }
        } else {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[h][r] = rnd<H>(v[h][r]);
          bf16* arow = p.aux + bz * p.sAux + m * p.ldaux + cw;
          *(u32x4*)(arow + np * 32 + sw) = pair_to_u4<H>(v[0], v[1]);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; r += 2) {
            if constexpr (H) {
              v[h][r] = gelu_of<H>(v[h][r]);
              v[h][r + 1] = gelu_of<H>(v[h][r + 1]);
            } else {
              const f32x2 y = gelu_erf2(f32x2{v[h][r], v[h][r + 1]});
              v[h][r] = y.x;
              v[h][r + 1] = y.y;
            }
          }
        bf16* crow = (bf16*)p.C + bz * p.sC + m * p.ldc + cw;
        *(u32x4*)(crow + np * 32 + sw) = pair_to_u4<H>(v[0], v[1]);
      } else if constexpr (KIND == EPI_DGELU) {
        // the generic epilogue's sequence: round the product, times gelu'(pre-activation), round
        float x[4], y[4];
        u4_to_pair<H>(rb[np], x, y);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[0][r] = rnd<H>((rd ? rnd<H>(v[0][r]) : v[0][r]) * gelu_grad_of<H>(x[r]));
          v[1][r] = rnd<H>((rd ? rnd<H>(v[1][r]) : v[1][r]) * gelu_grad_of<H>(y[r]));
        }
        bf16* crow = (bf16*)p.C + bz * p.sC + m * p.ldc + cw;
        *(u32x4*)(crow + np * 32 + sw) = pair_to_u4<H>(v[0], v[1]);
      } else if constexpr (KIND == EPI_RES_BF16) {
        float x[4], y[4];
        u4_to_pair<H>(rb[np], x, y);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[0][r] = (rd ? rnd<H>(v[0][r]) : v[0][r]) + x[r];
          v[1][r] = (rd ? rnd<H>(v[1][r]) : v[1][r]) + y[r];
        }
        if (p.flags & F_CLAMP16) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[0][r] = clamp_f16_stream(rnd<H>(v[0][r]));
            v[1][r] = clamp_f16_stream(rnd<H>(v[1][r]));
          }
        }
        bf16* crow = (bf16*)p.C + bz * p.sC + m * p.ldc + cw;
        *(u32x4*)(crow + np * 32 + sw) = pair_to_u4<H>(v[0], v[1]);
      } else {   // EPI_RES_F32
        float* crow = (float*)p.C + bz * p.sC + m * p.ldc + cw;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (rd ? rnd<H>(v[h][r]) : v[h][r]) + rf[2 * np + h][r];
          *(f32x4*)(crow + (2 * np + h) * 16 + 4 * g) = o;
        }
      }
    }
  }
  }
}

// DG: the kernel runs dX products (transposed B), the only ones with a GELU-backward epilogue
template <bool H, int BM, int BN, int WM, int WN, int MI0 = 0, int MI1 = -1, bool DG = false>
__device__ __forceinline__ void epilogue(const GemmP& p, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                         int n0, int wm, int wn, int lane, int bz) {
  const bool full = (m0 + BM <= p.M) && (n0 + BN <= p.N);
  const int k = full ? p.epi : EPI_GENERIC;
  if constexpr (DG) {
    if (k == EPI_DGELU) {
      epilogue_fast<H, BM, BN, WM, WN, EPI_DGELU, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
      return;
    }
  }
  if (k == EPI_STORE_BF16) epilogue_fast<H, BM, BN, WM, WN, EPI_STORE_BF16, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_STORE_F32) epilogue_fast<H, BM, BN, WM, WN, EPI_STORE_F32, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_GELU) epilogue_fast<H, BM, BN, WM, WN, EPI_GELU, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_GELU_AUX) epilogue_fast<H, BM, BN, WM, WN, EPI_GELU_AUX, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_RES_BF16) epilogue_fast<H, BM, BN, WM, WN, EPI_RES_BF16, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_RES_F32) epilogue_fast<H, BM, BN, WM, WN, EPI_RES_F32, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  else epilogue_generic<H, BM, BN, WM, WN, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
}

// The same with the kind fixed at compile time (KIND < 0: the runtime dispatch above); ragged tiles
// take the generic form.
template <bool H, int BM, int BN, int WM, int WN, int KIND, int MI0 = 0, int MI1 = -1, bool PB = false>
__device__ __forceinline__ void epilogue_k(const GemmP& p, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                           int n0, int wm, int wn, int lane, int bz, const bf16* braw = nullptr) {
  if constexpr (KIND < 0) {
    epilogue<H, BM, BN, WM, WN, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  } else if constexpr (KIND == EPI_GENERIC) {
    epilogue_generic<H, BM, BN, WM, WN, MI0, MI1>(p, acc, m0, n0, wm, wn, lane, bz);
  } else {
    if constexpr (H && PB) {
      // fp16 persistent kernel: full tiles only (the host launches it for M, N multiples of 256).  Compiling
      // the generic edge-tile epilogue into the fp16 instantiations spilled their accumulators (528 B of
      // scratch, 3-5x slower on c4's encoder): the fp16 rounding barrier of f2e keeps every per-element path
      // of that epilogue from folding, and its register demand spills the whole kernel.
      epilogue_fast<H, BM, BN, WM, WN, KIND, MI0, MI1, PB>(p, acc, m0, n0, wm, wn, lane, bz, braw);
    } else if ((m0 + BM <= p.M) && (n0 + BN <= p.N)) {
      epilogue_fast<H, BM, BN, WM, WN, KIND, MI0, MI1, PB>(p, acc, m0, n0, wm, wn, lane, bz, braw);
    } else {
      epilogue_generic<H, BM, BN, WM, WN, MI0, MI1, true>(p, acc, m0, n0, wm, wn, lane, bz);
    }
  }
}

__device__ __forceinline__ bool pp_tile(const GemmP& p, int i, int& m0, int& n0, int& bz) {
  const int vb = blockIdx.x + gridDim.x * i;
  if (vb >= p.tiles_total) return false;
  const int nwg = p.tiles_total;
  const int q = nwg / 8, rr = nwg % 8, xcd = vb % 8;
  const int tid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + vb / 8;
  bz = tid / p.tiles_mn;
  int mt, nt;
  tile_coords(tid - bz * p.tiles_mn, p, mt, nt);
  m0 = mt * 256;
  n0 = nt * 256;
  return true;
}

}  // namespace twg
