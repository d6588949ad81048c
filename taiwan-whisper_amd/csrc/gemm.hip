// bf16 MFMA GEMM with fused epilogues (gfx950).
//
//   C[b][m][n] = epilogue( alpha * sum_k A[b][m][k] * B[b][n][k] )
//
// A is K-major ([M][K], lda) or MN-major ([K][M], lda) — template AT;
// B is K-major ([N][K], ldb, the nn.Linear weight layout) or MN-major ([K][N]) — BT.
// So one kernel serves forward (AT=0,BT=0: X·Wᵀ), dX (AT=0,BT=1: dY·W) and
// dW (AT=1,BT=1: dYᵀ·X) of every Linear / conv-as-GEMM of the Whisper step
// (SURVEY.md §2.2 K2/K4/K6/K8/K10).
//
// Tiling: 128x128x64 per 256-thread workgroup (2x2 waves of 64x64), v_mfma_f32_16x16x32_bf16,
// operands staged HBM->LDS with buffer_load ... lds (16 B per lane, out-of-range lanes
// read zero through the buffer descriptor), two LDS stages (64 KiB), one barrier per K-step.
// K-major LDS images: 128-B rows, 16-B chunk c of row r at c ^ (r & 7) (ds_read_b128
// conflict-free).  MN-major images: 256-B k-rows, 32-B slot s of k-row r at
// s ^ ((r & 3) | ((r >> 3) & 1) << 2), read with ds_read_b64_tr_b16 (conflict-free).
// The MFMA is issued with operands swapped (Bfrag, Afrag) so each lane ends up holding
// 4 consecutive output columns of one row: 8/16-B stores in the epilogue.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <vector>

namespace {

constexpr int BK = 64;

enum {
  F_BIAS = 1,      // v += bias[n]            (bias bf16, autocast casts it)
  F_ROUND = 2,     // v = bf16(v)             (autocast Linear output)
  F_GELU = 4,      // [aux = v]; v = bf16(gelu(v))
  F_RES = 8,       // v = res[m % res_mod][n] + v
  F_ACCUM = 16,    // v += C_old
  F_AUX_OUT = 32,  // store pre-activation to aux (with F_GELU)
  F_DGELU = 64,    // v = bf16(v * gelu'(aux[m][n]))  (gelu backward, aux = pre-activation)
};

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
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void epilogue_generic(const GemmP& p, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                         int n0, int wm, int wn, int lane, int bz) {
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  const int g = lane >> 4, li = lane & 15;
  const int flags = p.flags;
  char* C = (char*)p.C;
  const bool full_tile = (m0 + BM <= p.M) && (n0 + BN <= p.N) && ((p.ldc & 3) == 0) &&
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
        for (int r = 0; r < 4; ++r) bv[ni][r] = bf2f(t[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[ni][r] = 0.f;
      }
    }
#pragma unroll
    for (int mi = 0; mi < FM; ++mi) {
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
            for (int r = 0; r < 4; ++r) ex[ni][r] = bf2f(t[r]);
          } else {
            const bool res = flags & F_RES;
            const void* src = res ? p.res : (const void*)C;
            const int dt = res ? p.res_dtype : p.c_dtype;
            const int64_t o = res ? bz * p.sR + (int64_t)m * p.ldr + n : bz * p.sC + (int64_t)m * p.ldc + n;
            if (dt == TW_BF16) {
              const bf16x4 t = *(const bf16x4*)((const bf16*)src + o);
#pragma unroll
              for (int r = 0; r < 4; ++r) ex[ni][r] = bf2f(t[r]);
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
          if (flags & F_ROUND) v[r] = rbf(v[r]);
          if (flags & F_DGELU) v[r] = rbf(v[r] * gelu_erf_grad(ex[ni][r]));
        }
        if (flags & F_GELU) {
          if (flags & F_AUX_OUT)
            *(bf16x4*)(p.aux + bz * p.sAux + (int64_t)m * p.ldaux + n) =
                bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = rbf(gelu_erf(v[r]));
        }
        if (flags & (F_RES | F_ACCUM)) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += ex[ni][r];
        }
        const int64_t co = bz * p.sC + (int64_t)m * p.ldc + n;
        if (p.c_dtype == TW_BF16) *(bf16x4*)((bf16*)C + co) = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
        else *(f32x4*)((float*)C + co) = f32x4{v[0], v[1], v[2], v[3]};
      }
    }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < FM; ++mi) {
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
        for (int r = 0; r < nv; ++r) v[r] += bf2f(p.bias[n + r]);
      }
      if (flags & F_ROUND) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = rbf(v[r]);
      }
      if (flags & F_DGELU) {
        const bf16* ax = p.aux + bz * p.sAux + (int64_t)m * p.ldaux + n;
        for (int r = 0; r < nv; ++r) v[r] = rbf(v[r] * gelu_erf_grad(bf2f(ax[r])));
      }
      if (flags & F_GELU) {
        if (flags & F_AUX_OUT) {
          bf16* ax = p.aux + bz * p.sAux + (int64_t)m * p.ldaux + n;
          for (int r = 0; r < nv; ++r) ax[r] = f2bf(v[r]);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = rbf(gelu_erf(v[r]));
      }
      if (flags & F_RES) {
        const int mr = p.res_mod > 0 ? (m % p.res_mod) : m;
        const int64_t ro = bz * p.sR + (int64_t)mr * p.ldr + n;
        for (int r = 0; r < nv; ++r) v[r] += ld_as_f32(p.res, p.res_dtype, ro + r);
      }
      const int64_t co = bz * p.sC + (int64_t)m * p.ldc + n;
      if (flags & F_ACCUM) {
        for (int r = 0; r < nv; ++r) v[r] += ld_as_f32(C, p.c_dtype, co + r);
      }
      if (p.c_dtype == TW_BF16) {
        bf16* cp = (bf16*)C + co;
        if (full && ((co & 3) == 0)) {
          *(bf16x4*)cp = bf16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
        } else {
          for (int r = 0; r < nv; ++r) cp[r] = f2bf(v[r]);
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
enum { EPI_GENERIC = 0, EPI_STORE_BF16, EPI_STORE_F32, EPI_GELU, EPI_GELU_AUX, EPI_RES_BF16, EPI_RES_F32 };

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  return __builtin_bit_cast(uint32_t, bf16x2{f2bf(a), f2bf(b)});
}
__device__ __forceinline__ float lo_bf(uint32_t u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __builtin_bit_cast(float, u & 0xffff0000u); }

// fragments X (ni) and Y (ni+1), 4 floats each -> this lane's 16 B of the pair (swapped layout)
__device__ __forceinline__ u32x4 pair_to_u4(const float (&x)[4], const float (&y)[4]) {
  const uint32_t x0 = pack2(x[0], x[1]), x1 = pack2(x[2], x[3]);
  const uint32_t y0 = pack2(y[0], y[1]), y1 = pack2(y[2], y[3]);
  const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
  return u32x4{s0[0], s1[0], s0[1], s1[1]};
}
// inverse: this lane's 16 B of the pair (swapped layout) -> fragments X, Y as floats
__device__ __forceinline__ void u4_to_pair(u32x4 r, float (&x)[4], float (&y)[4]) {
  const auto s0 = __builtin_amdgcn_permlane16_swap(r[0], r[2], false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(r[1], r[3], false, false);
  x[0] = lo_bf(s0[0]); x[1] = hi_bf(s0[0]); x[2] = lo_bf(s1[0]); x[3] = hi_bf(s1[0]);
  y[0] = lo_bf(s0[1]); y[1] = hi_bf(s0[1]); y[2] = lo_bf(s1[1]); y[3] = hi_bf(s1[1]);
}

template <int BM, int BN, int WM, int WN, int KIND>
__device__ __forceinline__ void epilogue_fast(const GemmP& p, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                              int n0, int wm, int wn, int lane, int bz) {
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  static_assert(FN % 2 == 0, "fragment pairs");
  const int g = lane >> 4, li = lane & 15;
  const int cw = n0 + wn * (BN / WN);                 // wave's first column
  const int sw = (g & 1) * 16 + (g >> 1) * 8;        // this lane's column in a swapped pair
  const bool rnd = p.flags & F_ROUND;
  float bv[FN][4];
#pragma unroll
  for (int ni = 0; ni < FN; ++ni) {
    if (p.flags & F_BIAS) {
      const bf16x4 t = *(const bf16x4*)(p.bias + cw + ni * 16 + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[ni][r] = bf2f(t[r]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[ni][r] = 0.f;
    }
  }
#pragma unroll
  for (int mi = 0; mi < FM; ++mi) {
    const int64_t m = m0 + wm * (BM / WM) + mi * 16 + li;
    // residual operand of the whole row block, loaded before any store of it
    u32x4 rb[FN / 2];
    f32x4 rf[FN];
    if constexpr (KIND == EPI_RES_BF16) {
      const bf16* rrow = (const bf16*)p.res + bz * p.sR + m * p.ldr + cw;
#pragma unroll
      for (int np = 0; np < FN / 2; ++np) rb[np] = *(const u32x4*)(rrow + np * 32 + sw);
    }
    if constexpr (KIND == EPI_RES_F32) {
      const float* rrow = (const float*)p.res + bz * p.sR + m * p.ldr + cw;
#pragma unroll
      for (int ni = 0; ni < FN; ++ni) rf[ni] = *(const f32x4*)(rrow + ni * 16 + 4 * g);
    }
#pragma unroll
    for (int np = 0; np < FN / 2; ++np) {
      float v[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[h][r] = p.alpha * acc[mi][2 * np + h][r] + bv[2 * np + h][r];
      if constexpr (KIND == EPI_STORE_BF16) {
        bf16* crow = (bf16*)p.C + bz * p.sC + m * p.ldc + cw;
        *(u32x4*)(crow + np * 32 + sw) = pair_to_u4(v[0], v[1]);
      } else if constexpr (KIND == EPI_STORE_F32) {
        float* crow = (float*)p.C + bz * p.sC + m * p.ldc + cw;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = rnd ? rbf(v[h][r]) : v[h][r];
          *(f32x4*)(crow + (2 * np + h) * 16 + 4 * g) = o;
        }
      } else if constexpr (KIND == EPI_GELU || KIND == EPI_GELU_AUX) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[h][r] = rbf(v[h][r]);     // autocast: Linear output is bf16
        if constexpr (KIND == EPI_GELU_AUX) {
          bf16* arow = p.aux + bz * p.sAux + m * p.ldaux + cw;
          *(u32x4*)(arow + np * 32 + sw) = pair_to_u4(v[0], v[1]);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int r = 0; r < 4; ++r) v[h][r] = gelu_erf(v[h][r]);
        bf16* crow = (bf16*)p.C + bz * p.sC + m * p.ldc + cw;
        *(u32x4*)(crow + np * 32 + sw) = pair_to_u4(v[0], v[1]);
      } else if constexpr (KIND == EPI_RES_BF16) {
        float x[4], y[4];
        u4_to_pair(rb[np], x, y);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[0][r] = (rnd ? rbf(v[0][r]) : v[0][r]) + x[r];
          v[1][r] = (rnd ? rbf(v[1][r]) : v[1][r]) + y[r];
        }
        bf16* crow = (bf16*)p.C + bz * p.sC + m * p.ldc + cw;
        *(u32x4*)(crow + np * 32 + sw) = pair_to_u4(v[0], v[1]);
      } else {   // EPI_RES_F32
        float* crow = (float*)p.C + bz * p.sC + m * p.ldc + cw;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x4 o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (rnd ? rbf(v[h][r]) : v[h][r]) + rf[2 * np + h][r];
          *(f32x4*)(crow + (2 * np + h) * 16 + 4 * g) = o;
        }
      }
    }
  }
}

template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void epilogue(const GemmP& p, const f32x4 (&acc)[BM / WM / 16][BN / WN / 16], int m0,
                                         int n0, int wm, int wn, int lane, int bz) {
  const bool full = (m0 + BM <= p.M) && (n0 + BN <= p.N);
  const int k = full ? p.epi : EPI_GENERIC;
  if (k == EPI_STORE_BF16) epilogue_fast<BM, BN, WM, WN, EPI_STORE_BF16>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_STORE_F32) epilogue_fast<BM, BN, WM, WN, EPI_STORE_F32>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_GELU) epilogue_fast<BM, BN, WM, WN, EPI_GELU>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_GELU_AUX) epilogue_fast<BM, BN, WM, WN, EPI_GELU_AUX>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_RES_BF16) epilogue_fast<BM, BN, WM, WN, EPI_RES_BF16>(p, acc, m0, n0, wm, wn, lane, bz);
  else if (k == EPI_RES_F32) epilogue_fast<BM, BN, WM, WN, EPI_RES_F32>(p, acc, m0, n0, wm, wn, lane, bz);
  else epilogue_generic<BM, BN, WM, WN>(p, acc, m0, n0, wm, wn, lane, bz);
}

// STAGES-deep LDS ring, prefetch distance STAGES-1; waits are counted (vmcnt = loads of the
// stages allowed to stay in flight) and the barrier is a raw s_barrier, so in-flight LDS-DMA
// survives it (a __syncthreads() would drain vmcnt(0)).
template <bool AT, bool BT, int BM, int BN, int WM, int WN, int STAGES>
__global__ __launch_bounds__(WM * WN * 64, 1) void gemm_kernel(GemmP p) {
  constexpr int NW = WM * WN;
  constexpr int FM = BM / WM / 16, FN = BN / WN / 16;
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int PD = STAGES - 1;                          // prefetch distance (K-steps)
  constexpr int LPS = BM / 8 / NW + BN / 8 / NW;          // LDS-DMA instructions per stage per wave
  __shared__ __attribute__((aligned(16))) char smem[STAGES * (A_BYTES + B_BYTES)];
  const int lane = lane_id();
  const int wave = wave_id_uniform();
  const int wm = wave / WN, wn = wave % WN;
  const int bz = blockIdx.z;
  // XCD-aware bijective remap of the linear tile id
  const int nwg = p.tiles_mn, bid = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = bid % 8;
  const int tid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  int mt, nt;
  tile_coords(tid, p, mt, nt);
  const int n0 = nt * BN, m0 = mt * BM;

  const bf16* A = p.A + bz * p.sA;
  const bf16* B = p.B + bz * p.sB;
  const int K = p.K;
  const int nk = (K + BK - 1) / BK;

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int buf, int kt) {
    char* As = smem + buf * (A_BYTES + B_BYTES);
    char* Bs = As + A_BYTES;
    const int k0 = kt * BK;
    if (AT) stage_mn<BM, NW>(A + (int64_t)k0 * p.lda + m0, p.lda, p.M - m0, K - k0, As, wave, lane);
    else    stage_k<BM, NW>(A + (int64_t)m0 * p.lda + k0, p.lda, p.M - m0, K - k0, As, wave, lane);
    if (BT) stage_mn<BN, NW>(B + (int64_t)k0 * p.ldb + n0, p.ldb, p.N - n0, K - k0, Bs, wave, lane);
    else    stage_k<BN, NW>(B + (int64_t)n0 * p.ldb + k0, p.ldb, p.N - n0, K - k0, Bs, wave, lane);
  };

  for (int s = 0; s < PD; ++s)
    if (s < nk) stage(s, s);
  if (nk >= PD) wait_vm_lgkm0<(PD - 1) * LPS>();     // stage 0 landed, later ones may fly
  else wait_vm_lgkm0<0>();
  __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % STAGES;
    const int nxt = (kt + PD) % STAGES;
    const char* As = smem + cur * (A_BYTES + B_BYTES);
    const char* Bs = As + A_BYTES;
    if constexpr (AT || BT) {
      // transposed (ds_read_b64_tr_b16) reads: fetch both k-halves BEFORE the next stage's
      // LDS-DMA is issued, else the compiler cannot prove they do not alias the DMA and
      // drains vmcnt(0) mid-step (the whole load latency exposed every K-step)
      bf16x8 a[2][FM], b[2][FN];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int ni = 0; ni < FN; ++ni)
          b[kk][ni] = BT ? frag_mn<BN>(Bs, wn * (BN / WN) + ni * 16, kk, lane)
                         : frag_k(Bs, wn * (BN / WN) + ni * 16, kk, lane);
#pragma unroll
        for (int mi = 0; mi < FM; ++mi)
          a[kk][mi] = AT ? frag_mn<BM>(As, wm * (BM / WM) + mi * 16, kk, lane)
                         : frag_k(As, wm * (BM / WM) + mi * 16, kk, lane);
      }
      if (kt + PD < nk) stage(nxt, kt + PD);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int mi = 0; mi < FM; ++mi)
#pragma unroll
          for (int ni = 0; ni < FN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[kk][ni], a[kk][mi], acc[mi][ni], 0, 0, 0);
    } else {
      if (kt + PD < nk) stage(nxt, kt + PD);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 a[FM], b[FN];
#pragma unroll
        for (int ni = 0; ni < FN; ++ni) b[ni] = frag_k(Bs, wn * (BN / WN) + ni * 16, kk, lane);
#pragma unroll
        for (int mi = 0; mi < FM; ++mi) a[mi] = frag_k(As, wm * (BM / WM) + mi * 16, kk, lane);
#pragma unroll
        for (int mi = 0; mi < FM; ++mi)
#pragma unroll
          for (int ni = 0; ni < FN; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[ni], a[mi], acc[mi][ni], 0, 0, 0);
      }
    }
    // stage kt+1 must have landed; stages kt+2 .. kt+PD (when issued) may stay in flight
    if (kt + PD < nk) wait_vm_lgkm0<(PD - 1) * LPS>();
    else wait_vm_lgkm0<0>();
    __builtin_amdgcn_s_barrier();
  }

  epilogue<BM, BN, WM, WN>(p, acc, m0, n0, wm, wn, lane, bz);
}

// ---------------------------------------------------------------------------------------------
// Ping-pong 256x256 kernel for K-major A and B (the forward X·Wᵀ of every Linear).
//
// 8 waves as 2 (rows) x 4 (cols), each wave owns 128x64 of C = 4 quadrants of 64x32.  A K-tile
// (BK = 64) is consumed in 4 phases, one quadrant per phase (16 MFMAs):
//   q(0,0): read A-half 0 + B-quarter 0    q(0,1): read B-quarter 1
//   q(1,1): read A-half 1                  q(1,0): read B-quarter 0 again
// LDS = 2 buffers (even / odd K-tile) x 4 regions of 16 KiB:
//   A-half h    : rows  wr*128 + h*64 + [0,64)  for wr = 0,1   (the rows quadrant-row h reads)
//   B-quarter q : cols  wc*64  + q*32 + [0,32)  for wc = 0..3  (the cols quadrant-col q reads)
// so each region's last read in a K-tile is one phase (A-h0: 1, B-q1: 2, A-h1: 3, B-q0: 4), and
// every phase restages exactly one region (2 LDS-DMA per lane) for the K-tile two ahead in the
// same buffer, one phase after that region's last read (reads are retired by lgkmcnt(0) before
// the barrier that ends the reading section).  Waits: vmcnt(6) at phases 4 and 8 = three
// regions left in flight across the barrier (raw s_barrier, never __syncthreads()).
// The two wave rows run one barrier apart (wave-row 1 takes an extra barrier up front): on each
// SIMD (waves w and w+4) one wave issues its 16 MFMAs while the other issues LDS reads and DMA.
// ---------------------------------------------------------------------------------------------
constexpr int PP_REGION = 16384;

// Stage one 16-KiB region (128 source rows x 64 k) with 2 LDS-DMA per lane; region row R maps to
// source row (R >> S) * GS + off + (R & (2^S - 1)).  128-B rows, chunk c of row R at c ^ (R & 7).
template <int S, int GS>
__device__ __forceinline__ void pp_stage(const bf16* base, int64_t ld, int rows_left, int k_left, int off,
                                         char* region, int wave, int lane) {
  const auto rs = make_rsrc(base);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pce = wave + 8 * i;
    const int R = pce * 8 + (lane >> 3);
    const int row = (R >> S) * GS + off + (R & ((1 << S) - 1));
    const int c = (lane & 7) ^ (R & 7);
    const bool ok = (row < rows_left) && (c * 8 < k_left);
    const uint32_t o = ok ? (uint32_t)(((int64_t)row * ld + c * 8) * 2) : TW_OOB;
    buf_load_lds16(rs, region + pce * 1024, o);
  }
}

// Persistent form: gridDim.x (a multiple of 8, <= CUs) workgroups; workgroup b takes the tiles
// of virtual block ids b, b + G, b + 2G, ... (G = gridDim.x), each mapped through the same
// XCD-aware bijective remap as a one-tile-per-block launch, so an XCD keeps walking its own
// contiguous chunk.  The K-tile stream is continuous across tiles (nk rounded up to even; the
// pad K-tile stages zeros), so the next tile's first K-tiles are already in flight while the
// finished tile's epilogue runs (between phases, beside the other wave-row's MFMAs).
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

__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmP p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * PP_REGION];
  const int lane = lane_id();
  const int wave = wave_id_uniform();
  const int wm = wave >> 2, wn = wave & 3;
  const int K = p.K, nk = (K + BK - 1) / BK, nke = (nk + 1) & ~1;
  const int G = gridDim.x;
  const int my_tiles = ((int)blockIdx.x < p.tiles_total) ? (p.tiles_total - (int)blockIdx.x + G - 1) / G : 0;
  const int total = my_tiles * nke;                       // K-tiles this workgroup consumes

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // region r of buffer b: 0,1 = A-half 0,1; 2,3 = B-quarter 0,1.  K-tile g of the stream goes to
  // buffer g & 1.  Tile state is carried incrementally (one pp_tile() per tile); a K-tile past
  // the stream or the pad K-tile stages zeros, keeping the vmcnt counts uniform.
  // (plain scalars, no struct: a struct select here is promoted to LDS by the compiler, and any
  // LDS access it cannot disambiguate from the DMA costs a vmcnt(0) drain)
  auto tile_info = [&](int i, int& m0, int& n0, int& bz, int& kl) {
    const bool live = i < my_tiles && pp_tile(p, i, m0, n0, bz);
    if (!live) { m0 = 0; n0 = 0; bz = 0; }
    kl = live ? K : 0;                       // K extent seen by the stager (0: stage zeros)
  };
  auto reg = [&](int b, int r) -> char* { return smem + (b * 4 + r) * PP_REGION; };
  auto stage = [&](int m0, int n0, int bz, int kl, int kt, int buf, int r) {
    const int k_left = kl - kt * BK;
    if (r < 2)
      pp_stage<6, 128>(p.A + bz * p.sA + (int64_t)m0 * p.lda + kt * BK, p.lda, p.M - m0, k_left, r * 64,
                       reg(buf, r), wave, lane);
    else
      pp_stage<5, 64>(p.B + bz * p.sB + (int64_t)n0 * p.ldb + kt * BK, p.ldb, p.N - n0, k_left, (r - 2) * 32,
                      reg(buf, r), wave, lane);
  };

  bf16x8 a[2][4], bb[2][2];
  auto rdA = [&](int b, int h) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) a[kk][mi] = frag_k(reg(b, h), wm * 64 + mi * 16, kk, lane);
  };
  auto rdB = [&](int b, int qq) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) bb[kk][ni] = frag_k(reg(b, 2 + qq), wn * 32 + ni * 16, kk, lane);
  };
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mma = [&](int qm, int qn) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[qm * 4 + mi][qn * 2 + ni] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[kk][ni], a[kk][mi], acc[qm * 4 + mi][qn * 2 + ni], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };

  // prologue: K-tile 0 whole into buffer 0, K-tile 1 without B-quarter 0 into buffer 1
  int cm, cn, cb, ck;                        // current tile: m0, n0, batch, K extent
  tile_info(0, cm, cn, cb, ck);
  int kt = 0, ti = 0;
  stage(cm, cn, cb, ck, 0, 0, 0); stage(cm, cn, cb, ck, 0, 0, 1);
  stage(cm, cn, cb, ck, 0, 0, 2); stage(cm, cn, cb, ck, 0, 0, 3);
  stage(cm, cn, cb, ck, 1, 1, 0); stage(cm, cn, cb, ck, 1, 1, 3); stage(cm, cn, cb, ck, 1, 1, 1);
  asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
  sync();
  if (wm == 1) sync();                       // stagger the wave rows by one barrier

  for (int g = 0; g < total; g += 2) {
    // K-tiles g, g+1 = (cur, kt), (cur, kt+1); g+2, g+3 = (nxt, k2), (nxt, k2+1)
    const bool last = kt + 2 >= nke;
    int nm = cm, nn = cn, nb = cb, nkl = ck, k2 = kt + 2;
    if (last) {
      tile_info(ti + 1, nm, nn, nb, nkl);
      k2 = 0;
    }
    // even K-tile g from buffer 0
    rdB(0, 0); rdA(0, 0); stage(cm, cn, cb, ck, kt + 1, 1, 2);  mma(0, 0);
    rdB(0, 1);            stage(nm, nn, nb, nkl, k2, 0, 0);     mma(0, 1);
    rdA(0, 1);            stage(nm, nn, nb, nkl, k2, 0, 3);     mma(1, 1);
    rdB(0, 0);            stage(nm, nn, nb, nkl, k2, 0, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");            mma(1, 0);
    // odd K-tile g+1 from buffer 1
    rdB(1, 0); rdA(1, 0); stage(nm, nn, nb, nkl, k2, 0, 2);     mma(0, 0);
    rdB(1, 1);            stage(nm, nn, nb, nkl, k2 + 1, 1, 0); mma(0, 1);
    rdA(1, 1);            stage(nm, nn, nb, nkl, k2 + 1, 1, 3); mma(1, 1);
    rdB(1, 0);            stage(nm, nn, nb, nkl, k2 + 1, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");            mma(1, 0);
    if (last) {                                                 // tile finished
      if (!(p.flags & 4096) || acc[0][0][0] != acc[0][0][0])    // 4096: diagnostic, skip epilogue
        epilogue<256, 256, 2, 4>(p, acc, cm, cn, wm, wn, lane, cb);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      ++ti;
    }
    cm = nm; cn = nn; cb = nb; ck = nkl;
    kt = k2;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");             // no LDS-DMA may outlive the block
  if (wm == 0) sync();                       // balance the stagger barrier
}

template <bool AT, bool BT, int BM, int BN, int WM, int WN, int STAGES>
void launch(GemmP p, int batch, hipStream_t stream) {
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_mn = p.tiles_n * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_kernel<AT, BT, BM, BN, WM, WN, STAGES>), dim3(p.tiles_mn, 1, batch), dim3(WM * WN * 64), 0,
                     stream, p);
}

// ---------------------------------------------------------------------------------------------
// Skinny GEMM for the decode step (M <= 128 rows = the batch of one greedy step, A and B K-major):
// weight streaming.  One 256-thread workgroup per 16-column slice of W (all M rows), the K range
// split over the 4 waves; W fragments load straight from HBM (16 B per lane, each W byte read
// once per step), A fragments from L2 (A is at most 128 x K bf16), MFMA 16x16x32 with swapped
// operands, the 4 wave partials summed through LDS, then the per-element epilogue (every flag).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void epi_element(const GemmP& p, int m, int n, float v) {
  const int flags = p.flags;
  v *= p.alpha;
  if (flags & F_BIAS) v += bf2f(p.bias[n]);
  if (flags & F_ROUND) v = rbf(v);
  if (flags & F_DGELU) v = rbf(v * gelu_erf_grad(bf2f(p.aux[(int64_t)m * p.ldaux + n])));
  if (flags & F_GELU) {
    if (flags & F_AUX_OUT) p.aux[(int64_t)m * p.ldaux + n] = f2bf(v);
    v = rbf(gelu_erf(v));
  }
  if (flags & F_RES) {
    const int mr = p.res_mod > 0 ? (m % p.res_mod) : m;
    v += ld_as_f32(p.res, p.res_dtype, (int64_t)mr * p.ldr + n);
  }
  const int64_t co = (int64_t)m * p.ldc + n;
  if (flags & F_ACCUM) v += ld_as_f32(p.C, p.c_dtype, co);
  if (p.c_dtype == TW_BF16) ((bf16*)p.C)[co] = f2bf(v);
  else ((float*)p.C)[co] = v;
}

template <int MF>
__global__ __launch_bounds__(256, 1) void gemm_skinny_kernel(GemmP p) {
  __shared__ float part[4][MF * 16][17];
  const int lane = lane_id(), wave = wave_id_uniform();
  const int n0 = blockIdx.x * 16;
  const int li = lane & 15, g = lane >> 4;
  const int nk = (p.K + 31) / 32;                         // 32-deep k-steps
  // this workgroup's K chunk (split-K over gridDim.y when the launch has too few workgroups to
  // keep enough weight loads in flight), then split over the 4 waves
  const int cper = (nk + (int)gridDim.y - 1) / (int)gridDim.y;
  const int c_beg = (int)blockIdx.y * cper, c_end = min(nk, c_beg + cper);
  const int per = (c_end - c_beg + 3) / 4;
  const int k_beg = min(c_end, c_beg + wave * per), k_end = min(c_end, k_beg + per);
  f32x4 acc[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wrow = n0 + li;
  const bool wok = wrow < p.N;
  const bf16* wp = p.B + (int64_t)(wok ? wrow : 0) * p.ldb + 8 * g;
  const bf16* ap[MF];
  bool aok[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int m = i * 16 + li;
    aok[i] = m < p.M;
    ap[i] = p.A + (int64_t)(aok[i] ? m : 0) * p.lda + 8 * g;
  }
  auto ldk = [&](const bf16* base, int ks, bool ok) -> bf16x8 {
    const int k = ks * 32 + 8 * g;
    return (ok && k < p.K) ? *(const bf16x8*)(base + ks * 32) : bf16x8{};
  };
  // software pipeline: the fragments of 4 k-steps in flight while the previous 4 compute (the
  // W bytes come from HBM once; a 2-deep loop left the per-k-step latency exposed)
  constexpr int D = 4;
  bf16x8 wb[2][D], ab[2][D][MF];
  auto load_group = [&](int buf, int k0) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const bool in = k0 + j < k_end;
      wb[buf][j] = ldk(wp, k0 + j, wok && in);
#pragma unroll
      for (int i = 0; i < MF; ++i) ab[buf][j][i] = ldk(ap[i], k0 + j, aok[i] && in);
    }
  };
  auto mma_group = [&](int buf) {
#pragma unroll
    for (int j = 0; j < D; ++j)
#pragma unroll
      for (int i = 0; i < MF; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[buf][j], ab[buf][j][i], acc[i], 0, 0, 0);
  };
  if (k_beg < k_end) {
    load_group(0, k_beg);
    int k0 = k_beg;
    for (; k0 + D < k_end; k0 += 2 * D) {
      load_group(1, k0 + D);
      mma_group(0);
      if (k0 + 2 * D < k_end) load_group(0, k0 + 2 * D);
      mma_group(1);
    }
    if (k0 < k_end) mma_group(0);
  }
  // lane holds C[16i + li][n0 + 4g + r]
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wave][i * 16 + li][4 * g + r] = acc[i][r];
  __syncthreads();
  for (int e = threadIdx.x; e < MF * 16 * 16; e += 256) {
    const int m = e >> 4, c = e & 15, n = n0 + c;
    if (m < p.M && n < p.N) {
      const float v = part[0][m][c] + part[1][m][c] + part[2][m][c] + part[3][m][c];
      if (p.ws) p.ws[((int64_t)blockIdx.y * p.M + m) * p.N + n] = v;
      else epi_element(p, m, n, v);
    }
  }
}

// sum of the split-K partials of the skinny kernel (in chunk order) + the full epilogue
__global__ __launch_bounds__(256) void skinny_reduce_kernel(GemmP p, int S) {
  const int64_t total = (int64_t)p.M * p.N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    float v = p.ws[i];
    for (int s = 1; s < S; ++s) v += p.ws[s * total + i];
    epi_element(p, (int)(i / p.N), (int)(i % p.N), v);
  }
}

void launch_skinny(GemmP p, hipStream_t stream, int S = 1) {
  const dim3 grid((p.N + 15) / 16, S);
  const int mf = (p.M + 15) / 16;
  switch (mf) {
    case 1: hipLaunchKernelGGL(gemm_skinny_kernel<1>, grid, dim3(256), 0, stream, p); break;
    case 2: hipLaunchKernelGGL(gemm_skinny_kernel<2>, grid, dim3(256), 0, stream, p); break;
    case 3:
    case 4: hipLaunchKernelGGL(gemm_skinny_kernel<4>, grid, dim3(256), 0, stream, p); break;
    default: hipLaunchKernelGGL(gemm_skinny_kernel<8>, grid, dim3(256), 0, stream, p); break;
  }
}

// Host: the specialised epilogue a call qualifies for (alignment for 16-B vectors included).
int pick_epilogue(const GemmP& p, int batch) {
  const int f = p.flags & 0xff;
  auto a16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  const bool c8 = (p.ldc % 8) == 0 && (batch == 1 || (p.sC % 8) == 0) && a16(p.C);
  const bool c4 = (p.ldc % 4) == 0 && (batch == 1 || (p.sC % 4) == 0) && a16(p.C);
  const bool b4 = !(f & F_BIAS) || ((uintptr_t)p.bias & 7) == 0;
  if (!b4) return EPI_GENERIC;
  if ((f & ~(F_BIAS | F_ROUND)) == 0) {
    if (p.c_dtype == TW_BF16 && c8) return EPI_STORE_BF16;
    if (p.c_dtype == TW_F32 && c4) return EPI_STORE_F32;
    return EPI_GENERIC;
  }
  if ((f & ~(F_BIAS | F_AUX_OUT)) == (F_ROUND | F_GELU) && p.c_dtype == TW_BF16 && c8) {
    if (!(f & F_AUX_OUT)) return EPI_GELU;
    const bool x8 = (p.ldaux % 8) == 0 && (batch == 1 || (p.sAux % 8) == 0) && a16(p.aux);
    return x8 ? EPI_GELU_AUX : EPI_GENERIC;
  }
  if ((f & ~(F_BIAS | F_ROUND)) == F_RES && p.res_mod == 0 && p.res_dtype == p.c_dtype) {
    if (p.c_dtype == TW_BF16 && c8 && (p.ldr % 8) == 0 && (batch == 1 || (p.sR % 8) == 0) && a16(p.res))
      return EPI_RES_BF16;
    if (p.c_dtype == TW_F32 && c4 && (p.ldr % 4) == 0 && (batch == 1 || (p.sR % 4) == 0) && a16(p.res))
      return EPI_RES_F32;
  }
  return EPI_GENERIC;
}

void launch_pp(GemmP p, int batch, hipStream_t stream) {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n >= 8 ? n : 8;
  }();
  p.tiles_n = (p.N + 255) / 256;
  p.tiles_mn = p.tiles_n * ((p.M + 255) / 256);
  p.tiles_total = p.tiles_mn * batch;
  int grid = p.tiles_total <= cus ? p.tiles_total : (cus & ~7);
  if (p.flags & 8192) grid = p.tiles_total;   // diagnostic: one tile per workgroup
  hipLaunchKernelGGL(gemm_pp_kernel, dim3(grid), dim3(512), 0, stream, p);
}

// ---------------------------------------------------------------------------------------------
// Split-K for weight gradients (dW = dYᵀ·X: both operands MN-major, K = tokens, few output tiles):
// the K range is cut into S chunks run as S batch entries of the 128x128 kernel into an fp32
// workspace, then one pass sums the chunks in order and applies the epilogue
//     C = [C +] round?(alpha * sum_s ws[s])
// (bf16 rounding point of the autocast product as in the unsplit kernel; the fp32 sum over K is
// regrouped by chunk).  Workspace: splitk_workspace (per device, never freed).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int S, int64_t split_stride,
                                                            float* __restrict__ C, int64_t ldc, int M, int N,
                                                            float alpha, int round, int accum) {
  const int n4 = N >> 2;
  const int64_t total = (int64_t)M * n4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / n4), c = (int)(i - (int64_t)m * n4) * 4;
    const float* w = ws + (int64_t)m * N + c;
    f32x4 a = *(const f32x4*)w;
    for (int s = 1; s < S; ++s) a += *(const f32x4*)(w + s * split_stride);
    float* cp = C + (int64_t)m * ldc + c;
    f32x4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = round ? rbf(alpha * a[r]) : alpha * a[r];
    if (accum) o += *(const f32x4*)cp;
    *(f32x4*)cp = o;
  }
}

// Split-K workspace: one block per device, grown (never freed: a captured HIP graph may hold the
// pointer of an older block, so old blocks are kept) outside stream capture only.  GEMMs of one
// device are issued from one stream at a time (the trainer's and the decoder's current stream).
void* splitk_workspace(hipStream_t stream, size_t bytes) {
  static std::mutex mu;
  static std::vector<std::pair<int, std::pair<void*, size_t>>> cur;   // device -> (ptr, bytes)
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream, &cap);
  std::lock_guard<std::mutex> lock(mu);
  for (auto& e : cur)
    if (e.first == dev) {
      if (e.second.second >= bytes) return e.second.first;
      if (cap != hipStreamCaptureStatusNone) return nullptr;
      void* ptr = nullptr;
      if (hipMalloc(&ptr, bytes) != hipSuccess) return nullptr;
      e.second = {ptr, bytes};                                           // the old block stays allocated
      return ptr;
    }
  if (cap != hipStreamCaptureStatusNone) return nullptr;
  void* ptr = nullptr;
  if (hipMalloc(&ptr, bytes) != hipSuccess) return nullptr;
  cur.push_back({dev, {ptr, bytes}});
  return ptr;
}

// S for a dW-shaped call, 0 = no split: fewer than 512 128x128 tiles, K split into S equal chunks of
// >= 1024 until >= 512 workgroups; fp32 output, flags within {ROUND, ACCUM}.
int splitk_factor(const GemmP& p, int batch, int a_trans, int b_trans) {
  if (!a_trans || !b_trans || batch != 1 || p.c_dtype != TW_F32) return 0;
  if (p.flags & ~(F_ROUND | F_ACCUM) & 0xff) return 0;
  if ((p.N & 3) || (p.ldc & 3) || ((uintptr_t)p.C & 15)) return 0;
  const int64_t tiles = (int64_t)((p.M + 127) / 128) * ((p.N + 127) / 128);
  if (tiles >= 512) return 0;
  for (int S = 2; S <= 16; S *= 2) {
    if (p.K % S != 0 || p.K / S < 1024) break;      // chunk tails are masked like any K tail
    if (tiles * S >= 512) return S;
  }
  return 0;
}

template <bool AT, bool BT>
void dispatch(GemmP p, int batch, hipStream_t stream, int tile) {
  if (tile == 2562 && !AT && !BT) launch_pp(p, batch, stream);
  else if (tile == 256) launch<AT, BT, 256, 256, 2, 4, 2>(p, batch, stream);
  else if (tile == 2561) launch<AT, BT, 256, 128, 4, 2, 3>(p, batch, stream);
  else launch<AT, BT, 128, 128, 2, 2, 2>(p, batch, stream);
}

}  // namespace

extern "C" int tw_gemm_bf16(const void* A, int64_t lda, int a_trans, const void* B, int64_t ldb, int b_trans,
                            void* C, int64_t ldc, int c_dtype, int M, int N, int K, int batch,
                            int64_t sA, int64_t sB, int64_t sC, float alpha, const void* bias,
                            const void* res, int64_t ldr, int64_t sR, int res_dtype, int res_mod,
                            void* aux, int64_t ldaux, int64_t sAux, int flags, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return TW_OK;
  if (K <= 0) return TW_EINVAL;
  if ((!a_trans || !b_trans) && (K % 8) != 0) return TW_EINVAL;  // 16-B k-chunks of K-major operands
  if (a_trans && (M % 8) != 0) return TW_EINVAL;                // 16-B column chunks
  if (b_trans && (N % 8) != 0) return TW_EINVAL;
  if ((lda % 8) != 0 || (ldb % 8) != 0) return TW_EINVAL;       // 16-B aligned rows / k-rows
  if (((uintptr_t)A & 15) || ((uintptr_t)B & 15)) return TW_EINVAL;
  if ((flags & F_BIAS) && !bias) return TW_EINVAL;
  if ((flags & F_RES) && !res) return TW_EINVAL;
  if ((flags & (F_AUX_OUT | F_DGELU)) && !aux) return TW_EINVAL;
  if (c_dtype != TW_F32 && c_dtype != TW_BF16) return TW_EUNSUPPORTED;
  GemmP p;
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.C = C;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.sA = sA; p.sB = sB; p.sC = sC; p.alpha = alpha; p.bias = (const bf16*)bias;
  p.res = res; p.ldr = ldr; p.sR = sR; p.res_dtype = res_dtype; p.res_mod = res_mod;
  p.aux = (bf16*)aux; p.ldaux = ldaux; p.sAux = sAux; p.c_dtype = c_dtype; p.flags = flags;
  p.ws = nullptr;
  static const int env_group = [] {
    const char* e = getenv("TW_GEMM_GROUP_M");   // A/B sweeps only (tools/bench_gemm.py)
    return e ? atoi(e) : 0;
  }();
  p.group_m = env_group > 0 ? env_group : 1;
  p.epi = pick_epilogue(p, batch);
  // 256x256 tiles (8 waves) when the problem has enough tiles to fill the chip, else 128x128
  const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256) * batch;
  // measured crossovers (tools/bench_gemm.py, r01, specialised epilogues): the persistent 256x256
  // ping-pong kernel wins every large K-major/K-major shape (1.05-1.27 PFLOP/s); the 2-stage
  // 256x256 tile the large transposed ones; 128x128 the small grids (< ~1000 256-tiles).  The
  // 256x128 3-stage ring is kept as a forced variant only.
  int tile = (t256 >= 1000 && K >= 256) ? 256 : 128;
  if (tile == 256 && !a_trans && !b_trans) tile = 2562;
  if (flags & 256) tile = 128;        // forced tile (benchmarking / A-B comparisons)
  if (flags & 512) tile = 256;
  if (flags & 1024) tile = 2561;      // 256x128, 3-stage ring
  if (flags & 2048) tile = 2562;      // 256x256 ping-pong (K-major A and B only)
  const int64_t ntiles = (tile == 256 || tile == 2562) ? t256 / batch : (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (ntiles > 0x7fffffff || ntiles * batch > 0x7fffffff || batch > 65535) return TW_EINVAL;
  // decode-step GEMMs (tools/bench_skinny.py, r01): the weight-streaming kernel wins for N <= 3840
  // (and N <= 8192 at M <= 64); the LM head and wide M=128 GEMMs stream faster as 128x128 tiles
  const bool skinny = !a_trans && !b_trans && batch == 1 && M <= 128 && (N <= 4096 || (M <= 64 && N <= 8192)) &&
                      !(flags & (256 | 512 | 1024 | 2048));
  if (skinny && ((uintptr_t)A & 15) == 0) {
    // decode-step GEMMs: stream W once.  With fewer than 512 workgroups and M > 32 the K range is
    // also split over workgroups (chunks of >= 4 k-steps) into fp32 partials, reduced with the
    // epilogue (c4 batch 64 / 128: -3 / -4 % per step; at batch 1 the extra launch loses 9 %).
    p.ws = nullptr;
    const int nwg = (N + 15) / 16, nk = (K + 31) / 32;
    int S = std::min((512 + nwg - 1) / nwg, nk / 4);
    if ((flags & 16384) || M <= 32) S = 1;          // small batches: the reduce launch costs more than it saves
    void* ws = S > 1 ? splitk_workspace(stream, (size_t)S * M * N * sizeof(float)) : nullptr;
    if (ws) {
      p.ws = (float*)ws;
      launch_skinny(p, stream, S);
      TW_CHECK_LAUNCH();
      const int64_t total = (int64_t)M * N;
      hipLaunchKernelGGL(skinny_reduce_kernel, dim3((int)std::min<int64_t>((total + 255) / 256, 2048)), dim3(256), 0,
                         stream, p, S);
    } else {
      launch_skinny(p, stream);
    }
    TW_CHECK_LAUNCH();
    return TW_OK;
  }
  if (!(flags & (16384 | 256 | 512 | 1024 | 2048))) {   // 16384: no split-K; forced tiles: A/B runs
    const int S = splitk_factor(p, batch, a_trans, b_trans);
    const size_t bytes = (size_t)S * M * N * sizeof(float);
    void* ws = (S > 0 && bytes <= ((size_t)1 << 30)) ? splitk_workspace(stream, bytes) : nullptr;
    if (ws) {
      GemmP q = p;
      const int Kc = K / S;
      q.K = Kc;
      q.sA = (int64_t)Kc * lda;                      // A is [K][M] (lda), B is [K][N] (ldb)
      q.sB = (int64_t)Kc * ldb;
      q.C = ws; q.ldc = N; q.sC = (int64_t)M * N; q.c_dtype = TW_F32;
      q.alpha = 1.f; q.flags = 0; q.bias = nullptr; q.res = nullptr; q.aux = nullptr;
      q.epi = pick_epilogue(q, S);
      launch<true, true, 128, 128, 2, 2, 2>(q, S, stream);
      TW_CHECK_LAUNCH();
      const int64_t work = (int64_t)M * (N / 4);
      const int grid = (int)std::min<int64_t>((work + 255) / 256, 4096);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, stream, (const float*)ws, S,
                         (int64_t)M * N, (float*)C, ldc, M, N, alpha, (flags & F_ROUND) ? 1 : 0,
                         (flags & F_ACCUM) ? 1 : 0);
      TW_CHECK_LAUNCH();
      return TW_OK;
    }
  }
  if (!a_trans && !b_trans) dispatch<false, false>(p, batch, stream, tile);
  else if (!a_trans && b_trans) dispatch<false, true>(p, batch, stream, tile);
  else if (a_trans && !b_trans) dispatch<true, false>(p, batch, stream, tile);
  else dispatch<true, true>(p, batch, stream, tile);
  TW_CHECK_LAUNCH();
  return TW_OK;
}
