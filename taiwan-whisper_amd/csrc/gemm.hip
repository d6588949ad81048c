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
  int tiles_n, tiles_mn;
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
  const int mt = tid / p.tiles_n, nt = tid % p.tiles_n;
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

  // ---- epilogue: lane holds C[m][n..n+3] per fragment
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

template <bool AT, bool BT, int BM, int BN, int WM, int WN, int STAGES>
void launch(GemmP p, int batch, hipStream_t stream) {
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_mn = p.tiles_n * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_kernel<AT, BT, BM, BN, WM, WN, STAGES>), dim3(p.tiles_mn, 1, batch), dim3(WM * WN * 64), 0,
                     stream, p);
}

template <bool AT, bool BT>
void dispatch(GemmP p, int batch, hipStream_t stream, int tile) {
  if (tile == 256) launch<AT, BT, 256, 256, 2, 4, 2>(p, batch, stream);
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
  // 256x256 tiles (8 waves) when the problem has enough tiles to fill the chip, else 128x128
  const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256) * batch;
  const int64_t t2561 = (int64_t)((M + 255) / 256) * ((N + 127) / 128) * batch;
  // measured crossovers (tools/bench_gemm.py, r01): the 3-stage 256x128 ring wins by 8-12% on
  // the K<=4096 NN/NT shapes; long-K reductions (dW, dX of the vocab head) keep the 2-stage
  // 256x256 tile, small grids the 128x128 one.
  int tile = (t256 >= 1000 && K >= 256) ? 256 : 128;
  if (!a_trans && K >= 256 && K <= 4096 && t2561 >= 1500) tile = 2561;
  if (flags & 256) tile = 128;        // forced tile (benchmarking / A-B comparisons)
  if (flags & 512) tile = 256;
  if (flags & 1024) tile = 2561;      // 256x128, 3-stage ring
  const int64_t ntiles = tile == 256 ? t256 / batch : (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (ntiles > 0x7fffffff || batch > 65535) return TW_EINVAL;
  if (!a_trans && !b_trans) dispatch<false, false>(p, batch, stream, tile);
  else if (!a_trans && b_trans) dispatch<false, true>(p, batch, stream, tile);
  else if (a_trans && !b_trans) dispatch<true, false>(p, batch, stream, tile);
  else dispatch<true, true>(p, batch, stream, tile);
  TW_CHECK_LAUNCH();
  return TW_OK;
}
