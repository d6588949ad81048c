// Flash attention, head dim 64, bf16 in/out, fp32 softmax:
//   encoder self-attention (1500 x 1500), decoder causal self-attention (447 x 447) and
//   cross-attention (447 x 1500) of HF WhisperAttention (modeling_whisper.py:265-350;
//   q pre-scaled by hd^-0.5 -> here `scale` is applied to the fp32 scores, identical
//   because 2^-3 scaling is exact).
//
// Layout: rows of [B*T][ld] with head h at columns h*64 .. h*64+63, so Q/K/V are read
// in place from the fused QKV (or KV) projection output and O is written where out_proj
// reads it.  LSE [B][H][Tq] (natural log of the scaled-score row sum) is kept for the
// backward pass.
//
// MFMA v_mfma_f32_16x16x32_bf16 in the "swapped" orientation: S^T = K·Q^T, so each lane
// holds 4 keys of one query; the probabilities then ARE the B operand of O^T = V^T·P^T
// (accumulator-as-operand, keys in permuted order 4g+r / 16+4g+r) and V^T comes from
// ds_read_b64_tr_b16 reads of a row-major V tile.  Every LDS tile is [64 rows][64] bf16
// with 16-B chunk c of row r stored at c ^ (r & 7): conflict-free for both the ds_read_b128
// row reads and the transposed reads.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace {

constexpr int QW = 32;          // query rows per wave
constexpr int QB = 4 * QW;      // query rows per workgroup
constexpr int KT = 64;          // keys per LDS tile
constexpr int TB = KT * 64 * 2; // bytes per [64][64] bf16 tile

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int swz(int r, int c) { return r * 128 + ((c ^ (r & 7)) << 4); }

// [64 rows][64 cols] tile from rows row0.. of a [rows][ld] matrix; rows >= rows_valid read 0.
__device__ __forceinline__ void stage_tile(const bf16* base, int64_t ld, int rows_valid, char* lds, int wave,
                                           int lane) {
  const auto rs = make_rsrc(base);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pce = wave + 4 * i;
    const int r = pce * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const uint32_t off = r < rows_valid ? (uint32_t)(((int64_t)r * ld + c * 8) * 2) : TW_OOB;
    buf_load_lds16(rs, lds + pce * 1024, off);
  }
}

// row fragment: lane gives T[rbase + (l&15)][kk*32 + 8*(l>>4) .. +7]
__device__ __forceinline__ bf16x8 rd_row(const char* t, int rbase, int kk, int lane) {
  const int r = rbase + (lane & 15);
  return *(const bf16x8*)(t + swz(r, kk * 4 + (lane >> 4)));
}

// transposed fragment for k-step s over rows: lane gives T^T[cbase + i][rows perm(s)]
//   elements 0..3: rows s*32 + 4g + 0..3 ; elements 4..7: rows s*32 + 16 + 4g + 0..3
__device__ __forceinline__ bf16x8 rd_tr(const char* t, int cbase, int s, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = cbase + 4 * (i & 3);
  const int r0 = s * 32 + 4 * g + (i >> 2);
  const int r1 = r0 + 16;
  const int ch = col >> 3, inoff = (col & 7) * 2;
  const char* a0 = t + swz(r0, ch) + inoff;
  const char* a1 = t + swz(r1, ch) + inoff;
  s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(uint32_t)(uintptr_t)a0);
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(uint32_t)(uintptr_t)a1);
  s16x8 v = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// global fragment: lane gives M[row0 + (l&15)][kk*32 + 8*(l>>4) .. +7] (zero past rows_valid)
__device__ __forceinline__ bf16x8 ld_frag(const bf16* base, int64_t ld, int row, int rows_valid, int kk, int lane) {
  if (row >= rows_valid) return bf16x8{};
  return *(const bf16x8*)(base + (int64_t)row * ld + kk * 32 + 8 * (lane >> 4));
}

// P as the 16-bit operand type of the instantiation (bf16 words, or fp16 words for the fp16 path)
template <bool H>
__device__ __forceinline__ bf16x8 pack8e(const f32x4& a, const f32x4& b) {
  return bf16x8{f2e<H>(a[0]), f2e<H>(a[1]), f2e<H>(a[2]), f2e<H>(a[3]),
                f2e<H>(b[0]), f2e<H>(b[1]), f2e<H>(b[2]), f2e<H>(b[3])};
}

struct AttnP {
  const bf16* Q; const bf16* K; const bf16* V; bf16* O; float* lse;
  const bf16* dO; float* Dv; bf16* dQ; bf16* dK; bf16* dV;
  int64_t ldq, ldk, ldv, ldo, lddo, lddq, lddk, lddv;
  int B, H, Tq, Tk, causal;
  float scale, scale_log2;
};

constexpr float LOG2E = 1.4426950408889634f;

// XCD-aware bijective remap of a 2-D (blocks_per_head, heads) grid: the blocks of one
// (batch, head) land on one XCD (blocks b and b+8 share one), so its K/V (or Q/dO) tiles are
// fetched into that XCD's L2 once instead of once per XCD.
__device__ __forceinline__ void remap_bh(int& xblk, int& bh) {
  const int nx = gridDim.x, nwg = gridDim.x * gridDim.y;
  const int bid = blockIdx.y * nx + blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = bid % 8;
  const int tid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  bh = tid / nx;
  xblk = tid % nx;
}
constexpr float NEG_BIG = -1e30f;

__device__ __forceinline__ float fmx(float a, float b) { return __builtin_elementwise_maximum(a, b); }

// ------------------------------------------------------------------------------------
// H = false: bf16 Q/K/V/O (autocast); H = true: fp16 (the fp16 decode path: P rounded to fp16 for PV,
// as SDPA's fp16 flash kernel rounds it)
// K/V arrive in a 3-deep LDS ring: two tiles in flight (prefetch distance 2: the DMA of tile kt+2 overlaps the
// compute of tiles kt and kt+1), counted vmcnt + a raw s_barrier (a __syncthreads() would drain every DMA in
// flight).  (Round 3's opt-in lazy max and the 2-stage ring were deleted in round 4: DESIGN.md, Attention.)
template <bool H>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnP p) {
  constexpr int ST = 3;
  __shared__ __attribute__((aligned(16))) char smem[ST * 2 * TB];   // [ST stages][K, V]
  const int lane = lane_id(), wave = wave_id_uniform();
  const int g = lane >> 4, li = lane & 15;
  int xblk, bh;
  remap_bh(xblk, bh);
  const int b = bh / p.H, h = bh % p.H;
  const int qblk = xblk * QB;
  const int qw = qblk + wave * QW;
  const bf16* Qb = p.Q + (int64_t)b * p.Tq * p.ldq + h * 64;
  const bf16* Kb = p.K + (int64_t)b * p.Tk * p.ldk + h * 64;
  const bf16* Vb = p.V + (int64_t)b * p.Tk * p.ldv + h * 64;
  const int off = p.Tk - p.Tq;   // causal diagonal offset

  bf16x8 qf[2][2];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qf[qi][kk] = ld_frag(Qb, p.ldq, qw + qi * 16 + li, p.Tq, kk, lane);

  f32x4 o[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) o[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {NEG_BIG, NEG_BIG}, l[2] = {0.f, 0.f};

  int nkt = (p.Tk + KT - 1) / KT;
  if (p.causal) {
    const int qmax = min(p.Tq - 1, qblk + QB - 1);
    const int kend = qmax + off + 1;
    nkt = min(nkt, (kend + KT - 1) / KT);
  }

  auto stage = [&](int buf, int kt) {
    char* Ks = smem + buf * 2 * TB;
    const int k0 = kt * KT;
    stage_tile(Kb + (int64_t)k0 * p.ldk, p.ldk, p.Tk - k0, Ks, wave, lane);
    stage_tile(Vb + (int64_t)k0 * p.ldv, p.ldv, p.Tk - k0, Ks + TB, wave, lane);
  };
  // S^T = K Q^T for one tile, boundary tiles masked (key tail / causal diagonal)
  auto scores = [&](const bf16x8 (&kf)[4][2], f32x4 (&s)[4][2], int k0) {
#pragma unroll
    for (int kj = 0; kj < 4; ++kj) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      s[kj][0] = mma16<H>(kf[kj][1], qf[0][1], mma16<H>(kf[kj][0], qf[0][0], z));
      s[kj][1] = mma16<H>(kf[kj][1], qf[1][1], mma16<H>(kf[kj][0], qf[1][0], z));
    }
    const bool need_mask = (k0 + KT > p.Tk) || (p.causal && k0 + KT - 1 > qw + off);
    if (need_mask) {
#pragma unroll
      for (int qi = 0; qi < 2; ++qi) {
        const int q = qw + qi * 16 + li;
#pragma unroll
        for (int kj = 0; kj < 4; ++kj)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + kj * 16 + 4 * g + r;
            const bool ok = key < p.Tk && (!p.causal || key <= q + off);
            if (!ok) s[kj][qi][r] = -INFINITY;
          }
      }
    }
  };
  // online softmax (log2 domain), per query column: max on raw scores (scale > 0); p = exp2(s*c - m) is
  // one FMA + one exp; O is rescaled only when some row max of this wave grew.  Returns the lane-partial
  // sums of the weights (added to l by the caller).
  auto exact = [&](f32x4 (&s)[4][2], float (&ls)[2]) {
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      // row max: a tree over the lane's 16 scores, then across the 4 lanes of the query column
      // (l, l^16, l^32, l^48) with v_permlane16/32_swap (VALU) instead of two ds_bpermute trips
      // (a chain of 3-input maxes: 8 v_maximum3_f32 for the 16 scores.  IEEE maximum, not fmaxf: fmaxf in the
      // kernels' IEEE mode first quiets each MFMA result with a v_max_f32 x, x; maximum needs none and propagates
      // a NaN score, which the weights would carry to O and l anyway)
      float tmax = fmx(fmx(s[0][qi][0], s[0][qi][1]), s[0][qi][2]);
#pragma unroll
      for (int e = 3; e < 15; e += 2)
        tmax = fmx(fmx(tmax, s[e >> 2][qi][e & 3]), s[(e + 1) >> 2][qi][(e + 1) & 3]);
      tmax = fmx(tmax, s[3][qi][3]);
      {
        const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(tmax), __float_as_uint(tmax), false, false);
        tmax = fmx(__uint_as_float(a[0]), __uint_as_float(a[1]));
        const auto c = __builtin_amdgcn_permlane32_swap(__float_as_uint(tmax), __float_as_uint(tmax), false, false);
        tmax = fmx(__uint_as_float(c[0]), __uint_as_float(c[1]));
      }
      const float mn = fmaxf(m[qi], tmax * p.scale_log2);
      if (__any(mn > m[qi])) {
        const float alpha = __builtin_amdgcn_exp2f(m[qi] - mn);
        l[qi] *= alpha;
#pragma unroll
        for (int hj = 0; hj < 4; ++hj) o[hj][qi] *= alpha;
      }
      m[qi] = mn;
      float a = 0.f;      // sequential (a 4-way split moved the micro-config KL by 1e-3 vs the oracle)
      // s*c - m as one scalar v_fma_f32 per score (a v_pk_fma_f32 costs more issue cycles than two
      // v_fma_f32 beside MFMAs: MI355X_MICROARCH constants table), then v_exp_f32 on it directly
      const float nm = -mn;
#pragma unroll
      for (int kj = 0; kj < 4; ++kj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float e = __builtin_amdgcn_exp2f(fmaf(s[kj][qi][r], p.scale_log2, nm));
          s[kj][qi][r] = e;
          a += e;
        }
      ls[qi] = a;
    }
  };
  stage(0, 0);
  if (nkt > 1) {
    stage(1, 1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");      // tile 0 landed (4 DMA per tile per wave), tile 1 flies
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();

  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt % 3;
    const char* Ks = smem + cur * 2 * TB;
    const char* Vs = Ks + TB;
    // all K and V fragments of this tile into registers BEFORE the next tile's LDS-DMA is
    // issued: otherwise the compiler cannot prove the DMA does not alias these reads and
    // drains vmcnt(0) in the middle of the tile (exposing the whole load latency)
    bf16x8 kf[4][2], vf[4][2];
#pragma unroll
    for (int kj = 0; kj < 4; ++kj)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) kf[kj][kk] = rd_row(Ks, kj * 16, kk, lane);
#pragma unroll
    for (int hj = 0; hj < 4; ++hj)
#pragma unroll
      for (int ss = 0; ss < 2; ++ss) vf[hj][ss] = rd_tr(Vs, hj * 16, ss, lane);
    if (kt + 2 < nkt) stage((kt + 2) % 3, kt + 2);          // the slot tile kt-1 was read from
    const int k0 = kt * KT;
    f32x4 s[4][2];
    scores(kf, s, k0);
    float ls[2];
    exact(s, ls);
    l[0] += ls[0];
    l[1] += ls[1];
    // O^T += V^T P^T
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 p0 = pack8e<H>(s[2 * ss][0], s[2 * ss + 1][0]);
      const bf16x8 p1 = pack8e<H>(s[2 * ss][1], s[2 * ss + 1][1]);
#pragma unroll
      for (int hj = 0; hj < 4; ++hj) {
        o[hj][0] = mma16<H>(vf[hj][ss], p0, o[hj][0]);
        o[hj][1] = mma16<H>(vf[hj][ss], p1, o[hj][1]);
      }
    }
    // tile kt+1 must have landed for every wave; tile kt+2 (issued this iteration) may stay in flight
    if (kt + 2 < nkt) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  // epilogue
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const float lt = swap32_sum(swap16_sum(l[qi]));   // xor 16 then 32 on permlane swaps (bit-identical: common.h)
    const int q = qw + qi * 16 + li;
    if (q < p.Tq) {
      const float inv = 1.f / lt;
      bf16* Ob = p.O + ((int64_t)b * p.Tq + q) * p.ldo + h * 64;
#pragma unroll
      for (int hj = 0; hj < 4; ++hj) {
        const f32x4 v = o[hj][qi] * inv;
        *(bf16x4*)(Ob + hj * 16 + 4 * g) = bf16x4{f2e<H>(v[0]), f2e<H>(v[1]), f2e<H>(v[2]), f2e<H>(v[3])};
      }
      if (g == 0 && p.lse) p.lse[(int64_t)bh * p.Tq + q] = (m[qi] + log2f(lt)) / LOG2E;
    }
  }
}


// ------------------------------------------------------------------------------------
// dQ: per query block, loop over key tiles (K, V in LDS).  Also computes D[q] = sum_e dO[q][e] O[q][e] for its rows
// (each lane's 16 products, then the 4 lanes of a row by xor-16 / xor-32 swaps) and stores it for the dK/dV kernel,
// which runs after it: no separate pass over dO and O.
template <bool H>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(AttnP p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TB];
  const int lane = lane_id(), wave = wave_id_uniform();
  const int g = lane >> 4, li = lane & 15;
  int xblk, bh;
  remap_bh(xblk, bh);
  const int b = bh / p.H, h = bh % p.H;
  const int qblk = xblk * QB;
  const int qw = qblk + wave * QW;
  const bf16* Qb = p.Q + (int64_t)b * p.Tq * p.ldq + h * 64;
  const bf16* dOb = p.dO + (int64_t)b * p.Tq * p.lddo + h * 64;
  const bf16* Kb = p.K + (int64_t)b * p.Tk * p.ldk + h * 64;
  const bf16* Vb = p.V + (int64_t)b * p.Tk * p.ldv + h * 64;
  const int off = p.Tk - p.Tq;

  const bf16* Ob = p.O + (int64_t)b * p.Tq * p.ldo + h * 64;
  bf16x8 qf[2][2], dof[2][2];
  float lse2[2], Dq[2];
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int q = qw + qi * 16 + li;
    float dd = 0.f;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[qi][kk] = ld_frag(Qb, p.ldq, q, p.Tq, kk, lane);
      dof[qi][kk] = ld_frag(dOb, p.lddo, q, p.Tq, kk, lane);
      const bf16x8 of = ld_frag(Ob, p.ldo, q, p.Tq, kk, lane);
#pragma unroll
      for (int e = 0; e < 8; ++e) dd += e2f<H>(dof[qi][kk][e]) * e2f<H>(of[e]);
    }
    lse2[qi] = q < p.Tq ? p.lse[(int64_t)bh * p.Tq + q] * LOG2E : 0.f;
    Dq[qi] = swap32_sum(swap16_sum(dd));                 // rows past Tq: zero fragments, D = 0
    if (g == 0 && q < p.Tq) p.Dv[(int64_t)bh * p.Tq + q] = Dq[qi];
  }
  f32x4 dq[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) dq[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int nkt = (p.Tk + KT - 1) / KT;
  if (p.causal) {
    const int qmax = min(p.Tq - 1, qblk + QB - 1);
    nkt = min(nkt, (qmax + off + 1 + KT - 1) / KT);
  }
  auto stage = [&](int buf, int kt) {
    char* Ks = smem + buf * 2 * TB;
    const int k0 = kt * KT;
    stage_tile(Kb + (int64_t)k0 * p.ldk, p.ldk, p.Tk - k0, Ks, wave, lane);
    stage_tile(Vb + (int64_t)k0 * p.ldv, p.ldv, p.Tk - k0, Ks + TB, wave, lane);
  };
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nkt; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nkt) stage(cur ^ 1, kt + 1);
    const char* Ks = smem + cur * 2 * TB;
    const char* Vs = Ks + TB;
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int kj = 0; kj < 4; ++kj) {
      s[kj][0] = s[kj][1] = dp[kj][0] = dp[kj][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 kf = rd_row(Ks, kj * 16, kk, lane);
        const bf16x8 vf = rd_row(Vs, kj * 16, kk, lane);
        s[kj][0] = mma16<H>(kf, qf[0][kk], s[kj][0]);
        s[kj][1] = mma16<H>(kf, qf[1][kk], s[kj][1]);
        dp[kj][0] = mma16<H>(vf, dof[0][kk], dp[kj][0]);
        dp[kj][1] = mma16<H>(vf, dof[1][kk], dp[kj][1]);
      }
    }
    const int k0 = kt * KT;
    // P recomputed with the forward's exp2 (v_exp_f32) and, on interior tiles (no key tail, no query tail, not on
    // the causal diagonal: wave-uniform), without the per-element mask
    const bool need_mask = (k0 + KT > p.Tk) || (qw + QW > p.Tq) || (p.causal && k0 + KT - 1 > qw + off);
#pragma unroll
    for (int qi = 0; qi < 2; ++qi) {
      const int q = qw + qi * 16 + li;
#pragma unroll
      for (int kj = 0; kj < 4; ++kj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + kj * 16 + 4 * g + r;
          const bool ok = !need_mask || (key < p.Tk && q < p.Tq && (!p.causal || key <= q + off));
          // masked scores as exp2(-inf) = 0: a select, not a branch per element (interior tiles: ok is always true)
          const float pr = __builtin_amdgcn_exp2f(ok ? s[kj][qi][r] * p.scale_log2 - lse2[qi] : -INFINITY);
          s[kj][qi][r] = pr * (dp[kj][qi][r] - Dq[qi]);   // dS^T
        }
    }
    // dQ^T += K^T dS^T
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 d0 = pack8e<H>(s[2 * ss][0], s[2 * ss + 1][0]);
      const bf16x8 d1 = pack8e<H>(s[2 * ss][1], s[2 * ss + 1][1]);
#pragma unroll
      for (int hj = 0; hj < 4; ++hj) {
        const bf16x8 kt_ = rd_tr(Ks, hj * 16, ss, lane);
        dq[hj][0] = mma16<H>(kt_, d0, dq[hj][0]);
        dq[hj][1] = mma16<H>(kt_, d1, dq[hj][1]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int qi = 0; qi < 2; ++qi) {
    const int q = qw + qi * 16 + li;
    if (q < p.Tq) {
      bf16* out = p.dQ + ((int64_t)b * p.Tq + q) * p.lddq + h * 64;
#pragma unroll
      for (int hj = 0; hj < 4; ++hj) {
        const f32x4 v = dq[hj][qi] * p.scale;
        *(bf16x4*)(out + hj * 16 + 4 * g) = bf16x4{f2e<H>(v[0]), f2e<H>(v[1]), f2e<H>(v[2]), f2e<H>(v[3])};
      }
    }
  }
}

// dK, dV: per key block (32 keys per wave, 128 per workgroup), loop over query tiles
// Two workgroups per CU (round 4): 218 VGPRs, two waves per SIMD hide each other's LDS / exp / MFMA latencies.  At
// one workgroup per CU (round 3: 268-276 VGPRs, accumulators shuffled through AGPRs) the encoder-shape backward
// took 6.1 ms against 4.6 ms now (tools/bench_attn.py, same box, profiles/r04_h_attn_bwd_ab.log).
template <bool H>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(AttnP p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * TB + 2 * 2 * 64 * 4];
  const int lane = lane_id(), wave = wave_id_uniform();
  const int g = lane >> 4, li = lane & 15;
  int xblk, bh;
  remap_bh(xblk, bh);
  const int b = bh / p.H, h = bh % p.H;
  const int kblk = xblk * QB;
  const int kw = kblk + wave * QW;
  const bf16* Qb = p.Q + (int64_t)b * p.Tq * p.ldq + h * 64;
  const bf16* dOb = p.dO + (int64_t)b * p.Tq * p.lddo + h * 64;
  const bf16* Kb = p.K + (int64_t)b * p.Tk * p.ldk + h * 64;
  const bf16* Vb = p.V + (int64_t)b * p.Tk * p.ldv + h * 64;
  const int off = p.Tk - p.Tq;
  float* rowc = (float*)(smem + 4 * TB);   // [2 stages][lse2 64 | D 64]

  bf16x8 kf[2][2], vf[2][2];
#pragma unroll
  for (int kj = 0; kj < 2; ++kj)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kf[kj][kk] = ld_frag(Kb, p.ldk, kw + kj * 16 + li, p.Tk, kk, lane);
      vf[kj][kk] = ld_frag(Vb, p.ldv, kw + kj * 16 + li, p.Tk, kk, lane);
    }
  f32x4 dk[4][2], dv[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) dk[i][j] = dv[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nqt_all = (p.Tq + KT - 1) / KT;
  int qt0 = 0;
  if (p.causal) {
    const int qmin = kblk - off;   // first query that can see this key block
    qt0 = qmin > 0 ? qmin / KT : 0;
  }
  auto stage = [&](int buf, int qt) {
    char* Qs = smem + buf * 2 * TB;
    const int q0 = qt * KT;
    stage_tile(Qb + (int64_t)q0 * p.ldq, p.ldq, p.Tq - q0, Qs, wave, lane);
    stage_tile(dOb + (int64_t)q0 * p.lddo, p.lddo, p.Tq - q0, Qs + TB, wave, lane);
    if (threadIdx.x < 64) {
      const int q = q0 + threadIdx.x;
      rowc[buf * 128 + threadIdx.x] = q < p.Tq ? p.lse[(int64_t)bh * p.Tq + q] * LOG2E : 0.f;
      rowc[buf * 128 + 64 + threadIdx.x] = q < p.Tq ? p.Dv[(int64_t)bh * p.Tq + q] : 0.f;
    }
  };
  if (qt0 < nqt_all) {
    stage(0, qt0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int qt = qt0; qt < nqt_all; ++qt) {
    const int cur = (qt - qt0) & 1;
    if (qt + 1 < nqt_all) stage(cur ^ 1, qt + 1);
    const char* Qs = smem + cur * 2 * TB;
    const char* dOs = Qs + TB;
    const float* lrow = rowc + cur * 128;
    const int q0 = qt * KT;
    // S[q][key], dP[q][key] for 64 q x 32 keys
    f32x4 s[4][2], dp[4][2];
#pragma unroll
    for (int qf = 0; qf < 4; ++qf) {
      s[qf][0] = s[qf][1] = dp[qf][0] = dp[qf][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 qa = rd_row(Qs, qf * 16, kk, lane);
        const bf16x8 da = rd_row(dOs, qf * 16, kk, lane);
        s[qf][0] = mma16<H>(qa, kf[0][kk], s[qf][0]);
        s[qf][1] = mma16<H>(qa, kf[1][kk], s[qf][1]);
        dp[qf][0] = mma16<H>(da, vf[0][kk], dp[qf][0]);
        dp[qf][1] = mma16<H>(da, vf[1][kk], dp[qf][1]);
      }
    }
    // interior tiles (no query tail, no key tail, not on the causal diagonal: wave-uniform) skip the mask
    const bool need_mask = (q0 + KT > p.Tq) || (kw + QW > p.Tk) || (p.causal && kw + QW - 1 > q0 + off);
#pragma unroll
    for (int qf = 0; qf < 4; ++qf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = qf * 16 + 4 * g + r;
        const int q = q0 + ql;
        const float l2 = lrow[ql], Dq = lrow[64 + ql];
#pragma unroll
        for (int kj = 0; kj < 2; ++kj) {
          const int key = kw + kj * 16 + li;
          const bool ok = !need_mask || (q < p.Tq && key < p.Tk && (!p.causal || key <= q + off));
          const float pr = __builtin_amdgcn_exp2f(ok ? s[qf][kj][r] * p.scale_log2 - l2 : -INFINITY);   // select, no branch
          s[qf][kj][r] = pr;                              // P
          dp[qf][kj][r] = pr * (dp[qf][kj][r] - Dq);      // dS
        }
      }
    // dV^T += dO^T P ; dK^T += Q^T dS
#pragma unroll
    for (int ss = 0; ss < 2; ++ss) {
      const bf16x8 p0 = pack8e<H>(s[2 * ss][0], s[2 * ss + 1][0]);
      const bf16x8 p1 = pack8e<H>(s[2 * ss][1], s[2 * ss + 1][1]);
      const bf16x8 d0 = pack8e<H>(dp[2 * ss][0], dp[2 * ss + 1][0]);
      const bf16x8 d1 = pack8e<H>(dp[2 * ss][1], dp[2 * ss + 1][1]);
#pragma unroll
      for (int hj = 0; hj < 4; ++hj) {
        const bf16x8 dot = rd_tr(dOs, hj * 16, ss, lane);
        const bf16x8 qt_ = rd_tr(Qs, hj * 16, ss, lane);
        dv[hj][0] = mma16<H>(dot, p0, dv[hj][0]);
        dv[hj][1] = mma16<H>(dot, p1, dv[hj][1]);
        dk[hj][0] = mma16<H>(qt_, d0, dk[hj][0]);
        dk[hj][1] = mma16<H>(qt_, d1, dk[hj][1]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int kj = 0; kj < 2; ++kj) {
    const int key = kw + kj * 16 + li;
    if (key < p.Tk) {
      bf16* ok_ = p.dK + ((int64_t)b * p.Tk + key) * p.lddk + h * 64;
      bf16* ov_ = p.dV + ((int64_t)b * p.Tk + key) * p.lddv + h * 64;
#pragma unroll
      for (int hj = 0; hj < 4; ++hj) {
        const f32x4 a = dk[hj][kj] * p.scale;
        const f32x4 c = dv[hj][kj];
        *(bf16x4*)(ok_ + hj * 16 + 4 * g) = bf16x4{f2e<H>(a[0]), f2e<H>(a[1]), f2e<H>(a[2]), f2e<H>(a[3])};
        *(bf16x4*)(ov_ + hj * 16 + 4 * g) = bf16x4{f2e<H>(c[0]), f2e<H>(c[1]), f2e<H>(c[2]), f2e<H>(c[3])};
      }
    }
  }
}

bool check_common(const void* Q, const void* K, const void* V, int64_t ldq, int64_t ldk, int64_t ldv) {
  if (((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V) & 15) return false;
  if ((ldq | ldk | ldv) & 7) return false;
  return true;
}

}  // namespace

extern "C" int tw_attn_fwd(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv, void* O,
                           int64_t ldo, float* lse, int B, int H, int Tq, int Tk, int head_dim, int causal, float scale,
                           hipStream_t stream) {
  if (head_dim != 64) return TW_EUNSUPPORTED;
  if (B <= 0 || Tq <= 0 || Tk <= 0) return TW_OK;
  if (!check_common(Q, K, V, ldq, ldk, ldv) || (ldo & 3)) return TW_EINVAL;
  if (causal && Tq > Tk) return TW_EINVAL;
  AttnP p = {};
  p.Q = (const bf16*)Q; p.K = (const bf16*)K; p.V = (const bf16*)V; p.O = (bf16*)O; p.lse = lse;
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo;
  p.B = B; p.H = H; p.Tq = Tq; p.Tk = Tk; p.causal = causal;
  p.scale = scale; p.scale_log2 = scale * LOG2E;
  hipLaunchKernelGGL(attn_fwd_kernel<false>, dim3((Tq + QB - 1) / QB, B * H), dim3(256), 0, stream, p);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// fp16 Q/K/V/O (HF Whisper with torch_dtype=float16: SDPA over fp16 projections, run_eval.py:99,500-509)
extern "C" int tw_attn_fwd_f16(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv,
                               void* O, int64_t ldo, float* lse, int B, int H, int Tq, int Tk, int head_dim, int causal,
                               float scale, hipStream_t stream) {
  if (head_dim != 64) return TW_EUNSUPPORTED;
  if (B <= 0 || Tq <= 0 || Tk <= 0) return TW_OK;
  if (!check_common(Q, K, V, ldq, ldk, ldv) || (ldo & 3)) return TW_EINVAL;
  if (causal && Tq > Tk) return TW_EINVAL;
  AttnP p = {};
  p.Q = (const bf16*)Q; p.K = (const bf16*)K; p.V = (const bf16*)V; p.O = (bf16*)O; p.lse = lse;
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo;
  p.B = B; p.H = H; p.Tq = Tq; p.Tk = Tk; p.causal = causal;
  p.scale = scale; p.scale_log2 = scale * LOG2E;
  hipLaunchKernelGGL(attn_fwd_kernel<true>, dim3((Tq + QB - 1) / QB, B * H), dim3(256), 0, stream, p);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

namespace {
// workspace: B*H*Tq floats (the D = rowsum(dO*O) vector); half: fp16 words (fp16-autocast training), else bf16
int attn_bwd_run(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv, const void* O,
                 int64_t ldo, const void* dO, int64_t lddo, const float* lse, void* dQ, int64_t lddq, void* dK,
                 int64_t lddk, void* dV, int64_t lddv, int B, int H, int Tq, int Tk, int head_dim, int causal,
                 float scale, float* workspace, bool half, hipStream_t stream) {
  if (head_dim != 64) return TW_EUNSUPPORTED;
  if (B <= 0 || Tq <= 0 || Tk <= 0) return TW_OK;
  if (!check_common(Q, K, V, ldq, ldk, ldv) || ((uintptr_t)dO & 15) || (lddo & 7) || ((uintptr_t)O & 15) || (ldo & 7))
    return TW_EINVAL;
  if (causal && Tq > Tk) return TW_EINVAL;
  AttnP p = {};
  p.Q = (const bf16*)Q; p.K = (const bf16*)K; p.V = (const bf16*)V; p.lse = (float*)lse; p.O = (bf16*)O;
  p.dO = (const bf16*)dO; p.Dv = workspace; p.dQ = (bf16*)dQ; p.dK = (bf16*)dK; p.dV = (bf16*)dV;
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo; p.lddo = lddo; p.lddq = lddq; p.lddk = lddk; p.lddv = lddv;
  p.B = B; p.H = H; p.Tq = Tq; p.Tk = Tk; p.causal = causal;
  p.scale = scale; p.scale_log2 = scale * LOG2E;
  // dQ (and D, which the dK/dV kernel reads) first, then dK/dV
  if (half) {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<true>, dim3((Tq + QB - 1) / QB, B * H), dim3(256), 0, stream, p);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<true>, dim3((Tk + QB - 1) / QB, B * H), dim3(256), 0, stream, p);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_kernel<false>, dim3((Tq + QB - 1) / QB, B * H), dim3(256), 0, stream, p);
    hipLaunchKernelGGL(attn_bwd_dkdv_kernel<false>, dim3((Tk + QB - 1) / QB, B * H), dim3(256), 0, stream, p);
  }
  TW_CHECK_LAUNCH();
  return TW_OK;
}
}  // namespace

extern "C" int tw_attn_bwd(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv,
                           const void* O, int64_t ldo, const void* dO, int64_t lddo, const float* lse, void* dQ,
                           int64_t lddq, void* dK, int64_t lddk, void* dV, int64_t lddv, int B, int H, int Tq, int Tk,
                           int head_dim, int causal, float scale, float* workspace, hipStream_t stream) {
  return attn_bwd_run(Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse, dQ, lddq, dK, lddk, dV, lddv, B, H, Tq, Tk,
                      head_dim, causal, scale, workspace, false, stream);
}

// fp16 Q/K/V/O/dO/dQ/dK/dV (the student's SDPA backward under fp16 autocast, run_distillation.py:815-817
// mixed_precision="fp16"): the bf16 kernels instantiated for fp16 words (P and dS rounded to fp16 for their MFMAs)
extern "C" int tw_attn_bwd_f16(const void* Q, int64_t ldq, const void* K, int64_t ldk, const void* V, int64_t ldv,
                               const void* O, int64_t ldo, const void* dO, int64_t lddo, const float* lse, void* dQ,
                               int64_t lddq, void* dK, int64_t lddk, void* dV, int64_t lddv, int B, int H, int Tq,
                               int Tk, int head_dim, int causal, float scale, float* workspace, hipStream_t stream) {
  return attn_bwd_run(Q, ldq, K, ldk, V, ldv, O, ldo, dO, lddo, lse, dQ, lddq, dK, lddk, dV, lddv, B, H, Tq, Tk,
                      head_dim, causal, scale, workspace, true, stream);
}
