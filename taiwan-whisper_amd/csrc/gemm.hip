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
#include "gemm_impl.h"
#include "gemv_impl.h"


namespace {

using namespace twg;

// STAGES-deep LDS ring, prefetch distance STAGES-1; waits are counted (vmcnt = loads of the
// stages allowed to stay in flight) and the barrier is a raw s_barrier, so in-flight LDS-DMA
// survives it (a __syncthreads() would drain vmcnt(0)).
template <bool H, bool AT, bool BT, int BM, int BN, int WM, int WN, int STAGES>
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
            acc[mi][ni] = mma16<H>(b[kk][ni], a[kk][mi], acc[mi][ni]);
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
            acc[mi][ni] = mma16<H>(b[ni], a[mi], acc[mi][ni]);
      }
    }
    // stage kt+1 must have landed; stages kt+2 .. kt+PD (when issued) may stay in flight
    if (kt + PD < nk) wait_vm_lgkm0<(PD - 1) * LPS>();
    else wait_vm_lgkm0<0>();
    __builtin_amdgcn_s_barrier();
  }

  epilogue<H, BM, BN, WM, WN, 0, -1, BT && !AT>(p, acc, m0, n0, wm, wn, lane, bz);
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

// The same for a whole 64-deep K-tile (every k valid): the lane part of the source offset is loop-invariant -- piece
// row (lane >> 3), 16-B chunk (lane & 7) ^ (lane >> 3), since a piece's first region row is a multiple of 8 -- so it
// is computed once per kernel (`lane_off`); the piece's row adds one scalar term and the K-tile goes into the scalar
// offset.  Rows past the operand (a ragged last tile) read zeros through the descriptor's bound (`bytes` = the
// valid rows x ld from the tile base; the K offset never leaves a valid row), so there is no per-lane compare (the
// checked form's row / bound arithmetic ran in the load segments, beside the partner wave's MFMAs).
__device__ __forceinline__ uint32_t pp_lane_off(int64_t ld, int lane) {
  const int r = lane >> 3;
  return (uint32_t)(((int64_t)r * ld + ((lane & 7) ^ r) * 8) * 2);
}
template <int S, int GS>
__device__ __forceinline__ void pp_stage_full(const bf16* base, int64_t ld, int rows_left, uint32_t lane_off, int kt,
                                              int off, char* region, int wave) {
  // (only this tile's 256 rows are ever addressed: the bound stays 32-bit, <= 256 x ld x 2 bytes)
  const int bytes = rows_left > 0 ? (rows_left < 256 ? rows_left : 256) * (int)ld * 2 : 0;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int pce = wave + 8 * i;
    const int R0 = pce * 8;
    const int row0 = (R0 >> S) * GS + off + (R0 & ((1 << S) - 1));
    const uint32_t voff = lane_off + (uint32_t)(row0 * (int)ld * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(region + pce * 1024), 16, voff, (uint32_t)(kt * BK * 2), 0, 0);
  }
}

// Epilogue of fragment rows MI0 .. MI1-1 of finished tile `ti` of this workgroup, then those accumulators
// are zeroed for the next tile.  Debug flags: 4096 skips the stores, 1 << 20 stores every tile to tile 0.
template <bool H, int KIND, int MI0, int MI1>
__device__ __forceinline__ void pp_epi_part(const GemmP& p, f32x4 (&acc)[8][4], int ti, int wm, int wn, int lane,
                                            const bf16* braw) {
  if (!(p.flags & 4096) || acc[MI0][0][0] != acc[MI0][0][0]) {
    int m0, n0, bz;
    pp_tile(p, ti, m0, n0, bz);
    if (p.flags & (1 << 20)) { m0 = 0; n0 = 0; }
    epilogue_k<H, 256, 256, 2, 4, KIND, MI0, MI1, true>(p, acc, m0, n0, wm, wn, lane, bz, braw);
  }
#pragma unroll
  for (int i = MI0; i < MI1; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// Persistent form: gridDim.x (a multiple of 8, <= CUs) workgroups; workgroup b takes the tiles
// of virtual block ids b, b + G, b + 2G, ... (G = gridDim.x), each mapped through the same
// XCD-aware bijective remap as a one-tile-per-block launch, so an XCD keeps walking its own
// contiguous chunk.  The K-tile stream is continuous across tiles (nk rounded up to even; the
// pad K-tile stages zeros), so the next tile's first K-tiles are already in flight while the
// finished tile's epilogue runs (between phases, beside the other wave-row's MFMAs).

// PRIO (variant; flags bits 15-17 select it, see launch_pp): 0 = four 16-MFMA phases per K-tile,
// prio 1 around each MFMA phase; 1 = the same with static prio 1 for the trailing wave row
// (waves 4-7), no flips; 2 = diagnostic: every MFMA phase issued twice (wrong results; measures
// the fixed per-phase cost); 4 = two 32-MFMA phases per K-tile (default: +4-8 % main loop)
// KF: K is a multiple of 64 (every launch of the model's shapes but the conv stem's K = 240): staging without per-lane
// bound arithmetic (pp_stage_full).  KF = false keeps the checked stager for a K tail (generic epilogue only).
template <bool H, int PRIO, int KIND = -1, bool KF = true>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(GemmP p) {
  // + 2 x 1 KiB: the bias slice of the current tile (by tile parity), for the fast epilogue (one array:
  // a second __shared__ object can make the compiler drain vmcnt before LDS reads)
  __shared__ __attribute__((aligned(16))) char smem[2 * 4 * PP_REGION + 2048];
  const int lane = lane_id();
  const int wave = wave_id_uniform();
  const int wm = wave >> 2, wn = wave & 3;
  const int K = p.K, nk = (K + BK - 1) / BK, nke = (nk + 1) & ~1;
  const int G = gridDim.x;
  const int my_tiles = ((int)blockIdx.x < p.tiles_total) ? (p.tiles_total - (int)blockIdx.x + G - 1) / G : 0;
  const int total = my_tiles * nke;                       // K-tiles this workgroup consumes

  int si = 0;                                // current tile of this workgroup
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
  // Tile state: the operand base pointers at k = 0, the rows / columns left and the K extent
  // (0 past the stream: the stager then fills zeros); per K-tile the stager only adds kt * BK.
  auto tile_info = [&](int i, const bf16*& pa, const bf16*& pb, int& rows, int& cols, int& kl) {
    int m0 = 0, n0 = 0, bz = 0;
    const bool live = i < my_tiles && pp_tile(p, i, m0, n0, bz);
#ifdef TW_PP_DIAG_VARIANTS
    // diagnostic build only, flag 1 << 22: every tile stages the panels of its workgroup's XCD-first tile (A rows and
    // B columns of one 256 x 256 block per XCD, L2-resident): the main loop without L2 misses (wrong results)
    if (p.flags & (1 << 22)) { m0 = p.M >= 2048 ? ((int)blockIdx.x & 7) * 256 : 0; n0 = 0; bz = 0; }
#endif
    pa = p.A + bz * p.sA + (int64_t)m0 * p.lda;
    pb = p.B + bz * p.sB + (int64_t)n0 * p.ldb;
    rows = p.M - m0;
    cols = p.N - n0;
    kl = live ? K : 0;
  };
  auto reg = [&](int b, int r) -> char* { return smem + (b * 4 + r) * PP_REGION; };
  const uint32_t lane_off_a = KF ? pp_lane_off(p.lda, lane) : 0u, lane_off_b = KF ? pp_lane_off(p.ldb, lane) : 0u;
  auto stage = [&](const bf16* pa, const bf16* pb, int rows, int cols, int kl, int kt, int buf, int r) {
    const int k_left = kl - kt * BK;
    if constexpr (KF) {
      // a whole K-tile, or none (a dead tile or the pad K-tile: k_left <= 0 -> zero valid rows -> zeros)
      const int valid = k_left > 0 ? 1 : 0;
      if (r < 2) pp_stage_full<6, 128>(pa, p.lda, rows * valid, lane_off_a, kt, r * 64, reg(buf, r), wave);
      else pp_stage_full<5, 64>(pb, p.ldb, cols * valid, lane_off_b, kt, (r - 2) * 32, reg(buf, r), wave);
    } else {
      if (r < 2) pp_stage<6, 128>(pa + kt * BK, p.lda, rows, k_left, r * 64, reg(buf, r), wave, lane);
      else pp_stage<5, 64>(pb + kt * BK, p.ldb, cols, k_left, (r - 2) * 32, reg(buf, r), wave, lane);
    }
  };

  // PRIO 6: diagnostic, no restaging in the main loop (timing of everything but the DMA)
  auto stg = [&](const bf16* pa, const bf16* pb, int rows, int cols, int kl, int kt, int buf, int r) {
    if constexpr (PRIO != 6) stage(pa, pb, rows, cols, kl, kt, buf, r);
  };
  bf16x8 a[2][4], bb[2][2];
  bf16x8 bq[2][2][2];                        // PRIO 4: both B-quarters of the K-tile
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
  auto rdB2 = [&](int b) {
#pragma unroll
    for (int qq = 0; qq < 2; ++qq)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) bq[qq][kk][ni] = frag_k(reg(b, 2 + qq), wn * 32 + ni * 16, kk, lane);
  };
  auto sync = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  // PRIO 4: one phase = one A-half x both B-quarters (32 MFMAs)
  auto mma2 = [&](int qm) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sync();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int qq = 0; qq < 2; ++qq)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
            acc[qm * 4 + mi][qq * 2 + ni] =
                mma16<H>(bq[qq][kk][ni], a[kk][mi], acc[qm * 4 + mi][qq * 2 + ni]);
    __builtin_amdgcn_s_setprio(0);
    sync();
  };
  auto mma = [&](int qm, int qn) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    sync();
    if constexpr (PRIO == 0 || PRIO == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int rep = 0; rep < (PRIO == 2 ? 2 : 1); ++rep)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
          acc[qm * 4 + mi][qn * 2 + ni] =
              mma16<H>(bb[kk][ni], a[kk][mi], acc[qm * 4 + mi][qn * 2 + ni]);
    if constexpr (PRIO == 0 || PRIO == 2) __builtin_amdgcn_s_setprio(0);
    sync();
  };

  // prologue: K-tile 0 whole into buffer 0, K-tile 1 without B-quarter 0 into buffer 1
  const bf16 *cpa, *cpb;                     // current tile (see tile_info)
  int cr, cc, ck;
  tile_info(0, cpa, cpb, cr, cc, ck);
  int kt = 0;
  stage(cpa, cpb, cr, cc, ck, 0, 0, 0); stage(cpa, cpb, cr, cc, ck, 0, 0, 1);
  stage(cpa, cpb, cr, cc, ck, 0, 0, 2); stage(cpa, cpb, cr, cc, ck, 0, 0, 3);
  if constexpr (PRIO >= 3) {                 // K-tile 1 without its A-half 1 (staged in the first phase)
    stage(cpa, cpb, cr, cc, ck, 1, 1, 0); stage(cpa, cpb, cr, cc, ck, 1, 1, 2); stage(cpa, cpb, cr, cc, ck, 1, 1, 3);
  } else {
    stage(cpa, cpb, cr, cc, ck, 1, 1, 0); stage(cpa, cpb, cr, cc, ck, 1, 1, 3); stage(cpa, cpb, cr, cc, ck, 1, 1, 1);
  }
  asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
  sync();
  if (wm == 1) sync();                       // stagger the wave rows by one barrier
  if constexpr (PRIO == 1) { if (wm == 1) __builtin_amdgcn_s_setprio(1); }

  for (int g = 0; g < total; g += 2) {
    // K-tiles g, g+1 = (cur, kt), (cur, kt+1); g+2, g+3 = (nxt, k2), (nxt, k2+1)
    const bool last = kt + 2 >= nke;                            // this pair ends the tile
    const bf16 *npa = cpa, *npb = cpb;
    int nr = cr, nc = cc, nkl = ck, k2 = kt + 2;
    if (last) {
      tile_info(si + 1, npa, npb, nr, nc, nkl);
      k2 = 0;
    }
    if constexpr (PRIO >= 3) {
      // Two phases per K-tile (A-half 0, then A-half 1, each against both B-quarters): the load
      // segment before phase X reads A0, B0, B1 and stages A1 of the next K-tile; the one before
      // phase Y reads A1 and stages A0, B0, B1 of the K-tile two ahead (their last readers, the
      // other wave row's X-segment, finished one barrier earlier).  Waits, counted: at an X
      // segment the A1 staged one segment-pair ago (6 DMA staged since), at a Y segment the
      // A0/B0/B1 staged one pair ago (2 since) — each published by the barriers before its
      // readers' segments.
      if constexpr (PRIO != 7) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // PRIO 7: diagnostic, no waits
      rdA(0, 0); rdB2(0); stg(cpa, cpb, cr, cc, ck, kt + 1, 1, 1);
      // a tile's first K-tile pair: wave 0 stages its 256 bias words (LDS-DMA, no registers).  The next-but-one
      // counted wait of wave 0 covers it and a barrier follows, long before the tile's epilogue reads it;
      // the extra DMA only makes wave 0's counted waits stricter.
      if (kt == 0 && (p.flags & F_BIAS) && wave == 0) {
        int m0, n0, bz;
        if (pp_tile(p, si, m0, n0, bz)) {
          const int c = n0 + lane * 8;                          // 8 words per lane, lanes 0..31
          const uint32_t o = (lane < 32 && c < p.N) ? (uint32_t)(c * 2) : TW_OOB;
          buf_load_lds16(make_rsrc(p.bias), smem + 8 * PP_REGION + (si & 1) * 1024, o);
        }
      }
      mma2(0);
      if constexpr (PRIO != 7) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      if constexpr (PRIO == 4 || PRIO == 3) rdA(0, 1);      // PRIO 5: diagnostic, A-half 1 not read (LDS-read cost)
      stg(npa, npb, nr, nc, nkl, k2, 0, 0); stg(npa, npb, nr, nc, nkl, k2, 0, 2); stg(npa, npb, nr, nc, nkl, k2, 0, 3);
      mma2(1);
      if constexpr (PRIO != 7) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");   // PRIO 7: diagnostic, no waits
      rdA(1, 0); rdB2(1); stg(npa, npb, nr, nc, nkl, k2, 0, 1);
      mma2(0);
      if constexpr (PRIO != 7) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      if constexpr (PRIO == 4 || PRIO == 3) rdA(1, 1);
      stg(npa, npb, nr, nc, nkl, k2 + 1, 1, 0); stg(npa, npb, nr, nc, nkl, k2 + 1, 1, 2); stg(npa, npb, nr, nc, nkl, k2 + 1, 1, 3);
      mma2(1);
    } else {
    // even K-tile g from buffer 0
    rdB(0, 0); rdA(0, 0); stage(cpa, cpb, cr, cc, ck, kt + 1, 1, 2);  mma(0, 0);
    rdB(0, 1);            stage(npa, npb, nr, nc, nkl, k2, 0, 0);     mma(0, 1);
    rdA(0, 1);            stage(npa, npb, nr, nc, nkl, k2, 0, 3);     mma(1, 1);
    rdB(0, 0);            stage(npa, npb, nr, nc, nkl, k2, 0, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");            mma(1, 0);
    // odd K-tile g+1 from buffer 1
    rdB(1, 0); rdA(1, 0); stage(npa, npb, nr, nc, nkl, k2, 0, 2);     mma(0, 0);
    rdB(1, 1);            stage(npa, npb, nr, nc, nkl, k2 + 1, 1, 0); mma(0, 1);
    rdA(1, 1);            stage(npa, npb, nr, nc, nkl, k2 + 1, 1, 3); mma(1, 1);
    rdB(1, 0);            stage(npa, npb, nr, nc, nkl, k2 + 1, 1, 1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");            mma(1, 0);
    }
    if (last) {                                                 // tile finished
      pp_epi_part<H, KIND, 0, 8>(p, acc, si, wm, wn, lane, (const bf16*)(smem + 8 * PP_REGION + (si & 1) * 1024));
      ++si;
    }
    cpa = npa; cpb = npb; cr = nr; cc = nc; ck = nkl;
    kt = k2;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");             // no LDS-DMA may outlive the block
  if (wm == 0) sync();                       // balance the stagger barrier
}


template <bool H, bool AT, bool BT, int BM, int BN, int WM, int WN, int STAGES>
void launch(GemmP p, int batch, hipStream_t stream) {
  p.tiles_n = (p.N + BN - 1) / BN;
  p.tiles_mn = p.tiles_n * ((p.M + BM - 1) / BM);
  hipLaunchKernelGGL((gemm_kernel<H, AT, BT, BM, BN, WM, WN, STAGES>), dim3(p.tiles_mn, 1, batch), dim3(WM * WN * 64), 0,
                     stream, p);
}

// ---------------------------------------------------------------------------------------------
// Skinny GEMM for the decode step (M <= 128 rows = the batch of one greedy step, A and B K-major):
// weight streaming.  One 256-thread workgroup per 16-column slice of W (all M rows), the K range
// split over the 4 waves; W fragments load straight from HBM (16 B per lane, each W byte read
// once per step), A fragments from L2 (A is at most 128 x K bf16), MFMA 16x16x32 with swapped
// operands, the 4 wave partials summed through LDS, then the per-element epilogue (every flag).
// ---------------------------------------------------------------------------------------------
template <bool H>
__device__ __forceinline__ void epi_element(const GemmP& p, int m, int n, float v) {
  v = epi_value<H>(p, m, n, v);
  const int64_t co = (int64_t)m * p.ldc + n;
  if (p.c_dtype == TW_BF16) ((bf16*)p.C)[co] = f2e<H>(v);
  else ((float*)p.C)[co] = v;
}

template <bool H, int MF>
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
  const int mbase = (int)blockIdx.z * MF * 16;              // row block (batches of 65..128 rows: 2 x 64)
  const bf16* ap[MF];
  bool aok[MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int m = mbase + i * 16 + li;
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
        acc[i] = mma16<H>(wb[buf][j], ab[buf][j][i], acc[i]);
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
    const int ml = e >> 4, c = e & 15, n = n0 + c, m = mbase + ml;
    if (m < p.M && n < p.N) {
      const float v = part[0][ml][c] + part[1][ml][c] + part[2][ml][c] + part[3][ml][c];
      if (p.ws) p.ws[((int64_t)blockIdx.y * p.M + m) * p.N + n] = v;
      else epi_element<H>(p, m, n, v);
    }
  }
}

// sum of the split-K partials of the skinny kernel (in chunk order) + the full epilogue
template <bool H>
__global__ __launch_bounds__(256) void skinny_reduce_kernel(GemmP p, int S) {
  const int64_t total = (int64_t)p.M * p.N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    float v = p.ws[i];
    for (int s = 1; s < S; ++s) v += p.ws[s * total + i];
    epi_element<H>(p, (int)(i / p.N), (int)(i % p.N), v);
  }
}

// the same, 4 consecutive columns per thread (N % 4 == 0, ldc / ws rows 16-B aligned): the split-K tail
// of the mid-sized forward GEMMs
template <bool H>
__global__ __launch_bounds__(256) void sk_reduce_kernel(GemmP p, int S) {
  const int n4 = p.N >> 2;
  const int64_t total = (int64_t)p.M * p.N, work = (int64_t)p.M * n4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < work; i += (int64_t)gridDim.x * blockDim.x) {
    const int m = (int)(i / n4), n = (int)(i - (int64_t)m * n4) * 4;
    const float* w = p.ws + (int64_t)m * p.N + n;
    f32x4 a = *(const f32x4*)w;
    for (int s = 1; s < S; ++s) a += *(const f32x4*)(w + s * total);
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = epi_value<H>(p, m, n + r, a[r]);
    const int64_t co = (int64_t)m * p.ldc + n;
    if (p.c_dtype == TW_BF16)
      *(bf16x4*)((bf16*)p.C + co) = bf16x4{f2e<H>(v[0]), f2e<H>(v[1]), f2e<H>(v[2]), f2e<H>(v[3])};
    else *(f32x4*)((float*)p.C + co) = f32x4{v[0], v[1], v[2], v[3]};
  }
}

// GEMV for the batch <= 8 decode step: the body (LN staging, column dots, epilogue) lives in gemv_impl.h
template <bool H, int MR, int CPW, int PRE>
__global__ __launch_bounds__(256) void gemv_kernel(GemmP p, const float* __restrict__ lnw, const float* __restrict__ lnb,
                                                   float eps, GemvKV kv) {
  extern __shared__ __attribute__((aligned(16))) char gemv_smem[];
  bf16* xs = (bf16*)gemv_smem;                         // [MR][K] bf16
  const int lane = lane_id(), wave = wave_id_uniform();
  const int n0 = (blockIdx.x * 4 + wave) * CPW;
  // LayerNorm'd rows (K <= 1280, K % 256 == 0): the LN weight and bias go to LDS behind the rows ([2][K] fp32) by
  // LDS-DMA issued first, so they travel with the weight preload and the row loads instead of after the statistics
  float* lnp = nullptr;
  if (lnw && p.K <= 1280) {
    lnp = (float*)(gemv_smem + (size_t)MR * p.K * 2);
    const int per = p.K / 256;                         // 64-lane x 16-B pieces per array
    for (int i = wave; i < 2 * per; i += 4) {
      const float* src = i < per ? lnw : lnb;
      const int pc = (i % per) * 64;
      buf_load_lds16(make_rsrc(src), lnp + (i < per ? 0 : p.K) + pc * 4, (uint32_t)(pc + lane) * 16);
    }
  }
  bf16x8 wpre[CPW][PRE];
  gemv_preload<H, CPW, PRE>(p, n0, lane, wpre);
  gemv_stage_rows<H, MR>(p, lnw, lnb, eps, xs, wave, 4, lane, lnp);
  __syncthreads();
  if (n0 >= p.N) return;
  gemv_finish<H, MR, CPW, PRE>(p, kv, xs, n0, lane, wpre);
}

// Row blocks per skinny launch: batches of 65..128 rows run as 2 blocks of 64 (blockIdx.z) -- the
// 128-row form loads 8 A fragments per W fragment and measured 18 / 31 us on the large-v2 decode
// out_proj / fc2 at M = 128 against 14.5 / 18 us at M = 64 (tools/bench_decode_gemm.py); W is then read
// twice, the second time from L2.
constexpr int SKINNY_ROWS = 64;
int skinny_block_rows() { return SKINNY_ROWS; }
int skinny_row_blocks(int M) { return M > SKINNY_ROWS ? (M + SKINNY_ROWS - 1) / SKINNY_ROWS : 1; }

template <bool H>
void launch_skinny(GemmP p, hipStream_t stream, int S = 1) {
  const int zb = skinny_row_blocks(p.M);
  const dim3 grid((p.N + 15) / 16, S, zb);
  const int mf = zb > 1 ? skinny_block_rows() / 16 : (p.M + 15) / 16;
  switch (mf) {
    case 1: hipLaunchKernelGGL((gemm_skinny_kernel<H, 1>), grid, dim3(256), 0, stream, p); break;
    case 2: hipLaunchKernelGGL((gemm_skinny_kernel<H, 2>), grid, dim3(256), 0, stream, p); break;
    case 3:
    case 4: hipLaunchKernelGGL((gemm_skinny_kernel<H, 4>), grid, dim3(256), 0, stream, p); break;
    default: hipLaunchKernelGGL((gemm_skinny_kernel<H, 8>), grid, dim3(256), 0, stream, p); break;
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
  if (f == (F_ROUND | F_DGELU) && p.c_dtype == TW_BF16 && c8 && (p.ldaux % 8) == 0 &&
      (batch == 1 || (p.sAux % 8) == 0) && a16(p.aux))
    return EPI_DGELU;             // (the dX kernels: gemm_kernel's epilogue<..., DG>; elsewhere the generic form)
  if ((f & ~(F_BIAS | F_ROUND | F_CLAMP16)) == F_RES && p.res_mod == 0 && p.res_dtype == p.c_dtype) {
    if (p.c_dtype == TW_BF16 && c8 && (p.ldr % 8) == 0 && (batch == 1 || (p.sR % 8) == 0) && a16(p.res))
      return EPI_RES_BF16;
    if (f & F_CLAMP16) return EPI_GENERIC;
    if (p.c_dtype == TW_F32 && c4 && (p.ldr % 4) == 0 && (batch == 1 || (p.sR % 4) == 0) && a16(p.res))
      return EPI_RES_F32;
  }
  return EPI_GENERIC;
}

// the production variants are specialised on the epilogue kind (one fast epilogue + the generic one for
// ragged tiles per kernel: the split epilogue's three inlined parts stay within the register budget)
template <bool H, int PRIO>
void launch_pp_kind(const GemmP& p, int grid, hipStream_t stream) {
  if (p.K % BK) {     // a K tail (the conv stem's K = 240): the checked stager with the generic epilogue
    hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_GENERIC, false>), dim3(grid), dim3(512), 0, stream, p);
    return;
  }
  switch (p.epi) {
    case EPI_STORE_BF16: hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_STORE_BF16>), dim3(grid), dim3(512), 0, stream, p); break;
    case EPI_STORE_F32: hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_STORE_F32>), dim3(grid), dim3(512), 0, stream, p); break;
    case EPI_GELU: hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_GELU>), dim3(grid), dim3(512), 0, stream, p); break;
    case EPI_GELU_AUX: hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_GELU_AUX>), dim3(grid), dim3(512), 0, stream, p); break;
    case EPI_RES_BF16: hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_RES_BF16>), dim3(grid), dim3(512), 0, stream, p); break;
    case EPI_RES_F32: hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_RES_F32>), dim3(grid), dim3(512), 0, stream, p); break;
    default: hipLaunchKernelGGL((gemm_pp_kernel<H, PRIO, EPI_GENERIC>), dim3(grid), dim3(512), 0, stream, p); break;
  }
}

template <bool H>
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
  // default: two 32-MFMA phases per K-tile (PRIO 4); flags bits 15-17 select the diagnostic variants
  // (the round-2 variants PRIO 0/1/2/5/6/7 stay in the source but are instantiated only in a diagnostic build:
  // each is a full copy of the kernel; -DTW_PP_DIAG_VARIANTS brings them back, tools/bench_pp_prio.py)
  switch ((p.flags >> 15) & 7) {
#ifdef TW_PP_DIAG_VARIANTS
    case 1: hipLaunchKernelGGL((gemm_pp_kernel<H, 0>), dim3(grid), dim3(512), 0, stream, p); break;
    case 2: hipLaunchKernelGGL((gemm_pp_kernel<H, 2>), dim3(grid), dim3(512), 0, stream, p); break;
    case 3: hipLaunchKernelGGL((gemm_pp_kernel<H, 1>), dim3(grid), dim3(512), 0, stream, p); break;
    case 5: hipLaunchKernelGGL((gemm_pp_kernel<H, 5>), dim3(grid), dim3(512), 0, stream, p); break;
    case 6: hipLaunchKernelGGL((gemm_pp_kernel<H, 6>), dim3(grid), dim3(512), 0, stream, p); break;
    case 7: hipLaunchKernelGGL((gemm_pp_kernel<H, 7>), dim3(grid), dim3(512), 0, stream, p); break;
#endif
    default: launch_pp_kind<H, 4>(p, grid, stream); break;
  }
}

// ---------------------------------------------------------------------------------------------
// Split-K for weight gradients (dW = dYᵀ·X: both operands MN-major, K = tokens, few output tiles):
// the K range is cut into S chunks run as S batch entries of the 128x128 kernel into an fp32
// workspace, then one pass sums the chunks in order and applies the epilogue
//     C = [C +] round?(alpha * sum_s ws[s])
// (16-bit rounding point of the autocast product as in the unsplit kernel -- round 1: bf16, 2: fp16; the fp32
// sum over K is regrouped by chunk).  Workspace: splitk_workspace (per device, never freed).
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
    for (int r = 0; r < 4; ++r) o[r] = round == 2 ? rnd<true>(alpha * a[r]) : round ? rbf(alpha * a[r]) : alpha * a[r];
    if (accum) o += *(const f32x4*)cp;
    *(f32x4*)cp = o;
  }
}

// Split-K workspace: one block per device, grown (never freed: a captured HIP graph may hold the
// pointer of an older block, so old blocks are kept) outside stream capture only.  GEMMs of one
// device are issued from one stream at a time (the trainer's and the decoder's current stream).
// (gemm_f16.hip compiles this file again for the fp16 entry points and uses this TU's block)
#ifdef TW_GEMM_TU_F16
}  // namespace
void* tw_device_workspace(hipStream_t stream, size_t bytes);
namespace {
void* splitk_workspace(hipStream_t stream, size_t bytes) { return tw_device_workspace(stream, bytes); }
#else
void* splitk_workspace(hipStream_t stream, size_t bytes) {
  // at least 4 MiB per allocation: the small users (decode-attention partials, selection partials) then
  // find the block already large enough inside a captured decode step once any eager call has run
  bytes = std::max(bytes, (size_t)4 << 20);
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
#endif

int pp_grid_cus();

// S for a dW-shaped call, 0 = no split: fewer than 512 128x128 tiles, K split into S equal chunks; fp32 output, flags
// within {ROUND, ACCUM}.  The 128x128 split kernel holds two workgroups per CU (64 KiB of LDS each), so a grid of
// tiles x S workgroups runs in ceil(tiles x S / (2 x CUs)) rounds of K / S steps each; the 256x256 one holds one per
// CU at R times the 128 tile's rate per CU (R = 1.4 measured from the unsplit LM-head dW against the split dW
// products; TW_SK256_R overrides it, 0 = never), so ceil(tiles256 x S / CUs) rounds of 4 x K / S / R.  S (2..16,
// K % S == 0, >= 512 k per chunk) and the tile minimise that, the smaller S and the 128 tile on ties.  (Round 6.
// Powers of two before: c2's encoder 768 x 3072 weight gradients -- 144 tiles, K = 48 000 -- ran S = 4, 576
// workgroups = 1.125 rounds of 12 000 k; with the 128 tile alone S = 10, with the 256 tile S = 6 on 216 workgroups.
// c2 +1.3 %, c3 +0.3 % same-box, profiles/r06_al_ab.log.  Each chunk's fp32 sum is regrouped, as any split.)
int splitk_factor(const GemmP& p, int batch, int a_trans, int b_trans, int* tile) {
  *tile = 128;
  if (!a_trans || !b_trans || batch != 1 || p.c_dtype != TW_F32) return 0;
  if (p.flags & ~(F_ROUND | F_ACCUM) & 0xff) return 0;
  if ((p.N & 3) || (p.ldc & 3) || ((uintptr_t)p.C & 15)) return 0;
  const int64_t tiles = (int64_t)((p.M + 127) / 128) * ((p.N + 127) / 128);
  if (tiles >= 512) return 0;
  const int64_t cus = pp_grid_cus();
  const int64_t slots = 2 * cus;
  // time units: one CU's 128x128 x 1k of work at the 128-tile rate.  A 128-tile round holds two workgroups per CU
  // (2 units per k); a 256-tile round one workgroup of four times the area at R times the 128-tile rate.
  static const double R = [] {
    const char* e = getenv("TW_SK256_R");
    return e ? atof(e) : 1.4;
  }();
  const int64_t tiles256 = (int64_t)((p.M + 255) / 256) * ((p.N + 255) / 256);
  double best_cost = (double)((tiles + slots - 1) / slots) * 2.0 * p.K;   // unsplit: rounds x K
  int best = 0;
  for (int S = 2; S <= 16; ++S) {
    if (p.K % S != 0 || p.K / S < 512) continue;
    const double kc = (double)(p.K / S);
    const double c128 = (double)((tiles * S + slots - 1) / slots) * 2.0 * kc;
    if (c128 < best_cost) { best_cost = c128; best = S; *tile = 128; }
    if (R > 0) {
      const double c256 = (double)((tiles256 * S + cus - 1) / cus) * 4.0 * kc / R;
      if (c256 < best_cost) { best_cost = c256; best = S; *tile = 256; }
    }
  }
  return best;
}

template <bool H, bool AT, bool BT>
void dispatch(GemmP p, int batch, hipStream_t stream, int tile) {
  if constexpr (H && (AT || BT)) {
    // fp16 training's dX / dW products: the 2-stage 256x256 and 128x128 tiles only (the 256x128 rings are forced
    // A/B variants of the bf16 kernels; not instantiating them for fp16 keeps the library's build time down)
    if (tile == 256) launch<H, AT, BT, 256, 256, 2, 4, 2>(p, batch, stream);
    else launch<H, AT, BT, 128, 128, 2, 2, 2>(p, batch, stream);
    return;
  }
  if (tile == 2562 && !AT && !BT) launch_pp<H>(p, batch, stream);
  else if (tile == 1284) {
    if constexpr (!AT && !BT) launch<H, AT, BT, 128, 128, 2, 2, 4>(p, batch, stream);   // 4-stage ring
  }
  else if (tile == 256) launch<H, AT, BT, 256, 256, 2, 4, 2>(p, batch, stream);
  else if (tile == 2561) launch<H, AT, BT, 256, 128, 4, 2, 3>(p, batch, stream);
  else if (tile == 2563) launch<H, AT, BT, 256, 128, 4, 2, 2>(p, batch, stream);
  else launch<H, AT, BT, 128, 128, 2, 2, 2>(p, batch, stream);
}

int pp_grid_cus() {
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n >= 8 ? n : 8;
  }();
  return cus & ~7;
}

// ---------------------------------------------------------------------------------------------
// Data-parallel + split-K tail for the mid-sized forward GEMMs (the decoder's N = 1280 Linears at
// M = 64 x 447: 560 256-tiles = 2.19 rounds of the 256 persistent workgroups).  The m-tile rows that
// fill whole rounds run as ordinary persistent tiles (full epilogue); the remaining m-tile rows are cut
// into S equal K chunks run as S batch entries of the same kernel into fp32 partials (one round),
// then skinny_reduce_kernel sums the chunks in order and applies the full epilogue to those rows.
// Returns S (0 = no plan: the caller takes the 128x128 path).  Numerics: the tail rows' fp32 sum over
// K is regrouped by chunk (as the dW split-K); every other row is the unsplit kernel's.
// ---------------------------------------------------------------------------------------------
int sk_tail_plan(const GemmP& p, int batch, int& m_dp) {
  if (batch != 1 || p.res_mod != 0 || (p.N & 3) || (p.ldc & 3) || ((uintptr_t)p.C & 15)) return 0;
  const int G = pp_grid_cus();
  const int tn = (p.N + 255) / 256, tm = (p.M + 255) / 256;
  const int64_t T = (int64_t)tn * tm;
  if (T < G && p.M >= 256) {
    // less than one round (the decode step's fc2 at a 512-clip batch: 10 tiles of K = 5120, 60 us on 40
    // 128x128 tiles): every tile split into up to 16 K-chunks, no whole-round part
    m_dp = 0;
    int best = 0;
    for (int S = 2; S <= 16; ++S)
      if (p.K % (64 * S) == 0 && T * S <= G && p.K / S >= 256) best = S;
    return best;
  }
  if (T < G || T >= 4 * G) return 0;                  // < 1 round: nothing to fill; many rounds: tail small
  m_dp = (int)((T / G) * G / tn);                      // m-tile rows of whole rounds
  const int tail = (tm - m_dp) * tn;
  if (tail <= 0 || m_dp <= 0) return 0;
  int best = 0;
  for (int S = 2; S <= 8; ++S)
    if (p.K % (64 * S) == 0 && (int64_t)tail * S <= G && p.K / S >= 256) best = S;
  return best;
}

template <bool H>
int launch_sk_tail(GemmP p, int S, int m_dp, hipStream_t stream) {
  const int Mt = p.M - m_dp * 256;
  const size_t bytes = (size_t)S * Mt * p.N * sizeof(float);
  float* ws = (float*)splitk_workspace(stream, bytes);
  if (!ws) return 0;
  if (m_dp > 0) {
    GemmP d = p;                                       // whole rounds: the unsplit kernel
    d.M = m_dp * 256;
    launch_pp<H>(d, 1, stream);
    TW_CHECK_LAUNCH();
  }
  GemmP q = p;                                         // tail rows: S K-chunks -> fp32 partials
  const int64_t r0 = (int64_t)m_dp * 256;
  q.A = p.A + r0 * p.lda;
  q.M = Mt;
  q.K = p.K / S;
  q.sA = q.K;                                          // chunk s starts at column s*K/S of A and B
  q.sB = q.K;
  q.C = ws; q.ldc = p.N; q.sC = (int64_t)Mt * p.N; q.c_dtype = TW_F32;
  q.alpha = 1.f; q.flags = 0; q.bias = nullptr; q.res = nullptr; q.aux = nullptr; q.ws = nullptr;
  q.group_m = 1;
  q.epi = pick_epilogue(q, S);
  launch_pp<H>(q, S, stream);
  TW_CHECK_LAUNCH();
  GemmP r = p;                                         // ordered chunk sum + the full epilogue
  const int csz = p.c_dtype == TW_BF16 ? 2 : 4;
  r.C = (char*)p.C + r0 * p.ldc * csz;
  if (p.res) r.res = (const char*)p.res + r0 * p.ldr * (p.res_dtype == TW_BF16 ? 2 : 4);
  if (p.aux) r.aux = p.aux + r0 * p.ldaux;
  r.M = Mt;
  r.ws = ws;
  const int64_t work = (int64_t)Mt * (p.N / 4);
  hipLaunchKernelGGL(sk_reduce_kernel<H>, dim3((int)std::min<int64_t>((work + 255) / 256, 4096)), dim3(256), 0,
                     stream, r, S);
  TW_CHECK_LAUNCH();
  return 1;
}

// ---------------------------------------------------------------------------------------------
// Whole rounds persistent + a 128x128 tail: for grids whose last round of 256-tiles would leave most of the
// persistent kernel's workgroups idle (the decoder's N = 1280 projections at M = 64 x 447: 560 256-tiles = 2.19
// rounds, of which the third runs 48 tiles on 256 CUs), the m-tile rows of whole rounds run on the persistent
// kernel and the remaining rows as 128x128 tiles on the 4-stage ring -- when they fit one round of it.  Both
// kernels accumulate every output in the same K order (tests/test_kernels_gpu.py forced-tile identity), so the
// result is bit-identical to either kernel alone.  Returns 0 (no plan) or 1, m_dp = m-tile rows of whole rounds.
int dp_tail_plan(const GemmP& p, int batch, int& m_dp) {
  if (batch != 1 || p.res_mod != 0) return 0;
  const int G = pp_grid_cus();
  const int tn = (p.N + 255) / 256, tm = (p.M + 255) / 256;
  const int64_t T = (int64_t)tn * tm;
  if (T < G || T >= 8 * G) return 0;
  const int64_t rest = T % G;                            // 256-tiles of the last, partial round
  if (rest == 0 || rest * 10 > (int64_t)G * 6) return 0;  // last round >= 60 % busy: keep it
  m_dp = (int)((T / G) * G / tn);
  const int rows = p.M - m_dp * 256;
  const int64_t t128 = (int64_t)((rows + 127) / 128) * ((p.N + 127) / 128);
  return (m_dp > 0 && rows > 0 && t128 <= G) ? 1 : 0;
}

template <bool H>
int launch_dp_tail(const GemmP& p, int m_dp, hipStream_t stream) {
  GemmP d = p;                                           // whole rounds: the persistent kernel
  d.M = m_dp * 256;
  launch_pp<H>(d, 1, stream);
  TW_CHECK_LAUNCH();
  GemmP q = p;                                           // the remaining rows: 128x128 tiles, 4-stage ring
  const int64_t r0 = (int64_t)m_dp * 256;
  const int csz = p.c_dtype == TW_BF16 ? 2 : 4;
  q.A = p.A + r0 * p.lda;
  q.M = p.M - (int)r0;
  q.C = (char*)p.C + r0 * p.ldc * csz;
  if (p.res) q.res = (const char*)p.res + r0 * p.ldr * (p.res_dtype == TW_BF16 ? 2 : 4);
  if (p.aux) q.aux = p.aux + r0 * p.ldaux;
  q.epi = pick_epilogue(q, 1);
  launch<H, false, false, 128, 128, 2, 2, 4>(q, 1, stream);
  TW_CHECK_LAUNCH();
  return 1;
}

// ---------------------------------------------------------------------------------------------
// fp16 grids ragged in M or N (the fp16 teacher decoder's M = B x 447 rows, the LM head's N = 51 904): the whole
// 256x256 tiles [0, Mf) x [0, Nf) on the persistent kernel, the right strip [0, M) x [Nf, N) and the bottom strip
// [Mf, M) x [0, Nf) on the 128x128 kernel.  Every output keeps the K order of either kernel: bit-identical to the
// 128x128 kernel alone (tests/test_fp16_train_gpu.py).
// ---------------------------------------------------------------------------------------------
template <bool H>
int launch_pp_edges(const GemmP& p, hipStream_t stream) {
  const int Mf = p.M / 256 * 256, Nf = p.N / 256 * 256;
  const int csz = p.c_dtype == TW_BF16 ? 2 : 4, rsz = p.res_dtype == TW_BF16 ? 2 : 4;
  auto sub = [&](int m0, int n0, int M, int N) {
    GemmP q = p;
    q.A = p.A + (int64_t)m0 * p.lda;
    q.B = p.B + (int64_t)n0 * p.ldb;
    q.C = (char*)p.C + ((int64_t)m0 * p.ldc + n0) * csz;
    if (p.bias) q.bias = p.bias + n0;
    if (p.res) q.res = (const char*)p.res + ((int64_t)m0 * p.ldr + n0) * rsz;
    if (p.aux) q.aux = p.aux + (int64_t)m0 * p.ldaux + n0;
    q.M = M;
    q.N = N;
    q.epi = pick_epilogue(q, 1);
    return q;
  };
  launch_pp<H>(sub(0, 0, Mf, Nf), 1, stream);
  TW_CHECK_LAUNCH();
  if (Nf < p.N) {
    launch<H, false, false, 128, 128, 2, 2, 2>(sub(0, Nf, p.M, p.N - Nf), 1, stream);
    TW_CHECK_LAUNCH();
  }
  if (Mf < p.M) {
    launch<H, false, false, 128, 128, 2, 2, 2>(sub(Mf, 0, p.M - Mf, Nf), 1, stream);
    TW_CHECK_LAUNCH();
  }
  return TW_OK;
}

}  // namespace

// the same per-device block for other stream-ordered scratch users (decode attention split partials)
#ifndef TW_GEMM_TU_F16
void* tw_device_workspace(hipStream_t stream, size_t bytes) { return splitk_workspace(stream, bytes); }
#endif

namespace {

// H = false: tw_gemm_bf16; H = true: tw_gemm_f16 (the fp16 model's forward products, and since round 6 the
// transposed dX / dW products of fp16-autocast training: the same kernels instantiated for fp16 words)
template <bool H>
int gemm_run(const void* A, int64_t lda, int a_trans, const void* B, int64_t ldb, int b_trans, void* C, int64_t ldc,
             int c_dtype, int M, int N, int K, int batch, int64_t sA, int64_t sB, int64_t sC, float alpha,
             const void* bias, const void* res, int64_t ldr, int64_t sR, int res_dtype, int res_mod, void* aux,
             int64_t ldaux, int64_t sAux, int flags, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return TW_OK;
  if (H) {
    if ((c_dtype != TW_F32 && c_dtype != TW_F16) || ((flags & F_RES) && res_dtype != TW_F32 && res_dtype != TW_F16))
      return TW_EUNSUPPORTED;
    // inside the kernels the 16-bit code means "the operand type" (gemm_impl.h)
    if (c_dtype == TW_F16) c_dtype = TW_BF16;
    if (res_dtype == TW_F16) res_dtype = TW_BF16;
  } else if (flags & F_CLAMP16) {
    return TW_EINVAL;
  }
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
  if (res_dtype != TW_F32 && res_dtype != TW_BF16) res_dtype = TW_F32;   // unused without F_RES
  GemmP p;
  p.A = (const bf16*)A; p.B = (const bf16*)B; p.C = C;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.sA = sA; p.sB = sB; p.sC = sC; p.alpha = alpha; p.bias = (const bf16*)bias;
  p.res = res; p.ldr = ldr; p.sR = sR; p.res_dtype = res_dtype; p.res_mod = res_mod;
  p.aux = (bf16*)aux; p.ldaux = ldaux; p.sAux = sAux; p.c_dtype = c_dtype; p.flags = flags;
  p.ws = nullptr;
  // tile order: runs of 8 m-tiles walked n-tile by n-tile for the tall, short-K forward GEMMs (the
  // encoder's M = B x 1500 projections: +3-5 % from L2 reuse of the weight panels,
  // tools/bench_pp_prio.py with TW_GEMM_GROUP_M); plain row-major elsewhere (K = 5120 and the
  // decoder's M = B x 447 shapes lose with grouping: round 4, profiles/r04_b_l2_epilogue_study.txt)
  const bool grouped = !a_trans && !b_trans && batch == 1 && M >= 65536 && K <= 2048;
  p.group_m = grouped ? 8 : 1;
  if ((flags >> 24) & 15) p.group_m = (flags >> 24) & 15;     // forced tile order (A/B runs: tools/bench_group.py)
  p.epi = pick_epilogue(p, batch);
  // 256x256 tiles (8 waves) when the problem has enough tiles to fill the chip, else 128x128
  const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256) * batch;
  // measured crossovers (tools/bench_gemm.py, r01, specialised epilogues): the persistent 256x256
  // ping-pong kernel wins every large K-major/K-major shape (1.05-1.27 PFLOP/s); the 2-stage
  // 256x256 tile the large transposed ones; 128x128 the small grids (< ~1000 256-tiles).  The
  // 256x128 3-stage ring is kept as a forced variant only.
  int tile = (t256 >= 1000 && K >= 256) ? 256 : 128;
  // very long K (the LM-head input gradient, K = 51 904): the persistent kernel wins from one round up
  // (3356 vs 4006 us on 560 tiles, tools/bench_head_bwd.py), its per-tile fixed cost being amortised
  if (!a_trans && !b_trans && K >= 8192 && t256 >= pp_grid_cus()) tile = 256;
  // ... and its transposed-B form (the student's LM-head dX = dlogits . E, K = 51 904, 560 tiles) on the 2-stage
  // 256x256 tile: 4059 vs 4370 us on the 128x128 one (tools/bench_gemm.py "dX head", profiles/r06_a_gemm.log)
  if (!a_trans && b_trans && K >= 8192 && t256 >= pp_grid_cus() / 2) tile = 256;   // c2's: 168 tiles, 1297 vs 1643 us
  // K-major forward grids of 1-4 rounds whose rounds are well filled (c2's B = 32 shapes: the teacher encoder's
  // N = 1280 Linears at M = 48 000, 940 256-tiles = 3.67 rounds, 92 % of the workgroup-rounds busy; the student
  // decoder's fused QKV and fc1): the persistent kernel.  Grids with a mostly idle last round take the whole-round
  // + 128x128 tail split below (dp_tail_plan).  Fill threshold 85 % (c2 +0.6 %, c3 unchanged: same box, round 4)
  // (K >= 1024: at c2's student decoder K = 768 -- 12 K-tiles per tile -- the 128x128 kernel wins: fused QKV 69 vs
  // 85 us, fc1 90 vs 105 us, profiles/r06_l_gemm_c2.log)
  if (!a_trans && !b_trans && tile == 128 && K >= 1024) {
    const int64_t G = pp_grid_cus();
    if (t256 >= G && t256 * 100 >= ((t256 + G - 1) / G) * G * 85) tile = 256;
  }
  if (tile == 256 && !a_trans && !b_trans) tile = 2562;
  if (flags & 256) tile = 128;        // forced tile (benchmarking / A-B comparisons)
  if (flags & 512) tile = 256;
  if (flags & 1024) tile = 2561;      // 256x128, 3-stage ring
  if (flags & 2048) tile = 2562;      // 256x256 ping-pong (K-major A and B only)
  // the fp16 persistent kernel is compiled with the fast full-tile epilogues only (gemm_impl.h epilogue_k): a grid
  // ragged in M or N runs its whole 256x256 tiles there and the edge strips on the 128x128 kernel (tile 2564,
  // launch_pp_edges); K tails, batches, row-periodic residuals and the generic epilogue kind take the 128x128 kernel
  if (H && tile == 2562 && ((M % 256) || (N % 256))) {
    const bool edges = (K % BK) == 0 && p.epi != EPI_GENERIC && batch == 1 && res_mod == 0 && M >= 256 && N >= 256;
    tile = edges ? 2564 : 128;
  }
  if (H && tile == 2562 && ((K % BK) || p.epi == EPI_GENERIC)) tile = 128;
  const int64_t ntiles = (tile == 256 || tile == 2562 || tile == 2564) ? t256 / batch
                                                                       : (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (ntiles > 0x7fffffff || ntiles * batch > 0x7fffffff || batch > 65535) return TW_EINVAL;
  // decode-step GEMMs (tools/bench_skinny.py, r01): the weight-streaming kernel wins for N <= 3840
  // (and N <= 8192 at M <= 64); the LM head and wide M=128 GEMMs stream faster as 128x128 tiles
  // (row-blocked skinny launches above 128 rows measured slower at M = 512, tools/bench_decode_gemm.py: qkv 50 vs
  // 21 us, fc2 69 vs 60 us against the 128x128 tiles)
  const bool skinny = !a_trans && !b_trans && batch == 1 && M <= 128 && (N <= 4096 || (M <= 64 && N <= 8192)) &&
                      !(flags & (256 | 512 | 1024 | 2048));
  if (skinny && ((uintptr_t)A & 15) == 0) {
    // decode-step GEMMs: stream W once.  With fewer than 512 workgroups and M > 32 the K range is
    // also split over workgroups (chunks of >= 4 k-steps) into fp32 partials, reduced with the
    // epilogue (c4 batch 64 / 128: -3 / -4 % per step; at batch 1 the extra launch loses 9 %).
    p.ws = nullptr;
    const int nwg = (N + 15) / 16 * skinny_row_blocks(M), nk = (K + 31) / 32;
    int S = std::min((512 + nwg - 1) / nwg, nk / 4);
    if ((flags & 16384) || M <= 32) S = 1;          // small batches: the reduce launch costs more than it saves
    void* ws = S > 1 ? splitk_workspace(stream, (size_t)S * M * N * sizeof(float)) : nullptr;
    if (ws) {
      p.ws = (float*)ws;
      launch_skinny<H>(p, stream, S);
      TW_CHECK_LAUNCH();
      const int64_t total = (int64_t)M * N;
      hipLaunchKernelGGL(skinny_reduce_kernel<H>, dim3((int)std::min<int64_t>((total + 255) / 256, 2048)), dim3(256), 0,
                         stream, p, S);
    } else {
      launch_skinny<H>(p, stream);
    }
    TW_CHECK_LAUNCH();
    return TW_OK;
  }
  if (!(flags & (16384 | 256 | 512 | 1024 | 2048))) {   // 16384: no split-K; forced tiles: A/B runs
    int sk_tile = 128;
    const int S = splitk_factor(p, batch, a_trans, b_trans, &sk_tile);
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
      if (sk_tile == 256) launch<H, true, true, 256, 256, 2, 4, 2>(q, S, stream);
      else launch<H, true, true, 128, 128, 2, 2, 2>(q, S, stream);
      TW_CHECK_LAUNCH();
      const int64_t work = (int64_t)M * (N / 4);
      const int grid = (int)std::min<int64_t>((work + 255) / 256, 4096);
      hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid), dim3(256), 0, stream, (const float*)ws, S,
                         (int64_t)M * N, (float*)C, ldc, M, N, alpha, (flags & F_ROUND) ? (H ? 2 : 1) : 0,
                         (flags & F_ACCUM) ? 1 : 0);
      TW_CHECK_LAUNCH();
      return TW_OK;
    }
  }
  // mid-sized forward grids (1-4 rounds of 256-tiles): whole rounds persistent + a split-K tail
  // (flag 262144 forces the 256x128 2-stage tile)
  if (flags & 262144) tile = 2563;
  // (tools/bench_gemm_dec.py: fc2 K = 5120 417 -> 347 us; at K = 1280 the split's fp32 round trip costs
  // more than the third round it saves, 125 -> 140 us, so short K stays on the 128x128 kernel; grids of less than
  // one round, the 512-clip decode step's Linears, follow the same K >= 3072 rule)
  if (!a_trans && !b_trans && tile == 128 && K >= 3072 &&
      !(flags & (16384 | 256 | 512 | 1024 | 2048 | 262144))) {
    int m_dp = 0;
    const int S = sk_tail_plan(p, batch, m_dp);
    // (fp16: the persistent kernel runs full tiles only, so both parts must be whole 256-row blocks)
    const bool full = !H || ((N % 256) == 0 && ((M - m_dp * 256) % 256) == 0 && p.epi != EPI_GENERIC);
    if (S > 0 && full && launch_sk_tail<H>(p, S, m_dp, stream)) return TW_OK;
  }
  // whole rounds persistent + a 128x128 tail (dp_tail_plan)
  if (!a_trans && !b_trans && !(flags & (16384 | 256 | 512 | 1024 | 2048 | 262144))) {
    int m_dp = 0;
    // (fp16: the persistent part must be whole 256x256 tiles with a fast epilogue)
    if (dp_tail_plan(p, batch, m_dp) && (!H || ((N % 256) == 0 && (K % BK) == 0 && p.epi != EPI_GENERIC)) &&
        launch_dp_tail<H>(p, m_dp, stream))
      return TW_OK;
  }
  // Grids of at most one 128x128 tile per CU (the 512-clip decode step's Linears: 40-160 tiles, one workgroup per
  // CU anyway) run on a 4-stage ring: three K-steps in flight instead of one hide the load latency that bounds a
  // 20-K-step tile.  Same tile, same K order: bit-identical.  c4 fp16 155.8 -> 158.5 utt/s, c5 16.93 -> 17.09
  // audio s/s (same box, profiles/r03_s_gemm_deep_ab.log).  Flag 256 (forced 128x128) keeps the 2-stage kernel.
  if (tile == 128 && !a_trans && !b_trans && !(flags & 256) &&
      (int64_t)((M + 127) / 128) * ((N + 127) / 128) * batch <= pp_grid_cus())
    tile = 1284;
  if (tile == 2564) return launch_pp_edges<H>(p, stream);
  if (!a_trans && !b_trans) dispatch<H, false, false>(p, batch, stream, tile);
  else if (!a_trans && b_trans) dispatch<H, false, true>(p, batch, stream, tile);
  else if (a_trans && !b_trans) dispatch<H, true, false>(p, batch, stream, tile);
  else dispatch<H, true, true>(p, batch, stream, tile);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

template <bool H>
int gemv_run(const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps, const void* W, int64_t ldw,
             void* C, int64_t ldc, int c_dtype, int M, int N, int K, const void* bias, const void* res, int64_t ldr,
             int res_dtype, void* aux, int64_t ldaux, int flags, void* kv_cache, int64_t kv_sb, int64_t kv_ld,
             int kv_col0, const int* t_dev, hipStream_t stream) {
  if (M <= 0 || N <= 0) return TW_OK;
  if (H) {
    if ((c_dtype != TW_F32 && c_dtype != TW_F16) || ((flags & F_RES) && res_dtype != TW_F32 && res_dtype != TW_F16))
      return TW_EUNSUPPORTED;
    if (c_dtype == TW_F16) c_dtype = TW_BF16;
    if (res_dtype == TW_F16) res_dtype = TW_BF16;
  } else if (flags & F_CLAMP16) {
    return TW_EINVAL;
  }
  if (M > 8 || K <= 0 || (K % 8) || (ldx % 8) || (ldw % 8)) return TW_EINVAL;
  if (((uintptr_t)x & 15) || ((uintptr_t)W & 15)) return TW_EINVAL;
  if (ln_w && (!ln_b || (K % 256) || (((uintptr_t)ln_w | (uintptr_t)ln_b) & 15))) return TW_EINVAL;
  if ((flags & F_BIAS) && !bias) return TW_EINVAL;
  if ((flags & F_RES) && !res) return TW_EINVAL;
  if ((flags & (F_AUX_OUT | F_DGELU)) && !aux) return TW_EINVAL;
  if (c_dtype != TW_F32 && c_dtype != TW_BF16) return TW_EUNSUPPORTED;
  const int mr = M == 1 ? 1 : M == 2 ? 2 : M <= 4 ? 4 : 8;
  if ((size_t)mr * K * 2 > 80 * 1024) return TW_EUNSUPPORTED;        // A rows in LDS
  if (kv_cache && (!t_dev || kv_col0 < 0 || kv_col0 >= N)) return TW_EINVAL;
  const GemvKV kv{kv_cache, kv_sb, kv_ld, kv_col0, t_dev};
  GemmP p = {};
  p.A = (const bf16*)x; p.B = (const bf16*)W; p.C = C;
  p.lda = ldx; p.ldb = ldw; p.ldc = ldc; p.M = M; p.N = N; p.K = K;
  p.alpha = 1.f; p.bias = (const bf16*)bias;
  p.res = res; p.ldr = ldr; p.res_dtype = res_dtype; p.res_mod = 0;
  p.aux = (bf16*)aux; p.ldaux = ldaux; p.c_dtype = c_dtype; p.flags = flags;
  // one output column per wave; 8 for very wide N (the LM head: fewer workgroups repeating the A prologue), 4 of
  // them at 5..8 rows (8 x 8 accumulators and their preloads cap a wave at 2 per SIMD); 2 for the wide decode Linears
  // (fc1, QKV) at 3..8 rows, so each LDS read of the staged rows feeds two columns.  The per-output arithmetic does
  // not depend on the column count (tests/test_kernels_gpu.py::test_gemv_rows_independent_of_batch)
  const int cpw = N >= 16384 ? (mr == 8 || mr == 1 ? 4 : 8) : (mr >= 4 && N >= 3072 && K <= 1536) ? 2 : 1;
  const dim3 grid((N + 4 * cpw - 1) / (4 * cpw));
  const size_t lds = (size_t)mr * K * 2 + (ln_w && K <= 1280 ? (size_t)2 * K * 4 : 0);
#define TW_GEMV(MR_, CPW_, PRE_) \
  hipLaunchKernelGGL((gemv_kernel<H, MR_, CPW_, PRE_>), grid, dim3(256), lds, stream, p, ln_w, ln_b, eps, kv)
  if (cpw == 8) {
    if (mr == 1) TW_GEMV(1, 8, 3);
    else if (mr == 2) TW_GEMV(2, 8, 3);
    else TW_GEMV(4, 8, 3);
  } else if (cpw == 4) {
    if (mr == 1) TW_GEMV(1, 4, 3);
    else TW_GEMV(8, 4, 3);
  } else if (cpw == 2) {
    if (mr == 4) TW_GEMV(4, 2, 3);
    else TW_GEMV(8, 2, 3);
  } else if (K <= 1536) {
    if (mr == 1) TW_GEMV(1, 1, 3);
    else if (mr == 2) TW_GEMV(2, 1, 3);
    else if (mr == 4) TW_GEMV(4, 1, 3);
    else TW_GEMV(8, 1, 3);
  } else {
    if (mr == 1) TW_GEMV(1, 1, 10);
    else if (mr == 2) TW_GEMV(2, 1, 10);
    else if (mr == 4) TW_GEMV(4, 1, 10);
    else TW_GEMV(8, 1, 10);
  }
#undef TW_GEMV
  TW_CHECK_LAUNCH();
  return TW_OK;
}

}  // namespace

#ifndef TW_GEMM_TU_F16
extern "C" int tw_gemm_bf16(const void* A, int64_t lda, int a_trans, const void* B, int64_t ldb, int b_trans,
                            void* C, int64_t ldc, int c_dtype, int M, int N, int K, int batch,
                            int64_t sA, int64_t sB, int64_t sC, float alpha, const void* bias,
                            const void* res, int64_t ldr, int64_t sR, int res_dtype, int res_mod,
                            void* aux, int64_t ldaux, int64_t sAux, int flags, hipStream_t stream) {
  return gemm_run<false>(A, lda, a_trans, B, ldb, b_trans, C, ldc, c_dtype, M, N, K, batch, sA, sB, sC, alpha, bias,
                         res, ldr, sR, res_dtype, res_mod, aux, ldaux, sAux, flags, stream);
}

extern "C" int tw_gemv_bf16(const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps, const void* W,
                            int64_t ldw, void* C, int64_t ldc, int c_dtype, int M, int N, int K, const void* bias,
                            const void* res, int64_t ldr, int res_dtype, void* aux, int64_t ldaux, int flags,
                            void* kv_cache, int64_t kv_sb, int64_t kv_ld, int kv_col0, const int* t_dev,
                            hipStream_t stream) {
  return gemv_run<false>(x, ldx, ln_w, ln_b, eps, W, ldw, C, ldc, c_dtype, M, N, K, bias, res, ldr, res_dtype, aux,
                         ldaux, flags, kv_cache, kv_sb, kv_ld, kv_col0, t_dev, stream);
}

#else
extern "C" int tw_gemm_f16(const void* A, int64_t lda, int a_trans, const void* B, int64_t ldb, int b_trans,
                           void* C, int64_t ldc, int c_dtype, int M, int N, int K, int batch,
                           int64_t sA, int64_t sB, int64_t sC, float alpha, const void* bias,
                           const void* res, int64_t ldr, int64_t sR, int res_dtype, int res_mod,
                           void* aux, int64_t ldaux, int64_t sAux, int flags, hipStream_t stream) {
  return gemm_run<true>(A, lda, a_trans, B, ldb, b_trans, C, ldc, c_dtype, M, N, K, batch, sA, sB, sC, alpha, bias,
                        res, ldr, sR, res_dtype, res_mod, aux, ldaux, sAux, flags, stream);
}

extern "C" int tw_gemv_f16(const void* x, int64_t ldx, const float* ln_w, const float* ln_b, float eps, const void* W,
                           int64_t ldw, void* C, int64_t ldc, int c_dtype, int M, int N, int K, const void* bias,
                           const void* res, int64_t ldr, int res_dtype, void* aux, int64_t ldaux, int flags,
                           void* kv_cache, int64_t kv_sb, int64_t kv_ld, int kv_col0, const int* t_dev,
                           hipStream_t stream) {
  return gemv_run<true>(x, ldx, ln_w, ln_b, eps, W, ldw, C, ldc, c_dtype, M, N, K, bias, res, ldr, res_dtype, aux,
                        ldaux, flags, kv_cache, kv_sb, kv_ld, kv_col0, t_dev, stream);
}
#endif
