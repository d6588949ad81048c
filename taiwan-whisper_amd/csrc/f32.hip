// fp32 arithmetic path (mixed_precision = "no": the reference's default --dtype float32,
// training/run_distillation.py:815-823, and the fp32 decode whose greedy token ids must equal HF
// fp32 generate bit for bit).  Every Linear / Conv1d-as-GEMM / attention product runs on the
// exact-fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 operands, fp32 accumulate -- the same
// instruction log-mel's DFT uses); nothing is rounded to bf16.
//
//  * tw_gemm_f32: C[b] = epi(alpha * op(A[b]) op(B[b])^T), 128x128 tiles, 4 waves of 64x64
//    (4x4 MFMA blocks), BK = 16 through a two-stage LDS ring ([k][m] images, row pitch 144 floats:
//    fragment reads conflict-free), register-prefetched global loads.  Two batch levels
//    (outer b, inner h: the attention products run over (batch, head) pairs with head columns
//    interleaved in the activation rows).  Epilogue: alpha -> +bias -> x gelu'(aux) (DGELU) ->
//    aux := v, v = gelu(v) (GELU; erf form with libm erff, HF ACT2FN["gelu"]) -> +res -> +C_old.
//  * tw_attn_fwd_f32 / tw_attn_bwd_f32: SDPA (HF modeling_whisper.py:265-350) composed from
//    those GEMMs and two row kernels over a caller-provided score workspace: S = scale Q K^T,
//    P = softmax(S) (exact two-pass, global row max, causal mask, lse out), O = P V; backward
//    P = exp(scale Q K^T - lse), dP = dO V^T, dS = scale P (dP - rowsum(dO o O)), dV = P^T dO,
//    dQ = dS K, dK = dS^T Q.  (B, H) pairs are processed in chunks that fit the workspace.
//  * conv-stem helpers in fp32: mel -> time-major conv1 input, im2col, GELU backward.
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 16, LDP = 144, NT = 256;

enum { F_BIAS = 1, F_GELU = 4, F_RES = 8, F_ACCUM = 16, F_AUX_OUT = 32, F_DGELU = 64 };

struct G32P {
  const float* A; int64_t lda; int at;
  const float* B; int64_t ldb; int bt;
  float* C; int64_t ldc;
  int M, N, K, tiles_n, batch_in;
  int64_t sA, sB, sC, sAi, sBi, sCi;
  float alpha;
  const float* bias;
  const float* res; int64_t ldr, sR; int res_mod;
  float* aux; int64_t ldaux, sAux;
  int flags;
};

__device__ __forceinline__ float gelu_exact(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f)); }
__device__ __forceinline__ float gelu_exact_grad(float x) {
  const float cdf = 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  const float pdf = expf(-0.5f * x * x) * 0.39894228040143267794f;
  return cdf + x * pdf;
}

// Stage loader: 128 rows (m or n) x 16 k of X into registers (8 floats per thread).
//   !trans: element (r, k) at X[r * ld + k]  -- thread t: rows t/4 and t/4 + 64, k chunk 4*(t%4)
//    trans: element (r, k) at X[k * ld + r]  -- thread t: k rows t/32 and t/32 + 8, r chunk 4*(t%32)
struct Regs { float v[8]; };

__device__ __forceinline__ void load_stage(const float* __restrict__ X, int64_t ld, int trans, int rows, int K, int r0,
                                           int k0, Regs& R) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (!trans) {
      const int r = r0 + t / 4 + 64 * i, k = k0 + 4 * (t % 4);
      if (r < rows && k + 3 < K) {
        const f32x4 w = *(const f32x4*)(X + (int64_t)r * ld + k);
        R.v[4 * i] = w[0]; R.v[4 * i + 1] = w[1]; R.v[4 * i + 2] = w[2]; R.v[4 * i + 3] = w[3];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) R.v[4 * i + j] = (r < rows && k + j < K) ? X[(int64_t)r * ld + k + j] : 0.f;
      }
    } else {
      const int k = k0 + t / 32 + 8 * i, r = r0 + 4 * (t % 32);
      if (k < K && r + 3 < rows) {
        const f32x4 w = *(const f32x4*)(X + (int64_t)k * ld + r);
        R.v[4 * i] = w[0]; R.v[4 * i + 1] = w[1]; R.v[4 * i + 2] = w[2]; R.v[4 * i + 3] = w[3];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) R.v[4 * i + j] = (k < K && r + j < rows) ? X[(int64_t)k * ld + r + j] : 0.f;
      }
    }
  }
}

__device__ __forceinline__ void store_stage(float (*s)[LDP], int trans, const Regs& R) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if (!trans) {
      const int r = t / 4 + 64 * i, k = 4 * (t % 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) s[k + j][r] = R.v[4 * i + j];
    } else {
      const int k = t / 32 + 8 * i, r = 4 * (t % 32);
      *(f32x4*)&s[k][r] = f32x4{R.v[4 * i], R.v[4 * i + 1], R.v[4 * i + 2], R.v[4 * i + 3]};
    }
  }
}

__global__ __launch_bounds__(NT) void gemm_f32_kernel(G32P p) {
  __shared__ float sA[2][BK][LDP];
  __shared__ float sB[2][BK][LDP];
  const int tile = blockIdx.x;
  const int mt = tile / p.tiles_n, nt = tile % p.tiles_n;
  const int bz = blockIdx.y;
  const int bo = bz / p.batch_in, bi = bz % p.batch_in;
  const float* A = p.A + bo * p.sA + bi * p.sAi;
  const float* B = p.B + bo * p.sB + bi * p.sBi;
  float* C = p.C + bo * p.sC + bi * p.sCi;
  const int m0 = mt * BM, n0 = nt * BN;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 15, kr = lane >> 4;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  Regs ra, rb;
  load_stage(A, p.lda, p.at, p.M, p.K, m0, 0, ra);
  load_stage(B, p.ldb, p.bt, p.N, p.K, n0, 0, rb);
  store_stage(sA[0], p.at, ra);
  store_stage(sB[0], p.bt, rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      load_stage(A, p.lda, p.at, p.M, p.K, m0, (kt + 1) * BK, ra);
      load_stage(B, p.ldb, p.bt, p.N, p.K, n0, (kt + 1) * BK, rb);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int k = 4 * kk + kr;
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = sA[cur][k][wm * 64 + i * 16 + li];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = sB[cur][k][wn * 64 + j * 16 + li];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      store_stage(sA[cur ^ 1], p.at, ra);
      store_stage(sB[cur ^ 1], p.bt, rb);
    }
    __syncthreads();
  }

  // epilogue: lane holds C[m = .. + 4*kr + r][n = .. + li] of each 16x16 block
  const int flags = p.flags;
  const float* res = p.res ? p.res + bo * p.sR : nullptr;
  float* aux = p.aux ? p.aux + bo * p.sAux : nullptr;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + li;
    if (n >= p.N) continue;
    const float bv = (flags & F_BIAS) ? p.bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + 4 * kr + r;
        if (m >= p.M) continue;
        float v = acc[i][j][r] * p.alpha + bv;
        if (flags & F_DGELU) v *= gelu_exact_grad(aux[(int64_t)m * p.ldaux + n]);
        if (flags & F_GELU) {
          if (flags & F_AUX_OUT) aux[(int64_t)m * p.ldaux + n] = v;
          v = gelu_exact(v);
        }
        if (flags & F_RES) {
          const int mr = p.res_mod > 0 ? m % p.res_mod : m;
          v += res[(int64_t)mr * p.ldr + n];
        }
        float* c = C + (int64_t)m * p.ldc + n;
        if (flags & F_ACCUM) v += *c;
        *c = v;
      }
    }
  }
}

int launch_gemm(const G32P& q, int batch, hipStream_t stream) {
  G32P p = q;
  p.tiles_n = (p.N + BN - 1) / BN;
  const int64_t tiles = (int64_t)((p.M + BM - 1) / BM) * p.tiles_n;
  if (tiles > 0x7fffffff || batch > 65535) return TW_EINVAL;
  hipLaunchKernelGGL(gemm_f32_kernel, dim3((unsigned)tiles, batch), dim3(NT), 0, stream, p);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// ------------------------------------------------------------------------------- attention rows
// S rows of one chunk: row r -> (bl, hl, q) = (r / (nh*Tq), (r / Tq) % nh, r % Tq); ld = row pitch.
// softmax in place (exact: global max, expf, fp32 sum), causal: key j > q + (Tk - Tq) masked;
// pad columns [Tk, ld) zeroed (they are K-range operands of the P.V GEMM only up to Tk, but keep
// them finite); lse[(b*H + h)*Tq + q] = max + log(sum).
__global__ __launch_bounds__(256) void softmax_rows_kernel(float* __restrict__ S, int64_t ld, int64_t rows, int Tq,
                                                           int Tk, int nh, int H, int b0, int h0, int causal,
                                                           float* __restrict__ lse) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const int q = r % Tq;
  const int hl = (r / Tq) % nh, bl = r / ((int64_t)Tq * nh);
  const int lim = causal ? min(Tk, q + (Tk - Tq) + 1) : Tk;
  float* row = S + r * ld;
  float m = -INFINITY;
  for (int j = lane; j < lim; j += 64) m = fmaxf(m, row[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < lim; j += 64) s += expf(row[j] - m);
  s = wave_sum(s);
  const float inv = 1.0f / s;
  for (int j = lane; j < ld; j += 64) row[j] = j < lim ? expf(row[j] - m) * inv : 0.f;
  if (lane == 0 && lse) lse[((int64_t)(b0 + bl) * H + h0 + hl) * Tq + q] = m + logf(s);
}

// backward rows: P = exp(S - lse) (in place in S), dS = scale * P * (dP - sum_j dO[j] O[j]) (in place in dP)
__global__ __launch_bounds__(256) void dsoftmax_rows_kernel(float* __restrict__ S, float* __restrict__ dP, int64_t ld,
                                                            int64_t rows, int Tq, int Tk, int nh, int H, int b0, int h0,
                                                            int causal, const float* __restrict__ lse,
                                                            const float* __restrict__ O, int64_t ldo,
                                                            const float* __restrict__ dO, int64_t lddo, float scale) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  const int q = r % Tq;
  const int hl = (r / Tq) % nh, bl = r / ((int64_t)Tq * nh);
  const int b = b0 + bl, h = h0 + hl;
  const int lim = causal ? min(Tk, q + (Tk - Tq) + 1) : Tk;
  const int64_t orow = (int64_t)b * Tq + q;
  const float D = wave_sum(O[orow * ldo + h * 64 + lane] * dO[orow * lddo + h * 64 + lane]);
  const float l = lse[((int64_t)b * H + h) * Tq + q];
  float* srow = S + r * ld;
  float* drow = dP + r * ld;
  for (int j = lane; j < ld; j += 64) {
    const float pj = j < lim ? expf(srow[j] - l) : 0.f;
    srow[j] = pj;
    drow[j] = j < lim ? scale * pj * (drow[j] - D) : 0.f;
  }
}

int64_t ws_pitch(int Tk) { return ((int64_t)Tk + 3) / 4 * 4; }

// ------------------------------------------------------------------------------- conv helpers
__global__ void mel_to_conv_input_f32_kernel(const float* __restrict__ mel, float* __restrict__ xt, int B, int nmel,
                                             int T) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)B * (T + 2) * nmel;
  if (i >= n) return;
  const int c = i % nmel;
  const int64_t r = i / nmel;
  const int b = r / (T + 2), tt = r % (T + 2);
  xt[i] = (tt >= 1 && tt <= T) ? mel[((int64_t)b * nmel + c) * T + (tt - 1)] : 0.f;
}

__global__ void im2col_f32_kernel(const float* __restrict__ src, int64_t src_rows, float* __restrict__ dst, int B,
                                  int T_out, int stride, int C) {
  const int64_t row = blockIdx.x;
  if (row >= (int64_t)B * T_out) return;
  const int b = row / T_out, t = row % T_out;
  for (int j = threadIdx.x; j < 3 * C; j += blockDim.x) {
    const int k = j / C, c = j % C;
    dst[row * 3 * C + j] = src[((int64_t)b * src_rows + (int64_t)t * stride + k) * C + c];
  }
}

__global__ void gelu_bwd_f32_kernel(const float* __restrict__ g, const float* __restrict__ pre, float* __restrict__ out,
                                    int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = g[i] * gelu_exact_grad(pre[i]);
}

inline int nblk(int64_t n, int bs, int cap = 8192) {
  int64_t b = (n + bs - 1) / bs;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

bool al16(const void* x) { return ((uintptr_t)x & 15) == 0; }

}  // namespace

extern "C" int tw_gemm_f32(const float* A, int64_t lda, int a_trans, const float* B, int64_t ldb, int b_trans, float* C,
                           int64_t ldc, int M, int N, int K, int batch, int64_t sA, int64_t sB, int64_t sC,
                           int batch_inner, int64_t sA_in, int64_t sB_in, int64_t sC_in, float alpha, const float* bias,
                           const float* res, int64_t ldr, int64_t sR, int res_mod, float* aux, int64_t ldaux,
                           int64_t sAux, int flags, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return TW_OK;
  if (K <= 0 || batch_inner <= 0 || (batch % batch_inner) != 0) return TW_EINVAL;
  if ((lda & 3) || (ldb & 3) || !al16(A) || !al16(B)) return TW_EINVAL;     // 16-B vector loads
  if ((flags & F_BIAS) && !bias) return TW_EINVAL;
  if ((flags & F_RES) && !res) return TW_EINVAL;
  if ((flags & (F_AUX_OUT | F_DGELU)) && !aux) return TW_EINVAL;
  G32P p;
  p.A = A; p.lda = lda; p.at = a_trans; p.B = B; p.ldb = ldb; p.bt = b_trans; p.C = C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.batch_in = batch_inner;
  p.sA = sA; p.sB = sB; p.sC = sC; p.sAi = sA_in; p.sBi = sB_in; p.sCi = sC_in;
  p.alpha = alpha; p.bias = bias; p.res = res; p.ldr = ldr; p.sR = sR; p.res_mod = res_mod;
  p.aux = aux; p.ldaux = ldaux; p.sAux = sAux; p.flags = flags & (F_BIAS | F_GELU | F_RES | F_ACCUM | F_AUX_OUT | F_DGELU);
  return launch_gemm(p, batch, stream);
}

namespace {
G32P plain(const float* A, int64_t lda, int at, const float* B, int64_t ldb, int bt, float* C, int64_t ldc, int M,
           int N, int K, float alpha) {
  G32P p{};
  p.A = A; p.lda = lda; p.at = at; p.B = B; p.ldb = ldb; p.bt = bt; p.C = C; p.ldc = ldc;
  p.M = M; p.N = N; p.K = K; p.alpha = alpha; p.batch_in = 1; p.flags = 0;
  return p;
}

// chunking of (b, h) pairs over a workspace holding `per` floats per (b, h) per buffer
bool chunks(int64_t ws_floats, int64_t per, int B, int H, int& cb, int& ch) {
  const int64_t fit = ws_floats / per;
  if (fit < 1) return false;
  if (fit >= H) { ch = H; cb = (int)std::min<int64_t>(fit / H, (int64_t)B); }
  else { ch = (int)fit; cb = 1; }
  cb = std::min(cb, 65535 / std::max(ch, 1));
  return cb >= 1;
}
}  // namespace

extern "C" int tw_attn_fwd_f32(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv,
                               float* O, int64_t ldo, float* lse, int B, int H, int Tq, int Tk, int head_dim,
                               int causal, float scale, float* ws, int64_t ws_floats, hipStream_t stream) {
  if (head_dim != 64) return TW_EUNSUPPORTED;
  if (B <= 0 || H <= 0 || Tq <= 0) return TW_OK;
  if (Tk <= 0 || (causal && Tk < Tq) || !ws) return TW_EINVAL;
  if ((ldq | ldk | ldv) & 3) return TW_EINVAL;
  const int64_t ldS = ws_pitch(Tk);
  const int64_t per = (int64_t)Tq * ldS;
  int cb, ch;
  if (!chunks(ws_floats, per, B, H, cb, ch)) return TW_EINVAL;
  for (int b0 = 0; b0 < B; b0 += cb) {
    const int nb = std::min(cb, B - b0);
    for (int h0 = 0; h0 < H; h0 += ch) {
      const int nh = std::min(ch, H - h0);
      // S = scale * Q K^T   (outer: b, inner: h)
      G32P s = plain(Q + (int64_t)b0 * Tq * ldq + h0 * 64, ldq, 0, K + (int64_t)b0 * Tk * ldk + h0 * 64, ldk, 0, ws,
                     ldS, Tq, Tk, 64, scale);
      s.batch_in = nh; s.sA = (int64_t)Tq * ldq; s.sAi = 64; s.sB = (int64_t)Tk * ldk; s.sBi = 64;
      s.sC = nh * per; s.sCi = per;
      int rc = launch_gemm(s, nb * nh, stream);
      if (rc) return rc;
      const int64_t rows = (int64_t)nb * nh * Tq;
      hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, ws, ldS, rows, Tq,
                         Tk, nh, H, b0, h0, causal, lse);
      // O = P V   (V stored [Tk][64]: the [K][N] operand)
      G32P o = plain(ws, ldS, 0, V + (int64_t)b0 * Tk * ldv + h0 * 64, ldv, 1, O + (int64_t)b0 * Tq * ldo + h0 * 64, ldo,
                     Tq, 64, Tk, 1.0f);
      o.batch_in = nh; o.sA = nh * per; o.sAi = per; o.sB = (int64_t)Tk * ldv; o.sBi = 64;
      o.sC = (int64_t)Tq * ldo; o.sCi = 64;
      rc = launch_gemm(o, nb * nh, stream);
      if (rc) return rc;
    }
  }
  TW_CHECK_LAUNCH();
  return TW_OK;
}

// workspace >= 2 * Tq * round_up(Tk, 4) floats (more: several (b, h) pairs per pass)
extern "C" int tw_attn_bwd_f32(const float* Q, int64_t ldq, const float* K, int64_t ldk, const float* V, int64_t ldv,
                               const float* O, int64_t ldo, const float* dO, int64_t lddo, const float* lse, float* dQ,
                               int64_t lddq, float* dK, int64_t lddk, float* dV, int64_t lddv, int B, int H, int Tq,
                               int Tk, int head_dim, int causal, float scale, float* ws, int64_t ws_floats,
                               hipStream_t stream) {
  if (head_dim != 64) return TW_EUNSUPPORTED;
  if (B <= 0 || H <= 0 || Tq <= 0) return TW_OK;
  if (Tk <= 0 || (causal && Tk < Tq) || !ws || !lse) return TW_EINVAL;
  if ((ldq | ldk | ldv | lddo) & 3) return TW_EINVAL;
  const int64_t ldS = ws_pitch(Tk);
  const int64_t per = (int64_t)Tq * ldS;
  int cb, ch;
  if (!chunks(ws_floats / 2, per, B, H, cb, ch)) return TW_EINVAL;
  for (int b0 = 0; b0 < B; b0 += cb) {
    const int nb = std::min(cb, B - b0);
    for (int h0 = 0; h0 < H; h0 += ch) {
      const int nh = std::min(ch, H - h0);
      float* S = ws;
      float* dP = ws + (int64_t)nb * nh * per;
      const float* Qc = Q + (int64_t)b0 * Tq * ldq + h0 * 64;
      const float* Kc = K + (int64_t)b0 * Tk * ldk + h0 * 64;
      const float* Vc = V + (int64_t)b0 * Tk * ldv + h0 * 64;
      const float* dOc = dO + (int64_t)b0 * Tq * lddo + h0 * 64;
      // S = scale Q K^T ; dP = dO V^T
      G32P s = plain(Qc, ldq, 0, Kc, ldk, 0, S, ldS, Tq, Tk, 64, scale);
      s.batch_in = nh; s.sA = (int64_t)Tq * ldq; s.sAi = 64; s.sB = (int64_t)Tk * ldk; s.sBi = 64;
      s.sC = nh * per; s.sCi = per;
      int rc = launch_gemm(s, nb * nh, stream);
      if (rc) return rc;
      G32P d = plain(dOc, lddo, 0, Vc, ldv, 0, dP, ldS, Tq, Tk, 64, 1.0f);
      d.batch_in = nh; d.sA = (int64_t)Tq * lddo; d.sAi = 64; d.sB = (int64_t)Tk * ldv; d.sBi = 64;
      d.sC = nh * per; d.sCi = per;
      rc = launch_gemm(d, nb * nh, stream);
      if (rc) return rc;
      const int64_t rows = (int64_t)nb * nh * Tq;
      hipLaunchKernelGGL(dsoftmax_rows_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, S, dP, ldS, rows,
                         Tq, Tk, nh, H, b0, h0, causal, lse, O, ldo, dO, lddo, scale);
      // dV = P^T dO   (P^T: A stored [K = Tq][M = Tk]; dO: B stored [K = Tq][N = 64])
      G32P v = plain(S, ldS, 1, dOc, lddo, 1, dV + (int64_t)b0 * Tk * lddv + h0 * 64, lddv, Tk, 64, Tq, 1.0f);
      v.batch_in = nh; v.sA = nh * per; v.sAi = per; v.sB = (int64_t)Tq * lddo; v.sBi = 64;
      v.sC = (int64_t)Tk * lddv; v.sCi = 64;
      rc = launch_gemm(v, nb * nh, stream);
      if (rc) return rc;
      // dQ = dS K   (K stored [K = Tk][N = 64])
      G32P q = plain(dP, ldS, 0, Kc, ldk, 1, dQ + (int64_t)b0 * Tq * lddq + h0 * 64, lddq, Tq, 64, Tk, 1.0f);
      q.batch_in = nh; q.sA = nh * per; q.sAi = per; q.sB = (int64_t)Tk * ldk; q.sBi = 64;
      q.sC = (int64_t)Tq * lddq; q.sCi = 64;
      rc = launch_gemm(q, nb * nh, stream);
      if (rc) return rc;
      // dK = dS^T Q
      G32P k = plain(dP, ldS, 1, Qc, ldq, 1, dK + (int64_t)b0 * Tk * lddk + h0 * 64, lddk, Tk, 64, Tq, 1.0f);
      k.batch_in = nh; k.sA = nh * per; k.sAi = per; k.sB = (int64_t)Tq * ldq; k.sBi = 64;
      k.sC = (int64_t)Tk * lddk; k.sCi = 64;
      rc = launch_gemm(k, nb * nh, stream);
      if (rc) return rc;
    }
  }
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_mel_to_conv_input_f32(const float* mel, float* xt, int B, int nmel, int T, hipStream_t stream) {
  const int64_t n = (int64_t)B * (T + 2) * nmel;
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(mel_to_conv_input_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, mel, xt, B,
                     nmel, T);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_im2col3_f32(const float* src, int64_t src_rows, float* dst, int B, int T_out, int stride, int C,
                              hipStream_t stream) {
  if (B <= 0 || T_out <= 0) return TW_OK;
  hipLaunchKernelGGL(im2col_f32_kernel, dim3((unsigned)((int64_t)B * T_out)), dim3(256), 0, stream, src, src_rows, dst,
                     B, T_out, stride, C);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_gelu_bwd_f32(const float* g, const float* pre, float* out, int64_t n, hipStream_t stream) {
  if (n <= 0) return TW_OK;
  hipLaunchKernelGGL(gelu_bwd_f32_kernel, dim3(nblk(n, 256)), dim3(256), 0, stream, g, pre, out, n);
  TW_CHECK_LAUNCH();
  return TW_OK;
}
