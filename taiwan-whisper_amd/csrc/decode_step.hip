// Persistent decoder-step kernel (the long-form / small-batch decode of
// run_eval.py:659-685 through HF generation_whisper.py's per-token loop): every decoder layer of one greedy
// step -- LN + fused QKV + KV append, self-attention over the cache, out_proj + residual, LN + cross-q,
// cross-attention over the encoder K/V (split over keys + combine), out_proj + residual, LN + fc1 + GELU,
// fc2 + residual -- in ONE launch of one workgroup per CU, the stages separated by grid-wide barriers.
//
// Why: at batch <= 8 a decode step is ~10 dependent launches per layer (~330 for large-v2), each a few
// microseconds of work behind a launch + drain + fill (DESIGN.md §5 Decode); here a stage boundary is a
// counter arrival + poll + one cache invalidate instead.
//
// Arithmetic: the stages call the same device bodies as the per-launch kernels (gemv_impl.h: LN staging,
// per-lane k-ordered fp32 dots, epilogue; decode_impl.h: two-pass attention body, chunk combine), so the
// outputs are bit-identical to the per-launch path (tests/test_decode_step_gpu.py).
//
// Hand-off protocol (cdna_hip_programming.md Guideline 16, fan-in form R1): every value a later stage reads
// is stored write-through (WT: global_store_* sc1, no L2 write-back needed), every storing wave drains
// (s_waitcnt vmcnt(0)) before the workgroup barrier, one lane adds 1 to the arrival counter (agent-scope
// relaxed atomic) and polls it (relaxed, s_sleep between polls) until all G workgroups of this phase have
// arrived, then ONE agent-scope acquire (buffer_inv sc1: this CU's stale L1/L2 lines dropped) before the
// workgroup barrier that releases the other waves' loads.  Residual operands (read by lane 0 of a wave at a
// wave-uniform address) go through an agent-scope atomic load, never the scalar cache.  Every spin is bounded:
// on a timeout the kernel records an error word and every workgroup leaves at its next barrier, so a lost
// workgroup cannot hang the device (the host raises on the error word).  Co-residency: grid = CU count with
// one 256-thread workgroup per CU admitted by the occupancy API (checked on the host).
#include "decode_impl.h"
#include "gemv_impl.h"

#include <type_traits>

namespace {

using namespace twg;
using namespace twd;

// one decoder layer's operands (device-resident table, tw_decoder_layers' `layers`): 21 pointers
struct DsLayer {
  const float* ln1w; const float* ln1b;
  const bf16* wqkv; const bf16* bqkv;            // fused [3d][d] / [3d]
  const bf16* wo; const bf16* bo;
  const float* ln2w; const float* ln2b;
  const bf16* wq; const bf16* bq;
  const bf16* xk; const bf16* xv;                // cross K, V head-major [B*H][Tk][64]
  const bf16* wco; const bf16* bco;
  const float* ln3w; const float* ln3b;
  const bf16* w1; const bf16* b1;
  const bf16* w2; const bf16* b2;
  bf16* self_kv;                                 // [B][T_max][2d] (k | v)
};

struct DsP {
  const DsLayer* layers; int L;
  bf16* x; bf16* qkv; bf16* o; bf16* q; bf16* h;  // residual stream [B][d] (16-bit) and stage outputs
  float* part;                                   // cross-attention chunk partials [B*H][nchunk][66]
  int B, d, H, ffn, T_max, Tk, nchunk;
  const int* t_dev;                              // step index (cache row, self-attention length - 1)
  float eps, c;                                  // LN eps; scale * log2(e)
  unsigned* ctr;                                 // arrival counter (zeroed before every launch)
  unsigned* err;                                 // sticky error word (spin timeout)
  int kmax;                                      // max(d, ffn): the LDS row length
};

constexpr unsigned DS_SPIN_LIMIT = 1u << 23;     // polls (s_sleep 2 each, ~0.1 us) before giving up (~1 s)

// Grid barrier number `phase` (1, 2, ...): true when every workgroup arrived, false after a timeout / error.
__device__ __forceinline__ bool ds_barrier(const DsP& p, unsigned phase, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this wave's write-through stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    __hip_atomic_fetch_add(p.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = phase * gridDim.x;
    unsigned n = 0;
    while (__hip_atomic_load(p.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if ((++n & 255u) == 0) {
        if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) { ok = 0; break; }
        if (n >= DS_SPIN_LIMIT) {
          __hip_atomic_store(p.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    *flag = ok;
  }
  __syncthreads();
  return *flag != 0;
}

// One Linear stage: rows of A (LayerNorm'd when lnw) against W, CPW columns per wave over the whole grid.
template <bool H, int MR, int CPW, int PRE>
__device__ __forceinline__ void ds_linear(const GemmP& g, const float* lnw, const float* lnb, float eps,
                                          const GemvKV& kv, bf16* xs, int wave, int lane) {
  const int ngroups = (g.N + CPW - 1) / CPW;
  const int nvw = gridDim.x * 4;
  int grp = blockIdx.x * 4 + wave;
  if ((int)blockIdx.x * 4 >= ngroups) return;          // no columns for this workgroup (uniform)
  bf16x8 wpre[CPW][PRE];
  if (grp < ngroups) gemv_preload<H, CPW, PRE>(g, grp * CPW, lane, wpre);
  gemv_stage_rows<H, MR>(g, lnw, lnb, eps, xs, wave, 4, lane);
  __syncthreads();
  while (grp < ngroups) {
    gemv_finish<H, MR, CPW, PRE, true>(g, kv, xs, grp * CPW, lane, wpre);
    grp += nvw;
    if (grp < ngroups) gemv_preload<H, CPW, PRE>(g, grp * CPW, lane, wpre);
  }
  __syncthreads();                                      // xs is restaged by the next Linear of this workgroup
}

__device__ __forceinline__ GemmP ds_gemm(const bf16* A, int64_t lda, const bf16* W, void* C, int64_t ldc, int M, int N,
                                         int K, const bf16* bias, const void* res, int flags) {
  GemmP g = {};
  g.A = A; g.B = W; g.C = C;
  g.lda = lda; g.ldb = K; g.ldc = ldc; g.M = M; g.N = N; g.K = K;
  g.alpha = 1.f; g.bias = bias; g.res = res; g.ldr = ldc; g.res_dtype = TW_BF16; g.res_mod = 0;
  g.c_dtype = TW_BF16; g.flags = flags | F_BIAS | F_ROUND | (res ? F_RES : 0);
  return g;
}

template <bool H, int MR>
__global__ __launch_bounds__(256, 1) void decoder_layers_kernel(DsP p) {
  extern __shared__ __attribute__((aligned(16))) char ds_smem[];
  bf16* xs = (bf16*)ds_smem;                           // [MR][kmax] staged A rows
  int* flag = (int*)(ds_smem + (size_t)MR * p.kmax * 2);
  using E = std::conditional_t<H, f16, bf16>;
  const int lane = lane_id(), wave = wave_id_uniform();
  const int G = gridDim.x, wg = blockIdx.x;
  const int B = p.B, d = p.d, H3 = p.H;
  const int BH = B * H3;
  unsigned phase = 0;
  const int t = *p.t_dev;
  int tk_self = 1 + t;
  if (tk_self > DA_MAX_TK) tk_self = DA_MAX_TK;
  const GemvKV nokv{nullptr, 0, 0, 0, nullptr};
  for (int l = 0; l < p.L; ++l) {
    const DsLayer& w = p.layers[l];
    const int64_t sb = (int64_t)p.T_max * 2 * d;
    // 1. LN1 + fused QKV; k, v of this step to cache row t
    {
      const GemmP g = ds_gemm(p.x, d, w.wqkv, p.qkv, 3 * d, B, 3 * d, d, w.bqkv, nullptr, 0);
      const GemvKV kv{w.self_kv, sb, 2 * d, d, p.t_dev};
      ds_linear<H, MR, 4, 3>(g, w.ln1w, w.ln1b, p.eps, kv, xs, wave, lane);
    }
    if (!ds_barrier(p, ++phase, flag)) return;
    // 2. self-attention over cache rows 0..t, one (clip, head) per workgroup
    {
      DecP a;
      a.q = p.qkv; a.sqb = 3 * d;
      a.k = w.self_kv; a.ldk = 2 * d; a.skb = sb;
      a.v = w.self_kv + d; a.ldv = 2 * d; a.svb = sb;
      a.o = p.o; a.sob = d; a.H = H3; a.Tk = 1; a.tk_dev = p.t_dev; a.c = p.c;
      for (int it = wg; it < BH; it += G) {
        decode_attn_body<E, true>(a, it / H3, it % H3, 0, tk_self, nullptr);
        __syncthreads();                                // the body's LDS is reused by the next item
      }
    }
    if (!ds_barrier(p, ++phase, flag)) return;
    // 3. self out_proj + residual (in place on x)
    ds_linear<H, MR, 2, 3>(ds_gemm(p.o, d, w.wo, p.x, d, B, d, d, w.bo, p.x, 0), nullptr, nullptr, p.eps, nokv, xs,
                           wave, lane);
    if (!ds_barrier(p, ++phase, flag)) return;
    // 4. LN2 + cross-attention q
    ds_linear<H, MR, 2, 3>(ds_gemm(p.x, d, w.wq, p.q, d, B, d, d, w.bq, nullptr, 0), w.ln2w, w.ln2b, p.eps, nokv, xs,
                           wave, lane);
    if (!ds_barrier(p, ++phase, flag)) return;
    // 5. cross-attention over the encoder K/V (head-major: (clip, head) = one row of H = 1), split into chunks
    //    of DA_SPLIT keys as tw_decode_attn splits below 640 pairs
    DecP xa;
    xa.q = p.q; xa.sqb = 64;
    xa.k = w.xk; xa.ldk = 64; xa.skb = (int64_t)p.Tk * 64;
    xa.v = w.xv; xa.ldv = 64; xa.svb = (int64_t)p.Tk * 64;
    xa.o = p.o; xa.sob = 64; xa.H = 1; xa.Tk = p.Tk; xa.tk_dev = nullptr; xa.c = p.c;
    for (int it = wg; it < BH * p.nchunk; it += G) {
      const int bh = it / p.nchunk, ch = it % p.nchunk;
      const int lo = ch * DA_SPLIT, hi = min(p.Tk, lo + DA_SPLIT);
      float* part = p.part + ((int64_t)bh * p.nchunk + ch) * 66;
      if (lo >= hi) {
        if (threadIdx.x < 64) st_wt<true>(part + threadIdx.x, 0.f);
        if (threadIdx.x == 0) {
          st_wt<true>(part + 64, -INFINITY);
          st_wt<true>(part + 65, 0.f);
        }
      } else {
        decode_attn_body<E, true>(xa, bh, 0, lo, hi, part);
      }
      __syncthreads();
    }
    if (!ds_barrier(p, ++phase, flag)) return;
    // 6. chunk combine, one (clip, head) per wave
    for (int it = wg * 4 + wave; it < BH; it += G * 4)
      combine_row<E, true>(xa, it, p.nchunk, p.part + (int64_t)it * p.nchunk * 66);
    if (!ds_barrier(p, ++phase, flag)) return;
    // 7. cross out_proj + residual
    ds_linear<H, MR, 2, 3>(ds_gemm(p.o, d, w.wco, p.x, d, B, d, d, w.bco, p.x, 0), nullptr, nullptr, p.eps, nokv, xs,
                           wave, lane);
    if (!ds_barrier(p, ++phase, flag)) return;
    // 8. LN3 + fc1 + GELU
    ds_linear<H, MR, 8, 3>(ds_gemm(p.x, d, w.w1, p.h, p.ffn, B, p.ffn, d, w.b1, nullptr, F_GELU), w.ln3w, w.ln3b,
                           p.eps, nokv, xs, wave, lane);
    if (!ds_barrier(p, ++phase, flag)) return;
    // 9. fc2 + residual
    ds_linear<H, MR, 2, 10>(ds_gemm(p.h, p.ffn, w.w2, p.x, d, B, d, p.ffn, w.b2, p.x, 0), nullptr, nullptr, p.eps,
                            nokv, xs, wave, lane);
    if (l + 1 < p.L && !ds_barrier(p, ++phase, flag)) return;
  }
}

int ds_grid(int dev) {
  static int cus[64] = {0};
  if (dev < 0 || dev >= 64) return 0;
  if (!cus[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    cus[dev] = n;
  }
  return cus[dev];
}

template <bool H, int MR>
int ds_launch(const DsP& p, hipStream_t stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return TW_EHIP;
  const int G = ds_grid(dev);
  if (G <= 0) return TW_EHIP;
  const size_t lds = (size_t)MR * p.kmax * 2 + 16;
  // every workgroup must be resident at once (grid barriers): one per CU, admitted by the occupancy API
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decoder_layers_kernel<H, MR>, 256, lds) != hipSuccess ||
      per_cu < 1)
    return TW_EUNSUPPORTED;
  if (hipMemsetAsync(p.ctr, 0, 16, stream) != hipSuccess) return TW_EHIP;
  hipLaunchKernelGGL((decoder_layers_kernel<H, MR>), dim3(G), dim3(256), lds, stream, p);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

}  // namespace

// include/tw_hip.h
extern "C" int tw_decoder_layers(const void* layers, int L, void* x, void* qkv, void* o, void* q, void* h, float* part,
                                 int B, int d, int H, int ffn, int T_max, int Tk, const int* t_dev, float eps,
                                 float scale, unsigned* sync, int dtype, hipStream_t stream) {
  if (L <= 0) return TW_OK;
  if (dtype != TW_BF16 && dtype != TW_F16) return TW_EUNSUPPORTED;
  if (B < 1 || B > 8 || H * 64 != d || d % 256 || ffn % 256) return TW_EUNSUPPORTED;
  if (T_max < 1 || T_max > DA_MAX_TK || Tk < 1 || Tk > DA_MAX_TK) return TW_EUNSUPPORTED;
  if (!layers || !x || !qkv || !o || !q || !h || !part || !t_dev || !sync) return TW_EINVAL;
  if (((uintptr_t)layers | (uintptr_t)x | (uintptr_t)qkv | (uintptr_t)o | (uintptr_t)q | (uintptr_t)h |
       (uintptr_t)part | (uintptr_t)sync) & 15)
    return TW_EINVAL;
  const int nchunk = (Tk + DA_SPLIT - 1) / DA_SPLIT;
  if (nchunk > DA_MAX_CHUNK) return TW_EUNSUPPORTED;
  DsP p;
  p.layers = (const DsLayer*)layers; p.L = L;
  p.x = (bf16*)x; p.qkv = (bf16*)qkv; p.o = (bf16*)o; p.q = (bf16*)q; p.h = (bf16*)h; p.part = part;
  p.B = B; p.d = d; p.H = H; p.ffn = ffn; p.T_max = T_max; p.Tk = Tk; p.nchunk = nchunk;
  p.t_dev = t_dev; p.eps = eps; p.c = scale * 1.4426950408889634f;
  p.ctr = sync; p.err = sync + 4;
  p.kmax = d > ffn ? d : ffn;
  const int mr = B == 1 ? 1 : B == 2 ? 2 : B <= 4 ? 4 : 8;
#define TW_DS(H_, MR_) return ds_launch<H_, MR_>(p, stream)
  if (dtype == TW_F16) {
    if (mr == 1) TW_DS(true, 1);
    if (mr == 2) TW_DS(true, 2);
    if (mr == 4) TW_DS(true, 4);
    TW_DS(true, 8);
  }
  if (mr == 1) TW_DS(false, 1);
  if (mr == 2) TW_DS(false, 2);
  if (mr == 4) TW_DS(false, 4);
  TW_DS(false, 8);
#undef TW_DS
}
