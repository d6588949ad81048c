// Fused distillation loss head: for every decoder position with
// label >= 0, from the student / teacher logit rows (bf16 under autocast, fp32 on the fp32 path) (the reference's fp32 logits are
// exactly these bf16 values upcast, ACC:accelerator.py:1818-1829):
//   ce_row = logsumexp(s) - s[label]                                (HF:modeling_whisper.py:1082-1087)
//   kl_row = sum_v p_v (log p_v - log q_v),  p = softmax(t/T), log q = log_softmax(s/T)
//                                                              (run_distillation.py:1507-1516,1542-1546)
// and, when requested, the gradient of loss = ce_w * mean(ce) + kl_w * T^2 * sum(kl)/N:
//   dlogits_v = gs/N * [ ce_w (softmax(s)_v - 1[v=label]) + kl_w * T (q_v - p_v) ]  (bf16)
// One workgroup per row; pass 1 keeps online (max, sum) statistics for softmax(s),
// softmax(s/T), softmax(t/T) and sum_v e_v (t_v - s_v); pass 2 writes the gradient row.
// None of the seven [B,447,V] fp32 tensors of the reference is materialised.
#include "common.h"

namespace {

constexpr int NT = 256;

struct Stats {
  float ms, z1, zt;      // student: max, sum exp(s-ms), sum exp((s-ms)/T)
  float mt, ztt, a;      // teacher: max, sum exp((t-mt)/T), sum exp((t-mt)/T)*(t-s)
};

__device__ __forceinline__ void merge(Stats& x, const Stats& y, float invT) {
  const float ms = fmaxf(x.ms, y.ms);
  if (ms != -INFINITY) {
    const float zx1 = x.ms == -INFINITY ? 0.f : x.z1 * __expf(x.ms - ms);
    const float zy1 = y.ms == -INFINITY ? 0.f : y.z1 * __expf(y.ms - ms);
    const float zxt = x.ms == -INFINITY ? 0.f : x.zt * __expf((x.ms - ms) * invT);
    const float zyt = y.ms == -INFINITY ? 0.f : y.zt * __expf((y.ms - ms) * invT);
    x.z1 = zx1 + zy1; x.zt = zxt + zyt; x.ms = ms;
  }
  const float mt = fmaxf(x.mt, y.mt);
  if (mt != -INFINITY) {
    const float ex = x.mt == -INFINITY ? 0.f : __expf((x.mt - mt) * invT);
    const float ey = y.mt == -INFINITY ? 0.f : __expf((y.mt - mt) * invT);
    x.ztt = x.ztt * ex + y.ztt * ey;
    x.a = x.a * ex + y.a * ey;
    x.mt = mt;
  }
}

__device__ __forceinline__ Stats shfl_stats(const Stats& s, int o) {
  Stats r;
  r.ms = __shfl_xor(s.ms, o, 64); r.z1 = __shfl_xor(s.z1, o, 64); r.zt = __shfl_xor(s.zt, o, 64);
  r.mt = __shfl_xor(s.mt, o, 64); r.ztt = __shfl_xor(s.ztt, o, 64); r.a = __shfl_xor(s.a, o, 64);
  return r;
}

template <typename E>
__global__ __launch_bounds__(NT) void klce_kernel(const E* __restrict__ S, const E* __restrict__ Tl, int64_t ld,
                                                  const int64_t* __restrict__ labels, int V, float T, float ce_w,
                                                  float kl_w, const int* __restrict__ n_valid, float grad_scale,
                                                  float* __restrict__ row_out, E* __restrict__ dS) {
  __shared__ Stats red[NT / 64];
  const int64_t row = blockIdx.x;
  const int64_t lab = labels[row];
  const int tid = threadIdx.x;
  const int nch = (V + 7) / 8;          // 8-wide chunks covering [0, V)
  const int nch_ld = (int)(ld / 8);     // chunks covering the padded row
  const E* srow = S + row * ld;
  const E* trow = Tl + row * ld;
  const float zero8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (lab < 0) {
    if (tid == 0) { row_out[row * 2] = 0.f; row_out[row * 2 + 1] = 0.f; }
    if (dS)
      for (int c = tid; c < nch_ld; c += NT) store8(dS + row * ld + c * 8, zero8);
    return;
  }
  const float invT = 1.f / T;
  Stats st = {-INFINITY, 0.f, 0.f, -INFINITY, 0.f, 0.f};
  for (int c = tid; c < nch; c += NT) {
    float sv[8], tv[8];
    load8(srow + c * 8, sv);
    load8(trow + c * 8, tv);
    float s[8], t[8];
    float cms = -INFINITY, cmt = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const bool ok = c * 8 + j < V;
      s[j] = ok ? sv[j] : -INFINITY;
      t[j] = ok ? tv[j] : -INFINITY;
      cms = fmaxf(cms, s[j]);
      cmt = fmaxf(cmt, t[j]);
    }
    if (cms > st.ms) {
      const float d = st.ms - cms;
      st.z1 *= __expf(d); st.zt *= __expf(d * invT); st.ms = cms;
    }
    if (cmt > st.mt) {
      const float f = __expf((st.mt - cmt) * invT);
      st.ztt *= f; st.a *= f; st.mt = cmt;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (c * 8 + j < V) {
        st.z1 += __expf(s[j] - st.ms);
        st.zt += __expf((s[j] - st.ms) * invT);
        const float e = __expf((t[j] - st.mt) * invT);
        st.ztt += e;
        st.a += e * (t[j] - s[j]);
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Stats y = shfl_stats(st, o);
    merge(st, y, invT);
  }
  if ((tid & 63) == 0) red[tid >> 6] = st;
  __syncthreads();
  Stats tot = red[0];
#pragma unroll
  for (int w = 1; w < NT / 64; ++w) merge(tot, red[w], invT);

  const float lse1 = tot.ms + __logf(tot.z1);                // logsumexp(s)
  const float lsesT = tot.ms * invT + __logf(tot.zt);        // logsumexp(s/T)
  const float lsetT = tot.mt * invT + __logf(tot.ztt);       // logsumexp(t/T)
  if (tid == 0) {
    row_out[row * 2] = lse1 - to_f32(srow[lab]);
    row_out[row * 2 + 1] = (tot.a / tot.ztt) * invT - lsetT + lsesT;
  }
  if (!dS) return;
  // dS may alias S (the trainer writes the gradient over the student logits, which nothing reads afterwards): every
  // chunk below is read and then written by the same thread; the barrier orders thread 0's read of s[label] first
  __syncthreads();
  const float N = (float)max(*n_valid, 1);
  const float gce = grad_scale * ce_w / N;
  const float gkl = grad_scale * kl_w * T / N;
  E* drow = dS + row * ld;
  for (int c = tid; c < nch_ld; c += NT) {
    float out[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (c < nch) {
      float sv[8], tv[8];
      load8(srow + c * 8, sv);
      load8(trow + c * 8, tv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int v = c * 8 + j;
        if (v < V) {
          const float s = sv[j], t = tv[j];
          const float sm1 = __expf(s - lse1);
          const float q = __expf(s * invT - lsesT);
          const float pp = __expf(t * invT - lsetT);
          out[j] = gce * (sm1 - (v == lab ? 1.f : 0.f)) + gkl * (q - pp);
        }
      }
    }
    store8(drow + c * 8, out);
  }
}

// out[0] = ce_w*ce + kl_w*kl ; out[1] = ce ; out[2] = kl  (kl already x T^2)
__global__ void klce_reduce_kernel(const float* __restrict__ row_out, int64_t rows, const int* __restrict__ n_valid,
                                   float T, float ce_w, float kl_w, float* __restrict__ out) {
  __shared__ float red[2][16];
  double a = 0.0, b = 0.0;
  for (int64_t r = threadIdx.x; r < rows; r += blockDim.x) { a += row_out[r * 2]; b += row_out[r * 2 + 1]; }
  float fa = (float)a, fb = (float)b;
  fa = wave_sum(fa); fb = wave_sum(fb);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = fa; red[1][threadIdx.x >> 6] = fb; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sa = 0.f, sb = 0.f;
    for (int w = 0; w < (int)(blockDim.x / 64); ++w) { sa += red[0][w]; sb += red[1][w]; }
    const float N = (float)max(*n_valid, 1);
    const float ce = sa / N, kl = sb / N * T * T;
    out[0] = ce_w * ce + kl_w * kl; out[1] = ce; out[2] = kl;
  }
}

}  // namespace

// row_out: rows*2 floats workspace; out3: [loss, ce, kl]; dlogits may be null (eval / no grad) or s_logits itself.
extern "C" int tw_kl_ce(const void* s_logits, const void* t_logits, int64_t ld, int logits_dtype,
                        const int64_t* labels, int64_t rows, int V, float T, float ce_w, float kl_w, const int* n_valid,
                        float grad_scale, float* row_out, float* out3, void* dlogits, hipStream_t stream) {
  if (rows <= 0) return TW_OK;
  if ((ld % 8) != 0 || ld < V) return TW_EINVAL;
  if ((((uintptr_t)s_logits) | ((uintptr_t)t_logits) | ((uintptr_t)dlogits)) & 15) return TW_EINVAL;
  if (logits_dtype == TW_BF16)
    hipLaunchKernelGGL(klce_kernel<bf16>, dim3(rows), dim3(NT), 0, stream, (const bf16*)s_logits, (const bf16*)t_logits,
                       ld, labels, V, T, ce_w, kl_w, n_valid, grad_scale, row_out, (bf16*)dlogits);
  else if (logits_dtype == TW_F16)      // the fp16 model's eval CE (HF upcasts fp16 logits to fp32)
    hipLaunchKernelGGL(klce_kernel<f16>, dim3(rows), dim3(NT), 0, stream, (const f16*)s_logits, (const f16*)t_logits,
                       ld, labels, V, T, ce_w, kl_w, n_valid, grad_scale, row_out, (f16*)dlogits);
  else if (logits_dtype == TW_F32)
    hipLaunchKernelGGL(klce_kernel<float>, dim3(rows), dim3(NT), 0, stream, (const float*)s_logits,
                       (const float*)t_logits, ld, labels, V, T, ce_w, kl_w, n_valid, grad_scale, row_out,
                       (float*)dlogits);
  else
    return TW_EUNSUPPORTED;
  hipLaunchKernelGGL(klce_reduce_kernel, dim3(1), dim3(1024), 0, stream, row_out, rows, n_valid, T, ce_w, kl_w, out3);
  TW_CHECK_LAUNCH();
  return TW_OK;
}
