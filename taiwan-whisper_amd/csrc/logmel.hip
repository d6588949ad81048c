// Whisper log-mel front end on the GPU (replaces the CPU
// WhisperFeatureExtractor call at training/run_distillation.py:1217, HF
// feature_extraction_whisper.py:135-170): center reflect pad 200, 400-pt periodic Hann
// frames every 160 samples, |DFT|^2 (201 bins), slaney mel (80), log10(max(x,1e-10)),
// max(x, clip_max - 8), (x + 4) / 4.
//
// Clips are n_samples long (480 000 = 30 s for the training / short-form path; any length for the
// long-form path, HF __call__(truncation=False, padding="longest"), run_eval.py:572-581), giving
// n_samples / 160 frames.
//
// Kernel 1: one workgroup = 64 frames of one clip.  The 10 480 samples the frames span
// are staged in LDS (coalesced reads, reflect padding resolved there); the windowed DFT
// runs on the exact-fp32 MFMA (v_mfma_f32_16x16x4_f32) against a [400][416] basis with the
// Hann window folded in (cos bins in columns 0..207, sin bins in 208..415); |X|^2 goes to
// LDS, the sparse mel projection + log10 is done per (frame, mel) and a per-clip max is
// kept with an order-preserving atomicMax.  Kernel 2 applies the clamp/scale and also
// emits the time-major bf16 conv1 input [B][3002][80] (zero rows 0 and 3001) that the
// encoder's zero-copy conv stem reads.
#include "common.h"

namespace {

constexpr int NFFT = 400, HOP = 160, NBIN = 201, NMEL = 80;
constexpr int FPB = 64;                        // frames per block
constexpr int NSAMP = (FPB - 1) * HOP + NFFT;  // 10480
constexpr int NCOL = 416;                      // 13 tiles cos + 13 tiles sin
constexpr int MELW = 32;                       // max taps per mel filter

typedef __attribute__((ext_vector_type(4))) float v4f;

__global__ __launch_bounds__(256, 1) void logmel_kernel(const float* __restrict__ wav, const float* __restrict__ basis,
                                                        const int* __restrict__ mel_start,
                                                        const float* __restrict__ mel_w, float* __restrict__ out,
                                                        uint32_t* __restrict__ clip_max, int64_t NS, int NFR) {
  __shared__ float samp[NSAMP];
  __shared__ float pw[FPB][NBIN + 3];
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FPB;
  const float* x = wav + (int64_t)b * NS;
  const int lane = lane_id(), wave = threadIdx.x >> 6;
  // stage samples of padded positions [f0*HOP, f0*HOP + NSAMP) with reflect padding
  for (int j = threadIdx.x; j < NSAMP; j += 256) {
    int64_t i = (int64_t)f0 * HOP + j - NFFT / 2;
    if (i < 0) i = -i;
    if (i >= NS) i = 2 * (NS - 1) - i;
    samp[j] = (i >= 0 && i < NS) ? x[i] : 0.f;
  }
  __syncthreads();

  // DFT: rows = frames (4 row tiles), cols = this wave's cos tiles + matching sin tiles
  v4f acc[4][4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c][0] = acc[a][c][1] = v4f{0.f, 0.f, 0.f, 0.f};
  const int ntile = wave == 0 ? 4 : 3;   // cos tiles wave, wave+4, wave+8, (wave+12 for wave 0)
  const int kr = lane >> 4, li = lane & 15;
  for (int k0 = 0; k0 < NFFT; k0 += 4) {
    const int n = k0 + kr;
    float av[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) av[rt] = samp[(rt * 16 + li) * HOP + n];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      if (ct < ntile) {
        const int col = (wave + 4 * ct) * 16 + li;
        const float bc = basis[n * NCOL + col];
        const float bs = basis[n * NCOL + 208 + col];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          acc[rt][ct][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[rt], bc, acc[rt][ct][0], 0, 0, 0);
          acc[rt][ct][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[rt], bs, acc[rt][ct][1], 0, 0, 0);
        }
      }
    }
  }
  // power -> LDS: lane holds D[frame = rt*16 + 4*(lane>>4) + r][bin = tile*16 + (lane&15)]
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    if (ct < ntile) {
      const int bin = (wave + 4 * ct) * 16 + li;
      if (bin < NBIN) {
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float re = acc[rt][ct][0][r], im = acc[rt][ct][1][r];
            pw[rt * 16 + 4 * kr + r][bin] = re * re + im * im;
          }
      }
    }
  }
  __syncthreads();
  // mel + log10: thread -> frame (t & 63), mels (t >> 6) + 4*j
  const int fr = threadIdx.x & 63;
  const int f = f0 + fr;
  float lmax = -INFINITY;
  for (int m = threadIdx.x >> 6; m < NMEL; m += 4) {
    const int s0 = mel_start[m];
    float acc_m = 0.f;
#pragma unroll 8
    for (int j = 0; j < MELW; ++j) {
      const float wgt = mel_w[m * MELW + j];
      const int bin = s0 + j;
      if (wgt != 0.f && bin < NBIN) acc_m += pw[fr][bin] * wgt;
    }
    const float lv = log10f(fmaxf(acc_m, 1e-10f));
    if (f < NFR) {
      out[((int64_t)b * NMEL + m) * NFR + f] = lv;
      lmax = fmaxf(lmax, lv);
    }
  }
  lmax = wave_max(lmax);
  if (lane == 0 && lmax > -INFINITY) atomicMax(clip_max + b, f2ord(lmax));
}

__global__ void logmel_finalize_kernel(float* __restrict__ mel, const uint32_t* __restrict__ clip_max,
                                       bf16* __restrict__ xt, int B, int NFR) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)B * NMEL * NFR;
  if (i < n) {
    const int b = i / ((int64_t)NMEL * NFR);
    const float floor_v = ord2f(clip_max[b]) - 8.f;
    const float v = (fmaxf(mel[i], floor_v) + 4.f) / 4.f;
    mel[i] = v;
    if (xt) {
      const int m = (i / NFR) % NMEL;
      const int t = i % NFR;
      xt[((int64_t)b * (NFR + 2) + t + 1) * NMEL + m] = f2bf(v);
    }
  }
  // zero pad rows of the conv input
  if (xt && i < (int64_t)B * 2 * NMEL) {
    const int b = i / (2 * NMEL), which = (i / NMEL) % 2, m = i % NMEL;
    xt[((int64_t)b * (NFR + 2) + (which ? NFR + 1 : 0)) * NMEL + m] = f2bf(0.f);
  }
}

}  // namespace

// wav [B][n_samples] f32 (already padded/truncated); basis [400][416]; mel_start [80]; mel_w [80][32]
// mel_out [B][80][n_samples/160] f32; conv_in (optional) [B][n_samples/160 + 2][80] bf16; workspace >= B uint32
extern "C" int tw_logmel_len(const float* wav, int B, int64_t n_samples, const float* basis, const int* mel_start,
                             const float* mel_w, float* mel_out, void* conv_in, void* workspace, hipStream_t stream) {
  if (B <= 0) return TW_OK;
  if (n_samples < NFFT / 2 + 1 || n_samples / HOP > (1 << 30) / NMEL) return TW_EINVAL;   // reflect pad needs > 200
  const int nfr = (int)(n_samples / HOP);
  uint32_t* cm = (uint32_t*)workspace;
  if (hipMemsetAsync(cm, 0, sizeof(uint32_t) * B, stream) != hipSuccess) return TW_EHIP;
  hipLaunchKernelGGL(logmel_kernel, dim3((nfr + FPB - 1) / FPB, B), dim3(256), 0, stream, wav, basis, mel_start, mel_w,
                     mel_out, cm, n_samples, nfr);
  const int64_t n = (int64_t)B * NMEL * nfr;
  hipLaunchKernelGGL(logmel_finalize_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, mel_out, cm, (bf16*)conv_in,
                     B, nfr);
  TW_CHECK_LAUNCH();
  return TW_OK;
}

extern "C" int tw_logmel(const float* wav, int B, const float* basis, const int* mel_start, const float* mel_w,
                         float* mel_out, void* conv_in, void* workspace, hipStream_t stream) {
  return tw_logmel_len(wav, B, 480000, basis, mel_start, mel_w, mel_out, conv_in, workspace, stream);
}
