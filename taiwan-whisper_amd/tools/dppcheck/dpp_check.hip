// Unit check of the DPP / permlane-swap reductions in csrc/common.h against the __shfl_xor butterflies they
// replace: bitwise per lane, random data, full waves.  hipcc --offload-arch=gfx950 -O3 -I../../csrc dpp_check.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "common.h"

__global__ void k(const float* in, float* out, int n) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x;
  float v = in[w * 64 + lane];
  float r[12];
  // reference butterflies
  float a = v;
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  r[0] = a;
  r[1] = wave_sum_dpp(v);
  a = v;
  a += __shfl_xor(a, 1, 64); a += __shfl_xor(a, 2, 64); a += __shfl_xor(a, 4, 64);
  r[2] = a;
  r[3] = oct_sum_dpp(v);
  a = v;
  a += __shfl_xor(a, 8, 64); a += __shfl_xor(a, 16, 64); a += __shfl_xor(a, 32, 64);
  r[4] = a;
  r[5] = stride8_sum_dpp(v);
  a = v;
  for (int o = 32; o > 0; o >>= 1) a = fmaxf(a, __shfl_xor(a, o, 64));
  r[6] = a;
  r[7] = wave_max_dpp(v);
  r[8] = __shfl(v, 5, 64);
  r[9] = readlane_f(v, 5);
  a = v;
  for (int o = 16; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
  r[10] = a;
  r[11] = half_sum_dpp(v);
  for (int i = 0; i < 12; ++i) out[(w * 12 + i) * 64 + lane] = r[i];
}

int main() {
  const int W = 64;
  float* h = (float*)malloc(W * 64 * 4);
  srand(1);
  for (int i = 0; i < W * 64; ++i) h[i] = ((rand() / (float)RAND_MAX) - 0.5f) * powf(2.f, (rand() % 20) - 10);
  float *din, *dout;
  hipMalloc(&din, W * 64 * 4);
  hipMalloc(&dout, W * 768 * 4);
  hipMemcpy(din, h, W * 64 * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(W), dim3(64), 0, 0, din, dout, W);
  float* o = (float*)malloc(W * 768 * 4);
  hipMemcpy(o, dout, W * 768 * 4, hipMemcpyDeviceToHost);
  const char* names[] = {"wave_sum", "oct_sum", "stride8_sum", "wave_max", "readlane", "half_sum"};
  int bad_total = 0;
  for (int t = 0; t < 6; ++t) {
    int bad = 0, first = -1;
    for (int w = 0; w < W; ++w)
      for (int l = 0; l < 64; ++l) {
        const float x = o[(w * 12 + 2 * t) * 64 + l], y = o[(w * 12 + 2 * t + 1) * 64 + l];
        if (memcmp(&x, &y, 4)) { if (first < 0) first = w * 64 + l; ++bad; }
      }
    printf("%-12s mismatching lanes %d / %d", names[t], bad, W * 64);
    if (first >= 0) {
      const int w = first / 64, l = first % 64;
      printf("  first: wave %d lane %d ref %.9g dpp %.9g", w, l, o[(w * 12 + 2 * t) * 64 + l], o[(w * 12 + 2 * t + 1) * 64 + l]);
    }
    printf("\n");
    bad_total += bad;
  }
  return bad_total ? 1 : 0;
}
