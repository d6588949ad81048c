// Store-shape microbenchmark for the GEMM epilogue (standalone: hipcc --offload-arch=gfx950 -O3).
// Writes an M x N bf16 matrix tile by tile (256x256 per 512-thread workgroup, 8 waves as 2x4,
// 128x64 per wave) in the shapes a swapped-operand 16x16 MFMA epilogue can produce:
//   P1  8 B per lane: lane (li, g) -> row li, cols 16*ni + 4g .. +3   (16 rows x 32 B per instr)
//   P2  16 B per lane after v_permlane16_swap of fragment pairs      (16 rows x 64 B per instr)
//   P3  16 B per lane, 8 rows x 128 B per instr (what an LDS transpose gives)
// Prints GB/s per pattern.  Not part of the library; a measurement aid for tools/ and DESIGN.md.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>

#include <cstdio>
#include <cstdint>

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int P>
__global__ __launch_bounds__(512) void store_kernel(uint16_t* C, int M, int N, int tiles_n) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int mt = blockIdx.x / tiles_n, nt = blockIdx.x % tiles_n;
  const int r0 = mt * 256 + wm * 128, c0 = nt * 256 + wn * 64;
  const int li = lane & 15, g = lane >> 4;
  const uint32_t v = 0x3f803f80u ^ (blockIdx.x * 2654435761u);
  if (P == 1) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        uint16_t* p = C + (int64_t)(r0 + mi * 16 + li) * N + c0 + ni * 16 + 4 * g;
        *(u32x2*)p = u32x2{v + mi, v + ni};
      }
  } else if (P == 2) {
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        u32x2 x = {v + mi, v + pr}, y = {v + mi + 1, v + pr + 1};
        auto s0 = __builtin_amdgcn_permlane16_swap(x[0], y[0], false, false);
        auto s1 = __builtin_amdgcn_permlane16_swap(x[1], y[1], false, false);
        uint16_t* p = C + (int64_t)(r0 + mi * 16 + li) * N + c0 + pr * 32 + (g & 1) * 16 + (g >> 1) * 8;
        *(u32x4*)p = u32x4{s0[0], s1[0], s0[1], s1[1]};
      }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint16_t* p = C + (int64_t)(r0 + i * 8 + (lane >> 3)) * N + c0 + (lane & 7) * 8;
      *(u32x4*)p = u32x4{v + i, v, v, v};
    }
  }
}

int main() {
  const int M = 96000, N = 5120;
  uint16_t* C;
  if (hipMalloc(&C, (size_t)M * N * 2) != hipSuccess) return 1;
  const int tiles_n = N / 256, tiles = (M / 256) * tiles_n;   // M, N multiples of 256 here
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int round = 0; round < 3; ++round) {
    for (int p = 1; p <= 3; ++p) {
      auto launch = [&] {
        if (p == 1) hipLaunchKernelGGL(store_kernel<1>, dim3(tiles), dim3(512), 0, 0, C, M, N, tiles_n);
        else if (p == 2) hipLaunchKernelGGL(store_kernel<2>, dim3(tiles), dim3(512), 0, 0, C, M, N, tiles_n);
        else hipLaunchKernelGGL(store_kernel<3>, dim3(tiles), dim3(512), 0, 0, C, M, N, tiles_n);
      };
      launch();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      printf("round %d P%d: %8.1f us  %7.1f GB/s\n", round, p, ms * 1e3, (double)M * N * 2 / (ms * 1e-3) / 1e9);
    }
  }
  (void)hipFree(C);
  return 0;
}
