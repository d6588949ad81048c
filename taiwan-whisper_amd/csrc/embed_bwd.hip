// Token-embedding backward, deterministic (replaces the autograd of HF WhisperDecoder's
// nn.Embedding(vocab, d, padding_idx = pad_token_id) lookup, modeling_whisper.py decoder embed_tokens; the
// tied LM-head part of the same gradient is a GEMM in the trainer).  dE[id] += sum over positions t with
// ids[t] == id of dh[t], summed in position order for every id -- the result does not depend on scheduling
// (PyTorch's CUDA embedding backward is likewise sort-based and deterministic); a float-atomic scatter
// would not be.  Positions holding padding_idx contribute nothing (nn.Embedding's padding_idx rule): they
// sort last under an out-of-range key and are never summed -- which also keeps the padded tail of a
// batch (~45 % of the positions at c3) out of one long serial group.
//
//   1. keys = ids (uint32), values = positions, stable radix sort (hipCUB) -> positions grouped by id,
//      ascending within a group;
//   2. one workgroup per sorted index that starts a group: sum the group's rows (fp32, position order),
//      one read-modify-write of dE[id] (each id has exactly one writer: no atomics).
// Rows whose gradient is exactly zero (padding after the last label, HF's padding_idx rows) add 0.
// Scratch: the per-device block (tw_device_workspace), stream-ordered.
#include "common.h"

#include <hipcub/hipcub.hpp>

namespace {

constexpr uint32_t SKIP = 0xffffffffu;

__global__ void embed_keys_kernel(const int64_t* __restrict__ ids, uint32_t* __restrict__ keys,
                                  uint32_t* __restrict__ pos, int rows, int64_t padding_idx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < rows) {
    keys[i] = ids[i] == padding_idx ? SKIP : (uint32_t)ids[i];
    pos[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256) void embed_group_sum_kernel(const uint32_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ pos,
                                                              const float* __restrict__ dh, float* __restrict__ dE,
                                                              int rows, int D) {
  const int i = blockIdx.x;
  const uint32_t id = keys[i];
  if (id == SKIP || (i > 0 && keys[i - 1] == id)) return;   // padding_idx, or not the first of its group
  int j_end = i + 1;
  while (j_end < rows && keys[j_end] == id) ++j_end;
  for (int e = threadIdx.x; e < D; e += blockDim.x) {
    float acc = 0.f;
#pragma unroll 8
    for (int j = i; j < j_end; ++j) acc += dh[(int64_t)pos[j] * D + e];
    dE[(int64_t)id * D + e] += acc;
  }
}

}  // namespace

extern "C" int tw_embed_bwd(const int64_t* ids, const float* dh, float* dE, int rows, int D, int64_t padding_idx,
                            hipStream_t stream) {
  if (rows <= 0) return TW_OK;
  size_t sort_bytes = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, rows, 0, 32, stream) !=
      hipSuccess)
    return TW_EHIP;
  const size_t arr = ((size_t)rows * sizeof(uint32_t) + 255) / 256 * 256;
  char* ws = (char*)tw_device_workspace(stream, 4 * arr + sort_bytes);
  if (!ws) return TW_EHIP;
  uint32_t *k_in = (uint32_t*)ws, *p_in = (uint32_t*)(ws + arr), *k_out = (uint32_t*)(ws + 2 * arr),
           *p_out = (uint32_t*)(ws + 3 * arr);
  hipLaunchKernelGGL(embed_keys_kernel, dim3((rows + 255) / 256), dim3(256), 0, stream, ids, k_in, p_in, rows,
                     padding_idx);
  if (hipcub::DeviceRadixSort::SortPairs(ws + 4 * arr, sort_bytes, k_in, k_out, p_in, p_out, rows, 0, 32, stream) !=
      hipSuccess)
    return TW_EHIP;
  hipLaunchKernelGGL(embed_group_sum_kernel, dim3(rows), dim3(256), 0, stream, k_out, p_out, dh, dE, rows, D);
  TW_CHECK_LAUNCH();
  return TW_OK;
}
