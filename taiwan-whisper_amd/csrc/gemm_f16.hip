// The fp16 entry points of gemm.hip (tw_gemm_f16 / tw_gemv_f16: the fp16 decode path and fp16-autocast
// training) as their own translation unit: the same source, compiled with TW_GEMM_TU_F16, instantiates the H = true
// kernels only, so the two halves of the GEMM library build in parallel.
#define TW_GEMM_TU_F16 1
#include "gemm.hip"
