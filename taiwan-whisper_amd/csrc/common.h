// Shared device helpers for the tw HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((address_space(3))) void lds_void;

// status codes of the C-ABI (include/tw_hip.h)
#define TW_OK 0
#define TW_EINVAL 1
#define TW_EUNSUPPORTED 2
#define TW_EHIP 3

#define TW_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t e__ = hipGetLastError();                     \
    if (e__ != hipSuccess) return TW_EHIP;                  \
  } while (0)

// dtype codes shared with the host side
enum { TW_F32 = 0, TW_BF16 = 1, TW_F16 = 2 };

typedef _Float16 f16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }
__device__ __forceinline__ float rbf(float x) { return (float)(bf16)x; }   // round-trip through bf16 (RNE)

// ---- 16-bit operand codec of the MFMA kernels.  Their operands and 16-bit outputs are moved as raw 16-bit
// words (typed `bf16` in the kernels: loads, LDS images, fragments); H selects what the words hold:
// H = false: bf16 (the CUDA-autocast path), H = true: IEEE fp16 (the reference's torch_dtype=float16
// decode path, run_eval.py:99,500-509 / run_pseudo_labelling.py:461-463).  Rounding is RNE either way.
template <bool H>
__device__ __forceinline__ float e2f(bf16 x) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, x);
  else return (float)x;
}
template <bool H>
__device__ __forceinline__ bf16 f2e(float x) {
  if constexpr (H) {
    // x is materialised as an fp32 value first: without this the backend folds fptrunc(fma(a, b, c)) into
    // v_fma_mixlo_f16, which rounds the exact a*b+c to fp16 ONCE -- the reference (an fp32 GEMM epilogue, then
    // the cast) rounds twice, and the two differ on ~2e-5 of the outputs (tests/test_fp16_gpu.py)
    asm("" : "+v"(x));
    return __builtin_bit_cast(bf16, (_Float16)x);
  } else {
    return (bf16)x;
  }
}
template <bool H>
__device__ __forceinline__ float rnd(float x) { return e2f<H>(f2e<H>(x)); }
// v_mfma_f32_16x16x32_{bf16,f16}: A, B = 8 16-bit words per lane, fp32 accumulate
template <bool H>
__device__ __forceinline__ f32x4 mma16(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (H)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// fp16 saturation of HF WhisperEncoderLayer (modeling_whisper.py:409-411: clamp to finfo(fp16).max - 1000 after
// the MLP residual when the stream is fp16); applied to the fp16-rounded value, so +-inf -> the bound too
__device__ __forceinline__ float clamp_f16_stream(float x) {
  return fminf(fmaxf(x, -64504.0f), 64504.0f);
}

// 8 consecutive elements of a bf16 / fp32 row as fp32 (16-B / 2 x 16-B vector loads; the caller
// guarantees alignment), and the inverse store
__device__ __forceinline__ void load8(const bf16* p, float* o) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = bf2f(v[j]);
}
__device__ __forceinline__ void load8(const float* p, float* o) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = a[3]; o[4] = b[0]; o[5] = b[1]; o[6] = b[2]; o[7] = b[3];
}
__device__ __forceinline__ void store8(bf16* p, const float* v) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
  *(bf16x8*)p = o;
}
__device__ __forceinline__ void store8(float* p, const float* v) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void load8(const f16* p, float* o) {
  const f16x8 v = *(const f16x8*)p;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (float)v[j];
}
__device__ __forceinline__ void store8(f16* p, const float* v) {
  f16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (_Float16)v[j];
  *(f16x8*)p = o;
}
__device__ __forceinline__ float to_f32(bf16 x) { return bf2f(x); }
__device__ __forceinline__ float to_f32(f16 x) { return (float)x; }
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ void from_f32(bf16& d, float x) { d = f2bf(x); }
__device__ __forceinline__ void from_f32(f16& d, float x) { d = (_Float16)x; }
__device__ __forceinline__ void from_f32(float& d, float x) { d = x; }

template <typename E> __device__ __forceinline__ E e_from_f32(float x) { E d; from_f32(d, x); return d; }

__device__ __forceinline__ float ld_as_f32(const void* p, int dtype, int64_t i) {
  return dtype == TW_BF16 ? (float)((const bf16*)p)[i]
       : dtype == TW_F16  ? (float)((const f16*)p)[i] : ((const float*)p)[i];
}
__device__ __forceinline__ void st_from_f32(void* p, int dtype, int64_t i, float v) {
  if (dtype == TW_BF16) ((bf16*)p)[i] = f2bf(v);
  else if (dtype == TW_F16) ((f16*)p)[i] = (_Float16)v;
  else ((float*)p)[i] = v;
}

// erf, branch-free (Abramowitz & Stegun 7.1.26: |error| <= 1.5e-7 absolute, ~14 VALU, no
// divergent polynomial pair as in the libm erff): GELU sits in GEMM epilogues, where every VALU
// of a 256x256 tile is exposed.
__device__ __forceinline__ float erf_fast(float z) {
  const float a = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float q = fmaf(1.061405429f, t, -1.453152027f);
  q = fmaf(q, t, 1.421413741f);
  q = fmaf(q, t, -0.284496736f);
  q = fmaf(q, t, 0.254829592f);
  q *= t;
  const float e = __builtin_amdgcn_exp2f(-(a * a) * 1.44269504088896341f);
  return copysignf(fmaf(-q, e, 1.0f), z);
}
// Two GELUs at once in the Phi form, gelu(x) = x * Phi(x) with Phi(x) = 1 - h (x >= 0), h (x < 0),
// h = erfc(|x|/sqrt2) / 2 = (t * P(t) / 2) * exp(-x^2/2) (the A&S 7.1.26 polynomial as above,
// coefficients pre-halved): the FMA/MUL chain runs as packed fp32 (v_pk_fma_f32 / v_pk_mul_f32,
// two lanes' worth per instruction), only rcp / exp2 / the select stay scalar.  Same error
// bound as gelu_erf; for x < 0 it avoids the 1 - (1 - small) cancellation.
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 gelu_erf2(f32x2 x) {
  const f32x2 ax = {__builtin_fabsf(x.x), __builtin_fabsf(x.y)};
  const f32x2 a = ax * 0.70710678118654752440f;
  const f32x2 d = a * 0.3275911f + 1.0f;
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 q = t * 0.5307027145f + -0.7265760135f;
  q = q * t + 0.7107068705f;
  q = q * t + -0.142248368f;
  q = q * t + 0.127414796f;
  q = q * t;
  const f32x2 w = (x * x) * -0.72134752044448170f;          // -x^2/2 * log2(e)
  const f32x2 e = {__builtin_amdgcn_exp2f(w.x), __builtin_amdgcn_exp2f(w.y)};
  const f32x2 h = q * e;
  const f32x2 g = 1.0f - h;
  const f32x2 phi = {x.x >= 0.f ? g.x : h.x, x.y >= 0.f ? g.y : h.y};
  return x * phi;
}
// GELU (HF ACT2FN["gelu"], erf form), one value: the operation sequence of gelu_erf2, so every
// epilogue (packed fast path, generic, per-element) rounds identically
__device__ __forceinline__ float gelu_erf(float x) {
  const float a = __builtin_fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(a * 0.3275911f + 1.0f);
  float q = t * 0.5307027145f + -0.7265760135f;
  q = q * t + 0.7107068705f;
  q = q * t + -0.142248368f;
  q = q * t + 0.127414796f;
  q = q * t;
  const float h = q * __builtin_amdgcn_exp2f((x * x) * -0.72134752044448170f);
  return x * (x >= 0.f ? 1.0f - h : h);
}

// GELU of the instantiation's operand type: bf16 -> the branch-free polynomial above (every bf16 result within
// 1 ulp of torch's fp32 formula, tools/gelu_sweep.py); fp16 (10-bit mantissa, subnormals down to 6e-8) -> torch's
// own formula x/2 (1 + erf(x/sqrt2)) with the device erff: the polynomial's 1.5e-7 absolute error is ~2 fp16
// ulps of the small negative outputs, where the reference's fp32 formula is what it is
template <bool H>
__device__ __forceinline__ float gelu_of(float x) {
  if constexpr (H) return x * 0.5f * (1.0f + erff(x * 0.70710678118654752440f));
  else return gelu_erf(x);
}

__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.0f + erf_fast(x * 0.70710678118654752440f));
  const float pdf = 0.39894228040143267794f * __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);
  return cdf + x * pdf;
}
// GELU derivative of the instantiation's operand type: bf16 -> the polynomial erf above (its 1.5e-7 absolute error is
// far below a bf16 ulp of any product); fp16 -> the device erff / expf (torch's gelu backward formula): for x < -3 the
// polynomial's error is ~1e-4 of gelu'(x), a third of an fp16 ulp, and flips roundings of fp16-autocast gradients
template <bool H>
__device__ __forceinline__ float gelu_grad_of(float x) {
  if constexpr (H)
    return 0.5f * (1.0f + erff(x * 0.70710678118654752440f)) + x * 0.39894228040143267794f * expf(-0.5f * x * x);
  else
    return gelu_erf_grad(x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- the same butterflies on the VALU (DPP row rotations / mirrors, v_permlane16/32_swap) instead of ds_bpermute
// round trips.  Each keeps the xor pairing order of the __shfl_xor form it replaces; where a rotation reaches a lane
// other than the xor partner, that lane already holds the partner's value (the earlier steps made the lanes of each
// merged class equal), and IEEE addition is commutative, so the results are bit-identical.
#define TW_DPP(v, ctrl) __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), (ctrl), 0xf, 0xf, false))
#define TW_ROW_ROR(n) (0x120 + (n))
#define TW_QUAD_XOR1 0xB1          // quad_perm [1,0,3,2]
#define TW_QUAD_XOR2 0x4E          // quad_perm [2,3,0,1]
#define TW_ROW_HALF_MIRROR 0x141   // lane i <-> 7 - i within each 8 (xor 4 once the quads are merged)
__device__ __forceinline__ float swap32_sum(float v) {
  const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
__device__ __forceinline__ float swap16_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(a[0]) + __uint_as_float(a[1]);
}
// wave_sum: xor 32, 16, 8, 4, 2, 1
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v = swap32_sum(v);
  v = swap16_sum(v);
  v += TW_DPP(v, TW_ROW_ROR(8));
  v += TW_DPP(v, TW_ROW_ROR(4));
  v += TW_DPP(v, TW_ROW_ROR(2));
  v += TW_DPP(v, TW_ROW_ROR(1));
  return v;
}
// xor 1, 2, 4 (a sum over each 8-lane group)
__device__ __forceinline__ float oct_sum_dpp(float v) {
  v += TW_DPP(v, TW_QUAD_XOR1);
  v += TW_DPP(v, TW_QUAD_XOR2);
  v += TW_DPP(v, TW_ROW_HALF_MIRROR);
  return v;
}
// xor 8, 16, 32 (a sum over the lanes with equal lane & 7)
__device__ __forceinline__ float stride8_sum_dpp(float v) {
  v += TW_DPP(v, TW_ROW_ROR(8));
  v = swap16_sum(v);
  return swap32_sum(v);
}
// xor 16, 8, 4, 2, 1 (a sum over each 32-lane half)
__device__ __forceinline__ float half_sum_dpp(float v) {
  v = swap16_sum(v);
  v += TW_DPP(v, TW_ROW_ROR(8));
  v += TW_DPP(v, TW_ROW_ROR(4));
  v += TW_DPP(v, TW_ROW_ROR(2));
  v += TW_DPP(v, TW_ROW_ROR(1));
  return v;
}
// lane c's value (c wave-uniform); the builtin is int-typed, so the bits go through as an int
__device__ __forceinline__ float readlane_f(float v, int c) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), c));
}
// wave_max (max is order-independent)
__device__ __forceinline__ float wave_max_dpp(float v) {
  {
    const auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  }
  {
    const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  }
  v = fmaxf(v, TW_DPP(v, TW_ROW_ROR(8)));
  v = fmaxf(v, TW_DPP(v, TW_ROW_ROR(4)));
  v = fmaxf(v, TW_DPP(v, TW_ROW_ROR(2)));
  v = fmaxf(v, TW_DPP(v, TW_ROW_ROR(1)));
  return v;
}

// raw buffer descriptor: out-of-range per-lane offsets (>= num_records) read as zero.
#define TW_OOB 0x80000000u
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)0x80000000, 0x00020000);
}

// 16-byte buffer load straight into LDS: lane l writes lds_base + 16*l (wave-uniform base).
__device__ __forceinline__ void buf_load_lds16(__amdgpu_buffer_rsrc_t r, void* lds_base, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_base, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id_uniform() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// order-preserving float <-> uint mapping for atomicMax on floats
__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// Per-device scratch block (gemm.hip): grown outside stream capture only, never freed (a captured graph
// may hold an older block); users on one stream are ordered, so they may share it.  nullptr when it
// cannot grow (e.g. during capture): callers fall back to a path without scratch.
void* tw_device_workspace(hipStream_t stream, size_t bytes);
