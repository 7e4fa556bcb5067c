// Shared device helpers for the vision-pt MI355X (gfx950) kernel library.
// bf16 storage is `unsigned short`; math is f32. MFMA fragment typedefs follow
// the gfx950 intrinsic signatures (see /opt/skills/guides/cdna_hip_programming.md §3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define VPT_LDS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((uint32_t)x) << 16); }

// Round-to-nearest-even f32 -> bf16 (NaN preserved by the hardware cvt at -O3).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ float h2f(unsigned short h) {
  _Float16 v = __builtin_bit_cast(_Float16, h);
  return (float)v;
}
__device__ __forceinline__ unsigned short f2h(float f) {
  _Float16 v = (_Float16)f;
  return __builtin_bit_cast(unsigned short, v);
}

typedef float float2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// Two f32 -> packed bf16 pair (RNE) as ONE v_cvt_pk_bf16_f32 (a per-element cast costs a convert per
// half plus an OR to merge).
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  const float2_t v = {lo, hi};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}

// Logistic sigmoid on the hardware transcendental units: rcp(1 + 2^(-x log2 e)) = v_exp_f32 + v_rcp_f32
// (~1 ulp each), instead of libm expf + IEEE division (~30 instructions). Used by the SwiGLU forward and
// backward (fused GEMM epilogues and the elementwise kernels alike, so the two paths stay bit-identical);
// against torch's bf16 silu (expf + division in f32) the bf16 results differ by at most one bf16 ulp.
// Limits: x -> -inf gives 2^inf = inf, rcp(inf) = 0; x -> +inf gives rcp(1) = 1; NaN propagates.
__device__ __forceinline__ float sigmoid_hw(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}

// SwiGLU element math shared by the fused GEMM epilogues (gemm.hip) and the elementwise kernels (misc.hip),
// with FP contraction off so both compile to the same operations (the two paths are tested bit-identical).
// Forward: h = bf16(bf16(silu(x1)) * x2) (the reference's silu(x1) * x2 on bf16 tensors, denoiser.py:480-506).
__device__ __forceinline__ float swiglu_fwd1(float x1, float x2) {
#pragma clang fp contract(off)
  const float s = x1 * sigmoid_hw(x1);
  return bf2f(f2bf(s)) * x2;
}
// Backward of one element: dh (bf16 value) -> dx1 = bf16(dh * x2) * silu'(x1), dx2 = dh * bf16(silu(x1)).
__device__ __forceinline__ void swiglu_bwd1(float gd, float a, float b, float& d1, float& d2) {
#pragma clang fp contract(off)
  const float sg = sigmoid_hw(a);
  const float sv = bf2f(f2bf(a * sg));
  const float ds = bf2f(f2bf(gd * b));
  d2 = gd * sv;
  d1 = ds * (sg * (1.f + a * (1.f - sg)));
}

// Per-head QK-RMSNorm + RoPE forward math on one lane's 8 consecutive head dims (4 RoPE pairs), shared by
// qknorm_rope_fwd_kernel (norm.hip) and the QKV GEMM's fused epilogue (gemm.hip), contraction off so both compile to
// the same operations (tested bitwise equal). qkn_sumsq8: the lane's part of the sum of squares (the callers add the
// other 7 lanes' parts by xor-shuffles 1, 2, 4); qkn_rope8: y = rope(bf16(x r w)) * osc with r = rsqrt(ss / 64 + eps).
__device__ __forceinline__ float qkn_sumsq8(const float (&f)[8]) {
#pragma clang fp contract(off)
  float ss = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) ss += f[e] * f[e];
  return ss;
}
__device__ __forceinline__ float qkn_rstd(float ss, float eps) {
#pragma clang fp contract(off)
  return rsqrtf(ss * (1.f / 64.f) + eps);
}
__device__ __forceinline__ void qkn_rope8(const float (&f)[8], float r, const float (&w)[8], const float (&c)[4],
                                          const float (&sn)[4], float osc, float (&y)[8]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = bf2f(f2bf((f[2 * i] * r) * w[2 * i]));
    const float b = bf2f(f2bf((f[2 * i + 1] * r) * w[2 * i + 1]));
    y[2 * i] = (a * c[i] - b * sn[i]) * osc;
    y[2 * i + 1] = (a * sn[i] + b * c[i]) * osc;
  }
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

// 16-byte vector of 8 bf16 viewed as uint4.
__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  uint4 r;
  r.x = pack_bf16x2(f[0], f[1]); r.y = pack_bf16x2(f[2], f[3]);
  r.z = pack_bf16x2(f[4], f[5]); r.w = pack_bf16x2(f[6], f[7]);
  return r;
}

// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies row q / cols 4p..4p+3 of a
// 4x16 block; lane i receives column i of the 4 rows (element q = row q).
__device__ __forceinline__ uint2 lds_read_tr16(const VPT_LDS void* p) {
  short4_t v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((VPT_LDS short4_t*)p);
  return __builtin_bit_cast(uint2, v);
}

__device__ __forceinline__ bf16x8 as_frag(uint4 v) { return __builtin_bit_cast(bf16x8, v); }
__device__ __forceinline__ bf16x8 as_frag2(uint2 a, uint2 b) {
  uint4 v = make_uint4(a.x, a.y, b.x, b.y);
  return __builtin_bit_cast(bf16x8, v);
}

// Error codes shared by every C-ABI entry point (include/vpt_hip.h).
#define VPT_OK 0
#define VPT_EINVAL 1
#define VPT_EUNSUPPORTED 2
#define VPT_ELAUNCH 3

extern "C" void vpt_set_error(const char* msg);

#define VPT_CHECK_ARG(cond, msg)            \
  do {                                      \
    if (!(cond)) {                          \
      vpt_set_error(msg);                   \
      return VPT_EINVAL;                    \
    }                                       \
  } while (0)

#define VPT_LAUNCH_CHECK()                                   \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) {                                  \
      vpt_set_error(hipGetErrorString(_e));                  \
      return VPT_ELAUNCH;                                    \
    }                                                        \
  } while (0)

// Column sums of a [R][C] f32 partial set for columns [16 cb, 16 cb + 16): out[c] (=|+=) sum_r in[r][c]. One block of
// 4 * RG threads (4 lanes x float4 = 16 columns, RG row groups): each row group strides over the rows in a fixed
// order, then a fixed pairwise tree over the row groups in `red` (deterministic, no atomics). Used by vpt_reduce_rows
// and, as an extra job riding a weight gradient's split-K reduce launch, by vpt_linear_wgrad_rr.
template <int RG>
__device__ __forceinline__ void colsum_block(const float* __restrict__ in, int R, int C, float* __restrict__ out,
                                             int accumulate, int cb, floatx4 (&red)[RG][4]) {
  const int cl = threadIdx.x & 3, rg = threadIdx.x >> 2;
  const int c = cb * 16 + cl * 4;
  floatx4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    if (C % 4 == 0) {
#pragma unroll 4
      for (int r = rg; r < R; r += RG) s += *reinterpret_cast<const floatx4*>(in + (long)r * C + c);
    } else {
      for (int r = rg; r < R; r += RG)
        for (int e = 0; e < 4; ++e)
          if (c + e < C) s[e] += in[(long)r * C + c + e];
    }
  }
  red[rg][cl] = s;
  __syncthreads();
#pragma unroll
  for (int st = RG / 2; st >= 1; st >>= 1) {
    if (rg < st) red[rg][cl] += red[rg + st][cl];
    __syncthreads();
  }
  if (rg == 0 && c < C) {
    const floatx4 t = red[0][cl];
    for (int e = 0; e < 4 && c + e < C; ++e) out[c + e] = accumulate ? out[c + e] + t[e] : t[e];
  }
}
