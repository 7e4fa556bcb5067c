// SDXL QLoRA transformer-block kernels for gfx950:
//   LayerNorm fwd/bwd        nn.LayerNorm (norm1/2/3, src/models/sdxl/denoiser.py:254-256), eps 1e-5, affine
//   GeGLU fwd/bwd            GeGLU.forward (denoiser.py:174-186): hidden * gelu(gate), exact (erf) GELU
//   NF4 dequant / quantize   bitsandbytes 0.48.2 nf4 (src/modules/quant/bnb.py:37-129 wraps it): blocksize 64,
//                            nested absmax (8-bit blockwise over the signed dynamic map, blocksize 256, + offset)
// Row kernels: one wave per row, 16-B (8 x bf16) vector accesses, up to 4 chunks per lane (D <= 2048).
#include "common.h"
#include "../../include/vpt_hip.h"  // C-ABI types (VptNf4Job)

namespace {

constexpr int MAXC = 4;  // 16-B chunks per lane: D <= 64 * 8 * 4 = 2048

// ---------------------------------------------------------------- LayerNorm
// y = (x - mean) * rstd * w + b, statistics in f32 (nn.LayerNorm runs in f32 under autocast).
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(const bf16_t* __restrict__ x, long ldx,
                                                            const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                            bf16_t* __restrict__ y, long ldy, float* __restrict__ mean_out,
                                                            float* __restrict__ rstd_out, int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = D >> 3;
  float f[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      unpack8(*reinterpret_cast<const uint4*>(x + row * ldx + c * 8), f[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += f[i][e];
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    if (lane + 64 * i < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = f[i][e] - mean;
        ss += d * d;
      }
    }
  }
  const float r = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float wf[8], bf[8], o[8];
      unpack8(*reinterpret_cast<const uint4*>(w + c * 8), wf);
      unpack8(*reinterpret_cast<const uint4*>(b + c * 8), bf);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (f[i][e] - mean) * r * wf[e] + bf[e];
      *reinterpret_cast<uint4*>(y + row * ldy + c * 8) = pack8(o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = r;
  }
}

// LayerNorm + the LoRA down-projections of its output (the q|k|v adapters of norm1's output, attn2.to_q's of
// norm2's, ff.net.0.proj's of norm3's): ds[m][16 gi + j] = bf16(alpha * y[m] . down_gi[j]) for gi < G, written
// by the same launch that writes y -- the separate vpt_lora_proj launch (one per use, ~8 us) gone. Each block
// owns 16 rows: every wave normalises 4 rows exactly as layernorm_fwd_kernel (same arithmetic) into y and into an
// LDS image of the 16 bf16 rows; then the projection runs in lora_proj's order (csrc/gemm.hip lora_proj_kernel,
// w_kmajor: wave w takes the 128-wide K chunks w, w + 4, ..., four 16x16x32 MFMAs per chunk; the waves' sums
// added in wave order), so ds is bit-identical to layernorm_fwd + vpt_lora_proj(_grouped).
constexpr int LNL_KC = 128;  // K chunk (lora_proj's LKC)
constexpr int LNL_MAXG = 3;
__global__ __launch_bounds__(256) void layernorm_lora_fwd_kernel(const bf16_t* __restrict__ x, long ldx,
                                                                 const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                                 bf16_t* __restrict__ y, long ldy, float* __restrict__ mean_out,
                                                                 float* __restrict__ rstd_out, int M, int D, float eps,
                                                                 const bf16_t* __restrict__ down, long w_goff, int G,
                                                                 bf16_t* __restrict__ ds, long ldds, float alpha) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lnl_tile[];  // [16][D + 8]
  __shared__ __attribute__((aligned(16))) floatx4 red[4][LNL_MAXG][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g4 = lane >> 4, j = lane & 15;
  const int TS = D + 8;  // padded row (bf16): 16-B offset per row spreads the fragment reads over the banks
  const int nch = D >> 3;
  const long row0 = (long)blockIdx.x * 16;
  // the wave's 4 rows loaded up front (one memory latency for all of them), then normalised one by one
  uint4 raw[4][MAXC];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const long row = row0 + wid * 4 + rr;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      raw[rr][i] = row < M && c < nch ? *reinterpret_cast<const uint4*>(x + row * ldx + c * 8) : make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int lr = wid * 4 + rr;  // tile row
    const long row = row0 + lr;
    bf16_t* trow = lnl_tile + lr * TS;
    if (row >= M) {  // past the end: zeros (their projections are never stored)
      for (int c = lane; c < nch; c += 64) *reinterpret_cast<uint4*>(trow + c * 8) = make_uint4(0, 0, 0, 0);
      continue;
    }
    float f[MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        unpack8(raw[rr][i], f[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) s += f[i][e];
      }
    }
    const float mean = wave_sum(s) / (float)D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      if (lane + 64 * i < nch) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = f[i][e] - mean;
          ss += d * d;
        }
      }
    }
    const float r = rsqrtf(wave_sum(ss) / (float)D + eps);
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float wf[8], bf[8], o[8];
        unpack8(*reinterpret_cast<const uint4*>(w + c * 8), wf);
        unpack8(*reinterpret_cast<const uint4*>(b + c * 8), bf);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (f[i][e] - mean) * r * wf[e] + bf[e];
        const uint4 pk = pack8(o);
        *reinterpret_cast<uint4*>(y + row * ldy + c * 8) = pk;
        *reinterpret_cast<uint4*>(trow + c * 8) = pk;
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = r;
    }
  }
  __syncthreads();
  // projections: wave wid takes K chunks wid, wid + 4, ... (<= 4 of them: D <= 2048)
  const int nkc = D / LNL_KC;
  const int ncw = (nkc - wid + 3) / 4;
  for (int gi = 0; gi < G; ++gi) {
    const bf16_t* wr = down + gi * w_goff + (long)j * D + 8 * g4;  // down_gi row j
    uint4 wb[4][LNL_KC / 32];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < ncw)
#pragma unroll
        for (int s2 = 0; s2 < LNL_KC / 32; ++s2)
          wb[u][s2] = *reinterpret_cast<const uint4*>(wr + (wid + 4 * u) * LNL_KC + 32 * s2);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < ncw) {
        const int c = wid + 4 * u;
#pragma unroll
        for (int s2 = 0; s2 < LNL_KC / 32; ++s2) {
          const uint4 xa = *reinterpret_cast<const uint4*>(lnl_tile + j * TS + c * LNL_KC + 32 * s2 + 8 * g4);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(xa), as_frag(wb[u][s2]), acc, 0, 0, 0);
        }
      }
    red[wid][gi][lane] = acc;
  }
  __syncthreads();
  if (wid != 0) return;
  for (int gi = 0; gi < G; ++gi) {
    floatx4 acc = red[0][gi][lane];
#pragma unroll
    for (int w2 = 1; w2 < 4; ++w2) acc += red[w2][gi][lane];
    // D[m][j]: lane holds rows 4 g4 .. 4 g4 + 3 of the 16, column j
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long m = row0 + 4 * g4 + r;
      if (m < M) ds[m * ldds + 16 * gi + j] = f2bf(acc[r] * alpha);
    }
  }
}

// dx = dres + rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * w; per-block partials of
// dw = sum dy * xhat and db = sum dy (reduced by vpt_reduce_rows).
__global__ __launch_bounds__(256) void layernorm_bwd_kernel(const bf16_t* __restrict__ dy, long lddy,
                                                            const bf16_t* __restrict__ x, long ldx,
                                                            const float* __restrict__ mean_in,
                                                            const float* __restrict__ rstd_in,
                                                            const bf16_t* __restrict__ w,
                                                            const bf16_t* __restrict__ dres, long ldr,
                                                            bf16_t* __restrict__ dx, long lddx,
                                                            float* __restrict__ dw_part, float* __restrict__ db_part,
                                                            int M, int D) {
  __shared__ float red[4][2048];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = D >> 3;
  float dwp[MAXC][8], dbp[MAXC][8], wf[MAXC][8];
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + 64 * i;
#pragma unroll
    for (int e = 0; e < 8; ++e) dwp[i][e] = dbp[i][e] = 0.f;
    if (c < nch) unpack8(*reinterpret_cast<const uint4*>(w + c * 8), wf[i]);
  }
  for (long row = (long)blockIdx.x * 4 + wid; row < M; row += (long)gridDim.x * 4) {
    const float mu = mean_in[row], r = rstd_in[row];
    float xh[MAXC][8], gg[MAXC][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float fx[8], fd[8];
        unpack8(*reinterpret_cast<const uint4*>(x + row * ldx + c * 8), fx);
        unpack8(*reinterpret_cast<const uint4*>(dy + row * lddy + c * 8), fd);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[i][e] = (fx[e] - mu) * r;
          gg[i][e] = fd[e] * wf[i][e];
          sg += gg[i][e];
          sgx += gg[i][e] * xh[i][e];
          dwp[i][e] += fd[e] * xh[i][e];
          dbp[i][e] += fd[e];
        }
      }
    }
    const float mg = wave_sum(sg) / (float)D, mgx = wave_sum(sgx) / (float)D;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[8], fr[8];
        if (dres) unpack8(*reinterpret_cast<const uint4*>(dres + row * ldr + c * 8), fr);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = r * (gg[i][e] - mg - xh[i][e] * mgx);
          o[e] = dres ? fr[e] + bf2f(f2bf(d)) : d;  // residual and norm branch grads are bf16 tensors
        }
        *reinterpret_cast<uint4*>(dx + row * lddx + c * 8) = pack8(o);
      }
    }
  }
  // dw then db partials, each reduced across the 4 waves through LDS
  for (int pass = 0; pass < 2; ++pass) {
    float* dst = pass == 0 ? dw_part : db_part;
    if (!dst) continue;
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch)
#pragma unroll
        for (int e = 0; e < 8; ++e) red[wid][c * 8 + e] = pass == 0 ? dwp[i][e] : dbp[i][e];
    }
    __syncthreads();
    for (int d = threadIdx.x; d < D; d += 256)
      dst[(long)blockIdx.x * D + d] = red[0][d] + red[1][d] + red[2][d] + red[3][d];
    __syncthreads();
  }
}

// LayerNorm backward (frozen affine weights: no dw / db partials) and, in the same launch, the rank-16 LoRA
// up-side projection of its output -- vs[m][j] = bf16(alpha * dx[m] . up[:, j]), up [D][16]: the input-gradient
// operand of the LoRALinear that consumes dx as its output gradient (attn1.to_out.0 after norm2, attn2.to_out.0
// after norm3). 16 rows per block: every wave computes 4 rows exactly as layernorm_bwd_kernel (same arithmetic) into
// dx and an LDS image; each 128-row chunk of up is transposed through the wave's LDS image (as lora_proj's up
// path); the projection then runs in lora_proj's order (wave w: 128-wide K chunks w, w + 4, ...; four 16x16x32 MFMAs per chunk; waves summed in order)
// -- dx and vs bit-identical to vpt_layernorm_bwd + vpt_lora_proj(w_kmajor = 0).
template <int NC>  // 16-B chunks per lane: D <= 512 NC
__global__ __launch_bounds__(256) void layernorm_bwd_lora_kernel(const bf16_t* __restrict__ dy, long lddy,
                                                                 const bf16_t* __restrict__ x, long ldx,
                                                                 const float* __restrict__ mean_in,
                                                                 const float* __restrict__ rstd_in,
                                                                 const bf16_t* __restrict__ w,
                                                                 const bf16_t* __restrict__ dres, long ldr,
                                                                 bf16_t* __restrict__ dx, long lddx, int M, int D,
                                                                 const bf16_t* __restrict__ up, bf16_t* __restrict__ vs,
                                                                 long ldvs, float alpha) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lbl_smem[];  // tile [16][D + 8]
  __shared__ __attribute__((aligned(16))) bf16_t wsa[4][16 * (LNL_KC + 8)];  // per-wave transposed up chunk
  __shared__ __attribute__((aligned(16))) floatx4 red[4][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g4 = lane >> 4, j = lane & 15;
  const int TS = D + 8;
  bf16_t* tile = lbl_smem;
  bf16_t* ws = wsa[wid];
  const int nch = D >> 3;
  const long row0 = (long)blockIdx.x * 16;
  // the wave's four rows of x / dy (/ dres) in flight before any arithmetic (one block = 16 rows = 1 wave per SIMD:
  // latency, not bandwidth, bounds a row at a time)
  uint4 rx[4][NC], rd[4][NC], rr_[4][NC];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long row = row0 + wid * 4 + q;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + 64 * i;
      if (row < M && c < nch) {
        rx[q][i] = *reinterpret_cast<const uint4*>(x + row * ldx + c * 8);
        rd[q][i] = *reinterpret_cast<const uint4*>(dy + row * lddy + c * 8);
        if (dres) rr_[q][i] = *reinterpret_cast<const uint4*>(dres + row * ldr + c * 8);
      }
    }
  }
  float wf[NC][8];
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) unpack8(*reinterpret_cast<const uint4*>(w + c * 8), wf[i]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int lr = wid * 4 + q;
    const long row = row0 + lr;
    bf16_t* trow = tile + lr * TS;
    if (row >= M) {
      for (int c = lane; c < nch; c += 64) *reinterpret_cast<uint4*>(trow + c * 8) = make_uint4(0, 0, 0, 0);
      continue;
    }
    const float mu = mean_in[row], r = rstd_in[row];
    float xh[NC][8], gg[NC][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float fx[8], fd[8];
        unpack8(rx[q][i], fx);
        unpack8(rd[q][i], fd);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[i][e] = (fx[e] - mu) * r;
          gg[i][e] = fd[e] * wf[i][e];
          sg += gg[i][e];
          sgx += gg[i][e] * xh[i][e];
        }
      }
    }
    const float mg = wave_sum(sg) / (float)D, mgx = wave_sum(sgx) / (float)D;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[8], fr[8];
        if (dres) unpack8(rr_[q][i], fr);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = r * (gg[i][e] - mg - xh[i][e] * mgx);
          o[e] = dres ? fr[e] + bf2f(f2bf(d)) : d;
        }
        const uint4 pk = pack8(o);
        *reinterpret_cast<uint4*>(dx + row * lddx + c * 8) = pk;
        *reinterpret_cast<uint4*>(trow + c * 8) = pk;
      }
    }
  }
  __syncthreads();
  const int ncw = (D / LNL_KC - wid + 3) / 4;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int u = 0; u < ncw; ++u) {
    const int c = wid + 4 * u;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // up rows c*128 + kr, kr < 128 -> ws [16][128 + 8] (lora_proj's up path)
      const int kr = lane + 64 * h;
      const uint4 a0 = *reinterpret_cast<const uint4*>(up + (long)(c * LNL_KC + kr) * 16);
      const uint4 a1 = *reinterpret_cast<const uint4*>(up + (long)(c * LNL_KC + kr) * 16 + 8);
      const uint32_t v[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ws[(2 * e) * (LNL_KC + 8) + kr] = (bf16_t)(v[e] & 0xffff);
        ws[(2 * e + 1) * (LNL_KC + 8) + kr] = (bf16_t)(v[e] >> 16);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s2 = 0; s2 < LNL_KC / 32; ++s2) {
      const uint4 xa = *reinterpret_cast<const uint4*>(tile + j * TS + c * LNL_KC + 32 * s2 + 8 * g4);
      const uint4 wb = *reinterpret_cast<const uint4*>(ws + j * (LNL_KC + 8) + 32 * s2 + 8 * g4);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(xa), as_frag(wb), acc, 0, 0, 0);
    }
  }
  red[wid][lane] = acc;
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int w2 = 1; w2 < 4; ++w2) acc += red[w2][lane];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const long m = row0 + 4 * g4 + r;
    if (m < M) vs[m * ldvs + j] = f2bf(acc[r] * alpha);
  }
}

// ---------------------------------------------------------------- GeGLU
__device__ __forceinline__ float rbf(float v) { return bf2f(f2bf(v)); }
__device__ __forceinline__ float gelu_erf(float g) { return 0.5f * g * (1.f + erff(g * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_erf_grad(float g) {  // d/dg gelu = cdf + g * pdf (torch GeluBackward)
  const float cdf = 0.5f * (1.f + erff(g * 0.70710678118654752f));
  const float pdf = __expf(-0.5f * g * g) * 0.3989422804014327f;
  return cdf + g * pdf;
}
// gelu_erf(g) and gelu_erf_grad(g) from ONE erff (hipcc does not merge the two calls: 3 exponentials per element
// instead of 2 in the GeGLU backward) -- the same operations, so the same values.
__device__ __forceinline__ void gelu_erf_both(float g, float& gelu, float& grad) {
  const float e = erff(g * 0.70710678118654752f);
  gelu = 0.5f * g * (1.f + e);
  const float cdf = 0.5f * (1.f + e);
  const float pdf = __expf(-0.5f * g * g) * 0.3989422804014327f;
  grad = cdf + g * pdf;
}

// out[m][j] = h * gelu(gate), h = x12[m][j], gate = x12[m][F + j] (chunk(2, -1) order), bf16 tensors:
// out = bf16(h * bf16(gelu(gate))).
__global__ void geglu_fwd_kernel(const bf16_t* __restrict__ x12, long ldx, int F, long M, bf16_t* __restrict__ out) {
  const int nch = F >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= M * nch) return;
  const long m = gid / nch;
  const int c = gid % nch;
  float h[8], g[8], o[8];
  unpack8(*reinterpret_cast<const uint4*>(x12 + m * ldx + c * 8), h);
  unpack8(*reinterpret_cast<const uint4*>(x12 + m * ldx + F + c * 8), g);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = h[e] * rbf(gelu_erf(g[e]));
  *reinterpret_cast<uint4*>(out + m * (long)F + c * 8) = pack8(o);
}

// Autograd of the bf16 graph: dh = bf16(dy * bf16(gelu(g))), dgate = bf16(bf16(dy * h) * gelu'(g)).
__global__ void geglu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x12, long ldx, int F, long M,
                                 bf16_t* __restrict__ dx12, long lddx) {
  const int nch = F >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= M * nch) return;
  const long m = gid / nch;
  const int c = gid % nch;
  float d[8], h[8], g[8], oh[8], og[8];
  unpack8(*reinterpret_cast<const uint4*>(dy + m * (long)F + c * 8), d);
  unpack8(*reinterpret_cast<const uint4*>(x12 + m * ldx + c * 8), h);
  unpack8(*reinterpret_cast<const uint4*>(x12 + m * ldx + F + c * 8), g);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float ge, gd;
    gelu_erf_both(g[e], ge, gd);
    oh[e] = d[e] * rbf(ge);
    og[e] = rbf(d[e] * h[e]) * gd;
  }
  *reinterpret_cast<uint4*>(dx12 + m * lddx + c * 8) = pack8(oh);
  *reinterpret_cast<uint4*>(dx12 + m * lddx + F + c * 8) = pack8(og);
}

// GeGLU backward (as geglu_bwd_kernel: bit-identical dx12) and, in the same launch, the rank-16 LoRA projection of
// its output through the up of the Linear that produced x12 (ff.net.0.proj): vs[m][j] = bf16(alpha * dx12[m] .
// up[:, j]), up [2F][16] -- the input-gradient operand of that Linear's backward, without re-reading dx12 (2F wide).
// Work unit = 16 rows x one 128-column chunk pair c (columns [128c, +128) of dh and of dgate), one per wave; a block
// is GBW waves = GBW consecutive chunk pairs of one 16-row block, so a launch is (M / 16) x (F / 128 / GBW) small
// blocks that the dispatcher spreads evenly. (The form with one 16-wave block per 16 rows ran its 264 blocks of
// config 5's bucketed M = 4224 as two rounds on 256 CUs: 72 us, 48 us at M = 4096; r06tail.) Each lane computes
// exactly the 8 elements of its MFMA A fragment (row lane & 15, columns 32s + 8 (lane >> 4) of k step s), so dx12
// goes from registers to memory and into the MFMAs with no LDS image; both halves' up rows are loaded with the
// chunk and transposed in turn through the wave's LDS image as in lora_proj. Reduction over the chunk pairs: the
// block's waves meet in LDS in wave order, the block writes its 16 x 16 f32 partial (write-through), and the block
// of the row block that arrives last (ticket counter, guide 'In-launch split-K reduction', sc1 form) sums the
// partials in block order, writes vs and resets the counter -- deterministic for any placement; a different f32
// summation order than vpt_lora_proj (within bf16 rounding of it).
constexpr int GBW = 4;
constexpr int GBP = 136;  // padded transposed-up row (bf16)
#ifndef VPT_GB_ABL
#define VPT_GB_ABL 0  // timing ablations (lib variants only, wrong results): 1 = every chunk reads up rows 0..255
#endif
#ifndef VPT_GF_COAL
#define VPT_GF_COAL 1  // 1: geglu_fwd_lora moves x12 / out in row segments, A fragments through LDS (0: fragment-direct)
#endif
#ifndef VPT_GB_COAL
#define VPT_GB_COAL 1  // 1: geglu_bwd_lora moves dy / x12 / dx12 in row segments, A fragments through LDS (0: fragment-direct)
#endif
#ifndef VPT_GB_UG_LATE
#define VPT_GB_UG_LATE 0  // A/B: the dgate half's up rows loaded after the dh half's MFMAs (fewer VGPRs)
#endif

// up rows [r0, r0 + 128) ([K][16]): lane's two rows (lane, lane + 64), 32 B each
struct UpRows {
  uint4 v[2][2];
};
__device__ __forceinline__ UpRows gb_up_load(const bf16_t* __restrict__ up, long r0, int lane) {
  UpRows u;
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const bf16_t* ur = up + (r0 + lane + 64 * hh) * 16;
    u.v[hh][0] = *reinterpret_cast<const uint4*>(ur);
    u.v[hh][1] = *reinterpret_cast<const uint4*>(ur + 8);
  }
  return u;
}
// ... -> the wave's image ws [16][GBP]
__device__ __forceinline__ void gb_up_store(const UpRows& u, bf16_t* ws, int lane) {
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    const int kr = lane + 64 * hh;
    const uint32_t v[8] = {u.v[hh][0].x, u.v[hh][0].y, u.v[hh][0].z, u.v[hh][0].w,
                           u.v[hh][1].x, u.v[hh][1].y, u.v[hh][1].z, u.v[hh][1].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ws[(2 * e) * GBP + kr] = (bf16_t)(v[e] & 0xffff);
      ws[(2 * e + 1) * GBP + kr] = (bf16_t)(v[e] >> 16);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
  __builtin_amdgcn_wave_barrier();
}

// The in-launch reduction of a row block's chunk partials (geglu_bwd_lora / geglu_fwd_lora): the block's GBW waves
// meet in LDS in wave order, wave 0 writes the block's 16 x 16 f32 partial (sc1 store: write-through, visible to a
// reducer on any XCD) to part[rb][b] and counts it in on the row block's ticket (guide 'In-launch split-K reduction',
// sc1 form); the block that draws the last ticket resets it and returns true, its wave 0 holding in s the nb partials
// summed in block order (sc1 loads) -- deterministic for any placement. Other blocks / waves return false.
__device__ __forceinline__ bool rowblock_reduce(floatx4 acc, floatx4 (&red)[GBW][64], float* __restrict__ part,
                                                unsigned* __restrict__ cnt, int rb, int b, int nb, int wid, int lane,
                                                floatx4& s) {
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
  red[wid][lane] = acc;
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      part + (long)rb * nb * 256, (short)0, nb * 1024, 0x00020000);
  if (wid == 0) {
#pragma unroll
    for (int w2 = 1; w2 < GBW; ++w2) acc += red[w2][lane];
    __builtin_amdgcn_raw_buffer_store_b128(
        u32x4_t{__float_as_uint(acc[0]), __float_as_uint(acc[1]), __float_as_uint(acc[2]), __float_as_uint(acc[3])},
        rs, lane * 16 + b * 1024, 0, 16);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1");  // the store's data registers stay untouched after issue (store_b128_padded)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial is in memory before the ticket
  }
  __syncthreads();
  int* flag = reinterpret_cast<int*>(&red[0][0]);  // red is consumed
  if (threadIdx.x == 0)
    *flag = __hip_atomic_fetch_add(cnt + rb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(nb - 1);
  __syncthreads();
  if (!*flag || wid != 0) return false;
  if (lane == 0) __hip_atomic_store(cnt + rb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
  // block order, 8 partials per round trip; offsets past the row block's nb partials read 0 (buffer range check)
  // and add exact zeros after the last one
  for (int b0 = 0; b0 < nb; b0 += 8) {
    u32x4_t u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + (b0 + k) * 1024, 0, 16);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const floatx4 v = {__uint_as_float(u[k][0]), __uint_as_float(u[k][1]), __uint_as_float(u[k][2]),
                         __uint_as_float(u[k][3])};
      s = (b0 + k == 0) ? v : s + v;
    }
  }
  return true;
}

// part: [M / 16 * nb][64] floatx4 block partials; cnt: [M / 16] tickets, zero on entry and on exit
__global__ __launch_bounds__(64 * GBW) void geglu_bwd_lora_kernel(const bf16_t* __restrict__ dy,
                                                                 const bf16_t* __restrict__ x12, long ldx, int F, int M,
                                                                 bf16_t* __restrict__ dx12, long lddx,
                                                                 const bf16_t* __restrict__ up, bf16_t* __restrict__ vs,
                                                                 long ldvs, float alpha, float* __restrict__ part,
                                                                 unsigned* __restrict__ cnt) {
  __shared__ __attribute__((aligned(16))) bf16_t wsa[GBW][16 * GBP];
  __shared__ __attribute__((aligned(16))) floatx4 red[GBW][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g4 = lane >> 4, i = lane & 15;
  bf16_t* ws = wsa[wid];
  const int nchp = F / 128, nb = (nchp + GBW - 1) / GBW;
  const int rb = blockIdx.x / nb, b = blockIdx.x - rb * nb;
  const long row0 = (long)rb * 16;
  const long row = row0 + i;
  const bool row_ok = row < M;
  const long rowc = row_ok ? row : (long)M - 1;
  const int c = b * GBW + wid;  // this wave's chunk pair
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#if VPT_GB_COAL
  // dy / x12 / dx12 moved in full 256-B row segments (16 lanes per row, 4 rows per instruction); the A fragments read
  // back from an LDS image of the wave's 16 x 128 dh tile, then of its dgate tile (same image, same MFMA order)
  __shared__ __attribute__((aligned(16))) bf16_t gbt[GBW][16 * GBP];
  if (c < nchp) {
    bf16_t* t = gbt[wid];
    const int lr = lane >> 4, lc = (lane & 15) * 8;
    const UpRows uh = gb_up_load(up, VPT_GB_ABL == 1 ? 0L : (long)c * 128, lane);      // the dh half's up rows
    const UpRows ug = gb_up_load(up, VPT_GB_ABL == 1 ? 128L : (long)F + c * 128, lane);  // the dgate half's
    uint4 d[4], h[4], gt[4], pg[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long r = row0 + 4 * q + lr;
      const long rc = r < M ? r : (long)M - 1;
      d[q] = *reinterpret_cast<const uint4*>(dy + rc * F + c * 128 + lc);
      h[q] = *reinterpret_cast<const uint4*>(x12 + rc * ldx + c * 128 + lc);
      gt[q] = *reinterpret_cast<const uint4*>(x12 + rc * ldx + F + c * 128 + lc);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long r = row0 + 4 * q + lr;
      float fd[8], fh[8], fg[8], oh[8], og[8];
      unpack8(d[q], fd);
      unpack8(h[q], fh);
      unpack8(gt[q], fg);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float ge, gd;
        gelu_erf_both(fg[e], ge, gd);
        oh[e] = fd[e] * rbf(ge);
        og[e] = rbf(fd[e] * fh[e]) * gd;
      }
      const uint4 ph = pack8(oh);
      pg[q] = pack8(og);
      if (r < M) {
        *reinterpret_cast<uint4*>(dx12 + r * lddx + c * 128 + lc) = ph;
        *reinterpret_cast<uint4*>(dx12 + r * lddx + F + c * 128 + lc) = pg[q];
      }
      *reinterpret_cast<uint4*>(t + (4 * q + lr) * GBP + lc) = ph;
    }
    gb_up_store(uh, ws, lane);  // its lgkmcnt(0) wait also lands the dh tile
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const uint4 a = *reinterpret_cast<const uint4*>(t + i * GBP + 32 * s2 + 8 * g4);
      const uint4 bh = *reinterpret_cast<const uint4*>(&ws[i * GBP + 32 * s2 + 8 * g4]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(bh), acc, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<uint4*>(t + (4 * q + lr) * GBP + lc) = pg[q];
    gb_up_store(ug, ws, lane);  // ... and the dgate tile
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const uint4 a = *reinterpret_cast<const uint4*>(t + i * GBP + 32 * s2 + 8 * g4);
      const uint4 bg = *reinterpret_cast<const uint4*>(&ws[i * GBP + 32 * s2 + 8 * g4]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(bg), acc, 0, 0, 0);
    }
  }
#else
  if (c < nchp) {
    const bf16_t* dyr = dy + rowc * F + 8 * g4;
    const bf16_t* xr = x12 + rowc * ldx + 8 * g4;
    bf16_t* dxr = dx12 + rowc * lddx + 8 * g4;
    const UpRows uh = gb_up_load(up, VPT_GB_ABL == 1 ? 0L : (long)c * 128, lane);      // the dh half's up rows
#if !VPT_GB_UG_LATE
    const UpRows ug = gb_up_load(up, VPT_GB_ABL == 1 ? 128L : (long)F + c * 128, lane);  // the dgate half's
#endif
    uint4 d[4], h[4], gt[4], pg[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int col = c * 128 + 32 * s2;
      d[s2] = *reinterpret_cast<const uint4*>(dyr + col);
      h[s2] = *reinterpret_cast<const uint4*>(xr + col);
      gt[s2] = *reinterpret_cast<const uint4*>(xr + F + col);
    }
    gb_up_store(uh, ws, lane);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      float fd[8], fh[8], fg[8], oh[8], og[8];
      unpack8(d[s2], fd);
      unpack8(h[s2], fh);
      unpack8(gt[s2], fg);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float ge, gd;
        gelu_erf_both(fg[e], ge, gd);
        oh[e] = fd[e] * rbf(ge);
        og[e] = rbf(fd[e] * fh[e]) * gd;
      }
      const uint4 ph = pack8(oh);
      pg[s2] = pack8(og);
      const int col = c * 128 + 32 * s2;
      if (row_ok) {
        *reinterpret_cast<uint4*>(dxr + col) = ph;
        *reinterpret_cast<uint4*>(dxr + F + col) = pg[s2];
      }
      const uint4 bh = *reinterpret_cast<const uint4*>(&ws[i * GBP + 32 * s2 + 8 * g4]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(ph), as_frag(bh), acc, 0, 0, 0);
    }
#if VPT_GB_UG_LATE
    const UpRows ug = gb_up_load(up, VPT_GB_ABL == 1 ? 128L : (long)F + c * 128, lane);
#endif
    gb_up_store(ug, ws, lane);
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const uint4 bg = *reinterpret_cast<const uint4*>(&ws[i * GBP + 32 * s2 + 8 * g4]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(pg[s2]), as_frag(bg), acc, 0, 0, 0);
    }
  }
#endif
  floatx4 s;
  if (!rowblock_reduce(acc, red, part, cnt, rb, b, nb, wid, lane, s)) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const long m = row0 + 4 * g4 + r;
    if (m < M) vs[m * ldvs + i] = f2bf(s[r] * alpha);
  }
}

// GeGLU forward (as geglu_fwd_kernel: bit-identical out) and, in the same launch, the rank-16 LoRA down-projection of
// its output for the Linear that consumes it (ff.net.2): ds[m][j] = bf16(alpha * out[m] . down[j, :]), down [16][F]
// -- that Linear's forward operand, without re-reading out. Work unit = 16 rows x one 128-column chunk, one per wave,
// GBW consecutive chunks per block; each lane computes exactly the 8 outputs of its MFMA A fragment, and its B
// fragment is 16 B of down row (lane & 15) straight from memory (k-major: no LDS image). The chunks' partials meet as
// in geglu_bwd_lora (rowblock_reduce: fixed order; a different f32 summation order than vpt_lora_proj).
__global__ __launch_bounds__(64 * GBW) void geglu_fwd_lora_kernel(const bf16_t* __restrict__ x12, long ldx, int F,
                                                                 int M, bf16_t* __restrict__ out, long ldo,
                                                                 const bf16_t* __restrict__ down,
                                                                 bf16_t* __restrict__ ds, long ldds, float alpha,
                                                                 float* __restrict__ part,
                                                                 unsigned* __restrict__ cnt) {
  __shared__ __attribute__((aligned(16))) floatx4 red[GBW][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g4 = lane >> 4, i = lane & 15;
  const int nch = F / 128, nb = (nch + GBW - 1) / GBW;
  const int rb = blockIdx.x / nb, b = blockIdx.x - rb * nb;
  const long row0 = (long)rb * 16;
  const long row = row0 + i;
  const bool row_ok = row < M;
  const long rowc = row_ok ? row : (long)M - 1;
  const int c = b * GBW + wid;  // this wave's chunk
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#if VPT_GF_COAL
  // x12 / out moved in full 256-B row segments (16 lanes per row, 4 rows per instruction) and the A fragments
  // read back from an LDS image of the wave's 16 x 128 output tile
  __shared__ __attribute__((aligned(16))) bf16_t gft[GBW][16 * GBP];
  if (c < nch) {
    bf16_t* t = gft[wid];
    const int lr = lane >> 4, lc = (lane & 15) * 8;
    const bf16_t* dr = down + (long)i * F + c * 128 + 8 * g4;
    uint4 h[4], gt[4], wd[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long r = row0 + 4 * q + lr;
      const bf16_t* xr = x12 + (r < M ? r : (long)M - 1) * ldx + c * 128 + lc;
      h[q] = *reinterpret_cast<const uint4*>(xr);
      gt[q] = *reinterpret_cast<const uint4*>(xr + F);
      wd[q] = *reinterpret_cast<const uint4*>(dr + 32 * q);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const long r = row0 + 4 * q + lr;
      float fh[8], fg[8], o[8];
      unpack8(h[q], fh);
      unpack8(gt[q], fg);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fh[e] * rbf(gelu_erf(fg[e]));
      const uint4 po = pack8(o);
      if (r < M) *reinterpret_cast<uint4*>(out + r * ldo + c * 128 + lc) = po;
      *reinterpret_cast<uint4*>(t + (4 * q + lr) * GBP + lc) = po;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const uint4 a = *reinterpret_cast<const uint4*>(t + i * GBP + 32 * s2 + 8 * g4);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(a), as_frag(wd[s2]), acc, 0, 0, 0);
    }
  }
#else
  if (c < nch) {
    const bf16_t* xr = x12 + rowc * ldx + c * 128 + 8 * g4;
    const bf16_t* dr = down + (long)i * F + c * 128 + 8 * g4;
    bf16_t* orow = out + rowc * ldo + c * 128 + 8 * g4;
    uint4 h[4], gt[4], wd[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      h[s2] = *reinterpret_cast<const uint4*>(xr + 32 * s2);
      gt[s2] = *reinterpret_cast<const uint4*>(xr + F + 32 * s2);
      wd[s2] = *reinterpret_cast<const uint4*>(dr + 32 * s2);
    }
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      float fh[8], fg[8], o[8];
      unpack8(h[s2], fh);
      unpack8(gt[s2], fg);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = fh[e] * rbf(gelu_erf(fg[e]));
      const uint4 po = pack8(o);
      if (row_ok) *reinterpret_cast<uint4*>(orow + 32 * s2) = po;
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(po), as_frag(wd[s2]), acc, 0, 0, 0);
    }
  }
#endif
  floatx4 s;
  if (!rowblock_reduce(acc, red, part, cnt, rb, b, nb, wid, lane, s)) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const long m = row0 + 4 * g4 + r;
    if (m < M) ds[m * ldds + i] = f2bf(s[r] * alpha);
  }
}

// ---------------------------------------------------------------- NF4
__constant__ float kNF4[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                               -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                               0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                               0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                               0.7229568362236023f, 1.0f};

// W[i] = NF4[code_i] * absmax[i / 64], absmax[j] = code2[qabsmax[j]] * absmax2[j / 256] + offset (bnb's
// dequantize_blockwise of the nested absmax, then `absmax += offset`: a product and a sum, each rounded -- no
// FMA); bf16 output in the original [out][in] layout, ready as the B operand of the GEMM. Byte -> (NF4[hi],
// NF4[lo]) from a 256-entry LDS table (nf4_dequant_dwords below). HBM-bound: 0.5 B in + 2 B out per weight.
__device__ __forceinline__ float nf4_absmax(float c2, float a2, float off) {
#pragma clang fp contract(off)
  return c2 * a2 + off;
}

struct Nf4Batch {
  VptNf4Job job[16];
  long block0[17];  // first block of each job (prefix over ceil(n / 8192): 1,024 packed dwords per block)
  int njobs;
};

// A block dequantises 1,024 consecutive packed dwords (8 weights each) of one tensor: thread t takes dwords
// t, t + 256, t + 512, t + 768 of the block's range, so every load instruction reads 256 contiguous bytes and every
// 16-B store instruction writes 1 KB contiguously (one chunk of 16 packed bytes per thread wrote four 16-B pieces 64 B
// apart per instruction: 23.1 -> 15.8 us per C5 batch launch). The nested-absmax code table and offset are staged in
// LDS with the NF4 pair table (c2s, offs: filled by the caller before its barrier).
// The packed words and their absmax codes are loaded BEFORE the block fills its LDS tables (nf4_dq_load), so the table
// fill's own global read (code2) and its barrier overlap them: one memory round trip per block instead of two.
struct Nf4Regs4 {
  uint32_t w[4];
  uint8_t qv[4];
  float a2[4];
};
__device__ __forceinline__ Nf4Regs4 nf4_dq_load(const uint32_t* __restrict__ pk, const uint8_t* __restrict__ qa,
                                                const float* __restrict__ absmax2, long ndw, long d0) {
  Nf4Regs4 r;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long d = d0 + 256 * q;
    r.w[q] = d < ndw ? pk[d] : 0u;
    r.qv[q] = d < ndw ? qa[d >> 3] : 0;            // absmax block of 64 weights = 8 dwords
    r.a2[q] = d < ndw ? absmax2[d >> 11] : 0.f;   // absmax2 per 256 blocks = 2,048 dwords
  }
  return r;
}
__device__ __forceinline__ void nf4_dequant_dwords(const Nf4Regs4& r, const float* c2s, float off, const float2_t* lut,
                                                   long ndw, long d0, bf16_t* __restrict__ out) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long d = d0 + 256 * q;
    if (d >= ndw) break;
    const float am = nf4_absmax(c2s[r.qv[q]], r.a2[q], off);
    float v[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float2_t pr = lut[(r.w[q] >> (8 * k)) & 0xffu];  // first weight in the high nibble
      v[2 * k] = pr[0] * am;
      v[2 * k + 1] = pr[1] * am;
    }
    reinterpret_cast<uint4*>(out)[d] = pack8(v);
  }
}

__global__ __launch_bounds__(256) void nf4_dequant_batch_kernel(Nf4Batch b) {
  __shared__ float2_t lut[256];
  __shared__ float c2s[256];
  __shared__ float offs;
  int j = 0;
  while (j + 1 < b.njobs && (long)blockIdx.x >= b.block0[j + 1]) ++j;  // wave-uniform
  const VptNf4Job& jb = b.job[j];
  const long d0 = ((long)blockIdx.x - b.block0[j]) * 1024 + threadIdx.x;
  const Nf4Regs4 r = nf4_dq_load((const uint32_t*)jb.packed, (const uint8_t*)jb.qabsmax, jb.absmax2, jb.n / 8, d0);
  lut[threadIdx.x] = float2_t{kNF4[threadIdx.x >> 4], kNF4[threadIdx.x & 15]};
  c2s[threadIdx.x] = jb.code2[threadIdx.x];
  if (threadIdx.x == 0) offs = jb.offset[0];
  __syncthreads();
  nf4_dequant_dwords(r, c2s, offs, lut, jb.n / 8, d0, (bf16_t*)jb.out);
}

__global__ __launch_bounds__(256) void nf4_dequant_kernel(const uint8_t* __restrict__ packed,
                                                          const uint8_t* __restrict__ qabsmax,
                                                          const float* __restrict__ absmax2,
                                                          const float* __restrict__ code2,
                                                          const float* __restrict__ offset, long nchunks,
                                                          bf16_t* __restrict__ out) {
  __shared__ float2_t lut[256];
  __shared__ float c2s[256];
  __shared__ float offs;
  const long d0 = (long)blockIdx.x * 1024 + threadIdx.x;
  const Nf4Regs4 r = nf4_dq_load((const uint32_t*)packed, qabsmax, absmax2, nchunks * 4, d0);
  lut[threadIdx.x] = float2_t{kNF4[threadIdx.x >> 4], kNF4[threadIdx.x & 15]};
  c2s[threadIdx.x] = code2[threadIdx.x];
  if (threadIdx.x == 0) offs = offset[0];
  __syncthreads();
  nf4_dequant_dwords(r, c2s, offs, lut, nchunks * 4, d0, out);
}

// Pass 1 of quantize_4bit: per 64-block absmax (one wave per block), nearest NF4 code of w / absmax
// (first minimum of |v - code|, as argmin), packed pairs.
__global__ __launch_bounds__(256) void nf4_quant_kernel(const bf16_t* __restrict__ w, long nblocks,
                                                        uint8_t* __restrict__ packed, float* __restrict__ absmax) {
  const int lane = threadIdx.x & 63;
  const long blk = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (blk >= nblocks) return;
  const float v = bf2f(w[blk * 64 + lane]);
  const float am = wave_max(fabsf(v));
  const float sv = v / fmaxf(am, 1e-30f);
  int best = 0;
  float bd = fabsf(sv - kNF4[0]);
#pragma unroll
  for (int k = 1; k < 16; ++k) {
    const float d = fabsf(sv - kNF4[k]);
    if (d < bd) { bd = d; best = k; }
  }
  const int other = __shfl_xor(best, 1, 64);
  if ((lane & 1) == 0) packed[blk * 32 + (lane >> 1)] = (uint8_t)((best << 4) | other);
  if (lane == 0) absmax[blk] = am;
}

// Pass 2: offset = mean(absmax) (one block, fixed-order tree), then nested 8-bit blockwise
// quantisation of absmax - offset over the dynamic map (blocksize 256; nearest code, first minimum).
__global__ __launch_bounds__(256) void nf4_nested_kernel(const float* __restrict__ absmax, long nblocks,
                                                         const float* __restrict__ code2, uint8_t* __restrict__ qabsmax,
                                                         float* __restrict__ absmax2, float* __restrict__ offset) {
  __shared__ float red[256];
  __shared__ float code[256];
  __shared__ float off_s;
  const int tid = threadIdx.x;
  code[tid] = code2[tid];
  float s = 0.f;
  for (long j = tid; j < nblocks; j += 256) s += absmax[j];
  red[tid] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (tid < h) red[tid] += red[tid + h];
    __syncthreads();
  }
  if (tid == 0) {
    off_s = red[0] / (float)nblocks;
    offset[0] = off_s;
  }
  __syncthreads();
  const float off = off_s;
  const long nb2 = (nblocks + 255) / 256;
  for (long b2 = 0; b2 < nb2; ++b2) {
    const long j = b2 * 256 + tid;
    const float a = j < nblocks ? absmax[j] - off : 0.f;
    red[tid] = fabsf(a);
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (tid < h) red[tid] = fmaxf(red[tid], red[tid + h]);
      __syncthreads();
    }
    const float am2 = red[0];
    __syncthreads();
    if (tid == 0) absmax2[b2] = am2;
    if (j < nblocks) {
      const float sv = a / fmaxf(am2, 1e-30f);
      int best = 0;
      float bd = fabsf(sv - code[0]);
      for (int k = 1; k < 256; ++k) {
        const float d = fabsf(sv - code[k]);
        if (d < bd) { bd = d; best = k; }
      }
      qabsmax[j] = (uint8_t)best;
    }
  }
}

// ---------------------------------------------------------------- SpatialTransformer (denoiser.py:283-365)
// GroupNorm(32, C, eps 1e-6, affine) on the NCHW stage activation: one workgroup per (batch, group) -- a group
// is cpg * HW contiguous elements. f32 statistics (two passes: mean, then centred variance), output
// bf16((x - mean) * rstd * w[c] + b[c]) in NCHW; the transpose to tokens is transpose_add_kernel.
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int wid = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[wid] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void groupnorm_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ y,
                                                            float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                            int C, int G, long HW, float eps) {
  __shared__ float red[4];
  const int bg = blockIdx.x, g = bg % G, cpg = C / G;
  const long n = (long)cpg * HW;
  const long base = (long)bg * n;  // (b * C + g * cpg) * HW
  const int tid = threadIdx.x;
  float s = 0.f;
  for (long i = tid * 8L; i < n; i += 256 * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(x + base + i), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[e];
  }
  const float mean = block_sum256(s, red) / (float)n;
  float q = 0.f;
  for (long i = tid * 8L; i < n; i += 256 * 8) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(x + base + i), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) q += (v[e] - mean) * (v[e] - mean);
  }
  const float rstd = rsqrtf(block_sum256(q, red) / (float)n + eps);
  if (tid == 0) { mean_out[bg] = mean; rstd_out[bg] = rstd; }
  for (long i = tid * 8L; i < n; i += 256 * 8) {
    const int c = g * cpg + (int)(i / HW);  // HW % 8 == 0: the 8 elements share a channel
    const float wc = bf2f(w[c]) * rstd, bc = bf2f(bias[c]);
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(x + base + i), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (v[e] - mean) * wc + bc;
    *reinterpret_cast<uint4*>(y + base + i) = pack8(v);
  }
}

// dx = rstd * (g - (sum g + xh * sum g xh) / n) (+ dres), g = w[c] * dy, xh = (x - mean) * rstd, per group;
// NCHW in and out (the affine weights are frozen under QLoRA: no dw / db).
__global__ __launch_bounds__(256) void groupnorm_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                            const float* __restrict__ mean_in,
                                                            const float* __restrict__ rstd_in,
                                                            const bf16_t* __restrict__ w, const bf16_t* __restrict__ dres,
                                                            bf16_t* __restrict__ dx, int C, int G, long HW) {
  __shared__ float red[4];
  const int bg = blockIdx.x, g = bg % G, cpg = C / G;
  const long n = (long)cpg * HW;
  const long base = (long)bg * n;
  const int tid = threadIdx.x;
  const float mean = mean_in[bg], rstd = rstd_in[bg];
  float sg = 0.f, sgx = 0.f;
  for (long i = tid * 8L; i < n; i += 256 * 8) {
    const float wc = bf2f(w[g * cpg + (int)(i / HW)]);
    float d[8], v[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + base + i), d);
    unpack8(*reinterpret_cast<const uint4*>(x + base + i), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gg = wc * d[e];
      sg += gg;
      sgx += gg * (v[e] - mean) * rstd;
    }
  }
  const float mg = block_sum256(sg, red) / (float)n;
  const float mgx = block_sum256(sgx, red) / (float)n;
  for (long i = tid * 8L; i < n; i += 256 * 8) {
    const float wc = bf2f(w[g * cpg + (int)(i / HW)]);
    float d[8], v[8], r[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + base + i), d);
    unpack8(*reinterpret_cast<const uint4*>(x + base + i), v);
    if (dres) unpack8(*reinterpret_cast<const uint4*>(dres + base + i), r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float xh = (v[e] - mean) * rstd;
      v[e] = rstd * (wc * d[e] - mg - xh * mgx) + (dres ? r[e] : 0.f);
    }
    *reinterpret_cast<uint4*>(dx + base + i) = pack8(v);
  }
}

// dst[b][s][r] = src[b][r][s] (+ add[b][s][r]), bf16, 64 x 64 tiles through LDS: the NCHW <-> token-major
// permutes of SpatialTransformer.forward (denoiser.py:339-345, 356-363), the residual add fused. R and S are
// multiples of 8 (16-B chunks); edge tiles (aspect-ratio buckets: HW = 28 x 36 = 1008 tokens) guard by chunk.
__global__ __launch_bounds__(256) void transpose_add_kernel(const bf16_t* __restrict__ src, const bf16_t* __restrict__ add,
                                                            bf16_t* __restrict__ dst, int R, int S) {
  __shared__ float t[64][65];
  const int b = blockIdx.z, r0 = blockIdx.y * 64, s0 = blockIdx.x * 64, tid = threadIdx.x;
  const int nr = min(64, R - r0), ns = min(64, S - s0);
  const bf16_t* sb = src + (long)b * R * S;
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // 64 rows x 8 chunks of 8
    const int idx = tid + 256 * k, rr = idx >> 3, ch = idx & 7;
    float v[8];
    if (rr < nr && ch * 8 < ns) {
      unpack8(*reinterpret_cast<const uint4*>(sb + (long)(r0 + rr) * S + s0 + ch * 8), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) t[rr][ch * 8 + e] = v[e];
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int idx = tid + 256 * k, ss = idx >> 3, ch = idx & 7;
    if (ss >= ns || ch * 8 >= nr) continue;
    const long o = (long)b * R * S + (long)(s0 + ss) * R + r0 + ch * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = t[ch * 8 + e][ss];
    if (add) {
      float a[8];
      unpack8(*reinterpret_cast<const uint4*>(add + o), a);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(v[e])) + a[e];  // bf16 tensor + bf16 residual
    }
    *reinterpret_cast<uint4*>(dst + o) = pack8(v);
  }
}

inline dim3 grid1(long n, int threads = 256) { return dim3((unsigned)((n + threads - 1) / threads)); }

}  // namespace

extern "C" int vpt_layernorm_fwd(const void* x, long ldx, const void* w, const void* b, void* y, long ldy, float* mean,
                                 float* rstd, int M, int D, float eps, void* stream) {
  VPT_CHECK_ARG(x && w && b && y && mean && rstd, "vpt_layernorm_fwd: null pointer");
  VPT_CHECK_ARG(D % 8 == 0 && D <= 2048 && M >= 0, "vpt_layernorm_fwd: D must be a multiple of 8, <= 2048");
  if (M == 0) return VPT_OK;
  hipLaunchKernelGGL(layernorm_fwd_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     ldx, (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, ldy, mean, rstd, M, D, eps);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_layernorm_lora_fwd(const void* x, long ldx, const void* w, const void* b, void* y, long ldy,
                                      float* mean, float* rstd, int M, int D, float eps, const void* down, long w_goff,
                                      int G, void* ds, long ldds, float alpha, void* stream) {
  VPT_CHECK_ARG(x && w && b && y && mean && rstd && down && ds, "vpt_layernorm_lora_fwd: null pointer");
  VPT_CHECK_ARG(D % LNL_KC == 0 && D <= 2048 && M >= 0 && ldx % 8 == 0 && ldy % 8 == 0,
                "vpt_layernorm_lora_fwd: D % 128 == 0, D <= 2048, 16-B leading dims");
  VPT_CHECK_ARG(G >= 1 && G <= LNL_MAXG && ldds >= 16 * G && w_goff % 8 == 0, "vpt_layernorm_lora_fwd: 1..3 groups");
  if (M == 0) return VPT_OK;
  const size_t lds = (size_t)16 * (D + 8) * sizeof(bf16_t);
  hipLaunchKernelGGL(layernorm_lora_fwd_kernel, dim3((M + 15) / 16), dim3(256), lds, (hipStream_t)stream,
                     (const bf16_t*)x, ldx, (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, ldy, mean, rstd, M, D, eps,
                     (const bf16_t*)down, w_goff, G, (bf16_t*)ds, ldds, alpha);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_layernorm_bwd_blocks(int M) {
  const int b = (M + 3) / 4;
  return b < 512 ? (b < 1 ? 1 : b) : 512;
}

extern "C" int vpt_layernorm_bwd(const void* dy, long lddy, const void* x, long ldx, const float* mean,
                                 const float* rstd, const void* w, const void* dres, long ldr, void* dx, long lddx,
                                 float* dw_part, float* db_part, int M, int D, void* stream) {
  VPT_CHECK_ARG(dy && x && mean && rstd && w && dx, "vpt_layernorm_bwd: null pointer");
  VPT_CHECK_ARG(D % 8 == 0 && D <= 2048, "vpt_layernorm_bwd: D must be a multiple of 8, <= 2048");
  if (M == 0) return VPT_OK;
  hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(vpt_layernorm_bwd_blocks(M)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, mean, rstd, (const bf16_t*)w,
                     (const bf16_t*)dres, ldr, (bf16_t*)dx, lddx, dw_part, db_part, M, D);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_layernorm_bwd_lora(const void* dy, long lddy, const void* x, long ldx, const float* mean,
                                      const float* rstd, const void* w, const void* dres, long ldr, void* dx, long lddx,
                                      int M, int D, const void* up, void* vs, long ldvs, float alpha, void* stream) {
  VPT_CHECK_ARG(dy && x && mean && rstd && w && dx && up && vs, "vpt_layernorm_bwd_lora: null pointer");
  VPT_CHECK_ARG(D % LNL_KC == 0 && D <= 2048 && lddy % 8 == 0 && ldx % 8 == 0 && lddx % 8 == 0 && (!dres || ldr % 8 == 0)
                    && ldvs >= 16, "vpt_layernorm_bwd_lora: D % 128 == 0, D <= 2048, 16-B leading dims");
  if (M == 0) return VPT_OK;
  const size_t lds = (size_t)16 * (D + 8) * sizeof(bf16_t);
  const int nc = (D / 8 + 63) / 64;
  auto k = nc <= 2 ? layernorm_bwd_lora_kernel<2> : nc == 3 ? layernorm_bwd_lora_kernel<3> : layernorm_bwd_lora_kernel<4>;
  hipLaunchKernelGGL(k, dim3((M + 15) / 16), dim3(256), lds, (hipStream_t)stream, (const bf16_t*)dy, lddy,
                     (const bf16_t*)x, ldx, mean, rstd, (const bf16_t*)w, (const bf16_t*)dres, ldr, (bf16_t*)dx, lddx, M,
                     D, (const bf16_t*)up, (bf16_t*)vs, ldvs, alpha);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_geglu_fwd(const void* x12, long ldx, int F, long M, void* out, void* stream) {
  VPT_CHECK_ARG(x12 && out && F % 8 == 0 && ldx % 8 == 0, "vpt_geglu_fwd: bad args");
  if (M == 0) return VPT_OK;
  hipLaunchKernelGGL(geglu_fwd_kernel, grid1(M * (F / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x12, ldx,
                     F, M, (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

// Workspaces of vpt_geglu_bwd_lora / vpt_geglu_fwd_lora: tickets = (M + 15) / 16 u32 row-block counters, zero when
// allocated and left zero by every launch (a launch touches only its own row blocks' counters, so one zeroed buffer
// serves every shape); partials = vpt_geglu_lora_partials_bytes(M, F), uninitialised.
extern "C" long vpt_geglu_lora_partials_bytes(int M, int F) {
  if (M <= 0 || F <= 0) return 0;
  return (long)((M + 15) / 16) * ((F / 128 + GBW - 1) / GBW) * 1024;
}

namespace {
int geglu_lora_check(const char* fn, int F, int M, const void* tickets, const void* partials) {
  VPT_CHECK_ARG(tickets && partials, fn);
  VPT_CHECK_ARG(((uintptr_t)tickets & 3) == 0 && ((uintptr_t)partials & 15) == 0, fn);
  const long R = (M + 15) / 16, nb = (F / 128 + GBW - 1) / GBW;
  VPT_CHECK_ARG(R * nb < (1L << 31) && nb * 1024 < (1L << 30), fn);
  return VPT_OK;
}
}  // namespace

extern "C" int vpt_geglu_fwd_lora(const void* x12, long ldx, int F, int M, void* out, long ldo, const void* down,
                                  void* ds, long ldds, float alpha, void* tickets, void* partials, void* stream) {
  VPT_CHECK_ARG(x12 && out && down && ds, "vpt_geglu_fwd_lora: null pointer");
  VPT_CHECK_ARG(F > 0 && F % 128 == 0 && ldx % 8 == 0 && ldo % 8 == 0 && ldx >= 2L * F && ldo >= F && ldds >= 16,
                "vpt_geglu_fwd_lora: F % 128 == 0, 16-B leading dims (x12 >= 2F, out >= F)");
  if (M <= 0) return VPT_OK;
  if (int rc = geglu_lora_check("vpt_geglu_fwd_lora: tickets / partials (null, misaligned or too many blocks)", F, M,
                                tickets, partials))
    return rc;
  const long R = (M + 15) / 16, nb = (F / 128 + GBW - 1) / GBW;
  hipLaunchKernelGGL(geglu_fwd_lora_kernel, dim3((unsigned)(R * nb)), dim3(64 * GBW), 0, (hipStream_t)stream,
                     (const bf16_t*)x12, ldx, F, M, (bf16_t*)out, ldo, (const bf16_t*)down, (bf16_t*)ds, ldds, alpha,
                     (float*)partials, (unsigned*)tickets);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_geglu_bwd_lora(const void* dy, const void* x12, long ldx, int F, int M, void* dx12, long lddx,
                                  const void* up, void* vs, long ldvs, float alpha, void* tickets, void* partials,
                                  void* stream) {
  VPT_CHECK_ARG(dy && x12 && dx12 && up && vs, "vpt_geglu_bwd_lora: null pointer");
  VPT_CHECK_ARG(F > 0 && F % 128 == 0 && ldx % 8 == 0 && lddx % 8 == 0 && ldx >= 2L * F && lddx >= 2L * F && ldvs >= 16,
                "vpt_geglu_bwd_lora: F % 128 == 0, 16-B leading dims >= 2F");
  if (M <= 0) return VPT_OK;
  if (int rc = geglu_lora_check("vpt_geglu_bwd_lora: tickets / partials (null, misaligned or too many blocks)", F, M,
                                tickets, partials))
    return rc;
  const long R = (M + 15) / 16, nb = (F / 128 + GBW - 1) / GBW;
  hipLaunchKernelGGL(geglu_bwd_lora_kernel, dim3((unsigned)(R * nb)), dim3(64 * GBW), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, (const bf16_t*)x12, ldx, F, M, (bf16_t*)dx12, lddx, (const bf16_t*)up,
                     (bf16_t*)vs, ldvs, alpha, (float*)partials, (unsigned*)tickets);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_geglu_bwd(const void* dy, const void* x12, long ldx, int F, long M, void* dx12, long lddx,
                             void* stream) {
  VPT_CHECK_ARG(dy && x12 && dx12 && F % 8 == 0 && ldx % 8 == 0 && lddx % 8 == 0, "vpt_geglu_bwd: bad args");
  if (M == 0) return VPT_OK;
  hipLaunchKernelGGL(geglu_bwd_kernel, grid1(M * (F / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                     (const bf16_t*)x12, ldx, F, M, (bf16_t*)dx12, lddx);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_nf4_dequant(const void* packed, const void* qabsmax, const float* absmax2, const float* code2,
                               const float* offset, long n, void* out, void* stream) {
  VPT_CHECK_ARG(packed && qabsmax && absmax2 && code2 && offset && out && n % 64 == 0 && n > 0,
                "vpt_nf4_dequant: n must be a positive multiple of 64");
  const long chunks = n / 32;
  hipLaunchKernelGGL(nf4_dequant_kernel, dim3((unsigned)((chunks + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)packed, (const uint8_t*)qabsmax, absmax2, code2, offset, chunks, (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_nf4_dequant_batch(const VptNf4Job* jobs, int njobs, void* stream) {
  VPT_CHECK_ARG(jobs && njobs > 0 && njobs <= 16, "vpt_nf4_dequant_batch: 1..16 jobs");
  Nf4Batch b = {};
  b.njobs = njobs;
  long blocks = 0;
  for (int j = 0; j < njobs; ++j) {
    const VptNf4Job& jb = jobs[j];
    VPT_CHECK_ARG(jb.packed && jb.qabsmax && jb.absmax2 && jb.code2 && jb.offset && jb.out && jb.n > 0 && jb.n % 64 == 0,
                  "vpt_nf4_dequant_batch: job n must be a positive multiple of 64");
    b.job[j] = jb;
    b.block0[j] = blocks;
    blocks += (jb.n / 32 + 255) / 256;
  }
  b.block0[njobs] = blocks;
  hipLaunchKernelGGL(nf4_dequant_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, b);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_nf4_quantize(const void* w, long n, const float* code2, void* packed, void* qabsmax, float* absmax2,
                                float* offset, float* absmax_scratch, void* stream) {
  VPT_CHECK_ARG(w && code2 && packed && qabsmax && absmax2 && offset && absmax_scratch && n % 64 == 0 && n > 0,
                "vpt_nf4_quantize: n must be a positive multiple of 64");
  const long nb = n / 64;
  hipLaunchKernelGGL(nf4_quant_kernel, dim3((unsigned)((nb + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)w, nb, (uint8_t*)packed, absmax_scratch);
  VPT_LAUNCH_CHECK();
  hipLaunchKernelGGL(nf4_nested_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, absmax_scratch, nb, code2,
                     (uint8_t*)qabsmax, absmax2, offset);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_groupnorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int B,
                                 int C, int G, long HW, float eps, void* stream) {
  VPT_CHECK_ARG(x && w && b && y && mean && rstd, "vpt_groupnorm_fwd: null pointer");
  VPT_CHECK_ARG(B > 0 && G > 0 && C % G == 0 && HW % 8 == 0, "vpt_groupnorm_fwd: C % G == 0, HW % 8 == 0");
  hipLaunchKernelGGL(groupnorm_fwd_kernel, dim3(B * G), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, mean, rstd, C, G, HW, eps);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_groupnorm_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const void* w,
                                 const void* dres, void* dx, int B, int C, int G, long HW, void* stream) {
  VPT_CHECK_ARG(dy && x && mean && rstd && w && dx, "vpt_groupnorm_bwd: null pointer");
  VPT_CHECK_ARG(B > 0 && G > 0 && C % G == 0 && HW % 8 == 0, "vpt_groupnorm_bwd: C % G == 0, HW % 8 == 0");
  hipLaunchKernelGGL(groupnorm_bwd_kernel, dim3(B * G), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dy,
                     (const bf16_t*)x, mean, rstd, (const bf16_t*)w, (const bf16_t*)dres, (bf16_t*)dx, C, G, HW);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_transpose_add(const void* src, const void* add, void* dst, int B, int R, int S, void* stream) {
  VPT_CHECK_ARG(src && dst && src != dst, "vpt_transpose_add: null or aliased pointer");
  VPT_CHECK_ARG(B > 0 && R > 0 && S > 0 && R % 8 == 0 && S % 8 == 0, "vpt_transpose_add: R, S multiples of 8");
  hipLaunchKernelGGL(transpose_add_kernel, dim3((S + 63) / 64, (R + 63) / 64, B), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)src, (const bf16_t*)add, (bf16_t*)dst, R, S);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
