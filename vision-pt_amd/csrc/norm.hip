// RMSNorm (hidden dim) and fused per-head QK-RMSNorm + RoPE, forward and backward, for gfx950.
//
// Replaces:
//   FP32RMSNorm.forward      src/modules/norm.py:20-27 (norm1/norm2 at denoiser.py:600,625,
//                            norm_final at denoiser.py:521): y = bf16((x_f32 * rstd) * w)
//   q_norm / k_norm + apply_rope   src/models/jit/denoiser.py:307-316, 369-373, 98-111:
//                            per head (hd = 64) RMSNorm, rounded to bf16, then the interleaved
//                            complex rotation (x_{2i} + i x_{2i+1}) * (cos + i sin) in f32,
//                            rounded to bf16 (`type_as`).
// Math is f32, I/O bf16, vectorised 16 B per lane (guide G13). Weight gradients are reduced
// per block into f32 partial rows and summed by vpt_reduce_rows (deterministic, no atomics).
#include "common.h"

namespace {

// ---------------------------------------------------------------- RMSNorm over D (D % 8 == 0, D <= 1024)
__global__ __launch_bounds__(256) void rmsnorm_fwd_kernel(const bf16_t* __restrict__ x, long ldx,
                                                          const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                          long ldy, float* __restrict__ rstd_out, int M, int D,
                                                          float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = D >> 3;
  uint4 v[2];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      v[i] = *reinterpret_cast<const uint4*>(x + row * ldx + c * 8);
      float f[8];
      unpack8(v[i], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) ss += f[e] * f[e];
    }
  }
  ss = wave_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float f[8], wf[8];
      unpack8(v[i], f);
      unpack8(*reinterpret_cast<const uint4*>(w + c * 8), wf);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = (f[e] * r) * wf[e];
      *reinterpret_cast<uint4*>(y + row * ldy + c * 8) = pack8(f);
    }
  }
  if (lane == 0 && rstd_out) rstd_out[row] = r;
}

// The same with two rows per wave, 32 lanes per row and NC 16-B chunks per lane (D = 256 NC: every lane busy; the
// one-row form leaves half the lanes idle in its second chunk at D = 768). Sum of squares: the lane's 8 NC products in
// order, then xor-shuffles 1 .. 16 within the row's 32 lanes. At the C3 shape (M = 8 x 4154, D = 768; tools/
// hbm_kernels.py, r06i, two interleaved runs each): 18.8 vs 20.16 us, 0.68 vs 0.63 of 8 TB/s. Knob VPT_RMS_FWD32.
template <int NC>
__global__ __launch_bounds__(256) void rmsnorm_fwd32_kernel(const bf16_t* __restrict__ x, long ldx,
                                                            const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                                                            long ldy, float* __restrict__ rstd_out, int M, int D,
                                                            float eps) {
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const long row = (long)blockIdx.x * 8 + (threadIdx.x >> 6) * 2 + (lane >> 5);
  const bool ok = row < M;
  uint4 v[NC], wv[NC];  // the weight pieces loaded up front too: no load follows a store (tools/isa_store_hazard.py)
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    v[i] = ok ? *reinterpret_cast<const uint4*>(x + row * ldx + (hl + 32 * i) * 8) : make_uint4(0, 0, 0, 0);
    wv[i] = *reinterpret_cast<const uint4*>(w + (hl + 32 * i) * 8);
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    float f[8];
    unpack8(v[i], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += f[e] * f[e];
  }
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) ss += __shfl_xor(ss, o, 64);
  const float r = rsqrtf(ss / (float)D + eps);
  if (!ok) return;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const int c = hl + 32 * i;
    float f[8], wf[8];
    unpack8(v[i], f);
    unpack8(wv[i], wf);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = (f[e] * r) * wf[e];
    *reinterpret_cast<uint4*>(y + row * ldy + c * 8) = pack8(f);
  }
  if (hl == 0 && rstd_out) rstd_out[row] = r;
}
#ifndef VPT_RMS_FWD32
#define VPT_RMS_FWD32 1
#endif

// dx = dres + rstd * (g - xhat * mean(g * xhat)), g = dy * w; dw partial per block.
__global__ __launch_bounds__(256) void rmsnorm_bwd_kernel(const bf16_t* __restrict__ dy, long lddy,
                                                          const bf16_t* __restrict__ x, long ldx,
                                                          const float* __restrict__ rstd,
                                                          const bf16_t* __restrict__ w,
                                                          const bf16_t* __restrict__ dres, long ldr,
                                                          bf16_t* __restrict__ dx, long lddx,
                                                          float* __restrict__ dw_part, int M, int D) {
  __shared__ float red[4][1024];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int nch = D >> 3;
  float dwp[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) dwp[i][e] = 0.f;
  float wf[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) unpack8(*reinterpret_cast<const uint4*>(w + c * 8), wf[i]);
  }
  // Two rows per wave per iteration: all loads of both rows (x, dy, dres) are issued before any use,
  // doubling the bytes in flight per wave (the kernel is HBM-latency-bound at one row).
  const long stride = (long)gridDim.x * 4;
  for (long row0 = (long)blockIdx.x * 4 + wid; row0 < M; row0 += 2 * stride) {
    long rows[2] = {row0, row0 + stride};
    uint4 vx[2][2], vd[2][2], vr[2][2];
    float r[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool ok = rows[k] < M;
      r[k] = ok ? rstd[rows[k]] : 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = lane + 64 * i;
        const bool in = ok && c < nch;
        vx[k][i] = in ? *reinterpret_cast<const uint4*>(x + rows[k] * ldx + c * 8) : make_uint4(0, 0, 0, 0);
        vd[k][i] = in ? *reinterpret_cast<const uint4*>(dy + rows[k] * lddy + c * 8) : make_uint4(0, 0, 0, 0);
        vr[k][i] = in && dres ? *reinterpret_cast<const uint4*>(dres + rows[k] * ldr + c * 8) : make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (rows[k] >= M) break;
      const long row = rows[k];
      float xh[2][8], gg[2][8];
      float dot = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
          float fx[8], fd[8];
          unpack8(vx[k][i], fx);
          unpack8(vd[k][i], fd);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            xh[i][e] = fx[e] * r[k];
            gg[i][e] = fd[e] * wf[i][e];
            dot += gg[i][e] * xh[i][e];
            dwp[i][e] += fd[e] * xh[i][e];
          }
        }
      }
      dot = wave_sum(dot) / (float)D;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
          float o[8], fr[8];
          unpack8(vr[k][i], fr);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = r[k] * (gg[i][e] - xh[i][e] * dot);
            // reference: the residual branch and the norm branch gradients are bf16 tensors summed
            o[e] = dres ? fr[e] + bf2f(f2bf(d)) : d;
          }
          *reinterpret_cast<uint4*>(dx + row * lddx + c * 8) = pack8(o);
        }
      }
    }
  }
  if (!dw_part) return;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i;
    if (c < nch)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wid][c * 8 + e] = dwp[i][e];
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += 256)
    dw_part[(long)blockIdx.x * D + d] = red[0][d] + red[1][d] + red[2][d] + red[3][d];
}

// ---------------------------------------------------------------- QK-norm + RoPE (head_dim 64)
// Thread t of a (2*D/8)-thread block owns sub = t: which = sub/(D/8) (q,k), head, part = sub%8
// (dims 8*part..8*part+7). Rows are tokens; token position in its sequence = row % rows_per_seq.
__device__ __forceinline__ void rope_load(const float* __restrict__ cs, const float* __restrict__ sn, long pos, int part,
                                          float (&c)[4], float (&s)[4]) {
  const floatx4 c4 = *reinterpret_cast<const floatx4*>(cs + pos * 32 + part * 4);
  const floatx4 s4 = *reinterpret_cast<const floatx4*>(sn + pos * 32 + part * 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) { c[i] = c4[i]; s[i] = s4[i]; }
}

__global__ __launch_bounds__(256) void qknorm_rope_fwd_kernel(const bf16_t* __restrict__ qkv, long ldin,
                                                              const bf16_t* __restrict__ wq, const bf16_t* __restrict__ wk,
                                                              const float* __restrict__ cs, const float* __restrict__ sn,
                                                              bf16_t* __restrict__ out, long ldout, int M,
                                                              int rows_per_seq, int D, float eps, float q_scale) {
  const int sub = threadIdx.x, per = D >> 3;   // blockDim = 2 * D / 8
  const int which = sub / per, head = (sub % per) >> 3, part = sub & 7;
  const bf16_t* w = which ? wk : wq;
  const float osc = which ? 1.f : q_scale;  // q leaves pre-multiplied (one rounding) for the attention kernels
  float wf[8];
  unpack8(*reinterpret_cast<const uint4*>(w + part * 8), wf);
  for (long row = blockIdx.x; row < M; row += gridDim.x) {
    const long pos = row % rows_per_seq;
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(qkv + row * ldin + which * D + head * 64 + part * 8), f);
    float ss = qkn_sumsq8(f);
    ss += __shfl_xor(ss, 1, 64);
    ss += __shfl_xor(ss, 2, 64);
    ss += __shfl_xor(ss, 4, 64);
    const float r = qkn_rstd(ss, eps);
    float c[4], s[4];
    rope_load(cs, sn, pos, part, c, s);
    float o[8];
    qkn_rope8(f, r, wf, c, s, osc, o);
    *reinterpret_cast<uint4*>(out + row * ldout + which * D + head * 64 + part * 8) = pack8(o);
  }
}

__global__ __launch_bounds__(256) void qknorm_rope_bwd_kernel(const bf16_t* __restrict__ dqk, long lddqk,
                                                              const bf16_t* __restrict__ qkv, long ldin,
                                                              const bf16_t* __restrict__ wq, const bf16_t* __restrict__ wk,
                                                              const float* __restrict__ cs, const float* __restrict__ sn,
                                                              bf16_t* __restrict__ dqkv, long lddqkv,
                                                              float* __restrict__ dw_part, int M, int rows_per_seq,
                                                              int D, float eps, int n_valid) {
  __shared__ float red[256][8];
  const int sub = threadIdx.x, per = D >> 3;   // blockDim = 2 * D / 8
  const int which = sub / per, head = (sub % per) >> 3, part = sub & 7;
  const bf16_t* w = which ? wk : wq;
  float wf[8];
  unpack8(*reinterpret_cast<const uint4*>(w + part * 8), wf);
  float dwp[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) dwp[e] = 0.f;
  for (long row = blockIdx.x; row < M; row += gridDim.x) {
    const long pos = row % rows_per_seq;
    if (pos >= n_valid) {  // rows past the attention's n (a pre-context block's context rows): zero q | k | v gradients
      bf16_t* dst = dqkv + row * lddqkv + which * D + head * 64 + part * 8;
      *reinterpret_cast<uint4*>(dst) = make_uint4(0, 0, 0, 0);
      if (which == 0) *reinterpret_cast<uint4*>(dst + 2 * D) = make_uint4(0, 0, 0, 0);
      continue;
    }
    float fx[8], fg[8];
    unpack8(*reinterpret_cast<const uint4*>(qkv + row * ldin + which * D + head * 64 + part * 8), fx);
    unpack8(*reinterpret_cast<const uint4*>(dqk + row * lddqk + which * D + head * 64 + part * 8), fg);
    float c[4], s[4];
    rope_load(cs, sn, pos, part, c, s);
    float dy[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // rotate back by the conjugate
      dy[2 * i] = fg[2 * i] * c[i] + fg[2 * i + 1] * s[i];
      dy[2 * i + 1] = -fg[2 * i] * s[i] + fg[2 * i + 1] * c[i];
    }
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) ss += fx[e] * fx[e];
    ss += __shfl_xor(ss, 1, 64);
    ss += __shfl_xor(ss, 2, 64);
    ss += __shfl_xor(ss, 4, 64);
    const float r = rsqrtf(ss * (1.f / 64.f) + eps);
    float xh[8], gg[8], dot = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xh[e] = fx[e] * r;
      gg[e] = dy[e] * wf[e];
      dot += gg[e] * xh[e];
      dwp[e] += dy[e] * xh[e];
    }
    dot += __shfl_xor(dot, 1, 64);
    dot += __shfl_xor(dot, 2, 64);
    dot += __shfl_xor(dot, 4, 64);
    dot *= (1.f / 64.f);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = r * (gg[e] - xh[e] * dot);
    *reinterpret_cast<uint4*>(dqkv + row * lddqkv + which * D + head * 64 + part * 8) = pack8(o);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[sub][e] = dwp[e];
  __syncthreads();
  for (int o = sub; o < 128; o += blockDim.x) {  // o -> (which, dim)
    const int wch = o >> 6, d = o & 63, pt = d >> 3, e = d & 7;
    const int nheads = D / 64;
    float acc = 0.f;
    for (int hh = 0; hh < nheads; ++hh) acc += red[wch * per + hh * 8 + pt][e];
    dw_part[(long)blockIdx.x * 128 + o] = acc;
  }
}

// Sum rows of a [R][C] f32 matrix: out[c] (=|+=) sum_r in[r][c]. Block = 16 columns (4 lanes x float4, 64 B per row
// segment) x RG row groups; each row group strides over the rows in a fixed order, then a fixed pairwise tree over the
// row groups (deterministic, no atomics). The partial sets are short and wide (512 x 768 for an RMSNorm weight, 256 x N
// for a bias): 16-column blocks give C/16 workgroups and RG = 256 leaves each lane 2-4 rows, all loads in flight at once.
template <int RG>
__global__ __launch_bounds__(4 * RG) void reduce_rows_kernel(const float* __restrict__ in, int R, int C,
                                                             float* __restrict__ out, int accumulate) {
  __shared__ floatx4 red[RG][4];
  colsum_block<RG>(in, R, C, out, accumulate, blockIdx.x, red);
}

}  // namespace

extern "C" int vpt_rmsnorm_fwd(const void* x, long ldx, const void* w, void* y, long ldy, float* rstd, int M, int D,
                               float eps, void* stream) {
  VPT_CHECK_ARG(x && w && y, "vpt_rmsnorm_fwd: null pointer");
  VPT_CHECK_ARG(D % 8 == 0 && D <= 1024 && M >= 0, "vpt_rmsnorm_fwd: D must be a multiple of 8, <= 1024");
  if (M == 0) return VPT_OK;
  if (VPT_RMS_FWD32 && (D == 768 || D == 1024)) {
    auto kern = D == 768 ? rmsnorm_fwd32_kernel<3> : rmsnorm_fwd32_kernel<4>;
    hipLaunchKernelGGL(kern, dim3((M + 7) / 8), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x, ldx,
                       (const bf16_t*)w, (bf16_t*)y, ldy, rstd, M, D, eps);
  } else {
    hipLaunchKernelGGL(rmsnorm_fwd_kernel, dim3((M + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       (const bf16_t*)x, ldx, (const bf16_t*)w, (bf16_t*)y, ldy, rstd, M, D, eps);
  }
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_rmsnorm_bwd_blocks(int M) {
  int b = (M + 3) / 4;
  return b < 512 ? (b < 1 ? 1 : b) : 512;
}

extern "C" int vpt_rmsnorm_bwd(const void* dy, long lddy, const void* x, long ldx, const float* rstd, const void* w,
                               const void* dres, long ldr, void* dx, long lddx, float* dw_part, int M, int D,
                               void* stream) {
  VPT_CHECK_ARG(dy && x && rstd && w && dx, "vpt_rmsnorm_bwd: null pointer");
  VPT_CHECK_ARG(D % 8 == 0 && D <= 1024, "vpt_rmsnorm_bwd: D must be a multiple of 8, <= 1024");
  if (M == 0) return VPT_OK;
  hipLaunchKernelGGL(rmsnorm_bwd_kernel, dim3(vpt_rmsnorm_bwd_blocks(M)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, rstd, (const bf16_t*)w, (const bf16_t*)dres, ldr,
                     (bf16_t*)dx, lddx, dw_part, M, D);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_qknorm_rope_blocks(int M) { return M < 1024 ? (M < 1 ? 1 : M) : 1024; }

extern "C" int vpt_qknorm_rope_fwd(const void* qkv, long ldin, const void* wq, const void* wk, const float* cos_t,
                                   const float* sin_t, void* out, long ldout, int M, int rows_per_seq, int D,
                                   float eps, float q_scale, void* stream) {
  VPT_CHECK_ARG(qkv && wq && wk && cos_t && sin_t && out, "vpt_qknorm_rope_fwd: null pointer");
  VPT_CHECK_ARG(D % 64 == 0 && D <= 1024, "vpt_qknorm_rope_fwd: heads x 64 with D <= 1024");
  if (M == 0) return VPT_OK;
  hipLaunchKernelGGL(qknorm_rope_fwd_kernel, dim3(M < 8192 ? M : 8192), dim3(D / 4), 0, (hipStream_t)stream,
                     (const bf16_t*)qkv, ldin, (const bf16_t*)wq, (const bf16_t*)wk, cos_t, sin_t, (bf16_t*)out, ldout,
                     M, rows_per_seq, D, eps, q_scale);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_qknorm_rope_bwd_rows(const void* dqk, long lddqk, const void* qkv, long ldin, const void* wq,
                                        const void* wk, const float* cos_t, const float* sin_t, void* dqkv, long lddqkv,
                                        float* dw_part, int M, int rows_per_seq, int n_valid, int D, float eps,
                                        void* stream) {
  VPT_CHECK_ARG(dqk && qkv && wq && wk && cos_t && sin_t && dqkv && dw_part, "vpt_qknorm_rope_bwd: null pointer");
  VPT_CHECK_ARG(D % 64 == 0 && D <= 1024, "vpt_qknorm_rope_bwd: heads x 64 with D <= 1024");
  VPT_CHECK_ARG(n_valid >= 0 && n_valid <= rows_per_seq, "vpt_qknorm_rope_bwd: 0 <= n_valid <= rows_per_seq");
  VPT_CHECK_ARG(n_valid == rows_per_seq || lddqkv >= 3 * D, "vpt_qknorm_rope_bwd: n_valid < rows needs dqkv's v part");
  if (M == 0) return VPT_OK;
  hipLaunchKernelGGL(qknorm_rope_bwd_kernel, dim3(vpt_qknorm_rope_blocks(M)), dim3(D / 4), 0, (hipStream_t)stream,
                     (const bf16_t*)dqk, lddqk, (const bf16_t*)qkv, ldin, (const bf16_t*)wq, (const bf16_t*)wk, cos_t,
                     sin_t, (bf16_t*)dqkv, lddqkv, dw_part, M, rows_per_seq, D, eps, n_valid);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_qknorm_rope_bwd(const void* dqk, long lddqk, const void* qkv, long ldin, const void* wq,
                                   const void* wk, const float* cos_t, const float* sin_t, void* dqkv, long lddqkv,
                                   float* dw_part, int M, int rows_per_seq, int D, float eps, void* stream) {
  return vpt_qknorm_rope_bwd_rows(dqk, lddqk, qkv, ldin, wq, wk, cos_t, sin_t, dqkv, lddqkv, dw_part, M, rows_per_seq,
                                  rows_per_seq, D, eps, stream);
}

extern "C" int vpt_reduce_rows(const float* in, int R, int C, float* out, int accumulate, void* stream) {
  VPT_CHECK_ARG(in && out && R > 0 && C > 0, "vpt_reduce_rows: bad args");
  if (R >= 256)
    hipLaunchKernelGGL(reduce_rows_kernel<256>, dim3((C + 15) / 16), dim3(1024), 0, (hipStream_t)stream, in, R, C, out,
                       accumulate);
  else
    hipLaunchKernelGGL(reduce_rows_kernel<64>, dim3((C + 15) / 16), dim3(256), 0, (hipStream_t)stream, in, R, C, out,
                       accumulate);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
