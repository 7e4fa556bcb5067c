// SDXL flow-matching step pieces around the UNet (BASELINE config 5), for gfx950. HBM-bound elementwise work,
// 16-B vectorised. Reference call sites replaced:
//   t * 1000 sampling + noising   train/sdxl/flow_match.py:127-149, src/modules/loss/flow_match.py:60-74
//                                 (prepare_scaled_noised_latents: eps = randn_like(latents) * noise_scale,
//                                 z = t x + (1 - t) eps, or (1 - t) x + t eps with clean_at_zero)
//   velocity MSE + its gradient   src/modules/loss/flow_match.py:85-96 (loss_with_predicted_velocity:
//                                 mse(v, eps - latents)), called by flow_match.py:163-169 (treat_loss)
//   sinusoidal embeddings         src/models/sdxl/denoiser.py:1117-1123 (get_timestep_embedding, any even dim,
//                                 flip_sin_to_cos=True, downscale_freq_shift=0) for t*1000 (dim 320) and the
//                                 six size conditions (dim 256), src/models/sdxl/denoiser.py:1125-1170
//   pixel (un)shuffle             the NCHW <-> token-major maps of the UNet skeleton around the transformer stacks
//                                 (vpt/sdxl_flow.py): space-to-depth by r with feature order (c, i, j)
#include "common.h"

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// Standard normal for element `idx` of stream `seed` (Box-Muller on a counter hash).
__device__ __forceinline__ float gauss(uint64_t seed, uint64_t idx) {
  const uint64_t h = mix64(seed * 0x632be59bd9b4e019ull ^ mix64(idx));
  const float u1 = ((float)(uint32_t)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
  const float u2 = (float)((uint32_t)h & 0xffffffu) * (1.0f / 16777216.0f);
  return sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// 8 latents per thread: eps = bf16(bf16(randn) * s) (randn_like on bf16 latents, then the bf16 multiply), or
// the caller's eps; z = f32 lerp (t is an f32 tensor: the products promote to f32) rounded to bf16 for the
// bf16 model.
__global__ void flow_noise_kernel(const bf16_t* __restrict__ x, const float* __restrict__ t, long n_per, long total,
                                  float noise_scale, int clean_at_zero, uint64_t seed, const bf16_t* __restrict__ eps_in,
                                  bf16_t* __restrict__ z, bf16_t* __restrict__ eps_out) {
#pragma clang fp contract(off)  // torch: two f32 products and one add, each rounded (no FMA)
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= total) return;
  const float tb = t[i / n_per];
  const float a = clean_at_zero ? 1.f - tb : tb, c = clean_at_zero ? tb : 1.f - tb;
  float xv[8], ev[8], zv[8];
  unpack8(*reinterpret_cast<const uint4*>(x + i), xv);
  if (eps_in) {
    unpack8(*reinterpret_cast<const uint4*>(eps_in + i), ev);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) ev[e] = bf2f(f2bf(bf2f(f2bf(gauss(seed, (uint64_t)(i + e)))) * noise_scale));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) zv[e] = a * xv[e] + c * ev[e];
  *reinterpret_cast<uint4*>(z + i) = pack8(zv);
  if (eps_out && !eps_in) *reinterpret_cast<uint4*>(eps_out + i) = pack8(ev);
}

// loss = mean((v - bf16(eps - x))^2) in f32 (autocast mse_loss on the bf16 tensors), dv = bf16(2 d / n);
// per-block partial sums (fixed order) reduced by flow_loss_reduce_kernel.
constexpr int kLossBlocks = 1024;
__global__ __launch_bounds__(256) void velocity_loss_kernel(const bf16_t* __restrict__ v, const bf16_t* __restrict__ x,
                                                            const bf16_t* __restrict__ eps, long total, float two_over_n,
                                                            bf16_t* __restrict__ dv, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < total; i += (long)gridDim.x * blockDim.x * 8) {
    float vv[8], xv[8], ev[8], g[8];
    unpack8(*reinterpret_cast<const uint4*>(v + i), vv);
    unpack8(*reinterpret_cast<const uint4*>(x + i), xv);
    unpack8(*reinterpret_cast<const uint4*>(eps + i), ev);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = vv[e] - bf2f(f2bf(ev[e] - xv[e]));
      s += d * d;
      g[e] = two_over_n * d;
    }
    if (dv) *reinterpret_cast<uint4*>(dv + i) = pack8(g);
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ void loss_reduce_kernel(const float* __restrict__ part, int n, float inv_n, float* __restrict__ loss) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) *loss = ((red[0] + red[1]) + (red[2] + red[3])) * inv_n;
}

// out[r][j] = cos(v_r f_j) (j < half), sin(v_r f_{j-half}) (j >= half), f_j = exp(-ln(1e4) j / half)
__global__ void sinusoid_kernel(const float* __restrict__ vals, int R, int dim, bf16_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * dim) return;
  const int half = dim >> 1, r = i / dim, j = i % dim, f = j < half ? j : j - half;
  const float arg = vals[r] * expf((-9.210340371976184f * (float)f) / (float)half);
  out[i] = f2bf(j < half ? cosf(arg) : sinf(arg));
}

// NCHW [B][C][H][W] <-> token-major [B][(H/r)(W/r)][C r r], feature index (c r + i) r + j for pixel
// (y r + i, x r + j) of token (y, x): torch.nn.functional.pixel_unshuffle followed by the NCHW->tokens permute.
// One thread per token-side element (coalesced on the token side).
__global__ void space_to_depth_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int B, int C, int H,
                                      int W, int r, int inverse) {
  const int Ht = H / r, Wt = W / r, F = C * r * r;
  const long total = (long)B * Ht * Wt * F;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int f = gid % F;
  const long tok = gid / F;
  const int b = tok / ((long)Ht * Wt), p = tok % ((long)Ht * Wt), y = p / Wt, x = p % Wt;
  const int c = f / (r * r), ij = f % (r * r), i = ij / r, j = ij % r;
  const long nchw = (((long)b * C + c) * H + (y * r + i)) * W + (x * r + j);
  if (inverse)
    dst[nchw] = src[gid];  // tokens -> NCHW (pixel_shuffle): the adjoint permutation
  else
    dst[gid] = src[nchw];
}

}  // namespace

extern "C" int vpt_flow_noise(const void* x, const float* t, long n_per_sample, int B, float noise_scale,
                              int clean_at_zero, unsigned long long seed, const void* eps_in, void* z, void* eps_out,
                              void* stream) {
  VPT_CHECK_ARG(x && t && z && (eps_in || eps_out), "vpt_flow_noise: null pointer");
  VPT_CHECK_ARG(B > 0 && n_per_sample > 0 && n_per_sample % 8 == 0, "vpt_flow_noise: n_per_sample % 8 == 0");
  const long total = (long)B * n_per_sample;
  hipLaunchKernelGGL(flow_noise_kernel, dim3((unsigned)((total / 8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, t, n_per_sample, total, noise_scale, clean_at_zero, (uint64_t)seed,
                     (const bf16_t*)eps_in, (bf16_t*)z, (bf16_t*)eps_out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_velocity_loss_blocks(void) { return kLossBlocks; }

extern "C" int vpt_velocity_loss(const void* v, const void* x, const void* eps, long n, void* dv, float* part,
                                 float* loss, void* stream) {
  VPT_CHECK_ARG(v && x && eps && part && loss && n > 0 && n % 8 == 0, "vpt_velocity_loss: bad args");
  hipLaunchKernelGGL(velocity_loss_kernel, dim3(kLossBlocks), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)v,
                     (const bf16_t*)x, (const bf16_t*)eps, n, (float)(2.0 / (double)n), (bf16_t*)dv, part);
  hipLaunchKernelGGL(loss_reduce_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, kLossBlocks,
                     (float)(1.0 / (double)n), loss);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_sinusoid_embed(const float* vals, int R, int dim, void* out, void* stream) {
  VPT_CHECK_ARG(vals && out && R > 0 && dim > 0 && dim % 2 == 0, "vpt_sinusoid_embed: bad args");
  hipLaunchKernelGGL(sinusoid_kernel, dim3((R * dim + 255) / 256), dim3(256), 0, (hipStream_t)stream, vals, R, dim,
                     (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_space_to_depth(const void* src, void* dst, int B, int C, int H, int W, int r, int inverse,
                                  void* stream) {
  VPT_CHECK_ARG(src && dst && B > 0 && C > 0 && r > 0 && H % r == 0 && W % r == 0, "vpt_space_to_depth: bad shape");
  const long total = (long)B * C * H * W;
  hipLaunchKernelGGL(space_to_depth_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)src, (bf16_t*)dst, B, C, H, W, r, inverse);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
