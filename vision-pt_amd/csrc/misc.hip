// HBM-bound helper kernels of the JiT training step, for gfx950 (all 16-B vectorised where the
// layout allows). Reference call sites replaced:
//   noise + lerp            src/modules/loss/flow_match.py:60-74 (prepare_scaled_noised_latents)
//   patchify for proj_1     src/models/jit/denoiser.py:36-49 (Conv2d k=16 s=16 -> im2col (c,ky,kx))
//   unpatchify              src/models/jit/denoiser.py:828-860 ((py,px,c) per patch -> NCHW)
//   x-/v-loss + its grad    train/jit/arb_class_to_image.py:108-151, src/models/jit/pipeline.py:253-260
//   timestep embedding      src/modules/timestep/embedding.py:10-62 (flip_sin_to_cos=True, shift 0)
//   token assembly          src/models/jit/denoiser.py:982-1005, 1078-1113 (time/size/context tokens)
//   SwiGLU activation       src/models/jit/denoiser.py:499-504
//   class embedding         src/models/jit/class_encoder.py:139 (nn.Embedding, padding_idx rows get no grad)
//   RAdamScheduleFree step  schedulefree==1.4.1 (configs/jit/x-loss/config.yml:74-78), see DESIGN.md
#include "common.h"

namespace {

// ---------------------------------------------------------------- counter-based gaussian noise
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// Counter-based standard normals, rounded to fp16 like randn_like(fp16 image): pixel pair j = idx / 2 is one
// Box-Muller draw from ONE keyed 32-bit hash of j (lowbias32: 2 multiplies, 3 xor-shifts; a bijection of j for a
// fixed key, so no two pairs of an image share a hash), its high half the radius uniform u1 and its low half the
// angle u2 (16 bits each: radii up to 4.85 sigma, 65536 angles -- finer than the fp16 result), element 2j taking
// r cos(2 pi u2), element 2j+1 r sin(2 pi u2). On the transcendental units: v_log_f32 (log2; ln u1 = ln2 log2 u1),
// v_sqrt_f32, v_cos_f32 / v_sin_f32 (argument in revolutions: no range reduction). The 32-bit multiplies are the
// expensive integer ops here (two per pair; the two-hash form had seven with its counter mixing). A pure function
// of (seed, idx): the loss regenerates the forward's noise.
struct NoiseKey {
  uint32_t a, b;
};
__device__ __forceinline__ NoiseKey noise_key(uint64_t seed) {
  const uint64_t m = mix64(seed);
  return {(uint32_t)m, (uint32_t)(m >> 32)};
}
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t pair_counter(uint64_t idx) {
  const uint64_t j = idx >> 1;
  return (uint32_t)j ^ (uint32_t)(j >> 32);  // pairs past 2^32 (batches > 8 G pixels) folded in without a multiply
}
// (radius, angle in revolutions) of pair j
__device__ __forceinline__ float2 gauss_polar(NoiseKey k, uint32_t j) {
  const uint32_t h = lowbias32((j ^ k.a) + k.b);
  const float u1 = ((float)(h >> 16) + 0.5f) * (1.0f / 65536.0f);  // (0,1)
  const float u2 = (float)(h & 0xffffu) * (1.0f / 65536.0f);       // [0,1)
  return {__builtin_amdgcn_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1)), u2};
}
// both elements of pair j (fp16-rounded)
__device__ __forceinline__ void gauss_pair_fp16(NoiseKey k, uint32_t j, float& g0, float& g1) {
  const float2 ra = gauss_polar(k, j);
  // both fp16 roundings (RNE) in one v_cvt_pk_f16_f32
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef _Float16 h2v __attribute__((ext_vector_type(2)));
  const f2v g = {ra.x * __builtin_amdgcn_cosf(ra.y), ra.x * __builtin_amdgcn_sinf(ra.y)};
  const h2v h = __builtin_convertvector(g, h2v);
  g0 = (float)h[0];
  g1 = (float)h[1];
}
// Strips: up to kStripP horizontally adjacent 16x16 patches of one patch row, i.e. 3 x 16 image rows of up to
// 64 pixels (128 B per row piece: whole cache lines). patchify and the loss stage a strip's pixels through LDS by
// coalesced 16-B row reads and map them onto the patch layouts from there (the patch layouts' 16-B pieces are 8
// pixels of one row (patchify) or 2.67 pixels x 3 channels (prediction): read from the NCHW image directly they
// were 32-B or 2-B gathers).
constexpr int kStripP = 4;
struct Strip {
  int b, py, px0, np;  // batch, patch row, first patch column, patches in the strip
};
__device__ __forceinline__ Strip strip_of(long s, int hp, int wp) {
  const int spr = (wp + kStripP - 1) / kStripP;
  Strip r;
  r.b = (int)(s / ((long)hp * spr));
  const int rem = (int)(s - (long)r.b * hp * spr);
  r.py = rem / spr;
  r.px0 = (rem - r.py * spr) * kStripP;
  r.np = min(kStripP, wp - r.px0);
  return r;
}
// Image-row piece i (< 384) of a strip with cpr in {2, 4, 6, 8} 16-B pieces per row -> row rr = c * 16 + ky and
// piece cc: rr = i / cpr as a 24-bit multiply by the block's rounded-up reciprocal (exact for i < 2^15), no division
// or 32-bit multiply per piece; and the piece's element offset in the image, (c * H + ky) * W + 8 cc (< 2^31).
struct PieceMap {
  int cpr, magic, H, W;
};
__device__ __forceinline__ PieceMap piece_map(int np, int H, int W) {
  return {2 * np, (65536 + 2 * np - 1) / (2 * np), H, W};
}
__device__ __forceinline__ void piece_of(const PieceMap& m, int i, int& c, int& ky, int& cc, int& off) {
  const int rr = (int)(__umul24((unsigned)i, (unsigned)m.magic) >> 16);
  cc = i - (int)__umul24((unsigned)rr, (unsigned)m.cpr);
  c = rr >> 4;
  ky = rr & 15;
  off = (int)__umul24((unsigned)(__umul24((unsigned)c, (unsigned)m.H) + ky), (unsigned)m.W) + cc * 8;
}
// z = t*x + (1-t)*eps written in patch-major im2col layout (col = c*P*P + ky*P + kx).
// in_kind 0: x fp16 + noise (generated or explicit fp16 `noise`), in_kind 1: x bf16 copied as is.
// An output piece (8 kx of one (c, ky)) is one 16-B piece of an image row, so no transposition is needed -- only
// the thread order: threads walk a strip's image-row pieces in row order (a wave reads 8 image rows x 128 B, whole
// lines) and write each piece to its patch row (per wave 4 runs of 256 B).
// One 128-thread block per strip (blockIdx.x = strip, decoded once in scalar registers); a thread takes the strip's
// pieces i = tid + 128 k (k < 3: 48 rows x 8 pieces of a full strip), all its image (and explicit-noise) loads issued
// before any arithmetic. (The earlier grid-stride form decoded every piece's strip with 64-bit divisions by runtime
// values and held one load in flight per thread: its integer index math and latency, not HBM, set its time.)
constexpr int kPatchThreads = 128, kPatchPer = 96 * kStripP / kPatchThreads;
// MODE (compile time, so the element loop carries no source branches): 0 = generated noise at noise_scale 1 (the
// draw is already fp16-rounded, so the reference's second rounding of randn * 1.0 is the identity and is skipped),
// 1 = generated noise at another scale, 2 = explicit fp16 noise, 3 = a bf16 image copied as is (in_kind 1).
template <int MODE>
__global__ __launch_bounds__(kPatchThreads) void patchify_kernel(const unsigned short* __restrict__ img,
                                                                 const unsigned short* __restrict__ noise,
                                                                 const float* __restrict__ t, float noise_scale,
                                                                 uint64_t seed, int B, int H, int W,
                                                                 bf16_t* __restrict__ out) {
  const int hp = H / 16, wp = W / 16;
  const Strip st = strip_of(blockIdx.x, hp, wp);
  const PieceMap pm = piece_map(st.np, H, W);
  const long img0 = ((long)st.b * 3 * H + st.py * 16) * W + st.px0 * 16;  // (c = 0, ky = 0, strip column 0)
  bf16_t* const out0 = out + (((long)st.b * hp + st.py) * wp + st.px0) * 768;
  const unsigned short* const im = img + img0;
  uint4 v[kPatchPer], nv[kPatchPer];
#pragma unroll
  for (int k = 0; k < kPatchPer; ++k) {
    const int i = threadIdx.x + k * kPatchThreads;
    int c, ky, cc, off;
    piece_of(pm, i, c, ky, cc, off);
    const bool ok = i < 48 * pm.cpr;
    v[k] = ok ? *reinterpret_cast<const uint4*>(im + off) : make_uint4(0, 0, 0, 0);
    if (MODE == 2) nv[k] = ok ? *reinterpret_cast<const uint4*>(noise + img0 + off) : make_uint4(0, 0, 0, 0);
  }
  const NoiseKey key = noise_key(seed);
  const float tb = MODE == 3 ? 0.f : t[st.b];
#pragma unroll
  for (int k = 0; k < kPatchPer; ++k) {
    const int i = threadIdx.x + k * kPatchThreads;
    if (i >= 48 * pm.cpr) continue;
    int c, ky, cc, off;
    piece_of(pm, i, c, ky, cc, off);
    const int pl = cc >> 1, kx0 = (cc & 1) * 8;
    const unsigned short* vs = reinterpret_cast<const unsigned short*>(&v[k]);
    float o[8];
    if (MODE == 3) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = bf2f(vs[e]);
    } else {
      float nz[8];
      if (MODE == 2) {
        const unsigned short* ns = reinterpret_cast<const unsigned short*>(&nv[k]);
#pragma unroll
        for (int e = 0; e < 8; ++e) nz[e] = h2f(f2h(h2f(ns[e]) * noise_scale));
      } else {
        const uint32_t j0 = pair_counter((uint64_t)(img0 + off));  // even (W, x multiples of 8)
#pragma unroll
        for (int e = 0; e < 4; ++e) gauss_pair_fp16(key, j0 + e, nz[2 * e], nz[2 * e + 1]);
        if (MODE == 1) {
#pragma unroll
          for (int e = 0; e < 8; ++e) nz[e] = h2f(f2h(nz[e] * noise_scale));
        }
      }
      const float ct = 1.f - tb;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = tb * h2f(vs[e]) + ct * nz[e];
    }
    *reinterpret_cast<uint4*>(out0 + pl * 768 + c * 256 + ky * 16 + kx0) = pack8(o);
  }
}

// lowres_loss inputs (train/jit/arb_class_to_image.py:228-264): F.interpolate(mode="area", scale_factor=1/k) of the
// fp16 image, of the fp16 noise and of the f32 noisy image z = t x + (1-t) eps, for an integer factor k (even: whole
// pixel pairs of the counter-based noise) -- adaptive average pooling over k x k windows, f32 sums. Writes the
// resized image and noise as fp16 (the reference's fp16 tensors) and the resized noisy image as bf16 (the model input,
// lowres_noisy_image.to(bf16)). noise = NULL: the full-resolution noise regenerated from `seed` exactly as patchify
// and the loss generate it. One thread per output pixel, one 4-B image (and noise) load per pixel pair.
__global__ void area_lowres_kernel(const unsigned short* __restrict__ img, const unsigned short* __restrict__ noise,
                                   const float* __restrict__ t, float noise_scale, uint64_t seed, int B, int H, int W,
                                   int k, unsigned short* __restrict__ img_lr, unsigned short* __restrict__ noise_lr,
                                   bf16_t* __restrict__ z_lr) {
  const int h = H / k, w = W / k;
  const long total = (long)B * 3 * h * w;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int X = i % w, Y = (i / w) % h;
  const long bc = i / ((long)w * h);  // b * 3 + c
  const float tb = t[bc / 3];
  const NoiseKey key = noise_key(seed);
  float sx = 0.f, se = 0.f, sz = 0.f;
  for (int dy = 0; dy < k; ++dy) {
    const long row = (bc * H + (long)Y * k + dy) * W + (long)X * k;
    for (int dx = 0; dx < k; dx += 2) {
      const long idx = row + dx;  // even
      const uint32_t xv = *reinterpret_cast<const uint32_t*>(img + idx);
      float n0, n1;
      if (noise) {
        const uint32_t nv = *reinterpret_cast<const uint32_t*>(noise + idx);
        n0 = h2f((unsigned short)(nv & 0xffffu));
        n1 = h2f((unsigned short)(nv >> 16));
      } else {
        gauss_pair_fp16(key, pair_counter((uint64_t)idx), n0, n1);
      }
      const float x0 = h2f((unsigned short)(xv & 0xffffu)), x1 = h2f((unsigned short)(xv >> 16));
      const float e0 = h2f(f2h(n0 * noise_scale)), e1 = h2f(f2h(n1 * noise_scale));
      sx += x0 + x1;
      se += e0 + e1;
      sz += (tb * x0 + (1.f - tb) * e0) + (tb * x1 + (1.f - tb) * e1);
    }
  }
  const float inv = 1.f / (float)(k * k);
  img_lr[i] = f2h(sx * inv);
  noise_lr[i] = f2h(se * inv);
  z_lr[i] = f2bf(sz * inv);
}

// The counter-based noise itself as an fp16 tensor (element idx of a flat [B][3][H][W] image = exactly the draw
// patchify, the loss and the lowres resize regenerate in-kernel at that index): randn_like(latents) * noise_scale of
// prepare_scaled_noised_latents (flow_match.py:60-74), for callers that need the tensor (explicit-noise paths, tests).
__global__ void gauss_noise_kernel(long n2, uint64_t seed, float noise_scale, unsigned short* __restrict__ out) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;  // pixel pair
  if (j >= n2) return;
  float g0, g1;
  gauss_pair_fp16(noise_key(seed), pair_counter((uint64_t)(2 * j)), g0, g1);
  const uint32_t v = (uint32_t)f2h(g0 * noise_scale) | ((uint32_t)f2h(g1 * noise_scale) << 16);
  reinterpret_cast<uint32_t*>(out)[j] = v;
}

// Patch rows [B*np][P*P*3] (col = (ky*P + kx)*3 + c) <-> image [B][3][H][W] (bf16), P = 16.
__global__ void unpatchify_kernel(const bf16_t* __restrict__ patches, int B, int H, int W, bf16_t* __restrict__ img,
                                  int reverse) {
  const long total = (long)B * 3 * H * W;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = i % W;
  const int y = (i / W) % H;
  const int c = (i / ((long)W * H)) % 3;
  const int b = i / ((long)3 * W * H);
  const int wp = W / 16;
  const long prow = (long)b * (H / 16) * wp + (y / 16) * wp + (x / 16);
  const int col = ((y % 16) * 16 + (x % 16)) * 3 + c;
  if (reverse) const_cast<bf16_t*>(patches)[prow * 768 + col] = img[i];
  else img[i] = patches[prow * 768 + col];
}

// One Euler step of the sampler with classifier-free guidance (JiTModel.generate,
// src/models/jit/pipeline.py:436-477): z <- z + v * (t_next - t) over the [B,3,H,W] bf16 image, v from
// the model prediction read straight from the patch layout [(n*np), 768] (the unpatchify index map,
// denoiser.py:828-860; positive half rows [0, B*np), negative half [B*np, 2B*np)). Every binary op
// rounds to bf16 as the reference's bf16 tensor arithmetic does: image_to_velocity (:254-260)
// v = bf16(bf16(x - z) / clamp(1 - t, 1e-5)), CFG (:351-357) v = bf16(vp + bf16(s * bf16(vp - vn))),
// update bf16(z + bf16(v * dt)).
__device__ __forceinline__ float rbf(float x) { return bf2f(f2bf(x)); }

__global__ void euler_cfg_kernel(bf16_t* __restrict__ z, const bf16_t* __restrict__ pred, int B, int H, int W,
                                 int cfg, float cfg_scale, int mode, float t, float dt) {
  const long total = (long)B * 3 * H * W;
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int x = i % W, y = (i / W) % H, c = (i / ((long)W * H)) % 3, b = i / ((long)3 * W * H);
  const int wp = W / 16;
  const long np_ = (long)(H / 16) * wp;
  const long prow = b * np_ + (y / 16) * wp + (x / 16);
  const int col = ((y % 16) * 16 + (x % 16)) * 3 + c;
  const float zf = bf2f(z[i]);
  const float den = fmaxf(1.f - t, 1e-5f);
  auto to_v = [&](float p) { return mode == 0 ? rbf(rbf(p - zf) / den) : p; };
  const float vp = to_v(bf2f(pred[prow * 768 + col]));
  float v = vp;
  if (cfg) {
    const float vn = to_v(bf2f(pred[(prow + (long)B * np_) * 768 + col]));
    v = rbf(vp + rbf(cfg_scale * rbf(vp - vn)));
  }
  z[i] = f2bf(zf + rbf(v * dt));
}

// out = bf16(a + b) and out = bf16(s * a) over n bf16 elements (n % 8 == 0): the residual sums and the
// LoRA output-scale gradient of the SDXL block (bf16 tensor arithmetic of the reference).
__global__ void add_bf16_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b, long n8,
                                bf16_t* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float fa[8], fb[8];
  unpack8(reinterpret_cast<const uint4*>(a)[i], fa);
  unpack8(reinterpret_cast<const uint4*>(b)[i], fb);
#pragma unroll
  for (int e = 0; e < 8; ++e) fa[e] += fb[e];
  reinterpret_cast<uint4*>(out)[i] = pack8(fa);
}
__global__ void scale_bf16_kernel(const bf16_t* __restrict__ a, long n8, float s, bf16_t* __restrict__ out) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  float fa[8];
  unpack8(reinterpret_cast<const uint4*>(a)[i], fa);
#pragma unroll
  for (int e = 0; e < 8; ++e) fa[e] *= s;
  reinterpret_cast<uint4*>(out)[i] = pack8(fa);
}

// The same on a [rows][cols] block of a row-strided matrix (in place allowed): the attention query pre-scale of
// a q that is one column block of a fused q | k | v projection.
__global__ void scale_bf16_2d_kernel(const bf16_t* __restrict__ a, long lda, long rows, int cols8, float s,
                                     bf16_t* __restrict__ out, long ldo) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * cols8) return;
  const long r = i / cols8, c = (i - r * cols8) * 8;
  float fa[8];
  unpack8(*reinterpret_cast<const uint4*>(a + r * lda + c), fa);
#pragma unroll
  for (int e = 0; e < 8; ++e) fa[e] *= s;
  *reinterpret_cast<uint4*>(out + r * ldo + c) = pack8(fa);
}

// Flow-matching MSE over patch-layout predictions; also writes d(loss)/d(pred) (bf16, patch layout).
// target 0 ("image"): mse(pred, x); target 1 ("velocity"): mse((pred-z)/c, (x-z)/c), c = clamp(1-t, eps);
// target 2 (model_pred="velocity", class_to_image.py:146-156): mse(pred, fp16(x - eps)) -- the fp16 image minus the
// fp16 noise rounded to fp16 as the reference's fp16 tensor subtraction, no timestep clamp.
// One 128-thread block per strip (grid-stride past the grid, fixed assignment), patchify's shape: a thread takes the
// strip's prediction pieces i = tid + 128 k and its image-row pieces (k < 3 for a full strip), every load (and the
// explicit noise's) issued before the strip is staged through LDS; then each 16-B prediction piece
// (col = (ky*16 + kx)*3 + c) is mapped onto the staged strip. Per-thread sums in a fixed order, one partial per block:
// deterministic. (The 256-thread form staged its image pieces only after its prediction loads and a barrier, two
// strips per block in sequence.)
#ifndef VPT_LOSS_BLOCKS
#define VPT_LOSS_BLOCKS 4096  // grid cap = partials (4096: 30.5 us, 8192: 32.8, 2048: 30.8 at C3, r05zu)
#endif
constexpr int kLossThreads = 128, kLossPer = 96 * kStripP / kLossThreads, kLossBlocks = VPT_LOSS_BLOCKS;
template <int TARGET>
__global__ __launch_bounds__(kLossThreads) void loss_kernel(const bf16_t* __restrict__ pred,
                                                            const unsigned short* __restrict__ img,
                                                            const unsigned short* __restrict__ noise,
                                                            const float* __restrict__ t, float noise_scale,
                                                            uint64_t seed, float t_eps, int B, int H, int W,
                                                            float inv_numel, bf16_t* __restrict__ dpred,
                                                            float* __restrict__ part) {
  __shared__ float red[kLossThreads];
  __shared__ __attribute__((aligned(16))) unsigned short px[3][16][16 * kStripP];
  __shared__ __attribute__((aligned(16))) unsigned short eps[TARGET ? 3 : 1][16][16 * kStripP];
  const int hp = H / 16, wp = W / 16;
  const long strips = (long)B * hp * ((wp + kStripP - 1) / kStripP);
  const NoiseKey key = noise_key(seed);
  float acc = 0.f;
  for (long s = blockIdx.x; s < strips; s += gridDim.x) {
    const Strip st = strip_of(s, hp, wp);
    const PieceMap pm = piece_map(st.np, H, W);
    const long img0 = ((long)st.b * 3 * H + st.py * 16) * W + st.px0 * 16;
    const long row0 = ((long)st.b * hp + st.py) * wp + st.px0;
    const bf16_t* const pr0 = pred + row0 * 768;
    uint4 pv[kLossPer], iv[kLossPer], nv[kLossPer];
#pragma unroll
    for (int k = 0; k < kLossPer; ++k) {
      const int i = threadIdx.x + k * kLossThreads;
      pv[k] = i < st.np * 96 ? *reinterpret_cast<const uint4*>(pr0 + i * 8) : make_uint4(0, 0, 0, 0);
      int c, ky, cc, off;
      piece_of(pm, i, c, ky, cc, off);
      const bool ok = i < 48 * pm.cpr;
      iv[k] = ok ? *reinterpret_cast<const uint4*>(img + img0 + off) : make_uint4(0, 0, 0, 0);
      nv[k] = TARGET && ok && noise ? *reinterpret_cast<const uint4*>(noise + img0 + off) : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();  // the previous strip's LDS reads are done
#pragma unroll
    for (int k = 0; k < kLossPer; ++k) {
      const int i = threadIdx.x + k * kLossThreads;
      if (i >= 48 * pm.cpr) continue;
      int c, ky, cc, off;
      piece_of(pm, i, c, ky, cc, off);
      *reinterpret_cast<uint4*>(&px[c][ky][cc * 8]) = iv[k];
      if (!TARGET) continue;
      float nz[8];
      if (noise) {
        const unsigned short* ns = reinterpret_cast<const unsigned short*>(&nv[k]);
#pragma unroll
        for (int e = 0; e < 8; ++e) nz[e] = h2f(ns[e]);
      } else {
        const uint32_t j0 = pair_counter((uint64_t)(img0 + off));  // even
#pragma unroll
        for (int e = 0; e < 4; ++e) gauss_pair_fp16(key, j0 + e, nz[2 * e], nz[2 * e + 1]);
      }
      unsigned short ev[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) ev[e] = f2h(nz[e] * noise_scale);
      *reinterpret_cast<uint4*>(&eps[TARGET ? c : 0][ky][cc * 8]) = *reinterpret_cast<const uint4*>(ev);
    }
    __syncthreads();
    const float tb = t[st.b];
    const float cl = fmaxf(1.f - tb, t_eps);
#pragma unroll
    for (int k = 0; k < kLossPer; ++k) {
      const int i = threadIdx.x + k * kLossThreads;
      if (i >= st.np * 96) continue;
      const int pl = i / 96, chunk = i - pl * 96;
      float pr[8], g[8];
      unpack8(pv[k], pr);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int col = chunk * 8 + e, pix = col / 3, c = col - pix * 3;
        const int ky = pix >> 4, kx = pl * 16 + (pix & 15);
        const float xv = h2f(px[c][ky][kx]);
        float diff;
        if (!TARGET) {
          diff = pr[e] - xv;
          g[e] = 2.f * diff * inv_numel;
        } else if (TARGET == 2) {
          diff = pr[e] - h2f(f2h(xv - h2f(eps[TARGET ? c : 0][ky][kx])));
          g[e] = 2.f * diff * inv_numel;
        } else {
          const float z = tb * xv + (1.f - tb) * h2f(eps[TARGET ? c : 0][ky][kx]);
          diff = (pr[e] - z) / cl - (xv - z) / cl;
          g[e] = 2.f * diff * inv_numel / cl;
        }
        acc += diff * diff;
      }
      *reinterpret_cast<uint4*>(dpred + row0 * 768 + i * 8) = pack8(g);
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kLossThreads / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// The block partials' sum, in a fixed order: a 1024-thread block, each thread's partials (k-strided by 1024) loaded
// 8 at a time before any add (a load-add loop waits one L2 round trip per partial: ~0.35 us each), then a tree.
constexpr int kFinThreads = 1024;
__global__ __launch_bounds__(kFinThreads) void loss_finalize_kernel(const float* __restrict__ part, int n,
                                                                    float inv_numel, float* __restrict__ loss) {
  __shared__ float red[kFinThreads];
  float s = 0.f;
  for (int i0 = threadIdx.x; i0 < n; i0 += 8 * kFinThreads) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = i0 + k * kFinThreads < n ? part[i0 + k * kFinThreads] : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = kFinThreads / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] * inv_numel;
}

// ---------------------------------------------------------------- timestep / image-size embedding
__global__ void timestep_embed_kernel(const float* __restrict__ vals, int R, bf16_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * 256) return;
  const int r = i >> 8, j = i & 255, f = j & 127;
  const float expo = (-9.210340371976184f * (float)f) / 128.f;
  const float arg = vals[r] * expf(expo);
  out[i] = f2bf(j < 128 ? cosf(arg) : sinf(arg));
}

// ---------------------------------------------------------------- token assembly
// x[b][n] rows: [0,np) patches | [np,np+6) image-size | [np+6,np+10) time (+pos) | [np+10, rows) context.
// D = hidden size (multiple of 8); one thread per 16-byte chunk.
__global__ void assemble_kernel(const bf16_t* __restrict__ patches, const bf16_t* __restrict__ size_emb,
                                const bf16_t* __restrict__ time_emb, const bf16_t* __restrict__ tpe,
                                const bf16_t* __restrict__ ctx, int n_ctx, int B, int np_, int rows, int D,
                                bf16_t* __restrict__ x) {
  const int nch = D >> 3;
  const long total = (long)B * rows * nch;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const long row = gid / nch;
  const int ch = gid % nch;
  const int b = row / rows, n = row % rows;
  uint4 v = make_uint4(0, 0, 0, 0);
  if (n < np_) {
    v = *reinterpret_cast<const uint4*>(patches + ((long)b * np_ + n) * D + ch * 8);
  } else if (n < np_ + 6) {
    v = *reinterpret_cast<const uint4*>(size_emb + ((long)b * 6 + n - np_) * D + ch * 8);
  } else if (n < np_ + 10) {
    float a[8], p[8];
    unpack8(*reinterpret_cast<const uint4*>(time_emb + (long)b * D + ch * 8), a);
    unpack8(*reinterpret_cast<const uint4*>(tpe + (long)(n - np_ - 6) * D + ch * 8), p);
#pragma unroll
    for (int e = 0; e < 8; ++e) a[e] += p[e];
    v = pack8(a);
  } else if (ctx && n - np_ - 10 < n_ctx) {
    v = *reinterpret_cast<const uint4*>(ctx + ((long)b * n_ctx + n - np_ - 10) * D + ch * 8);
  }
  *reinterpret_cast<uint4*>(x + row * D + ch * 8) = v;
}

// Backward of assemble: split dx into d(patches), d(size tokens), d(time_embed) (sum over the 4
// time tokens) and d(time_position_embeds) (sum over the batch, written by the b == 0 threads).
__global__ void disassemble_kernel(const bf16_t* __restrict__ dx, int B, int np_, int rows, int D,
                                   bf16_t* __restrict__ dpatches, bf16_t* __restrict__ dsize,
                                   bf16_t* __restrict__ dtime, float* __restrict__ dtpe) {
  const int nch = D >> 3;
  const long total = (long)B * (np_ + 7) * nch;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int ch = gid % nch;
  const long r = gid / nch;
  const int b = r / (np_ + 7), n = r % (np_ + 7);
  const bf16_t* src = dx + ((long)b * rows) * D + ch * 8;
  if (n < np_) {
    *reinterpret_cast<uint4*>(dpatches + ((long)b * np_ + n) * D + ch * 8) =
        *reinterpret_cast<const uint4*>(src + (long)n * D);
  } else if (n < np_ + 6) {
    *reinterpret_cast<uint4*>(dsize + ((long)b * 6 + n - np_) * D + ch * 8) =
        *reinterpret_cast<const uint4*>(src + (long)n * D);
  } else {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < 4; ++j) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(src + (long)(np_ + 6 + j) * D), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += f[e];
    }
    *reinterpret_cast<uint4*>(dtime + (long)b * D + ch * 8) = pack8(s);
    if (b == 0 && dtpe) {
      for (int j = 0; j < 4; ++j) {
        float t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int bb = 0; bb < B; ++bb) {
          float f[8];
          unpack8(*reinterpret_cast<const uint4*>(dx + ((long)bb * rows + np_ + 6 + j) * D + ch * 8), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] += f[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) dtpe[j * D + ch * 8 + e] = t[e];
      }
    }
  }
}

// Context rows [row0, row0+n_ctx) of every sequence: fwd copies ctx in; bwd accumulates dx into
// the f32 context-gradient accumulator and zeroes those dx rows (they are stripped after each block).
__global__ void ctx_rows_kernel(bf16_t* __restrict__ x, int B, int row0, int rows, int D,
                                const bf16_t* __restrict__ ctx, float* __restrict__ dctx, int n_ctx, int backward) {
  const int nch = D >> 3;
  const long total = (long)B * n_ctx * nch;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= total) return;
  const int ch = gid % nch;
  const long r = gid / nch;
  const int b = r / n_ctx, j = r % n_ctx;
  bf16_t* xr = x + ((long)b * rows + row0 + j) * D + ch * 8;
  if (!backward) {
    *reinterpret_cast<uint4*>(xr) = *reinterpret_cast<const uint4*>(ctx + r * D + ch * 8);
  } else {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(xr), f);
    floatx4* d = reinterpret_cast<floatx4*>(dctx + r * D + ch * 8);
    if (backward == 2) {  // the first refresh block of the backward: dctx = instead of += (no zero pass before)
      d[0] = floatx4{f[0], f[1], f[2], f[3]};
      d[1] = floatx4{f[4], f[5], f[6], f[7]};
    } else {
      d[0] += floatx4{f[0], f[1], f[2], f[3]};
      d[1] += floatx4{f[4], f[5], f[6], f[7]};
    }
    *reinterpret_cast<uint4*>(xr) = make_uint4(0, 0, 0, 0);
  }
}

// ---------------------------------------------------------------- SwiGLU
__device__ __forceinline__ float silu_f(float x) { return x / (1.f + expf(-x)); }

__global__ void swiglu_fwd_kernel(const bf16_t* __restrict__ x12, long M, int F, bf16_t* __restrict__ h) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nch = F >> 3;
  if (gid >= M * nch) return;
  const long row = gid / nch;
  const int ch = gid % nch;
  float a[8], b[8], o[8];
  unpack8(*reinterpret_cast<const uint4*>(x12 + row * 2 * F + ch * 8), a);
  unpack8(*reinterpret_cast<const uint4*>(x12 + row * 2 * F + F + ch * 8), b);
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = swiglu_fwd1(a[e], b[e]);
  *reinterpret_cast<uint4*>(h + row * F + ch * 8) = pack8(o);
}

__global__ void swiglu_bwd_kernel(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ x12, long M, int F,
                                  bf16_t* __restrict__ dx12) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int nch = F >> 3;
  if (gid >= M * nch) return;
  const long row = gid / nch;
  const int ch = gid % nch;
  float a[8], b[8], g[8], d1[8], d2[8];
  unpack8(*reinterpret_cast<const uint4*>(x12 + row * 2 * F + ch * 8), a);
  unpack8(*reinterpret_cast<const uint4*>(x12 + row * 2 * F + F + ch * 8), b);
  unpack8(*reinterpret_cast<const uint4*>(dh + row * F + ch * 8), g);
#pragma unroll
  for (int e = 0; e < 8; ++e) swiglu_bwd1(g[e], a[e], b[e], d1[e], d2[e]);
  *reinterpret_cast<uint4*>(dx12 + row * 2 * F + ch * 8) = pack8(d1);
  *reinterpret_cast<uint4*>(dx12 + row * 2 * F + F + ch * 8) = pack8(d2);
}

// ---------------------------------------------------------------- column sums (bias grads)
// Column sums of a bf16 [M][N] matrix into f32 partial rows part[slice][N]. Grid (N/256, slices);
// block = 32 lanes x 16-B chunks (256 columns, 512 B per row segment) x 8 row groups.
// Column sums of a bf16 [M][N] matrix into per-slice partials part[S][N] (grid: N/256 column blocks x
// S row slices); vpt_bias_grad then sums the S partial rows in slice order (deterministic).
__global__ __launch_bounds__(256) void colsum_kernel(const bf16_t* __restrict__ in, long ld, long M, int N,
                                                     long rows_per_slice, float* __restrict__ part) {
  __shared__ float red[8][257];
  const int cl = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int col = blockIdx.x * 256 + cl * 8;
  const long r0 = (long)blockIdx.y * rows_per_slice;
  const long r1 = min(M, r0 + rows_per_slice);
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (col < N) {
    long r = r0 + rg;
    for (; r + 24 < r1; r += 32) {  // 4 independent 16-B loads in flight per lane
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(in + (r + 8 * u) * ld + col);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float f[8];
        unpack8(v[u], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += f[e];
      }
    }
    for (; r < r1; r += 8) {
      float f[8];
      unpack8(*reinterpret_cast<const uint4*>(in + r * ld + col), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] += f[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rg][cl * 8 + e] = s[e];
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c < N) {
    float t = red[0][threadIdx.x];
#pragma unroll
    for (int g = 1; g < 8; ++g) t += red[g][threadIdx.x];
    part[(long)blockIdx.y * N + c] = t;
  }
}

// ---------------------------------------------------------------- embedding
__global__ void embed_gather_kernel(const bf16_t* __restrict__ table, const int64_t* __restrict__ ids, long R, int D,
                                    bf16_t* __restrict__ out) {
  const int nch = D >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= R * nch) return;
  const long r = gid / nch;
  const int ch = gid % nch;
  *reinterpret_cast<uint4*>(out + r * D + ch * 8) = *reinterpret_cast<const uint4*>(table + ids[r] * D + ch * 8);
}

__global__ void embed_scatter_kernel(const bf16_t* __restrict__ drows, const int64_t* __restrict__ ids, long R, int D,
                                     long pad_id, float* __restrict__ dtable) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= R * D) return;
  const long r = gid / D;
  const int d = gid % D;
  const long id = ids[r];
  if (id == pad_id) return;
  atomicAdd(dtable + id * D + d, bf2f(drows[gid]));
}

// The class-embedding gradient in one deterministic pass (replaces a fill of the whole table + the atomic scatter):
// each block owns kEmbRows table rows and builds, per row, the list of positions p whose id names it, in ascending p
// without a sort: thread t scans the contiguous position chunk [t*ch, (t+1)*ch), counts its hits per row, an exclusive
// scan over the threads (per row) gives each thread its offsets, and a second scan of the chunk writes the positions
// there -- O(R) per block however many ids share a row. Every row is then the sum of its drows rows in position order
// -- zeros for rows no id names and for the padding row (nn.Embedding padding_idx, as the scatter skips it). accumulate:
// the old value plus that sum (torch's .grad += of the dense embedding gradient); rows no id names are left as they
// are. Dynamic LDS: R ints (the lists), R <= 16384.
constexpr int kEmbRows = 8, kEmbThreads = 256;
__global__ __launch_bounds__(kEmbThreads) void embed_grad_set_kernel(const bf16_t* __restrict__ drows,
                                                                     const int64_t* __restrict__ ids, int R, int D,
                                                                     long pad_id, long V, int accumulate,
                                                                     float* __restrict__ dtable) {
  extern __shared__ int elist[];  // [R] positions, grouped by row, ascending within a row
  __shared__ int cnt[kEmbRows][kEmbThreads + 1];
  __shared__ int start[kEmbRows + 1];
  const long r0 = (long)blockIdx.x * kEmbRows;
  const int ch = (R + kEmbThreads - 1) / kEmbThreads;
  const int lo = min(R, (int)threadIdx.x * ch), hi = min(R, lo + ch);
  int c[kEmbRows];
#pragma unroll
  for (int ro = 0; ro < kEmbRows; ++ro) c[ro] = 0;
  for (int p = lo; p < hi; ++p) {
    const long id = ids[p];
    if (id >= r0 && id < r0 + kEmbRows && id != pad_id) {
#pragma unroll
      for (int ro = 0; ro < kEmbRows; ++ro) c[ro] += (id - r0) == ro;
    }
  }
#pragma unroll
  for (int ro = 0; ro < kEmbRows; ++ro) cnt[ro][threadIdx.x] = c[ro];
  __syncthreads();
  if (threadIdx.x < kEmbRows) {  // row ro: exclusive scan over the threads; the total in cnt[ro][kEmbThreads]
    int run = 0;
    for (int t = 0; t < kEmbThreads; ++t) {
      const int v = cnt[threadIdx.x][t];
      cnt[threadIdx.x][t] = run;
      run += v;
    }
    cnt[threadIdx.x][kEmbThreads] = run;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int ro = 0; ro < kEmbRows; ++ro) {
      start[ro] = run;
      run += cnt[ro][kEmbThreads];
    }
    start[kEmbRows] = run;
  }
  __syncthreads();
  {
    int o[kEmbRows];
#pragma unroll
    for (int ro = 0; ro < kEmbRows; ++ro) o[ro] = start[ro] + cnt[ro][threadIdx.x];
    for (int p = lo; p < hi; ++p) {
      const long id = ids[p];
      if (id >= r0 && id < r0 + kEmbRows && id != pad_id) {
#pragma unroll
        for (int ro = 0; ro < kEmbRows; ++ro)
          if ((id - r0) == ro) elist[o[ro]++] = p;
      }
    }
  }
  __syncthreads();
  const int nc = D >> 2;
  for (int idx = threadIdx.x; idx < kEmbRows * nc; idx += blockDim.x) {
    const int ro = idx / nc, c4 = idx % nc;
    if (r0 + ro >= V) break;
    const int e0 = start[ro], e1 = start[ro + 1];
    if (accumulate && e0 == e1) continue;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int e = e0; e < e1; ++e) {
      const uint2 w = *reinterpret_cast<const uint2*>(drows + (long)elist[e] * D + 4 * c4);
      acc += floatx4{__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                     __uint_as_float(w.y & 0xffff0000u)};
    }
    floatx4* dst = reinterpret_cast<floatx4*>(dtable + (r0 + ro) * D + 4 * c4);
    if (accumulate) acc = *dst + acc;
    *dst = acc;
  }
}

// The JiT step's small per-batch inputs in one launch (jit_train.JiTTrainer.step; replaces ~10 torch element-wise
// launches): t_vals = bf16(bf16(t) * scale) as f32 (arb_class_to_image.py:207's timesteps.to(bf16) * scale), size_vals
// = [original | target | crop] per sample as f32, and the key-bias rows: 0 over the n_pre image / token rows, 0 / -inf
// over the n_ctx context rows by the padding mask (all valid without one).
__global__ void step_inputs_kernel(const float* __restrict__ t, int B, float tscale, const int64_t* __restrict__ orig,
                                   const int64_t* __restrict__ target, const int64_t* __restrict__ crop,
                                   float* __restrict__ t_vals, float* __restrict__ size_vals,
                                   const int64_t* __restrict__ mask, int n_ctx, int n_pre, int rows,
                                   float* __restrict__ kbias) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nk = (long)B * (n_pre + n_ctx);
  if (gid < nk) {
    const int b = gid / (n_pre + n_ctx), c = gid % (n_pre + n_ctx);
    float v = 0.f;
    if (c >= n_pre && mask && mask[(long)b * n_ctx + c - n_pre] == 0) v = -__builtin_huge_valf();
    kbias[(long)b * rows + c] = v;
  } else if (gid < nk + B) {
    const int b = gid - nk;
    t_vals[b] = bf2f(f2bf(bf2f(f2bf(t[b])) * tscale));
  } else if (gid < nk + 7L * B) {
    const int i = gid - nk - B, b = i / 6, j = i % 6;
    const int64_t* src = j < 2 ? orig : j < 4 ? target : crop;
    size_vals[i] = (float)src[2 * b + (j & 1)];
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ in, long n, bf16_t* __restrict__ out) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  const floatx4 v = *reinterpret_cast<const floatx4*>(in + i);
  uint2 w;
  w.x = pack_bf16x2(v[0], v[1]);
  w.y = pack_bf16x2(v[2], v[3]);
  *reinterpret_cast<uint2*>(out + i) = w;
}

// ---------------------------------------------------------------- RAdamScheduleFree
struct SfScalars {
  float beta2, bias_correction2, eps, ckp1, adaptive_y_lr, lr, decay, grad_scale;
  int adam;
  const float* clip_coef;  // device scalar (global-norm clip coefficient) or null
  float clip_value;        // clamp(g, -clip_value, clip_value) when > 0
};
// One element of the update (shared by the scalar and the 4-wide kernel, so both round identically).
__device__ __forceinline__ void sf_elem(float g, float& vv, float& yy, float& zz, const SfScalars& s) {
  g *= s.grad_scale;
  // after_backward (for_training.py:98-109): clip_grad_norm_ then clip_grad_value_ on the (mean) gradient
  if (s.clip_coef) g *= *s.clip_coef;
  if (s.clip_value > 0.f) g = fminf(fmaxf(g, -s.clip_value), s.clip_value);
  vv = vv * s.beta2 + (1.f - s.beta2) * g * g;
  if (s.adam) g = g / (sqrtf(vv / s.bias_correction2) + s.eps);
  if (s.decay != 0.f) g += s.decay * yy;
  const float z0 = zz;
  yy = bf2f(f2bf(yy + s.ckp1 * (z0 - yy)));  // y.lerp_(z, ckp1) on the bf16 parameter
  yy = yy + s.adaptive_y_lr * g;
  zz = z0 - s.lr * g;
}
// GB: the gradient arrives as bf16 (the all-reduced bf16 wire buffer, vpt.ddp.GradSync wire="bf16").
template <bool GB>
__device__ __forceinline__ float sf_grad(const void* grad, long i) {
  return GB ? bf2f(reinterpret_cast<const bf16_t*>(grad)[i]) : reinterpret_cast<const float*>(grad)[i];
}
template <bool GB>
__global__ void radam_sf_step_kernel(bf16_t* __restrict__ y, const void* __restrict__ grad, float* __restrict__ z,
                                     float* __restrict__ v, long n, SfScalars s) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float vv = v[i], yy = bf2f(y[i]), zz = z[i];
  sf_elem(sf_grad<GB>(grad, i), vv, yy, zz, s);
  v[i] = vv;
  z[i] = zz;
  y[i] = f2bf(yy);
}
// 4 elements per thread (16-B z / v / f32-grad, 8-B y / bf16-grad accesses) when every base is aligned for
// them: one element per lane moved 2-B y pieces and ran at ~4.4 TB/s. The last n % 4 go element-wise.
template <bool GB>
__global__ void radam_sf_step4_kernel(bf16_t* __restrict__ y, const void* __restrict__ grad, float* __restrict__ z,
                                      float* __restrict__ v, long n, SfScalars s) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  if (i + 4 > n) {
    for (long j = i; j < n; ++j) {
      float vv = v[j], yy = bf2f(y[j]), zz = z[j];
      sf_elem(sf_grad<GB>(grad, j), vv, yy, zz, s);
      v[j] = vv;
      z[j] = zz;
      y[j] = f2bf(yy);
    }
    return;
  }
  floatx4 g;
  if (GB) {
    const uint2 w = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(grad) + i);
    g[0] = __uint_as_float(w.x << 16); g[1] = __uint_as_float(w.x & 0xffff0000u);
    g[2] = __uint_as_float(w.y << 16); g[3] = __uint_as_float(w.y & 0xffff0000u);
  } else {
    g = *reinterpret_cast<const floatx4*>(reinterpret_cast<const float*>(grad) + i);
  }
  floatx4 vv = *reinterpret_cast<const floatx4*>(v + i), zz = *reinterpret_cast<const floatx4*>(z + i);
  const uint2 yw = *reinterpret_cast<const uint2*>(y + i);
  floatx4 yy;
  yy[0] = __uint_as_float(yw.x << 16); yy[1] = __uint_as_float(yw.x & 0xffff0000u);
  yy[2] = __uint_as_float(yw.y << 16); yy[3] = __uint_as_float(yw.y & 0xffff0000u);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float a = vv[e], b = yy[e], c = zz[e];
    sf_elem(g[e], a, b, c, s);
    vv[e] = a; yy[e] = b; zz[e] = c;
  }
  *reinterpret_cast<floatx4*>(v + i) = vv;
  *reinterpret_cast<floatx4*>(z + i) = zz;
  uint2 o;
  o.x = (uint32_t)f2bf(yy[0]) | ((uint32_t)f2bf(yy[1]) << 16);
  o.y = (uint32_t)f2bf(yy[2]) | ((uint32_t)f2bf(yy[3]) << 16);
  *reinterpret_cast<uint2*>(y + i) = o;
}

__global__ void lerp_to_z_kernel(bf16_t* __restrict__ y, const float* __restrict__ z, long n, float w) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float yy = bf2f(y[i]);
  y[i] = f2bf(yy + w * (z[i] - yy));
}

// EMA of the bf16 parameters (torch.optim.swa_utils.AveragedModel + get_ema_avg_fn, use_buffers=False, as
// src/trainer/common.py:211-216 / :385-386 run it on bf16 parameters): ema = bf16(bf16(d * ema) +
// bf16((1 - d) * p)) -- the foreach bf16 tensor arithmetic's roundings; the first update copies.
__global__ void ema_update_kernel(bf16_t* __restrict__ ema, const bf16_t* __restrict__ p, long n, float d, float omd,
                                  int copy) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (copy) { ema[i] = p[i]; return; }
  ema[i] = f2bf(bf2f(f2bf(d * bf2f(ema[i]))) + bf2f(f2bf(omd * bf2f(p[i]))));
}
// The same update 8 elements per thread (16-B accesses) when both bases are 16-B aligned; the tail element-wise.
__global__ void ema_update8_kernel(bf16_t* __restrict__ ema, const bf16_t* __restrict__ p, long n, float d, float omd,
                                   int copy) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  if (i + 8 > n) {
    for (long j = i; j < n; ++j)
      ema[j] = copy ? p[j] : f2bf(bf2f(f2bf(d * bf2f(ema[j]))) + bf2f(f2bf(omd * bf2f(p[j]))));
    return;
  }
  const uint4 pv = *reinterpret_cast<const uint4*>(p + i);
  if (copy) { *reinterpret_cast<uint4*>(ema + i) = pv; return; }
  const uint4 ev = *reinterpret_cast<const uint4*>(ema + i);
  const bf16_t* pe = reinterpret_cast<const bf16_t*>(&pv);
  const bf16_t* ee = reinterpret_cast<const bf16_t*>(&ev);
  uint4 o;
  bf16_t* oe = reinterpret_cast<bf16_t*>(&o);
#pragma unroll
  for (int e = 0; e < 8; ++e) oe[e] = f2bf(bf2f(f2bf(d * bf2f(ee[e]))) + bf2f(f2bf(omd * bf2f(pe[e]))));
  *reinterpret_cast<uint4*>(ema + i) = o;
}

__global__ void init_z_kernel(const bf16_t* __restrict__ y, float* __restrict__ z, float* __restrict__ v, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  z[i] = bf2f(y[i]);
  v[i] = 0.f;
}

// Copy rows [row0, row0+cnt) of every sequence of a [B][rows][D] matrix to a dense [B*cnt][D]
// matrix (reverse: the other way round, writing into the sequence layout).
__global__ void copy_rows_kernel(bf16_t* __restrict__ seq, long ld_seq, int rows, int row0, int cnt,
                                 bf16_t* __restrict__ dense, long ld_dense, int B, int D, int reverse) {
  const int nch = D >> 3;
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const int span = reverse == 2 ? rows : cnt;  // mode 2 walks every sequence row: the others are zeroed
  if (gid >= (long)B * span * nch) return;
  const int ch = gid % nch;
  const long r = gid / nch;
  const int b = r / span, jr = r % span, j = reverse == 2 ? jr - row0 : jr;
  bf16_t* s = seq + ((long)b * rows + (reverse == 2 ? jr : row0 + j)) * ld_seq + ch * 8;
  if (reverse == 2 && (j < 0 || j >= cnt)) {
    *reinterpret_cast<uint4*>(s) = make_uint4(0, 0, 0, 0);
    return;
  }
  bf16_t* d = dense + ((long)b * cnt + j) * ld_dense + ch * 8;
  if (reverse) *reinterpret_cast<uint4*>(s) = *reinterpret_cast<const uint4*>(d);
  else *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
}

// y = bf16(silu(x)); backward dx = dy * silu'(x) (x is the bf16 pre-activation).
__global__ void silu_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, bf16_t* __restrict__ out,
                            long n, int backward) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 8;
  if (i >= n) return;
  float a[8], o[8];
  unpack8(*reinterpret_cast<const uint4*>(x + i), a);
  if (!backward) {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = silu_f(a[e]);
  } else {
    float g[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + i), g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = 1.f / (1.f + expf(-a[e]));
      o[e] = g[e] * (sg * (1.f + a[e] * (1.f - sg)));
    }
  }
  *reinterpret_cast<uint4*>(out + i) = pack8(o);
}

inline dim3 grid1(long n, int threads = 256) { return dim3((unsigned)((n + threads - 1) / threads)); }

}  // namespace

extern "C" int vpt_copy_rows(void* seq, long ld_seq, int rows, int row0, int cnt, void* dense, long ld_dense, int B,
                             int D, int reverse, void* stream) {
  VPT_CHECK_ARG(seq && dense && D % 8 == 0 && row0 >= 0 && row0 + cnt <= rows && reverse >= 0 && reverse <= 2,
                "vpt_copy_rows: bad args");
  hipLaunchKernelGGL(copy_rows_kernel, grid1((long)B * (reverse == 2 ? rows : cnt) * (D / 8)), dim3(256), 0,
                     (hipStream_t)stream,
                     (bf16_t*)seq, ld_seq, rows, row0, cnt, (bf16_t*)dense, ld_dense, B, D, reverse);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_silu(const void* x, const void* dy, void* out, long n, int backward, void* stream) {
  VPT_CHECK_ARG(x && out && n % 8 == 0 && (!backward || dy), "vpt_silu: bad args");
  hipLaunchKernelGGL(silu_kernel, grid1(n / 8), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     (const bf16_t*)dy, (bf16_t*)out, n, backward);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_patchify(const void* img, int in_kind, const void* noise, const float* t, float noise_scale,
                            unsigned long long seed, int B, int H, int W, void* out, void* stream) {
  VPT_CHECK_ARG(img && out && B > 0, "vpt_patchify: bad args");
  VPT_CHECK_ARG(H % 16 == 0 && W % 16 == 0, "vpt_patchify: H and W must be multiples of the 16-px patch");
  VPT_CHECK_ARG(in_kind == 1 || t, "vpt_patchify: noising needs t");
  const long strips = (long)B * (H / 16) * ((W / 16 + kStripP - 1) / kStripP);
  VPT_CHECK_ARG(strips < (1L << 31), "vpt_patchify: too many strips");
  auto kern = in_kind == 1 ? patchify_kernel<3> : noise ? patchify_kernel<2> : noise_scale == 1.f ? patchify_kernel<0>
                                                                                                  : patchify_kernel<1>;
  hipLaunchKernelGGL(kern, dim3((unsigned)strips), dim3(kPatchThreads), 0, (hipStream_t)stream,
                     (const unsigned short*)img, (const unsigned short*)noise, t, noise_scale, (uint64_t)seed, B, H, W,
                     (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_unpatchify(const void* patches, int B, int H, int W, void* img, int reverse, void* stream) {
  VPT_CHECK_ARG(patches && img && H % 16 == 0 && W % 16 == 0, "vpt_unpatchify: bad args");
  const long total = (long)B * 3 * H * W;
  hipLaunchKernelGGL(unpatchify_kernel, grid1(total), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)patches, B, H,
                     W, (bf16_t*)img, reverse);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_euler_cfg_step(void* z, const void* pred, int B, int H, int W, int cfg, float cfg_scale, int mode,
                                  float t, float dt, void* stream) {
  VPT_CHECK_ARG(z && pred && B > 0 && H % 16 == 0 && W % 16 == 0 && (mode == 0 || mode == 1),
                "vpt_euler_cfg_step: bad args");
  const long total = (long)B * 3 * H * W;
  hipLaunchKernelGGL(euler_cfg_kernel, grid1(total), dim3(256), 0, (hipStream_t)stream, (bf16_t*)z,
                     (const bf16_t*)pred, B, H, W, cfg, cfg_scale, mode, t, dt);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_add_bf16(const void* a, const void* b, long n, void* out, void* stream) {
  VPT_CHECK_ARG(a && b && out && n % 8 == 0, "vpt_add_bf16: n must be a multiple of 8");
  hipLaunchKernelGGL(add_bf16_kernel, grid1(n / 8), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)a,
                     (const bf16_t*)b, n / 8, (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_scale_bf16(const void* a, long n, float s, void* out, void* stream) {
  VPT_CHECK_ARG(a && out && n % 8 == 0, "vpt_scale_bf16: n must be a multiple of 8");
  hipLaunchKernelGGL(scale_bf16_kernel, grid1(n / 8), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)a, n / 8, s,
                     (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_scale_bf16_2d(const void* a, long lda, long rows, int cols, float s, void* out, long ldo,
                                 void* stream) {
  VPT_CHECK_ARG(a && out && rows > 0 && cols > 0 && cols % 8 == 0 && lda % 8 == 0 && ldo % 8 == 0,
                "vpt_scale_bf16_2d: cols and leading dims must be multiples of 8");
  const long n8 = rows * (cols / 8);
  hipLaunchKernelGGL(scale_bf16_2d_kernel, grid1(n8), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)a, lda, rows,
                     cols / 8, s, (bf16_t*)out, ldo);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_area_lowres(const void* img, const void* noise, const float* t, float noise_scale,
                               unsigned long long seed, int B, int H, int W, int k, void* img_lr, void* noise_lr,
                               void* z_lr, void* stream) {
  VPT_CHECK_ARG(img && t && img_lr && noise_lr && z_lr && B > 0, "vpt_area_lowres: null pointer");
  VPT_CHECK_ARG(k >= 2 && k % 2 == 0 && H % k == 0 && W % k == 0,
                "vpt_area_lowres: the factor must be even and divide H and W");
  const long n = (long)B * 3 * (H / k) * (W / k);
  hipLaunchKernelGGL(area_lowres_kernel, grid1(n), dim3(256), 0, (hipStream_t)stream, (const unsigned short*)img,
                     (const unsigned short*)noise, t, noise_scale, (uint64_t)seed, B, H, W, k,
                     (unsigned short*)img_lr, (unsigned short*)noise_lr, (bf16_t*)z_lr);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_gauss_noise(long n, unsigned long long seed, float noise_scale, void* out, void* stream) {
  VPT_CHECK_ARG(out && n >= 0 && n % 2 == 0, "vpt_gauss_noise: n must be even");
  if (n == 0) return VPT_OK;
  hipLaunchKernelGGL(gauss_noise_kernel, grid1(n / 2), dim3(256), 0, (hipStream_t)stream, n / 2, (uint64_t)seed,
                     noise_scale, (unsigned short*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_loss_blocks(void) { return kLossBlocks; }

extern "C" int vpt_flow_loss(const void* pred, const void* img, const void* noise, const float* t, float noise_scale,
                             unsigned long long seed, int target, float t_eps, int B, int H, int W, void* dpred,
                             float* part, float* loss, void* stream) {
  VPT_CHECK_ARG(pred && img && t && dpred && part && loss, "vpt_flow_loss: null pointer");
  VPT_CHECK_ARG(target >= 0 && target <= 2,
                "vpt_flow_loss: target must be 0 (image), 1 (velocity of an image prediction) or 2 (velocity prediction)");
  VPT_CHECK_ARG(B > 0 && H % 16 == 0 && W % 16 == 0, "vpt_flow_loss: H and W must be multiples of the 16-px patch");
  const float numel = (float)B * 3.f * H * W;
  const long strips = (long)B * (H / 16) * ((W / 16 + kStripP - 1) / kStripP);
  const int blocks = (int)(strips < kLossBlocks ? strips : kLossBlocks);  // partials part[0, blocks)
  hipStream_t s = (hipStream_t)stream;
  auto kern = target == 0 ? loss_kernel<0> : target == 1 ? loss_kernel<1> : loss_kernel<2>;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kLossThreads), 0, s, (const bf16_t*)pred, (const unsigned short*)img,
                     (const unsigned short*)noise, t, noise_scale, (uint64_t)seed, t_eps, B, H, W, 1.f / numel,
                     (bf16_t*)dpred, part);
  VPT_LAUNCH_CHECK();
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(kFinThreads), 0, s, part, blocks, 1.f / numel, loss);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_timestep_embed(const float* vals, int R, void* out, void* stream) {
  VPT_CHECK_ARG(vals && out && R > 0, "vpt_timestep_embed: bad args");
  hipLaunchKernelGGL(timestep_embed_kernel, grid1((long)R * 256), dim3(256), 0, (hipStream_t)stream, vals, R,
                     (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_assemble_tokens(const void* patches, const void* size_emb, const void* time_emb, const void* tpe,
                                   const void* ctx, int n_ctx, int B, int np_, int rows, int D, void* x,
                                   void* stream) {
  VPT_CHECK_ARG(patches && size_emb && time_emb && tpe && x, "vpt_assemble_tokens: null pointer");
  VPT_CHECK_ARG(rows >= np_ + 10 && D % 8 == 0 && D > 0, "vpt_assemble_tokens: rows too small or D % 8 != 0");
  hipLaunchKernelGGL(assemble_kernel, grid1((long)B * rows * (D / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)patches, (const bf16_t*)size_emb, (const bf16_t*)time_emb, (const bf16_t*)tpe,
                     (const bf16_t*)ctx, n_ctx, B, np_, rows, D, (bf16_t*)x);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_disassemble_tokens(const void* dx, int B, int np_, int rows, int D, void* dpatches, void* dsize,
                                      void* dtime, float* dtpe, void* stream) {
  VPT_CHECK_ARG(dx && dpatches && dsize && dtime && D % 8 == 0 && D > 0, "vpt_disassemble_tokens: bad args");
  hipLaunchKernelGGL(disassemble_kernel, grid1((long)B * (np_ + 7) * (D / 8)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)dx, B, np_, rows, D, (bf16_t*)dpatches, (bf16_t*)dsize, (bf16_t*)dtime, dtpe);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_ctx_rows(void* x, int B, int row0, int rows, int D, const void* ctx, float* dctx, int n_ctx,
                            int backward, void* stream) {
  VPT_CHECK_ARG(x && n_ctx > 0 && D % 8 == 0 && row0 + n_ctx <= rows && (backward ? dctx != nullptr : ctx != nullptr),
                "vpt_ctx_rows: bad args");
  hipLaunchKernelGGL(ctx_rows_kernel, grid1((long)B * n_ctx * (D / 8)), dim3(256), 0, (hipStream_t)stream, (bf16_t*)x,
                     B, row0, rows, D, (const bf16_t*)ctx, dctx, n_ctx, backward);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_swiglu_fwd(const void* x12, long M, int F, void* h, void* stream) {
  VPT_CHECK_ARG(x12 && h && F % 8 == 0, "vpt_swiglu_fwd: bad args");
  hipLaunchKernelGGL(swiglu_fwd_kernel, grid1(M * (F / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x12, M,
                     F, (bf16_t*)h);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_swiglu_bwd(const void* dh, const void* x12, long M, int F, void* dx12, void* stream) {
  VPT_CHECK_ARG(dh && x12 && dx12 && F % 8 == 0, "vpt_swiglu_bwd: bad args");
  hipLaunchKernelGGL(swiglu_bwd_kernel, grid1(M * (F / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)dh,
                     (const bf16_t*)x12, M, F, (bf16_t*)dx12);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_colsum_blocks(long M) {  // number of partial rows written by vpt_colsum
  // up to 256 row slices of >= 128 rows: with the (N/256)-wide column grid this keeps >= 3 blocks per
  // CU even at N = 768
  long b = (M + 127) / 128;
  return (int)(b > 256 ? 256 : (b < 1 ? 1 : b));
}

extern "C" int vpt_reduce_rows(const float* in, int R, int C, float* out, int accumulate, void* stream);

extern "C" int vpt_bias_grad(const void* in, long ld, long M, int N, float* part, float* out, int accumulate,
                             void* stream) {
  VPT_CHECK_ARG(in && part && out && N % 8 == 0 && M > 0, "vpt_bias_grad: bad args");
  const int nb = vpt_colsum_blocks(M);
  const long per = (M + nb - 1) / nb;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 255) / 256, nb), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)in,
                     ld, M, N, per, part);
  VPT_LAUNCH_CHECK();
  return vpt_reduce_rows(part, nb, N, out, accumulate, stream);
}

extern "C" int vpt_embed_gather(const void* table, const long long* ids, long R, int D, void* out, void* stream) {
  VPT_CHECK_ARG(table && ids && out && D % 8 == 0, "vpt_embed_gather: bad args");
  hipLaunchKernelGGL(embed_gather_kernel, grid1(R * (D / 8)), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)table,
                     (const int64_t*)ids, R, D, (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_embed_scatter_add(const void* drows, const long long* ids, long R, int D, long long pad_id,
                                     float* dtable, void* stream) {
  VPT_CHECK_ARG(drows && ids && dtable, "vpt_embed_scatter_add: bad args");
  hipLaunchKernelGGL(embed_scatter_kernel, grid1(R * D), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)drows,
                     (const int64_t*)ids, R, D, (long)pad_id, dtable);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_embed_grad_set(const void* drows, const long long* ids, long R, int D, long long pad_id, long V,
                                  int accumulate, float* dtable, void* stream) {
  VPT_CHECK_ARG((drows || R == 0) && (ids || R == 0) && dtable && D % 4 == 0 && V > 0, "vpt_embed_grad_set: bad args");
  VPT_CHECK_ARG(R >= 0 && R <= 16384, "vpt_embed_grad_set: R <= 16384 ids (LDS position lists)");
  hipLaunchKernelGGL(embed_grad_set_kernel, dim3((unsigned)((V + kEmbRows - 1) / kEmbRows)), dim3(kEmbThreads),
                     (size_t)(R > 0 ? R : 1) * sizeof(int), (hipStream_t)stream, (const bf16_t*)drows,
                     (const int64_t*)ids, (int)R, D, (long)pad_id, V, accumulate, dtable);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_step_inputs(const float* t, int B, float tscale, const long long* orig, const long long* target,
                               const long long* crop, float* t_vals, float* size_vals, const long long* mask, int n_ctx,
                               int n_pre, int rows, float* kbias, void* stream) {
  VPT_CHECK_ARG(t && orig && target && crop && t_vals && size_vals && kbias && B > 0 && n_ctx >= 0 && n_pre >= 0 &&
                n_pre + n_ctx <= rows, "vpt_step_inputs: bad args");
  const long n = (long)B * (n_pre + n_ctx) + 7L * B;
  hipLaunchKernelGGL(step_inputs_kernel, grid1(n), dim3(256), 0, (hipStream_t)stream, t, B, tscale,
                     (const int64_t*)orig, (const int64_t*)target, (const int64_t*)crop, t_vals, size_vals,
                     (const int64_t*)mask, n_ctx, n_pre, rows, kbias);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_cast_f32_bf16(const float* in, long n, void* out, void* stream) {
  VPT_CHECK_ARG(in && out && n % 4 == 0, "vpt_cast_f32_bf16: n must be a multiple of 4");
  hipLaunchKernelGGL(cast_f32_bf16_kernel, grid1(n / 4), dim3(256), 0, (hipStream_t)stream, in, n, (bf16_t*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_radam_sf_step(void* y, const void* grad, int grad_bf16, float* z, float* v, long n, float beta2,
                                 float bias_correction2, float eps, float ckp1, float adaptive_y_lr, float lr,
                                 float decay, float grad_scale, int adam, const float* clip_coef, float clip_value,
                                 void* stream) {
  VPT_CHECK_ARG(y && grad && z && v && n >= 0 && clip_value >= 0.f, "vpt_radam_sf_step: bad args");
  if (n == 0) return VPT_OK;
  SfScalars s{beta2, bias_correction2, eps, ckp1, adaptive_y_lr, lr, decay, grad_scale, adam, clip_coef, clip_value};
  auto al = [](const void* p, uintptr_t a) { return ((uintptr_t)p & (a - 1)) == 0; };
  const bool vec = al(y, 8) && al(z, 16) && al(v, 16) && al(grad, grad_bf16 ? 8 : 16);
  hipStream_t st = (hipStream_t)stream;
  if (vec && grad_bf16)
    hipLaunchKernelGGL(radam_sf_step4_kernel<true>, grid1((n + 3) / 4), dim3(256), 0, st, (bf16_t*)y, grad, z, v, n, s);
  else if (vec)
    hipLaunchKernelGGL(radam_sf_step4_kernel<false>, grid1((n + 3) / 4), dim3(256), 0, st, (bf16_t*)y, grad, z, v, n, s);
  else if (grad_bf16)
    hipLaunchKernelGGL(radam_sf_step_kernel<true>, grid1(n), dim3(256), 0, st, (bf16_t*)y, grad, z, v, n, s);
  else
    hipLaunchKernelGGL(radam_sf_step_kernel<false>, grid1(n), dim3(256), 0, st, (bf16_t*)y, grad, z, v, n, s);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

// ---------------------------------------------------------------- gradient clipping (global L2 norm)
// Per-bucket partial sums of squares: block j of kGradNormBlocks grid-strides over the bucket and writes
// its sum to part[j] (fixed assignment and order -> deterministic; no atomics).
constexpr int kGradNormBlocks = 256;
template <bool GB>
__global__ void grad_sumsq_kernel(const void* __restrict__ g, long n, float scale, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = (GB ? bf2f(reinterpret_cast<const bf16_t*>(g)[i]) : reinterpret_cast<const float*>(g)[i]) * scale;
    s += x * x;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
// coef = min(1, max_norm / (sqrt(sum of all partials) + 1e-6)) (torch.nn.utils.clip_grad_norm_), one block;
// norm_out (optional) receives the total norm.
__global__ void clip_coef_kernel(const float* __restrict__ part, int n, float max_norm, float* __restrict__ coef,
                                 float* __restrict__ norm_out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf((red[0] + red[1]) + (red[2] + red[3]));
    *coef = fminf(max_norm / (norm + 1e-6f), 1.f);
    if (norm_out) *norm_out = norm;
  }
}

extern "C" int vpt_grad_norm_blocks(void) { return kGradNormBlocks; }

extern "C" int vpt_grad_sumsq(const void* g, int g_bf16, long n, float scale, float* part, void* stream) {
  VPT_CHECK_ARG(g && part && n >= 0, "vpt_grad_sumsq: bad args");
  if (g_bf16)
    hipLaunchKernelGGL(grad_sumsq_kernel<true>, dim3(kGradNormBlocks), dim3(256), 0, (hipStream_t)stream, g, n, scale,
                       part);
  else
    hipLaunchKernelGGL(grad_sumsq_kernel<false>, dim3(kGradNormBlocks), dim3(256), 0, (hipStream_t)stream, g, n, scale,
                       part);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_clip_coef(const float* part, int n, float max_norm, float* coef, float* norm_out, void* stream) {
  VPT_CHECK_ARG(part && coef && n > 0 && max_norm > 0.f, "vpt_clip_coef: bad args");
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, n, max_norm, coef, norm_out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_sf_lerp(void* y, const float* z, long n, float w, void* stream) {
  VPT_CHECK_ARG(y && z, "vpt_sf_lerp: bad args");
  if (n == 0) return VPT_OK;
  hipLaunchKernelGGL(lerp_to_z_kernel, grid1(n), dim3(256), 0, (hipStream_t)stream, (bf16_t*)y, z, n, w);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_ema_update(void* ema, const void* param, long n, float decay, float one_minus_decay, int first,
                              void* stream) {
  VPT_CHECK_ARG(ema && param && decay >= 0.f && decay <= 1.f && one_minus_decay >= 0.f && one_minus_decay <= 1.f,
                "vpt_ema_update: bad args");
  if (n == 0) return VPT_OK;
  if ((((uintptr_t)ema | (uintptr_t)param) & 15) == 0)
    hipLaunchKernelGGL(ema_update8_kernel, grid1((n + 7) / 8), dim3(256), 0, (hipStream_t)stream, (bf16_t*)ema,
                       (const bf16_t*)param, n, decay, one_minus_decay, first);
  else
    hipLaunchKernelGGL(ema_update_kernel, grid1(n), dim3(256), 0, (hipStream_t)stream, (bf16_t*)ema,
                       (const bf16_t*)param, n, decay, one_minus_decay, first);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_sf_init(const void* y, float* z, float* v, long n, void* stream) {
  VPT_CHECK_ARG(y && z && v, "vpt_sf_init: bad args");
  if (n == 0) return VPT_OK;
  hipLaunchKernelGGL(init_z_kernel, grid1(n), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)y, z, v, n);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
