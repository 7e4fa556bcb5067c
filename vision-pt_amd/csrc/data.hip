// Bucketed-batch image preparation on the device: decoded uint8 RGB images become the
// fp16 [3][h][w] crops of their aspect-ratio bucket, written straight into the training batch.
//
// Replaces, per image, the reference's CPU transform chain (src/dataset/text_to_image.py:145-158,
// :164-177, :199-213): PILToTensor -> ToDtype(float16, scale=True) -> Normalize(0.5, 0.5) ->
// ObjectCoverResize (src/dataset/transform.py:11-55: bicubic, antialias, to the smallest size that covers
// the bucket) -> RandomCrop to the bucket. Only the crop window is computed: the horizontal pass covers
// the input rows the vertical filter of the cropped output rows touches.
//
// Arithmetic follows the ATen antialiased bicubic kernel that torchvision's resize calls for float
// images (separable, horizontal pass first into an f32 temporary, Keys a = -0.5 filter stretched by the
// downscale factor, weights normalised to sum 1, a dimension of unchanged size is not resampled), on the
// fp16-rounded normalised input; the f32 result is rounded to fp16 once.
#include "common.h"

#include <algorithm>

namespace {

constexpr int MAX_TAPS = 64;  // support of a 15x downscale

__device__ __forceinline__ float aa_bicubic(float x) {
  const float a = -0.5f;
  x = fabsf(x);
  if (x < 1.f) return ((a + 2.f) * x - (a + 3.f)) * x * x + 1.f;
  if (x < 2.f) return ((a * x - 5.f * a) * x + 8.f * a) * x - 4.f * a;
  return 0.f;
}

// Weight table of a resize in_size -> out_size restricted to output indices [i0, i0 + count): row k holds
// (first input index, tap count) as ints, then up to MAX_TAPS normalised weights (ATen
// _compute_indices_min_size_weights_aa order: center, support, xmin / xsize truncations, sum, divide).
constexpr int TAB = 2 + MAX_TAPS;
__global__ void aa_table_kernel(int in_size, int out_size, int i0, int count, float* __restrict__ tab) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= count) return;
  float* row = tab + (long)k * TAB;
  const int i = i0 + k;
  if (in_size == out_size) {  // unchanged dimension: not resampled
    row[0] = __int_as_float(i);
    row[1] = __int_as_float(1);
    row[2] = 1.f;
    return;
  }
  const float scale = (float)in_size / (float)out_size;
  const float support = scale >= 1.f ? 2.f * scale : 2.f;
  const float invscale = scale >= 1.f ? 1.f / scale : 1.f;
  const float center = scale * (i + 0.5f);
  const int xmin = max((int)(center - support + 0.5f), 0);
  const int xsize = min(min((int)(center + support + 0.5f), in_size) - xmin, MAX_TAPS);
  float total = 0.f;
  for (int j = 0; j < xsize; ++j) {
    const float v = aa_bicubic((j + xmin - center + 0.5f) * invscale);
    row[2 + j] = v;
    total += v;
  }
  if (total != 0.f)
    for (int j = 0; j < xsize; ++j) row[2 + j] /= total;
  row[0] = __int_as_float(xmin);
  row[1] = __int_as_float(xsize);
}

// PILToTensor -> ToDtype(float16, scale=True) -> Normalize(mean 0.5, std 0.5), each step rounded to fp16
// as the reference's fp16 tensors are.
__device__ __forceinline__ float norm_u8(unsigned v) {
  const float x = h2f(f2h((float)v * (1.f / 255.f)));
  return h2f(f2h(h2f(f2h(x - 0.5f)) / 0.5f));
}

// Horizontal pass: tmp[r - r0][c][x] for input rows r in [r0, r0 + rows), cropped output columns
// x in [0, out_w) of the width-resampled image (htab row x = output column left + x).
__global__ void resize_h_kernel(const unsigned char* __restrict__ img, int in_w, const float* __restrict__ htab,
                                int r0, int rows, int out_w, float* __restrict__ tmp) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= out_w) return;
  const float* tw = htab + (long)x * TAB;
  const int xmin = __float_as_int(tw[0]), n = __float_as_int(tw[1]);
  for (int r = blockIdx.y; r < rows; r += gridDim.y) {
    const unsigned char* p = img + ((long)(r0 + r) * in_w + xmin) * 3;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int j = 0; j < n; ++j) {
      const float wj = tw[2 + j];
#pragma unroll
      for (int c = 0; c < 3; ++c) acc[c] += wj * norm_u8(p[3 * j + c]);
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) tmp[((long)r * 3 + c) * out_w + x] = acc[c];
  }
}

// Vertical pass: out[c][y][x] = sum_j wv_j * tmp[ymin + j - r0][c][x], rounded to fp16 once.
__global__ void resize_v_kernel(const float* __restrict__ tmp, const float* __restrict__ vtab, int r0, int out_h,
                                int out_w, unsigned short* __restrict__ out) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= out_w || y >= out_h) return;
  const float* tw = vtab + (long)y * TAB;
  const int ymin = __float_as_int(tw[0]), n = __float_as_int(tw[1]);
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float acc = 0.f;
    for (int j = 0; j < n; ++j) acc += tw[2 + j] * tmp[((long)(ymin + j - r0) * 3 + c) * out_w + x];
    out[((long)c * out_h + y) * out_w + x] = f2h(acc);
  }
}

// Input rows [r0, r1) that the vertical filter of output rows [top, top + out_h) reads, with one row of
// slack each side (the device computes the exact ranges; the slack absorbs host/device rounding).
void v_rows(int in_h, int scaled_h, int top, int out_h, int& r0, int& r1) {
  if (scaled_h == in_h) {
    r0 = top;
    r1 = top + out_h;
    return;
  }
  const float scale = (float)in_h / (float)scaled_h;
  const float support = scale >= 1.f ? 2.f * scale : 2.f;
  const float c0 = scale * (top + 0.5f), c1 = scale * (top + out_h - 1 + 0.5f);
  r0 = std::max((int)(c0 - support + 0.5f) - 1, 0);
  r1 = std::min((int)(c1 + support + 0.5f) + 1, in_h);
}

int taps_ok(int in_size, int out_size) {
  const float scale = (float)in_size / (float)out_size;
  return (scale >= 1.f ? 4.f * scale + 2.f : 6.f) <= (float)MAX_TAPS;
}

}  // namespace

extern "C" long vpt_cover_resize_crop_workspace(int in_h, int in_w, int scaled_h, int scaled_w, int top, int out_h,
                                                int out_w) {
  (void)in_w; (void)scaled_w;
  int r0, r1;
  v_rows(in_h, scaled_h, top, out_h, r0, r1);
  return ((long)(r1 - r0) * 3 * out_w + (long)(out_w + out_h) * TAB) * (long)sizeof(float);
}

// img: uint8 [in_h][in_w][3] (RGB, HWC as decoded); the image is resized to (scaled_h, scaled_w) and the
// window rows [top, top + out_h) x columns [left, left + out_w) is written to out: fp16 [3][out_h][out_w]
// (one slot of the [B][3][h][w] batch). workspace: vpt_cover_resize_crop_workspace() bytes.
extern "C" int vpt_cover_resize_crop(const void* img, int in_h, int in_w, int scaled_h, int scaled_w, int top, int left,
                                     int out_h, int out_w, void* workspace, void* out, void* stream) {
  VPT_CHECK_ARG(img && workspace && out, "vpt_cover_resize_crop: null pointer");
  VPT_CHECK_ARG(in_h > 0 && in_w > 0 && out_h > 0 && out_w > 0, "vpt_cover_resize_crop: empty shape");
  VPT_CHECK_ARG(top >= 0 && left >= 0 && top + out_h <= scaled_h && left + out_w <= scaled_w,
                "vpt_cover_resize_crop: crop window outside the resized image");
  VPT_CHECK_ARG(taps_ok(in_h, scaled_h) && taps_ok(in_w, scaled_w),
                "vpt_cover_resize_crop: downscale factor above 15 (filter taps)");
  int r0, r1;
  v_rows(in_h, scaled_h, top, out_h, r0, r1);
  float* tmp = (float*)workspace;
  float* htab = tmp + (long)(r1 - r0) * 3 * out_w;
  float* vtab = htab + (long)out_w * TAB;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(aa_table_kernel, dim3((out_w + 127) / 128), dim3(128), 0, s, in_w, scaled_w, left, out_w, htab);
  hipLaunchKernelGGL(aa_table_kernel, dim3((out_h + 127) / 128), dim3(128), 0, s, in_h, scaled_h, top, out_h, vtab);
  VPT_LAUNCH_CHECK();
  const dim3 gh((out_w + 127) / 128, std::min(r1 - r0, 1024));
  hipLaunchKernelGGL(resize_h_kernel, gh, dim3(128), 0, s, (const unsigned char*)img, in_w, (const float*)htab, r0,
                     r1 - r0, out_w, tmp);
  VPT_LAUNCH_CHECK();
  const dim3 gv((out_w + 127) / 128, out_h);
  hipLaunchKernelGGL(resize_v_kernel, gv, dim3(128), 0, s, (const float*)tmp, (const float*)vtab, r0, out_h, out_w,
                     (unsigned short*)out);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
