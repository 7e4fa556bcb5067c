// MFMA bf16 GEMM for gfx950: C[M,N] = sum_k A(m,k) * B(n,k)  (+bias, +residual, SiLU).
//
// Replaces every nn.Linear / 1x1-conv matmul on the JiT training path
// (reference: src/models/jit/denoiser.py:36-49,59-65 patch-embed convs, :80-84 time MLP,
// :318-323/:360-366/:391-395 attention projections, :492-504 SwiGLU, :535-543 final layer)
// in all three directions of a Linear:
//   forward  Y  = X  . W^T : A = X  [M][K] (k-major),  B = W [N][K] (k-major)
//   dgrad    dX = dY . W   : A = dY [M][N] (k-major),  B = W [N][K] stored [red][out] (mn-major)
//   wgrad    dW = dY^T . X : A = dY stored [red][out], B = X stored [red][out] (both mn-major)
//
// Tile 128x128x64, 256 threads = 4 waves in 2x2, each wave 64x64 = 4x4 MFMA 16x16x32 bf16.
// k-major tiles are staged [row][64k] (128 B rows, 16-B chunk XOR swizzle, read with
// ds_read_b128); mn-major tiles are staged in their global [k][128mn] orientation (256 B rows,
// 8-B unit XOR swizzle) and read with ds_read_b64_tr_b16, which delivers the transpose.
// Register-staged double buffering, one barrier per K step, XCD-aware block remap,
// epilogue staged through LDS so bias/residual/activation and stores are 8-16 B per lane.
// Optional split-K writes f32 partial slabs (reduced by vpt_splitk_reduce).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int EPI_LD = 68;                         // f32 staging row stride (floats), conflict-free
constexpr int LDS_MAIN = 2 * 2 * 16384;            // [buf][A/B] 16 KB tiles
constexpr int LDS_EPI = 4 * 64 * EPI_LD * 4;       // 4 waves x 64x68 f32
constexpr int LDS_BYTES = LDS_MAIN > LDS_EPI ? LDS_MAIN : LDS_EPI;

enum { OUT_BF16 = 0, OUT_F32 = 1, OUT_F32_ACC = 2 };
enum { ACT_NONE = 0, ACT_SILU = 1 };

struct GemmArgs {
  const bf16_t* A; long lda;
  const bf16_t* B; long ldb;
  void* C; long ldc;
  const bf16_t* bias;
  const bf16_t* resid; long ldr;
  int M, N, K;
  int k_split;          // reduction length per split slice (multiple of BK)
  long split_stride;    // elements between partial slabs (f32 outputs)
  int out_mode, act;
};

__device__ __forceinline__ int kmaj_off(int row, int chunk) {  // bytes in a [128][64] bf16 tile
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ int mnmaj_f(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
__device__ __forceinline__ int mnmaj_off(int krow, int unit) {   // bytes in a [64][128] bf16 tile
  return krow * 256 + ((unit ^ (mnmaj_f(krow) << 2)) << 3);
}

// Loads one operand tile (rows = output dim, 128 of them; 64 along k) into 4 uint4 registers.
template <bool KMAJ>
__device__ __forceinline__ void load_tile(uint4 (&r)[4], const bf16_t* __restrict__ base, long ld,
                                          int row0, int nrows, int k0, int kend, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    if (KMAJ) {
      const int row = c >> 3, kc = c & 7;
      const int gr = row0 + row, gk = k0 + kc * 8;
      if (gr < nrows && gk < kend)
        r[i] = *reinterpret_cast<const uint4*>(base + (long)gr * ld + gk);
      else
        r[i] = make_uint4(0, 0, 0, 0);
    } else {
      const int krow = c >> 4, mc = c & 15;
      const int gk = k0 + krow, gm = row0 + mc * 8;
      if (gk < kend && gm < nrows)
        r[i] = *reinterpret_cast<const uint4*>(base + (long)gk * ld + gm);
      else
        r[i] = make_uint4(0, 0, 0, 0);
    }
  }
}

template <bool KMAJ>
__device__ __forceinline__ void store_tile(char* lds, const uint4 (&r)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + 256 * i;
    int off;
    if (KMAJ) {
      off = kmaj_off(c >> 3, c & 7);
    } else {
      off = mnmaj_off(c >> 4, (c & 15) * 2);
    }
    *reinterpret_cast<uint4*>(lds + off) = r[i];
  }
}

// LDS-DMA staging of one full 64-deep operand tile (16 KB = 16 wave-instructions of 1 KB; wave `wid`
// issues 4). The LDS image is written lane-linearly (dst = base + 16*lane), so the XOR swizzle of
// kmaj_off / mnmaj_off is applied to each lane's GLOBAL source address instead (guide rule 21).
// Rows past the matrix edge are clamped to a valid row: they only feed output rows/cols that are
// never stored. K must be a full tile here (partial K tiles go through load_tile/store_tile).
// One 16-B-per-lane LDS-DMA (1 KB per wave) in inline asm, so that hipcc's waitcnt pass does not
// serialise it against the ds_reads of the other buffer (it cannot prove the two do not alias);
// completion is waited for explicitly with `s_waitcnt vmcnt(0)` before the K-step barrier.
// M0 holds the wave-uniform LDS destination and is restored (guide §5.7 LDS-DMA recipe).
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_addr)
               : "memory");
}

template <bool KMAJ>
__device__ __forceinline__ void glds_tile(char* lds, const bf16_t* __restrict__ base, long ld, int row0, int nrows,
                                          int k0, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wid * 4 + i;
    const bf16_t* src;
    if (KMAJ) {
      const int row = q * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((row >> 1) & 7);
      int gr = row0 + row;
      gr = gr < nrows ? gr : nrows - 1;
      src = base + (long)gr * ld + k0 + c * 8;
    } else {
      const int krow = q * 4 + (lane >> 4);
      const int c = (lane & 15) ^ (mnmaj_f(krow) << 1);
      int gm = row0 + c * 8;
      gm = gm < nrows ? gm : 0;
      src = base + (long)(k0 + krow) * ld + gm;
    }
    const uint32_t dst = (uint32_t)(uintptr_t)(VPT_LDS char*)(lds + q * 1024);
    glds16((const void*)src, __builtin_amdgcn_readfirstlane(dst));
  }
}

// Fragment for a 16(row) x 32(k) MFMA operand: lane holds row (lane&15), k = 8*(lane>>4)+0..7.
template <bool KMAJ>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int row_base, int kk, int lane) {
  if (KMAJ) {
    const int row = row_base + (lane & 15);
    const int chunk = kk * 4 + (lane >> 4);
    return as_frag(*reinterpret_cast<const uint4*>(lds + kmaj_off(row, chunk)));
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int unit = (row_base >> 2) + p;
    const int k0 = kk * 32 + 8 * g + q;
    uint2 lo = lds_read_tr16((const VPT_LDS void*)(lds + mnmaj_off(k0, unit)));
    uint2 hi = lds_read_tr16((const VPT_LDS void*)(lds + mnmaj_off(k0 + 4, unit)));
    return as_frag2(lo, hi);
  }
}

// One 64-deep K step of the block tile: each wave reads its 4 A and 4 B fragments per 32-k half
// and issues 16 MFMA 16x16x32 into its 64x64 accumulator.
template <bool AK, bool BK_>
__device__ __forceinline__ void mma_tile(const char* la, floatx4 (&acc)[4][4], int wm, int wn, int lane) {
  const char* lb = la + 16384;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = read_frag<AK>(la, wm * 64 + i * 16, kk, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = read_frag<BK_>(lb, wn * 64 + j * 16, kk, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
  }
}

template <bool AK, bool BK_>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_n = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tm = wgid / tiles_n, tn = wgid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const int kbeg = blockIdx.y * g.k_split;
  const int kend = min(g.K, kbeg + g.k_split);
  const int nfull = (kend - kbeg) / BK;
  const bool ktail = (kend - kbeg) % BK != 0;
  const int nk = nfull + (ktail ? 1 : 0);

  floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Main loop over the full K tiles: LDS-DMA only (no ordinary VGPR loads in the loop, so hipcc
  // does not insert a vmcnt(0) ahead of the ds_reads); the next tile lands while this one computes.
  int cur = 0;
  if (nfull > 0) {
    glds_tile<AK>(smem, g.A, g.lda, m0, g.M, kbeg, wid, lane);
    glds_tile<BK_>(smem + 16384, g.B, g.ldb, n0, g.N, kbeg, wid, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int kt = 0; kt < nfull; ++kt) {
    if (kt + 1 < nfull) {
      char* nb = smem + (cur ^ 1) * 32768;
      const int kn = kbeg + (kt + 1) * BK;
      glds_tile<AK>(nb, g.A, g.lda, m0, g.M, kn, wid, lane);
      glds_tile<BK_>(nb + 16384, g.B, g.ldb, n0, g.N, kn, wid, lane);
    }
    mma_tile<AK, BK_>(smem + cur * 32768, acc, wm, wn, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA for tile kt+1 has landed
    __syncthreads();                                   // ... and every other wave's too
    cur ^= 1;
  }
  // Partial last K tile (wgrad over a token count that is not a multiple of 64): zero-filled
  // register loads into the free buffer.
  if (ktail) {
    uint4 ra[4], rb[4];
    const int kn = kbeg + nfull * BK;
    load_tile<AK>(ra, g.A, g.lda, m0, g.M, kn, kend, tid);
    load_tile<BK_>(rb, g.B, g.ldb, n0, g.N, kn, kend, tid);
    store_tile<AK>(smem + cur * 32768, ra, tid);
    store_tile<BK_>(smem + cur * 32768 + 16384, rb, tid);
    __syncthreads();
    mma_tile<AK, BK_>(smem + cur * 32768, acc, wm, wn, lane);
    __syncthreads();
  }

  // ---- epilogue: stage the wave's 64x64 f32 tile in LDS, then vectorised row pass ----
  float* st = reinterpret_cast<float*>(smem) + wid * 64 * EPI_LD;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        st[(i * 16 + (lane >> 4) * 4 + r) * EPI_LD + j * 16 + (lane & 15)] = acc[i][j][r];
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes retired
  __builtin_amdgcn_wave_barrier();

  const int col = n0 + wn * 64 + (lane & 15) * 4;
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  const bool col_ok = col < g.N;
  if (g.bias && col_ok) {
    const uint2 bv = *reinterpret_cast<const uint2*>(g.bias + col);
    bias4[0] = __uint_as_float(bv.x << 16); bias4[1] = __uint_as_float(bv.x & 0xffff0000u);
    bias4[2] = __uint_as_float(bv.y << 16); bias4[3] = __uint_as_float(bv.y & 0xffff0000u);
  }
  for (int pass = 0; pass < 16; ++pass) {
    const int lr = pass * 4 + (lane >> 4);
    const int row = m0 + wm * 64 + lr;
    if (row >= g.M || !col_ok) continue;
    floatx4 v = *reinterpret_cast<const floatx4*>(st + lr * EPI_LD + (lane & 15) * 4);
    float o[4] = {v[0] + bias4[0], v[1] + bias4[1], v[2] + bias4[2], v[3] + bias4[3]};
    if (g.act == ACT_SILU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = o[e] / (1.f + __expf(-o[e]));
    }
    if (g.out_mode == OUT_BF16) {
      bf16_t* C = reinterpret_cast<bf16_t*>(g.C);
      if (g.resid) {
        const uint2 rv = *reinterpret_cast<const uint2*>(g.resid + (long)row * g.ldr + col);
        // reference semantics: residual + bf16(linear output), rounded again to bf16
        o[0] = bf2f(f2bf(o[0])) + __uint_as_float(rv.x << 16);
        o[1] = bf2f(f2bf(o[1])) + __uint_as_float(rv.x & 0xffff0000u);
        o[2] = bf2f(f2bf(o[2])) + __uint_as_float(rv.y << 16);
        o[3] = bf2f(f2bf(o[3])) + __uint_as_float(rv.y & 0xffff0000u);
      }
      uint2 w;
      w.x = pack_bf16x2(o[0], o[1]);
      w.y = pack_bf16x2(o[2], o[3]);
      *reinterpret_cast<uint2*>(C + (long)row * g.ldc + col) = w;
    } else {
      float* C = reinterpret_cast<float*>(g.C) + (long)blockIdx.y * g.split_stride;
      floatx4* dst = reinterpret_cast<floatx4*>(C + (long)row * g.ldc + col);
      floatx4 ov = {o[0], o[1], o[2], o[3]};
      if (g.out_mode == OUT_F32_ACC) ov += *dst;
      *dst = ov;
    }
  }
}

template <bool AK, bool BK_>
int launch(const GemmArgs& g, int splits, hipStream_t s) {
  const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN);
  dim3 grid(tiles, splits);
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BK_>), grid, dim3(256), LDS_BYTES, s, g);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

__global__ void splitk_reduce_kernel(const float* __restrict__ part, long n, int splits, long stride,
                                     void* out, int out_mode) {
  const long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  floatx4 s = *reinterpret_cast<const floatx4*>(part + i4);
  for (int z = 1; z < splits; ++z) s += *reinterpret_cast<const floatx4*>(part + z * stride + i4);
  if (out_mode == OUT_BF16) {
    uint2 w;
    w.x = pack_bf16x2(s[0], s[1]);
    w.y = pack_bf16x2(s[2], s[3]);
    *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(out) + i4) = w;
  } else {
    floatx4* d = reinterpret_cast<floatx4*>(reinterpret_cast<float*>(out) + i4);
    if (out_mode == OUT_F32_ACC) s += *d;
    *d = s;
  }
}

}  // namespace

extern "C" int vpt_gemm_bf16(const void* A, long lda, int a_kmajor, const void* B, long ldb,
                             int b_kmajor, void* C, long ldc, int M, int N, int K,
                             const void* bias, const void* resid, long ldr, int out_mode, int act,
                             int splits, void* workspace, void* stream) {
  VPT_CHECK_ARG(A && B && C, "vpt_gemm_bf16: null operand");
  VPT_CHECK_ARG(M > 0 && N > 0 && K > 0, "vpt_gemm_bf16: empty shape");
  VPT_CHECK_ARG(N % 4 == 0, "vpt_gemm_bf16: N%4 required");
  VPT_CHECK_ARG((!a_kmajor && !b_kmajor) || K % 8 == 0, "vpt_gemm_bf16: k-major operands need K%8==0");
  VPT_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "vpt_gemm_bf16: leading dims must be 16B multiples");
  VPT_CHECK_ARG(a_kmajor || M % 8 == 0, "vpt_gemm_bf16: mn-major A needs M%8==0");
  VPT_CHECK_ARG(b_kmajor || N % 8 == 0, "vpt_gemm_bf16: mn-major B needs N%8==0");
  VPT_CHECK_ARG(out_mode >= 0 && out_mode <= 2, "vpt_gemm_bf16: bad out_mode");
  VPT_CHECK_ARG(!resid || out_mode == OUT_BF16, "vpt_gemm_bf16: residual only with bf16 output");
  if (splits < 1) splits = 1;
  GemmArgs g;
  g.A = (const bf16_t*)A; g.lda = lda;
  g.B = (const bf16_t*)B; g.ldb = ldb;
  g.bias = (const bf16_t*)bias;
  g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.M = M; g.N = N; g.K = K;
  g.act = act;
  hipStream_t s = (hipStream_t)stream;
  int final_mode = out_mode;
  if (splits > 1) {
    VPT_CHECK_ARG(workspace != nullptr, "vpt_gemm_bf16: split-K needs a workspace");
    VPT_CHECK_ARG(!bias && !resid && act == ACT_NONE, "vpt_gemm_bf16: split-K has no fused epilogue");
    VPT_CHECK_ARG(ldc == N, "vpt_gemm_bf16: split-K needs dense C");
    int per = (K + splits - 1) / splits;
    per = (per + BK - 1) / BK * BK;
    splits = (K + per - 1) / per;
    g.k_split = per;
    g.C = workspace; g.ldc = N;
    g.split_stride = (long)M * N;
    g.out_mode = OUT_F32;
  } else {
    g.k_split = K;
    g.C = C; g.ldc = ldc;
    g.split_stride = 0;
    g.out_mode = out_mode;
  }
  int rc;
  if (a_kmajor && b_kmajor) rc = launch<true, true>(g, splits, s);
  else if (a_kmajor && !b_kmajor) rc = launch<true, false>(g, splits, s);
  else if (!a_kmajor && b_kmajor) rc = launch<false, true>(g, splits, s);
  else rc = launch<false, false>(g, splits, s);
  if (rc != VPT_OK || splits == 1) return rc;
  const long n = (long)M * N;
  const int threads = 256;
  const long blocks = (n / 4 + threads - 1) / threads;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(blocks), dim3(threads), 0, s,
                     (const float*)workspace, n, splits, (long)M * N, C, final_mode);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" long vpt_gemm_workspace_bytes(int M, int N, int K, int splits) {
  (void)K;
  if (splits <= 1) return 0;
  return (long)splits * M * N * 4;
}
