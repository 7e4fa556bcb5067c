// The 256x128 ring GEMM ("R2"), two blocks per CU, for gfx950.
//
// Same operands, epilogues and results as the 256x256 ring (gemm.hip; every nn.Linear of the JiT step, reference
// src/models/jit/denoiser.py:318-323, 391-395, 480-506), in a geometry that leaves room for a second block on each CU:
//   4 waves (2 x 2) of 128 x 64 -- the same wave tile, fragment reads and 32 MFMAs (16x16x32 bf16) per 32-deep K step
//   as the 8-wave ring -- over a 3-stage LDS ring of 24 KB stages (A 256x32 + B 128x32), 72 KB per block, <= 256
//   VGPRs per lane: two blocks fit on a CU (2 waves per SIMD, one of each block).
// Why: the 256x256 ring holds all of a CU's registers and 128 KB of its LDS, so every item's epilogue (LDS staging,
// the stores, and for the SwiGLU backward 512 KB of x12 loads / dx12 stores per item) runs while that CU's matrix
// cores idle. With two independent blocks per CU, one block's epilogue overlaps the other block's K loop.
// One block per (256x128 tile, split-K slice) item, XCD-aware bijective item order (as the ring). Per K step: LDS-DMA of
// tile t+2 into the stage tile t-1 used (6 x 1-KB pieces per wave: A 4, B 2), fragment reads of tile t, 32 MFMAs,
// a counted wait for this wave's pieces of tile t+1 (tile t+2's six stay in flight) and one barrier.
#include "gemm_common.h"

namespace vptg {
namespace {

constexpr int R2TN = 128;                   // block tile columns
constexpr int R2NW = 4;                     // waves per block
constexpr int R2ST = 3;                     // ring stages
// TM = block tile rows: 256 (the 256x128 ring) or 128 (128x128 tiles, 4 waves of 64x64: the small-grid GEMMs of config 5)
template <int TM> constexpr int r2_a_bytes() { return TM * RBK * 2; }                     // A stage bytes (16 / 8 KB)
template <int TM> constexpr int r2_stage() { return r2_a_bytes<TM>() + R2TN * RBK * 2; }  // + B (8 KB)
template <int TM> constexpr int r2_lds() { return R2ST * r2_stage<TM>(); }                // 72 / 48 KB
constexpr int R2A = r2_a_bytes<256>();
constexpr int R2STAGE = r2_stage<256>();
constexpr int R2LDS = r2_lds<256>();
// K-step schedule knobs (compile-time; A/B builds of this unit only): PRIO = s_setprio 1 around the MFMAs; SPLIT = the
// fragment reads in two halves (B + A 0-3, then A 4-7 behind the first 16 MFMAs); DMAMID = tile t+2's DMA issued after
// the first half of the MFMAs instead of at the top of the step.
#ifndef VPT_R2_PRIO
#define VPT_R2_PRIO 1
#endif
#ifndef VPT_R2_SPLIT
#define VPT_R2_SPLIT 0
#endif
#ifndef VPT_R2_DMAMID
#define VPT_R2_DMAMID 0
#endif

struct R2Item {
  int m0, n0, split, kbeg, kend, nk, klast;
  uint32_t va[4], vb[2];  // loop-invariant per-lane DMA piece offsets of full K tiles
};

// Six 1-KB pieces of one K tile (A: 4, B: 2) in one asm statement: one hazard pad for the SGPR operands (which may come
// from v_readfirstlane), M0 set per piece, restored at the end (as glds_step).
__device__ __forceinline__ void glds_step6(const void* abase, const void* bbase, const uint32_t (&va)[4],
                                           const uint32_t (&vb)[2], uint32_t la, uint32_t lb) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %9\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %7\n\t"
      "s_mov_b32 m0, %10\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %7\n\t"
      "s_mov_b32 m0, %11\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %3, %7\n\t"
      "s_mov_b32 m0, %12\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %4, %7\n\t"
      "s_mov_b32 m0, %13\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %5, %8\n\t"
      "s_mov_b32 m0, %14\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %6, %8\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(va[0]), "v"(va[1]), "v"(va[2]), "v"(va[3]), "v"(vb[0]), "v"(vb[1]), "s"(abase), "s"(bbase), "s"(la),
        "s"(la + 1024), "s"(la + 2048), "s"(la + 3072), "s"(lb), "s"(lb + 1024)
      : "memory");
}

template <bool AK, bool BK_, int SW, int TM = 256>
__device__ __forceinline__ void r2_voffs(const GemmArgs& g, long lda, long ldb, int m0, int n0, int nrows_b, int kv,
                                         int wid, int lane, uint32_t (&va)[4], uint32_t (&vb)[2]) {
#pragma unroll
  for (int i = 0; i < TM / 64; ++i) va[i] = tile_voff<AK, TM, R2NW>(lda, m0, g.M, kv, wid, lane, i);
#pragma unroll
  for (int i = 0; i < 2; ++i)
    vb[i] = SW ? tile_voff_sw<R2TN, R2NW>(ldb, n0, g.N / 2, kv, wid, lane, i)
               : tile_voff<BK_, R2TN, R2NW>(ldb, n0, nrows_b, kv, wid, lane, i);
}

template <bool AK, bool BK_, int SW, int TM = 256>
__device__ __forceinline__ R2Item r2_item(const GemmArgs& g, int item, int items, int tiles, int tiles_n, int wid,
                                          int lane) {
  const int q8 = items >> 3, r8 = items & 7, xcd = item & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (item >> 3);
  R2Item it;
  it.split = wgid / tiles;
  const int tile = wgid - it.split * tiles;
  it.m0 = tile / tiles_n * TM;
  it.n0 = tile % tiles_n * (SW ? R2TN / 2 : R2TN);  // SW: first output feature of the tile
  it.kbeg = it.split * g.k_split;
  it.kend = min(g.K, it.kbeg + g.k_split);
  it.nk = (it.kend - it.kbeg + RBK - 1) / RBK;
  it.klast = it.kend - it.kbeg - (it.nk - 1) * RBK;
  if (g.K2 > 0 && it.split == g.splits - 1) {  // K-extension tiles after the main K (as ring_item)
    const int ne = (g.K2 + RBK - 1) / RBK;
    it.nk += ne;
    it.klast = g.K2 - (ne - 1) * RBK;
  }
  r2_voffs<AK, BK_, SW, TM>(g, g.lda, g.ldb, it.m0, it.n0, g.N, RBK, wid, lane, it.va, it.vb);
  return it;
}

// K tile t of the item by LDS-DMA into ring stage t % 3: this wave's A pieces at (TM / 64) wid + i, B pieces at
// 2 wid + i.
template <bool AK, bool BK_, int SW, int TM = 256>
__device__ __forceinline__ void r2_dma(const void* ab, const void* bb, const uint32_t (&va)[4], const uint32_t (&vb)[2],
                                       uint32_t la, uint32_t lb) {
  if constexpr (TM == 256) glds_step6(ab, bb, va, vb, la, lb);
  else glds_step(ab, bb, va[0], va[1], vb[0], vb[1], la, la + 1024, lb, lb + 1024);
}

template <bool AK, bool BK_, int SW, int TM = 256>
__device__ __forceinline__ void r2_issue(const GemmArgs& g, const R2Item& it, int t, uint32_t smem0, int wid,
                                         int lane) {
  const uint32_t st = smem0 + (uint32_t)(t % R2ST) * r2_stage<TM>();
  const uint32_t la = __builtin_amdgcn_readfirstlane(st + wid * (TM * 16));
  const uint32_t lb = __builtin_amdgcn_readfirstlane(st + r2_a_bytes<TM>() + wid * 2048);
  const int k0 = it.kbeg + t * RBK;
  if (k0 >= it.kend) {  // K-extension tile (A2 / B2), masked like a partial last tile
    const int e0 = k0 - it.kend, kv = min(RBK, g.K2 - e0);
    const int grp = g.g_n > 0 ? it.n0 / g.g_n : 0;
    const bf16_t* b2 = g.g_n > 0 ? (g.B2g[0] ? g.B2g[grp] : g.B2 + (long)grp * g.g_n * g.ldb2) : g.B2;
    const int nb0 = it.n0 - grp * g.g_n, nrows = g.g_n > 0 ? g.g_n : g.N;
    uint32_t va[4], vb[2];
    r2_voffs<AK, BK_, 0, TM>(g, g.lda2, g.ldb2, it.m0, nb0, nrows, kv, wid, lane, va, vb);
    r2_dma<AK, BK_, SW, TM>(uniform_ptr(tile_ptr<AK>(g.A2 + grp * g.K2, g.lda2, it.m0, e0)),
                            uniform_ptr(tile_ptr<BK_>(b2, g.ldb2, nb0, e0)), va, vb, la, lb);
    return;
  }
  const int kv = min(RBK, it.kend - k0);
  const void* ab = uniform_ptr(tile_ptr<AK>(g.A, g.lda, it.m0, k0));
  const void* bb = uniform_ptr(tile_ptr<BK_>(g.B, g.ldb, SW ? 0 : it.n0, k0));
  if (kv == RBK) {
    r2_dma<AK, BK_, SW, TM>(ab, bb, it.va, it.vb, la, lb);
  } else {
    uint32_t va[4], vb[2];
    r2_voffs<AK, BK_, SW, TM>(g, g.lda, g.ldb, it.m0, it.n0, g.N, kv, wid, lane, va, vb);
    r2_dma<AK, BK_, SW, TM>(ab, bb, va, vb, la, lb);
  }
}

template <bool AK, bool BK_, int SW, int EPI, bool RS, int TM = 256>
__global__ __launch_bounds__(256, 2) void gemm_r2_kernel(GemmArgs g) {
  static_assert(TM == 256 || (TM == 128 && SW == 0 && !RS && EPI != EPI_QKN && !epi_swb(EPI)),
                "128-row tiles: plain / residual / accumulate epilogues");
  constexpr int MI = TM / 32, WR = TM / 2;  // fragments and rows of a wave tile (128 x 64 or 64 x 64)
  constexpr int PCS = TM / 64 + 2;          // LDS-DMA pieces per wave and K tile (A + B)
  constexpr int STG = r2_stage<TM>(), AB = r2_a_bytes<TM>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (g.N + R2TN - 1) / R2TN;
  const int tiles = ((g.M + TM - 1) / TM) * tiles_n;
  const int items = tiles * g.splits;
  if ((int)blockIdx.x >= items) return;
  // The two blocks a CU starts with begin together and, equal in length, would keep reaching their epilogues together.
  // g.stagger > 0 (10-ns ticks, diagnostic build): the CUs' second blocks of the first wave of the grid (ids 256-511
  // under the dispatcher's order) start that much later, so the two blocks of a CU alternate K loop and epilogue.
  if (g.stagger > 0 && blockIdx.x >= 256 && blockIdx.x < 512) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)g.stagger) __builtin_amdgcn_s_sleep(2);
  }
  const uint32_t smem0 = (uint32_t)(uintptr_t)(VPT_LDS char*)smem;
  const R2Item it = r2_item<AK, BK_, SW, TM>(g, blockIdx.x, items, tiles, tiles_n, wid, lane);
  const int nk = it.nk;

  uint4 braw = make_uint4(0, 0, 0, 0), braw2 = make_uint4(0, 0, 0, 0);
  if (SW) {
    const int c = it.n0 + wn * 32 + (lane & 3) * 8;
    if (g.bias) {
      braw = *reinterpret_cast<const uint4*>(g.bias + c);
      braw2 = *reinterpret_cast<const uint4*>(g.bias + g.N / 2 + c);
    }
  } else {
    const int bcol = it.n0 + wn * 64 + (lane & 7) * 8;
    if (g.bias && bcol < g.N) braw = *reinterpret_cast<const uint4*>(g.bias + bcol);
  }
  // bias values in registers before the first LDS-DMA (the compiler cannot see the asm DMAs; its wait for these loads,
  // placed at their first use, would be a vmcnt(0) that also drains the ring)
  float bias8[8], bias8b[8];
  unpack8(braw, bias8);
  unpack8(braw2, bias8b);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    asm volatile("" : "+v"(bias8[e]));
    if (SW) asm volatile("" : "+v"(bias8b[e]));
  }

  floatx4 acc[8][4];  // [MI][4] used
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  // RS (fused bias gradient): the items of the first N tile also sum their A rows over k (MFMAs against an all-ones
  // fragment); wave (wm, wn) takes fragments 4 wn .. 4 wn + 3 of its 128 rows (4 extra MFMAs per K step)
  floatx4 racc[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) racc[f] = floatx4{0.f, 0.f, 0.f, 0.f};
  const bool rs_on = RS && it.n0 == 0;
  const int wn_u = __builtin_amdgcn_readfirstlane(wn);

  r2_issue<AK, BK_, SW, TM>(g, it, 0, smem0, wid, lane);
  if (nk > 1) {
    r2_issue<AK, BK_, SW, TM>(g, it, 1, smem0, wid, lane);
    // tile 0 landed (this wave); tile 1's pieces in flight
    if constexpr (PCS == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    // tile kt + 2 into the stage of tile kt - 1, which every wave finished reading before the last barrier
    if (!VPT_R2_DMAMID && kt + 2 < nk) r2_issue<AK, BK_, SW, TM>(g, it, kt + 2, smem0, wid, lane);
    const char* st = smem + (kt % R2ST) * STG;
    const bool mask = kt == nk - 1 && it.klast < RBK;
    bf16x8 bfr[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[j] = read_frag32<BK_, R2TN>(st + AB, SW ? ((j & 2) ? R2TN / 2 : 0) + wn * 32 + (j & 1) * 16 : wn * 64 + j * 16,
                                      lane);
#pragma unroll
    for (int i = 0; i < (VPT_R2_SPLIT ? MI / 2 : MI); ++i) {
      af[i] = read_frag32<AK, TM>(st, wm * WR + i * 16, lane);
      if (mask) af[i] = mask_k(af[i], 8 * (lane >> 4), it.klast);
    }
    if (VPT_R2_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MI / 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (VPT_R2_SPLIT) {
#pragma unroll
      for (int i = MI / 2; i < MI; ++i) {
        af[i] = read_frag32<AK, TM>(st, wm * WR + i * 16, lane);
        if (mask) af[i] = mask_k(af[i], 8 * (lane >> 4), it.klast);
      }
    }
    if (VPT_R2_DMAMID && kt + 2 < nk) r2_issue<AK, BK_, SW, TM>(g, it, kt + 2, smem0, wid, lane);
#pragma unroll
    for (int i = MI / 2; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    if (rs_on) {
      const bf16x8 ones = as_frag(make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u));
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const bf16x8 r = wn_u == 0 ? af[f] : af[4 + f];
        racc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r, ones, racc[f], 0, 0, 0);
      }
    }
    if (VPT_R2_PRIO) __builtin_amdgcn_s_setprio(0);
    if (kt + 1 < nk) {
      // this wave's pieces of tile kt + 1 landed (tile kt + 2's younger ones may still fly), then every wave's
      if (kt + 2 < nk) {
        if constexpr (PCS == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
    }
  }
  if (rs_on && (lane & 15) == 0) {  // D layout of the ones-MFMA: lane holds rows 4 (lane >> 4) + r of the fragment
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int row = it.m0 + wm * 128 + (4 * wn_u + f) * 16 + 4 * (lane >> 4);
      float* dst = g.rsum + (long)it.split * g.M + row;
      if (row + 3 < g.M && (g.M & 3) == 0) {
        *reinterpret_cast<floatx4*>(dst) = racc[f];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row + r < g.M) dst[r] = racc[f][r];
      }
    }
  }
  // Epilogue staging: this wave's 4 KB slice of the stage of tile nk - 3 (or an unused stage): every wave finished
  // reading it before the barrier that ended step nk - 2, and no DMA targets it after that.
  char* stg = smem + (nk % R2ST) * STG + wid * 4096;
  RingItem ri;
  ri.m0 = it.m0; ri.n0 = it.n0; ri.split = it.split;
  if (SW) {
    epilogue_ring_swf(g, acc, stg, lane, ri, wm, wn, bias8, bias8b);
    return;
  }
  EpiAddr ea = epi_addr(g, ri, wm, wn, lane, WR);
  EpiPre pre, pre2;
  if constexpr (TM == 128) {  // 4 fragments per wave
    if constexpr (epi_frags(EPI) == 4) {
      epi_preload<EPI, 0>(g, ea, pre);
      epilogue_ring<EPI, 0, 4>(g, acc, stg, lane, ea, bias8, pre);
    } else if constexpr (epi_frags(EPI) == 2) {
      epi_preload<EPI, 0>(g, ea, pre);
      epilogue_ring<EPI, 0, 2>(g, acc, stg, lane, ea, bias8, pre);
      epi_preload<EPI, 2>(g, ea, pre);
      epilogue_ring<EPI, 2, 4>(g, acc, stg, lane, ea, bias8, pre);
    } else {
      epilogue_ring<EPI, 0, 4>(g, acc, stg, lane, ea, bias8, pre);
    }
    return;
  }
  if (EPI == EPI_QKN) {
    epilogue_ring_qkn(g, acc, stg, lane, ea, bias8, ri, wm, wn);
  } else if (EPI == EPI_SWB) {
    epi_preload<EPI, 0>(g, ea, pre);
    epi_preload<EPI, 2>(g, ea, pre2);
    __builtin_amdgcn_s_waitcnt(0x0f78);  // vmcnt(8): the first group landed; the second may be in flight
    epilogue_ring<EPI, 0, 2>(g, acc, stg, lane, ea, bias8, pre);
    epi_preload<EPI, 4>(g, ea, pre);
    epilogue_ring<EPI, 2, 4>(g, acc, stg, lane, ea, bias8, pre2);
    epi_preload<EPI, 6>(g, ea, pre2);
    epilogue_ring<EPI, 4, 6>(g, acc, stg, lane, ea, bias8, pre);
    epilogue_ring<EPI, 6, 8>(g, acc, stg, lane, ea, bias8, pre2);
  } else if (epi_frags(EPI) == 2) {
    epi_preload<EPI, 0>(g, ea, pre);
    epilogue_ring<EPI, 0, 2>(g, acc, stg, lane, ea, bias8, pre);
    epi_preload<EPI, 2>(g, ea, pre);
    epilogue_ring<EPI, 2, 4>(g, acc, stg, lane, ea, bias8, pre);
    epi_preload<EPI, 4>(g, ea, pre);
    epilogue_ring<EPI, 4, 6>(g, acc, stg, lane, ea, bias8, pre);
    epi_preload<EPI, 6>(g, ea, pre);
    epilogue_ring<EPI, 6, 8>(g, acc, stg, lane, ea, bias8, pre);
  } else if (epi_frags(EPI) == 4) {
    epi_preload<EPI, 0>(g, ea, pre);
    epilogue_ring<EPI, 0, 4>(g, acc, stg, lane, ea, bias8, pre);
    epi_preload<EPI, 4>(g, ea, pre);
    epilogue_ring<EPI, 4, 8>(g, acc, stg, lane, ea, bias8, pre);
  } else {
    epilogue_ring<EPI, 0, 8>(g, acc, stg, lane, ea, bias8, pre);
  }
}

template <bool AK, bool BK_, int SW, int EPI, bool RS, int TM = 256>
int r2_launch(const GemmArgs& g, int items, hipStream_t s) {
  hipLaunchKernelGGL((gemm_r2_kernel<AK, BK_, SW, EPI, RS, TM>), dim3(items), dim3(256), r2_lds<TM>(), s, g);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

template <bool AK, bool BK_>
int r2_dispatch(const GemmArgs& g, int items, hipStream_t s) {
  if (g.sw == 1) {
    if constexpr (AK && BK_) return r2_launch<true, true, 1, EPI_PLAIN, false>(g, items, s);
    VPT_CHECK_ARG(false, "gemm r2: the fused SwiGLU forward is a k-major x k-major mode");
  }
  const int epi = epi_mode(g);
  if (!AK && g.rsum) {  // fused bias gradient (wgrad direction)
    if (epi == EPI_ACC) return r2_launch<AK, BK_, 0, EPI_ACC, true>(g, items, s);
    return r2_launch<AK, BK_, 0, EPI_PLAIN, true>(g, items, s);
  }
  if (epi == EPI_RESID) return r2_launch<AK, BK_, 0, EPI_RESID, false>(g, items, s);
  if (epi == EPI_ACC) return r2_launch<AK, BK_, 0, EPI_ACC, false>(g, items, s);
  if (epi == EPI_SWB) {
    if constexpr (AK && !BK_) return r2_launch<true, false, 0, EPI_SWB, false>(g, items, s);
    VPT_CHECK_ARG(false, "gemm r2: the fused SwiGLU backward is a k-major x mn-major mode");
  }
  if (epi == EPI_QKN) {
    if constexpr (AK && BK_) return r2_launch<true, true, 0, EPI_QKN, false>(g, items, s);
    VPT_CHECK_ARG(false, "gemm r2: the QK-norm epilogue is a forward (k-major x k-major) mode");
  }
  return r2_launch<AK, BK_, 0, EPI_PLAIN, false>(g, items, s);
}

// 128x128 tiles (TM = 128): plain, residual or accumulate epilogue, no fused bias gradient / SwiGLU / QK-norm.
template <bool AK, bool BK_>
int r2_128_dispatch(const GemmArgs& g, int items, hipStream_t s) {
  VPT_CHECK_ARG(g.sw == 0 && g.qk_d == 0 && !g.rsum, "gemm r2 128x128: plain / residual / accumulate epilogues only");
  const int epi = epi_mode(g);
  if (epi == EPI_RESID) return r2_launch<AK, BK_, 0, EPI_RESID, false, 128>(g, items, s);
  if (epi == EPI_ACC) return r2_launch<AK, BK_, 0, EPI_ACC, false, 128>(g, items, s);
  return r2_launch<AK, BK_, 0, EPI_PLAIN, false, 128>(g, items, s);
}

}  // namespace

// The 128x128 form of the R2 ring: the config-5 GEMMs whose 256-wide grids cover few CUs (2 blocks per CU, 48 KB of
// LDS each; the same K order as the 128x128 T128 kernel, so the same sums).
int launch_r2_128(const GemmArgs& g, bool ak, bool bk, hipStream_t s) {
  VPT_CHECK_ARG(g.N % 8 == 0, "gemm r2 128x128: N % 8 == 0 (8-column epilogue chunks)");
  VPT_CHECK_ARG(g.g_n % R2TN == 0 && g.alpha_cols % R2TN == 0, "gemm r2 128x128: groups / alpha columns in 128-column tiles");
  const int items = ((g.M + 127) / 128) * ((g.N + R2TN - 1) / R2TN) * g.splits;
  if (ak && bk) return r2_128_dispatch<true, true>(g, items, s);
  if (ak) return r2_128_dispatch<true, false>(g, items, s);
  if (bk) return r2_128_dispatch<false, true>(g, items, s);
  return r2_128_dispatch<false, false>(g, items, s);
}

// The 256x128 ring for an argument block the 256x256 ring would run (gemm.hip launch_ring: same GemmArgs, one block per
// item, ring_grid ignored). Tiles never straddle a LoRA group or an alpha column block: g_n, alpha_cols % 128 == 0.
int launch_r2(const GemmArgs& g, bool ak, bool bk, hipStream_t s) {
  VPT_CHECK_ARG(g.N % 8 == 0, "gemm r2: N % 8 == 0 (8-column epilogue chunks)");
  VPT_CHECK_ARG(g.g_n % R2TN == 0 && g.alpha_cols % R2TN == 0, "gemm r2: groups / alpha columns in 128-column tiles");
  const int items = ((g.M + 255) / 256) * ((g.N + R2TN - 1) / R2TN) * g.splits;
  if (ak && bk) return r2_dispatch<true, true>(g, items, s);
  if (ak) return r2_dispatch<true, false>(g, items, s);
  if (bk) return r2_dispatch<false, true>(g, items, s);
  return r2_dispatch<false, false>(g, items, s);
}

}  // namespace vptg
