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
// Two geometries of one kernel template, BK = 64, MFMA 16x16x32 bf16:
//   T128: 128x128 block tile, 4 waves (2x2) of 64x64, 2 blocks/CU   (small grids / N = 768)
//   T256: 256x256 block tile, 8 waves (2x4) of 128x64, 1 block/CU   (large grids): 64 MFMA per wave
//         per K step cover the LDS-DMA latency of the next tile, and 128x64 wave tiles cut LDS read
//         traffic per FLOP by 25 % vs 64x64.
// k-major tiles are staged [row][64k] (128 B rows, 16-B chunk XOR swizzle, read with ds_read_b128);
// mn-major tiles keep their global [k][mn] orientation (8-B unit XOR swizzle) and are read with
// ds_read_b64_tr_b16, which delivers the transpose. Full K tiles arrive by LDS-DMA
// (global_load_lds_dwordx4, swizzle moved to the source address), issued one K step ahead into a
// 2-stage ring; one barrier per K step; the partial last K tile (wgrad over a token count) is DMA'd
// with clamped addresses and its out-of-range part zeroed in LDS. XCD-aware bijective block remap. Epilogue staged through
// LDS (f32, 64 rows at a time) so bias / residual / SiLU and stores are 8-16 B per lane. Optional
// split-K writes f32 partial slabs, summed in a fixed order by splitk_reduce_kernel.
#include "common.h"
#include "../../include/vpt_hip.h"  // C-ABI types (VptLoraReduceJob)
#include "gemm_common.h"

using namespace vptg;

namespace vptg {
int launch_r2(const GemmArgs& g, bool ak, bool bk, hipStream_t s);  // gemm_r2.hip: the 256x128 two-blocks-per-CU ring
int launch_r2_128(const GemmArgs& g, bool ak, bool bk, hipStream_t s);  // gemm_r2.hip: its 128x128 form
// geometry 1281 of the C-ABI: the 128x128 tiles on the R2 ring's pipeline (3-stage LDS-DMA ring, counted waits)
constexpr int kGeoR2x128 = 1281;
}

namespace {

// Ring launches that take the 256x128 two-blocks-per-CU ring (gemm_r2.hip) instead, by kind: bit 0 = k-major A (forward /
// input gradient: plain, residual), bit 1 = mn-major A (weight gradients), bit 2 = fused SwiGLU forward, bit 3 = fused
// SwiGLU backward, bit 4 = fused QK-norm + RoPE forward. Production: the SwiGLU backward only -- bitwise equal to the
// 256x256 ring on every kind, 212 -> 193 us at the C3 shape (its x12 / dx12 epilogue traffic overlaps the CU's other
// block's K loop), while the other kinds measured level or slower (r05i-r05k, tools/r2_ab.py).
constexpr int kR2Kinds = 8;
#ifdef VPT_DIAG
int g_r2 = kR2Kinds;  // vpt_gemm_set_r2 (A/B)
#else
constexpr int g_r2 = kR2Kinds;
#endif
inline bool use_r2(const GemmArgs& g, bool ak) {
  const int kind = g.sw == 1 ? 4 : g.sw == 2 ? 8 : g.qk_d > 0 ? 16 : ak ? 1 : 2;
  return (g_r2 & kind) != 0;
}

template <int TM_, int TN_, int WGM, int WGN>
struct Geo {
  static constexpr int TM = TM_, TN = TN_;
  static constexpr int NW = WGM * WGN, T = 64 * NW;
  static constexpr int WR = TM / WGM, WC = TN / WGN;       // wave tile
  static constexpr int MI = WR / 16, NI = WC / 16;         // MFMA fragments per wave
  static constexpr int A_BYTES = TM * BK * 2, B_BYTES = TN * BK * 2, STAGE = A_BYTES + B_BYTES;
  // epilogue staging: SLAB fragments (16 * SLAB rows) per round, f32 rows of ELD floats (WC + 4: 68 for the
  // 64-wide wave tiles, conflict-free for the column writes)
  static constexpr int SLAB = MI < 4 ? MI : 4, ELD = WC + 4;
  static constexpr int EPI = NW * 16 * SLAB * ELD * 4;
  static constexpr int LDS = 2 * STAGE > EPI ? 2 * STAGE : EPI;
};

// One 64-deep K step: per 32-k half each wave reads MI A and NI B fragments, issues MI*NI MFMAs.
template <bool AK, bool BK_, typename G>
__device__ __forceinline__ void mma_tile(const char* la, floatx4 (&acc)[G::MI][G::NI], int wm, int wn, int lane) {
  const char* lb = la + G::A_BYTES;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 bfr[G::NI];
#pragma unroll
    for (int j = 0; j < G::NI; ++j) bfr[j] = read_frag<BK_, G::TN>(lb, wn * G::WC + j * 16, kk, lane);
#pragma unroll
    for (int i = 0; i < G::MI; ++i) {
      const bf16x8 af = read_frag<AK, G::TM>(la, wm * G::WR + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < G::NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
    }
  }
}

// Epilogue: per 64-row slab of the wave tile, stage the f32 accumulators in the wave's own LDS region,
// then a vectorised row pass applies bias / SiLU / residual and stores 8-16 B per lane.
template <typename G>
__device__ __forceinline__ void epilogue(const GemmArgs& g, floatx4 (&acc)[G::MI][G::NI], char* smem, int wid, int lane,
                                         int m0, int n0, int wm, int wn, int split) {
  constexpr int SLAB = G::SLAB, ELD = G::ELD;
  float* st = reinterpret_cast<float*>(smem) + wid * 16 * SLAB * ELD;
  const int colw = (lane & 15) * 4;
#pragma unroll
  for (int h = 0; h < G::MI / SLAB; ++h) {
#pragma unroll
    for (int i = 0; i < SLAB; ++i)
#pragma unroll
      for (int j = 0; j < G::NI; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          st[(i * 16 + (lane >> 4) * 4 + r) * ELD + j * 16 + (lane & 15)] = acc[SLAB * h + i][j][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes retired
    __builtin_amdgcn_wave_barrier();
    for (int cb = 0; cb < G::WC; cb += 64) {
      const int col = n0 + wn * G::WC + cb + colw;
      const bool col_ok = cb + colw < G::WC && col < g.N;  // (an 80-wide wave tile: 16 columns in round 2)
      float bias4[4] = {0.f, 0.f, 0.f, 0.f};
      const float alpha = g.alpha_cols > 0 && col >= g.alpha_cols ? 1.f : g.alpha;
      if (g.bias && col_ok) {
        const uint2 bv = *reinterpret_cast<const uint2*>(g.bias + col);
        bias4[0] = __uint_as_float(bv.x << 16); bias4[1] = __uint_as_float(bv.x & 0xffff0000u);
        bias4[2] = __uint_as_float(bv.y << 16); bias4[3] = __uint_as_float(bv.y & 0xffff0000u);
      }
      for (int pass = 0; pass < 4 * SLAB; ++pass) {
        const int lr = pass * 4 + (lane >> 4);
        const int row = m0 + wm * G::WR + h * 16 * SLAB + lr;
        if (row >= g.M || !col_ok) continue;
        floatx4 v = *reinterpret_cast<const floatx4*>(st + lr * ELD + cb + colw);
        float o[4] = {v[0] * alpha + bias4[0], v[1] * alpha + bias4[1], v[2] * alpha + bias4[2],
                      v[3] * alpha + bias4[3]};
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
          float* C = reinterpret_cast<float*>(g.C) + (long)split * g.split_stride;
          floatx4* dst = reinterpret_cast<floatx4*>(C + (long)row * g.ldc + col);
          floatx4 ov = {o[0], o[1], o[2], o[3]};
          if (g.out_mode == OUT_F32_ACC) ov += *dst;
          *dst = ov;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <bool AK, bool BK_, int TM, int TN, int WGM, int WGN>
__global__ __launch_bounds__(64 * WGM * WGN, 2) void gemm_bf16_kernel(GemmArgs g) {
  using G = Geo<TM, TN, WGM, WGN>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;

  const int tiles_n = (g.N + TN - 1) / TN;
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int tm = wgid / tiles_n, tn = wgid % tiles_n;
  const int m0 = tm * TM, n0 = tn * TN;

  const int kbeg = blockIdx.y * g.k_split;
  const int kend = min(g.K, kbeg + g.k_split);
  const int nfull = (kend - kbeg) / BK;
  const bool ktail = (kend - kbeg) % BK != 0;
  // K-extension tiles (K % BK == 0): in the last split's K loop only
  const int next = g.K2 > 0 && (int)blockIdx.y == g.splits - 1 ? (g.K2 + BK - 1) / BK : 0;

  floatx4 acc[G::MI][G::NI];
#pragma unroll
  for (int i = 0; i < G::MI; ++i)
#pragma unroll
    for (int j = 0; j < G::NI; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  // Main loop: LDS-DMA only (no ordinary VGPR loads in the loop), next tile in flight while this one
  // computes. A partial last K tile (wgrad over a token count) is DMA'd with clamped addresses and
  // its out-of-range k rows / chunks are zeroed in LDS before it is consumed.
  const int nkm = nfull + (ktail ? 1 : 0);  // main K tiles
  const int nk = nkm + next;
  // tile t -> its valid k and the DMA of both operands into `buf` (main K, then the K-extension)
  auto issue = [&](char* buf, int t) -> int {
    if (t < nkm) {
      const int k0 = kbeg + t * BK, kv = min(BK, kend - k0);
      glds_tile<AK, TM, G::NW>(buf, tile_ptr<AK>(g.A, g.lda, m0, k0), g.lda, m0, g.M, kv, wid, lane);
      glds_tile<BK_, TN, G::NW>(buf + G::A_BYTES, tile_ptr<BK_>(g.B, g.ldb, n0, k0), g.ldb, n0, g.N, kv, wid, lane);
      return kv;
    }
    const int e0 = (t - nkm) * BK, kv = min(BK, g.K2 - e0);
    const int grp = g.g_n > 0 ? n0 / g.g_n : 0;  // grouped extension: this tile's target
    const bf16_t* b2 = g.g_n > 0 ? (g.B2g[0] ? g.B2g[grp] : g.B2 + (long)grp * g.g_n * g.ldb2) : g.B2;
    const int nb0 = n0 - grp * g.g_n, nrows = g.g_n > 0 ? g.g_n : g.N;
    glds_tile<AK, TM, G::NW>(buf, tile_ptr<AK>(g.A2 + grp * g.K2, g.lda2, m0, e0), g.lda2, m0, g.M, kv, wid, lane);
    glds_tile<BK_, TN, G::NW>(buf + G::A_BYTES, tile_ptr<BK_>(b2, g.ldb2, nb0, e0), g.ldb2, nb0, nrows, kv, wid, lane);
    return kv;
  };
  int cur = 0;
  {
    const int kv = issue(smem, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kv < BK) {
      zero_k_tail<AK, TM, G::T>(smem, kv, tid);
      zero_k_tail<BK_, TN, G::T>(smem + G::A_BYTES, kv, tid);
      __syncthreads();
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* nb = smem + (cur ^ 1) * G::STAGE;
    const int kv = kt + 1 < nk ? issue(nb, kt + 1) : 0;  // valid k rows of the next tile (0: no next tile)
    mma_tile<AK, BK_, G>(smem + cur * G::STAGE, acc, wm, wn, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's LDS-DMA for tile kt+1 has landed
    __syncthreads();                                   // ... and every other wave's too
    if (kv > 0 && kv < BK) {
      zero_k_tail<AK, TM, G::T>(nb, kv, tid);
      zero_k_tail<BK_, TN, G::T>(nb + G::A_BYTES, kv, tid);
      __syncthreads();
    }
    cur ^= 1;
  }

  epilogue<G>(g, acc, smem, wid, lane, m0, n0, wm, wn, blockIdx.y);
}


using GR = Geo<256, 256, 2, 4>;

// STAMP (diagnostic build, geometry 2566): per-wave cycle sums of the K-step segments (DMA issue,
// ds_reads, vmcnt wait, barrier Y, MFMA issue, barrier X) to g.dbg[(block*8 + wave)*8 + seg]; read the
// shares, not the length (the stamps' lgkmcnt(0) forbids overlaps the real kernel has).
//
// PERSISTENT grid: min(items, 256) blocks walk work items (tile, split-K slice) with a stride of
// gridDim.x; item -> tile uses the same bijective XCD remap as a one-tile-per-block launch of `items`
// blocks (block b runs on XCD b % 8 and only sees items == b mod 8). Item seam: after the last K step
// the block DMAs the NEXT item's K tiles 0-2 into ring stages 0-2, then runs this item's epilogue out of
// stage 3, so the next item's operand latency and this item's store drain overlap the epilogue and
// the next item's first K steps (its waits for tiles 0-2 count the epilogue stores as younger).
// TL (diagnostic build, geometry 2567): wave 0 of each block writes s_memrealtime (100 MHz) stamps of its
// first 4 items to g.dbg[(block*4 + k)*4 + phase]: phase 0 item start, 1 tile 0 ready (after X_0),
// 2 K loop done, 3 epilogue issued.
__device__ __forceinline__ void tl_stamp(const GemmArgs& g, int k, int phase, int wid, int lane) {
  if (wid == 0 && lane == 0 && k < 4)
    g.dbg[((long)blockIdx.x * 4 + k) * 4 + phase] = __builtin_amdgcn_s_memrealtime();
}

template <bool AK, bool BK_, bool PP, int ABL = 0, bool DMAC = false, bool STAMP = false, bool TL = false, int SW = 0,
          int EPI = EPI_PLAIN, bool RS = false>
__global__ __launch_bounds__(512, 1) void gemm_ring_kernel(GemmArgs g) {
  using G = GR;
  constexpr int A32 = 256 * RBK * 2, STAGE32 = 2 * A32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / 4, wn = wid % 4;

  const int tiles_n = (g.N + 255) / 256;
  const int tiles = ((g.M + 255) / 256) * tiles_n;
  const int items = tiles * g.splits;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(VPT_LDS char*)smem + wid * 2048;
  char* stg = smem + 3 * STAGE32 + wid * 4096;  // this wave's epilogue staging slice (ring stage 3)
  const int S = ring_stores(g);

  int item = blockIdx.x;
  if (item >= items) return;
  RingItem it = ring_item<AK, BK_, SW>(g, item, items, tiles, tiles_n, wid, lane);
  ring_issue<AK, BK_, SW>(g, it, 0, lds0, wid, lane);
  if (it.nk > 1) ring_issue<AK, BK_, SW>(g, it, 1, lds0, wid, lane);
  if (it.nk > 2) ring_issue<AK, BK_, SW>(g, it, 2, lds0, wid, lane);
  // Epilogue de-synchronisation: with every block on the same item length all 256 CUs reach their store
  // (and residual / x12 load) bursts together, which then run at the chip's HBM rate while no MFMA works.
  // Delaying half the blocks by about half an epilogue (wave-uniform spin on the 100 MHz real-time
  // counter, the first tiles already in flight) makes the two halves alternate: one half's epilogue
  // traffic overlaps the other half's K loop.
  if (g.stagger > 0 && ((blockIdx.x >> 3) & 1)) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)g.stagger) __builtin_amdgcn_s_sleep(2);
  }
  int pend = 0;  // epilogue stores younger than this item's pre-issued tiles 0-2 (0 on the first item)
  int kth = 0;   // items done by this block (TL stamps)

  for (;;) {
    if (TL) tl_stamp(g, kth, 0, wid, lane);
    const int nk = it.nk;
    // bias of this item's 8 output columns (plain load; consumed after the K loop, when nothing is
    // outstanding, so the compiler's wait for it costs nothing)
    uint4 braw = make_uint4(0, 0, 0, 0), braw2 = make_uint4(0, 0, 0, 0);
    if (SW) {  // bias of the lane's 8 features in both halves (W1 at c, W2 at F + c)
      const int c = it.n0 + wn * 32 + (lane & 3) * 8;
      if (g.bias) {
        braw = *reinterpret_cast<const uint4*>(g.bias + c);
        braw2 = *reinterpret_cast<const uint4*>(g.bias + g.N / 2 + c);
      }
    } else {
      const int bcol = it.n0 + wn * 64 + (lane & 7) * 8;
      if (g.bias && bcol < g.N) braw = *reinterpret_cast<const uint4*>(g.bias + bcol);
    }

    floatx4 acc[G::MI][G::NI];
#pragma unroll
    for (int i = 0; i < G::MI; ++i)
#pragma unroll
      for (int j = 0; j < G::NI; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
    // RS (fused bias gradient): the items of the first N tile also sum their A rows over k, as MFMAs of
    // the A fragments against an all-ones B fragment; wave (wm, wn) takes fragments 2wn and 2wn + 1 of its
    // 128 rows (2 extra MFMAs per K step). wn is made wave-uniform so the fragment pick is a scalar branch.
    floatx4 racc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
    const bool rs_on = RS && it.n0 == 0;
    const int wn_u = __builtin_amdgcn_readfirstlane(wn);

    if (pend && nk >= 3) wait_vm_pend(pend);  // tile 0 landed: tiles 1, 2 and the stores are younger
    else wait_younger(min(2, nk - 1));
    if (PP && wm == 1) raw_barrier();
    raw_barrier();  // X_0
    if (TL) tl_stamp(g, kth, 1, wid, lane);

    unsigned long long seg[6] = {0, 0, 0, 0, 0, 0};
    for (int kt = 0; kt < nk; ++kt) {
      const char* st = smem + (kt & (RSTAGES - 1)) * STAGE32;
      unsigned long long t0 = 0, t1 = 0;
      if (STAMP) t0 = stamp();
      if (!DMAC && ABL != 1 && kt + 3 < nk) ring_issue<AK, BK_, SW>(g, it, kt + 3, lds0, wid, lane);
      if (STAMP) { t1 = stamp(); seg[0] += t1 - t0; t0 = t1; }
      bf16x8 bfr[G::NI], af[G::MI];
#pragma unroll
      for (int j = 0; j < G::NI; ++j)
        bfr[j] = read_frag32<BK_, 256>(st + A32, SW ? ((j & 2) << 6) + wn * 32 + (j & 1) * 16 : wn * G::WC + j * 16, lane);
#pragma unroll
      for (int i = 0; i < G::MI; ++i) af[i] = read_frag32<AK, 256>(st, wm * G::WR + i * 16, lane);
      if (kt == nk - 1 && it.klast < RBK) {
#pragma unroll
        for (int i = 0; i < G::MI; ++i) af[i] = mask_k(af[i], 8 * (lane >> 4), it.klast);
      }
      if (STAMP) { t1 = stamp(); seg[1] += t1 - t0; t0 = t1; }
      // tile kt+1 (if any) landed for this wave; the previous epilogue's stores are younger than tiles 0-2
      if (ABL != 2) {
        if (!DMAC && pend && kt < 2 && nk - 2 - kt >= 2) wait_vm_pend(pend);  // 8 + S younger
        else wait_younger(min(DMAC ? 1 : 2, nk - 2 - kt));  // (over-waits for the stores when pend)
      }
      if (STAMP) { t1 = stamp(); seg[2] += t1 - t0; t0 = t1; }
      if (DMAC) bare_barrier(); else raw_barrier();                // Y_kt
      if (STAMP) { t1 = stamp(); seg[3] += t1 - t0; t0 = t1; }
      if (DMAC && ABL != 1 && kt + 3 < nk) ring_issue<AK, BK_, SW>(g, it, kt + 3, lds0, wid, lane);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < G::MI; ++i)
#pragma unroll
        for (int j = 0; j < G::NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (rs_on) {
        const bf16x8 ones = as_frag(make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u));
        bf16x8 r0, r1;
        if (wn_u == 0) { r0 = af[0]; r1 = af[1]; }
        else if (wn_u == 1) { r0 = af[2]; r1 = af[3]; }
        else if (wn_u == 2) { r0 = af[4]; r1 = af[5]; }
        else { r0 = af[6]; r1 = af[7]; }
        racc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r0, ones, racc[0], 0, 0, 0);
        racc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(r1, ones, racc[1], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
      if (STAMP) { t1 = stamp(); seg[4] += t1 - t0; t0 = t1; }
      if (DMAC) bare_barrier(); else raw_barrier();  // X_kt+1
      if (STAMP) { t1 = stamp(); seg[5] += t1 - t0; }
    }
    if (STAMP && lane == 0 && item < 256 && it.split == 0) {
      unsigned long long* o = g.dbg + ((long)item * 8 + wid) * 8;
#pragma unroll
      for (int i = 0; i < 6; ++i) o[i] = seg[i];
      o[6] = nk;
    }
    if (PP && wm == 0) raw_barrier();
    if (TL) tl_stamp(g, kth, 2, wid, lane);
    if (rs_on && (lane & 15) == 0) {
      // D layout of the ones-MFMA: lane holds rows 4*(lane>>4) + r of the fragment (every column equal);
      // issued before the next item's DMA, so the counted waits never see these stores
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int row = it.m0 + wm * 128 + (2 * wn_u + f) * 16 + 4 * (lane >> 4);
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
    float bias8[8], bias8b[8];
    unpack8(braw, bias8);
    unpack8(braw2, bias8b);
    // The bias values must be in registers BEFORE the next item's LDS-DMA below: the compiler does not
    // see the asm DMA, places its wait for the bias loads at their first use (in the epilogue) as
    // vmcnt(0), and vmcnt retires in order -- that wait would drain the next item's prefetched tiles.
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      asm volatile("" : "+v"(bias8[e]));
      if (SW) asm volatile("" : "+v"(bias8b[e]));
    }
    // Every wave has passed its last K step (barrier X_nk), so ring stages 0-2 are free: DMA the next
    // item's first tiles before this item's epilogue (which stages through stage 3 only).
    // Epilogue operands read from memory (residual, SwiGLU x12, f32 accumulate) are loaded first and
    // waited for once, so no wait inside the epilogue drains those DMAs (in-order vmcnt; the compiler
    // does not see the asm DMAs). A second preload group (x12 / accumulate, fragments 4-7) is loaded
    // after the first group's stores: its wait also covers the DMAs, by then long in flight.
    const int next = item + gridDim.x;
    constexpr int GF = SW ? 0 : epi_frags(EPI);
    EpiAddr ea;
    EpiPre pre, pre2;
    if (!SW) {
      ea = epi_addr(g, it, wm, wn, lane);
      if (ABL == 4) ea.rs = __builtin_amdgcn_make_buffer_rsrc(g.C, (short)0, 0, 0x00020000);  // stores dropped
      if (ABL == 6 && epi_swb(EPI))  // every item's x12 operands from the first tile (L2-resident; timing only)
        ea.ra = __builtin_amdgcn_make_buffer_rsrc((void*)g.aux, (short)0, 256 * (int)g.ldaux * 2, 0x00020000);
      if (EPI == EPI_SWB) {
        // two groups in flight (the K loop's fragment registers are free now): group 0 waited for here, group 1
        // lands under group 0's epilogue, and each later group is loaded one group ahead of its use
        epi_preload<EPI, 0>(g, ea, pre);
        epi_preload<EPI, 2>(g, ea, pre2);
        __builtin_amdgcn_s_waitcnt(0x0f78);  // vmcnt(8): the first group landed; the second may be in flight
      } else if (GF) {
        epi_preload<EPI, 0>(g, ea, pre);
        __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the first group landed (nothing else in flight)
      }
    }
    RingItem nx;
    if (next < items && EPI != EPI_QKN) {
      nx = ring_item<AK, BK_, SW>(g, next, items, tiles, tiles_n, wid, lane);
      ring_issue<AK, BK_, SW>(g, nx, 0, lds0, wid, lane);
      if (nx.nk > 1) ring_issue<AK, BK_, SW>(g, nx, 1, lds0, wid, lane);
      if (nx.nk > 2) ring_issue<AK, BK_, SW>(g, nx, 2, lds0, wid, lane);
    }
    if (ABL == 3) {
      // diagnostic timing ablation (wrong results): no epilogue, but the accumulators stay live (a store
      // no real run takes) so the K loop's MFMAs are not dead code
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (s == 1.2345e37f) reinterpret_cast<float*>(g.C)[threadIdx.x] = s;
    } else if (SW) {
      epilogue_ring_swf(g, acc, stg, lane, it, wm, wn, bias8, bias8b);
    } else if (EPI == EPI_QKN) {
      epilogue_ring_qkn(g, acc, stg, lane, ea, bias8, it, wm, wn);
    } else if (EPI == EPI_SWB) {
      epilogue_ring<EPI, 0, 2>(g, acc, stg, lane, ea, bias8, pre);
      epi_preload<EPI, 4>(g, ea, pre);
      epilogue_ring<EPI, 2, 4>(g, acc, stg, lane, ea, bias8, pre2);
      epi_preload<EPI, 6>(g, ea, pre2);
      epilogue_ring<EPI, 4, 6>(g, acc, stg, lane, ea, bias8, pre);
      epilogue_ring<EPI, 6, 8>(g, acc, stg, lane, ea, bias8, pre2);
    } else if (GF == 2) {
      epilogue_ring<EPI, 0, 2>(g, acc, stg, lane, ea, bias8, pre);
      epi_preload<EPI, 2>(g, ea, pre);
      epilogue_ring<EPI, 2, 4>(g, acc, stg, lane, ea, bias8, pre);
      epi_preload<EPI, 4>(g, ea, pre);
      epilogue_ring<EPI, 4, 6>(g, acc, stg, lane, ea, bias8, pre);
      epi_preload<EPI, 6>(g, ea, pre);
      epilogue_ring<EPI, 6, 8>(g, acc, stg, lane, ea, bias8, pre);
    } else if (GF == 4) {
      epilogue_ring<EPI, 0, 4>(g, acc, stg, lane, ea, bias8, pre);
      epi_preload<EPI, 4>(g, ea, pre);
      epilogue_ring<EPI, 4, 8>(g, acc, stg, lane, ea, bias8, pre);
    } else {
      epilogue_ring<EPI, 0, 8, ABL == 5>(g, acc, stg, lane, ea, bias8, pre);
    }
    if (TL) tl_stamp(g, kth, 3, wid, lane);
    ++kth;
    if (next >= items) break;
    if (EPI == EPI_QKN) {  // the next item's first tiles after this epilogue (its table loads are compiler-waited)
      nx = ring_item<AK, BK_, SW>(g, next, items, tiles, tiles_n, wid, lane);
      ring_issue<AK, BK_, SW>(g, nx, 0, lds0, wid, lane);
      if (nx.nk > 1) ring_issue<AK, BK_, SW>(g, nx, 1, lds0, wid, lane);
      if (nx.nk > 2) ring_issue<AK, BK_, SW>(g, nx, 2, lds0, wid, lane);
    }
    // The next item's first LDS-DMA into stage 3 (tile 3, issued at its K step 0) follows its barrier
    // X_0, which every wave reaches only after its staging reads (raw_barrier: lgkmcnt(0) first).
    item = next;
    it = nx;
    // the epilogue's S stores are younger than the next item's pre-issued tiles 0-2 (EPI_QKN: older)
    pend = ABL == 3 || ABL == 5 || EPI == EPI_QKN ? 0 : S;
  }
}

template <bool AK, bool BK_, int TM, int TN, int WGM, int WGN>
int launch(const GemmArgs& g, int splits, hipStream_t s) {
  using G = Geo<TM, TN, WGM, WGN>;
  const int tiles = ((g.M + TM - 1) / TM) * ((g.N + TN - 1) / TN);
  dim3 grid(tiles, splits);
  hipLaunchKernelGGL((gemm_bf16_kernel<AK, BK_, TM, TN, WGM, WGN>), grid, dim3(G::T), G::LDS, s, g);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

// Epilogue stagger (GemmArgs::stagger, 10-ns ticks; diagnostic build only). Measured at the JiT-B/16 B=8
// shapes with 200-1500 ticks (profiles/r02/r02q_gemm_stagger_ab.json): no gain on any shape, larger delays
// only add their own length, i.e. the epilogues are not a chip-wide synchronized HBM burst. Off in
// production.
#ifdef VPT_DIAG
int g_stagger_override = 0;  // vpt_gemm_set_stagger
int g_swb_abl = 0;           // vpt_gemm_set_swb_ablation (SwiGLU-backward ring GEMM timing ablations, wrong results)
int g_swb_one_group = 0;     // vpt_gemm_set_swb_one_group (A/B: the SwiGLU-backward epilogue's older preload form)
#endif
inline int ring_stagger() {
#ifdef VPT_DIAG
  return g_stagger_override;
#else
  return 0;
#endif
}

template <bool AK, bool BK_, bool PP, int ABL = 0, bool DMAC = false, bool STAMP = false, bool TL = false, int SW = 0>
int launch_ring(const GemmArgs& g, int splits, hipStream_t s) {
  constexpr int LDS = RSTAGES * 2 * 256 * RBK * 2;  // the epilogue stages through ring stage 3
  const int items = ((g.M + 255) / 256) * ((g.N + 255) / 256) * splits;
  // the stamped / timeline diagnostic builds size their buffers for the persistent 256-block walk
  const int rg = g.ring_grid > 0 ? g.ring_grid : (STAMP || TL) ? 256 : items;
  const int grid = rg < items ? rg : items;
  const int epi = SW ? EPI_PLAIN : epi_mode(g);
  GemmArgs ga = g;
  ga.stagger = ring_stagger();
  const GemmArgs& gl = ga;
  if (!AK && !SW && g.rsum) {  // fused bias gradient (wgrad direction)
    if (epi == EPI_ACC)
      hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, 0, EPI_ACC, true>), dim3(grid), dim3(512), LDS,
                         s, gl);
    else
      hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, 0, EPI_PLAIN, true>), dim3(grid), dim3(512),
                         LDS, s, gl);
  } else if (epi == EPI_RESID)
    hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, SW, SW ? 0 : EPI_RESID>), dim3(grid), dim3(512),
                       LDS, s, gl);
#ifdef VPT_DIAG
  else if (epi == EPI_SWB && g_swb_one_group)
    hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, SW, SW ? 0 : EPI_SWB1>), dim3(grid), dim3(512),
                       LDS, s, gl);
#endif
  else if (epi == EPI_SWB)
    hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, SW, SW ? 0 : EPI_SWB>), dim3(grid), dim3(512),
                       LDS, s, gl);
  else if (epi == EPI_ACC)
    hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, SW, SW ? 0 : EPI_ACC>), dim3(grid), dim3(512),
                       LDS, s, gl);
  else if (epi == EPI_QKN) {
    if constexpr (AK && BK_ && SW == 0 && ABL == 0 && !STAMP && !TL && !DMAC)
      hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, 0, EPI_QKN>), dim3(grid), dim3(512), LDS, s,
                         gl);
    else
      VPT_CHECK_ARG(false, "gemm ring: the QK-norm epilogue is a forward (k-major x k-major) mode");
  } else
    hipLaunchKernelGGL((gemm_ring_kernel<AK, BK_, PP, ABL, DMAC, STAMP, TL, SW, EPI_PLAIN>), dim3(grid), dim3(512), LDS, s,
                       gl);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

#ifdef VPT_DIAG
#include "diag/gemm_ring4.inc"
#endif

// launch_r2 with the (diagnostic) start stagger of ring_stagger()
inline int launch_r2_st(const GemmArgs& g, bool ak, bool bk, hipStream_t s) {
  GemmArgs ga = g;
  ga.stagger = ring_stagger();
  return launch_r2(ga, ak, bk, s);
}

template <bool AK, bool BK_>
int launch_geo(const GemmArgs& g, int splits, int geo, hipStream_t s) {
  if (geo != 128 && geo != 2562 && g.N % 8 != 0) geo = 128;  // ring epilogue stores 8-column chunks
  if (geo == 256) return use_r2(g, AK) ? launch_r2_st(g, AK, BK_, s) : launch_ring<AK, BK_, true>(g, splits, s);
  if (geo == kGeoR2x128) return launch_r2_128(g, AK, BK_, s);
#ifdef VPT_DIAG
  // diagnostic build only (libvpt_hip_diag.so): A/B geometries, timing ablations with WRONG results
  // (2563, 2564), stamped / timeline builds
  if (geo == 2561) return launch_ring<AK, BK_, false>(g, splits, s);  // ring without the stagger (A/B only)
  if (AK && BK_ && geo == 2563) return launch_ring<AK, BK_, true, 1>(g, splits, s);  // ablation, wrong results
  if (AK && BK_ && geo == 2564) return launch_ring<AK, BK_, true, 2>(g, splits, s);  // ablation, wrong results
  if (geo == 2565) return launch_ring<AK, BK_, true, 0, true>(g, splits, s);  // DMA in the MFMA phase
  if (AK && BK_ && geo == 2566 && g.dbg) return launch_ring<AK, BK_, true, 0, false, true>(g, splits, s);  // stamps
  if (AK && BK_ && geo == 2567 && g.dbg) return launch_ring<AK, BK_, true, 0, false, false, true>(g, splits, s);
  if (geo == 2568) return launch_ring<AK, BK_, true, 3>(g, splits, s);  // no epilogue (wrong results)
  if (AK && BK_ && geo == 2572) return launch_ring<AK, BK_, true, 4>(g, splits, s);  // stores dropped (wrong)
  if (AK && BK_ && geo == 2573) return launch_ring<AK, BK_, true, 5>(g, splits, s);  // no stores (wrong)
  if (geo == 2569 && g.sw != 1 && !g.rsum) return launch_ring4<AK, BK_>(g, splits, s);  // 4-wave ring
  if (AK && BK_ && geo == 2570) return launch_ring4<AK, BK_, 1>(g, splits, s);  // 4-wave, no DMA (wrong results)
  if (AK && BK_ && geo == 2571) return launch_ring4<AK, BK_, 3>(g, splits, s);  // 4-wave, no epilogue (wrong)
  if (geo == 2562) return launch<AK, BK_, 256, 256, 2, 4>(g, splits, s);  // 2-stage BK=64 T256 (A/B only)
  // 128x160 tiles (M = 4096, N = 1280: 256 tiles, one per CU), k-major B only: 4 waves of 64x80 / 8 of 32x80
  if (AK && BK_ && geo == 1601) return launch<AK, BK_, 128, 160, 2, 2>(g, splits, s);
  if (AK && BK_ && geo == 1602) return launch<AK, BK_, 128, 160, 4, 2>(g, splits, s);
#endif
  return launch<AK, BK_, 128, 128, 2, 2>(g, splits, s);
}

// A column-sum job that rides a split-K reduce launch (vpt_linear_wgrad_rr): out[c] (=|+=) sum_r part[r][c].
struct ColSumJob {
  const float* part;
  int R, C;
  float* out;
  int acc;
};

// Fixed-order sum of the split-K partial slabs (blocks [0, cblocks)) and, in the same launch, of the
// per-split row sums of a fused bias gradient (blocks [cblocks, xblock0): rout[m] (+)= sum_z rpart[z][m]) and of an
// unrelated column-sum job (blocks from xblock0, 16 columns each: colsum_block<64>).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, long n, int splits,
                                                            long stride, void* out, int out_mode, long cblocks,
                                                            const float* __restrict__ rpart, int rsplits, int rn,
                                                            float* rout, int racc, const bf16_t* __restrict__ bias,
                                                            const bf16_t* __restrict__ resid, long ldr, int ncols,
                                                            long xblock0, ColSumJob xj) {
  if ((long)blockIdx.x >= xblock0) {
    __shared__ floatx4 red[64][4];
    colsum_block<64>(xj.part, xj.R, xj.C, xj.out, xj.acc, (int)((long)blockIdx.x - xblock0), red);
    return;
  }
  if ((long)blockIdx.x >= cblocks) {
    const long m = ((long)blockIdx.x - cblocks) * blockDim.x + threadIdx.x;
    if (m >= rn) return;
    float v = rpart[m];
    for (int z = 1; z < rsplits; ++z) v += rpart[(long)z * rn + m];
    rout[m] = racc ? rout[m] + v : v;
    return;
  }
  const long i4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  floatx4 s = *reinterpret_cast<const floatx4*>(part + i4);
  for (int z = 1; z < splits; ++z) s += *reinterpret_cast<const floatx4*>(part + z * stride + i4);
  if (bias || resid) {  // the GEMM epilogue's bias / residual, applied to the summed slabs (bf16 output)
    const long row = i4 / ncols, col = i4 - row * ncols;
    if (bias) {
      const uint2 bv = *reinterpret_cast<const uint2*>(bias + col);
      s[0] += __uint_as_float(bv.x << 16); s[1] += __uint_as_float(bv.x & 0xffff0000u);
      s[2] += __uint_as_float(bv.y << 16); s[3] += __uint_as_float(bv.y & 0xffff0000u);
    }
    if (resid) {  // reference semantics: residual + bf16(linear output), rounded again to bf16
      const uint2 rv = *reinterpret_cast<const uint2*>(resid + row * ldr + col);
      s[0] = bf2f(f2bf(s[0])) + __uint_as_float(rv.x << 16);
      s[1] = bf2f(f2bf(s[1])) + __uint_as_float(rv.x & 0xffff0000u);
      s[2] = bf2f(f2bf(s[2])) + __uint_as_float(rv.y << 16);
      s[3] = bf2f(f2bf(s[3])) + __uint_as_float(rv.y & 0xffff0000u);
    }
  }
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

// Geometry choice: the 256x256 ring when its grid (x split-K slices) fills most of the 256 CUs,
// otherwise 128x128 (2 blocks/CU, 4x the tiles). `req` (128 / 256) forces one (vpt_gemm_bf16_tiled).
#ifdef VPT_DIAG
int g_nf4_abl = 0;                    // vpt_gemm_set_nf4_ablation (timing only)
unsigned long long* g_dbg = nullptr;  // vpt_gemm_set_debug
int g_geo_override = 0;               // vpt_gemm_set_geometry
int g_ring_grid_override = 0;         // vpt_gemm_set_ring_grid
#endif
int pick_geo(int M, int N, int splits, int req) {
#ifdef VPT_DIAG
  if (g_geo_override) return g_geo_override;
#endif
  if (req) return req;
  const long t256 = (long)((M + 255) / 256) * ((N + 255) / 256) * splits;
  return t256 >= 160 ? 256 : 128;
}

int gemm_impl(const void* A, long lda, int a_kmajor, const void* B, long ldb, int b_kmajor, void* C, long ldc, int M,
              int N, int K, const void* bias, const void* resid, long ldr, int out_mode, int act, int splits,
              void* workspace, float alpha, int geo_req, int ring_grid, void* stream, float* rsum_out = nullptr,
              int rsum_acc = 0, bool* rsum_done = nullptr, const void* A2 = nullptr, long lda2 = 0,
              const void* B2 = nullptr, long ldb2 = 0, int K2 = 0, const void* const* B2g = nullptr, int G = 0,
              int g_n = 0, int alpha_cols = 0, const ColSumJob* xj = nullptr);

}  // namespace

extern "C" int vpt_gemm_bf16(const void* A, long lda, int a_kmajor, const void* B, long ldb,
                             int b_kmajor, void* C, long ldc, int M, int N, int K,
                             const void* bias, const void* resid, long ldr, int out_mode, int act,
                             int splits, void* workspace, float alpha, void* stream) {
  return gemm_impl(A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, M, N, K, bias, resid, ldr, out_mode, act, splits,
                   workspace, alpha, 0, 0, stream);
}

// C[M,N] = A . B (as vpt_gemm_bf16, one split) + A2 . B2 over K2 more reduction elements in the same f32
// accumulator: the LoRA term of LoRALinear (src/modules/peft/lora.py:92-104) as a K-extension of the base
// GEMM (forward: A2 = s * x . down^T [M][r], B2 = up [N][r]; input gradient: A2 = s * dy . up [M][r], B2 = down
// [r][K_in], the layout of B). A and A2 k-major; K % 64 == 0; K2 % 8 == 0, 0 < K2 <= 256. splits > 1: split-K
// (the extension rides the last slice; bias / residual applied by the slab reduce; vpt_gemm_workspace_bytes).
extern "C" int vpt_gemm_bf16_lora(const void* A, long lda, const void* B, long ldb, int b_kmajor, const void* A2,
                                  long lda2, const void* B2, long ldb2, int K2, void* C, long ldc, int M, int N, int K,
                                  const void* bias, const void* resid, long ldr, int out_mode, int splits,
                                  void* workspace, int geometry, void* stream) {
  VPT_CHECK_ARG(A2 && B2, "vpt_gemm_bf16_lora: null LoRA operand");
  VPT_CHECK_ARG(K % 64 == 0 && K2 > 0 && K2 <= 256 && K2 % 8 == 0, "vpt_gemm_bf16_lora: K % 64 == 0, K2 in 8..256, K2 % 8 == 0");
  VPT_CHECK_ARG(lda2 % 8 == 0 && ldb2 % 8 == 0 && lda2 >= K2 && (b_kmajor ? ldb2 >= K2 : ldb2 >= N),
                "vpt_gemm_bf16_lora: LoRA leading dims (16-B multiples, >= K2 / N)");
  VPT_CHECK_ARG(geometry == 0 || geometry == 128 || geometry == 256 || geometry == kGeoR2x128,
                "vpt_gemm_bf16_lora: geometry 0, 128, 256 or 1281");
  return gemm_impl(A, lda, 1, B, ldb, b_kmajor, C, ldc, M, N, K, bias, resid, ldr, out_mode, ACT_NONE, splits, workspace,
                   1.f, geometry, 0, stream, nullptr, 0, nullptr, A2, lda2, B2, ldb2, K2);
}

// G LoRA targets that read the same input, computed as ONE GEMM (the base weights stacked [G * g_n][K]): outputs
// C[:, g * g_n : (g + 1) * g_n] = A . W_g^T + A2[:, g * r : (g + 1) * r] . up_g^T (up_g = B2s[g], [g_n][r]).
extern "C" int vpt_gemm_bf16_lora_grouped(const void* A, long lda, const void* B, long ldb, const void* A2, long lda2,
                                          const void* const* B2s, int G, int r, void* C, long ldc, int M, int g_n,
                                          int K, const void* bias, const void* resid, long ldr, int splits,
                                          void* workspace, int geometry, void* stream) {
  VPT_CHECK_ARG(A2 && B2s && G > 0 && G <= 4, "vpt_gemm_bf16_lora_grouped: 1..4 groups");
  for (int i = 0; i < G; ++i) VPT_CHECK_ARG(B2s[i], "vpt_gemm_bf16_lora_grouped: null up");
  VPT_CHECK_ARG(K % 64 == 0 && r > 0 && r <= 64 && r % 8 == 0 && g_n % 128 == 0,
                "vpt_gemm_bf16_lora_grouped: K % 64 == 0, r in 8..64 (r % 8 == 0), g_n % 128 == 0");
  VPT_CHECK_ARG(lda2 % 8 == 0 && lda2 >= G * r, "vpt_gemm_bf16_lora_grouped: lda2 >= G * r (16-B multiple)");
  VPT_CHECK_ARG(geometry == 0 || geometry == 128 || geometry == 256 || geometry == kGeoR2x128,
                "vpt_gemm_bf16_lora_grouped: geometry 0, 128, 256 or 1281");
  return gemm_impl(A, lda, 1, B, ldb, 1, C, ldc, M, G * g_n, K, bias, resid, ldr, OUT_BF16, ACT_NONE, splits, workspace,
                   1.f, geometry, 0, stream, nullptr, 0, nullptr, A2, lda2, B2s[0], r, r, B2s, G, g_n);
}

// vpt_gemm_bf16_lora / vpt_gemm_bf16_lora_grouped with an output scale: alpha multiplies the f32 result (base +
// extension) of columns [0, alpha_cols) before bias / residual and the one bf16 rounding (alpha_cols = 0: every
// column; otherwise a multiple of 128) -- the attention q projection emitted pre-scaled for the attention kernels.
// splits must be 1.
extern "C" int vpt_gemm_bf16_lora_scaled(const void* A, long lda, const void* B, long ldb, int b_kmajor, const void* A2,
                                         long lda2, const void* B2, long ldb2, int K2, void* C, long ldc, int M, int N,
                                         int K, const void* bias, const void* resid, long ldr, int geometry, float alpha,
                                         int alpha_cols, void* stream) {
  VPT_CHECK_ARG(A2 && B2, "vpt_gemm_bf16_lora_scaled: null LoRA operand");
  VPT_CHECK_ARG(K % 64 == 0 && K2 > 0 && K2 <= 256 && K2 % 8 == 0, "vpt_gemm_bf16_lora_scaled: K % 64 == 0, K2 in 8..256, K2 % 8 == 0");
  VPT_CHECK_ARG(lda2 % 8 == 0 && ldb2 % 8 == 0 && lda2 >= K2 && (b_kmajor ? ldb2 >= K2 : ldb2 >= N),
                "vpt_gemm_bf16_lora_scaled: LoRA leading dims (16-B multiples, >= K2 / N)");
  VPT_CHECK_ARG(geometry == 0 || geometry == 128 || geometry == 256 || geometry == kGeoR2x128,
                "vpt_gemm_bf16_lora_scaled: geometry 0, 128, 256 or 1281");
  return gemm_impl(A, lda, 1, B, ldb, b_kmajor, C, ldc, M, N, K, bias, resid, ldr, OUT_BF16, ACT_NONE, 1, nullptr,
                   alpha, geometry, 0, stream, nullptr, 0, nullptr, A2, lda2, B2, ldb2, K2, nullptr, 0, 0, alpha_cols);
}

extern "C" int vpt_gemm_bf16_lora_grouped_scaled(const void* A, long lda, const void* B, long ldb, const void* A2,
                                                 long lda2, const void* const* B2s, int G, int r, void* C, long ldc,
                                                 int M, int g_n, int K, const void* bias, const void* resid, long ldr,
                                                 int geometry, float alpha, int alpha_cols, void* stream) {
  VPT_CHECK_ARG(A2 && B2s && G > 0 && G <= 4, "vpt_gemm_bf16_lora_grouped_scaled: 1..4 groups");
  for (int i = 0; i < G; ++i) VPT_CHECK_ARG(B2s[i], "vpt_gemm_bf16_lora_grouped_scaled: null up");
  VPT_CHECK_ARG(K % 64 == 0 && r > 0 && r <= 64 && r % 8 == 0 && g_n % 128 == 0,
                "vpt_gemm_bf16_lora_grouped_scaled: K % 64 == 0, r in 8..64 (r % 8 == 0), g_n % 128 == 0");
  VPT_CHECK_ARG(lda2 % 8 == 0 && lda2 >= G * r, "vpt_gemm_bf16_lora_grouped_scaled: lda2 >= G * r (16-B multiple)");
  VPT_CHECK_ARG(geometry == 0 || geometry == 128 || geometry == 256 || geometry == kGeoR2x128,
                "vpt_gemm_bf16_lora_grouped_scaled: geometry 0, 128, 256 or 1281");
  return gemm_impl(A, lda, 1, B, ldb, 1, C, ldc, M, G * g_n, K, bias, resid, ldr, OUT_BF16, ACT_NONE, 1, nullptr,
                   alpha, geometry, 0, stream, nullptr, 0, nullptr, A2, lda2, B2s[0], r, r, B2s, G, g_n, alpha_cols);
}

// Any number G of LoRA targets reading the same input, bases stacked [G * g_n][K] and adapters' ups stacked
// [G * g_n][r] (B2, ld r): C[:, g*g_n:(g+1)*g_n] = A . W_g^T + A2[:, g*r:(g+1)*r] . up_g^T. The cross-attention
// k / v projections of a fixed text context for every transformer block of a step as one GEMM.
extern "C" int vpt_gemm_bf16_lora_stacked(const void* A, long lda, const void* B, long ldb, const void* A2, long lda2,
                                          const void* B2, int G, int r, void* C, long ldc, int M, int g_n, int K,
                                          int splits, void* workspace, int geometry, void* stream) {
  VPT_CHECK_ARG(A2 && B2 && G > 0, "vpt_gemm_bf16_lora_stacked: null LoRA operand");
  VPT_CHECK_ARG(K % 64 == 0 && r > 0 && r <= 64 && r % 8 == 0 && g_n % 128 == 0,
                "vpt_gemm_bf16_lora_stacked: K % 64 == 0, r in 8..64 (r % 8 == 0), g_n % 128 == 0");
  VPT_CHECK_ARG(lda2 % 8 == 0 && lda2 >= (long)G * r, "vpt_gemm_bf16_lora_stacked: lda2 >= G * r (16-B multiple)");
  VPT_CHECK_ARG((long)G * g_n < (1L << 31), "vpt_gemm_bf16_lora_stacked: G * g_n < 2^31");
  VPT_CHECK_ARG(geometry == 0 || geometry == 128 || geometry == 256 || geometry == kGeoR2x128,
                "vpt_gemm_bf16_lora_stacked: geometry 0, 128, 256 or 1281");
  return gemm_impl(A, lda, 1, B, ldb, 1, C, ldc, M, G * g_n, K, nullptr, nullptr, 0, OUT_BF16, ACT_NONE, splits,
                   workspace, 1.f, geometry, 0, stream, nullptr, 0, nullptr, A2, lda2, B2, r, r, nullptr, G, g_n);
}

extern "C" int vpt_gemm_bf16_tiled(const void* A, long lda, int a_kmajor, const void* B, long ldb, int b_kmajor,
                                   void* C, long ldc, int M, int N, int K, const void* bias, const void* resid,
                                   long ldr, int out_mode, int act, int splits, void* workspace, float alpha,
                                   int geometry, int ring_grid, void* stream) {
  VPT_CHECK_ARG(geometry == 0 || geometry == 128 || geometry == 256 || geometry == kGeoR2x128,
                "vpt_gemm_bf16_tiled: geometry 0, 128, 256 or 1281");
  VPT_CHECK_ARG(ring_grid >= 0 && ring_grid <= 65536, "vpt_gemm_bf16_tiled: ring_grid 0..65536");
  return gemm_impl(A, lda, a_kmajor, B, ldb, b_kmajor, C, ldc, M, N, K, bias, resid, ldr, out_mode, act, splits,
                   workspace, alpha, geometry, ring_grid, stream);
}

// The JiT attention input projection with its per-head QK-RMSNorm + RoPE in the epilogue: qkv[M][3D] = x . W^T + b
// (bf16, as vpt_gemm_bf16) and qk[M][2D] = (rope(rms(q) wq) * q_scale | rope(rms(k) wk)) -- bitwise what
// vpt_qknorm_rope_fwd computes from that qkv (src/models/jit/denoiser.py:307-316, 318-323, 369-373, 98-111). Always
// the 256x256 ring (its epilogue owns whole 64-column heads).
extern "C" int vpt_linear_qknorm_rope(const void* x, long ldx, const void* w, long ldw, const void* bias, void* qkv,
                                      long ldqkv, void* qk, long ldqk, int M, int D, int K, const void* wq,
                                      const void* wk, const float* cos_t, const float* sin_t, int rows_per_seq,
                                      float eps, float q_scale, void* stream) {
  VPT_CHECK_ARG(x && w && qkv && qk && wq && wk && cos_t && sin_t, "vpt_linear_qknorm_rope: null pointer");
  VPT_CHECK_ARG(M > 0 && K > 0 && D > 0 && D % 64 == 0 && K % 8 == 0 && rows_per_seq > 0,
                "vpt_linear_qknorm_rope: heads of 64, K % 8 == 0");
  VPT_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0 && ldqkv % 8 == 0 && ldqk % 8 == 0 && ldqkv >= 3L * D && ldqk >= 2L * D,
                "vpt_linear_qknorm_rope: 16-B leading dims, qkv >= 3D and qk >= 2D columns");
  GemmArgs g = {};
  g.A = (const bf16_t*)x; g.lda = ldx;
  g.B = (const bf16_t*)w; g.ldb = ldw;
  g.bias = (const bf16_t*)bias;
  g.M = M; g.N = 3 * D; g.K = K;
  g.act = ACT_NONE;
  g.alpha = 1.f;
  g.k_split = K; g.splits = 1;
  g.C = qkv; g.ldc = ldqkv; g.out_mode = OUT_BF16;
  g.C2 = (bf16_t*)qk; g.ldc2 = ldqk;
  g.qk_d = D; g.rps = rows_per_seq;
  g.qk_wq = (const bf16_t*)wq; g.qk_wk = (const bf16_t*)wk;
  g.rcos = cos_t; g.rsin = sin_t;
  g.qk_scale = q_scale; g.qk_eps = eps;
  return launch_ring<true, true, true>(g, 1, (hipStream_t)stream);
}

namespace {
// rsum_out (wgrad direction, ring geometry only): also rsum_out[m] (+)= sum_k A(m, k) (the bias gradient),
// from per-split row sums in the workspace behind the split slabs; *rsum_done tells whether it was done.
int gemm_impl(const void* A, long lda, int a_kmajor, const void* B, long ldb, int b_kmajor, void* C, long ldc, int M,
              int N, int K, const void* bias, const void* resid, long ldr, int out_mode, int act, int splits,
              void* workspace, float alpha, int geo_req, int ring_grid, void* stream, float* rsum_out, int rsum_acc,
              bool* rsum_done, const void* A2, long lda2, const void* B2, long ldb2, int K2,
              const void* const* B2g, int G, int g_n, int alpha_cols, const ColSumJob* xj) {
  VPT_CHECK_ARG(A && B && C, "vpt_gemm_bf16: null operand");
  VPT_CHECK_ARG(alpha_cols >= 0 && alpha_cols % 128 == 0, "vpt_gemm_bf16: alpha_cols a multiple of 128");
  VPT_CHECK_ARG(M > 0 && N > 0 && K > 0, "vpt_gemm_bf16: empty shape");
  VPT_CHECK_ARG(N % 4 == 0, "vpt_gemm_bf16: N%4 required");
  VPT_CHECK_ARG((!a_kmajor && !b_kmajor) || K % 8 == 0, "vpt_gemm_bf16: k-major operands need K%8==0");
  VPT_CHECK_ARG(lda % 8 == 0 && ldb % 8 == 0 && ldc % 4 == 0, "vpt_gemm_bf16: leading dims must be 16B multiples");
  VPT_CHECK_ARG(a_kmajor || M % 8 == 0, "vpt_gemm_bf16: mn-major A needs M%8==0");
  VPT_CHECK_ARG(b_kmajor || N % 8 == 0, "vpt_gemm_bf16: mn-major B needs N%8==0");
  VPT_CHECK_ARG(out_mode >= 0 && out_mode <= 2, "vpt_gemm_bf16: bad out_mode");
  VPT_CHECK_ARG(!resid || out_mode == OUT_BF16, "vpt_gemm_bf16: residual only with bf16 output");
  if (splits < 1) splits = 1;
  GemmArgs g = {};
  g.A = (const bf16_t*)A; g.lda = lda;
  g.B = (const bf16_t*)B; g.ldb = ldb;
  g.bias = (const bf16_t*)bias;
  g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.M = M; g.N = N; g.K = K;
  g.act = act;
  g.alpha = alpha;
  g.alpha_cols = alpha_cols < N ? alpha_cols : 0;
  g.ring_grid = ring_grid;
  g.A2 = (const bf16_t*)A2; g.lda2 = lda2;
  g.B2 = (const bf16_t*)B2; g.ldb2 = ldb2;
  g.K2 = A2 ? K2 : 0;
  if (B2g && G > 0) {
    for (int i = 0; i < G; ++i) g.B2g[i] = (const bf16_t*)B2g[i];
    g.g_n = g_n;
  } else if (G > 0) {  // stacked groups: B2 = [G * g_n][K2]
    g.g_n = g_n;
  }
#ifdef VPT_DIAG
  g.dbg = g_dbg;
  if (g_ring_grid_override) g.ring_grid = g_ring_grid_override;
#endif
  hipStream_t s = (hipStream_t)stream;
  int final_mode = out_mode;
  if (splits > 1) {
    VPT_CHECK_ARG(workspace != nullptr, "vpt_gemm_bf16: split-K needs a workspace");
    VPT_CHECK_ARG(act == ACT_NONE && alpha == 1.f && (out_mode == OUT_BF16 || (!bias && !resid)),
                  "vpt_gemm_bf16: split-K epilogue: bias / residual with bf16 output only, no SiLU / alpha");
    VPT_CHECK_ARG(ldc == N, "vpt_gemm_bf16: split-K needs dense C");
    VPT_CHECK_ARG(N % 4 == 0 && (!resid || ldr % 4 == 0), "vpt_gemm_bf16: split-K epilogue needs N % 4 == 0");
    g.bias = nullptr;  // applied by the slab reduce
    g.resid = nullptr;
    int per = (K + splits - 1) / splits;
    per = (per + BK - 1) / BK * BK;
    splits = (K + per - 1) / per;
    g.k_split = per;
    g.splits = splits;
    g.C = workspace; g.ldc = N;
    g.split_stride = (long)M * N;
    g.out_mode = OUT_F32;
  } else {
    g.k_split = K;
    g.splits = 1;
    g.C = C; g.ldc = ldc;
    g.split_stride = 0;
    g.out_mode = out_mode;
  }
  int geo = pick_geo(M, N, splits, geo_req);
  if (geo == 256 && g.g_n > 0 && g.g_n % 256 != 0) geo = 128;  // grouped extension: a 256-wide tile would straddle
  if (geo == 256 && g.alpha_cols % 256 != 0) geo = 128;         // two groups; the ring applies alpha per 256-wide tile
  const bool rs = rsum_out && !a_kmajor && geo == 256 && N % 8 == 0 && workspace != nullptr;
  if (rsum_done) *rsum_done = rs;
  float* rpart = nullptr;
  if (rs) {  // per-split row sums behind the split slabs (16-B aligned)
    rpart = reinterpret_cast<float*>(workspace) + (splits > 1 ? ((long)splits * M * N + 3) / 4 * 4 : 0);
    g.rsum = rpart;
  }
  int rc;
  if (a_kmajor && b_kmajor) rc = launch_geo<true, true>(g, splits, geo, s);
  else if (a_kmajor && !b_kmajor) rc = launch_geo<true, false>(g, splits, geo, s);
  else if (!a_kmajor && b_kmajor) rc = launch_geo<false, true>(g, splits, geo, s);
  else rc = launch_geo<false, false>(g, splits, geo, s);
  if (rc != VPT_OK || (splits == 1 && !rs && !xj)) return rc;
  const long n = splits > 1 ? (long)M * N : 0;
  const int threads = 256;
  const long cblocks = (n / 4 + threads - 1) / threads;
  const long rblocks = rs ? (M + threads - 1) / threads : 0;
  const long xblocks = xj ? (xj->C + 15) / 16 : 0;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(cblocks + rblocks + xblocks), dim3(threads), 0, s,
                     (const float*)workspace, n, splits, (long)M * N, C, final_mode, cblocks, rpart, splits, M, rsum_out,
                     rsum_acc, splits > 1 ? (const bf16_t*)bias : nullptr, splits > 1 ? (const bf16_t*)resid : nullptr,
                     ldr, N, cblocks + rblocks, xj ? *xj : ColSumJob{});
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
}  // namespace

#ifdef VPT_DIAG
// ---- diagnostic build only (libvpt_hip_diag.so, include/vpt_hip_diag.h): process-wide switches ----
extern "C" int vpt_gemm_set_swb_one_group(int on) {
  g_swb_one_group = on;
  return VPT_OK;
}

extern "C" int vpt_gemm_set_r2(int mask) {
  VPT_CHECK_ARG(mask >= 0 && mask < 32, "vpt_gemm_set_r2: bit mask of 5 launch kinds");
  g_r2 = mask;
  return VPT_OK;
}

extern "C" int vpt_gemm_set_swb_ablation(int a) {
  VPT_CHECK_ARG(a == 0 || a == 3 || a == 4 || a == 6, "vpt_gemm_set_swb_ablation: 0, 3, 4 or 6");
  g_swb_abl = a;
  return VPT_OK;
}

extern "C" int vpt_gemm_set_geometry(int geo) {
  VPT_CHECK_ARG(geo == 0 || geo == 128 || geo == 256 || (geo >= 2561 && geo <= 2573) || geo == 1601 || geo == 1602,
                "vpt_gemm_set_geometry: 0, 128, 256 or 2561-2573");
  g_geo_override = geo;
  return VPT_OK;
}

// Ring grid size (blocks) for every ring GEMM: 0 restores the default (one block per item); 256 = the persistent walk
// with one block per CU.
extern "C" int vpt_gemm_set_ring_grid(int blocks) {
  VPT_CHECK_ARG(blocks >= 0 && blocks <= 65536, "vpt_gemm_set_ring_grid: 0..65536");
  g_ring_grid_override = blocks;
  return VPT_OK;
}

// Ring epilogue stagger in 10-ns ticks (0 = off, the production setting).
extern "C" int vpt_gemm_set_stagger(int ticks) {
  g_stagger_override = ticks;
  return VPT_OK;
}

// NF4 GEMM timing ablation (WRONG results): 0 off, 1 no dequant, 2 no NF4 loads and no dequant.
extern "C" int vpt_gemm_set_nf4_ablation(int a) {
  g_nf4_abl = a;
  return VPT_OK;
}

// Output buffer for the stamped ring build (geometry 2566), [256 blocks][8 waves][8] u64.
extern "C" int vpt_gemm_set_debug(unsigned long long* buf) {
  g_dbg = buf;
  return VPT_OK;
}

// Co-running-kernel probe: `blocks` one-wave workgroups that hold a CU each (dynamic LDS) for `ticks` of the 100-MHz
// constant clock and exit -- a stand-in for the RCCL / side-stream kernels that share the chip with a persistent GEMM.
namespace {
__global__ void occupy_kernel(long ticks, float* sink) {
  extern __shared__ float hold[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float acc = 0.f;
  while ((long)(__builtin_amdgcn_s_memrealtime() - t0) < ticks) {
    __builtin_amdgcn_s_sleep(4);
    acc += 1.f;
  }
  if (acc < 0.f) { hold[threadIdx.x] = acc; sink[threadIdx.x] = hold[threadIdx.x]; }  // never taken; keeps the LDS
}
}  // namespace

extern "C" int vpt_diag_occupy(int blocks, long ticks, int lds_bytes, float* sink, void* stream) {
  VPT_CHECK_ARG(blocks > 0 && blocks <= 4096 && ticks > 0 && ticks <= 1000000 && lds_bytes >= 0 && lds_bytes <= 163840,
                "vpt_diag_occupy: blocks 1..4096, ticks 1..1e6 (10 ms), lds <= 160 KB");
  hipLaunchKernelGGL(occupy_kernel, dim3(blocks), dim3(64), lds_bytes, (hipStream_t)stream, ticks, sink);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
#endif  // VPT_DIAG

extern "C" long vpt_gemm_workspace_bytes(int M, int N, int K, int splits) {
  (void)K;
  if (splits <= 1) return 0;
  return (long)splits * M * N * 4;
}

// ---- nn.Linear weight + bias gradient in one ring GEMM (torch autograd of F.linear; every Linear of
// denoiser.py, e.g. :318-323 / :492-504) -------------------------------------------------------------
// dw [N][K] (=|+=) dy^T . x and db [N] (=|+=) column sums of dy [M][N], both f32. On the 256x256 ring the
// column sums are row sums of the GEMM's mn-major A operand, taken by MFMAs against an all-ones fragment
// in the items of the first output tile and reduced with the split-K slabs in one launch; otherwise the
// colsum kernel (vpt_bias_grad) runs after the GEMM on the same workspace.
extern "C" int vpt_colsum_blocks(long M);
extern "C" int vpt_bias_grad(const void* in, long ld, long M, int N, float* part, float* out, int accumulate,
                             void* stream);

extern "C" long vpt_linear_wgrad_workspace_bytes(long M, int N, int K, int splits) {
  const int s = splits < 1 ? 1 : splits;
  const long slab = s > 1 ? ((long)s * N * K + 3) / 4 * 4 : 0;
  const long ring = (slab + (long)s * N) * 4;
  const long cs = (long)vpt_colsum_blocks(M) * N * 4;
  return ring > cs ? ring : cs;
}

namespace {
int linear_wgrad_impl(const void* dy, long lddy, const void* x, long ldx, float* dw, long lddw, float* db, long M,
                      int N, int K, int accumulate, int splits, void* workspace, int geometry, int ring_grid,
                      void* stream, const ColSumJob* xj) {
  VPT_CHECK_ARG(dy && x && dw && M > 0 && M < (1L << 31), "vpt_linear_wgrad: bad args");
  VPT_CHECK_ARG(!db || workspace, "vpt_linear_wgrad: a bias gradient needs the workspace");
  VPT_CHECK_ARG(geometry == 0 || geometry == 128 || geometry == 256, "vpt_linear_wgrad: geometry 0, 128 or 256");
  bool done = false;
  // the column-sum job (its own buffers) rides the reduce launch that follows the GEMM, which gemm_impl then issues
  // even without split-K slabs or bias row sums
  const int rc = gemm_impl(dy, lddy, 0, x, ldx, 0, dw, lddw, N, K, (int)M, nullptr, nullptr, 0,
                           accumulate ? OUT_F32_ACC : OUT_F32, ACT_NONE, splits, workspace, 1.f, geometry, ring_grid,
                           stream, db, accumulate, &done, nullptr, 0, nullptr, 0, 0, nullptr, 0, 0, 0, xj);
  if (rc != VPT_OK || !db || done) return rc;
  return vpt_bias_grad(dy, lddy, M, N, (float*)workspace, db, accumulate, stream);
}
}  // namespace

extern "C" int vpt_linear_wgrad(const void* dy, long lddy, const void* x, long ldx, float* dw, long lddw, float* db,
                                long M, int N, int K, int accumulate, int splits, void* workspace, int geometry,
                                int ring_grid, void* stream) {
  return linear_wgrad_impl(dy, lddy, x, ldx, dw, lddw, db, M, N, K, accumulate, splits, workspace, geometry, ring_grid,
                           stream, nullptr);
}

// vpt_linear_wgrad plus one unrelated column sum rr_out[c] (=|+=) sum_r rr_part[r][c] ([rr_R][rr_C] f32, e.g. an
// RMSNorm weight gradient's partial rows), computed by extra blocks of the weight gradient's split-K reduce launch
// instead of a launch of its own (vpt_reduce_rows semantics with its 64-row-group summation order, colsum_block<64>;
// vpt_reduce_rows itself switches to 256 row groups at R >= 256, so for such R the two sum in different, each fixed,
// orders: deterministic, not bitwise equal to the standalone reduce).
extern "C" int vpt_linear_wgrad_rr(const void* dy, long lddy, const void* x, long ldx, float* dw, long lddw, float* db,
                                   long M, int N, int K, int accumulate, int splits, void* workspace, int geometry,
                                   int ring_grid, const float* rr_part, int rr_R, int rr_C, float* rr_out, int rr_acc,
                                   void* stream) {
  VPT_CHECK_ARG(rr_part && rr_out && rr_R > 0 && rr_C > 0, "vpt_linear_wgrad_rr: bad column-sum job");
  const ColSumJob xj{rr_part, rr_R, rr_C, rr_out, rr_acc};
  return linear_wgrad_impl(dy, lddy, x, ldx, dw, lddw, db, M, N, K, accumulate, splits, workspace, geometry, ring_grid,
                           stream, &xj);
}

// ---- fused SwiGLU GEMMs (the JiT MLP, denoiser.py:480-506; FinalLayer 535-543) ---------------------
extern "C" int vpt_swiglu_fwd(const void* x12, long M, int F, void* h, void* stream);
extern "C" int vpt_swiglu_bwd(const void* dh, const void* x12, long M, int F, void* dx12, void* stream);

static bool swiglu_ring_ok(int M, int N) {
#ifdef VPT_DIAG
  if (g_geo_override && g_geo_override != 256) return false;
  if (g_geo_override == 256) return N % 256 == 0;
#endif
  return N % 256 == 0 && (long)((M + 255) / 256) * (N / 256) >= 160;
}

// x12 [M][2F] = x . W12^T + b12 (W12 = W1 | W2 [2F][K]) and h [M][F] = bf16(silu(x1)) * x2, from one ring
// GEMM whose epilogue pairs x1 / x2 (small shapes: the plain GEMM + vpt_swiglu_fwd, same roundings).
extern "C" int vpt_gemm_swiglu_fwd(const void* x, long ldx, const void* w12, long ldw, const void* b12, void* x12,
                                   long ldx12, void* h, long ldh, int M, int F, int K, void* stream) {
  VPT_CHECK_ARG(x && w12 && x12 && h, "vpt_gemm_swiglu_fwd: null pointer");
  VPT_CHECK_ARG(M > 0 && F > 0 && K > 0 && F % 8 == 0 && K % 8 == 0, "vpt_gemm_swiglu_fwd: bad shape");
  if (!swiglu_ring_ok(M, 2 * F) || ldx12 != 2 * F || ldh != F) {
    int rc = vpt_gemm_bf16(x, ldx, 1, w12, ldw, 1, x12, ldx12, M, 2 * F, K, b12, nullptr, 0, OUT_BF16, ACT_NONE, 1,
                           nullptr, 1.f, stream);
    if (rc) return rc;
    VPT_CHECK_ARG(ldx12 == 2 * F && ldh == F, "vpt_gemm_swiglu_fwd: dense x12 / h required");
    return vpt_swiglu_fwd(x12, M, F, h, stream);
  }
  VPT_CHECK_ARG(ldx % 8 == 0 && ldw % 8 == 0, "vpt_gemm_swiglu_fwd: leading dims must be 16B multiples");
  GemmArgs g = {};
  g.A = (const bf16_t*)x; g.lda = ldx;
  g.B = (const bf16_t*)w12; g.ldb = ldw;
  g.C = x12; g.ldc = ldx12;
  g.C2 = (bf16_t*)h; g.ldc2 = ldh;
  g.bias = (const bf16_t*)b12;
  g.M = M; g.N = 2 * F; g.K = K;
  g.k_split = K; g.splits = 1;
  g.out_mode = OUT_BF16; g.act = ACT_NONE; g.alpha = 1.f;
  g.sw = 1;
  if (use_r2(g, true)) return launch_r2_st(g, true, true, (hipStream_t)stream);
  return launch_ring<true, true, true, 0, false, false, false, 1>(g, 1, (hipStream_t)stream);
}

extern "C" long vpt_gemm_swiglu_bwd_workspace(int M, int F, int D) {
  (void)D;
  return swiglu_ring_ok(M, F) ? 0 : (long)M * F * 2;
}

// dx12 [M][2F] = SwiGLU backward of dh = dy . W3 (dy [M][D], W3 [D][F]) against x12, from one ring dgrad
// whose epilogue applies the SwiGLU derivative (small shapes: dgrad into `workspace` + vpt_swiglu_bwd).
extern "C" int vpt_gemm_swiglu_bwd(const void* dy, long lddy, const void* w3, long ldw3, const void* x12, long ldx12,
                                   void* dx12, long lddx12, int M, int F, int D, void* workspace, void* stream) {
  VPT_CHECK_ARG(dy && w3 && x12 && dx12, "vpt_gemm_swiglu_bwd: null pointer");
  VPT_CHECK_ARG(M > 0 && F > 0 && D > 0 && F % 8 == 0 && D % 8 == 0, "vpt_gemm_swiglu_bwd: bad shape");
  if (!swiglu_ring_ok(M, F) || ldx12 != 2 * F || lddx12 != 2 * F) {
    VPT_CHECK_ARG(workspace != nullptr, "vpt_gemm_swiglu_bwd: workspace required (vpt_gemm_swiglu_bwd_workspace)");
    VPT_CHECK_ARG(ldx12 == 2 * F && lddx12 == 2 * F, "vpt_gemm_swiglu_bwd: dense x12 / dx12 required");
    int rc = vpt_gemm_bf16(dy, lddy, 1, w3, ldw3, 0, workspace, F, M, F, D, nullptr, nullptr, 0, OUT_BF16, ACT_NONE, 1,
                           nullptr, 1.f, stream);
    if (rc) return rc;
    return vpt_swiglu_bwd(workspace, x12, M, F, dx12, stream);
  }
  VPT_CHECK_ARG(lddy % 8 == 0 && ldw3 % 8 == 0, "vpt_gemm_swiglu_bwd: leading dims must be 16B multiples");
  GemmArgs g = {};
  g.A = (const bf16_t*)dy; g.lda = lddy;
  g.B = (const bf16_t*)w3; g.ldb = ldw3;
  g.C = dx12; g.ldc = lddx12;
  g.aux = (const bf16_t*)x12; g.ldaux = ldx12;
  g.M = M; g.N = F; g.K = D;
  g.k_split = D; g.splits = 1;
  g.out_mode = OUT_BF16; g.act = ACT_NONE; g.alpha = 1.f;
  g.sw = 2;
#ifdef VPT_DIAG
  // timing ablations (WRONG results): 3 = no epilogue, 4 = dx12 stores dropped, 6 = x12 read from one L2-resident tile
  if (g_swb_abl == 3) return launch_ring<true, false, true, 3>(g, 1, (hipStream_t)stream);
  if (g_swb_abl == 4) return launch_ring<true, false, true, 4>(g, 1, (hipStream_t)stream);
  if (g_swb_abl == 6) return launch_ring<true, false, true, 6>(g, 1, (hipStream_t)stream);
#endif
  if (use_r2(g, true)) return launch_r2_st(g, true, false, (hipStream_t)stream);
  return launch_ring<true, false, true>(g, 1, (hipStream_t)stream);
}

// ---- NF4 dequant-in-GEMM with a fused LoRA K-extension (SDXL QLoRA, BASELINE config 5) ----------------
// Replaces, for every QLoRA target Linear (src/modules/peft/lora.py:92-104 over bnb Linear4bit,
// src/modules/quant/bnb.py:37-129), bnb's dequantize_4bit into a bf16 weight in HBM + the GEMM + the LoRA
// up-projection GEMM + the add, in both directions:
//   forward  y  = x . Wd^T (+ bias) + ds . up^T        Wd [N][K] NF4 (k-major B), ds = s * x . down^T [M][r]
//   dgrad    dx = dy . Wd       + vs . down            Wd read mn-major (B(n, k) = W[k][n]), vs = s * dy . up [M][r]
// The NF4 B tile (128 weight rows x one 64-element NF4 block each, or 64 rows x two half blocks) is loaded
// as packed codes + nested absmax into registers one K step ahead, dequantised exactly as bnb's
// dequantize_4bit (f32 NF4[code] * absmax, absmax = code2[qabsmax] * absmax2[blk / 256] + offset, then
// bf16) and written into the same LDS tile image the bf16 kernel uses; the activation operand arrives by
// LDS-DMA. No dequantised weight ever exists in HBM. The LoRA term is one extra K tile (r <= 64 valid k,
// zero-filled) from (ds | vs, up | down), so the sum is taken in the f32 accumulator before the single
// bf16 rounding. 128x128 tiles, 4 waves (T128 geometry), 2 LDS stages.
namespace {
struct Nf4Args {
  const uint8_t* packed;    // [N_w * K_w / 2]
  const uint8_t* qabsmax;   // [N_w * K_w / 64]
  const float* absmax2;     // [ceil(N_w * K_w / 64 / 256)]
  const float* code2;       // [256]
  const float* offset;      // [1]
  long kw;                  // K_w: input features of the quantised Linear (row length of W)
  const bf16_t* A2; long lda2;  // LoRA activation operand [M][r] (k-major) or null
  const bf16_t* B2; long ldb2;  // up [N][r] (k-major, forward) or down [r][K_w] (mn-major, dgrad)
  int r;
};

__constant__ float kNF4g[16] = {-1.0f, -0.6961928009986877f, -0.5250730514526367f, -0.39491748809814453f,
                                -0.28444138169288635f, -0.18477343022823334f, -0.09105003625154495f, 0.0f,
                                0.07958029955625534f, 0.16093020141124725f, 0.24611230194568634f,
                                0.33791524171829224f, 0.44070982933044434f, 0.5626170039176941f,
                                0.7229568362236023f, 1.0f};

// The 32 codes one thread dequantises per K step (16 packed bytes) and their block's nested absmax index.
struct Nf4Regs {
  uint4 codes;
  uint32_t q;   // qabsmax byte
  float a2;     // absmax2[blk / 256]
};

template <bool BKMAJ>
__device__ __forceinline__ long nf4_elem(const GemmArgs& g, const Nf4Args& f, int n0, int k0, int tid) {
  if (BKMAJ) {  // forward: B(n, k) = W[n][k]; thread -> weight row n0 + tid/2, k0 + 32 * (tid & 1)
    const int n = min(n0 + (tid >> 1), g.N - 1);
    return (long)n * f.kw + k0 + 32 * (tid & 1);
  } else {      // dgrad: B(n, k) = W[k][n]; thread -> weight row k0 + tid/4, columns n0 + 32 * (tid & 3)
    const int c = min(n0 + 32 * (tid & 3), g.N - 32);
    return (long)(k0 + (tid >> 2)) * f.kw + c;
  }
}

template <bool BKMAJ>
__device__ __forceinline__ Nf4Regs nf4_load(const GemmArgs& g, const Nf4Args& f, int n0, int k0, int tid) {
  const long e = nf4_elem<BKMAJ>(g, f, n0, k0, tid);  // first of 32 consecutive elements (one half block)
  const long blk = e >> 6;
  Nf4Regs r;
  r.codes = *reinterpret_cast<const uint4*>(f.packed + (e >> 1));
  r.q = f.qabsmax[blk];
  r.a2 = f.absmax2[blk >> 8];
  return r;
}

// Dequantise and write the thread's 32 elements into the stage's B image (k-major [128][64] or mn-major
// [64][128], the layouts read_frag expects).
template <bool BKMAJ>
__device__ __forceinline__ void nf4_store(char* lb, const Nf4Regs& r, const float* lut, const float* code2, float off,
                                          int tid) {
  float am;
  {
#pragma clang fp contract(off)  // bnb: dequantize_blockwise (a product), then absmax += offset (a sum)
    am = code2[r.q] * r.a2 + off;
  }
  const uint32_t w[4] = {r.codes.x, r.codes.y, r.codes.z, r.codes.w};
  const float2_t* lut2 = reinterpret_cast<const float2_t*>(lut);  // [256] (NF4[b >> 4], NF4[b & 15])
#pragma unroll
  for (int i = 0; i < 4; ++i) {  // 8 elements (4 packed bytes) per 16-B chunk
    float v[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float2_t pr = lut2[(w[i] >> (8 * j)) & 0xffu];  // one b64 read per packed byte
      v[2 * j] = pr[0] * am;       // first element in the high nibble
      v[2 * j + 1] = pr[1] * am;
    }
    const uint4 pk = pack8(v);
    if (BKMAJ) {
      *reinterpret_cast<uint4*>(lb + kmaj_off(tid >> 1, 4 * (tid & 1) + i)) = pk;
    } else {
      *reinterpret_cast<uint4*>(lb + mnmaj_off<128>(tid >> 2, 8 * (tid & 3) + 2 * i)) = pk;
    }
  }
}

// ABL (diagnostic build, timing only, WRONG results): 1 = no dequant (codes loaded, B tile not rewritten),
// 2 = no NF4 code loads either (B tile stale).
template <bool BKMAJ, int ABL = 0>
__global__ __launch_bounds__(256, 2) void gemm_nf4_kernel(GemmArgs g, Nf4Args f) {
  using G = Geo<128, 128, 2, 2>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* lut = reinterpret_cast<float*>(smem + G::LDS);  // byte -> NF4 pair table (256 x 2) + code2 (256)
  float* c2 = lut + 512;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / 2, wn = wid % 2;
  const int tiles_n = (g.N + 127) / 128;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int xcd = orig & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int m0 = wgid / tiles_n * 128, n0 = wgid % tiles_n * 128;

  lut[2 * tid] = kNF4g[tid >> 4];
  lut[2 * tid + 1] = kNF4g[tid & 15];
  c2[tid] = f.code2[tid];
  const float off = f.offset[0];

  floatx4 acc[G::MI][G::NI];
#pragma unroll
  for (int i = 0; i < G::MI; ++i)
#pragma unroll
    for (int j = 0; j < G::NI; ++j) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;  // K % 64 == 0 (checked on the host)
  Nf4Regs nr = nf4_load<BKMAJ>(g, f, n0, 0, tid);
  glds_tile<true, 128, 4>(smem, tile_ptr<true>(g.A, g.lda, m0, 0), g.lda, m0, g.M, BK, wid, lane);
  __syncthreads();  // lut / code2 visible
  nf4_store<BKMAJ>(smem + G::A_BYTES, nr, lut, c2, off, tid);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    char* nb = smem + (cur ^ 1) * G::STAGE;
    const bool more = kt + 1 < nk;
    if (more) {
      glds_tile<true, 128, 4>(nb, tile_ptr<true>(g.A, g.lda, m0, (kt + 1) * BK), g.lda, m0, g.M, BK, wid, lane);
      if (ABL < 2) nr = nf4_load<BKMAJ>(g, f, n0, (kt + 1) * BK, tid);
    } else if (f.A2) {
      // the LoRA K-extension tile (k in [0, r) of (A2, B2)) goes out under the last K step's MFMAs, into
      // the idle stage, instead of as an exposed load after the loop
      glds_tile<true, 128, 4>(nb, tile_ptr<true>(f.A2, f.lda2, m0, 0), f.lda2, m0, g.M, f.r, wid, lane);
      glds_tile<BKMAJ, 128, 4>(nb + G::A_BYTES, tile_ptr<BKMAJ>(f.B2, f.ldb2, n0, 0), f.ldb2, n0, g.N, f.r, wid, lane);
    }
    mma_tile<true, BKMAJ, G>(smem + cur * G::STAGE, acc, wm, wn, lane);
    if (more && ABL == 0) nf4_store<BKMAJ>(nb + G::A_BYTES, nr, lut, c2, off, tid);
    if (more && ABL == 1) asm volatile("" :: "v"(nr.codes.x), "v"(nr.codes.w), "v"(nr.q), "v"(nr.a2));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    cur ^= 1;
  }
  if (f.A2) {  // LoRA K-extension: k in [0, r) of (A2, B2) (loaded in the last K step), zero-filled to 64
    char* st = smem + cur * G::STAGE;
    zero_k_tail<true, 128, 256>(st, f.r, tid);
    zero_k_tail<BKMAJ, 128, 256>(st + G::A_BYTES, f.r, tid);
    __syncthreads();
    mma_tile<true, BKMAJ, G>(st, acc, wm, wn, lane);
    __syncthreads();
  }
  epilogue<G>(g, acc, smem, wid, lane, m0, n0, wm, wn, 0);
}
}  // namespace

// fwd (w_kmajor = 1): C[M][N] = A[M][K] . Wd[N][K]^T; dgrad (w_kmajor = 0): C[M][N] = A[M][K] . Wd[K][N]
// with Wd the NF4 weight of `kw` input features ([N][kw] forward, [K][kw = N] dgrad).
extern "C" int vpt_gemm_nf4(const void* A, long lda, const void* packed, const void* qabsmax, const float* absmax2,
                            const float* code2, const float* offset, long kw, int w_kmajor, const void* lora_a,
                            long lda2, const void* lora_b, long ldb2, int r, void* C, long ldc, int M, int N, int K,
                            const void* bias, const void* resid, long ldr, int out_mode, float alpha, void* stream) {
  VPT_CHECK_ARG(A && packed && qabsmax && absmax2 && code2 && offset && C, "vpt_gemm_nf4: null pointer");
  VPT_CHECK_ARG(M > 0 && N > 0 && K > 0, "vpt_gemm_nf4: empty shape");
  VPT_CHECK_ARG(K % 64 == 0 && lda % 8 == 0 && ldc % 4 == 0, "vpt_gemm_nf4: K % 64, 16-B leading dims");
  VPT_CHECK_ARG(w_kmajor ? (kw == K && N % 4 == 0) : (kw == N && N % 64 == 0),
                "vpt_gemm_nf4: forward needs kw == K; dgrad needs kw == N, N % 64 == 0");
  VPT_CHECK_ARG(!lora_a || (lora_b && r > 0 && r <= 64 && lda2 % 8 == 0 && ldb2 % 8 == 0 && (w_kmajor || N % 8 == 0)),
                "vpt_gemm_nf4: LoRA operands need 0 < r <= 64 and 16-B leading dims");
  VPT_CHECK_ARG(out_mode == OUT_BF16 || (out_mode == OUT_F32 && !resid), "vpt_gemm_nf4: out_mode bf16 or f32");
  GemmArgs g = {};
  g.A = (const bf16_t*)A; g.lda = lda;
  g.C = C; g.ldc = ldc;
  g.bias = (const bf16_t*)bias;
  g.resid = (const bf16_t*)resid; g.ldr = ldr;
  g.M = M; g.N = N; g.K = K;
  g.k_split = K; g.splits = 1; g.split_stride = 0;
  g.out_mode = out_mode; g.act = ACT_NONE; g.alpha = alpha;
  Nf4Args f = {(const uint8_t*)packed, (const uint8_t*)qabsmax, absmax2, code2, offset, kw,
               (const bf16_t*)lora_a, lda2, (const bf16_t*)lora_b, ldb2, r};
  using G = Geo<128, 128, 2, 2>;
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  const int lds = G::LDS + (512 + 256) * 4;
  hipStream_t s = (hipStream_t)stream;
#ifdef VPT_DIAG
  if (g_nf4_abl == 1) {
    if (w_kmajor) hipLaunchKernelGGL((gemm_nf4_kernel<true, 1>), dim3(tiles), dim3(256), lds, s, g, f);
    else hipLaunchKernelGGL((gemm_nf4_kernel<false, 1>), dim3(tiles), dim3(256), lds, s, g, f);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
  if (g_nf4_abl == 2) {
    if (w_kmajor) hipLaunchKernelGGL((gemm_nf4_kernel<true, 2>), dim3(tiles), dim3(256), lds, s, g, f);
    else hipLaunchKernelGGL((gemm_nf4_kernel<false, 2>), dim3(tiles), dim3(256), lds, s, g, f);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
#endif
  if (w_kmajor) hipLaunchKernelGGL(gemm_nf4_kernel<true>, dim3(tiles), dim3(256), lds, s, g, f);
  else hipLaunchKernelGGL(gemm_nf4_kernel<false>, dim3(tiles), dim3(256), lds, s, g, f);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

// ---- LoRA rank-r projections and their weight gradients (r = 16: QLoRA C5; lora.py:92-104) -------------
// Skinny shapes the 128x128 tile kernels waste 7/8 of a tile on: memory-bound reads of one [M][K] operand.
//   lora_proj:  Y[M][16] = alpha * sum_k X[m][k] W(j, k),  W = down [16][K] (w_kmajor) or up [K][16]
//   lora_wgrad: G (+)= alpha * sum_m X[m][n] S[m][j],       G [N][16] (up grad) or [16][N] (down grad)
// MFMA 16x16x32 bf16; W / S / X tiles transposed through padded LDS images; the wgrad reduction over the
// M tokens is split across workgroups into f32 slabs summed in a fixed order (deterministic).
namespace {
constexpr int LKC = 128;         // K chunk of W staged per step (lora_proj)
constexpr int LKP = LKC + 8;     // padded LDS row (bf16): conflict-free b128 row reads

// Four waves per 16 rows (LKS-wave workgroups, M/16 of them), each taking every LKS-th 128-k chunk with the
// activation fragments of its next LPD chunks in flight in registers (a 4-deep ring), so the memory latency
// is paid once, not per chunk; the LKS partial sums meet in LDS and wave 0 adds them in wave order
// (deterministic). (One wave per 16 rows left M = 4096 launches at one wave per CU: 12 us, latency-bound.)
// W = down [16][K]: B fragments straight from global memory (L2-resident, prefetched with the chunk);
// W = up [K][16]: each chunk transposed through the wave's LDS image.
constexpr int LPD = 4;
constexpr int LKS = 4;
#ifndef VPT_LP_COAL
#define VPT_LP_COAL 0  // A/B: activation rows loaded in 256-B segments, A fragments through LDS
#endif
// Grouped (blockIdx.y = group gy): X + gy * xgoff, W + gy * wgoff, output columns 16 gy .. 16 gy + 15 -- the
// q / k / v projections of one input (or of the three column blocks of one gradient) in one launch.
__global__ __launch_bounds__(64 * LKS) void lora_proj_kernel(const bf16_t* __restrict__ X, long ldx, long xgoff,
                                                             const bf16_t* __restrict__ W, int w_kmajor, long wgoff,
                                                             bf16_t* __restrict__ Y, long ldy, int M, int K, float alpha) {
  __shared__ __attribute__((aligned(16))) bf16_t wsa[LKS][16 * LKP];
  __shared__ __attribute__((aligned(16))) floatx4 red[LKS][64];
#if VPT_LP_COAL
  __shared__ __attribute__((aligned(16))) bf16_t xta[LKS][16 * LKP];  // the wave's 16 x 128 activation chunk
#endif
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, g = lane >> 4, j = lane & 15;
  X += blockIdx.y * xgoff;
  W += blockIdx.y * wgoff;
  Y += blockIdx.y * 16;
  bf16_t* ws = wsa[wid];
  const int row = blockIdx.x * 16 + j;
#if VPT_LP_COAL
  // rows in full 256-B segments (16 lanes per row, 4 rows per load), A fragments read back through LDS
  const bf16_t* xr = X + (long)min(blockIdx.x * 16 + g, M - 1) * ldx + (lane & 15) * 8;
  const long xq = 4 * ldx;  // next 4 rows
  const int lastq = (M - 1 - (int)blockIdx.x * 16 - g) / 4;  // loads past M re-read row M - 1
#else
  const bf16_t* xr = X + (long)min(row, M - 1) * ldx + 8 * g;
#endif
  const bf16_t* wr = W + (long)j * K + 8 * g;  // down: row j
  const int nch = K / LKC;
  const int ncw = (nch - wid + LKS - 1) / LKS;  // chunks wid, wid + LKS, ... of this wave
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  uint4 xb[LPD][LKC / 32], wb[LPD][LKC / 32];
#pragma unroll
  for (int u = 0; u < LPD; ++u)
    if (u < ncw) {
      const int c = wid + LKS * u;
#pragma unroll
      for (int s = 0; s < LKC / 32; ++s) {
#if VPT_LP_COAL
        xb[u][s] = *reinterpret_cast<const uint4*>(xr + (s <= lastq ? s : lastq) * xq + c * LKC);
#else
        xb[u][s] = *reinterpret_cast<const uint4*>(xr + c * LKC + 32 * s);
#endif
        if (w_kmajor) wb[u][s] = *reinterpret_cast<const uint4*>(wr + c * LKC + 32 * s);
      }
    }
  for (int t0 = 0; t0 < ncw; t0 += LPD) {
#pragma unroll
    for (int u = 0; u < LPD; ++u) {
      const int t = t0 + u;
      if (t < ncw) {
        const int c = wid + LKS * t;
        if (!w_kmajor) {  // up [K][16]: 128 rows of 32 B, two per lane, transposed into [16][k]
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int kr = lane + 64 * h;
            const uint4 a = *reinterpret_cast<const uint4*>(W + (long)(c * LKC + kr) * 16);
            const uint4 b = *reinterpret_cast<const uint4*>(W + (long)(c * LKC + kr) * 16 + 8);
            const uint32_t v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              ws[(2 * e) * LKP + kr] = (bf16_t)(v[e] & 0xffff);
              ws[(2 * e + 1) * LKP + kr] = (bf16_t)(v[e] >> 16);
            }
          }
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
          __builtin_amdgcn_wave_barrier();
        }
#if VPT_LP_COAL
        bf16_t* xt = xta[wid];
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int s = 0; s < LKC / 32; ++s) *reinterpret_cast<uint4*>(xt + (4 * s + g) * LKP + (lane & 15) * 8) = xb[u][s];
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes landed
        __builtin_amdgcn_wave_barrier();
#endif
#pragma unroll
        for (int s = 0; s < LKC / 32; ++s) {
          const bf16x8 bf = w_kmajor ? as_frag(wb[u][s])
                                     : as_frag(*reinterpret_cast<const uint4*>(&ws[j * LKP + 32 * s + 8 * g]));
#if VPT_LP_COAL
          const bf16x8 af = as_frag(*reinterpret_cast<const uint4*>(xt + j * LKP + 32 * s + 8 * g));
#else
          const bf16x8 af = as_frag(xb[u][s]);
#endif
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc, 0, 0, 0);
        }
        if (t + LPD < ncw) {
          const int cn = c + LKS * LPD;
#pragma unroll
          for (int s = 0; s < LKC / 32; ++s) {
#if VPT_LP_COAL
            xb[u][s] = *reinterpret_cast<const uint4*>(xr + (s <= lastq ? s : lastq) * xq + cn * LKC);
#else
            xb[u][s] = *reinterpret_cast<const uint4*>(xr + cn * LKC + 32 * s);
#endif
            if (w_kmajor) wb[u][s] = *reinterpret_cast<const uint4*>(wr + cn * LKC + 32 * s);
          }
        }
      }
    }
  }
  red[wid][lane] = acc;
  __syncthreads();
  if (wid != 0) return;
#pragma unroll
  for (int w = 1; w < LKS; ++w) acc += red[w][lane];
  // D[m][j]: lane holds rows 4g..4g+3 of the wave's 16, column j = lane & 15
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int m = blockIdx.x * 16 + 4 * g + r;
    if (m < M) Y[(long)m * ldy + j] = f2bf(acc[r] * alpha);
  }
}

constexpr int LMC = 128;  // m rows per wgrad stage (4 MFMA k-steps of 32 between two barriers)

// One wgrad job: G (+)= alpha * X[M][N]^T . S[M][16] (trans: G stored [16][N]); split over gridDim.y.
struct LoraWgradJob {
  const bf16_t* X; long ldx;
  const bf16_t* S; long lds;
  float* G;
  float* part;   // [splits][N][16]
  int N, trans, mchunk, splits;
};

// The MFMA operands run along m, the row index of both X and S: the tiles are staged row-major as loaded
// (one 16-B LDS store per chunk) and read back transposed by ds_read_b64_tr_b16 (lane i of a 16-lane group
// gets column i of 4 rows), 128 rows per stage with the next stage's loads in flight in registers.
constexpr int LXS = 72;  // X stage row stride (bf16): 64 columns + 16 B padding (spreads the tr reads' banks)
constexpr int LSS = 24;  // S stage row stride (bf16): 16 columns + 16 B
// Column block bx (64 columns) of split `split` of one job.
__device__ __forceinline__ void lora_wgrad_body(const LoraWgradJob& jb, int M, int bx, int split) {
  __shared__ __attribute__((aligned(16))) bf16_t xt[LMC * LXS];  // [m][n]
  __shared__ __attribute__((aligned(16))) bf16_t st[LMC * LSS];  // [m][j]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int n0 = bx * 64;
  const int mb = split * jb.mchunk, me = min(M, mb + jb.mchunk);
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  const int mr = tid >> 3, c = tid & 7;   // X: rows mr + 32u (u = 0..3), 16-B chunk c of the 64 columns
  const int sm = tid >> 1, hh = tid & 1;  // S: row sm, 16-B half hh of the 16 columns
  auto load = [&](int m0, uint4 (&xv)[4], uint4& sv) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = m0 + mr + 32 * u;
      xv[u] = m < me ? *reinterpret_cast<const uint4*>(jb.X + (long)m * jb.ldx + n0 + c * 8) : make_uint4(0, 0, 0, 0);
    }
    sv = m0 + sm < me ? *reinterpret_cast<const uint4*>(jb.S + (long)(m0 + sm) * jb.lds + hh * 8) : make_uint4(0, 0, 0, 0);
  };
  uint4 xv[4], sv;
  load(mb, xv, sv);
  for (int m0 = mb; m0 < me; m0 += LMC) {
#pragma unroll
    for (int u = 0; u < 4; ++u) *reinterpret_cast<uint4*>(&xt[(mr + 32 * u) * LXS + c * 8]) = xv[u];
    *reinterpret_cast<uint4*>(&st[sm * LSS + hh * 8]) = sv;
    if (m0 + LMC < me) load(m0 + LMC, xv, sv);  // next stage in flight during this one
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < LMC / 32; ++kk) {
      // A = X^T rows n = 16 wid + (lane & 15), k = m (8g .. 8g+7 of this 32); B = S, columns j = lane & 15
      const int r0 = 32 * kk + 8 * g + q;
      const uint2 a0 = lds_read_tr16((const VPT_LDS void*)(VPT_LDS char*)&xt[r0 * LXS + 16 * wid + 4 * p]);
      const uint2 a1 = lds_read_tr16((const VPT_LDS void*)(VPT_LDS char*)&xt[(r0 + 4) * LXS + 16 * wid + 4 * p]);
      const uint2 b0 = lds_read_tr16((const VPT_LDS void*)(VPT_LDS char*)&st[r0 * LSS + 4 * p]);
      const uint2 b1 = lds_read_tr16((const VPT_LDS void*)(VPT_LDS char*)&st[(r0 + 4) * LSS + 4 * p]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag2(a0, a1), as_frag2(b0, b1), acc, 0, 0, 0);
    }
    __syncthreads();
  }
  // D[n][j]: rows n = n0 + 16 wid + 4g + r, column j = lane & 15 -> part[split][n][j]
  float* pp = jb.part + ((long)split * jb.N + n0 + wid * 16 + 4 * g) * 16 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) pp[r * 16] = acc[r];
}

__global__ __launch_bounds__(256) void lora_wgrad_kernel(LoraWgradJob j0, LoraWgradJob j1, int M) {
  const LoraWgradJob jb = blockIdx.z ? j1 : j0;
  if ((int)blockIdx.x >= jb.N / 64 || (int)blockIdx.y >= jb.splits) return;
  lora_wgrad_body(jb, M, blockIdx.x, blockIdx.y);
}

// The slab launches of many jobs (several LoRA targets' up and down gradients, each with its own M) as one
// grid: job i owns the blocks [first[i], first[i + 1]), (N / 64) x splits of them, column block fastest.
constexpr int kLoraWgJobs = 24;
struct LoraWgBatch {
  LoraWgradJob j[kLoraWgJobs];
  int M[kLoraWgJobs];
  int first[kLoraWgJobs + 1];
  int njobs;
};
__global__ __launch_bounds__(256) void lora_wgrad_batch_kernel(LoraWgBatch b) {
  const int blk = blockIdx.x;
  int i = 0;
  while (i + 1 < b.njobs && blk >= b.first[i + 1]) ++i;  // wave-uniform scan over <= 24 entries
  const int local = blk - b.first[i], nbx = b.j[i].N / 64;
  lora_wgrad_body(b.j[i], b.M[i], local % nbx, local / nbx);
}

// G (+)= alpha * (sum of the split slabs in split order): deterministic; blockIdx.y selects the job.
__global__ void lora_wgrad_reduce_kernel(LoraWgradJob j0, LoraWgradJob j1, float alpha, int accumulate) {
  const LoraWgradJob jb = blockIdx.y ? j1 : j0;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // element (n, j) of [N][16]
  if (i >= jb.N * 16) return;
  float sum = 0.f;
  for (int z = 0; z < jb.splits; ++z) sum += jb.part[(long)z * jb.N * 16 + i];
  const int n = i >> 4, j = i & 15;
  float* d = jb.G + (jb.trans ? (long)j * jb.N + n : (long)i);
  *d = (accumulate ? *d : 0.f) + alpha * sum;
}
// Batched form of lora_wgrad_reduce_kernel: blockIdx.y selects one of up to kLoraRedJobs (part, G) jobs, so
// one launch finishes the adapter gradients of a whole transformer block (the per-target reduce launches
// cost more than their few MB of traffic).
constexpr int kLoraRedJobs = 32;
struct LoraRedBatch {
  const float* part[kLoraRedJobs];
  float* g[kLoraRedJobs];
  int n[kLoraRedJobs], splits[kLoraRedJobs], trans[kLoraRedJobs];
};
__global__ void lora_wgrad_reduce_batch_kernel(LoraRedBatch b, float alpha, int accumulate) {
  const int jb = blockIdx.y;
  const int N = b.n[jb], splits = b.splits[jb];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // element (n, j) of [N][16]
  if (i >= N * 16) return;
  const float* p = b.part[jb] + i;
  float sum = 0.f;
  for (int z = 0; z < splits; ++z) sum += p[(long)z * N * 16];  // split order: as lora_wgrad_reduce_kernel
  const int n = i >> 4, j = i & 15;
  float* d = b.g[jb] + (b.trans[jb] ? (long)j * N + n : (long)i);
  *d = (accumulate ? *d : 0.f) + alpha * sum;
}
}  // namespace

extern "C" int vpt_lora_proj(const void* X, long ldx, const void* W, int w_kmajor, void* Y, long ldy, int M, int K, int r,
                             float alpha, void* stream) {
  VPT_CHECK_ARG(X && W && Y, "vpt_lora_proj: null pointer");
  VPT_CHECK_ARG(r == 16, "vpt_lora_proj: rank 16 (the C5 configuration) only");
  VPT_CHECK_ARG(M > 0 && K > 0 && K % LKC == 0 && ldx % 8 == 0, "vpt_lora_proj: K % 128 == 0, 16-B leading dim");
  hipLaunchKernelGGL(lora_proj_kernel, dim3((M + 15) / 16), dim3(64 * LKS), 0, (hipStream_t)stream, (const bf16_t*)X, ldx,
                     0L, (const bf16_t*)W, w_kmajor, 0L, (bf16_t*)Y, ldy, M, K, alpha);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_lora_proj_grouped(const void* X, long ldx, long x_goff, const void* W, int w_kmajor, long w_goff,
                                     void* Y, long ldy, int M, int K, int r, int G, float alpha, void* stream) {
  VPT_CHECK_ARG(X && W && Y, "vpt_lora_proj_grouped: null pointer");
  VPT_CHECK_ARG(r == 16 && G >= 1 && G <= 64, "vpt_lora_proj_grouped: rank 16, 1..64 groups");
  VPT_CHECK_ARG(M > 0 && K > 0 && K % LKC == 0 && ldx % 8 == 0 && x_goff % 8 == 0 && w_goff % 8 == 0 && ldy >= 16 * G,
                "vpt_lora_proj_grouped: K % 128 == 0, 16-B leading dim / group offsets, ldy >= 16 G");
  hipLaunchKernelGGL(lora_proj_kernel, dim3((M + 15) / 16, G), dim3(64 * LKS), 0, (hipStream_t)stream,
                     (const bf16_t*)X, ldx, x_goff, (const bf16_t*)W, w_kmajor, w_goff, (bf16_t*)Y, ldy, M, K, alpha);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

// Rows per split slab at least: 2048 -- in the config-5 step the batched slab + reduce launches take 5.29 ms per
// step at 2048, 5.43 at 1024, 6.09 at 256 (rocprof, profiles/r03/r03zt, r03zu): fewer, longer slab blocks and
// fewer slabs to sum. A constant: the library holds no process-wide switches.
constexpr int kLoraWgradMinRows = 2048;

static int lora_wgrad_splits(int M, int N) {
  const int nb = N / 64;
  int splits = 1024 / (nb > 0 ? nb : 1);
  const int mr = kLoraWgradMinRows;
  const int maxs = (M + mr - 1) / mr;
  return splits < 1 ? 1 : (splits > maxs ? maxs : splits);
}

// f32 partial slabs [splits][N][16] of one wgrad.
extern "C" long vpt_lora_wgrad_workspace(int M, int N) { return (long)lora_wgrad_splits(M, N) * N * 16 * 4; }

static LoraWgradJob lora_job(const void* X, long ldx, const void* S, long lds_, float* G, int trans, int M, int N,
                             void* ws) {
  LoraWgradJob j;
  j.X = (const bf16_t*)X; j.ldx = ldx; j.S = (const bf16_t*)S; j.lds = lds_; j.G = G; j.part = (float*)ws;
  j.N = N; j.trans = trans;
  j.splits = lora_wgrad_splits(M, N);
  int mc = (M + j.splits - 1) / j.splits;
  j.mchunk = (mc + LMC - 1) / LMC * LMC;
  j.splits = (M + j.mchunk - 1) / j.mchunk;
  return j;
}

// Split-M slabs a wgrad of M rows and N columns writes (the `splits` of its vpt_lora_wgrad_reduce_batch job).
extern "C" int vpt_lora_wgrad_splits(int M, int N) {
  return M > 0 && N > 0 ? lora_job(nullptr, 0, nullptr, 0, nullptr, 0, M, N, nullptr).splits : 0;
}

// Both adapter gradients of one LoRA Linear in two launches (slabs, then the ordered sum):
//   G_up [N_out][16] (+)= alpha * dY[M][N_out]^T . dS[M][16]
//   G_down [16][N_in] (+)= alpha * X[M][N_in]^T . vS[M][16]     (ws_up / ws_down: lora_wgrad_workspace bytes)
static int lora_wgrad2_impl(const void* dY, long lddy, const void* dS, long ldds, float* g_up, int n_out,
                            const void* X, long ldx, const void* vS, long ldvs, float* g_down, int n_in, int M,
                            int accumulate, float alpha, void* ws_up, void* ws_down, bool deferred, void* stream) {
  VPT_CHECK_ARG(dY && dS && g_up && X && vS && g_down && ws_up && ws_down, "vpt_lora_wgrad2: null pointer");
  VPT_CHECK_ARG(M > 0 && n_out % 64 == 0 && n_in % 64 == 0 && lddy % 8 == 0 && ldx % 8 == 0 && ldds % 8 == 0 &&
                    ldvs % 8 == 0, "vpt_lora_wgrad2: widths % 64, 16-B leading dims");
  const LoraWgradJob j0 = lora_job(dY, lddy, dS, ldds, g_up, 0, M, n_out, ws_up);
  const LoraWgradJob j1 = lora_job(X, ldx, vS, ldvs, g_down, 1, M, n_in, ws_down);
  hipStream_t s = (hipStream_t)stream;
  const int gx = max(n_out, n_in) / 64, gy = max(j0.splits, j1.splits);
  hipLaunchKernelGGL(lora_wgrad_kernel, dim3(gx, gy, 2), dim3(256), 0, s, j0, j1, M);
  VPT_LAUNCH_CHECK();
  if (deferred) return VPT_OK;
  hipLaunchKernelGGL(lora_wgrad_reduce_kernel, dim3((max(n_out, n_in) * 16 + 255) / 256, 2), dim3(256), 0, s, j0, j1,
                     alpha, accumulate);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_lora_wgrad2(const void* dY, long lddy, const void* dS, long ldds, float* g_up, int n_out,
                               const void* X, long ldx, const void* vS, long ldvs, float* g_down, int n_in, int M,
                               int accumulate, float alpha, void* ws_up, void* ws_down, void* stream) {
  return lora_wgrad2_impl(dY, lddy, dS, ldds, g_up, n_out, X, ldx, vS, ldvs, g_down, n_in, M, accumulate, alpha, ws_up,
                          ws_down, false, stream);
}

extern "C" int vpt_lora_wgrad2_partial(const void* dY, long lddy, const void* dS, long ldds, int n_out, const void* X,
                                       long ldx, const void* vS, long ldvs, int n_in, int M, void* ws_up, void* ws_down,
                                       void* stream) {
  // g_up / g_down are only read by the reduce: any non-null placeholders pass the argument check
  float* const placeholder = reinterpret_cast<float*>(ws_up);
  return lora_wgrad2_impl(dY, lddy, dS, ldds, placeholder, n_out, X, ldx, vS, ldvs, placeholder, n_in, M, 1, 1.f, ws_up,
                          ws_down, true, stream);
}

extern "C" int vpt_lora_wgrad_partial_batch(const VptLoraWgradJob* jobs, int njobs, void* stream) {
  VPT_CHECK_ARG(jobs && njobs > 0 && njobs <= kLoraWgJobs, "vpt_lora_wgrad_partial_batch: 1..24 jobs");
  LoraWgBatch b = {};
  int total = 0;
  for (int i = 0; i < njobs; ++i) {
    const VptLoraWgradJob& q = jobs[i];
    VPT_CHECK_ARG(q.X && q.S && q.part && q.M > 0 && q.N > 0 && q.N % 64 == 0 && q.ldx % 8 == 0 && q.lds % 8 == 0,
                  "vpt_lora_wgrad_partial_batch: bad job (widths % 64, 16-B leading dims)");
    b.j[i] = lora_job(q.X, q.ldx, q.S, q.lds, nullptr, 0, q.M, q.N, q.part);
    b.M[i] = q.M;
    b.first[i] = total;
    total += (q.N / 64) * b.j[i].splits;
  }
  b.first[njobs] = total;
  b.njobs = njobs;
  hipLaunchKernelGGL(lora_wgrad_batch_kernel, dim3(total), dim3(256), 0, (hipStream_t)stream, b);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

extern "C" int vpt_lora_wgrad_reduce_batch(const VptLoraReduceJob* jobs, int njobs, float alpha, int accumulate,
                                           void* stream) {
  VPT_CHECK_ARG(jobs && njobs > 0 && njobs <= kLoraRedJobs, "vpt_lora_wgrad_reduce_batch: 1..32 jobs");
  LoraRedBatch b = {};
  int nmax = 0;
  for (int i = 0; i < njobs; ++i) {
    VPT_CHECK_ARG(jobs[i].part && jobs[i].g && jobs[i].n > 0 && jobs[i].splits > 0,
                  "vpt_lora_wgrad_reduce_batch: bad job");
    b.part[i] = jobs[i].part; b.g[i] = jobs[i].g;
    b.n[i] = jobs[i].n; b.splits[i] = jobs[i].splits; b.trans[i] = jobs[i].trans;
    nmax = max(nmax, jobs[i].n);
  }
  hipLaunchKernelGGL(lora_wgrad_reduce_batch_kernel, dim3((nmax * 16 + 255) / 256, njobs), dim3(256), 0,
                     (hipStream_t)stream, b, alpha, accumulate);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
