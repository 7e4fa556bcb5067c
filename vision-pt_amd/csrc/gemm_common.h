// Shared device code of the bf16 GEMM units (gemm.hip: the T128 kernel, the 256x256 ring and every C-ABI entry point;
// gemm_r2.hip: the 256x128 two-blocks-per-CU ring): kernel arguments, LDS image layouts, the LDS-DMA operand staging
// and the ring epilogues. Included by both translation units (named namespace vptg so that GemmArgs is one type).
#pragma once
#include "common.h"

namespace vptg {

constexpr int BK = 64;

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
  int splits;               // split-K slices (ring kernel work items = tiles * splits)
  float alpha;              // output scale applied to the accumulator before bias (LoRA alpha / rank)
  int ring_grid;            // persistent ring grid (0 = one block per CU)
  unsigned long long* dbg;  // stamp-diagnostic output (diagnostic build only)
  // fused SwiGLU (ring kernel only): sw = 1 forward (C = x12 [M][2F], C2 = h [M][F]; N = 2F, B = W1|W2),
  // sw = 2 backward of the W3 dgrad (C = dx12 [M][2F], aux = x12; N = F)
  int sw;
  bf16_t* C2; long ldc2;
  const bf16_t* aux; long ldaux;
  // row sums of A over this item's K slice (wgrad direction: the bias gradient sum_t dY[t][m]), f32 at
  // rsum[split * M + m]; ring kernel (RS instantiation) only
  float* rsum;
  // ring kernel: start delay (s_memrealtime ticks, 10 ns) of the blocks with bit 3 of blockIdx set, so
  // that half the CUs reach their (HBM-bound) epilogues while the other half run K loops (0 = off)
  int stagger;
  // K-extension (LoRA, vpt_gemm_bf16_lora): K2 more reduction elements from A2 (k-major [M][K2]) and B2 (the
  // layout of B: k-major [N][K2] or mn-major [K2][N]) after the K of A / B, in the same f32 accumulator.
  // K2 = 0: none. With K2 > 0: one split, K % 64 == 0.
  const bf16_t* A2; long lda2;
  const bf16_t* B2; long ldb2;
  int K2;
  // grouped K-extension (forward of several LoRA targets sharing one input, outputs side by side): output
  // columns [g * g_n, (g + 1) * g_n) take their extension from A2 columns [g * K2, (g + 1) * K2) and B2g[g]
  // ([g_n][K2], k-major), or with B2g[0] null from the stacked B2 rows [g * g_n, (g + 1) * g_n); g_n = 0:
  // ungrouped (B2). Tiles never straddle groups (g_n % tile width == 0).
  const bf16_t* B2g[4];
  int g_n;
  // alpha_cols > 0: alpha scales output columns [0, alpha_cols) only, the rest take 1 (the attention q block of a
  // fused q|k|v GEMM pre-scaled in its epilogue); a multiple of the ring tile width (256) or the T128 path is used
  int alpha_cols;
  // fused per-head QK-RMSNorm + RoPE forward (ring kernel, EPI_QKN; vpt_linear_qknorm_rope): qk_d > 0 marks output
  // columns [0, qk_d) as q and [qk_d, 2 qk_d) as k projections; each 64-column head of them is also normed (weights
  // qk_wq / qk_wk [64], eps qk_eps), roped (tables rcos / rsin [rps][32], position = row % rps), q times qk_scale,
  // and stored to C2 [M][ldc2] at the same column -- exactly qknorm_rope_fwd_kernel's arithmetic (csrc/norm.hip).
  int qk_d, rps;
  const bf16_t* qk_wq; const bf16_t* qk_wk;
  const float* rcos; const float* rsin;
  float qk_scale, qk_eps;
};

// ---- LDS images -----------------------------------------------------------------------------
__device__ __forceinline__ int kmaj_off(int row, int chunk) {  // [R][64] bf16, 128-B rows
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}
__device__ __forceinline__ int mnmaj_f(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }
template <int R>
__device__ __forceinline__ int mnmaj_off(int krow, int unit) {  // [64][R] bf16, 2R-byte rows
  return krow * (2 * R) + ((unit ^ (mnmaj_f(krow) << 2)) << 3);
}

// One 16-B-per-lane LDS-DMA (1 KB per wave) in inline asm, so that hipcc's waitcnt pass does not
// serialise it against the ds_reads of the other buffer (it cannot prove the two do not alias);
// completion is waited for explicitly with `s_waitcnt vmcnt(0)` before the K-step barrier.
// M0 holds the wave-uniform LDS destination and is restored (guide §5.7 LDS-DMA recipe).
// saddr form: wave-uniform 64-bit base in SGPRs + 32-bit per-lane byte offset in one VGPR. The base
// SGPRs come straight from v_readfirstlane: a VMEM read of a VALU-written SGPR needs wait states
// that hipcc does not insert inside asm, hence the opening `s_nop 4` (guide §5.7 item 2).
__device__ __forceinline__ void glds16(const void* sbase, uint32_t voff, uint32_t lds_addr) {
  unsigned keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_addr)
               : "memory");
}

// LDS-DMA of one full 64-deep operand tile of R rows (R*128 B = R/8 wave-instructions of 1 KB; each
// of the NW waves issues R/(8*NW)). The image is written lane-linearly, so the XOR swizzle is
// applied to each lane's GLOBAL source address (guide rule 21). Rows past the matrix edge are
// clamped to a valid row: they only feed output rows/cols that are never stored.
// `tile_base` is the wave-uniform address of element (row0, k0) [k-major] or (k0, row0) [mn-major].
template <bool KMAJ, int R, int NW>
__device__ __forceinline__ void glds_tile(char* lds, const bf16_t* tile_base, long ld, int row0, int nrows, int kvalid,
                                          int wid, int lane) {
  // pieces of 1 KB: contiguous per wave when they divide evenly, else strided (q = i * NW + wid, R = 160)
  constexpr bool EVEN = R % (8 * NW) == 0;
  constexpr int PER_WAVE = EVEN ? R / (8 * NW) : (R / 8 + NW - 1) / NW;
  const unsigned long long sb = (unsigned long long)tile_base;
  // readfirstlane returns int: go through `unsigned` so the low word is zero-extended (a sign-extended
  // low word with bit 31 set would OR 1s into the high word).
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)sb);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(sb >> 32));
  const bf16_t* sbase = (const bf16_t*)(((unsigned long long)hi << 32) | lo);
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int q = EVEN ? wid * PER_WAVE + i : i * NW + wid;
    if (!EVEN && q >= R / 8) break;  // wave-uniform
    uint32_t off;
    if (KMAJ) {
      const int row = q * 8 + (lane >> 3);
      int c = (lane & 7) ^ ((row >> 1) & 7);
      c = c * 8 < kvalid ? c : 0;  // k past the end: any valid chunk, zeroed in LDS afterwards
      int r = row0 + row < nrows ? row : nrows - 1 - row0;
      off = (uint32_t)(((long)r * ld + c * 8) * 2);
    } else {
      constexpr int CH = R / 8;  // 16-B chunks per k-row
      const int krow = q * (64 / CH) + lane / CH;
      const int c = (lane % CH) ^ (mnmaj_f(krow) << 1);
      const int m = row0 + c * 8 < nrows ? c * 8 : nrows - 8 - row0;  // >= 0 (nrows % 8 == 0)
      const int kr = krow < kvalid ? krow : kvalid - 1;               // zeroed in LDS afterwards
      off = (uint32_t)(((long)kr * ld + m) * 2);
    }
    const uint32_t dst = (uint32_t)(uintptr_t)(VPT_LDS char*)(lds + q * 1024);
    glds16((const void*)sbase, off, __builtin_amdgcn_readfirstlane(dst));
  }
}

template <bool KMAJ>
__device__ __forceinline__ const bf16_t* tile_ptr(const bf16_t* base, long ld, int row0, int k0) {
  return KMAJ ? base + (long)row0 * ld + k0 : base + (long)k0 * ld + row0;
}

// Zeroes the k >= kvalid part of a staged tile (k-major: chunks kc*8 >= kvalid of every row;
// mn-major: whole k-rows >= kvalid), so clamped DMA addresses never contribute to the product.
template <bool KMAJ, int R, int T>
__device__ __forceinline__ void zero_k_tail(char* lds, int kvalid, int tid) {
  if (KMAJ) {
    const int c0 = kvalid >> 3, nc = 8 - c0;
    for (int idx = tid; idx < R * nc; idx += T) {
      const int row = idx / nc, kc = c0 + idx % nc;
      *reinterpret_cast<uint4*>(lds + kmaj_off(row, kc)) = make_uint4(0, 0, 0, 0);
    }
  } else {
    constexpr int CH = R / 8;
    for (int idx = tid; idx < (BK - kvalid) * CH; idx += T) {
      const int krow = kvalid + idx / CH, ch = idx % CH;
      *reinterpret_cast<uint4*>(lds + krow * (2 * R) + ch * 16) = make_uint4(0, 0, 0, 0);
    }
  }
}

// Fragment for a 16(row) x 32(k) MFMA operand: lane holds row (lane&15), k = 8*(lane>>4)+0..7.
template <bool KMAJ, int R>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int row_base, int kk, int lane) {
  if (KMAJ) {
    const int row = row_base + (lane & 15);
    const int chunk = kk * 4 + (lane >> 4);
    return as_frag(*reinterpret_cast<const uint4*>(lds + kmaj_off(row, chunk)));
  } else {
    const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p = i16 & 3;
    const int unit = (row_base >> 2) + p;
    const int k0 = kk * 32 + 8 * g + q;
    uint2 lo = lds_read_tr16((const VPT_LDS void*)(lds + mnmaj_off<R>(k0, unit)));
    uint2 hi = lds_read_tr16((const VPT_LDS void*)(lds + mnmaj_off<R>(k0 + 4, unit)));
    return as_frag2(lo, hi);
  }
}

// ---- T256 ring kernel: 256x256 block tile, 8 waves (2x4) of 128x64, BK = 32 stages ------------
// A 4-deep LDS ring of 32-deep K tiles (32 KB each: A 256x32 + B 256x32) keeps up to three tiles of
// LDS-DMA in flight; waits are counted (`s_waitcnt vmcnt(8)`: the two younger tiles' 4 + 4 pieces
// per wave stay outstanding), never vmcnt(0) in the steady state (guide §5 "Pipelining across
// barriers", T3/T4). Each K step is two phases separated by raw s_barriers:
//   L_t: DMA tile t+3 into the stage of tile t-1; ds_read all A/B fragments of tile t into registers;
//        wait for this wave's pieces of tile t+1; barrier Y_t
//   C_t: 32 MFMAs from registers (s_setprio 1); barrier X_t+1
// PP (ping-pong): wave group 1 (waves 4-7, one per SIMD) executes one extra barrier up front and
// group 0 one at the end, so on every SIMD one wave is in C while the other is in L. The data wait for
// tile t+1 sits before Y_t (one phase earlier than an unstaggered loop needs), so that all 8 waves'
// pieces of a tile have landed before the earlier group's barrier that precedes its reads; a stage is
// re-filled in L_t only, after both groups' reads of it (L_t-1, each closed by lgkmcnt(0) + barrier).
// k-major stages are [row][32k] (64-B rows, chunk ^= 2*bit2(row): conflict-free for ds_read_b128's
// lane groups); mn-major stages are [32k][R] as in T128. A partial last K tile is DMA'd from clamped
// (finite, in-bounds) addresses and its k >= K lanes of the A fragments are zeroed in registers.
constexpr int RBK = 32;
constexpr int RSTAGES = 4;
// Default ring grid (GemmArgs::ring_grid = 0): one block per work item, the dispatcher placing each block wherever a CU
// is free. Against the persistent walk (256 blocks, one per CU, items at a stride of 256, the next item's first tiles
// DMA'd under the epilogue) it is level at N = 1 (r04za: +0.4 % over the 12 GEMMs of a block, -0.08 % per C3 step),
// +0.3 % per step with the optimizer on a side stream (r04zc), and it tolerates kernels beside it: with 8 CUs held for
// 150 us by another kernel, the persistent q|k|v forward took 204 us (its 8 displaced blocks started 150 us late)
// against 156 us (r04za) -- RCCL's all-reduce channels hold CUs that way during the N > 1 backward. ring_grid > 0
// keeps the persistent walk with that many blocks.
constexpr int kRingGrid = 256;  // the persistent walk: one block per CU (the 4-wave diagnostic ring's default)

__device__ __forceinline__ int kmaj32_off(int row, int chunk) {  // [R][32] bf16, 64-B rows
  return row * 64 + ((chunk ^ (((row >> 2) & 1) << 1)) << 4);
}

// One 32-deep operand tile of R rows = R*64 B = R/16 pieces of 1 KB; each of the 8 waves issues R/128
// = 2 (q = 2*wid + i). tile_voff gives lane's byte offset for piece i from the tile's (row0, k0)
// element: loop-invariant for full tiles, so it is computed once; only a partial last tile (kvalid <
// 32) recomputes it with k clamped. Rows past the matrix edge are clamped to a valid row.
template <bool KMAJ, int R, int NW = 8>  // NW waves share the tile's R / 16 pieces (the 256x128 ring: NW = 4)
__device__ __forceinline__ uint32_t tile_voff(long ld, int row0, int nrows, int kvalid, int wid, int lane, int i) {
  const int q = wid * (R / (16 * NW)) + i;
  if (KMAJ) {
    const int row = q * 16 + (lane >> 2);
    int c = (lane & 3) ^ (((row >> 2) & 1) << 1);
    c = c * 8 < kvalid ? c : 0;  // k past the end: any in-bounds chunk (masked in registers)
    const int r = row0 + row < nrows ? row : nrows - 1 - row0;
    return (uint32_t)(((long)r * ld + c * 8) * 2);
  } else {
    constexpr int CH = R / 8;  // 16-B chunks per k-row
    const int krow = q * (64 / CH) + lane / CH;
    const int c = (lane % CH) ^ (mnmaj_f(krow) << 1);
    const int m = row0 + c * 8 < nrows ? c * 8 : nrows - 8 - row0;
    const int kr = krow < kvalid ? krow : kvalid - 1;
    return (uint32_t)(((long)kr * ld + m) * 2);
  }
}

// The 4 pieces of one K tile (A: 2, B: 2) in one asm statement: one hazard pad for the SGPR operands
// (which may come from v_readfirstlane), M0 set per piece from precomputed SGPRs, restored at the end.
__device__ __forceinline__ void glds_step(const void* abase, const void* bbase, uint32_t va0, uint32_t va1,
                                          uint32_t vb0, uint32_t vb1, uint32_t la0, uint32_t la1, uint32_t lb0,
                                          uint32_t lb1) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %7\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %5\n\t"
      "s_mov_b32 m0, %8\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %5\n\t"
      "s_mov_b32 m0, %9\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %3, %6\n\t"
      "s_mov_b32 m0, %10\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %4, %6\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(va0), "v"(va1), "v"(vb0), "v"(vb1), "s"(abase), "s"(bbase), "s"(la0), "s"(la1), "s"(lb0), "s"(lb1)
      : "memory");
}

__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (const void*)(((unsigned long long)hi << 32) | lo);
}

template <bool KMAJ, int R>
__device__ __forceinline__ bf16x8 read_frag32(const char* lds, int row_base, int lane) {
  if (KMAJ) {
    const int row = row_base + (lane & 15);
    return as_frag(*reinterpret_cast<const uint4*>(lds + kmaj32_off(row, lane >> 4)));
  } else {
    return read_frag<false, R>(lds, row_base, 0, lane);
  }
}

// Zero the elements k = kbase + 0..7 of a fragment that lie at or past klast.
__device__ __forceinline__ unsigned keep2(int k, int klast) {
  return (k < klast ? 0x0000ffffu : 0u) | (k + 1 < klast ? 0xffff0000u : 0u);
}
__device__ __forceinline__ bf16x8 mask_k(bf16x8 f, int kbase, int klast) {
  uint4 v = __builtin_bit_cast(uint4, f);
  v.x &= keep2(kbase, klast);
  v.y &= keep2(kbase + 2, klast);
  v.z &= keep2(kbase + 4, klast);
  v.w &= keep2(kbase + 6, klast);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ void wait_younger(int younger) {  // 4 pieces per tile per wave
  if (younger >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}
__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
__device__ __forceinline__ void bare_barrier() {
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// ABL (timing-only ablations, wrong results): 1 = no LDS-DMA inside the loop, 2 = no vmcnt waits, 3 = no
// epilogue, 4 = epilogue stores dropped (zero-size buffer), 5 = no epilogue stores (plain bf16 output).
// DMAC: issue tile t+3's LDS-DMA at the start of the MFMA phase C_t instead of in L_t. It overwrites
// the stage of tile t-1, which every wave consumed by MFMAs before its previous barrier, so the
// barriers need no lgkmcnt(0) and L_t shrinks to the ds_reads; tile t+1 is then waited for with only
// tile t+2 younger (vmcnt(4)).
__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// Wait for a K tile with two younger tiles (8 pieces) and the previous item's S epilogue stores (issued
// after the tile) still allowed in flight: S = 16 (bf16 output) or 32 (f32).
__device__ __forceinline__ void wait_vm_pend(int S) {
  if (S == 16) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (S == 24) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
}

// One work item (tile, split-K slice) of the ring kernel.
struct RingItem {
  int m0, n0, split, kbeg, kend, nk, klast;
  uint32_t va0, va1, vb0, vb1;  // loop-invariant per-lane DMA piece offsets of full K tiles
};

// SW (fused SwiGLU forward): tile rows 0-127 of B are W1 rows c0.., rows 128-255 the matching W2 rows
// F + c0.. (F = N / 2, c0 = 128 * tile column), so each wave's fragments j = 0, 1 and 2, 3 hold x1 and x2
// of the same 32 output features; the staged output pairs them in the epilogue.
// (TN-wide tiles in general: rows [0, TN/2) W1, [TN/2, TN) W2; NW waves issue the TN / 16 pieces)
template <int TN = 256, int NW = 8>
__device__ __forceinline__ uint32_t tile_voff_sw(long ld, int c0, int F, int kvalid, int wid, int lane, int i) {
  const int q = wid * (TN / (16 * NW)) + i;
  const int row = q * 16 + (lane >> 2);
  int c = (lane & 3) ^ (((row >> 2) & 1) << 1);
  c = c * 8 < kvalid ? c : 0;
  const int srow = row < TN / 2 ? c0 + row : F + c0 + row - TN / 2;
  return (uint32_t)(((long)srow * ld + c * 8) * 2);
}

template <bool AK, bool BK_, int SW = 0>
__device__ __forceinline__ RingItem ring_item(const GemmArgs& g, int item, int items, int tiles, int tiles_n, int wid,
                                              int lane) {
  const int q8 = items >> 3, r8 = items & 7, xcd = item & 7;
  const int wgid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (item >> 3);
  RingItem it;
  it.split = wgid / tiles;
  const int tile = wgid - it.split * tiles;
  it.m0 = tile / tiles_n * 256;
  it.n0 = tile % tiles_n * (SW ? 128 : 256);  // SW: first output feature of the tile
  it.kbeg = it.split * g.k_split;
  it.kend = min(g.K, it.kbeg + g.k_split);
  it.nk = (it.kend - it.kbeg + RBK - 1) / RBK;
  it.klast = it.kend - it.kbeg - (it.nk - 1) * RBK;  // valid k of the last tile (1..32)
  if (g.K2 > 0 && it.split == g.splits - 1) {  // K-extension tiles after the main K (K % 64 == 0), last split
    const int ne = (g.K2 + RBK - 1) / RBK;
    it.nk += ne;
    it.klast = g.K2 - (ne - 1) * RBK;
  }
  it.va0 = tile_voff<AK, 256>(g.lda, it.m0, g.M, RBK, wid, lane, 0);
  it.va1 = tile_voff<AK, 256>(g.lda, it.m0, g.M, RBK, wid, lane, 1);
  if (SW) {
    it.vb0 = tile_voff_sw(g.ldb, it.n0, g.N / 2, RBK, wid, lane, 0);
    it.vb1 = tile_voff_sw(g.ldb, it.n0, g.N / 2, RBK, wid, lane, 1);
  } else {
    it.vb0 = tile_voff<BK_, 256>(g.ldb, it.n0, g.N, RBK, wid, lane, 0);
    it.vb1 = tile_voff<BK_, 256>(g.ldb, it.n0, g.N, RBK, wid, lane, 1);
  }
  return it;
}

// K tile t of item `it` by LDS-DMA into ring stage t % 4: 4 pieces per wave (A: 2, B: 2).
template <bool AK, bool BK_, int SW = 0>
__device__ __forceinline__ void ring_issue(const GemmArgs& g, const RingItem& it, int t, uint32_t lds0, int wid,
                                           int lane) {
  constexpr int A32 = 256 * RBK * 2, STAGE32 = 2 * A32;
  const uint32_t la = __builtin_amdgcn_readfirstlane(lds0 + (t & (RSTAGES - 1)) * STAGE32);
  const int k0 = it.kbeg + t * RBK;
  if (k0 >= it.kend) {  // K-extension tile (A2 / B2); its k >= K2 lanes are masked like a partial last tile
    const int e0 = k0 - it.kend, kv = min(RBK, g.K2 - e0);
    const int grp = g.g_n > 0 ? it.n0 / g.g_n : 0;  // grouped extension: this tile's target
    const bf16_t* b2 = g.g_n > 0 ? (g.B2g[0] ? g.B2g[grp] : g.B2 + (long)grp * g.g_n * g.ldb2) : g.B2;
    const int nb0 = it.n0 - grp * g.g_n, nrows = g.g_n > 0 ? g.g_n : g.N;
    const void* ab = uniform_ptr(tile_ptr<AK>(g.A2 + grp * g.K2, g.lda2, it.m0, e0));
    const void* bb = uniform_ptr(tile_ptr<BK_>(b2, g.ldb2, nb0, e0));
    glds_step(ab, bb, tile_voff<AK, 256>(g.lda2, it.m0, g.M, kv, wid, lane, 0),
              tile_voff<AK, 256>(g.lda2, it.m0, g.M, kv, wid, lane, 1),
              tile_voff<BK_, 256>(g.ldb2, nb0, nrows, kv, wid, lane, 0),
              tile_voff<BK_, 256>(g.ldb2, nb0, nrows, kv, wid, lane, 1), la, la + 1024, la + A32, la + A32 + 1024);
    return;
  }
  const int kv = min(RBK, it.kend - k0);
  const void* ab = uniform_ptr(tile_ptr<AK>(g.A, g.lda, it.m0, k0));
  const void* bb = uniform_ptr(tile_ptr<BK_>(g.B, g.ldb, SW ? 0 : it.n0, k0));
  if (kv == RBK) {
    glds_step(ab, bb, it.va0, it.va1, it.vb0, it.vb1, la, la + 1024, la + A32, la + A32 + 1024);
  } else if (SW) {
    glds_step(ab, bb, tile_voff<AK, 256>(g.lda, it.m0, g.M, kv, wid, lane, 0),
              tile_voff<AK, 256>(g.lda, it.m0, g.M, kv, wid, lane, 1), tile_voff_sw(g.ldb, it.n0, g.N / 2, kv, wid, lane, 0),
              tile_voff_sw(g.ldb, it.n0, g.N / 2, kv, wid, lane, 1), la, la + 1024, la + A32, la + A32 + 1024);
  } else {
    glds_step(ab, bb, tile_voff<AK, 256>(g.lda, it.m0, g.M, kv, wid, lane, 0),
              tile_voff<AK, 256>(g.lda, it.m0, g.M, kv, wid, lane, 1),
              tile_voff<BK_, 256>(g.ldb, it.n0, g.N, kv, wid, lane, 0),
              tile_voff<BK_, 256>(g.ldb, it.n0, g.N, kv, wid, lane, 1), la, la + 1024, la + A32, la + A32 + 1024);
  }
}

// Buffer descriptors and per-lane offsets of one item's epilogue (output, residual, SwiGLU x12).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
struct EpiAddr {
  __amdgpu_buffer_rsrc_t rs, rr, ra;
  uint32_t voff, rvoff, avoff;
  int rstride, rrstride, rastride;
  bool col_ok;
  float alpha;  // the output scale of this tile (GemmArgs::alpha / alpha_cols)
};

__device__ __forceinline__ EpiAddr epi_addr(const GemmArgs& g, const RingItem& it, int wm, int wn, int lane,
                                             int wr = 128) {  // wr: rows of a wave tile (the 128x128 R2 tiles: 64)
  EpiAddr e;
  const int es = g.out_mode == OUT_BF16 ? 2 : 4;
  const int rows_here = min(256, g.M - it.m0);
  char* cbase = (char*)g.C + ((long)it.split * g.split_stride + (long)it.m0 * g.ldc + it.n0) * es;
  e.rs = __builtin_amdgcn_make_buffer_rsrc(cbase, (short)0, rows_here * (int)g.ldc * es, 0x00020000);
  const int tcol = wn * 64 + (lane & 7) * 8;  // column within the tile
  e.col_ok = it.n0 + tcol < g.N;
  e.alpha = g.alpha_cols > 0 && it.n0 >= g.alpha_cols ? 1.f : g.alpha;
  const int lrow = wm * wr + (lane >> 3);  // tile row of (fragment 0, p = 0)
  // lane part of the store offset; fragment i / half p add the wave-uniform soffset (i*16 + p*8) rows
  e.voff = e.col_ok ? (uint32_t)((lrow * (int)g.ldc + tcol) * es) : 0x80000000u;
  e.rstride = (int)g.ldc * es;  // bytes per row
  // residual rows of this tile (bf16, leading dim ldr), addressed like C
  const bf16_t* rbase = g.resid ? g.resid + (long)it.m0 * g.ldr + it.n0 : g.resid;
  e.rr = __builtin_amdgcn_make_buffer_rsrc((void*)rbase, (short)0, g.resid ? rows_here * (int)g.ldr * 2 : 0, 0x00020000);
  e.rrstride = (int)g.ldr * 2;
  e.rvoff = e.col_ok ? (uint32_t)((lrow * (int)g.ldr + tcol) * 2) : 0x80000000u;
  // fused SwiGLU backward: x12 rows of this tile (bf16, leading dim ldaux)
  const bf16_t* abase = g.aux ? g.aux + (long)it.m0 * g.ldaux + it.n0 : g.aux;
  e.ra = __builtin_amdgcn_make_buffer_rsrc((void*)abase, (short)0, g.aux ? rows_here * (int)g.ldaux * 2 : 0, 0x00020000);
  e.rastride = (int)g.ldaux * 2;
  e.avoff = e.col_ok ? (uint32_t)((lrow * (int)g.ldaux + tcol) * 2) : 0x80000000u;
  return e;
}

// Epilogue operands read from memory (residual, SwiGLU-backward x12, f32 accumulate target) arrive in
// groups of 8 loads (32 VGPRs), waited for once per group. Issued per fragment inside the epilogue, each
// load's compiler-placed wait was a vmcnt(0) (16 serial HBM round trips per item) and, being younger than
// the prefetched tiles, drained them. The first group is loaded BEFORE the next item's LDS-DMA; a later
// group is loaded right after the previous group's stores (its wait then also covers the DMAs, by then
// long in flight). Residual: 2 loads per fragment, groups of 4 fragments; x12 / accumulate: 4 loads per
// fragment, groups of 2. Slot of fragment il (in its group), half p, part e: resid 2il + p, else 4il + 2p + e.
// Epilogue modes (a template parameter of the ring kernel, so that each mode gets its own register
// allocation): 0 = no loads (bf16 / f32 out, bias, SiLU), 1 = residual, 2 = fused SwiGLU backward (x12),
// 3 = f32 accumulate into C.
// EPI_SWB1: the SwiGLU-backward epilogue with its x12 operands loaded one group at a time (the form before the
// one-group-ahead preload; diagnostic build only, A/B)
enum { EPI_PLAIN = 0, EPI_RESID = 1, EPI_SWB = 2, EPI_ACC = 3, EPI_QKN = 4, EPI_SWB1 = 5 };
// Cache policy (buffer instruction aux bits) of the SwiGLU-backward epilogue's x12 loads and dx12 stores: both streams
// are touched once (270 MB each at C3), while the GEMM's B operand (W3, 3 MB) is re-read by every row tile of an XCD.
// nt (2) on the x12 loads, sc1 (16: the line leaves the XCD's L2) on the dx12 stores. In-process A/B at the C3 shape
// (tools/lib_ab.py swb, r06b; L2 / MALL flushed between launches, bitwise equal): 218.4 us default policy, 196.0 nt
// loads, 216.4 sc1 stores, 194.0 both. Compile-time knobs for such A/B builds.
#ifndef VPT_SWB_LD_AUX
#define VPT_SWB_LD_AUX 2
#endif
#ifndef VPT_SWB_ST_AUX
#define VPT_SWB_ST_AUX 16
#endif
// The same knobs for the residual epilogue's loads, the SwiGLU forward's x12 / h stores and the plain bf16 stores
// (A/B builds; default policy unless measured otherwise)
#ifndef VPT_RESID_LD_AUX
#define VPT_RESID_LD_AUX 0
#endif
#ifndef VPT_SWF_ST_AUX
#define VPT_SWF_ST_AUX 0
#endif
#ifndef VPT_EPI_ST_AUX
#define VPT_EPI_ST_AUX 0
#endif
__host__ __device__ constexpr bool epi_swb(int e) { return e == EPI_SWB || e == EPI_SWB1; }
__host__ __device__ constexpr int epi_frags(int epi) {  // fragments per preload group (0: no loads)
  return epi == EPI_RESID ? 4 : (epi_swb(epi) || epi == EPI_ACC) ? 2 : 0;
}
__host__ __device__ inline int epi_mode(const GemmArgs& g) {
  return g.sw == 2 ? EPI_SWB : g.out_mode == OUT_F32_ACC ? EPI_ACC : g.resid ? EPI_RESID : g.qk_d > 0 ? EPI_QKN : EPI_PLAIN;
}
struct EpiPre {
  u32x4 v[8];
};
template <int EPI, int I0>
__device__ __forceinline__ void epi_preload(const GemmArgs& g, const EpiAddr& e, EpiPre& pre) {
  if (epi_swb(EPI)) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int so = ((I0 + i) * 16 + p * 8) * e.rastride;
        pre.v[4 * i + 2 * p] = __builtin_amdgcn_raw_buffer_load_b128(e.ra, (int)e.avoff, so, VPT_SWB_LD_AUX);
        pre.v[4 * i + 2 * p + 1] = __builtin_amdgcn_raw_buffer_load_b128(
            e.ra, (int)(e.col_ok ? e.avoff + g.N * 2 : e.avoff), so, VPT_SWB_LD_AUX);
      }
  } else if (EPI == EPI_ACC) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int so = ((I0 + i) * 16 + p * 8) * e.rstride;
        pre.v[4 * i + 2 * p] = __builtin_amdgcn_raw_buffer_load_b128(e.rs, (int)e.voff, so, 0);
        pre.v[4 * i + 2 * p + 1] = __builtin_amdgcn_raw_buffer_load_b128(e.rs, (int)e.voff, so + 16, 0);
      }
  } else if (EPI == EPI_RESID) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int p = 0; p < 2; ++p)
        pre.v[2 * i + p] =
            __builtin_amdgcn_raw_buffer_load_b128(e.rr, (int)e.rvoff, ((I0 + i) * 16 + p * 8) * e.rrstride,
                                                  VPT_RESID_LD_AUX);
  }
}

// Ring epilogue over fragments [i0, i1). Per 16-row fragment of the wave's 128x64 sub-tile: stage the
// f32 accumulators in the wave's 4 KB slice of ring stage 3 (16 rows x 64 floats, 16-B slot ^= row & 1:
// conflict-free b128 reads, 2-way b32 writes), read back 2 rows x 8 consecutive columns per lane, apply
// alpha / bias / SiLU / residual / accumulate (operands from `pre`, group of i0), and store with buffer
// stores. Rows past M fall outside the buffer's num_records and columns past N carry an offset past it,
// so the hardware drops them without a branch: every wave issues exactly ring_stores(out_mode) store
// instructions, which the next item's counted vmcnt waits rely on (stores are younger than that item's
// first three K tiles).
__device__ __forceinline__ int ring_stores(const GemmArgs& g) {
  if (g.sw == 1) return 24;  // x1, x2, h per lane and fragment
  if (g.sw == 2) return 32;  // dx1, dx2 per lane, fragment and half
  return g.out_mode == OUT_BF16 ? 16 : 32;
}
__device__ __forceinline__ int stg_off(int row, int col) {
  return row * 256 + (((col >> 2) ^ (row & 1)) << 4) + ((col & 3) << 2);
}

// A 16-B buffer store whose data registers the next instruction may not overwrite: the store reads them
// after issue, and hipcc (ROCm 7.2, gfx950) emitted the SwiGLU-backward epilogue's first store followed
// directly by a VALU write of its data registers, with no wait state -- the stored dwords came out corrupted.
// The scheduling barrier pins the pad right behind the store (tools/isa_store_hazard.py checks the .s).
template <int AUX = 0>
__device__ __forceinline__ void store_b128_padded(u32x4 v, __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, voff, soff, AUX);
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1");
  __builtin_amdgcn_sched_barrier(0);
}

template <int EPI, int I0, int I1, bool NOST = false>
__device__ __forceinline__ void epilogue_ring(const GemmArgs& g, const floatx4 (&acc)[8][4], char* stg, int lane,
                                              const EpiAddr& e, const float (&bias8)[8], const EpiPre& pre) {
  const int cw = lane & 7;
#pragma unroll
  for (int i = I0; i < I1; ++i) {
    const int il = i - I0;  // fragment within the preload group
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float*>(stg + stg_off((lane >> 4) * 4 + r, j * 16 + (lane & 15))) = acc[i][j][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes retired
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int lr = p * 8 + (lane >> 3);
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, cw * 8));
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, cw * 8 + 4));
      float o[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = o[q] * e.alpha + bias8[q];
      if (g.act == ACT_SILU) {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = o[q] / (1.f + __expf(-o[q]));
      }
      const int soff = (i * 16 + p * 8) * e.rstride;
      if (epi_swb(EPI)) {
        // fused SwiGLU backward (the reference's SwiGLU autograd, denoiser.py:480-506, as swiglu_bwd_kernel):
        // o = dh; x1, x2 from x12; dx1 -> column c, dx2 -> column F + c of dx12 (F = N)
        const u32x4 a4 = pre.v[4 * il + 2 * p], b4 = pre.v[4 * il + 2 * p + 1];
        float a[8], b[8], d1[8], d2[8];
        unpack8(make_uint4(a4[0], a4[1], a4[2], a4[3]), a);
        unpack8(make_uint4(b4[0], b4[1], b4[2], b4[3]), b);
#pragma unroll
        for (int q = 0; q < 8; ++q) swiglu_bwd1(bf2f(f2bf(o[q])), a[q], b[q], d1[q], d2[q]);  // dh: a bf16 tensor
        const uint4 w1 = pack8(d1), w2 = pack8(d2);
        store_b128_padded<VPT_SWB_ST_AUX>(u32x4{w1.x, w1.y, w1.z, w1.w}, e.rs, (int)e.voff, soff);
        store_b128_padded<VPT_SWB_ST_AUX>(u32x4{w2.x, w2.y, w2.z, w2.w}, e.rs,
                                          (int)(e.col_ok ? e.voff + g.N * 2 : e.voff), soff);
      } else if (g.out_mode == OUT_BF16) {
        if (EPI == EPI_RESID) {
          // reference semantics: residual + bf16(linear output), rounded again to bf16. Out-of-range rows /
          // columns read 0 (their stores are dropped).
          const u32x4 r4 = pre.v[2 * il + p];
          float rv[8];
          unpack8(make_uint4(r4[0], r4[1], r4[2], r4[3]), rv);
#pragma unroll
          for (int q = 0; q < 8; ++q) o[q] = bf2f(f2bf(o[q])) + rv[q];
        }
        const uint4 w = pack8(o);
        if (NOST) asm volatile("" :: "v"(w.x), "v"(w.y), "v"(w.z), "v"(w.w));  // timing ablation: no store
        else store_b128_padded<VPT_EPI_ST_AUX>(u32x4{w.x, w.y, w.z, w.w}, e.rs, (int)e.voff, soff);
      } else {
        if (EPI == EPI_ACC) {
          const u32x4 a0 = pre.v[4 * il + 2 * p], a1 = pre.v[4 * il + 2 * p + 1];
#pragma unroll
          for (int q = 0; q < 4; ++q) { o[q] += __uint_as_float(a0[q]); o[4 + q] += __uint_as_float(a1[q]); }
        }
        store_b128_padded(
            u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3])}, e.rs,
            (int)e.voff, soff);
        store_b128_padded(
            u32x4{__float_as_uint(o[4]), __float_as_uint(o[5]), __float_as_uint(o[6]), __float_as_uint(o[7])}, e.rs,
            (int)e.voff, soff + 16);
      }
    }
  }
}

// Fused QK-RMSNorm + RoPE forward epilogue (EPI_QKN, bf16 output, no residual): as epilogue_ring's bf16 path, plus,
// for a wave whose 64-column slice is a q or k head, the head's rope(rms(x) w) (q: times qk_scale) of the bf16-rounded
// output row to C2. A lane holds 8 consecutive columns of one row and the row's 64 columns sit in the 8 lanes
// lane >> 3 == row: the sum of squares is 8 in-lane adds and xor-shuffles 1, 2, 4, the RoPE pairs are in-lane -- the
// operation order of qknorm_rope_fwd_kernel, so qk is bitwise what that kernel computes from the stored qkv. The RoPE
// table rows (L2-resident) are loaded one fragment ahead; this epilogue runs BEFORE the next item's tiles are DMA'd
// (its loads are waited for by the compiler, and vmcnt retires in order), so the item seam waits count no stores.
__device__ __forceinline__ void epilogue_ring_qkn(const GemmArgs& g, const floatx4 (&acc)[8][4], char* stg, int lane,
                                                  const EpiAddr& e, const float (&bias8)[8], const RingItem& it, int wm,
                                                  int wn) {
  const int cw = lane & 7;
  const int hcol = it.n0 + wn * 64;                    // first column of this wave's head slice
  const bool isq = hcol < g.qk_d, isk = !isq && hcol < 2 * g.qk_d;
  const bool qk = isq || isk;                          // wave-uniform
  const int rows_here = min(256, g.M - it.m0);
  const __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(
      (char*)g.C2 + ((long)it.m0 * g.ldc2 + (qk ? hcol : 0)) * 2, (short)0, rows_here * (int)g.ldc2 * 2, 0x00020000);
  const int lrow = wm * 128 + (lane >> 3);
  const uint32_t voff2 = (uint32_t)((lrow * (int)g.ldc2 + cw * 8) * 2);
  const int rstride2 = (int)g.ldc2 * 2;
  float wf[8];
  {
    uint4 wr = make_uint4(0, 0, 0, 0);
    if (qk) wr = *reinterpret_cast<const uint4*>((isq ? g.qk_wq : g.qk_wk) + cw * 8);
    unpack8(wr, wf);
  }
  const float osc = isq ? g.qk_scale : 1.f;
  // RoPE table pieces (4 cos + 4 sin of the lane's column pairs) of fragment i, halves p = 0, 1
  auto table = [&](int i, floatx4 (&c)[2], floatx4 (&sn)[2]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const long pos = (long)(it.m0 + lrow + i * 16 + p * 8) % g.rps;
      c[p] = *reinterpret_cast<const floatx4*>(g.rcos + pos * 32 + cw * 4);
      sn[p] = *reinterpret_cast<const floatx4*>(g.rsin + pos * 32 + cw * 4);
    }
  };
  floatx4 cc[2], sc[2];
  if (qk) table(0, cc, sc);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    floatx4 cn[2], sn[2];
    if (qk && i < 7) table(i + 1, cn, sn);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float*>(stg + stg_off((lane >> 4) * 4 + r, j * 16 + (lane & 15))) = acc[i][j][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes retired
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int lr = p * 8 + (lane >> 3);
      const floatx4 x0 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, cw * 8));
      const floatx4 x1 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, cw * 8 + 4));
      float o[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = bf2f(f2bf(o[q] * e.alpha + bias8[q]));  // the stored bf16 qkv values
      const int soff = (i * 16 + p * 8) * e.rstride;
      const uint4 w = pack8(o);
      store_b128_padded(u32x4{w.x, w.y, w.z, w.w}, e.rs, (int)e.voff, soff);
      if (qk) {
        float ss = qkn_sumsq8(o);
        ss += __shfl_xor(ss, 1, 64);
        ss += __shfl_xor(ss, 2, 64);
        ss += __shfl_xor(ss, 4, 64);
        const float rr = qkn_rstd(ss, g.qk_eps);
        const float c4[4] = {cc[p][0], cc[p][1], cc[p][2], cc[p][3]};
        const float s4[4] = {sc[p][0], sc[p][1], sc[p][2], sc[p][3]};
        float y[8];
        qkn_rope8(o, rr, wf, c4, s4, osc, y);
        const uint4 w2 = pack8(y);
        store_b128_padded(u32x4{w2.x, w2.y, w2.z, w2.w}, r2, (int)voff2, (i * 16 + p * 8) * rstride2);
      }
    }
    if (i < 7) {
#pragma unroll
      for (int p = 0; p < 2; ++p) { cc[p] = cn[p]; sc[p] = sn[p]; }
    }
  }
}

// Fused SwiGLU forward epilogue (SW): per 16-row fragment, stage as epilogue_ring (staged columns 0-31 =
// x1, 32-63 = x2 of the same 32 features), then each lane takes one row and 8 features: x1, x2 = bf16(acc
// + bias) stored to x12 (columns c and F + c) and h = bf16(bf16(silu(x1)) * x2) to C2 (column c) -- the
// reference's SwiGLU (denoiser.py:480-506) with the same roundings as swiglu_fwd_kernel. 24 stores per wave.
__device__ __forceinline__ void epilogue_ring_swf(const GemmArgs& g, const floatx4 (&acc)[8][4], char* stg, int lane,
                                                  const RingItem& it, int wm, int wn, const float (&b1)[8],
                                                  const float (&b2)[8]) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const int F = g.N / 2;
  const int rows_here = min(256, g.M - it.m0);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (char*)g.C + (long)it.m0 * g.ldc * 2, (short)0, rows_here * (int)g.ldc * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rh = __builtin_amdgcn_make_buffer_rsrc(
      (char*)g.C2 + (long)it.m0 * g.ldc2 * 2, (short)0, rows_here * (int)g.ldc2 * 2, 0x00020000);
  const int q = lane & 3, lr = lane >> 2;     // 8-feature chunk, fragment row
  const int col = it.n0 + wn * 32 + q * 8;     // first output feature of the lane
  const int lrow = wm * 128 + lr;
  const uint32_t vx = (uint32_t)((lrow * (int)g.ldc + col) * 2);
  const uint32_t vh = (uint32_t)((lrow * (int)g.ldc2 + col) * 2);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        *reinterpret_cast<float*>(stg + stg_off((lane >> 4) * 4 + r, j * 16 + (lane & 15))) = acc[i][j][r];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own-wave LDS writes retired
    __builtin_amdgcn_wave_barrier();
    const floatx4 a0 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, q * 8));
    const floatx4 a1 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, q * 8 + 4));
    const floatx4 c0 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, 32 + q * 8));
    const floatx4 c1 = *reinterpret_cast<const floatx4*>(stg + stg_off(lr, 32 + q * 8 + 4));
    float x1[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    float x2[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
    float hv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x1[e] = bf2f(f2bf(x1[e] * g.alpha + b1[e]));
      x2[e] = bf2f(f2bf(x2[e] * g.alpha + b2[e]));
      hv[e] = swiglu_fwd1(x1[e], x2[e]);
    }
    const int soff = i * 16 * (int)g.ldc * 2, soffh = i * 16 * (int)g.ldc2 * 2;
    const uint4 w1 = pack8(x1), w2 = pack8(x2), wh = pack8(hv);
    store_b128_padded<VPT_SWF_ST_AUX>(u32x4{w1.x, w1.y, w1.z, w1.w}, rs, (int)vx, soff);
    store_b128_padded<VPT_SWF_ST_AUX>(u32x4{w2.x, w2.y, w2.z, w2.w}, rs, (int)(vx + F * 2), soff);
    store_b128_padded<VPT_SWF_ST_AUX>(u32x4{wh.x, wh.y, wh.z, wh.w}, rh, (int)vh, soffh);
  }
}

}  // namespace vptg
