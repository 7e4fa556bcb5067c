// Flash attention (head_dim 64, bf16 in, f32 softmax) with a key-padding bias, for gfx950.
//
// Replaces src/modules/attention.py:98-129 (`scaled_dot_product_attention`, eager SDPA with a
// [B,H,N,N] bool mask built at src/models/jit/denoiser.py:375-381). Instead of materialising the
// expanded mask, keys carry an additive bias row (0 / -inf) per batch: keys < n_dense are always
// valid (patch / image-size / time tokens), keys in [n_dense, n) read `kbias[b][key]`, keys >= n
// are -inf. Softmax scale is 1/sqrt(64) (reference default scale=None). Queries (n rows) and keys
// (nk rows) may differ: SDXL cross-attention (src/models/sdxl/denoiser.py:101-171) attends image
// tokens to the text context.
//
// All products use v_mfma_f32_32x32x16_bf16 with the reduction axis chosen so that every
// accumulator is directly the next product's operand (guide §3 "accumulator tile as operand"):
//   forward : S^T = K.Q^T (query on the lane -> softmax is lane-local), O^T += V^T.P^T
//   dK/dV   : S = Q.K^T, dP = dO.V^T (key on the lane), dV^T += dO^T.P, dK^T += Q^T.dS
//   dQ      : S^T = K.Q^T, dP^T = V.dO^T, dQ^T += K^T.dS^T
// Row tiles [64][64] bf16 live in LDS with one XOR swizzle (sigma) that is conflict-free for both
// ds_read_b128 row reads and ds_read_b64_tr_b16 transposed reads.
//
// VALU diet (the softmax, not the MFMA, bounds head_dim 64): the caller passes the query pre-scaled by
// c = scale*log2(e) (vpt_qknorm_rope_fwd's q_scale), so every S product is in log2 units; the row
// constants (-m in the forward, -LSE and -delta in the backward, stored negated) are the MFMA chains'
// initial accumulators. Per score that leaves exp2 (+ row-sum add / max) in the forward and exp2 + one
// multiply in the backward.
#include "common.h"

namespace {

struct Tensor4 {       // element strides: batch, head, row; the 64 head dims are contiguous
  const bf16_t* p; long sb, sh, sr;
};
struct OTensor4 {
  bf16_t* p; long sb, sh, sr;
};

struct AttnArgs {
  Tensor4 q, k, v, dO;
  OTensor4 o, dq, dk, dv;
  float* lse; const float* delta_in; float* delta_out; long l_sb, l_sh;  // [B][H][*] f32
  const float* kbias; long kb_sb;                                         // [B][*] f32
  int n, nk, n_dense;  // query rows, key rows (cross-attention: nk != n), always-valid keys
  float scale, scale_log2;
  float tau;  // forward lazy-rescale threshold
  int kb0;    // start of the key-bias LDS array: n_dense rounded down to 64 (fwd, dq)
  float* dqacc; int nq_pad;  // fused backward: f32 dQ accumulator [B*H][nq_pad][64] (workspace)
  int H;
  // Fused QK-RMSNorm + RoPE backward (vpt_attn_bwd_qknorm; qkn = 0: dq / dk are plain gradients of the attention
  // inputs). dq / dk then receive d loss / d (raw q, k), the pre-norm projections read from xq / xk.
  int qkn;
  Tensor4 xq, xk;
  const bf16_t* wq; const bf16_t* wk;   // q_norm / k_norm weights [64]
  const float* rcos; const float* rsin; // RoPE tables [positions][32]
  float eps;
  float* dwq; float* dwk;               // per-workgroup partial weight gradients, rows of 64 at stride dw_ld
  long dw_ld;
  int xcd;  // block order: 1 = XCD-contiguous (xcd_remap), 0 = linear
  int pm;   // backward partner-wave treatment (diagnostic build only; 0 in production): bit 0 = s_setprio 1 for the
            // wave in an odd slot of its SIMD, bit 1 = that wave's block starts pm >> 2 ticks (10 ns) late
};

constexpr float kNegInf = -__builtin_huge_valf();
constexpr float kTau = 8.f;  // forward lazy-rescale threshold, log2 units
#ifdef VPT_DIAG
// diagnostic build only (libvpt_hip_diag.so): process-wide A/B switches
int g_variant = 0;  // backward kernel variant (vpt_attn_set_variant; 1, 2 = timing-only ablations)
int g_waves = 4;    // waves per block (vpt_attn_set_variant 3 -> 8-wave blocks, A/B only)
float g_tau = kTau; // forward lazy-rescale threshold (vpt_attn_set_rescale_threshold)
int g_bwd_nst = 2;  // backward LDS ring stages (vpt_attn_set_bwd_stages, A/B)
int g_fwd_ord = 1;  // forward S^T chain with its K fragments read first (vpt_attn_set_fwd_order, A/B)
int g_bwd_pf = 0;   // backward transposed-fragment prefetch (vpt_attn_set_bwd_prefetch bit mask, A/B)
int g_xcd = 1;      // block order of the forward / backward grids (vpt_attn_set_xcd_order, A/B)
int g_rows64 = 0;   // backward variants (vpt_attn_set_rows64 bit mask, A/B): 1 = 64-key dK/dV, 2 = 64-query dQ
                    // at 2 waves / SIMD, 4 = 64-query dQ at 1 wave / SIMD; 0 = the 32-row pair
int g_pm = 0;       // backward partner-wave priority / stagger (vpt_attn_set_bwd_partner, A/B)
int g_fwd_lsm = 0;  // QK-norm forward: row sums on the MFMA pipe (vpt_attn_set_fwd_lsum, A/B)
int g_mf16 = 7;     // backward bodies on the 16x16x32 MFMA (vpt_attn_set_bwd_mfma16: 0 = the 32x32x16 bodies, A/B)
int g_fwd16 = 0;    // QK-norm forward on the 16x16x32 MFMA (vpt_attn_set_fwd_mfma16, A/B)
#else
constexpr int g_variant = 0, g_waves = 4;
constexpr float g_tau = kTau;
// XCD-contiguous block order (r04s: -1.1 % fwd, -1.8 % bwd, 4x less HBM traffic; +0.38 % per C3 step, r04t) and the
// forward's S^T chain with its K fragments read first (+0.32 % per C3 step, r04t)
constexpr int g_xcd = 1, g_fwd_ord = 1;
// The QK-norm forward's row sums on the MFMA pipe (fwd_body LSM): forward +3.3 %, C3 step -0.49 % (r05n) -- the loop is
// not VALU-issue bound, and the extra MFMAs cost more than the 32 adds per tile they replace. Off.
constexpr int g_fwd_lsm = 0;
#endif

// Reductions over the lane pair (l, l^32) with v_permlane32_swap (VALU, no LDS round trip): the two
// results together hold both halves' values in every lane, whichever half the swap moves.
__device__ __forceinline__ float pair_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ int sigma(int r) { return ((r >> 1) & 7) ^ ((r & 2) << 1); }
// The 16x16x32 bodies' tile image (dkdv16_body / dq16_body): chunk c of row r at position c ^ (r & 6). Conflict-free for
// their ds_read_b128 row fragments (row 16t + (lane & 15), chunk 4ks + (lane >> 4): per lane group of the b128 read the
// 8 even rows -- and the 8 odd ones -- take 8 distinct slots) and their transposed ds_read_b64_tr_b16 reads (rows
// r0 + 4(lane >> 4) + 0..3 of units 4dt + 0..3: per 32 lanes, rows r0..r0+7 in 8 distinct chunk pairs). The 32x32
// bodies' sigma is 2-way conflicted on the 16-row pattern.
__device__ __forceinline__ int sigma16(int r) { return r & 6; }
template <int SW>
__device__ __forceinline__ int sig(int r) { return SW ? sigma16(r) : sigma(r); }
__device__ __forceinline__ int tile16_off(int row, int chunk) { return row * 128 + ((chunk ^ sigma16(row)) << 4); }
__device__ __forceinline__ int tile16_unit_off(int row, int unit) {
  return row * 128 + (((unit >> 1) ^ sigma16(row)) << 4) + ((unit & 1) << 3);
}
__device__ __forceinline__ int tile_off(int row, int chunk) { return row * 128 + ((chunk ^ sigma(row)) << 4); }
__device__ __forceinline__ int tile_unit_off(int row, int unit) {
  return row * 128 + (((unit >> 1) ^ sigma(row)) << 4) + ((unit & 1) << 3);
}

// ---- LDS-DMA staging (global_load_lds; guide §5.7): one wave-instruction moves 1 KB (dwordx4, 16 B
// per lane) or 256 B (dword) from a wave-uniform SGPR base + per-lane 32-bit offset straight into LDS
// at M0 + lane*width. No VGPR round trip and no ds_write; completion is `s_waitcnt vmcnt(0)` by the
// issuing wave, then a barrier. The opening s_nop covers SGPR operands written by v_readfirstlane.
__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (const void*)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(VPT_LDS const char*)p);
}
__device__ __forceinline__ void dma_x4(const void* sbase, uint32_t voff, uint32_t m0v) {
  unsigned keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(m0v) : "memory");
}
__device__ __forceinline__ void dma_x1(const void* sbase, uint32_t voff, uint32_t m0v) {
  unsigned keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(m0v) : "memory");
}
// Rows r0..r0+63 of a (b,h) slice -> the tile_off LDS image: 8 pieces of 1 KB (rows 8q..8q+7), 8/NW
// per wave (q = (8/NW)*wid + i). The image is written lane-linearly, so position p of a row receives its
// logical chunk p ^ sigma(row) (sigma-swizzle moved to the source address). Rows >= n are clamped to
// n-1: finite values the callers mask (keys: -inf bias; queries: zeroed rows).
template <int NW>
__device__ __forceinline__ void dma_rows(char* lds, const void* head, long sr, int r0, int n, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 8 / NW; ++i) {
    const int q = (8 / NW) * wid + i, row = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ sigma(row);
    const int r = min(r0 + row, n - 1);
    dma_x4(head, (uint32_t)(((long)r * sr + c * 8) * 2), lds_addr(lds + q * 1024));
  }
}
// dma_rows with the LDS tile given as a byte address (lds_tile, wave-uniform) and a fast path for full
// tiles (r0 + 64 <= n): the row advance goes into the scalar base (head + r0 rows) and the per-lane offsets
// (row * sr + chunk) * 2 come precomputed from a RowPlan (loop-invariant registers), so no clamp, 64-bit
// multiply, generic-to-LDS conversion or readfirstlane is issued per piece; only the last, partial tile takes
// the clamped path.
template <int NW>
struct RowPlan {
  uint32_t voff[8 / NW];
  uint32_t wq;  // this wave's first piece within a tile image (bytes)
};
template <int NW, int SW = 0>
__device__ __forceinline__ RowPlan<NW> row_plan(long sr, int wid, int lane) {
  RowPlan<NW> p;
#pragma unroll
  for (int i = 0; i < 8 / NW; ++i) {
    const int q = (8 / NW) * wid + i, row = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ sig<SW>(row);
    p.voff[i] = (uint32_t)((row * (int)sr + c * 8) * 2);
  }
  p.wq = __builtin_amdgcn_readfirstlane((uint32_t)((8 / NW) * wid * 1024));
  return p;
}
template <int NW, int SW = 0>
__device__ __forceinline__ void dma_rows_at(uint32_t lds_tile, const void* head, long sr, int r0, int n,
                                            const RowPlan<NW>& p, int wid, int lane) {
  if (r0 + 64 <= n) {
    const void* base = (const char*)head + (long)r0 * sr * 2;
#pragma unroll
    for (int i = 0; i < 8 / NW; ++i) dma_x4(base, p.voff[i], lds_tile + p.wq + i * 1024);
  } else {
#pragma unroll
    for (int i = 0; i < 8 / NW; ++i) {
      const int q = (8 / NW) * wid + i, row = 8 * q + (lane >> 3);
      const int c = (lane & 7) ^ sig<SW>(row);
      const int r = min(r0 + row, n - 1);
      dma_x4(head, (uint32_t)(((long)r * sr + c * 8) * 2), lds_tile + p.wq + i * 1024);
    }
  }
}
// 64 f32 statistics (rows r0..r0+63, clamped to n-1) -> lds, one 256-B piece.
__device__ __forceinline__ void dma_stat(float* lds, const void* head, int r0, int n, int lane) {
  dma_x1(head, (uint32_t)(min(r0 + lane, n - 1) * 4), lds_addr(lds));
}
// Zero rows nv..63 of a staged 64x64 tile (all 8 chunks of each row).
template <int NW>
__device__ __forceinline__ void zero_rows(char* lds, int nv, int tid) {
  for (int idx = tid; idx < (64 - nv) * 8; idx += 64 * NW)
    *reinterpret_cast<uint4*>(lds + (nv + (idx >> 3)) * 128 + (idx & 7) * 16) = make_uint4(0, 0, 0, 0);
}

// A-operand (32 rows x 16 k) read by rows: lane row = rbase + (lane&31), k = 16s + 8h + j.
__device__ __forceinline__ bf16x8 frag_rows(const char* lds, int rbase, int s, int lane) {
  const int row = rbase + (lane & 31);
  return as_frag(*reinterpret_cast<const uint4*>(lds + tile_off(row, 2 * s + (lane >> 5))));
}
// A-operand read transposed: rows = head dims d = 32*db + (lane&31); k = tile rows
// 16s' + 8(j>>2) + 4h + (j&3) where s' indexes 16-row steps of the 64-row tile.
__device__ __forceinline__ bf16x8 frag_tr(const char* lds, int db, int s16, int lane) {
  const int G = lane >> 4, i16 = lane & 15, qq = i16 >> 2, p = i16 & 3, h = lane >> 5;
  const int row = 16 * s16 + 4 * h + qq;
  const int unit = 8 * db + 4 * (G & 1) + p;
  uint2 lo = lds_read_tr16((const VPT_LDS void*)(lds + tile_unit_off(row, unit)));
  uint2 hi = lds_read_tr16((const VPT_LDS void*)(lds + tile_unit_off(row + 8, unit)));
  return as_frag2(lo, hi);
}
// 16x16x32 operands from a tile16 image. Rows: lane row = rbase + (lane&15), k = 32ks + 8(lane>>4) + j.
__device__ __forceinline__ bf16x8 frag16_rows(const char* lds, int rbase, int ks, int lane) {
  return as_frag(*reinterpret_cast<const uint4*>(lds + tile16_off(rbase + (lane & 15), 4 * ks + (lane >> 4))));
}
// Transposed: lane row = head dim 16dt + (lane&15); k slot j of lane group G = lane>>4 is tile row
// 32m + 16(j>>2) + 4G + (j&3) -- the order in which two row-adjacent 16x16 accumulators (rows 4G + e) pack.
__device__ __forceinline__ bf16x8 frag16_tr(const char* lds, int dt, int m, int lane) {
  const int i16 = lane & 15, row = 32 * m + 4 * (lane >> 4) + (i16 >> 2), unit = 4 * dt + (i16 & 3);
  uint2 lo = lds_read_tr16((const VPT_LDS void*)(lds + tile16_unit_off(row, unit)));
  uint2 hi = lds_read_tr16((const VPT_LDS void*)(lds + tile16_unit_off(row + 16, unit)));
  return as_frag2(lo, hi);
}
__device__ __forceinline__ floatx4 mfma16(bf16x8 a, bf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// Two row-adjacent 16x16 accumulators (rows 4G + e and 16 + 4G + e) as one bf16 operand (k slots as frag16_tr).
__device__ __forceinline__ bf16x8 pack16(const floatx4& a, const floatx4& b) {
  uint4 v;
  v.x = pack_bf16x2(a[0], a[1]);
  v.y = pack_bf16x2(a[2], a[3]);
  v.z = pack_bf16x2(b[0], b[1]);
  v.w = pack_bf16x2(b[2], b[3]);
  return as_frag(v);
}
// B operand held in registers for row `row` of a global tensor: lane col = row, d = 32ks + 8(lane>>4) + j.
__device__ __forceinline__ void load_row_frags16(bf16x8 (&f)[2], const bf16_t* base, long sr, int row, int n, int lane) {
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < n) v = *reinterpret_cast<const uint4*>(base + (long)row * sr + 32 * ks + 8 * (lane >> 4));
    f[ks] = as_frag(v);
  }
}
// B-operand held in registers for a row of a global tensor: lane col = row (lane&31),
// elements d = 16s + 8h + j.
__device__ __forceinline__ void load_row_frags(bf16x8 (&f)[4], const bf16_t* base, long sr, int row, int n, int lane) {
  const int h = lane >> 5;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (row < n) v = *reinterpret_cast<const uint4*>(base + (long)row * sr + 16 * s + 8 * h);
    f[s] = as_frag(v);
  }
}
// Pack accumulator registers 8s..8s+7 to a bf16 operand fragment.
__device__ __forceinline__ bf16x8 pack_acc(const floatx16& a, int s) {
  uint4 v;
  v.x = pack_bf16x2(a[8 * s + 0], a[8 * s + 1]);
  v.y = pack_bf16x2(a[8 * s + 2], a[8 * s + 3]);
  v.z = pack_bf16x2(a[8 * s + 4], a[8 * s + 5]);
  v.w = pack_bf16x2(a[8 * s + 6], a[8 * s + 7]);
  return as_frag(v);
}
__device__ __forceinline__ floatx16 mfma32(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ floatx16 splat16(float v) {
  floatx16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = v;
  return r;
}
// Accumulator-layout tile of 16 per-row constants from an LDS row vector: register 4*g4+e of lane
// holds row 8*g4 + 4*(lane>>5) + e (v_mfma_f32_32x32x16 D layout), rows offset by r0.
__device__ __forceinline__ floatx16 rows16(const float* v, int r0, int h) {
  floatx16 r;
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const floatx4 x = *reinterpret_cast<const floatx4*>(v + r0 + 8 * g4 + 4 * h);
#pragma unroll
    for (int e = 0; e < 4; ++e) r[4 * g4 + e] = x[e];
  }
  return r;
}
__device__ __forceinline__ float key_bias(const AttnArgs& g, int b, int key) {
  if (key >= g.nk) return kNegInf;
  if (key < g.n_dense || !g.kbias) return 0.f;
  return g.kbias[(long)b * g.kb_sb + key];
}
// Writes a [64 d][32 rows] transposed accumulator pair (rows on the lane) as row-major bf16; `zero`
// stores exact zeros instead (masked keys, whose accumulators may hold non-finite values).
__device__ __forceinline__ void store_T(const OTensor4& t, long base_off, const floatx16 (&acc)[2], float mul,
                                        int row, int n, int lane, bool zero) {
  if (row >= n) return;
  const int h = lane >> 5;
  bf16_t* dst = t.p + base_off + (long)row * t.sr;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      const int d = 32 * db + 8 * g4 + 4 * h;
      uint2 w;
      w.x = pack_bf16x2(acc[db][4 * g4 + 0] * mul, acc[db][4 * g4 + 1] * mul);
      w.y = pack_bf16x2(acc[db][4 * g4 + 2] * mul, acc[db][4 * g4 + 3] * mul);
      if (zero) w = make_uint2(0u, 0u);
      *reinterpret_cast<uint2*>(dst + d) = w;
    }
}
// store_T for four transposed 16x16 accumulators of one row (16x16x32 bodies): register e of acc[dt] of lane l holds
// dim 16dt + 4(l>>4) + e of the lane's row.
__device__ __forceinline__ void store16_T(const OTensor4& t, long base_off, const floatx4 (&acc)[4], float mul, int row,
                                          int n, int lane, bool zero) {
  if (row >= n) return;
  bf16_t* dst = t.p + base_off + (long)row * t.sr + 4 * (lane >> 4);
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) {
    uint2 w;
    w.x = pack_bf16x2(acc[dt][0] * mul, acc[dt][1] * mul);
    w.y = pack_bf16x2(acc[dt][2] * mul, acc[dt][3] * mul);
    if (zero) w = make_uint2(0u, 0u);
    *reinterpret_cast<uint2*>(dst + 16 * dt) = w;
  }
}

// ---- fused QK-RMSNorm + RoPE backward of one q / k row (JiT Attention.q_norm / k_norm + apply_rope,
// src/models/jit/denoiser.py:307-316, 98-111; the standalone form is qknorm_rope_bwd_kernel, csrc/norm.hip).
// The row's gradient arrives as a transposed accumulator pair (row on the lane, register 16 db + 4 g4 + e of lane l
// holding dim d = 32 db + 8 g4 + 4 h + e, h = l >> 5): g = mul * acc = d loss / d rope(rms(x) w), in f32 (never
// rounded to bf16 on the way). Lanes l and l + 32 hold the two halves of the row, so the two 64-dim sums are one
// permlane32 swap each. Writes dx = d loss / d x (bf16) and adds this row's dy * xhat to dwp (this lane's 32 dims).
__device__ __forceinline__ int qkn_dim(int v, int h) { return 32 * (v >> 4) + 8 * ((v >> 2) & 3) + 4 * h + (v & 3); }

__device__ __forceinline__ void qkn_load_w(const bf16_t* w, int lane, float (&wf)[32]) {
  const int h = lane >> 5;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint2 u = *reinterpret_cast<const uint2*>(w + qkn_dim(4 * q, h));
    wf[4 * q + 0] = __uint_as_float(u.x << 16); wf[4 * q + 1] = __uint_as_float(u.x & 0xffff0000u);
    wf[4 * q + 2] = __uint_as_float(u.y << 16); wf[4 * q + 3] = __uint_as_float(u.y & 0xffff0000u);
  }
}

__device__ __forceinline__ void qkn_bwd_row(const AttnArgs& g, const Tensor4& xs, const OTensor4& out, int b, int hd,
                                            const floatx16 (&acc)[2], float mul, const float (&wf)[32], int row, int n,
                                            int lane, bool zero, float (&dwp)[32]) {
  if (row >= n) return;  // both lanes of a row take the same branch (the swaps below pair l with l ^ 32)
  const int h = lane >> 5;
  const bf16_t* xr = xs.p + (long)b * xs.sb + (long)hd * xs.sh + (long)row * xs.sr;
  bf16_t* orow = out.p + (long)b * out.sb + (long)hd * out.sh + (long)row * out.sr;
  if (zero) {  // masked key: its gradient is exactly zero (and contributes nothing to the weight gradient)
#pragma unroll
    for (int q = 0; q < 8; ++q) *reinterpret_cast<uint2*>(orow + qkn_dim(4 * q, h)) = make_uint2(0u, 0u);
    return;
  }
  float x[32], cs[16], sn[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int d0 = qkn_dim(4 * q, h);
    const uint2 u = *reinterpret_cast<const uint2*>(xr + d0);
    x[4 * q + 0] = __uint_as_float(u.x << 16); x[4 * q + 1] = __uint_as_float(u.x & 0xffff0000u);
    x[4 * q + 2] = __uint_as_float(u.y << 16); x[4 * q + 3] = __uint_as_float(u.y & 0xffff0000u);
    const float2 c2 = *reinterpret_cast<const float2*>(g.rcos + (long)row * 32 + d0 / 2);
    const float2 s2 = *reinterpret_cast<const float2*>(g.rsin + (long)row * 32 + d0 / 2);
    cs[2 * q] = c2.x; cs[2 * q + 1] = c2.y; sn[2 * q] = s2.x; sn[2 * q + 1] = s2.y;
  }
  float ss = 0.f;
#pragma unroll
  for (int v = 0; v < 32; ++v) ss += x[v] * x[v];
  const float r = rsqrtf(pair_sum(ss) * (1.f / 64.f) + g.eps);
  float dy[32], xh[32], gg[32], dot = 0.f;
#pragma unroll
  for (int p = 0; p < 16; ++p) {  // RoPE backward: rotate the pair (2p, 2p + 1) back by the conjugate
    const int db = p >> 3, i = (p >> 1) & 3, e = 2 * (p & 1);
    const float a = acc[db][4 * i + e] * mul, c = acc[db][4 * i + e + 1] * mul;
    dy[2 * p] = a * cs[p] + c * sn[p];
    dy[2 * p + 1] = -a * sn[p] + c * cs[p];
  }
#pragma unroll
  for (int v = 0; v < 32; ++v) {
    xh[v] = x[v] * r;
    gg[v] = dy[v] * wf[v];
    dot += gg[v] * xh[v];
    dwp[v] += dy[v] * xh[v];
  }
  dot = pair_sum(dot) * (1.f / 64.f);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    uint2 w;
    w.x = pack_bf16x2(r * (gg[4 * q] - xh[4 * q] * dot), r * (gg[4 * q + 1] - xh[4 * q + 1] * dot));
    w.y = pack_bf16x2(r * (gg[4 * q + 2] - xh[4 * q + 2] * dot), r * (gg[4 * q + 3] - xh[4 * q + 3] * dot));
    *reinterpret_cast<uint2*>(orow + qkn_dim(4 * q, h)) = w;
  }
}

// The block's 128 rows' dwp (4 waves x 32 rows, two lanes per row) summed in a fixed order into dw[64] (one
// partial row per workgroup, reduced by vpt_reduce_rows). red: 32 KB of the staging LDS, red2: 1 KB.
template <int NW>
__device__ __forceinline__ void qkn_dw_partial(float* red, float* red2, const float (&dwp)[32], float* dw, int tid) {
  const int lane = tid & 63, wid = tid >> 6, h = lane >> 5;
  __syncthreads();  // every wave is done reading the staging tiles
#pragma unroll
  for (int q = 0; q < 8; ++q)
    *reinterpret_cast<floatx4*>(red + (wid * 32 + (lane & 31)) * 64 + qkn_dim(4 * q, h)) =
        floatx4{dwp[4 * q], dwp[4 * q + 1], dwp[4 * q + 2], dwp[4 * q + 3]};
  __syncthreads();
  {
    const int d = tid & 63, w = tid >> 6;
    float acc = 0.f;
    for (int r2 = 0; r2 < 32; ++r2) acc += red[(w * 32 + r2) * 64 + d];
    red2[w * 64 + d] = acc;
  }
  __syncthreads();
  if (tid < 64) {
    float acc = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) acc += red2[w * 64 + tid];
    dw[tid] = acc;
  }
}

// Key bias for keys [kb0, round_up(n, 64)) in LDS, filled once per block: 0 below n_dense,
// kbias[b][key] in [n_dense, n), -inf for the padding keys >= n. Dense tiles (kv0 + 64 <= n_dense)
// never read it.
// Bijective remap of a linear block id: the dispatcher deals blocks round-robin to the 8 XCDs (id % 8), so XCD x runs
// ids x, x + 8, ...; mapped here to the contiguous logical range [x * q8 + min(x, r8), ...). A (batch, head)'s blocks
// then run on one XCD, whose L2 holds that head's K / V (forward, dQ blocks) or Q / dO (dK / dV blocks) once.
__device__ __forceinline__ int xcd_remap(int id, int total) {
  const int q8 = total >> 3, r8 = total & 7, x = id & 7;
  return (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + (id >> 3);
}

template <int NW>
__device__ __forceinline__ void fill_key_bias(float* kbl, const AttnArgs& g, int b, int tid) {
  const int nk = (g.nk + 63) / 64 * 64 - g.kb0;
  for (int i = tid; i < nk; i += 64 * NW) kbl[i] = key_bias(g, b, g.kb0 + i);
}

// ------------------------------------------------------------------ forward
// NW waves per block, 32 query rows per wave: one K/V tile staged per block serves 32*NW queries.
// Occupancy: 134 VGPRs -> 3 waves per SIMD with 4-wave blocks (forcing <= 128 VGPRs for 4 waves
// spills inside the tile loop and measured slower: 749 vs 823 TFLOP/s).
//
// FIX (fixed reference point, vpt_attn_fwd_qknorm): when q and k are QK-RMSNormed (JiT, denoiser.py:307-316), every
// score is bounded by Cauchy-Schwarz: |q~.k| <= ||q~|| ||k|| <= (c 8 max|w_q|) (8 max|w_k|) = bound (log2 units, q~ the
// pre-scaled query, ||rms(x)|| <= 8 for 64 dims, RoPE a rotation; with margin for the bf16 roundings). Then
// p = exp2(s - bound) <= 1 needs no running row maximum: the per-tile fmax reduction, its lane-pair exchange and the
// rescale test -- a third of the loop's VALU at head_dim 64, where the softmax and not the MFMA bounds the loop --
// are gone. The caller's kernel takes this path only while bound < kFixMax (p >= 2^-2 bound stays a normal float:
// no underflow of the largest p); otherwise the online-max path below.
constexpr float kFixMax = 60.f;

// ORD: the S^T chain's 8 K fragments read from LDS before its MFMAs (one counted wait each), instead of hipcc's
// read-wait-MFMA order in one register quad (which exposes the LDS latency at every MFMA of the chain).
// LSM (with FIX; diagnostic A/B, off in production): the row sums l = sum_k p out of the MFMA pipe as a third O^T block,
// ones . P^T, from the same bf16 P the PV product uses (4 MFMAs per tile in place of 32 v_add_f32 per lane) --
// o = sum_k bf16(p) v / sum_k bf16(p). Measured slower (g_fwd_lsm).
template <int NW, bool FIX, bool ORD = false, bool LSM = false>
__device__ __forceinline__ void fwd_body(const AttnArgs& g, float bound, char (&lds)[2][2][8192], float* kbl, int bx,
                                         int hd, int b) {
  static_assert(!LSM || FIX, "MFMA row sums with the fixed reference point only");
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5;
  const int q0 = bx * (32 * NW) + wid * 32;
  const bf16_t* Q = g.q.p + b * g.q.sb + hd * g.q.sh;
  const bf16_t* K = g.k.p + b * g.k.sb + hd * g.k.sh;
  const bf16_t* V = g.v.p + b * g.v.sb + hd * g.v.sh;

  bf16x8 qf[4];  // pre-scaled query: K.Q^T is already in log2 units
  load_row_frags(qf, Q, g.q.sr, q0 + (lane & 31), g.n, lane);

  floatx16 oacc[2], lacc;
#pragma unroll
  for (int i = 0; i < 16; ++i) { oacc[0][i] = 0.f; oacc[1][i] = 0.f; lacc[i] = 0.f; }
  const bf16x8 ones = as_frag(make_uint4(0x3f803f80u, 0x3f803f80u, 0x3f803f80u, 0x3f803f80u));
  float m_c = FIX ? bound : 0.f, lsum = 0.f;  // reference point (log2 units), row sum
  floatx16 nm = splat16(-m_c);  // -m_c: the S^T chain's initial accumulator, so it ends at S - m_c

  const int nt = (g.nk + 63) / 64;
  const void* Ku = uniform_ptr(K);
  const void* Vu = uniform_ptr(V);
  fill_key_bias<NW>(kbl, g, b, tid);
  const uint32_t lb = lds_addr(&lds[0][0][0]);  // [buf][K / V] tiles of 8 KB
  const RowPlan<NW> pk = row_plan<NW>(g.k.sr, wid, lane), pv = row_plan<NW>(g.v.sr, wid, lane);
  dma_rows_at<NW>(lb, Ku, g.k.sr, 0, g.nk, pk, wid, lane);
  dma_rows_at<NW>(lb + 8192, Vu, g.v.sr, 0, g.nk, pv, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int cur = 0;
  for (int t = 0; t < nt; ++t) {
    const int kv0 = t * 64;
    const bool more = t + 1 < nt;
    if (more) {  // next K/V tile by LDS-DMA into the other buffer, in flight during this tile
      dma_rows_at<NW>(lb + (cur ^ 1) * 16384, Ku, g.k.sr, kv0 + 64, g.nk, pk, wid, lane);
      dma_rows_at<NW>(lb + (cur ^ 1) * 16384 + 8192, Vu, g.v.sr, kv0 + 64, g.nk, pv, wid, lane);
    }
    const char* lk = lds[cur][0];
    const char* lv = lds[cur][1];
    floatx16 sacc[2];  // S^T - m_c (log2 units) straight out of the MFMA chain
    if (ORD) {
      bf16x8 kr[2][4];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s = 0; s < 4; ++s) kr[kb][s] = frag_rows(lk, 32 * kb, s, lane);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        sacc[kb] = mfma32(kr[kb][0], qf[0], nm);
#pragma unroll
        for (int s = 1; s < 4; ++s) sacc[kb] = mfma32(kr[kb][s], qf[s], sacc[kb]);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        sacc[kb] = mfma32(frag_rows(lk, 32 * kb, 0, lane), qf[0], nm);
#pragma unroll
        for (int s = 1; s < 4; ++s) sacc[kb] = mfma32(frag_rows(lk, 32 * kb, s, lane), qf[s], sacc[kb]);
      }
    }
    if (kv0 + 64 > g.n_dense) {  // key bias 0 / -inf (context and padding tiles only)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const floatx4 bias = *reinterpret_cast<const floatx4*>(&kbl[kv0 - g.kb0 + 32 * kb + 8 * g4 + 4 * h]);
#pragma unroll
          for (int e = 0; e < 4; ++e) sacc[kb][4 * g4 + e] += bias[e];
        }
    }
    if (!FIX) {
      float mx = kNegInf;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) mx = fmaxf(mx, sacc[kb][i]);
      mx = pair_max(mx);
      // Lazy rescale: the reference point m_c moves only on the first tile and when a tile's max
      // exceeds it by more than tau (p <= 2^tau otherwise); wave-uniform branch, rarely taken after t=0.
      const bool up = t == 0 || mx > g.tau;
      if (__builtin_amdgcn_ballot_w64(up)) {
        const float sh = up && mx != kNegInf ? mx : 0.f;  // shift of the reference point
        if (t > 0) {
          const float alpha = __builtin_amdgcn_exp2f(-sh);
          lsum *= alpha;
#pragma unroll
          for (int i = 0; i < 16; ++i) { oacc[0][i] *= alpha; oacc[1][i] *= alpha; }
        }
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int i = 0; i < 16; ++i) sacc[kb][i] -= sh;
        m_c += sh;
        nm = splat16(-m_c);
      }
    }
    float ps = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = __builtin_amdgcn_exp2f(sacc[kb][i]);
        sacc[kb][i] = p;
        if (!LSM) ps += p;
      }
    if (!LSM) lsum += ps;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = pack_acc(sacc[kb], s);
#pragma unroll
        for (int db = 0; db < 2; ++db) oacc[db] = mfma32(frag_tr(lv, db, 2 * kb + s, lane), pf, oacc[db]);
        if (LSM) lacc = mfma32(ones, pf, lacc);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of the next tile landed
    __syncthreads();                                    // ... and every wave's; this tile fully read
    cur ^= 1;
  }
  const float l = LSM ? lacc[0] : pair_sum(lsum);  // LSM: every register of the lane holds its query's sum
  const float inv = 1.f / l;
  const int qrow = q0 + (lane & 31);
  store_T(g.o, (long)b * g.o.sb + hd * g.o.sh, oacc, inv, qrow, g.n, lane, false);
  if (lane < 32 && qrow < g.n) g.lse[b * g.l_sb + hd * g.l_sh + qrow] = -(m_c + __log2f(l));  // -LSE, log2
}

// Forward with the fixed reference point on the 16x16x32 MFMA (diagnostic A/B against fwd_body<FIX, ORD>, as
// dkdv16_body): 32 queries per wave as two query tiles qt on the lanes; per 64-key tile the 8 K row fragments read
// first, S^T - m_c as 2 x 2 x 2 accumulators (key half m, key tile u, query tile qt), the key bias on context / padding
// tiles, p = exp2, O^T (head-dim tile dt x qt) += V^T (frag16_tr) x P (pack16 of the two key tiles of a half). Each
// lane holds partial row sums over its 4-key groups; the four lane groups (lane >> 4) are summed once at the end.
template <int NW>
__device__ __forceinline__ void fwd16_body(const AttnArgs& g, float bound, char (&lds)[2][2][8192], float* kbl, int bx,
                                           int hd, int b) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, G = lane >> 4;
  const int q0 = bx * (32 * NW) + wid * 32;
  const bf16_t* Q = g.q.p + b * g.q.sb + hd * g.q.sh;
  const bf16_t* K = g.k.p + b * g.k.sb + hd * g.k.sh;
  const bf16_t* V = g.v.p + b * g.v.sb + hd * g.v.sh;

  bf16x8 qf[2][2];  // [qt][ks], pre-scaled query
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) load_row_frags16(qf[qt], Q, g.q.sr, q0 + 16 * qt + (lane & 15), g.n, lane);
  floatx4 oacc[2][4];  // [qt][dt]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int e = 0; e < 4; ++e) oacc[qt][dt][e] = 0.f;
  float lsum[2] = {0.f, 0.f};
  const float m_c = bound;

  const int nt = (g.nk + 63) / 64;
  const void* Ku = uniform_ptr(K);
  const void* Vu = uniform_ptr(V);
  fill_key_bias<NW>(kbl, g, b, tid);
  const uint32_t lb = lds_addr(&lds[0][0][0]);
  const RowPlan<NW> pk = row_plan<NW, 1>(g.k.sr, wid, lane), pv = row_plan<NW, 1>(g.v.sr, wid, lane);
  dma_rows_at<NW, 1>(lb, Ku, g.k.sr, 0, g.nk, pk, wid, lane);
  dma_rows_at<NW, 1>(lb + 8192, Vu, g.v.sr, 0, g.nk, pv, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  int cur = 0;
  for (int t = 0; t < nt; ++t) {
    const int kv0 = t * 64;
    if (t + 1 < nt) {
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384, Ku, g.k.sr, kv0 + 64, g.nk, pk, wid, lane);
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384 + 8192, Vu, g.v.sr, kv0 + 64, g.nk, pv, wid, lane);
    }
    const char* lk = lds[cur][0];
    const char* lv = lds[cur][1];
    bf16x8 kr[2][2][2];  // [m][u][ks]
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) kr[m][u][ks] = frag16_rows(lk, 32 * m + 16 * u, ks, lane);
    __builtin_amdgcn_sched_barrier(0);
    floatx4 sacc[2][2][2];  // [m][u][qt]: keys 32m + 16u + 4G + e, query 16qt + (lane & 15)
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) {
          floatx4 a;
#pragma unroll
          for (int e = 0; e < 4; ++e) a[e] = -m_c;
          a = mfma16(kr[m][u][0], qf[qt][0], a);
          sacc[m][u][qt] = mfma16(kr[m][u][1], qf[qt][1], a);
        }
    if (kv0 + 64 > g.n_dense) {  // key bias 0 / -inf (context and padding tiles only)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const floatx4 bias = *reinterpret_cast<const floatx4*>(&kbl[kv0 - g.kb0 + 32 * m + 16 * u + 4 * G]);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt)
#pragma unroll
            for (int e = 0; e < 4; ++e) sacc[m][u][qt][e] += bias[e];
        }
    }
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      float ps = 0.f;
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float p = __builtin_amdgcn_exp2f(sacc[m][u][qt][e]);
            sacc[m][u][qt][e] = p;
            ps += p;
          }
      lsum[qt] += ps;
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      bf16x8 pf[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) pf[qt] = pack16(sacc[m][0][qt], sacc[m][1][qt]);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 tv = frag16_tr(lv, dt, m, lane);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) oacc[qt][dt] = mfma16(tv, pf[qt], oacc[qt][dt]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    cur ^= 1;
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    float l = lsum[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const int qrow = q0 + 16 * qt + (lane & 15);
    store16_T(g.o, (long)b * g.o.sb + hd * g.o.sh, oacc[qt], 1.f / l, qrow, g.n, lane, false);
    if (G == 0 && qrow < g.n) g.lse[b * g.l_sb + hd * g.l_sh + qrow] = -(m_c + __log2f(l));
  }
}

template <int NW, bool QKN = false, bool ORD = false, bool LSM = false, bool M16 = false>
__global__ __launch_bounds__(64 * NW, 2) void attn_fwd_kernel(AttnArgs g) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][8192];
  extern __shared__ __attribute__((aligned(16))) float kbl[];  // key bias of keys kb0.. (fill_key_bias)
  int bx = blockIdx.x, hd = blockIdx.y, b = blockIdx.z;
  if (g.xcd) {
    const int nbx = gridDim.x, total = nbx * gridDim.y * gridDim.z;
    const int l = xcd_remap(bx + nbx * (hd + gridDim.y * b), total);
    bx = l % nbx;
    hd = (l / nbx) % gridDim.y;
    b = l / (nbx * gridDim.y);
  }
  if (QKN) {
    // score bound from the QK-norm weights (every wave computes the same value: wave-uniform branch)
    const int lane = threadIdx.x & 63;
    const float aq = fabsf(bf2f(g.wq[lane])), ak = fabsf(bf2f(g.wk[lane]));
    const float bound = g.scale_log2 * 64.f * wave_max(aq) * wave_max(ak) * 1.0625f;
    if (bound < kFixMax) {
      if constexpr (M16) fwd16_body<NW>(g, bound, lds, kbl, bx, hd, b);
      else fwd_body<NW, true, ORD, LSM>(g, bound, lds, kbl, bx, hd, b);
      return;
    }
  }
  fwd_body<NW, false, ORD>(g, 0.f, lds, kbl, bx, hd, b);
}

// ------------------------------------------------------------------ backward preprocess
// delta[b,h,q] = -sum_d dO[q,d] * O[q,d] (stored negated: it is the dP chains' initial accumulator);
// 8 lanes per (b,h,q) row.
__global__ void attn_bwd_pre_kernel(AttnArgs g, int H, long rows_total) {
#pragma clang fp contract(off)  // each product rounded, then summed (no fma): the results of the SLP-packed build
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long row = gid >> 3;
  const int part = gid & 7;
  float s = 0.f;
  long b = 0, hd = 0, q = 0;
  if (row < rows_total) {
    q = row % g.n; const long bh = row / g.n; hd = bh % H; b = bh / H;
    const uint4 a = *reinterpret_cast<const uint4*>(g.dO.p + b * g.dO.sb + hd * g.dO.sh + q * g.dO.sr + part * 8);
    const uint4 o = *reinterpret_cast<const uint4*>(g.o.p + b * g.o.sb + hd * g.o.sh + q * g.o.sr + part * 8);
    float fa[8], fo[8];
    unpack8(a, fa); unpack8(o, fo);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += fa[e] * fo[e];
  }
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  s += __shfl_xor(s, 4, 64);
  if (row < rows_total && part == 0) g.delta_out[b * g.l_sb + hd * g.l_sh + q] = -s;
}

// ------------------------------------------------------------------ backward dK, dV
// ABL (timing-only ablations, wrong results): 1 = no next-tile staging (global -> regs -> LDS) in
// the loop, 2 = transposed fragment reads replaced by row reads.
// Body of one dK/dV block (key block bx of head hd, batch b); lds = [buf][Q / dO] tiles, lstat = [buf][lse / delta].
// NST: LDS stages of the Q / dO ring (2: tile t+1 in flight during tile t; 3: tiles t+1 and t+2, counted vmcnt).
template <int ABL, int NW, int NST = 2>
__device__ __forceinline__ void dkdv_body(const AttnArgs& g, int bx, int hd, int b, char (&lds)[NST][2][8192],
                                          float (&lstat)[NST][2][64]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5;
  const int k0 = bx * (32 * NW) + wid * 32;
  const bf16_t* Q = g.q.p + b * g.q.sb + hd * g.q.sh;
  const bf16_t* dO = g.dO.p + b * g.dO.sb + hd * g.dO.sh;
  const float* LSE = g.lse + b * g.l_sb + hd * g.l_sh;
  const float* DEL = g.delta_in + b * g.l_sb + hd * g.l_sh;

  const int key = k0 + (lane & 31);
  bf16x8 kf[4], vf[4];
  load_row_frags(kf, g.k.p + b * g.k.sb + hd * g.k.sh, g.k.sr, key, g.nk, lane);
  load_row_frags(vf, g.v.p + b * g.v.sb + hd * g.v.sh, g.v.sr, key, g.nk, lane);
  const bool kmasked = key_bias(g, b, key) == kNegInf;
  // Retire those loads here, visibly to hipcc's wait placement: otherwise its wait for them sits at the
  // first MFMA inside the tile loop, runs every iteration, and -- vmcnt retiring in order -- also drains the
  // next tile's LDS-DMA issued just before it (the asm DMAs are invisible to the compiler).
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)

  floatx16 dvT[2], dkT[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dvT[0][i] = dvT[1][i] = dkT[0][i] = dkT[1][i] = 0.f; }

  const int nt = (g.n + 63) / 64;
  const void* Qu = uniform_ptr(Q);
  const void* Du = uniform_ptr(dO);
  const void* Lu = uniform_ptr(LSE);
  const void* Eu = uniform_ptr(DEL);
  // Q / dO tiles and their lse / delta rows by LDS-DMA (waves 0 and 1 also move one stats piece each).
  const uint32_t lb = lds_addr(&lds[0][0][0]);  // [buf][Q / dO] tiles of 8 KB
  const RowPlan<NW> pq = row_plan<NW>(g.q.sr, wid, lane), pd0 = row_plan<NW>(g.dO.sr, wid, lane);
  auto stage = [&](int buf, int r0) {
    dma_rows_at<NW>(lb + buf * 16384, Qu, g.q.sr, r0, g.n, pq, wid, lane);
    dma_rows_at<NW>(lb + buf * 16384 + 8192, Du, g.dO.sr, r0, g.n, pd0, wid, lane);
    if (wid == 0) dma_stat(lstat[buf][0], Lu, r0, g.n, lane);
    else if (wid == 1) dma_stat(lstat[buf][1], Eu, r0, g.n, lane);
  };
  // After the DMA into `buf` landed for every wave: a partial last query tile gets its padding rows of
  // Q and dO zeroed, so the clamped duplicates contribute nothing to dK (dS.Q) or dV (P^T.dO).
  // younger: a later tile's pieces were issued after this tile's (3-stage ring): wait only for this one's -- each
  // wave issues 4 pieces per tile (Q, dO) plus the stats piece on waves 0 and 1, and vmcnt retires in order.
  auto settle = [&](int buf, int r0, bool younger) {
    if (NST == 3 && younger) {
      if (wid < 2) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (g.n - r0 < 64) {
      zero_rows<NW>(lds[buf][0], g.n - r0, tid);
      zero_rows<NW>(lds[buf][1], g.n - r0, tid);
      __syncthreads();
    }
  };
  stage(0, 0);
  if (NST == 3 && ABL != 1 && nt > 1) stage(1, 64);
  settle(0, 0, NST == 3 && ABL != 1 && nt > 1);

  for (int t = 0; t < nt; ++t) {
    const int cur = NST == 2 ? (t & 1) : t % NST;
    const bool more = ABL != 1 && t + 1 < nt;
    if (NST == 2 && more) stage(cur ^ 1, (t + 1) * 64);
    if (NST == 3 && ABL != 1 && t + 2 < nt) stage((t + 2) % 3, (t + 2) * 64);
    const int nxt = NST == 2 ? (cur ^ 1) : (t + 1) % NST;
    const char* lq = lds[cur][0];
    const char* ld = lds[cur][1];
    if (ABL == 8 || ABL == 9 || ABL == 10) {
      // Explicitly ordered body: the row fragments and row constants of query block qb+1 are read while
      // block qb's S / dP chains run (s_setprio 1 around every MFMA group), P and dS are packed to bf16
      // as soon as they exist, and sched_barriers keep hipcc from sinking the reads back to their uses.
      floatx16 cs = rows16(lstat[cur][0], 0, h), cd = rows16(lstat[cur][1], 0, h);
      bf16x8 qa[4], da[4], pp[2][2], pd[2][2];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) { qa[ks] = frag_rows(lq, 0, ks, lane); da[ks] = frag_rows(ld, 0, ks, lane); }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        floatx16 s = cs, dp = cd;
        __builtin_amdgcn_sched_barrier(0);
        if (ABL != 10) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          s = mfma32(qa[ks], kf[ks], s);
          dp = mfma32(da[ks], vf[ks], dp);
        }
        if (ABL != 10) __builtin_amdgcn_s_setprio(0);
        if (qb == 0) {
          cs = rows16(lstat[cur][0], 32, h);
          cd = rows16(lstat[cur][1], 32, h);
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) { qa[ks] = frag_rows(lq, 32, ks, lane); da[ks] = frag_rows(ld, 32, ks, lane); }
        }
        __builtin_amdgcn_sched_barrier(0);
        floatx16 P, dS;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float p = __builtin_amdgcn_exp2f(s[i]);
          P[i] = p;
          dS[i] = p * dp[i];
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) { pp[qb][s2] = pack_acc(P, s2); pd[qb][s2] = pack_acc(dS, s2); }
      }
      __builtin_amdgcn_sched_barrier(0);
      if (ABL == 9) {
        // the transposed Q / dO fragments of step st + 1 are read before step st's four MFMAs (two register sets), so
        // no dV / dK MFMA waits on a read issued right before it
        bf16x8 tv[2][2], tq[2][2];
        auto rd = [&](int st) {
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            tv[st & 1][db] = frag_tr(ld, db, st, lane);
            tq[st & 1][db] = frag_tr(lq, db, st, lane);
          }
        };
        rd(0);
#pragma unroll
        for (int st = 0; st < 4; ++st) {
          if (st + 1 < 4) rd(st + 1);
          __builtin_amdgcn_sched_barrier(0);
          if (ABL != 10) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            dvT[db] = mfma32(tv[st & 1][db], pp[st >> 1][st & 1], dvT[db]);
            dkT[db] = mfma32(tq[st & 1][db], pd[st >> 1][st & 1], dkT[db]);
          }
          if (ABL != 10) __builtin_amdgcn_s_setprio(0);
          __builtin_amdgcn_sched_barrier(0);
        }
        if (more) settle(nxt, (t + 1) * 64, NST == 3 && t + 2 < nt);
        continue;
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 tv[2], tq[2];
#pragma unroll
          for (int db = 0; db < 2; ++db) { tv[db] = frag_tr(ld, db, 2 * qb + s2, lane); tq[db] = frag_tr(lq, db, 2 * qb + s2, lane); }
          if (ABL != 10) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int db = 0; db < 2; ++db) {
            dvT[db] = mfma32(tv[db], pp[qb][s2], dvT[db]);
            dkT[db] = mfma32(tq[db], pd[qb][s2], dkT[db]);
          }
          if (ABL != 10) __builtin_amdgcn_s_setprio(0);
        }
      if (more) settle(nxt, (t + 1) * 64, NST == 3 && t + 2 < nt);
      continue;
    }
    floatx16 P[2], dS[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      // Row constants as the initial accumulators (guide App. B): S' = Q~.K^T - LSE (Q~ pre-scaled, so
      // log2 units) and dP' = dO.V^T - delta leave the chains ready for p = exp2(S'), dS = p * dP'.
      floatx16 s = rows16(lstat[cur][0], 32 * qb, h), dp = rows16(lstat[cur][1], 32 * qb, h);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s = mfma32(ABL == 6 ? vf[ks] : frag_rows(lq, 32 * qb, ks, lane), kf[ks], s);
        dp = mfma32(ABL == 6 ? kf[ks] : frag_rows(ld, 32 * qb, ks, lane), vf[ks], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        // No key bias here: a masked key (bias -inf) only feeds its own lane's dK/dV columns, which
        // are stored as exact zeros below.
        const float p = ABL == 3 ? s[i] : __builtin_amdgcn_exp2f(s[i]);
        P[qb][i] = p;
        dS[qb][i] = p * dp[i];
      }
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const bf16x8 pp = pack_acc(P[qb], s2);
        const bf16x8 pd = pack_acc(dS[qb], s2);
        if (ABL == 4) {  // timing: one MFMA per (qb, s2) keeps P, dS alive in place of the 4 products
          dvT[0] = mfma32(pp, pd, dvT[0]);
          continue;
        }
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          if (ABL == 5) {  // timing: register operands in place of the transposed LDS reads
            dvT[db] = mfma32(kf[2 * db + s2], pp, dvT[db]);
            dkT[db] = mfma32(vf[2 * db + s2], pd, dkT[db]);
          } else if (ABL == 2) {
            dvT[db] = mfma32(frag_rows(ld, 32 * db, 2 * qb + s2, lane), pp, dvT[db]);
            dkT[db] = mfma32(frag_rows(lq, 32 * db, 2 * qb + s2, lane), pd, dkT[db]);
          } else {
            dvT[db] = mfma32(frag_tr(ld, db, 2 * qb + s2, lane), pp, dvT[db]);
            dkT[db] = mfma32(frag_tr(lq, db, 2 * qb + s2, lane), pd, dkT[db]);
          }
        }
      }
    if (more) settle(nxt, (t + 1) * 64, NST == 3 && t + 2 < nt);
  }
  store_T(g.dv, (long)b * g.dv.sb + hd * g.dv.sh, dvT, 1.f, key, g.nk, lane, kmasked);
  // dK = scale * dS^T.Q = (scale / c) * dS^T.Q~ with Q~ = c*Q, c = scale*log2(e): the factor is ln 2
  if (!g.qkn) {
    store_T(g.dk, (long)b * g.dk.sb + hd * g.dk.sh, dkT, 0.69314718055994531f, key, g.nk, lane, kmasked);
    return;
  }
  float wf[32], dwp[32];
  qkn_load_w(g.wk, lane, wf);
#pragma unroll
  for (int v = 0; v < 32; ++v) dwp[v] = 0.f;
  qkn_bwd_row(g, g.xk, g.dk, b, hd, dkT, 0.69314718055994531f, wf, key, g.nk, lane, kmasked, dwp);
  qkn_dw_partial<NW>(reinterpret_cast<float*>(&lds[0][0][0]), &lstat[0][0][0], dwp,
                     g.dwk + ((long)(b * g.H + hd) * ((g.nk + 32 * NW - 1) / (32 * NW)) + bx) * g.dw_ld, tid);
}

// dK/dV body on the 16x16x32 MFMA (diagnostic A/B against dkdv_body's 32x32x16: the same 32 keys per wave, 64-query
// tiles, products, LDS bytes and VALU; guide MI355X_MICROARCH 'DVFS give-back' item 7: under load the chip can hold a
// higher clock on one MFMA shape than on the other). Per tile and 32-query half m: S and dP as 2 x 2 accumulators
// (query tile u, key tile kt) of 2 K steps, P = exp2(S), dS = P dP packed per key tile into one 32-query operand
// (pack16), then dV^T / dK^T (head-dim tile dt x key tile kt) += dO^T / Q^T (frag16_tr) x P / dS. Self-attention
// inputs without the fused QK-norm epilogue (g.qkn == 0).
// ORD: explicitly ordered as dkdv_body's body 10 -- the row fragments of half m + 1 read while half m's S / dP chains
// run, P / dS of both halves packed before the dV / dK products, sched_barriers against hipcc's re-sinking.
template <int NW, bool ORD = false>
__device__ __forceinline__ void dkdv16_body(const AttnArgs& g, int bx, int hd, int b, char (&lds)[2][2][8192],
                                            float (&lstat)[2][2][64]) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, G = lane >> 4;
  const int k0 = bx * (32 * NW) + wid * 32;
  const bf16_t* Q = g.q.p + b * g.q.sb + hd * g.q.sh;
  const bf16_t* dO = g.dO.p + b * g.dO.sb + hd * g.dO.sh;
  const float* LSE = g.lse + b * g.l_sb + hd * g.l_sh;
  const float* DEL = g.delta_in + b * g.l_sb + hd * g.l_sh;

  bf16x8 kf[2][2], vf[2][2];
  bool kmasked[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + 16 * kt + (lane & 15);
    load_row_frags16(kf[kt], g.k.p + b * g.k.sb + hd * g.k.sh, g.k.sr, key, g.nk, lane);
    load_row_frags16(vf[kt], g.v.p + b * g.v.sb + hd * g.v.sh, g.v.sr, key, g.nk, lane);
    kmasked[kt] = key_bias(g, b, key) == kNegInf;
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): as in dkdv_body

  floatx4 dv[2][4], dk[2][4];  // [kt][dt]
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int e = 0; e < 4; ++e) { dv[kt][dt][e] = 0.f; dk[kt][dt][e] = 0.f; }

  const int nt = (g.n + 63) / 64;
  const void* Qu = uniform_ptr(Q);
  const void* Du = uniform_ptr(dO);
  const void* Lu = uniform_ptr(LSE);
  const void* Eu = uniform_ptr(DEL);
  const uint32_t lb = lds_addr(&lds[0][0][0]);
  const RowPlan<NW> pq = row_plan<NW, 1>(g.q.sr, wid, lane), pd0 = row_plan<NW, 1>(g.dO.sr, wid, lane);
  auto stage = [&](int buf, int r0) {
    dma_rows_at<NW, 1>(lb + buf * 16384, Qu, g.q.sr, r0, g.n, pq, wid, lane);
    dma_rows_at<NW, 1>(lb + buf * 16384 + 8192, Du, g.dO.sr, r0, g.n, pd0, wid, lane);
    if (wid == 0) dma_stat(lstat[buf][0], Lu, r0, g.n, lane);
    else if (wid == 1) dma_stat(lstat[buf][1], Eu, r0, g.n, lane);
  };
  auto settle = [&](int buf, int r0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (g.n - r0 < 64) {  // padding query rows zeroed: no dK / dV contribution
      zero_rows<NW>(lds[buf][0], g.n - r0, tid);
      zero_rows<NW>(lds[buf][1], g.n - r0, tid);
      __syncthreads();
    }
  };
  stage(0, 0);
  settle(0, 0);

  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    const bool more = t + 1 < nt;
    if (more) stage(cur ^ 1, (t + 1) * 64);
    const char* lq = lds[cur][0];
    const char* ld = lds[cur][1];
    if constexpr (ORD) {
      bf16x8 qa[2][2], da[2][2], pp[2][2], pd[2][2];  // qa / da [u][ks]; pp / pd [m][kt]
      auto rd = [&](int m) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            qa[u][ks] = frag16_rows(lq, 32 * m + 16 * u, ks, lane);
            da[u][ks] = frag16_rows(ld, 32 * m + 16 * u, ks, lane);
          }
      };
      rd(0);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        floatx4 s[2][2], dp[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const floatx4 cs = *reinterpret_cast<const floatx4*>(&lstat[cur][0][32 * m + 16 * u + 4 * G]);
          const floatx4 cd = *reinterpret_cast<const floatx4*>(&lstat[cur][1][32 * m + 16 * u + 4 * G]);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) { s[u][kt] = cs; dp[u][kt] = cd; }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int kt = 0; kt < 2; ++kt) {
              s[u][kt] = mfma16(qa[u][ks], kf[kt][ks], s[u][kt]);
              dp[u][kt] = mfma16(da[u][ks], vf[kt][ks], dp[u][kt]);
            }
        if (m == 0) rd(1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          floatx4 P[2], dS[2];
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float p = __builtin_amdgcn_exp2f(s[u][kt][e]);
              P[u][e] = p;
              dS[u][e] = p * dp[u][kt][e];
            }
          pp[m][kt] = pack16(P[0], P[1]);
          pd[m][kt] = pack16(dS[0], dS[1]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int dt = 0; dt < 4; ++dt) {
          const bf16x8 tv = frag16_tr(ld, dt, m, lane);
          const bf16x8 tq = frag16_tr(lq, dt, m, lane);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            dv[kt][dt] = mfma16(tv, pp[m][kt], dv[kt][dt]);
            dk[kt][dt] = mfma16(tq, pd[m][kt], dk[kt][dt]);
          }
        }
      if (more) settle(cur ^ 1, (t + 1) * 64);
      continue;
    }
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      floatx4 s[2][2], dp[2][2];  // [u][kt]: query rows 32m + 16u + 4G + e, key 16kt + (lane & 15)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const floatx4 cs = *reinterpret_cast<const floatx4*>(&lstat[cur][0][32 * m + 16 * u + 4 * G]);
        const floatx4 cd = *reinterpret_cast<const floatx4*>(&lstat[cur][1][32 * m + 16 * u + 4 * G]);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) { s[u][kt] = cs; dp[u][kt] = cd; }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 qa = frag16_rows(lq, 32 * m + 16 * u, ks, lane);
          const bf16x8 da = frag16_rows(ld, 32 * m + 16 * u, ks, lane);
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[u][kt] = mfma16(qa, kf[kt][ks], s[u][kt]);
            dp[u][kt] = mfma16(da, vf[kt][ks], dp[u][kt]);
          }
        }
      }
      bf16x8 pp[2], pd[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        floatx4 P[2], dS[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float p = __builtin_amdgcn_exp2f(s[u][kt][e]);
            P[u][e] = p;
            dS[u][e] = p * dp[u][kt][e];
          }
        pp[kt] = pack16(P[0], P[1]);
        pd[kt] = pack16(dS[0], dS[1]);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 tv = frag16_tr(ld, dt, m, lane);
        const bf16x8 tq = frag16_tr(lq, dt, m, lane);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          dv[kt][dt] = mfma16(tv, pp[kt], dv[kt][dt]);
          dk[kt][dt] = mfma16(tq, pd[kt], dk[kt][dt]);
        }
      }
    }
    if (more) settle(cur ^ 1, (t + 1) * 64);
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + 16 * kt + (lane & 15);
    store16_T(g.dv, (long)b * g.dv.sb + hd * g.dv.sh, dv[kt], 1.f, key, g.nk, lane, kmasked[kt]);
    store16_T(g.dk, (long)b * g.dk.sb + hd * g.dk.sh, dk[kt], 0.69314718055994531f, key, g.nk, lane, kmasked[kt]);
  }
}

// ------------------------------------------------------------------ backward dQ
// Body of one dQ block (query block bx of head hd, batch b); lds = [buf][K / V] tiles, kbl = key bias of keys kb0..
template <int ABL, int NW, int NST = 2>
__device__ __forceinline__ void dq_body(const AttnArgs& g, int bx, int hd, int b, char (&lds)[NST][2][8192], float* kbl,
                                        float* red2) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5;
  const int q0 = bx * (32 * NW) + wid * 32;
  const int qrow = q0 + (lane & 31);
  const bf16_t* K = g.k.p + b * g.k.sb + hd * g.k.sh;
  const bf16_t* V = g.v.p + b * g.v.sb + hd * g.v.sh;

  bf16x8 qf[4], df[4];
  load_row_frags(qf, g.q.p + b * g.q.sb + hd * g.q.sh, g.q.sr, qrow, g.n, lane);
  load_row_frags(df, g.dO.p + b * g.dO.sb + hd * g.dO.sh, g.dO.sr, qrow, g.n, lane);
  const long lo = b * g.l_sb + hd * g.l_sh + qrow;
  // -LSE and -delta of the lane's query as the S^T / dP^T chains' initial accumulators
  const floatx16 nlse = splat16(qrow < g.n ? g.lse[lo] : -__builtin_huge_valf());
  const floatx16 ndel = splat16(qrow < g.n ? g.delta_in[lo] : 0.f);

  floatx16 dqT[2];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dqT[0][i] = 0.f; dqT[1][i] = 0.f; }

  const int nt = (g.nk + 63) / 64;
  const void* Ku = uniform_ptr(K);
  const void* Vu = uniform_ptr(V);
  fill_key_bias<NW>(kbl, g, b, tid);
  const uint32_t lb = lds_addr(&lds[0][0][0]);  // [buf][K / V] tiles of 8 KB
  const RowPlan<NW> pk = row_plan<NW>(g.k.sr, wid, lane), pv = row_plan<NW>(g.v.sr, wid, lane);
  // the lse / delta / q / dO register loads above retire here, visibly to hipcc's wait placement (as in dkdv_body)
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  dma_rows_at<NW>(lb, Ku, g.k.sr, 0, g.nk, pk, wid, lane);
  dma_rows_at<NW>(lb + 8192, Vu, g.v.sr, 0, g.nk, pv, wid, lane);
  if (NST == 3 && ABL != 1 && nt > 1) {  // tile 1 in flight while tile 0 is waited for (4 pieces per wave)
    dma_rows_at<NW>(lb + 16384, Ku, g.k.sr, 64, g.nk, pk, wid, lane);
    dma_rows_at<NW>(lb + 16384 + 8192, Vu, g.v.sr, 64, g.nk, pv, wid, lane);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int kv0 = t * 64;
    const int cur = NST == 2 ? (t & 1) : t % NST;
    const bool more = ABL != 1 && t + 1 < nt;
    const int ahead = NST == 2 ? 1 : 2;  // the tile this iteration DMAs
    if (ABL != 1 && t + ahead < nt) {
      const int nb = (t + ahead) % NST;
      dma_rows_at<NW>(lb + nb * 16384, Ku, g.k.sr, kv0 + 64 * ahead, g.nk, pk, wid, lane);
      dma_rows_at<NW>(lb + nb * 16384 + 8192, Vu, g.v.sr, kv0 + 64 * ahead, g.nk, pv, wid, lane);
    }
    // at the end of this tile: wait for tile t + 1 with tile t + 2 (if any) still in flight (3-stage ring)
    const bool younger = NST == 3 && ABL != 1 && t + 2 < nt;
    const char* lk = lds[cur][0];
    const char* lv = lds[cur][1];
    const bool dense = kv0 + 64 <= g.n_dense;
    if (ABL == 8 || ABL == 10) {
      // Explicitly ordered body: both key halves' S^T / dP^T chains back to back (the second half's row fragments
      // read under the first chain), then the first half's exp / dS while the second chain drains, the dQ
      // products of the first half, the second half's exp / dS, its dQ products -- so no exp waits on the
      // chain it follows and no MFMA waits on a just-issued LDS read.
      bf16x8 ka[4], va[4], pd[2][2];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) { ka[ks] = frag_rows(lk, 0, ks, lane); va[ks] = frag_rows(lv, 0, ks, lane); }
      floatx16 sc[2], dp[2];
      sc[0] = nlse; dp[0] = ndel;
      __builtin_amdgcn_sched_barrier(0);
      if (ABL != 10) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc[0] = mfma32(ka[ks], qf[ks], sc[0]);
        dp[0] = mfma32(va[ks], df[ks], dp[0]);
      }
      if (ABL != 10) __builtin_amdgcn_s_setprio(0);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) { ka[ks] = frag_rows(lk, 32, ks, lane); va[ks] = frag_rows(lv, 32, ks, lane); }
      __builtin_amdgcn_sched_barrier(0);
      sc[1] = nlse; dp[1] = ndel;
      if (ABL != 10) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        sc[1] = mfma32(ka[ks], qf[ks], sc[1]);
        dp[1] = mfma32(va[ks], df[ks], dp[1]);
      }
      if (ABL != 10) __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        if (!dense) {
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const floatx4 bias = *reinterpret_cast<const floatx4*>(&kbl[kv0 - g.kb0 + 32 * kb + 8 * g4 + 4 * h]);
#pragma unroll
            for (int e = 0; e < 4; ++e) sc[kb][4 * g4 + e] += bias[e];
          }
        }
        floatx16 d;
#pragma unroll
        for (int i = 0; i < 16; ++i) d[i] = __builtin_amdgcn_exp2f(sc[kb][i]) * dp[kb][i];
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) pd[kb][s2] = pack_acc(d, s2);
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 tk[2];
#pragma unroll
          for (int db = 0; db < 2; ++db) tk[db] = frag_tr(lk, db, 2 * kb + s2, lane);
          if (ABL != 10) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int db = 0; db < 2; ++db) dqT[db] = mfma32(tk[db], pd[kb][s2], dqT[db]);
          if (ABL != 10) __builtin_amdgcn_s_setprio(0);
        }
      }
      if (younger) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      continue;
    }
    floatx16 dS[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      floatx16 s = nlse, dp = ndel;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        s = mfma32(frag_rows(lk, 32 * kb, ks, lane), qf[ks], s);
        dp = mfma32(frag_rows(lv, 32 * kb, ks, lane), df[ks], dp);
      }
      if (!dense) {  // scalar branch: only the context / padding key tiles carry a bias
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const floatx4 bias = *reinterpret_cast<const floatx4*>(&kbl[kv0 - g.kb0 + 32 * kb + 8 * g4 + 4 * h]);
#pragma unroll
          for (int e = 0; e < 4; ++e) s[4 * g4 + e] += bias[e];
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) dS[kb][i] = __builtin_amdgcn_exp2f(s[i]) * dp[i];
    }
    if (ABL == 9) {
      // the transposed K fragments of step st + 1 are read before step st's two MFMAs (two register sets)
      bf16x8 tk[2][2], pd[2][2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) pd[kb][s2] = pack_acc(dS[kb], s2);
#pragma unroll
      for (int db = 0; db < 2; ++db) tk[0][db] = frag_tr(lk, db, 0, lane);
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        if (st + 1 < 4) {
#pragma unroll
          for (int db = 0; db < 2; ++db) tk[(st + 1) & 1][db] = frag_tr(lk, db, st + 1, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int db = 0; db < 2; ++db) dqT[db] = mfma32(tk[st & 1][db], pd[st >> 1][st & 1], dqT[db]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const bf16x8 pd = pack_acc(dS[kb], s2);
#pragma unroll
          for (int db = 0; db < 2; ++db)
            dqT[db] = mfma32(ABL == 2 ? frag_rows(lk, 32 * db, 2 * kb + s2, lane) : frag_tr(lk, db, 2 * kb + s2, lane), pd,
                             dqT[db]);
        }
    }
    if (younger) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    (void)more;
  }
  if (!g.qkn) {
    store_T(g.dq, (long)b * g.dq.sb + hd * g.dq.sh, dqT, g.scale, qrow, g.n, lane, false);
    return;
  }
  float wf[32], dwp[32];
  qkn_load_w(g.wq, lane, wf);
#pragma unroll
  for (int v = 0; v < 32; ++v) dwp[v] = 0.f;
  qkn_bwd_row(g, g.xq, g.dq, b, hd, dqT, g.scale, wf, qrow, g.n, lane, false, dwp);
  qkn_dw_partial<NW>(reinterpret_cast<float*>(&lds[0][0][0]), red2,
                     dwp, g.dwq + ((long)(b * g.H + hd) * ((g.n + 32 * NW - 1) / (32 * NW)) + bx) * g.dw_ld, tid);
}

// dQ body on the 16x16x32 MFMA (diagnostic A/B against dq_body, as dkdv16_body): 32 queries per wave as two query
// tiles qt on the lanes; per key tile and 32-key half m, S^T / dP^T as 2 x 2 accumulators (key tile u, query tile qt)
// started at -LSE / -delta of the lane's query, the key bias on the context / padding tiles, dS^T packed per query tile,
// dQ^T (head-dim tile dt x query tile qt) += K^T (frag16_tr) x dS^T. Without the fused QK-norm epilogue.
template <int NW>
__device__ __forceinline__ void dq16_body(const AttnArgs& g, int bx, int hd, int b, char (&lds)[2][2][8192], float* kbl) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, G = lane >> 4;
  const int q0 = bx * (32 * NW) + wid * 32;
  const bf16_t* K = g.k.p + b * g.k.sb + hd * g.k.sh;
  const bf16_t* V = g.v.p + b * g.v.sb + hd * g.v.sh;

  bf16x8 qf[2][2], df[2][2];
  float nlse[2], ndel[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qrow = q0 + 16 * qt + (lane & 15);
    load_row_frags16(qf[qt], g.q.p + b * g.q.sb + hd * g.q.sh, g.q.sr, qrow, g.n, lane);
    load_row_frags16(df[qt], g.dO.p + b * g.dO.sb + hd * g.dO.sh, g.dO.sr, qrow, g.n, lane);
    const long lo = b * g.l_sb + hd * g.l_sh + qrow;
    nlse[qt] = qrow < g.n ? g.lse[lo] : -__builtin_huge_valf();
    ndel[qt] = qrow < g.n ? g.delta_in[lo] : 0.f;
  }
  floatx4 dq[2][4];  // [qt][dt]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int e = 0; e < 4; ++e) dq[qt][dt][e] = 0.f;

  const int nt = (g.nk + 63) / 64;
  const void* Ku = uniform_ptr(K);
  const void* Vu = uniform_ptr(V);
  fill_key_bias<NW>(kbl, g, b, tid);
  const uint32_t lb = lds_addr(&lds[0][0][0]);
  const RowPlan<NW> pk = row_plan<NW, 1>(g.k.sr, wid, lane), pv = row_plan<NW, 1>(g.v.sr, wid, lane);
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): as in dq_body
  dma_rows_at<NW, 1>(lb, Ku, g.k.sr, 0, g.nk, pk, wid, lane);
  dma_rows_at<NW, 1>(lb + 8192, Vu, g.v.sr, 0, g.nk, pv, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < nt; ++t) {
    const int kv0 = t * 64;
    const int cur = t & 1;
    if (t + 1 < nt) {
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384, Ku, g.k.sr, kv0 + 64, g.nk, pk, wid, lane);
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384 + 8192, Vu, g.v.sr, kv0 + 64, g.nk, pv, wid, lane);
    }
    const char* lk = lds[cur][0];
    const char* lv = lds[cur][1];
    const bool dense = kv0 + 64 <= g.n_dense;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      floatx4 s[2][2], dp[2][2];  // [u][qt]: key rows 32m + 16u + 4G + e, query 16qt + (lane & 15)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int e = 0; e < 4; ++e) { s[u][qt][e] = nlse[qt]; dp[u][qt][e] = ndel[qt]; }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 ka = frag16_rows(lk, 32 * m + 16 * u, ks, lane);
          const bf16x8 va = frag16_rows(lv, 32 * m + 16 * u, ks, lane);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) {
            s[u][qt] = mfma16(ka, qf[qt][ks], s[u][qt]);
            dp[u][qt] = mfma16(va, df[qt][ks], dp[u][qt]);
          }
        }
        if (!dense) {  // scalar branch: only the context / padding key tiles carry a bias
          const floatx4 bias = *reinterpret_cast<const floatx4*>(&kbl[kv0 - g.kb0 + 32 * m + 16 * u + 4 * G]);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt)
#pragma unroll
            for (int e = 0; e < 4; ++e) s[u][qt][e] += bias[e];
        }
      }
      bf16x8 pd[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        floatx4 dS[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) dS[u][e] = __builtin_amdgcn_exp2f(s[u][qt][e]) * dp[u][qt][e];
        pd[qt] = pack16(dS[0], dS[1]);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 tk = frag16_tr(lk, dt, m, lane);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) dq[qt][dt] = mfma16(tk, pd[qt], dq[qt][dt]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
    store16_T(g.dq, (long)b * g.dq.sb + hd * g.dq.sh, dq[qt], g.scale, q0 + 16 * qt + (lane & 15), g.n, lane, false);
}

// The production backward as ONE launch over both block kinds: the dK/dV blocks first (the longer ones),
// then the dQ blocks. Each kind alone is 3,168 equal blocks at B=8 1024^2 on 512 block slots (2 per CU):
// 6.19 waves of work run as 7, twice. In one grid the dQ blocks start on the slots the dK/dV tail frees,
// so the pair runs in ~(work of both) / slots instead of two rounded-up launches.
// DKDV: the dK/dV body (8 = explicitly ordered, 0 = compiler-scheduled). ORDER 1 (diagnostic A/B): per (batch,
// head) its nkb dK/dV blocks then its nqb dQ blocks, heads in sequence (a head's Q / dO / K / V shared in time).
// The 16x16x32 bodies with NW waves per block (diagnostic A/B of NW = 8: 256 keys / queries per block, one block of
// 8 waves per CU -- the same 2 waves per SIMD -- so each staged Q / dO (K / V) tile serves twice the waves).
template <int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void attn_bwd16_kernel(AttnArgs g, int nkb, int nqb, int B) {
  __shared__ __attribute__((aligned(16))) char lds[2][2][8192];
  __shared__ __attribute__((aligned(16))) float lstat[2][2][64];
  extern __shared__ __attribute__((aligned(16))) float kbl[];
  int bid = blockIdx.x;
  const int nk_blocks = nkb * g.H * B;
  const bool kv = bid < nk_blocks;
  if (!kv) bid -= nk_blocks;
  if (g.xcd) bid = xcd_remap(bid, kv ? nk_blocks : nqb * g.H * B);
  const int bx = kv ? bid % nkb : bid % nqb;
  const int r = kv ? bid / nkb : bid / nqb;
  if (kv) dkdv16_body<NW, true>(g, bx, r % g.H, r / g.H, lds, lstat);
  else dq16_body<NW>(g, bx, r % g.H, r / g.H, lds, kbl);
}

template <int DQ, int DKDV = 8, int ORDER = 0, int NST = 2>
__global__ __launch_bounds__(256, 2) void attn_bwd_kernel(AttnArgs g, int nkb, int nqb, int B) {
  __shared__ __attribute__((aligned(16))) char lds[NST][2][8192];
  __shared__ __attribute__((aligned(16))) float lstat[NST][2][64];
  extern __shared__ __attribute__((aligned(16))) float kbl[];
#ifdef VPT_DIAG
  if (g.pm) {
    // Two blocks share each CU, one wave of each per SIMD, running the same program: partner waves that start together
    // stay in step (both in their exp / pack phase, then both in their MFMA phase). The wave in an odd slot of its SIMD
    // (HW_ID[3:0]) takes static priority (guide: two waves per SIMD, item 4) and / or starts its block late (item 9).
    const unsigned slot = __builtin_amdgcn_s_getreg((3 << 11) | 4) & 15u;  // hwreg(HW_REG_HW_ID, 0, 4)
    if (slot & 1u) {
      if (g.pm & 1) __builtin_amdgcn_s_setprio(1);
      if (g.pm & 2) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)(g.pm >> 2)) __builtin_amdgcn_s_sleep(1);
      }
    }
  }
#endif
  int bid = blockIdx.x;
  bool kv;
  int bx, r;
  if (ORDER == 1) {
    r = bid / (nkb + nqb);
    const int j = bid - r * (nkb + nqb);
    kv = j < nkb;
    bx = kv ? j : j - nkb;
  } else {
    const int nk_blocks = nkb * g.H * B;
    kv = bid < nk_blocks;
    if (!kv) bid -= nk_blocks;
    if (g.xcd) bid = xcd_remap(bid, kv ? nk_blocks : nqb * g.H * B);
    bx = kv ? bid % nkb : bid % nqb;
    r = kv ? bid / nkb : bid / nqb;
  }
  static_assert((DKDV < 16 && DQ != 16) || NST == 2, "16x16x32 bodies: two-stage ring");
  if (kv) {
    if constexpr (DKDV == 16 || DKDV == 17) dkdv16_body<4, DKDV == 17>(g, bx, r % g.H, r / g.H, lds, lstat);
    else dkdv_body<DKDV, 4, NST>(g, bx, r % g.H, r / g.H, lds, lstat);
  } else {
    if constexpr (DQ == 16) dq16_body<4>(g, bx, r % g.H, r / g.H, lds, kbl);
    else dq_body<DQ, 4, NST>(g, bx, r % g.H, r / g.H, lds, kbl, &lstat[0][0][0]);
  }
}
// ------------------------------------------------------------------ backward, persistent work queue
// The same dK/dV and dQ items as attn_bwd_kernel<16, 17> (16x16x32 bodies, the dK/dV body explicitly ordered: the same
// products in the same order, so the results are bitwise those of the one-launch grid), run by a resident grid (two
// blocks per CU) that pulls items from per-XCD queues instead of one block per item:
//  - queue x holds the items xcd_remap deals to XCD x (a contiguous range of dK/dV items, then one of dQ items), so a
//    (batch, head)'s Q / dO (or K / V) stays in that XCD's L2 as before; a block reads its XCD from HW_REG_XCC_ID and
//    pulls from its own queue with one returning atomic add per item (in the item's prologue, beside the fragment
//    loads), taking from the other XCDs' queues only once its own is empty -- a dynamic fill, unlike the static
//    persistent walk (r05zzi: +3.0 % at C3, +4.5 % at C2: the tail lost the dispatcher's fill);
//  - the next item's first K / V (or Q / dO + LSE / delta) tile is DMA'd into the free LDS buffer during the current
//    item's last tile, so an item starts on staged data; the key-bias array is refilled only when the batch changes;
//    the per-block launch, first-tile round trip and retirement of the one-launch grid are gone.
// Queue words (caller's workspace, zero before the first launch): [0, 8) per-XCD tickets, [8] finished blocks. The block
// that finishes last resets them, so the next launch on the same workspace starts from zero (stream order). Every
// block ends once all queues are drained: no block ever waits for another.
constexpr int kPqWords = 16;
__device__ __forceinline__ int xcc_id() { return (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u); }

struct PqGeom {
  int nkb, nqb, nkv, nq;  // blocks per head (dK/dV, dQ), items of each kind
  __device__ __forceinline__ int kv_lo(int x) const { return x * (nkv >> 3) + min(x, nkv & 7); }
  __device__ __forceinline__ int q_lo(int x) const { return x * (nq >> 3) + min(x, nq & 7); }
  __device__ __forceinline__ int kv_len(int x) const { return (nkv >> 3) + (x < (nkv & 7)); }
  __device__ __forceinline__ int q_len(int x) const { return (nq >> 3) + (x < (nq & 7)); }
  // ticket t of queue x -> item id: [0, nkv) dK/dV logical ids, [nkv, nkv + nq) dQ logical ids + nkv; -1 past the end
  __device__ __forceinline__ int item(int x, unsigned t) const {
    const int lk = kv_len(x);
    if (t < (unsigned)lk) return kv_lo(x) + (int)t;
    if (t < (unsigned)(lk + q_len(x))) return nkv + q_lo(x) + ((int)t - lk);
    return -1;
  }
};

// One item from the block's own queue, else from the others in turn (-1: all drained). One lane.
__device__ __forceinline__ int pq_pull(unsigned* qws, const PqGeom& q, int x) {
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    const int xq = (x + i) & 7;
    const int it = q.item(xq, atomicAdd(qws + xq, 1u));
    if (it >= 0) return it;
  }
  return -1;
}

// Tile 0 of item `it` into LDS buffer `buf` (dK/dV: Q / dO rows and the LSE / delta rows; dQ: K / V rows).
// threadIdx.x hidden from the optimiser per call: the lane-dependent DMA offsets and fragment addresses of an item are
// then recomputed in each item instead of being hoisted out of the item loop, kept live across every item (spilled)
__device__ __forceinline__ int pq_opaque_tid() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

template <int NW>
__device__ __forceinline__ void pq_stage0(const AttnArgs& g, const PqGeom& q, int it, uint32_t lb, int buf,
                                          float (&lstat)[2][2][64], int wid, int lane) {
  lane = pq_opaque_tid() & 63;
  const bool kv = it < q.nkv;
  const int id = kv ? it : it - q.nkv;
  const int r = kv ? id / q.nkb : id / q.nqb, hd = r % g.H, b = r / g.H;
  if (kv) {
    dma_rows_at<NW, 1>(lb + buf * 16384, uniform_ptr(g.q.p + b * g.q.sb + hd * g.q.sh), g.q.sr, 0, g.n,
                       row_plan<NW, 1>(g.q.sr, wid, lane), wid, lane);
    dma_rows_at<NW, 1>(lb + buf * 16384 + 8192, uniform_ptr(g.dO.p + b * g.dO.sb + hd * g.dO.sh), g.dO.sr, 0, g.n,
                       row_plan<NW, 1>(g.dO.sr, wid, lane), wid, lane);
    if (wid == 0) dma_stat(lstat[buf][0], uniform_ptr(g.lse + b * g.l_sb + hd * g.l_sh), 0, g.n, lane);
    else if (wid == 1) dma_stat(lstat[buf][1], uniform_ptr(g.delta_in + b * g.l_sb + hd * g.l_sh), 0, g.n, lane);
  } else {
    dma_rows_at<NW, 1>(lb + buf * 16384, uniform_ptr(g.k.p + b * g.k.sb + hd * g.k.sh), g.k.sr, 0, g.nk,
                       row_plan<NW, 1>(g.k.sr, wid, lane), wid, lane);
    dma_rows_at<NW, 1>(lb + buf * 16384 + 8192, uniform_ptr(g.v.p + b * g.v.sb + hd * g.v.sh), g.v.sr, 0, g.nk,
                       row_plan<NW, 1>(g.v.sr, wid, lane), wid, lane);
  }
}

// Prologue shared by both item kinds, after the item's fragment loads were issued: every wave waits for its loads and
// tile-0 pieces; lane 0 publishes the next item into `slot` -- its ticket `pend` was taken one item earlier, so the
// atomic's round trip ran under that item (own queue drained: the others are tried in turn, at the tail only) -- and
// then takes the ticket after it, which returns while this item runs (only an explicit vmcnt(0) later waits for it,
// at this item's first tile). The barrier publishes the slot. Returns the next item (-1: none).
__device__ __forceinline__ int pq_prologue(unsigned* qws, const PqGeom& q, int x, volatile int* slot, unsigned& pend) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    int it = q.item(x, pend);
    if (it < 0) it = pq_pull(qws, q, x);
    *slot = it;
    pend = atomicAdd(qws + x, 1u);
  }
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*slot);  // the same in every lane: uniform for the compiler too
}

// dkdv16_body<NW, true> as a queue item: tile 0 staged (possibly still in flight) in buffer p0; the next item's tile 0
// is staged into the free buffer during this item's last tile. Returns the buffer of the next tile 0; *next = item.
template <int NW>
__device__ __forceinline__ int pq_dkdv(const AttnArgs& g, const PqGeom& q, int bx, int hd, int b, int p0,
                                       char (&lds)[2][2][8192], float (&lstat)[2][2][64], unsigned* qws, int x,
                                       volatile int* slot, unsigned& pend, int& next) {
  const int tid = pq_opaque_tid(), lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), G = lane >> 4;
  const int k0 = bx * (32 * NW) + wid * 32;
  bf16x8 kf[2][2], vf[2][2];
  bool kmasked[2];
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + 16 * kt + (lane & 15);
    load_row_frags16(kf[kt], g.k.p + b * g.k.sb + hd * g.k.sh, g.k.sr, key, g.nk, lane);
    load_row_frags16(vf[kt], g.v.p + b * g.v.sb + hd * g.v.sh, g.v.sr, key, g.nk, lane);
    kmasked[kt] = key_bias(g, b, key) == kNegInf;
  }
  const int nxt = pq_prologue(qws, q, x, slot, pend);
  next = nxt;
  if (g.n < 64) {  // padding query rows of the (only) tile zeroed
    zero_rows<NW>(lds[p0][0], g.n, tid);
    zero_rows<NW>(lds[p0][1], g.n, tid);
    __syncthreads();
  }
  floatx4 dv[2][4], dk[2][4];  // [kt][dt]
#pragma unroll
  for (int kt = 0; kt < 2; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int e = 0; e < 4; ++e) { dv[kt][dt][e] = 0.f; dk[kt][dt][e] = 0.f; }
  const int nt = (g.n + 63) / 64;
  const void* Qu = uniform_ptr(g.q.p + b * g.q.sb + hd * g.q.sh);
  const void* Du = uniform_ptr(g.dO.p + b * g.dO.sb + hd * g.dO.sh);
  const void* Lu = uniform_ptr(g.lse + b * g.l_sb + hd * g.l_sh);
  const void* Eu = uniform_ptr(g.delta_in + b * g.l_sb + hd * g.l_sh);
  const uint32_t lb = lds_addr(&lds[0][0][0]);
  const RowPlan<NW> pq = row_plan<NW, 1>(g.q.sr, wid, lane), pd0 = row_plan<NW, 1>(g.dO.sr, wid, lane);
  for (int t = 0; t < nt; ++t) {
    const int cur = (t + p0) & 1;
    const bool more = t + 1 < nt;
    if (more) {
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384, Qu, g.q.sr, (t + 1) * 64, g.n, pq, wid, lane);
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384 + 8192, Du, g.dO.sr, (t + 1) * 64, g.n, pd0, wid, lane);
      if (wid == 0) dma_stat(lstat[cur ^ 1][0], Lu, (t + 1) * 64, g.n, lane);
      else if (wid == 1) dma_stat(lstat[cur ^ 1][1], Eu, (t + 1) * 64, g.n, lane);
    } else if (nxt >= 0) {
      pq_stage0<NW>(g, q, nxt, lb, cur ^ 1, lstat, wid, lane);
    }
    const char* lq = lds[cur][0];
    const char* ld = lds[cur][1];
    bf16x8 qa[2][2], da[2][2], pp[2][2], pd[2][2];  // qa / da [u][ks]; pp / pd [m][kt]
    auto rd = [&](int m) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          qa[u][ks] = frag16_rows(lq, 32 * m + 16 * u, ks, lane);
          da[u][ks] = frag16_rows(ld, 32 * m + 16 * u, ks, lane);
        }
    };
    rd(0);
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      floatx4 s[2][2], dp[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const floatx4 cs = *reinterpret_cast<const floatx4*>(&lstat[cur][0][32 * m + 16 * u + 4 * G]);
        const floatx4 cd = *reinterpret_cast<const floatx4*>(&lstat[cur][1][32 * m + 16 * u + 4 * G]);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) { s[u][kt] = cs; dp[u][kt] = cd; }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) {
            s[u][kt] = mfma16(qa[u][ks], kf[kt][ks], s[u][kt]);
            dp[u][kt] = mfma16(da[u][ks], vf[kt][ks], dp[u][kt]);
          }
      if (m == 0) rd(1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        floatx4 P[2], dS[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float p = __builtin_amdgcn_exp2f(s[u][kt][e]);
            P[u][e] = p;
            dS[u][e] = p * dp[u][kt][e];
          }
        pp[m][kt] = pack16(P[0], P[1]);
        pd[m][kt] = pack16(dS[0], dS[1]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 tv = frag16_tr(ld, dt, m, lane);
        const bf16x8 tq = frag16_tr(lq, dt, m, lane);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          dv[kt][dt] = mfma16(tv, pp[m][kt], dv[kt][dt]);
          dk[kt][dt] = mfma16(tq, pd[m][kt], dk[kt][dt]);
        }
      }
    if (more) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      const int r1 = (t + 1) * 64;
      if (g.n - r1 < 64) {  // padding query rows zeroed: no dK / dV contribution
        zero_rows<NW>(lds[cur ^ 1][0], g.n - r1, tid);
        zero_rows<NW>(lds[cur ^ 1][1], g.n - r1, tid);
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    const int key = k0 + 16 * kt + (lane & 15);
    store16_T(g.dv, (long)b * g.dv.sb + hd * g.dv.sh, dv[kt], 1.f, key, g.nk, lane, kmasked[kt]);
    store16_T(g.dk, (long)b * g.dk.sb + hd * g.dk.sh, dk[kt], 0.69314718055994531f, key, g.nk, lane, kmasked[kt]);
  }
  return (nt + p0) & 1;
}

// dq16_body<NW> as a queue item (see pq_dkdv); kbl_b = the batch whose key biases kbl holds (-1: none yet).
template <int NW>
__device__ __forceinline__ int pq_dq(const AttnArgs& g, const PqGeom& q, int bx, int hd, int b, int p0,
                                     char (&lds)[2][2][8192], float (&lstat)[2][2][64], float* kbl, int& kbl_b,
                                     unsigned* qws, int x, volatile int* slot, unsigned& pend, int& next) {
  const int tid = pq_opaque_tid(), lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), G = lane >> 4;
  const int q0 = bx * (32 * NW) + wid * 32;
  bf16x8 qf[2][2], df[2][2];
  float nlse[2], ndel[2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int qrow = q0 + 16 * qt + (lane & 15);
    load_row_frags16(qf[qt], g.q.p + b * g.q.sb + hd * g.q.sh, g.q.sr, qrow, g.n, lane);
    load_row_frags16(df[qt], g.dO.p + b * g.dO.sb + hd * g.dO.sh, g.dO.sr, qrow, g.n, lane);
    const long lo = b * g.l_sb + hd * g.l_sh + qrow;
    nlse[qt] = qrow < g.n ? g.lse[lo] : -__builtin_huge_valf();
    ndel[qt] = qrow < g.n ? g.delta_in[lo] : 0.f;
  }
  if (b != kbl_b) {  // the previous item's last reads of kbl were before its last barrier
    fill_key_bias<NW>(kbl, g, b, tid);
    kbl_b = b;
  }
  const int nxt = pq_prologue(qws, q, x, slot, pend);
  next = nxt;
  floatx4 dq[2][4];  // [qt][dt]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int e = 0; e < 4; ++e) dq[qt][dt][e] = 0.f;
  const int nt = (g.nk + 63) / 64;
  const void* Ku = uniform_ptr(g.k.p + b * g.k.sb + hd * g.k.sh);
  const void* Vu = uniform_ptr(g.v.p + b * g.v.sb + hd * g.v.sh);
  const uint32_t lb = lds_addr(&lds[0][0][0]);
  const RowPlan<NW> pk = row_plan<NW, 1>(g.k.sr, wid, lane), pv = row_plan<NW, 1>(g.v.sr, wid, lane);
  for (int t = 0; t < nt; ++t) {
    const int kv0 = t * 64;
    const int cur = (t + p0) & 1;
    if (t + 1 < nt) {
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384, Ku, g.k.sr, kv0 + 64, g.nk, pk, wid, lane);
      dma_rows_at<NW, 1>(lb + (cur ^ 1) * 16384 + 8192, Vu, g.v.sr, kv0 + 64, g.nk, pv, wid, lane);
    } else if (nxt >= 0) {
      pq_stage0<NW>(g, q, nxt, lb, cur ^ 1, lstat, wid, lane);
    }
    const char* lk = lds[cur][0];
    const char* lv = lds[cur][1];
    const bool dense = kv0 + 64 <= g.n_dense;
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      floatx4 s[2][2], dp[2][2];  // [u][qt]: key rows 32m + 16u + 4G + e, query 16qt + (lane & 15)
#pragma unroll
      for (int u = 0; u < 2; ++u) {
#pragma unroll
        for (int qt = 0; qt < 2; ++qt)
#pragma unroll
          for (int e = 0; e < 4; ++e) { s[u][qt][e] = nlse[qt]; dp[u][qt][e] = ndel[qt]; }
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 ka = frag16_rows(lk, 32 * m + 16 * u, ks, lane);
          const bf16x8 va = frag16_rows(lv, 32 * m + 16 * u, ks, lane);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt) {
            s[u][qt] = mfma16(ka, qf[qt][ks], s[u][qt]);
            dp[u][qt] = mfma16(va, df[qt][ks], dp[u][qt]);
          }
        }
        if (!dense) {  // scalar branch: only the context / padding key tiles carry a bias
          const floatx4 bias = *reinterpret_cast<const floatx4*>(&kbl[kv0 - g.kb0 + 32 * m + 16 * u + 4 * G]);
#pragma unroll
          for (int qt = 0; qt < 2; ++qt)
#pragma unroll
            for (int e = 0; e < 4; ++e) s[u][qt][e] += bias[e];
        }
      }
      bf16x8 pd[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        floatx4 dS[2];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) dS[u][e] = __builtin_amdgcn_exp2f(s[u][qt][e]) * dp[u][qt][e];
        pd[qt] = pack16(dS[0], dS[1]);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const bf16x8 tk = frag16_tr(lk, dt, m, lane);
#pragma unroll
        for (int qt = 0; qt < 2; ++qt) dq[qt][dt] = mfma16(tk, pd[qt], dq[qt][dt]);
      }
    }
    if (t + 1 < nt) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
#pragma unroll
  for (int qt = 0; qt < 2; ++qt)
    store16_T(g.dq, (long)b * g.dq.sb + hd * g.dq.sh, dq[qt], g.scale, q0 + 16 * qt + (lane & 15), g.n, lane, false);
  return (nt + p0) & 1;
}

__global__ __launch_bounds__(256, 2) void attn_bwd_pq_kernel(AttnArgs g, int nkb, int nqb, int B, unsigned* qws) {
  constexpr int NW = 4;
  __shared__ __attribute__((aligned(16))) char lds[2][2][8192];
  __shared__ __attribute__((aligned(16))) float lstat[2][2][64];
  __shared__ int s_item[2];
  extern __shared__ __attribute__((aligned(16))) float kbl[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  PqGeom q;
  q.nkb = nkb;
  q.nqb = nqb;
  q.nkv = nkb * g.H * B;
  q.nq = nqb * g.H * B;
  const int x = xcc_id();
  volatile int* slots = s_item;
  unsigned pend = 0;  // lane 0: the ticket of the item after the current one (pq_prologue)
  if (tid == 0) {
    slots[0] = pq_pull(qws, q, x);
    pend = atomicAdd(qws + x, 1u);
  }
  __syncthreads();
  int it = __builtin_amdgcn_readfirstlane(slots[0]);
  int buf = 0, kbl_b = -1;
  if (it >= 0) pq_stage0<NW>(g, q, it, lds_addr(&lds[0][0][0]), 0, lstat, wid, lane);
  // item n's prologue writes slot (n + 1) & 1 (a wave can reach the next item's prologue before a slower wave has
  // passed this one's barrier, never two items ahead: every item has a barrier)
  for (int n = 0; it >= 0; ++n) {
    const bool kv = it < q.nkv;
    const int id = kv ? it : it - q.nkv;
    const int r = kv ? id / nkb : id / nqb;
    const int bx = kv ? id - r * nkb : id - r * nqb;
    int next;
    if (kv) buf = pq_dkdv<NW>(g, q, bx, r % g.H, r / g.H, buf, lds, lstat, qws, x, slots + ((n + 1) & 1), pend, next);
    else buf = pq_dq<NW>(g, q, bx, r % g.H, r / g.H, buf, lds, lstat, kbl, kbl_b, qws, x, slots + ((n + 1) & 1), pend,
                         next);
    it = next;
  }
  // queue reset by the block that finishes last (every block has taken its last, failing tickets before it counts)
  if (tid == 0 && atomicAdd(qws + 8, 1u) == gridDim.x - 1) {
#pragma unroll
    for (int i = 0; i < 9; ++i) atomicExch(qws + i, 0u);
  }
}

constexpr int kDqBody = 0;  // production dQ body (0 = compiler-scheduled, 8 = explicitly ordered)
// production dK/dV body: the explicitly ordered body without s_setprio around its MFMA groups (10); with them (8) the
// other wave on the SIMD waits out each prioritised MFMA group before its exp / pack phase can issue: kernel -1.1 %,
// +0.18 % per C3 step without (same-box A/B r04zg, bitwise equal)
constexpr int kDkdvBody = 10;
// Production backward (without the fused QK-norm epilogue): the 16x16x32 bodies, dK/dV explicitly ordered (mask 7 of
// vpt_attn_set_bwd_mfma16). Same products, LDS bytes and VALU as the 32x32x16 pair; the chip holds a higher clock on
// the smaller MFMA shape under this load (guide MI355X_MICROARCH 'DVFS give-back' item 7): backward -4.6 % (both
// compiler-scheduled) / -6.3 % (ordered dK/dV), C3 step +1.7 % (r05p, r05q).
constexpr int kBwdMf16 = 7;

// Dynamic LDS of the key-bias array (fill_key_bias); n <= 32768 keeps it within 128 KB.
size_t key_bias_lds_bytes(const AttnArgs& g) { return (size_t)((g.nk + 63) / 64 * 64 - g.kb0) * sizeof(float); }

int check_common(int B, int H, int n, int nk) {
  VPT_CHECK_ARG(B > 0 && H > 0 && n > 0 && nk > 0, "attention: empty shape");
  VPT_CHECK_ARG(nk <= 32768, "attention: nk <= 32768 (key-bias LDS array)");
  return VPT_OK;
}

#ifdef VPT_DIAG
#include "diag/attention_diag_kernels.inc"
#endif

}  // namespace

// The factor the caller applies to q before vpt_attn_fwd / vpt_attn_bwd.
extern "C" float vpt_attn_q_scale(float scale) { return scale * 1.4426950408889634f; }

// Strides are in elements; every tensor is addressed as p[b*sb + h*sh + row*sr + d], d in [0,64).
extern "C" int vpt_attn_fwd(const void* q, long q_sb, long q_sh, long q_sr,
                            const void* k, long k_sb, long k_sh, long k_sr,
                            const void* v, long v_sb, long v_sh, long v_sr,
                            void* o, long o_sb, long o_sh, long o_sr,
                            float* lse, long l_sb, long l_sh,
                            const float* kbias, long kb_sb,
                            int B, int H, int n, int nk, int n_dense, float scale, void* stream) {
  int rc = check_common(B, H, n, nk);
  if (rc) return rc;
  VPT_CHECK_ARG(q && k && v && o && lse, "vpt_attn_fwd: null pointer");
  AttnArgs g = {};
  g.xcd = g_xcd;
  g.q = {(const bf16_t*)q, q_sb, q_sh, q_sr};
  g.k = {(const bf16_t*)k, k_sb, k_sh, k_sr};
  g.v = {(const bf16_t*)v, v_sb, v_sh, v_sr};
  g.o = {(bf16_t*)o, o_sb, o_sh, o_sr};
  g.lse = lse; g.l_sb = l_sb; g.l_sh = l_sh;
  g.kbias = kbias; g.kb_sb = kb_sb;
  g.n = n; g.nk = nk; g.n_dense = n_dense < nk ? n_dense : nk;
  g.scale = scale; g.scale_log2 = scale * 1.4426950408889634f;
  g.tau = g_tau;
  g.kb0 = g.n_dense / 64 * 64;
  if (g_waves != 8 && g_fwd_ord)
    hipLaunchKernelGGL((attn_fwd_kernel<4, false, true>), dim3((n + 127) / 128, H, B), dim3(256), key_bias_lds_bytes(g),
                       (hipStream_t)stream, g);
  else if (g_waves != 8)
    hipLaunchKernelGGL((attn_fwd_kernel<4>), dim3((n + 127) / 128, H, B), dim3(256), key_bias_lds_bytes(g),
                       (hipStream_t)stream, g);
  else
    hipLaunchKernelGGL(attn_fwd_kernel<8>, dim3((n + 255) / 256, H, B), dim3(512), key_bias_lds_bytes(g),
                       (hipStream_t)stream, g);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

// vpt_attn_fwd for QK-RMSNormed q / k (JiT self-attention: q, k = rope(rms(x) w), q pre-scaled): the same results,
// computed with a fixed softmax reference point (the Cauchy-Schwarz bound of the scores from the q_norm / k_norm
// weights wq, wk [64]) while that bound is below kFixMax -- no running row maximum in the loop; larger weights take
// the online-maximum path.
extern "C" int vpt_attn_fwd_qknorm(const void* q, long q_sb, long q_sh, long q_sr,
                                   const void* k, long k_sb, long k_sh, long k_sr,
                                   const void* v, long v_sb, long v_sh, long v_sr,
                                   void* o, long o_sb, long o_sh, long o_sr,
                                   float* lse, long l_sb, long l_sh,
                                   const float* kbias, long kb_sb, const void* wq, const void* wk,
                                   int B, int H, int n, int nk, int n_dense, float scale, void* stream) {
  int rc = check_common(B, H, n, nk);
  if (rc) return rc;
  VPT_CHECK_ARG(q && k && v && o && lse && wq && wk, "vpt_attn_fwd_qknorm: null pointer");
  AttnArgs g = {};
  g.xcd = g_xcd;
  g.q = {(const bf16_t*)q, q_sb, q_sh, q_sr};
  g.k = {(const bf16_t*)k, k_sb, k_sh, k_sr};
  g.v = {(const bf16_t*)v, v_sb, v_sh, v_sr};
  g.o = {(bf16_t*)o, o_sb, o_sh, o_sr};
  g.lse = lse; g.l_sb = l_sb; g.l_sh = l_sh;
  g.kbias = kbias; g.kb_sb = kb_sb;
  g.n = n; g.nk = nk; g.n_dense = n_dense < nk ? n_dense : nk;
  g.scale = scale; g.scale_log2 = scale * 1.4426950408889634f;
  g.tau = g_tau;
  g.kb0 = g.n_dense / 64 * 64;
  g.wq = (const bf16_t*)wq; g.wk = (const bf16_t*)wk;
#ifdef VPT_DIAG
  if (g_fwd16) {
    hipLaunchKernelGGL((attn_fwd_kernel<4, true, true, false, true>), dim3((n + 127) / 128, H, B), dim3(256),
                       key_bias_lds_bytes(g), (hipStream_t)stream, g);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
#endif
  if (g_fwd_ord && g_fwd_lsm)
    hipLaunchKernelGGL((attn_fwd_kernel<4, true, true, true>), dim3((n + 127) / 128, H, B), dim3(256),
                       key_bias_lds_bytes(g), (hipStream_t)stream, g);
  else if (g_fwd_ord)
    hipLaunchKernelGGL((attn_fwd_kernel<4, true, true>), dim3((n + 127) / 128, H, B), dim3(256), key_bias_lds_bytes(g),
                       (hipStream_t)stream, g);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<4, true>), dim3((n + 127) / 128, H, B), dim3(256), key_bias_lds_bytes(g),
                       (hipStream_t)stream, g);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}


namespace {
int attn_bwd_impl(AttnArgs& g, int B, int H, int n, int nk, hipStream_t s);
int attn_bwd_pq_impl(AttnArgs& g, int B, int H, int n, int nk, unsigned* qws, hipStream_t s);
}

extern "C" int vpt_attn_bwd(const void* q, long q_sb, long q_sh, long q_sr,
                            const void* k, long k_sb, long k_sh, long k_sr,
                            const void* v, long v_sb, long v_sh, long v_sr,
                            const void* o, long o_sb, long o_sh, long o_sr,
                            const void* dO, long do_sb, long do_sh, long do_sr,
                            const float* lse, float* delta, long l_sb, long l_sh,
                            const float* kbias, long kb_sb,
                            void* dq, long dq_sb, long dq_sh, long dq_sr,
                            void* dk, long dk_sb, long dk_sh, long dk_sr,
                            void* dv, long dv_sb, long dv_sh, long dv_sr,
                            int B, int H, int n, int nk, int n_dense, float scale, void* stream) {
  int rc = check_common(B, H, n, nk);
  if (rc) return rc;
  VPT_CHECK_ARG(q && k && v && o && dO && lse && delta && dq && dk && dv, "vpt_attn_bwd: null pointer");
  AttnArgs g = {};
  g.xcd = g_xcd;
  g.q = {(const bf16_t*)q, q_sb, q_sh, q_sr};
  g.k = {(const bf16_t*)k, k_sb, k_sh, k_sr};
  g.v = {(const bf16_t*)v, v_sb, v_sh, v_sr};
  g.o = {(bf16_t*)o, o_sb, o_sh, o_sr};
  g.dO = {(const bf16_t*)dO, do_sb, do_sh, do_sr};
  g.dq = {(bf16_t*)dq, dq_sb, dq_sh, dq_sr};
  g.dk = {(bf16_t*)dk, dk_sb, dk_sh, dk_sr};
  g.dv = {(bf16_t*)dv, dv_sb, dv_sh, dv_sr};
  g.lse = (float*)lse; g.delta_in = delta; g.delta_out = delta; g.l_sb = l_sb; g.l_sh = l_sh;
  g.kbias = kbias; g.kb_sb = kb_sb;
  g.n = n; g.nk = nk; g.n_dense = n_dense < nk ? n_dense : nk;
  g.scale = scale; g.scale_log2 = scale * 1.4426950408889634f;
  g.kb0 = g.n_dense / 64 * 64;
  g.nq_pad = (n + 63) / 64 * 64;
  g.H = H;
#ifdef VPT_DIAG
  g.pm = g_pm;
#endif
  return attn_bwd_impl(g, B, H, n, nk, (hipStream_t)stream);
}

// vpt_attn_bwd on the persistent work-queue kernel (bitwise the same results): `queue` = 64 bytes of device memory owned
// by the caller, zero before its first use and left zero by every launch; one per stream that may run this concurrently.
extern "C" int vpt_attn_bwd_q(const void* q, long q_sb, long q_sh, long q_sr,
                              const void* k, long k_sb, long k_sh, long k_sr,
                              const void* v, long v_sb, long v_sh, long v_sr,
                              const void* o, long o_sb, long o_sh, long o_sr,
                              const void* dO, long do_sb, long do_sh, long do_sr,
                              const float* lse, float* delta, long l_sb, long l_sh,
                              const float* kbias, long kb_sb,
                              void* dq, long dq_sb, long dq_sh, long dq_sr,
                              void* dk, long dk_sb, long dk_sh, long dk_sr,
                              void* dv, long dv_sb, long dv_sh, long dv_sr,
                              int B, int H, int n, int nk, int n_dense, float scale, void* queue, void* stream) {
  int rc = check_common(B, H, n, nk);
  if (rc) return rc;
  VPT_CHECK_ARG(q && k && v && o && dO && lse && delta && dq && dk && dv && queue, "vpt_attn_bwd_q: null pointer");
  VPT_CHECK_ARG(((uintptr_t)queue & 63) == 0, "vpt_attn_bwd_q: queue must be 64-byte aligned");
  AttnArgs g = {};
  g.xcd = 1;
  g.q = {(const bf16_t*)q, q_sb, q_sh, q_sr};
  g.k = {(const bf16_t*)k, k_sb, k_sh, k_sr};
  g.v = {(const bf16_t*)v, v_sb, v_sh, v_sr};
  g.o = {(bf16_t*)o, o_sb, o_sh, o_sr};
  g.dO = {(const bf16_t*)dO, do_sb, do_sh, do_sr};
  g.dq = {(bf16_t*)dq, dq_sb, dq_sh, dq_sr};
  g.dk = {(bf16_t*)dk, dk_sb, dk_sh, dk_sr};
  g.dv = {(bf16_t*)dv, dv_sb, dv_sh, dv_sr};
  g.lse = (float*)lse; g.delta_in = delta; g.delta_out = delta; g.l_sb = l_sb; g.l_sh = l_sh;
  g.kbias = kbias; g.kb_sb = kb_sb;
  g.n = n; g.nk = nk; g.n_dense = n_dense < nk ? n_dense : nk;
  g.scale = scale; g.scale_log2 = scale * 1.4426950408889634f;
  g.kb0 = g.n_dense / 64 * 64;
  g.nq_pad = (n + 63) / 64 * 64;
  g.H = H;
  return attn_bwd_pq_impl(g, B, H, n, nk, (unsigned*)queue, (hipStream_t)stream);
}

extern "C" int vpt_attn_bwd_queue_bytes(void) { return kPqWords * 4; }

// Rows of the per-workgroup weight-gradient partials vpt_attn_bwd_qknorm writes for n rows (q: n = query rows,
// k: n = key rows): one 64-float row per 128-row block of every (batch, head).
extern "C" int vpt_attn_bwd_dw_rows(int B, int H, int n) { return B * H * ((n + 127) / 128); }

extern "C" int vpt_attn_bwd_qknorm(const void* q, long q_sb, long q_sh, long q_sr,
                                   const void* k, long k_sb, long k_sh, long k_sr,
                                   const void* v, long v_sb, long v_sh, long v_sr,
                                   const void* o, long o_sb, long o_sh, long o_sr,
                                   const void* dO, long do_sb, long do_sh, long do_sr,
                                   const float* lse, float* delta, long l_sb, long l_sh,
                                   const float* kbias, long kb_sb,
                                   const void* xq, const void* xk, long x_sb, long x_sh, long x_sr,
                                   const void* wq, const void* wk, const float* cos_t, const float* sin_t, float eps,
                                   void* dq, void* dk, long dqk_sb, long dqk_sh, long dqk_sr, float* dwq_part,
                                   float* dwk_part, long dw_ld, void* dv, long dv_sb, long dv_sh, long dv_sr,
                                   int B, int H, int n, int nk, int n_dense, float scale, void* stream) {
  int rc = check_common(B, H, n, nk);
  if (rc) return rc;
  VPT_CHECK_ARG(q && k && v && o && dO && lse && delta && dq && dk && dv, "vpt_attn_bwd_qknorm: null pointer");
  VPT_CHECK_ARG(xq && xk && wq && wk && cos_t && sin_t && dwq_part && dwk_part, "vpt_attn_bwd_qknorm: null pointer");
  VPT_CHECK_ARG(n == nk, "vpt_attn_bwd_qknorm: self-attention only (the RoPE position of a key is its row)");
  VPT_CHECK_ARG(x_sr % 4 == 0 && dqk_sr % 4 == 0 && x_sh % 4 == 0 && dqk_sh % 4 == 0 && x_sb % 4 == 0 &&
                dqk_sb % 4 == 0, "vpt_attn_bwd_qknorm: 8-byte aligned row pieces");
  AttnArgs g = {};
  g.xcd = g_xcd;
  g.q = {(const bf16_t*)q, q_sb, q_sh, q_sr};
  g.k = {(const bf16_t*)k, k_sb, k_sh, k_sr};
  g.v = {(const bf16_t*)v, v_sb, v_sh, v_sr};
  g.o = {(bf16_t*)o, o_sb, o_sh, o_sr};
  g.dO = {(const bf16_t*)dO, do_sb, do_sh, do_sr};
  g.dq = {(bf16_t*)dq, dqk_sb, dqk_sh, dqk_sr};
  g.dk = {(bf16_t*)dk, dqk_sb, dqk_sh, dqk_sr};
  g.dv = {(bf16_t*)dv, dv_sb, dv_sh, dv_sr};
  g.lse = (float*)lse; g.delta_in = delta; g.delta_out = delta; g.l_sb = l_sb; g.l_sh = l_sh;
  g.kbias = kbias; g.kb_sb = kb_sb;
  g.n = n; g.nk = nk; g.n_dense = n_dense < nk ? n_dense : nk;
  g.scale = scale; g.scale_log2 = scale * 1.4426950408889634f;
  g.kb0 = g.n_dense / 64 * 64;
  g.nq_pad = (n + 63) / 64 * 64;
  g.H = H;
  g.qkn = 1;
  g.xq = {(const bf16_t*)xq, x_sb, x_sh, x_sr};
  g.xk = {(const bf16_t*)xk, x_sb, x_sh, x_sr};
  g.wq = (const bf16_t*)wq; g.wk = (const bf16_t*)wk;
  g.rcos = cos_t; g.rsin = sin_t; g.eps = eps;
  VPT_CHECK_ARG(dw_ld >= 64, "vpt_attn_bwd_qknorm: dw_ld >= 64");
  g.dwq = dwq_part; g.dwk = dwk_part; g.dw_ld = dw_ld;
  return attn_bwd_impl(g, B, H, n, nk, (hipStream_t)stream);
}

namespace {
int attn_bwd_impl(AttnArgs& g, int B, int H, int n, int nk, hipStream_t s) {
  const long rows = (long)B * H * n;
  g.dqacc = nullptr;
#ifdef VPT_DIAG
  if (const int rc = diag_attn_bwd_variants(g, B, H, n, nk, s, rows); rc >= 0) return rc;
#endif
  // production: the split dK/dV pass (explicitly ordered body) + the dQ pass, launched as one grid
  // (attn_bwd_kernel: dK/dV blocks, then dQ blocks). The fused single pass
  // (attn_bwd_fused_kernel, diagnostic variant 13) does 5 products instead of 7 but its f32 dQ atomics
  // run at the chip-wide atomic rate (~1.3 TB/s: 3.4 GB per launch at B=8 1024^2, 128-key blocks):
  // measured 2.66 ms vs 1.55 ms for this pair (1.14 ms with the atomics removed).
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((rows * 8 + 255) / 256), dim3(256), 0, s, g, H, rows);
  VPT_LAUNCH_CHECK();
#ifdef VPT_DIAG
  if (const int rc = diag_attn_bwd_rows64(g, B, H, n, nk, s); rc >= 0) return rc;
#endif
  const int nkb = (nk + 127) / 128, nqb = (n + 127) / 128;
#ifdef VPT_DIAG
  if (g_rows64 & 32) {  // A/B: the software-pipelined dK/dV kernel (diag include), then the one-launch kernel's dQ blocks
    if (const int rc = diag_attn_bwd_pipe(g, nkb, H, B, s); rc != VPT_OK) return rc;
    hipLaunchKernelGGL((attn_bwd_kernel<kDqBody>), dim3(nqb * H * B), dim3(256), key_bias_lds_bytes(g), s, g, 0, nqb, B);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
  if (g_rows64 & (64 | 128)) {  // A/B: compiler-scheduled dK/dV body (64) / head-interleaved block order (128)
    const dim3 grid((nkb + nqb) * H * B);
    if ((g_rows64 & 192) == 64)
      hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, 0, 0>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    else if ((g_rows64 & 192) == 128)
      hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, 8, 1>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    else
      hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, 0, 1>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
  if (g_rows64 & 16) {  // A/B: the other dQ body in the one-launch kernel
    hipLaunchKernelGGL((attn_bwd_kernel<8 - kDqBody>), dim3((nkb + nqb) * H * B), dim3(256), key_bias_lds_bytes(g), s, g,
                       nkb, nqb, B);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
#endif
#ifdef VPT_DIAG
  if (g_mf16 && g_mf16 != kBwdMf16 && !g.qkn) {  // A/B: the 16x16x32 dK/dV (bit 1) / dQ (bit 2) bodies
    const dim3 grid((nkb + nqb) * H * B);
    const size_t kbl_bytes = key_bias_lds_bytes(g);
    if (g_mf16 == 15) {  // production bodies in 8-wave blocks
      const int nkb8 = (nk + 255) / 256, nqb8 = (n + 255) / 256;
      hipLaunchKernelGGL((attn_bwd16_kernel<8>), dim3((nkb8 + nqb8) * H * B), dim3(512), kbl_bytes, s, g, nkb8, nqb8, B);
    } else if (g_mf16 == 1)
      hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, 16>), grid, dim3(256), kbl_bytes, s, g, nkb, nqb, B);
    else if (g_mf16 == 2)
      hipLaunchKernelGGL((attn_bwd_kernel<16, kDkdvBody>), grid, dim3(256), kbl_bytes, s, g, nkb, nqb, B);
    else
      hipLaunchKernelGGL((attn_bwd_kernel<16, 16>), grid, dim3(256), kbl_bytes, s, g, nkb, nqb, B);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
  if (g_bwd_pf) {  // A/B: transposed-fragment prefetch in the dK/dV (bit 1) / dQ (bit 2) products
    const dim3 grid((nkb + nqb) * H * B);
    if (g_bwd_pf == 4)  // the ordered dK/dV body WITH s_setprio around its MFMA groups (the previous production body)
      hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, 8>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    else if (g_bwd_pf == 5)  // the explicitly ordered dQ body without s_setprio
      hipLaunchKernelGGL((attn_bwd_kernel<10, kDkdvBody>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    else if (g_bwd_pf == 1)
      hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, 9>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    else if (g_bwd_pf == 2)
      hipLaunchKernelGGL((attn_bwd_kernel<9, 8>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    else
      hipLaunchKernelGGL((attn_bwd_kernel<9, 9>), grid, dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
  if (g_bwd_nst == 3) {
    hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, 8, 0, 3>), dim3((nkb + nqb) * H * B), dim3(256), key_bias_lds_bytes(g),
                       s, g, nkb, nqb, B);
    VPT_LAUNCH_CHECK();
    return VPT_OK;
  }
  const int mf16 = g_mf16;
#else
  constexpr int mf16 = kBwdMf16;
#endif
  if (mf16 && !g.qkn)  // production: both bodies on the 16x16x32 MFMA, the dK/dV body explicitly ordered
    hipLaunchKernelGGL((attn_bwd_kernel<16, 17>), dim3((nkb + nqb) * H * B), dim3(256), key_bias_lds_bytes(g), s, g,
                       nkb, nqb, B);
  else  // the fused QK-norm epilogue reads the 32x32x16 accumulator layout
    hipLaunchKernelGGL((attn_bwd_kernel<kDqBody, kDkdvBody>), dim3((nkb + nqb) * H * B), dim3(256), key_bias_lds_bytes(g),
                       s, g, nkb, nqb, B);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}

// The persistent-queue backward (attn_bwd_pq_kernel): delta pre-pass, then two resident blocks per CU.
int attn_bwd_pq_impl(AttnArgs& g, int B, int H, int n, int nk, unsigned* qws, hipStream_t s) {
  const long rows = (long)B * H * n;
  g.dqacc = nullptr;
  hipLaunchKernelGGL(attn_bwd_pre_kernel, dim3((rows * 8 + 255) / 256), dim3(256), 0, s, g, H, rows);
  VPT_LAUNCH_CHECK();
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] == 0) {
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    cus[dev] = c;
  }
  const int nkb = (nk + 127) / 128, nqb = (n + 127) / 128;
  hipLaunchKernelGGL(attn_bwd_pq_kernel, dim3(2 * cus[dev]), dim3(256), key_bias_lds_bytes(g), s, g, nkb, nqb, B, qws);
  VPT_LAUNCH_CHECK();
  return VPT_OK;
}
}  // namespace

#ifdef VPT_DIAG
#include "diag/attention_diag_api.inc"
#endif  // VPT_DIAG
