/*
 * vpt_hip_diag.h — diagnostic-only entry points of libvpt_hip_diag.so.
 *
 * The diagnostic library is built from the same sources with -DVPT_DIAG (vpt/_build.py
 * build(diag=True)); it is used by tools/ for A/B timing, ablations and cycle stamps and is never
 * loaded by the product path (vpt/_lib.py loads it only when VPT_DIAG=1). These switches are
 * PROCESS-WIDE and some of them make results WRONG (timing-only ablations), which is why the
 * production library libvpt_hip.so does not export them (it is stateless and reentrant).
 * It exports everything vpt_hip.h declares, plus the functions below.
 */
#ifndef VPT_HIP_DIAG_H
#define VPT_HIP_DIAG_H
#include "vpt_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* GEMM tile geometry override: 0 = automatic; 128, 256; 2561 = ring unstaggered, 2562 = 256x256
 * 2-stage (A/B); 2563/2564 = timing-only ablations of the ring (WRONG results); 2565 = DMA in the
 * MFMA phase; 2566 / 2567 = stamped / timeline ring builds (need vpt_gemm_set_debug); 2568 = ring without
 * its epilogue (timing only, WRONG results; accumulators kept live so the MFMAs are not dead code). */
int vpt_gemm_set_geometry(int geo);
/* u64 buffer receiving per-wave K-step segment cycle sums (2566: [256][8][8]) or realtime stamps
 * (2567: [grid][4][4]); nullptr disables. */
int vpt_gemm_set_debug(unsigned long long* buf);
/* Ring grid override for every ring GEMM (0 = per-call / default: one block per item; 256 = the persistent walk with
 * one block per CU). */
int vpt_gemm_set_ring_grid(int blocks);
/* Ring epilogue stagger in 10-ns ticks: half the blocks start that much later (0 = off, production). */
int vpt_gemm_set_stagger(int ticks);
/* Forward lazy-rescale threshold in log2 units (default 8; 0 = rescale whenever the row max grows). */
int vpt_attn_set_rescale_threshold(float tau);
/* Attention kernel variant: 0 = production (split dK/dV + dQ kernels); 13 = fused single-pass backward
 * with f32 dQ atomics (correct); 10-12 = its timing ablations (WRONG results: no atomics / plain stores /
 * no dQ product); 1 / 2 = timing-only backward ablations (WRONG results);
 * 3 = 8-wave blocks (correct); 4-7 = dK/dV timing ablations (WRONG results); 8 = the previous
 * compiler-scheduled dK/dV body (correct). */
int vpt_attn_set_variant(int v);
/* f32 dQ accumulator of the fused backward variants 10-13: [B*H][round_up(n, 64)][64]. */
long vpt_attn_fused_workspace_bytes(int B, int H, int n);
int vpt_attn_set_fused_workspace(void* ws);
/* Backward kernel pair: 1 = 64 rows per wave (production default), 0 = the 32-row pair (A/B). */
int vpt_attn_set_rows64(int on);
int vpt_attn_set_bwd_stages(int n);
/* Attention forward / backward block order: 1 = XCD-contiguous (a (batch, head)'s blocks on one XCD), 0 = linear. */
int vpt_attn_set_xcd_order(int on);
/* QK-norm attention forward: S^T chain with its K fragments read before the MFMAs (1) or hipcc's order (0). */
int vpt_attn_set_fwd_order(int on);
/* Attention backward: transposed-fragment prefetch in the dK/dV (bit 1) / dQ (bit 2) products; 0 = production. */
int vpt_attn_set_bwd_prefetch(int mask);
/* Attention backward partner waves: bit 0 = s_setprio 1 for the odd-slot wave of each SIMD, bit 1 = its block starts
   (v >> 2) x 10 ns late; 0 = production. */
int vpt_attn_set_bwd_partner(int v);
/* QK-norm attention forward: row sums as a third MFMA block (1) or as f32 adds (0, production). */
int vpt_attn_set_fwd_lsum(int on);
// Backward bodies on the 16x16x32 MFMA: bit 1 dK/dV, bit 2 dQ, 7 = both with the ordered dK/dV body (production);
// 0 = the 32x32x16 bodies. Not with the fused QK-norm backward.
int vpt_attn_set_bwd_mfma16(int mask);
// The QK-norm forward's fixed-reference body on the 16x16x32 MFMA (0 = production 32x32x16).
int vpt_attn_set_fwd_mfma16(int on);
int vpt_gemm_set_swb_one_group(int on);
/* SwiGLU-backward ring GEMM timing ablations (WRONG results): 0 off, 3 = no epilogue, 4 = dx12 stores dropped,
   6 = every item's x12 operands from the first tile (L2-resident). */
int vpt_gemm_set_swb_ablation(int a);
/* 256x128 two-blocks-per-CU ring (gemm_r2.hip) in place of the 256x256 ring, by launch kind: bit 0 = k-major A (forward,
   input gradient), 1 = mn-major A (weight gradient), 2 = fused SwiGLU forward, 3 = fused SwiGLU backward, 4 = fused
   QK-norm + RoPE forward; production = 8. */
int vpt_gemm_set_r2(int mask);
/* NF4 GEMM timing ablations (WRONG results): 0 off, 1 = no dequant, 2 = no NF4 code loads / dequant. */
int vpt_gemm_set_nf4_ablation(int a);
/* Co-running-kernel probe: `blocks` one-wave workgroups holding a CU each (lds_bytes of LDS) for `ticks` of the 100-MHz
 * clock (sink: a device float[64], never written in practice). */
int vpt_diag_occupy(int blocks, long ticks, int lds_bytes, float* sink, void* stream);

#ifdef __cplusplus
}
#endif
#endif
