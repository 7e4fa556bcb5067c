/*
 * vpt_hip.h — C ABI of libvpt_hip.so, the MI355X (gfx950 / CDNA4) kernel library behind the
 * JiT rectified-flow training step of p1atdev/vision-pt.
 *
 * Conventions
 *  - Plain pointers to device memory, element strides / leading dimensions in ELEMENTS, sizes as
 *    int/long. bf16 tensors are 16-bit words, f32 tensors are float, fp16 images are 16-bit words.
 *  - Every call is enqueued on `stream` (a hipStream_t passed as void*), never synchronises the
 *    host, never allocates or frees device memory (callers own outputs and workspaces), and keeps
 *    no reference to its arguments after returning. Safe to capture in a hipGraph.
 *  - Status: 0 = OK, 1 = invalid argument, 2 = unsupported shape, 3 = HIP launch error; the
 *    message of the calling thread's last failure is vpt_last_error_string(). No C++ exception
 *    crosses the boundary.
 *  - Functions named *_blocks / *_bytes return sizes (partial-sum rows, workspace bytes).
 *
 * Reference interfaces replaced (paths relative to p1atdev/vision-pt):
 *  see the comment above each function.
 */
#ifndef VPT_HIP_H
#define VPT_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---- library ---------------------------------------------------------------------------- */
const char* vpt_last_error_string(void);
int vpt_abi_version(void);
const char* vpt_build_info(void);

/* ---- GEMM (MFMA bf16, f32 accumulate) -----------------------------------------------------
 * C[M,N] (=|+=) sum_k A(m,k) B(n,k) (+bias[n]) (+resid[m,n]) (SiLU).
 * A(m,k) = A[m*lda + k] if a_kmajor else A[k*lda + m]; same for B with n.
 * out_mode 0 = bf16 store, 1 = f32 store, 2 = f32 accumulate; act 0 = none, 1 = SiLU.
 * splits > 1: split-K into f32 slabs in `workspace` (vpt_gemm_workspace_bytes), deterministic sum; the
 * slab reduce applies bias / residual (bf16 output; no SiLU, alpha 1).
 * Replaces nn.Linear / 1x1 & patch Conv2d forward and their autograd backward:
 *   src/models/jit/denoiser.py:36-49,59-65 (BottleneckPatchEmbed), :80-84 (TimestepEmbedder MLP),
 *   :318-323,360-366,391-395 (Attention to_q/k/v/o), :492-504 (SwiGLU), :535-543 (FinalLayer),
 *   :715-719,997 (context_embedder). */
int vpt_gemm_bf16(const void* A, long lda, int a_kmajor, const void* B, long ldb, int b_kmajor, void* C,
                  long ldc, int M, int N, int K, const void* bias, const void* resid, long ldr, int out_mode,
                  int act, int splits, void* workspace, float alpha, void* stream);
long vpt_gemm_workspace_bytes(int M, int N, int K, int splits);
/* vpt_gemm_bf16 with an explicit tile geometry (stateless; same results contract): geometry 0 =
 * automatic, 128 = 128x128 2-stage, 256 = the persistent 256x256 ping-pong ring, whose
 * min(work items, ring_grid) blocks walk (tile, split-K slice) items (ring_grid 0 = one block per item).
 * 1281 = 128x128 tiles on the pipeline of the 256x128 ring (3-stage LDS-DMA ring, counted waits; bf16 / f32 /
 * f32-accumulate output with bias / residual, split-K; no fused bias gradient, SwiGLU or QK-norm epilogue): the
 * same K order as geometry 128, equal results. The LoRA entry points below take it as well.
 * Used by tests to cover both geometries and multi-item ring walks at small shapes. */
int vpt_gemm_bf16_tiled(const void* A, long lda, int a_kmajor, const void* B, long ldb, int b_kmajor, void* C,
                        long ldc, int M, int N, int K, const void* bias, const void* resid, long ldr, int out_mode,
                        int act, int splits, void* workspace, float alpha, int geometry, int ring_grid,
                        void* stream);
/* LoRALinear over a frozen base (src/modules/peft/lora.py:92-104; the QLoRA targets of
 * configs/sdxl/flow_match/config.yml), the base GEMM and the LoRA term in one f32 accumulator:
 * C[M,N] = A.B (+bias) (+resid, as vpt_gemm_bf16) + A2.B2 over K2 extra reduction elements.
 *   forward:        A = x [M][K], B = W [N][K] (b_kmajor 1), A2 = s*x.down^T [M][r], B2 = up [N][r]
 *   input gradient: A = dy [M][N_out], B = W [N_out][K_in] (b_kmajor 0), A2 = s*dy.up [M][r], B2 = down [r][K_in]
 * W is the bf16 base weight (for an NF4 base: vpt_nf4_dequant's output, exactly what bitsandbytes'
 * MatMul4Bit dequantises before its torch.nn.functional.linear). A, A2 k-major; K % 64 == 0; K2 % 8 == 0,
 * 0 < K2 <= 256 (several adapters side by side: K2 = their ranks summed, B2 block-diagonal); splits > 1:
 * split-K over `workspace` (vpt_gemm_workspace_bytes; the extension rides the last slice, bias / residual are
 * applied by the slab reduce); geometry as vpt_gemm_bf16_tiled (0 = automatic). Deterministic. */
int vpt_gemm_bf16_lora(const void* A, long lda, const void* B, long ldb, int b_kmajor, const void* A2, long lda2,
                       const void* B2, long ldb2, int K2, void* C, long ldc, int M, int N, int K, const void* bias,
                       const void* resid, long ldr, int out_mode, int splits, void* workspace, int geometry,
                       void* stream);
/* Several LoRA targets reading one input (the attention q / k / v projections of a TransformerBlock,
 * src/models/sdxl/denoiser.py:101-171 over lora.py:92-104) as ONE GEMM: B = the G base weights stacked
 * [G*g_n][K] (k-major), C[:, g*g_n:(g+1)*g_n] = A.W_g^T (+bias, +resid) + A2[:, g*r:(g+1)*r].up_g^T with
 * up_g = B2s[g] ([g_n][r], k-major). 1 <= G <= 4, r % 8 == 0, r <= 64, g_n % 128 == 0 (a 256-wide ring tile is
 * used only when g_n % 256 == 0), K % 64 == 0; splits / workspace / geometry as vpt_gemm_bf16_lora. */
int vpt_gemm_bf16_lora_grouped(const void* A, long lda, const void* B, long ldb, const void* A2, long lda2,
                               const void* const* B2s, int G, int r, void* C, long ldc, int M, int g_n, int K,
                               const void* bias, const void* resid, long ldr, int splits, void* workspace,
                               int geometry, void* stream);
/* vpt_gemm_bf16_lora / vpt_gemm_bf16_lora_grouped (splits = 1) with an output scale: alpha multiplies the f32
 * result (base + extension) of output columns [0, alpha_cols) -- every column when alpha_cols = 0; otherwise a
 * multiple of 128 -- before bias / residual and the one bf16 rounding: the attention q projection emitted already
 * multiplied by vpt_attn_q_scale (the attention kernels' pre-scaled q) instead of a separate scaling pass. */
int vpt_gemm_bf16_lora_scaled(const void* A, long lda, const void* B, long ldb, int b_kmajor, const void* A2, long lda2,
                              const void* B2, long ldb2, int K2, void* C, long ldc, int M, int N, int K,
                              const void* bias, const void* resid, long ldr, int geometry, float alpha, int alpha_cols,
                              void* stream);
int vpt_gemm_bf16_lora_grouped_scaled(const void* A, long lda, const void* B, long ldb, const void* A2, long lda2,
                                      const void* const* B2s, int G, int r, void* C, long ldc, int M, int g_n, int K,
                                      const void* bias, const void* resid, long ldr, int geometry, float alpha,
                                      int alpha_cols, void* stream);
/* The same with the G bases stacked [G*g_n][K] and the G ups stacked [G*g_n][r] (B2, leading dim r), any G:
 * the cross-attention to_k / to_v of every transformer block over one fixed text context as ONE GEMM per step
 * (src/models/sdxl/denoiser.py:101-171; the context is the same for all 70 blocks). */
int vpt_gemm_bf16_lora_stacked(const void* A, long lda, const void* B, long ldb, const void* A2, long lda2,
                               const void* B2, int G, int r, void* C, long ldc, int M, int g_n, int K, int splits,
                               void* workspace, int geometry, void* stream);
/* nn.Linear weight and bias gradient in one call (torch autograd of F.linear for every Linear of
 * src/models/jit/denoiser.py, e.g. :318-323 attention projections, :492-504 SwiGLU, :535-543 FinalLayer):
 * dw[N][K] (=|+=) dy[M][N]^T . x[M][K] and, if db != NULL, db[N] (=|+=) sum_m dy[m][N], both f32
 * (accumulate = 1 adds). On the 256x256 ring geometry the bias sums ride the GEMM (MFMAs of the dy fragments
 * against an all-ones fragment, reduced with the split-K slabs in one launch); otherwise the colsum path of
 * vpt_bias_grad runs after the GEMM. workspace: vpt_linear_wgrad_workspace_bytes(M, N, K, splits) bytes.
 * geometry / ring_grid as vpt_gemm_bf16_tiled (0 = automatic). Deterministic. */
int vpt_linear_wgrad(const void* dy, long lddy, const void* x, long ldx, float* dw, long lddw, float* db, long M,
                     int N, int K, int accumulate, int splits, void* workspace, int geometry, int ring_grid,
                     void* stream);
/* vpt_linear_wgrad plus one unrelated column sum rr_out[c] (=|+=) sum_r rr_part[r][c] over a [rr_R][rr_C] f32 partial
 * set (the vpt_reduce_rows job of, e.g., an RMSNorm weight gradient), done by extra blocks of the weight gradient's
 * split-K reduce launch instead of a launch of its own. Fixed summation order (deterministic). */
int vpt_linear_wgrad_rr(const void* dy, long lddy, const void* x, long ldx, float* dw, long lddw, float* db, long M,
                        int N, int K, int accumulate, int splits, void* workspace, int geometry, int ring_grid,
                        const float* rr_part, int rr_R, int rr_C, float* rr_out, int rr_acc, void* stream);
long vpt_linear_wgrad_workspace_bytes(long M, int N, int K, int splits);

/* Fused SwiGLU MLP GEMMs (src/models/jit/denoiser.py:480-506 SwiGLU, :535-543 FinalLayer):
 * forward: x12 [M][2F] = x.W12^T + b12 (W12 = w_1 | w_2 rows, [2F][K]) and h [M][F] =
 * bf16(bf16(silu(x1)) * x2) from one GEMM (the epilogue pairs x1 / x2 columns);
 * backward: dx12 [M][2F] from dh = dy.W3 (dy [M][D], W3 [D][F]) and x12, the SwiGLU derivative applied
 * in the dgrad epilogue (dh never reaches memory). Small shapes run the plain GEMM + the elementwise
 * kernel (backward: dh in `workspace`, vpt_gemm_swiglu_bwd_workspace bytes, 0 when not needed). */
int vpt_gemm_swiglu_fwd(const void* x, long ldx, const void* w12, long ldw, const void* b12, void* x12, long ldx12,
                        void* h, long ldh, int M, int F, int K, void* stream);
long vpt_gemm_swiglu_bwd_workspace(int M, int F, int D);
int vpt_gemm_swiglu_bwd(const void* dy, long lddy, const void* w3, long ldw3, const void* x12, long ldx12, void* dx12,
                        long lddx12, int M, int F, int D, void* workspace, void* stream);

/* The JiT attention input projection with the per-head QK-RMSNorm + RoPE fused into its epilogue: qkv [M][3D] =
 * x . W^T + b (W = to_q|to_k|to_v [3D][K], bf16 out) and qk [M][2D] = (rope(rms(q) wq) * q_scale | rope(rms(k) wk)),
 * bitwise what vpt_qknorm_rope_fwd computes from that qkv. Replaces Attention.to_q/to_k/to_v + q_norm/k_norm +
 * apply_rope, src/models/jit/denoiser.py:318-323, 307-316, 369-373, 98-111. */
int vpt_linear_qknorm_rope(const void* x, long ldx, const void* w, long ldw, const void* bias, void* qkv, long ldqkv,
                           void* qk, long ldqk, int M, int D, int K, const void* wq, const void* wk, const float* cos_t,
                           const float* sin_t, int rows_per_seq, float eps, float q_scale, void* stream);

/* ---- flash attention, head_dim 64 ---------------------------------------------------------
 * Tensors addressed p[b*sb + h*sh + row*sr + d]; n query rows, nk key rows (nk = n for
 * self-attention; SDXL cross-attention nk = context length). Keys < n_dense always valid; keys in
 * [n_dense, nk) get kbias[b*kb_sb + key] (0 or -inf); keys >= nk masked. lse/delta [b*l_sb+h*l_sh+q].
 * q must be PRE-SCALED by scale*log2(e) (vpt_qknorm_rope_fwd q_scale, or any bf16 scaling); k, v are
 * raw. The forward writes lse = -log2(sum_k exp(scale*q.k)) (negated, log2 units) for the backward;
 * delta is backward workspace. dq, dk, dv are gradients w.r.t. the UNSCALED q, k, v. */
float vpt_attn_q_scale(float scale);
/* Attention entry points:
 * Replaces src/modules/attention.py:98-159 scaled_dot_product_attention (eager SDPA with the
 * [B,H,N,N] bool mask of src/models/jit/denoiser.py:375-390) and its autograd backward. */
int vpt_attn_fwd(const void* q, long q_sb, long q_sh, long q_sr, const void* k, long k_sb, long k_sh, long k_sr,
                 const void* v, long v_sb, long v_sh, long v_sr, void* o, long o_sb, long o_sh, long o_sr,
                 float* lse, long l_sb, long l_sh, const float* kbias, long kb_sb, int B, int H, int n,
                 int nk, int n_dense, float scale, void* stream);
/* vpt_attn_fwd for QK-RMSNormed inputs (JiT: q, k = rope(rms(x) w), q pre-scaled; wq / wk the q_norm / k_norm
 * weights [64]): the same outputs computed with a fixed softmax reference point -- the scores' Cauchy-Schwarz bound
 * from the norm weights -- instead of a running row maximum, while that bound stays below 60 (log2 units). */
int vpt_attn_fwd_qknorm(const void* q, long q_sb, long q_sh, long q_sr, const void* k, long k_sb, long k_sh,
                        long k_sr, const void* v, long v_sb, long v_sh, long v_sr, void* o, long o_sb, long o_sh,
                        long o_sr, float* lse, long l_sb, long l_sh, const float* kbias, long kb_sb, const void* wq,
                        const void* wk, int B, int H, int n, int nk, int n_dense, float scale, void* stream);
int vpt_attn_bwd(const void* q, long q_sb, long q_sh, long q_sr, const void* k, long k_sb, long k_sh, long k_sr,
                 const void* v, long v_sb, long v_sh, long v_sr, const void* o, long o_sb, long o_sh, long o_sr,
                 const void* dO, long do_sb, long do_sh, long do_sr, const float* lse, float* delta, long l_sb,
                 long l_sh, const float* kbias, long kb_sb, void* dq, long dq_sb, long dq_sh, long dq_sr,
                 void* dk, long dk_sb, long dk_sh, long dk_sr, void* dv, long dv_sb, long dv_sh, long dv_sr,
                 int B, int H, int n, int nk, int n_dense, float scale, void* stream);
/* vpt_attn_bwd on a persistent work-queue kernel: the same dK/dV and dQ items and products, bitwise the same results,
 * run by two resident blocks per CU pulling items from per-XCD queues (dynamic fill; the next item's first tile staged
 * under the current item's last). queue = vpt_attn_bwd_queue_bytes() (64) bytes of 64-byte-aligned device memory owned
 * by the caller: zero before its first use, left zero by every launch; one per stream that may run it concurrently. */
int vpt_attn_bwd_q(const void* q, long q_sb, long q_sh, long q_sr, const void* k, long k_sb, long k_sh, long k_sr,
                   const void* v, long v_sb, long v_sh, long v_sr, const void* o, long o_sb, long o_sh, long o_sr,
                   const void* dO, long do_sb, long do_sh, long do_sr, const float* lse, float* delta, long l_sb,
                   long l_sh, const float* kbias, long kb_sb, void* dq, long dq_sb, long dq_sh, long dq_sr, void* dk,
                   long dk_sb, long dk_sh, long dk_sr, void* dv, long dv_sb, long dv_sh, long dv_sr, int B, int H, int n,
                   int nk, int n_dense, float scale, void* queue, void* stream);
int vpt_attn_bwd_queue_bytes(void);
/* The same backward with the per-head QK-RMSNorm + RoPE backward fused into its dQ / dK stores (JiT self-attention,
 * src/models/jit/denoiser.py:307-316, 98-111; replaces vpt_attn_bwd + vpt_qknorm_rope_bwd for that path): q, k are
 * the normed, roped (q pre-scaled) attention inputs as for vpt_attn_bwd; xq / xk the raw projections they came from
 * (same strides x_*), wq / wk the q_norm / k_norm weights [64], cos_t / sin_t the RoPE tables [positions][32] (a
 * row's position is its row: n == nk). dq / dk (strides dqk_*) receive d loss / d (raw q, k) in bf16, computed from
 * the f32 attention gradients; dwq_part / dwk_part receive per-workgroup partial q_norm / k_norm weight gradients,
 * vpt_attn_bwd_dw_rows(B, H, n) rows of 64 floats at row stride dw_ld (dwk_part = dwq_part + 64 with dw_ld = 128
 * interleaves them, so ONE vpt_reduce_rows over [rows][128] sums both in a fixed order). */
int vpt_attn_bwd_dw_rows(int B, int H, int n);
int vpt_attn_bwd_qknorm(const void* q, long q_sb, long q_sh, long q_sr, const void* k, long k_sb, long k_sh, long k_sr,
                        const void* v, long v_sb, long v_sh, long v_sr, const void* o, long o_sb, long o_sh, long o_sr,
                        const void* dO, long do_sb, long do_sh, long do_sr, const float* lse, float* delta, long l_sb,
                        long l_sh, const float* kbias, long kb_sb, const void* xq, const void* xk, long x_sb,
                        long x_sh, long x_sr, const void* wq, const void* wk, const float* cos_t, const float* sin_t,
                        float eps, void* dq, void* dk, long dqk_sb, long dqk_sh, long dqk_sr, float* dwq_part,
                        float* dwk_part, long dw_ld, void* dv, long dv_sb, long dv_sh, long dv_sr, int B, int H, int n, int nk,
                        int n_dense, float scale, void* stream);

/* ---- RMSNorm over the hidden dim -----------------------------------------------------------
 * Replaces FP32RMSNorm.forward src/modules/norm.py:20-27 (norm1/norm2/norm_final,
 * src/models/jit/denoiser.py:521,600,625) and its backward (dx = dres + RMSNorm'(dy);
 * dw_part[blocks][D] partial sums, reduce with vpt_reduce_rows). */
int vpt_rmsnorm_fwd(const void* x, long ldx, const void* w, void* y, long ldy, float* rstd, int M, int D, float eps,
                    void* stream);
int vpt_rmsnorm_bwd_blocks(int M);
int vpt_rmsnorm_bwd(const void* dy, long lddy, const void* x, long ldx, const float* rstd, const void* w,
                    const void* dres, long ldr, void* dx, long lddx, float* dw_part, int M, int D, void* stream);

/* ---- fused per-head QK-RMSNorm + RoPE --------------------------------------------------------
 * qkv [M][ldin] (q|k|v, D each) -> out [M][ldout] (rope(rms(q)) | rope(rms(k))).
 * Replaces Attention.q_norm/k_norm + apply_rope, src/models/jit/denoiser.py:307-316,369-373,98-111
 * (cos/sin tables [rows_per_seq][32] f32 replace the per-forward host RoPE gather 1013-1051). */
int vpt_qknorm_rope_blocks(int M);
/* q_scale multiplies the q half of the output before its bf16 rounding: the engine passes
 * vpt_attn_q_scale(1/sqrt(64)) so the result feeds vpt_attn_fwd/bwd directly (k is unscaled). */
int vpt_qknorm_rope_fwd(const void* qkv, long ldin, const void* wq, const void* wk, const float* cos_t,
                        const float* sin_t, void* out, long ldout, int M, int rows_per_seq, int D, float eps,
                        float q_scale, void* stream);
int vpt_qknorm_rope_bwd(const void* dqk, long lddqk, const void* qkv, long ldin, const void* wq, const void* wk,
                        const float* cos_t, const float* sin_t, void* dqkv, long lddqkv, float* dw_part, int M,
                        int rows_per_seq, int D, float eps, void* stream);
/* The same for the rows pos < n_valid of each sequence; rows past it get zero q | k | v gradients in dqkv (lddqkv >=
 * 3D) without dqk being read -- a pre-context block's context rows (denoiser.py:1092-1113), whose attention backward
 * covers only the n_valid rows. vpt_qknorm_rope_bwd = n_valid of rows_per_seq. */
int vpt_qknorm_rope_bwd_rows(const void* dqk, long lddqk, const void* qkv, long ldin, const void* wq, const void* wk,
                             const float* cos_t, const float* sin_t, void* dqkv, long lddqkv, float* dw_part, int M,
                             int rows_per_seq, int n_valid, int D, float eps, void* stream);
int vpt_reduce_rows(const float* in, int R, int C, float* out, int accumulate, void* stream);

/* ---- flow matching input / loss ----------------------------------------------------------------
 * patchify: z = t*x + (1-t)*eps (eps from `noise` fp16 or the counter RNG `seed`), written in the
 * Conv2d(k=16,s=16) im2col order; in_kind 1 copies a bf16 image. Replaces
 * prepare_scaled_noised_latents src/modules/loss/flow_match.py:60-74 + the proj_1 im2col.
 * flow_loss: mse(pred, x) (target 0) or mse(v(pred), v(x)) (target 1) with v = (. - z)/max(1-t, eps), or for a
 * velocity prediction mse(pred, fp16(x - eps)) (target 2; class_to_image.py:146-156, no timestep clamp),
 * writes d loss/d pred. Replaces treat_loss train/jit/arb_class_to_image.py:108-151,
 * JiTModel.image_to_velocity src/models/jit/pipeline.py:253-260, JiT._unpatchify denoiser.py:828-860. */
int vpt_patchify(const void* img, int in_kind, const void* noise, const float* t, float noise_scale,
                 unsigned long long seed, int B, int H, int W, void* out, void* stream);
int vpt_unpatchify(const void* patches, int B, int H, int W, void* img, int reverse, void* stream);
/* Sampler: one Euler step with classifier-free guidance over the bf16 image z [B,3,H,W], the
 * prediction read from the final-layer patch layout [n*np, 768] (n = 2B when cfg, positive half
 * first); mode 0 = image prediction (v = (x - z) / clamp(1 - t, 1e-5)), 1 = velocity prediction;
 * every op rounds to bf16 like the reference's bf16 tensors. Replaces the denoising loop body of
 * JiTModel.generate (src/models/jit/pipeline.py:436-477). */
int vpt_euler_cfg_step(void* z, const void* pred, int B, int H, int W, int cfg, float cfg_scale, int mode, float t,
                       float dt, void* stream);
int vpt_loss_blocks(void);
/* lowres_loss inputs (train/jit/arb_class_to_image.py:228-264): F.interpolate(mode="area", scale_factor=1/k), k even,
 * of the fp16 image -> img_lr fp16, of the fp16 noise (`noise`, or NULL = the counter RNG `seed` as patchify) ->
 * noise_lr fp16, and of the noisy image t x + (1-t) eps -> z_lr bf16 (the lowres model input); all [B][3][H/k][W/k]. */
/* The in-kernel noise as an fp16 tensor: element i of a flat [B][3][H][W] image (n = B*3*H*W, even) is exactly the
 * draw patchify / flow_loss / area_lowres generate at that index for `seed` -- torch.randn_like(latents) * noise_scale
 * of prepare_scaled_noised_latents (src/modules/loss/flow_match.py:60-74). */
int vpt_gauss_noise(long n, unsigned long long seed, float noise_scale, void* out, void* stream);
int vpt_area_lowres(const void* img, const void* noise, const float* t, float noise_scale, unsigned long long seed,
                    int B, int H, int W, int k, void* img_lr, void* noise_lr, void* z_lr, void* stream);
int vpt_flow_loss(const void* pred, const void* img, const void* noise, const float* t, float noise_scale,
                  unsigned long long seed, int target, float t_eps, int B, int H, int W, void* dpred, float* part,
                  float* loss, void* stream);

/* ---- embeddings and token assembly ----------------------------------------------------------
 * timestep_embed: get_timestep_embedding(flip_sin_to_cos=True, shift 0),
 *   src/modules/timestep/embedding.py:10-62.
 * assemble/disassemble/ctx_rows: token concatenation and per-block context append/strip,
 *   src/models/jit/denoiser.py:982-993,1078-1113 (+ their backward).
 * ctx_rows backward: 1 adds the context rows' gradient into dctx (f32), 2 writes it (the backward's first refresh
 *   block: no zero pass over dctx before); both zero those rows of x.
 * copy_rows: patch-token slice tokens[:, :N_p] (denoiser.py:1115). reverse 0: seq -> dense; 1: dense -> seq;
 *   2: dense -> seq and every other row of each sequence zeroed (the slice's backward into a fresh buffer).
 * embed_gather/scatter_add: nn.Embedding(padding_idx) of ClassEncoder, class_encoder.py:107-144. */
int vpt_timestep_embed(const float* vals, int R, void* out, void* stream);
int vpt_assemble_tokens(const void* patches, const void* size_emb, const void* time_emb, const void* tpe,
                        const void* ctx, int n_ctx, int B, int np_, int rows, int D, void* x, void* stream);
int vpt_disassemble_tokens(const void* dx, int B, int np_, int rows, int D, void* dpatches, void* dsize, void* dtime,
                           float* dtpe, void* stream);
int vpt_ctx_rows(void* x, int B, int row0, int rows, int D, const void* ctx, float* dctx, int n_ctx, int backward,
                 void* stream);
int vpt_copy_rows(void* seq, long ld_seq, int rows, int row0, int cnt, void* dense, long ld_dense, int B, int D,
                  int reverse, void* stream);
int vpt_embed_gather(const void* table, const long long* ids, long R, int D, void* out, void* stream);
int vpt_embed_scatter_add(const void* drows, const long long* ids, long R, int D, long long pad_id, float* dtable,
                          void* stream);
/* The same gradient written in one deterministic pass, each row summed in position order (O(R) position lists per
 * 8-row block; R <= 16384): accumulate = 0 overwrites the whole [V][D] table (zeros where no id points, the padding
 * row zero), accumulate = 1 adds the sum to the rows the ids name (torch's .grad += under gradient accumulation).
 * Replaces the zero_() of the class-embedding gradient + the scatter of arb_class_to_image.py's nn.Embedding backward
 * (class_encoder.py:16-90, :127-144). */
int vpt_embed_grad_set(const void* drows, const long long* ids, long R, int D, long long pad_id, long V, int accumulate,
                       float* dtable, void* stream);
/* The JiT step's per-batch inputs in one launch: t_vals = bf16(bf16(t) * tscale) as f32 (arb_class_to_image.py:207),
 * size_vals [B][6] f32 = original_size | target_size | crop_coords (int64 [B][2] each; denoiser.py's size embedder
 * input), and key-bias rows kbias[b][0, n_pre + n_ctx) (row stride rows): 0, then 0 / -inf by mask [B][n_ctx] int64
 * (NULL = all valid) -- the attention-mask expansion of denoiser.py:1078-1090. */
int vpt_step_inputs(const float* t, int B, float tscale, const long long* orig, const long long* target,
                    const long long* crop, float* t_vals, float* size_vals, const long long* mask, int n_ctx, int n_pre,
                    int rows, float* kbias, void* stream);

/* ---- activations / reductions ---------------------------------------------------------------
 * swiglu: silu(x1) * x2, SwiGLU.forward src/models/jit/denoiser.py:499-504 (+ backward).
 * silu: the TimestepEmbedder SiLU (denoiser.py:80-84). colsum: Linear bias gradients. */
int vpt_swiglu_fwd(const void* x12, long M, int F, void* h, void* stream);
int vpt_swiglu_bwd(const void* dh, const void* x12, long M, int F, void* dx12, void* stream);
int vpt_silu(const void* x, const void* dy, void* out, long n, int backward, void* stream);
int vpt_colsum_blocks(long M);
/* Linear bias gradient out[N] (=|+=) sum over M rows of in (bf16, row stride ld): column partials into
 * part [vpt_colsum_blocks(M)][N] f32 scratch, then a fixed-order row reduction (deterministic).
 * Replaces the autograd bias gradients of every nn.Linear on the path. */
int vpt_bias_grad(const void* in, long ld, long M, int N, float* part, float* out, int accumulate, void* stream);
int vpt_cast_f32_bf16(const float* in, long n, void* out, void* stream);

/* ---- optimizer -------------------------------------------------------------------------------
 * RAdamScheduleFree step over flat buffers (bf16 y, f32 z / v; grad f32, or bf16 when grad_bf16 = 1:
 * the all-reduced bf16 wire buffer of the data-parallel path); sf_lerp implements the
 * train()/eval() y<->x swap; sf_init lazily creates z = y, v = 0. Replaces schedulefree 1.4.1
 * RAdamScheduleFree (configs/jit/x-loss/config.yml:74-78, src/optimizer/util.py:5-31,
 * src/trainer/common.py:276-285,382-388). */
int vpt_radam_sf_step(void* y, const void* grad, int grad_bf16, float* z, float* v, long n, float beta2,
                      float bias_correction2, float eps, float ckp1, float adaptive_y_lr, float lr, float decay,
                      float grad_scale, int adam, const float* clip_coef, float clip_value, void* stream);
/* Gradient clipping (src/models/for_training.py:98-109 after_backward: accelerator.clip_grad_norm_ /
 * clip_grad_value_, src/config.py:74-75): the step above multiplies g by *clip_coef (device scalar; null =
 * none) and then clamps it to [-clip_value, clip_value] (0 = none). The global norm is taken over all
 * (all-reduced, mean) gradient buckets: vpt_grad_sumsq writes vpt_grad_norm_blocks() partial sums of
 * (scale * g)^2 of one bucket into part; vpt_clip_coef sums n partials in a fixed order and writes
 * coef = min(1, max_norm / (norm + 1e-6)) (torch.nn.utils.clip_grad_norm_) and, if norm_out, the norm. */
int vpt_grad_norm_blocks(void);
int vpt_grad_sumsq(const void* g, int g_bf16, long n, float scale, float* part, void* stream);
int vpt_clip_coef(const float* part, int n, float max_norm, float* coef, float* norm_out, void* stream);
int vpt_sf_lerp(void* y, const float* z, long n, float w, void* stream);
/* EMA copy of the flat bf16 parameters (swa_utils.AveragedModel(get_ema_avg_fn(decay)), use_buffers=False;
 * src/trainer/common.py:211-216, 385-386): first = 1 copies, else ema = bf16(bf16(d*ema) + bf16(omd*p)); omd = the caller's
 * f32 rounding of (1 - decay) formed in double (torch rounds the Python scalar 1 - decay, not 1 - f32(decay)). */
int vpt_ema_update(void* ema, const void* param, long n, float decay, float one_minus_decay, int first, void* stream);
int vpt_sf_init(const void* y, float* z, float* v, long n, void* stream);


/* ---- SDXL QLoRA transformer block ------------------------------------
 * LayerNorm: nn.LayerNorm norm1/2/3 (src/models/sdxl/denoiser.py:254-256), eps 1e-5, f32 statistics;
 * backward dx = dres + LN'(dy), per-block dw/db partials [vpt_layernorm_bwd_blocks(M)][D]. D <= 2048. */
int vpt_layernorm_fwd(const void* x, long ldx, const void* w, const void* b, void* y, long ldy, float* mean,
                      float* rstd, int M, int D, float eps, void* stream);
/* LayerNorm (as vpt_layernorm_fwd, bit-identical y / mean / rstd) and, in the same launch, the rank-16 LoRA
 * down-projections of its output: ds[m][16 g + j] = bf16(alpha * y[m] . down_g[j]) for g < G (<= 3), down_g =
 * down + g * w_goff ([16][D] each) -- bit-identical to vpt_lora_proj(_grouped) on y. D % 128 == 0. */
int vpt_layernorm_lora_fwd(const void* x, long ldx, const void* w, const void* b, void* y, long ldy, float* mean,
                           float* rstd, int M, int D, float eps, const void* down, long w_goff, int G, void* ds,
                           long ldds, float alpha, void* stream);
int vpt_layernorm_bwd_blocks(int M);
int vpt_layernorm_bwd(const void* dy, long lddy, const void* x, long ldx, const float* mean, const float* rstd,
                      const void* w, const void* dres, long ldr, void* dx, long lddx, float* dw_part, float* db_part,
                      int M, int D, void* stream);
/* LayerNorm backward with frozen affine weights (as vpt_layernorm_bwd without partials: bit-identical dx) and, in the
 * same launch, the rank-16 LoRA projection of dx through an up matrix: vs[m][j] = bf16(alpha * dx[m] . up[:, j]),
 * up [D][16] -- bit-identical to vpt_lora_proj(dx, up, w_kmajor = 0). D % 128 == 0. */
int vpt_layernorm_bwd_lora(const void* dy, long lddy, const void* x, long ldx, const float* mean, const float* rstd,
                           const void* w, const void* dres, long ldr, void* dx, long lddx, int M, int D, const void* up,
                           void* vs, long ldvs, float alpha, void* stream);
/* GeGLU (denoiser.py:174-186): out[M,F] = h * gelu_erf(gate), (h | gate) = x12[M, 2F] halves; backward
 * writes d(h) | d(gate) into dx12 [M, 2F]; bf16 rounding of the reference's bf16 tensor graph. */
int vpt_geglu_fwd(const void* x12, long ldx, int F, long M, void* out, void* stream);
int vpt_geglu_bwd(const void* dy, const void* x12, long ldx, int F, long M, void* dx12, long lddx, void* stream);
/* vpt_geglu_bwd (bit-identical dx12, dy [M][F] dense) and, in the same launch, the rank-16 LoRA projection of dx12
 * through up [2F][16] (the ff.net.0.proj adapter): vs[m][j] = bf16(alpha * dx12[m] . up[:, j]) -- within bf16
 * rounding of vpt_lora_proj(dx12, up, w_kmajor = 0) (per-chunk partial sums in a fixed order). F % 128 == 0.
 * tickets: (M + 15) / 16 u32, zero-filled when allocated and left zero by every launch (one zeroed buffer serves
 * every shape; one launch at a time per buffer); partials: vpt_geglu_lora_partials_bytes(M, F), 16-B aligned. */
long vpt_geglu_lora_partials_bytes(int M, int F);
int vpt_geglu_bwd_lora(const void* dy, const void* x12, long ldx, int F, int M, void* dx12, long lddx, const void* up,
                       void* vs, long ldvs, float alpha, void* tickets, void* partials, void* stream);
/* vpt_geglu_fwd (bit-identical out [M][F]) and, in the same launch, the rank-16 LoRA down-projection of out for the
 * Linear that consumes it (ff.net.2): ds[m][j] = bf16(alpha * out[m] . down[j, :]), down [16][F] -- within bf16
 * rounding of vpt_lora_proj(out, down, w_kmajor = 1). F % 128 == 0; tickets / partials as vpt_geglu_bwd_lora. */
int vpt_geglu_fwd_lora(const void* x12, long ldx, int F, int M, void* out, long ldo, const void* down, void* ds,
                       long ldds, float alpha, void* tickets, void* partials, void* stream);
/* NF4 weights in the bitsandbytes 0.48.2 layout (quant_type nf4, blocksize 64, compress_statistics):
 * packed uint8 [n/2] (first element in the high nibble), qabsmax uint8 [n/64], absmax2 f32 [ceil(n/64/256)],
 * code2 f32 [256] (signed dynamic map), offset f32 [1]. Dequant -> bf16 [n] in the original [out][in]
 * layout (replaces bnb dequantize_4bit inside Linear4bit.forward, src/modules/quant/bnb.py:37-129);
 * quantize (quantize_4bit, load time) uses absmax_scratch f32 [n/64]. */
int vpt_nf4_dequant(const void* packed, const void* qabsmax, const float* absmax2, const float* code2,
                    const float* offset, long n, void* out, void* stream);
/* Up to 16 NF4 tensors dequantised in one launch (a transformer block's LoRA bases before its forward or its
 * input-gradient GEMMs: bnb's per-call dequantize_4bit of each Linear4bit, batched); same values as
 * vpt_nf4_dequant. Each job: n % 64 == 0. */
typedef struct {
  const void* packed;
  const void* qabsmax;
  const float* absmax2;
  const float* code2;
  const float* offset;
  void* out;
  long n;
} VptNf4Job;
int vpt_nf4_dequant_batch(const VptNf4Job* jobs, int njobs, void* stream);
/* NF4 dequant-in-GEMM with the LoRA up-projection fused as one extra K tile (replaces, per QLoRA target,
 * LoRALinear.forward src/modules/peft/lora.py:92-104 = Linear4bit's dequantize_4bit + matmul
 * (src/modules/quant/bnb.py:37-129) + lora_up(lora_down(x)) * scale + add, and their input gradient).
 * W: the NF4 tensor above, [N_w][kw] (kw = input features). w_kmajor = 1 (forward): C[M][N] = A[M][K] .
 * Wd^T + bias + lora_a[M][r] . lora_b[N][r]^T with K = kw, N = N_w. w_kmajor = 0 (input gradient):
 * C[M][N] = A[M][K] . Wd + lora_a[M][r] . lora_b[r][N] with K = N_w, N = kw (N % 64 == 0). lora_a null:
 * no LoRA term; the caller pre-scales lora_a by alpha / rank. K % 64 == 0, 0 < r <= 64. The dequantised
 * weight never exists in HBM (bit-identical values to vpt_nf4_dequant, computed per tile in LDS).
 * out_mode 0 bf16 (resid: + bf16 residual, reference rounding) / 1 f32; alpha scales the accumulator. */
int vpt_gemm_nf4(const void* A, long lda, const void* packed, const void* qabsmax, const float* absmax2,
                 const float* code2, const float* offset, long kw, int w_kmajor, const void* lora_a, long lda2,
                 const void* lora_b, long ldb2, int r, void* C, long ldc, int M, int N, int K, const void* bias,
                 const void* resid, long ldr, int out_mode, float alpha, void* stream);
/* LoRA rank-16 skinny products (lora.py:92-104 lora_down / lora_up and their weight gradients):
 * lora_proj  Y[M][16] = alpha * X[M][K] . W^T, W = down [16][K] (w_kmajor = 1) or up [K][16] (0); K % 128 == 0.
 * lora_wgrad2 both adapter gradients of one LoRA Linear: g_up [N_out][16] (+)= alpha * dY^T . dS and
 * g_down [16][N_in] (+)= alpha * X^T . vS, f32; split-M partial sums in ws_up / ws_down
 * (lora_wgrad_workspace(M, N) bytes each), summed in a fixed order (deterministic). */
int vpt_lora_proj(const void* X, long ldx, const void* W, int w_kmajor, void* Y, long ldy, int M, int K, int r,
                  float alpha, void* stream);
/* G lora_proj in one launch: group g reads X + g * x_goff and W + g * w_goff (elements) and writes output columns
 * [16 g, 16 g + 16) of Y (the q / k / v adapters of one input: the downs stacked [3 * 16][K]; or of the three
 * column blocks of the q|k|v gradient: x_goff = dim, the ups stacked [3 * dim][16]). */
int vpt_lora_proj_grouped(const void* X, long ldx, long x_goff, const void* W, int w_kmajor, long w_goff, void* Y,
                          long ldy, int M, int K, int r, int G, float alpha, void* stream);
long vpt_lora_wgrad_workspace(int M, int N);
int vpt_lora_wgrad2(const void* dY, long lddy, const void* dS, long ldds, float* g_up, int n_out, const void* X,
                    long ldx, const void* vS, long ldvs, float* g_down, int n_in, int M, int accumulate, float alpha,
                    void* ws_up, void* ws_down, void* stream);
/* vpt_lora_wgrad2 in two steps, so that one launch reduces the adapter gradients of many targets:
 * _partial writes both gradients' split-M f32 slabs into ws_up / ws_down (vpt_lora_wgrad_workspace bytes each;
 * they must stay untouched until the reduce has run), vpt_lora_wgrad_splits(M, N) = the slabs of a width-N
 * gradient, and vpt_lora_wgrad_reduce_batch applies g (+)= alpha * (sum of the slabs in split order) for up
 * to 32 jobs in one launch (trans = 1: g stored [16][n], as g_down). Same results as vpt_lora_wgrad2. */
typedef struct {
  const float* part;
  float* g;
  int n, splits, trans, reserved;
} VptLoraReduceJob;
int vpt_lora_wgrad_splits(int M, int N);
int vpt_lora_wgrad2_partial(const void* dY, long lddy, const void* dS, long ldds, int n_out, const void* X, long ldx,
                            const void* vS, long ldvs, int n_in, int M, void* ws_up, void* ws_down, void* stream);
int vpt_lora_wgrad_reduce_batch(const VptLoraReduceJob* jobs, int njobs, float alpha, int accumulate, void* stream);
/* The slab half of up to 24 one-sided adapter-gradient jobs in ONE launch (a transformer block's ten targets,
 * deferred to the end of its backward): job i writes the split-M slabs of X[M][N]^T . S[M][16] into part
 * (vpt_lora_wgrad_workspace(M, N) bytes; vpt_lora_wgrad_splits(M, N) slabs), exactly as the matching side of
 * vpt_lora_wgrad2_partial (g_up: X = dY, S = dS; g_down: X = X, S = vS); reduced by vpt_lora_wgrad_reduce_batch. */
typedef struct {
  const void* X;
  long ldx;
  const void* S;
  long lds;
  float* part;
  int N, M;
} VptLoraWgradJob;
int vpt_lora_wgrad_partial_batch(const VptLoraWgradJob* jobs, int njobs, void* stream);
/* SpatialTransformer (src/models/sdxl/denoiser.py:283-365) around the transformer blocks:
 * GroupNorm(G, C, eps) on NCHW bf16 [B][C][HW] (f32 statistics mean / rstd [B*G] saved for the backward;
 * output NCHW bf16), its input gradient (affine weights frozen under QLoRA; dres: + a second NCHW gradient),
 * and dst[b][s][r] = src[b][r][s] (+ add) -- the NCHW <-> token-major permutes, the residual add fused (R, S
 * multiples of 8: any aspect-ratio bucket's stage HW). */
int vpt_groupnorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, int B, int C,
                      int G, long HW, float eps, void* stream);
int vpt_groupnorm_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const void* w,
                      const void* dres, void* dx, int B, int C, int G, long HW, void* stream);
int vpt_transpose_add(const void* src, const void* add, void* dst, int B, int R, int S, void* stream);
/* SDXL flow-matching step around the UNet (train/sdxl/flow_match.py:109-174):
 * vpt_flow_noise     prepare_scaled_noised_latents (src/modules/loss/flow_match.py:60-74) on bf16 latents x
 *                    [B][n_per_sample]: eps = bf16(bf16(randn) * noise_scale) from a counter RNG (seed), or the
 *                    caller's eps_in; z = t x + (1 - t) eps (clean_at_zero: (1 - t) x + t eps), f32 math,
 *                    bf16 out; t [B] f32 in (0, 1). eps_out receives the generated noise (needed by the loss).
 * vpt_velocity_loss  loss_with_predicted_velocity (flow_match.py:85-96): *loss = mean((v - bf16(eps - x))^2)
 *                    (f32, fixed-order block sums in part[vpt_velocity_loss_blocks()]); dv (optional) =
 *                    bf16(2 (v - target) / n), the gradient of the mean. n % 8 == 0.
 * vpt_sinusoid_embed get_timestep_embedding(vals, dim, flip_sin_to_cos=True, downscale_freq_shift=0)
 *                    (src/modules/timestep/embedding.py:10-62 via src/models/sdxl/denoiser.py:1117-1123) -> bf16.
 * vpt_space_to_depth NCHW bf16 [B][C][H][W] -> token-major [B][(H/r)(W/r)][C r r] (feature (c r + i) r + j =
 *                    pixel_unshuffle order); inverse = 1 maps tokens back to NCHW (pixel_shuffle), its adjoint. */
int vpt_flow_noise(const void* x, const float* t, long n_per_sample, int B, float noise_scale, int clean_at_zero,
                   unsigned long long seed, const void* eps_in, void* z, void* eps_out, void* stream);
int vpt_velocity_loss_blocks(void);
int vpt_velocity_loss(const void* v, const void* x, const void* eps, long n, void* dv, float* part, float* loss,
                      void* stream);
int vpt_sinusoid_embed(const float* vals, int R, int dim, void* out, void* stream);
int vpt_space_to_depth(const void* src, void* dst, int B, int C, int H, int W, int r, int inverse, void* stream);
/* Elementwise bf16: out = a + b (residual sums), out = s * a (LoRA scale gradient); n % 8 == 0. */
int vpt_add_bf16(const void* a, const void* b, long n, void* out, void* stream);
int vpt_scale_bf16(const void* a, long n, float s, void* out, void* stream);
/* out[r][c] = s * a[r][c] on a row-strided [rows][cols] block (in place allowed; cols, lda, ldo % 8 == 0): the
 * attention q pre-scale (vpt_attn_q_scale) of a q that is a column block of a fused q | k | v output. */
int vpt_scale_bf16_2d(const void* a, long lda, long rows, int cols, float s, void* out, long ldo, void* stream);
int vpt_nf4_quantize(const void* w, long n, const float* code2, void* packed, void* qabsmax, float* absmax2,
                     float* offset, float* absmax_scratch, void* stream);

/* ---- bucketed batch preparation ---------------------------------------------
 * One decoded uint8 RGB image [in_h][in_w][3] -> fp16 [3][out_h][out_w] batch slot: the reference's
 * PILToTensor -> ToDtype(float16, scale=True) -> Normalize(0.5, 0.5) -> ObjectCoverResize (bicubic,
 * antialias, to (scaled_h, scaled_w)) -> RandomCrop(top, left) chain, computed for the crop window only.
 * Replaces src/dataset/text_to_image.py:145-158,164-177,199-213 and src/dataset/transform.py:11-55
 * (torchvision / ATen antialiased bicubic on the CPU). workspace: *_workspace() bytes. */
long vpt_cover_resize_crop_workspace(int in_h, int in_w, int scaled_h, int scaled_w, int top, int out_h, int out_w);
int vpt_cover_resize_crop(const void* img, int in_h, int in_w, int scaled_h, int scaled_w, int top, int left,
                          int out_h, int out_w, void* workspace, void* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VPT_HIP_H */
