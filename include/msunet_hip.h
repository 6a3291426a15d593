/* msunet_hip.h -- C ABI of libmsunet_hip.so, the gfx950 (MI355X) kernels of the MS-UNet /
 * Swin training hot path.
 *
 * Plain pointers + sizes only (no torch types).  Every launch goes to `stream` (a
 * hipStream_t passed as void*), allocates nothing and never synchronises, so calls can be
 * captured into a hipGraph.  Device pointers are HIP device memory; scalars are host
 * values.  Return value: 0 on success, -2 bad shape/arguments, -3 unsupported mode,
 * -4 LDS budget exceeded, -1 launch error.
 *
 * dtype: 0 = f32 activations (parity mode), 1 = bf16 activations (training mode), 2 = f16
 * activations (the reference's torch.amp.autocast(float16) step, trainer.py:308).
 * Parameters, statistics and parameter gradients are always f32.
 *
 * The reference path is Python (network/model_parts.py, torchvision SwinTransformerBlock,
 * loss/DynamicLoss.py); each entry point names the reference operation it replaces.  The
 * reference has no FFI of its own -- the Python binding is semantic_segmentation_of_stylegan2_artifacts_amd/_lib.py
 * (ctypes) and INTEGRATION.md shows how a reference checkout would bind it.
 */
#ifndef MSUNET_HIP_H
#define MSUNET_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- LayerNorm family
 * nn.LayerNorm(C) over rows, with fused input addressing (mode):
 *   0 plain     torchvision block norm1/norm2 (model_parts.py:143-151 -> torchvision),
 *               PatchEmbed.norm (model_parts.py:213,224), MSUNetSys.norm / norm_up (:740-741,
 *               :813, :827)
 *   1 add       s = x + bscale[row / rows_per_sample] * b, y = LN(s); s stored to s_out.
 *               torchvision block residual `x + stochastic_depth(branch)` fused with the
 *               next norm
 *   2 merge     PatchMerging cat(x0,x1,x2,x3) + norm(4C) (model_parts.py:87-94); x is
 *               [B,H,W,Cin], C = 4*Cin
 *   3 d2s2      PatchExpand rearrange 'b h w (p1 p2 c) -> b (h p1) (w p2) c' + norm
 *               (model_parts.py:403-405); x is [B,H,W,4C]
 * mean / rstd: [rows] f32 saved for backward. */
int msu_layernorm_fwd(int dtype, int mode, const void* x, const void* b, const float* bscale,
                      long rows_per_sample, void* s_out, const float* gamma, const float* beta,
                      void* y, float* mean, float* rstd, long rows, int C, int H, int W, int Cin,
                      float eps, void* stream);
/* Backward: dx (scattered for merge / d2s2), optional dres added to dx (plain / add modes),
 * db = dx * bscale (add mode), dgamma/dbeta via nparts partial rows in `part`
 * ([nparts, 2, C] f32; nparts from msu_ln_part_blocks), written or (accumulate != 0) added
 * to dgamma/dbeta -- the latter lets a trainer accumulate straight into .grad. */
int msu_layernorm_bwd(int dtype, int mode, const void* dy, const void* x, const void* dres,
                      const float* gamma, const float* mean, const float* rstd, void* dx,
                      void* db, const float* bscale, long rows_per_sample, float* part,
                      int nparts, float* dgamma, float* dbeta, long rows, int C, int H, int W,
                      int Cin, int accumulate, void* stream);
/* As msu_layernorm_bwd with up to two more extra gradients (dres2, then dres3; null = none;
 * only with dres, plain / add modes) summed with dres in f32 before the one rounding of dx: a
 * stage input's other readers (skip fusion, PatchExpand Linear) hand their input gradients
 * to its first block's norm1 backward instead of autograd adds (model_parts.py:775-815). */
int msu_layernorm_bwd3(int dtype, int mode, const void* dy, const void* x, const void* dres,
                       const void* dres2, const void* dres3, const float* gamma, const float* mean,
                       const float* rstd, void* dx, void* db, const float* bscale, long rows_per_sample,
                       float* part, int nparts, float* dgamma, float* dbeta, long rows, int C, int H, int W,
                       int Cin, int accumulate, void* stream);
int msu_ln_part_blocks(long rows, int C);
/* nseg independent partial-row reductions in as few launches as fit (48 segments each):
 * out[j][i] (+)= sum over q < nparts[j] of part[j][q * stride[j] + i], i < n[j], in a fixed order.
 * Host arrays; n, stride multiples of 4, 16-B aligned rows.  With dgamma = dbeta = null,
 * msu_layernorm_bwd / _bwd3 write only their [nparts][2C] partials (dgamma row, then dbeta),
 * for such a batched reduction later (the deferred LayerNorm parameter gradients). */
int msu_colsum_batch(int nseg, const float* const* part, const long* stride, const int* nparts, const int* n,
                     float* const* out, int accumulate, void* stream);
/* 1 (default): the partial-row reductions of msu_layernorm_bwd / msu_head_bwd run inside the
 * kernel (its last blocks, in a fixed order); 0: a separate column-sum launch after it (A/B switch
 * MSU_TAIL).  Returns the previous mode. */
int msu_tail_reduce_mode(int mode);
int msu_reduce_rows(const float* part, int nparts, int n, long stride, float* out,
                    int accumulate, void* stream);

/* FinalPatchExpand_X4_V2.norm (model_parts.py:475) + bias-free 1x1 `output` conv
 * (model_parts.py:751, :846), num_classes == 1: logit[r] = <LN(z[r]), w> (f32). */
int msu_head_fwd(int dtype, const void* z, const float* gamma, const float* beta,
                 const float* w, float* logit, float* mean, float* rstd, long rows, int C,
                 float eps, void* stream);
int msu_head_bwd(int dtype, const float* dlogit, const void* z, const float* gamma,
                 const float* beta, const float* w, const float* mean, const float* rstd,
                 void* dz, float* part, int nparts, float* dgamma, float* dbeta, float* dw,
                 long rows, int C, void* stream);
/* accumulate != 0: dgamma / dbeta / dw are added to (the trainer's .grad: no autograd adds) */
int msu_head_bwd2(int dtype, const float* dlogit, const void* z, const float* gamma,
                  const float* beta, const float* w, const float* mean, const float* rstd,
                  void* dz, float* part, int nparts, float* dgamma, float* dbeta, float* dw,
                  long rows, int C, int accumulate, void* stream);

/* ---------------------------------------------------------------- window attention
 * torchvision shifted_window_attention core (called from SwinTransformerBlock at
 * model_parts.py:170 / :538): pad to 7 -> roll(-shift) -> 7x7 windows -> softmax(q k^T *
 * 32^-0.5 + B_rel + shift mask(-100)) -> dropout(p) -> @v -> reverse.  qkv: [B,H,W,3C]
 * (q|k|v, heads contiguous, head_dim 32), out: [B,H,W,C]; table [169, nh] f32 is
 * relative_position_bias_table; qkv_bias [3C] f32 supplies padded tokens' q,k,v.
 * Dropout masks: a counter hash of (seed, window, head, query i, key half) seeds a short
 * xorshift stream per query row (common.h); seed_dev (may be null) points at a device u64
 * mixed into the seed, so a replayed HIP graph draws new masks per step, and the backward reads
 * the forward's keep bits (keep buffer) or regenerates them from the same pair. */
long msu_win_count(int B, int H, int W);
/* f32 workspace elements (bf16: the per-head relative-bias image in MFMA C layout). */
long msu_win_attn_fwd_workspace(int dtype, int C, int nh);
/* u32 words of the dropout keep-bit buffer (16-bit dtypes: 128 per window x head, 0 for f32). */
long msu_win_attn_keep_words(int dtype, int B, int H, int W, int nh);
/* keep (may be null; 16-bit dtypes with p_drop > 0): the forward writes its dropout keep bits
 * there, the backward given the same buffer reads them instead of re-hashing. */
int msu_win_attn_fwd(int dtype, const void* qkv, const float* qkv_bias, const float* table,
                     void* out, float* workspace, int B, int H, int W, int C, int nh, int shift,
                     float p_drop, unsigned long long seed, const unsigned long long* seed_dev, void* keep,
                     void* stream);
long msu_win_attn_bwd_workspace(int dtype, int B, int H, int W, int C, int nh);
/* dqkv [B,H,W,3C]; dtable [169,nh] (overwritten); dqkv_bias_pad [3C]: padded tokens'
 * contribution to the qkv-bias gradient (overwritten). */
int msu_win_attn_bwd(int dtype, const void* qkv, const float* qkv_bias, const float* table,
                     const void* dout, void* dqkv, float* dtable, float* dqkv_bias_pad,
                     float* workspace, int B, int H, int W, int C, int nh, int shift,
                     float p_drop, unsigned long long seed, const unsigned long long* seed_dev, const void* keep,
                     void* stream);
/* As msu_win_attn_bwd; the parameter-gradient tail (relative-table and qkv-bias reductions)
 * runs on param_stream, ordered after the backward kernel by an event (null: on stream).
 * dqkv is complete when `stream` is; dtable / dqkv_bias_pad when `param_stream` is.
 * param_stream == (void*)-1: only the backward kernel is launched; the caller orders its own
 * stream after `stream` and issues msu_win_attn_bwd_tail (the HIP-graph-safe split).
 * 16-bit dtypes: table == null means the workspace is the forward's (msu_win_attn_fwd /
 * msu_win_attn_qkv_fwd2 with a workspace of max(fwd, bwd) floats), whose relative-bias image and
 * bias rows, built from the same table and qkv bias, are reused instead of rebuilt. */
int msu_win_attn_bwd2(int dtype, const void* qkv, const float* qkv_bias, const float* table,
                      const void* dout, void* dqkv, float* dtable, float* dqkv_bias_pad,
                      float* workspace, int B, int H, int W, int C, int nh, int shift,
                      float p_drop, unsigned long long seed, const unsigned long long* seed_dev, const void* keep,
                      void* stream, void* param_stream);
/* The parameter-gradient tail of msu_win_attn_bwd2 (dtable, dqkv_bias_pad) from the
 * workspace partials its backward kernel left, on `stream`. */
int msu_win_attn_bwd_tail(int dtype, float* workspace, float* dtable, float* dqkv_bias_pad, int B, int H, int W,
                          int C, int nh, void* stream);
/* As msu_win_attn_bwd_tail; accumulate != 0 adds into dtable / dqkv_bias_pad (a trainer's .grad)
 * instead of overwriting them. */
int msu_win_attn_bwd_tail2(int dtype, float* workspace, float* dtable, float* dqkv_bias_pad, int B, int H, int W,
                           int C, int nh, int accumulate, void* stream);

/* ---------------------------------------------------------------- refine convs
 * FinalPatchExpand_X4_V2.refine1 / refine2 (model_parts.py:447-448, :468-471): 3x3, pad 1,
 * NHWC implicit GEMM on MFMA.  in_mode bit0: GELU on the loaded input (model_parts.py:460,
 * :469); bit1: input is the pre-depth-to-space [B,H/4,W/4,16*Cin] expand output
 * (model_parts.py:464-465).  Wt: [9][Cout][roundup(Cin,32)] in the activation dtype. */
int msu_conv3x3_fwd(int dtype, int in_mode, const void* X, const void* Wt, const float* bias,
                    void* Y, int B, int H, int W, int Cin, int Cout, void* stream);
/* As msu_conv3x3_fwd; Y2 (may be null; only with in_mode bit0 clear) receives GELU(Y) from
 * the same epilogue, so the next refine conv loads its activation instead of converting its
 * halo (model_parts.py:469: refine2(act(refine1(.)))). */
int msu_conv3x3_fwd2(int dtype, int in_mode, const void* X, const void* Wt, const float* bias,
                     void* Y, void* Y2, int B, int H, int W, int Cin, int Cout, void* stream);
/* dX = conv(dY, Wflip) * GELU'(S) through the same input map (out_mode as in_mode);
 * Wflip [9][Cin][roundup(Cout,32)], Wflip[t][ci][co] = W[co][ci][8-t]. */
int msu_conv3x3_dgrad(int dtype, int out_mode, const void* dY, const void* Wflip, const void* S,
                      void* dX, int B, int H, int W, int Cin, int Cout, void* stream);
/* 1 (default): the 96-channel refine-conv kernel takes its tiles from a device queue (per-stream
 * counter slot, reset by the launch's last workgroup), so workgroups that start late beside
 * the side stream's kernels take fewer tiles; 0: the static schedule (A/B switch MSU_CONV_DYN).
 * Returns the previous mode. */
int msu_conv_mode(int mode);
long msu_conv3x3_wgrad_workspace(int nchunk, int Cin, int Cout, int dtype, int unused);
/* dW [Cout][Cin][3][3] f32, db [Cout] f32 (deterministic partial-sum reduction). */
int msu_conv3x3_wgrad(int dtype, int in_mode, const void* X, const void* dY, float* dW, float* db,
                      float* workspace, void* unused, int nchunk, int B, int H, int W, int Cin,
                      int Cout, void* stream);
/* The same with accumulate != 0: dW and db are added to (the trainer's .grad on the side stream:
 * no separate adds). */
int msu_conv3x3_wgrad2(int dtype, int in_mode, const void* X, const void* dY, float* dW, float* db,
                       float* workspace, int nchunk, int B, int H, int W, int Cin, int Cout, int accumulate,
                       void* stream);

/* ---------------------------------------------------------------- fused qkv Linear + window attention
 * Stage 0 of the Swin block (C = 96, 3 heads; model_parts.py:166-170 -> torchvision's qkv Linear and
 * shifted_window_attention in one kernel): out[B,H,W,C] = attention(x W_qkv^T + b_qkv), x the LN1
 * rows (16-bit), W_qkv [3C][C] 16-bit, b_qkv f32.  qkv_out (nullable) receives x W^T + b (the qkv
 * Linear's output, for the backward); dropout / keep bits / aux workspace as msu_win_attn_fwd. */
int msu_win_attn_qkv_supported(int C, int nh);
int msu_win_attn_qkv_fwd(int dtype, const void* x, const void* w_qkv, const float* b_qkv, const float* table,
                         void* out, void* qkv_out, void* keep, float* workspace, int B, int H, int W, int C, int nh,
                         int shift, float p_drop, unsigned long long seed, const unsigned long long* seed_dev,
                         void* stream);
/* The whole attention half of the block: out = (attention(x W_qkv^T + b_qkv)) W_proj^T + b_proj
 * (model_parts.py:166-170 with the proj Linear); o_out (nullable) receives the attention output
 * before proj (the proj weight gradient's input), qkv_out as above. */
int msu_win_attn_qkv_fwd2(int dtype, const void* x, const void* w_qkv, const float* b_qkv, const float* table,
                          const void* w_proj, const float* b_proj, void* out, void* o_out, void* qkv_out, void* keep,
                          float* workspace, int B, int H, int W, int C, int nh, int shift, float p_drop,
                          unsigned long long seed, const unsigned long long* seed_dev, void* stream);

/* ---------------------------------------------------------------- Linear weight gradient
 * Every nn.Linear on the path (torchvision block qkv / proj / mlp.0 / mlp.3,
 * PatchMerging.reduction model_parts.py:72, PatchExpand.expand :379, concat_back_dim
 * :639-641, FinalPatchExpand_X4_V2.expand :443, PatchEmbed.proj :211 as im2col GEMM):
 * dW[N][K] = sum_m dY[m][n] X[m][k], db[n] = sum_m dY[m][n] (db may be null), split over M
 * on MFMA; workspace f32 elements from msu_wgrad_workspace. */
int msu_wgrad_splits(long M, int N, int K);
long msu_wgrad_workspace(long M, int N, int K);
int msu_linear_wgrad(int dtype, const void* dY, const void* X, float* dW, float* db, float* workspace,
                     long M, int N, int K, int accumulate, void* stream);
/* Same, with dW a column slice of a wider row-major gradient (row stride ldw >= K): each input
 * half of a skip-fusion Linear (concat_back_dim, model_parts.py:639-641, applied to
 * torch.cat([x, skip], -1) at :792-794, :804-806, :823-824) accumulates straight into its
 * columns of the weight's gradient. */
int msu_linear_wgrad_ld(int dtype, const void* dY, const void* X, float* dW, long ldw, float* db,
                        float* workspace, long M, int N, int K, int accumulate, void* stream);

/* ---------------------------------------------------------------- Linear backward in one pass
 * Stage-0 Linears of the Swin block (qkv, proj, mlp.0, mlp.3; model_parts.py:143-151, called at
 * :170 / :538; (K, N) = (in, out) features in {(96, 288), (96, 96), (96, 384), (384, 96)}):
 * dX = dY . W (times GELU'(H) when H != null: mlp.3's input gradient through mlp.1, (384, 96)
 * only), dW[N][K] (+)= dY^T X and db[N] (+)= column sums of dY in ONE read of dY (replaces the
 * input-gradient GEMM plus msu_linear_wgrad).  Wt = W^T [K][N] 16-bit; dW / db f32, added to
 * when accumulate != 0 (db may be null); workspace f32 elements from msu_linear_bwd_workspace. */
int msu_linear_bwd_supported(long M, int K, int N);
long msu_linear_bwd_workspace(long M, int K, int N);
int msu_linear_bwd(int dtype, const void* dY, const void* X, const void* Wt, const void* H, void* dX, float* dW,
                   float* db, float* workspace, long M, int K, int N, int accumulate, void* stream);

/* ---------------------------------------------------------------- Linear forward / input gradient
 * Token GEMM (dtype 1 bf16 / 2 f16 in and out, f32 accumulate) for the same Linears as
 * msu_linear_wgrad:
 * Y[M][N] = epi(A[M][K] . W[N][K]^T + bias[N]); input gradients pass W^T ([K][N]).
 *   epi 0  plain, optional bias; A2 != null: A's columns [K1, K) come from A2 ([M][K-K1]) --
 *          the skip-fusion torch.cat([x, skip], -1) -> concat_back_dim (model_parts.py:792-794,
 *          :804-806, :823-824) without the concatenated copy (needs bias);
 *   epi 1  torchvision MLP mlp.0 + mlp.1 (Linear -> GELU): Y = H = A.W^T + b, Y2 = GELU(H);
 *   epi 2  input gradient of mlp.3 through mlp.1: Y = (A.W^T) * GELU'(H) (no bias).
 * msu_tok_gemm_supported() says whether a shape is covered (N % 32 == 0, K % 48 or 128 == 0
 * and an LDS plan exists), msu_tok_gemm_supported_epi() the same for one epilogue (the GELU
 * epilogues cap the column chunk); uncovered shapes are the caller's to route to a library GEMM. */
int msu_tok_gemm_supported(long M, int N, int K);
int msu_tok_gemm_supported_epi(long M, int N, int K, int epi);
int msu_tok_gemm(int dtype, const void* A, const void* A2, int K1, const void* W, const float* bias, void* Y,
                 void* Y2, const void* H, long M, int N, int K, int epi, void* stream);
int msu_tok_gemm_plan(long M, int N, int K, long* out6);
/* Persistent tiled NT GEMM (128 x 128 tiles, LDS-DMA double buffering, one flat K-step sequence per
 * workgroup) for the stage 1-3 Linears, whose wide weights do not fit the token GEMM's LDS: same
 * Y / epi semantics as msu_tok_gemm.  Covered: N % 32 == 0, K % 64 == 0. */
int msu_nt_gemm_supported(long M, int N, int K);
/* Tile msu_nt_gemm picks for an M x N output (rows * 1000 + columns; 128/256 x 128/192/256),
 * + 1000000 when the ping-pong kernel (gemm_pp.h) takes it. */
int msu_nt_gemm_plan(long M, int N);
/* bit 0: the ping-pong kernel where the shape tiles exactly (default off: the persistent
 * 2-barrier kernel everywhere; A/B switch MSU_NT_PP); bits 1-2: a forced tile form (timing
 * tools); bit 3: the 256 x 192 A3W2 ring; bit 4: the two-stage kernel claims its tiles from a
 * per-XCD device queue (opt-in MSU_NT_DYN=1: measured slower).  Returns the previous mode. */
int msu_nt_gemm_mode(int mode);
int msu_nt_gemm(int dtype, const void* A, const void* W, const float* bias, void* Y, void* Y2, const void* H,
                long M, int N, int K, int epi, void* stream);
/* Plain epilogue with the split-A input of msu_tok_gemm: A's columns [K1, K) from A2 (K1 % 64 == 0):
 * the wide skip fusions (concat_back_dim at stages 1-3, model_parts.py:792-794, :804-806, :823-824). */
int msu_nt_gemm_cat(int dtype, const void* A, const void* A2, int K1, const void* W, const float* bias, void* Y,
                    long M, int N, int K, void* stream);
/* The same with the weight given as Wk[K][N]: Y = epi(A . Wk + bias).  The input gradient of a
 * Linear, dX = dY . W with the forward weight W[N_fwd][K_fwd] (K = N_fwd, N = K_fwd) read in place
 * (transposed LDS fragment reads) instead of a W^T copy per call (torch F.linear backward,
 * replaced for the stage 1-3 Linears of model_parts.py:143-151, :72, :379, :639-641). */
int msu_nt_gemm_kn(int dtype, const void* A, const void* Wk, const float* bias, void* Y, void* Y2, const void* H,
                   long M, int N, int K, int epi, void* stream);

/* ---------------------------------------------------------------- streaming ops
 * nn.GELU() (exact erf): torchvision MLP activation, FinalPatchExpand_X4_V2.act. */
/* Stage-0 Swin MLP forward, fused (csrc/mlp_fused.hip; replaces mlp.0 -> GELU -> mlp.3 of
 * torchvision's block, model_parts.py:538): y = W2 GELU(W1 x + b1) + b2 with the hidden
 * activation kept on chip; h (nullable) receives the 16-bit pre-activation W1 x + b1 [M][384]
 * for the backward (training; null on the no-grad path: the reference's discarded branches
 * layers_cent1[-1] / layers_cent2[-1], model_parts.py:795 / :807, and evaluation).  x, y [M][96],
 * w1 [384][96], w2 [96][384] in the 16-bit format dtype, b1 / b2 f32, all 16-B aligned.
 * msu_mlp_fused_supported(C, Hd): 1 for C = 96, Hd = 384.  Returns 0, -2 (unsupported).
 * The backward's mlp.3 step is msu_linear_bwd with X = null and H = h. */
int msu_mlp_fused_supported(int C, int Hd);
/* No-grad second half of a stage-0 block: s_out = a + bscale[sample] * br (16-bit; bscale null = 1,
 * rows_per_sample rows per sample), y = mlp(LN(s) with gamma / beta / eps) -- the residual-add
 * LayerNorm (norm2) and the fused MLP above in one kernel, the normalised rows on chip. */
int msu_add_ln_mlp_fwd(int dtype, const void* a, const void* br, const float* bscale, long rows_per_sample,
                       const float* gamma, const float* beta, float eps, const void* w1, const float* b1,
                       const void* w2, const float* b2, void* s_out, void* y, long M, int C, int Hd, void* stream);
int msu_mlp_fused_fwd(int dtype, const void* x, const void* w1, const float* b1, const void* w2, const float* b2,
                      void* y, void* h, long M, int C, int Hd, void* stream);
int msu_gelu_fwd(int dtype, const void* x, void* y, long n, void* stream);
int msu_gelu_bwd(int dtype, const void* x, const void* dy, void* dx, long n, void* stream);
/* PatchEmbed.proj im2col (model_parts.py:211, :222): img [B,Cin,H,W] f32 ->
 * [B*(H/p)*(W/p), Cin*p*p] in (c, ky, kx) order. */
/* Batched 16-bit transpose: for each of nent entries {src offset, dst offset, N, K, first tile}
 * (int64, device memory; element offsets into src / dst; N, K multiples of 8; first tiles
 * ascending, entry e owning ceil(N/64) * ceil(K/64) tiles) dst[K][N] = src[N][K].  The
 * trainer's per-step transposed bf16 weight shadow: the Linear input gradients dX = dY . W
 * (model_parts.py:143-151 Linears' backward) read W^T with the forward GEMM's layout. */
int msu_transpose16_multi(const void* src, void* dst, const long long* table, int nent, int ntiles,
                          void* stream);
/* out = a + b * scale[i / per_sample] (a may be NULL: out = b * scale[...]); n, per_sample
 * multiples of 4.  The Swin block's residual add with StochasticDepth's per-sample scale
 * (torchvision SwinTransformerBlock: x + stochastic_depth(f(x))) and its branch gradient. */
int msu_residual(int dtype, const void* a, const void* b, const float* scale, void* out, long n, long per_sample,
                 void* stream);
int msu_patchify(int dtype, const float* img, void* out, int B, int Cin, int H, int W, int p,
                 void* stream);

/* DynamicLoss (loss/DynamicLoss.py:82-111): per-sample BCE-with-logits mean + Tversky
 * (smooth 1e-6) on non-empty masks, mixed (1-m)*bce + m*tversky, mean over samples;
 * binarise target at 127.5 iff max(target) > 1.  logits [B,N], target [B,N] f32.
 * loss[0] = loss, loss[1] = binarised flag; coef [4B] and part [B*nblk*12] scratch. */
int msu_dynloss_nblk(long N);
int msu_dynloss_fwd(int dtype, const void* logits, const float* target, int B, long N,
                    float alpha, float beta, float mix, float* part, int nblk, float* loss,
                    float* coef, void* stream);
/* dlogits [B,N] f32 = gout[0] * d loss / d logits (gout may be null = 1). */
int msu_dynloss_bwd(int dtype, const void* logits, const float* target, const float* coef,
                    const float* loss, const float* gout, int B, long N, float alpha, float beta,
                    float mix, float* dlogits, void* stream);
/* The same with the binarised flag in its own float (flag[0]): the loss is then a 1-element
 * buffer of its own (the 0-dim autograd output, no select and its backward's fill + copy). */
int msu_dynloss_fwd2(int dtype, const void* logits, const float* target, int B, long N,
                     float alpha, float beta, float mix, float* part, int nblk, float* loss, float* flag,
                     float* coef, void* stream);
int msu_dynloss_bwd2(int dtype, const void* logits, const float* target, const float* coef,
                     const float* flag, const float* gout, int B, long N, float alpha, float beta,
                     float mix, float* dlogits, void* stream);
/* fwd2 that also sets zero_out[0] = 0 (nullable) from its single-block final launch: the trainer's
 * non-finite flag is reset there each step, before the check after backward (no fill launch). */
int msu_dynloss_fwd3(int dtype, const void* logits, const float* target, int B, long N,
                     float alpha, float beta, float mix, float* part, int nblk, float* loss, float* flag,
                     float* coef, float* zero_out, void* stream);

/* Validation metrics (scripts/validation_functions.py:37-309): per image, p = sigmoid(logit),
 * pred_bin = p > threshold (:106-107), gt = label > 0 (:108).  out [B][12] f64 = sum(p g),
 * sum(p^2), sum(g), sum(p), soft fp / fn / tn (:219-222, :291-294), binary tp / fp / fn / tn
 * (:219-222, :267-270), 0 -- the host forms soft / binary Dice, IoU, recall, precision,
 * accuracy, FPR and Score (calculate_metrics_fake :247-309, calculate_metrics_real :214-244,
 * :180).  part [B * nblk * 12] f32 scratch, nblk from msu_metrics_nblk. */
int msu_metrics_nblk(long N);
int msu_seg_metrics(int dtype, const void* logits, const float* label, int B, long N, float threshold,
                    float* part, int nblk, double* out, void* stream);

/* AdamW step (trainer.py:143-152; torch.optim.AdamW, amsgrad=False) over a flat f32
 * parameter range; optional grad unscale (inv_scale) and skip-on-found_inf (GradScaler). */
int msu_adamw(float* p, const float* g, float* m, float* v, long n, float lr, float beta1,
              float beta2, float eps, float weight_decay, int step, const float* inv_scale,
              const float* found_inf, void* stream);
/* As msu_adamw with the per-step scalars in device memory, hyper = {lr, step} (f64): the
 * launch holds no host scalar that changes per step (HIP-graph replayable); scalars are
 * formed in double like torch.optim.AdamW's.  Skips when found_inf[0] != 0 (GradScaler.step,
 * trainer.py:182,315-316). */
int msu_adamw_dev(float* p, const float* g, float* m, float* v, long n, const double* hyper, double beta1,
                  double beta2, double eps, double weight_decay, const float* inv_scale, const float* found_inf,
                  void* stream);
/* msu_adamw_dev that also writes the updated parameters' 16-bit shadow (shadow_dtype 1 bf16 /
 * 2 f16; shadow null = none) and zeroes g after reading it (zero_grad; a skipped step zeroes it
 * too): the step's gradient reset and shadow refresh in the optimizer's own pass
 * (trainer.py:315-316 optimizer.step + zero_grad). */
int msu_adamw_dev2(float* p, float* g, float* m, float* v, long n, const double* hyper, double beta1, double beta2,
                   double eps, double weight_decay, const float* inv_scale, const float* found_inf, void* shadow,
                   int shadow_dtype, int zero_grad, void* stream);
/* hyper[1] += 1 unless found_inf[0] != 0 (the skipped step does not count, as torch's AdamW
 * `step` state is not advanced when GradScaler skips optimizer.step). */
int msu_step_advance(double* hyper, const float* found_inf, void* stream);
/* flag[0] = 1 if any element of x (x0[0:n0], x1[0:n1]) is inf/NaN; flag zeroed by the caller
 * (GradScaler's non-finite check, torch._amp_foreach_non_finite_check_and_unscale_). */
int msu_nonfinite(const float* x, long n, float* flag, void* stream);
int msu_nonfinite2(const float* x0, long n0, const float* x1, long n1, float* flag, void* stream);
int msu_cast(int dtype, const float* x, void* y, long n, void* stream);
/* The refine conv's f32 weight W [Cout][Cin][3][3] (model_parts.py:447-448) in the conv kernels'
 * layouts, in the activation dtype: flip 0 -> Wt of msu_conv3x3_fwd/_fwd2 [9][Cout][roundup(Cin,32)];
 * flip 1 -> Wflip of msu_conv3x3_dgrad [9][Cin][roundup(Cout,32)] (zero padding). */
int msu_conv3x3_weight(int dtype, const float* W, void* out, int Cout, int Cin, int flip, void* stream);

/* ---------------------------------------------------------------- input pipeline
 * The per-sample CPU transform of the reference's DataLoader workers (dataset/dataset.py:20-95
 * RandomGenerator: albumentations ToGray / RandomBrightnessContrast / HueSaturationValue /
 * OneOf(RandomGamma, GaussianBlur), random_flip, /255 and label > 127; :97-119 DataPrepartion)
 * as one pass over a decoded uint8 batch.  img [B, H, W, 3] u8 (PIL RGB), label [B, H, W] u8
 * (PIL "L") or null; ops [B][2] i32 = (bits: 1 gray, 2 brightness/contrast, 4 HSV, 8 gamma,
 * 16 hflip; blur ksize 0/3/5) and luts [B][5][256] u8 (brightness/contrast, hue, saturation,
 * value, gamma; built on the host as albumentations builds them), both null for normalisation
 * only; out [B, 3, H, W] f32 = u8/255, out_label [B, H, W] f32 in {0, 1}. */
int msu_augment_batch(const unsigned char* img, const unsigned char* label, const int* ops,
                      const unsigned char* luts, float* out, float* out_label, int B, int H, int W,
                      void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MSUNET_HIP_H */
