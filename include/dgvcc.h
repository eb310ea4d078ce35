/*
 * dgvcc.h — C-ABI of libdgvcc_hip.so, the MI355X (gfx950) kernels behind the
 * DGVCC crowd-density training hot path.
 *
 * Conventions (SURVEY.md §8b "C-ABI exports"):
 *   - every entry point returns int: DG_OK (0) or a negative DG_ERR_* code;
 *   - the library never allocates or owns tensors: callers pass device pointers
 *     (PyTorch caching allocator), sizes and a hipStream_t (as void*);
 *     workspaces are queried (`*_workspace`) then caller-allocated;
 *   - all launches are stream-ordered on the caller's stream; no implicit sync;
 *   - activations are NHWC with an explicit pixel stride `ld` (elements between
 *     consecutive pixels) so channel slices of concatenation buffers are
 *     addressed in place (replaces torch.cat, models/models.py:72,76,84);
 *   - dtype: DG_F32 (parity mode, exact-f32 MFMA), DG_BF16 (perf mode, bf16
 *     storage + bf16 MFMA, f32 accumulation/statistics) or DG_F16 (fp16 storage +
 *     f16 MFMA, f32 accumulation/statistics; configs/qnrf_final.yml's precision).
 *   - the library holds no tensors and no device memory and is safe to call from any
 *     thread; the pre-split f32 filter planes of the split-math convolutions live in
 *     the caller's workspace (dg_conv_fwd_workspace).
 */
#ifndef DGVCC_H
#define DGVCC_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define DG_OK 0
#define DG_ERR_INVALID (-1)     /* bad argument (null pointer, negative size, ...) */
#define DG_ERR_UNSUPPORTED (-2) /* shape/dtype combination not implemented */
#define DG_ERR_HIP (-3)         /* HIP launch/runtime error */

#define DG_F32 0
#define DG_BF16 1
#define DG_F16 2

/* ---- library ----------------------------------------------------------- */
int dg_version(void); /* returns DGVCC_ABI_VERSION */
/* writes the 16-hex-digit content hash of the sources the library was built from
 * (the csrc .hip/.h files and this header; dgvcc_amd/srchash.py) into out (cap > 16 bytes);
 * returns its length, or -1.  The Python binding refuses a library whose hash differs
 * from the sources beside it. */
int dg_source_hash(char* out, int cap);
/* diagnostic hook: with DGVCC_PSPLIT_STAMP set, the f16 x3 256-pixel pre-split forward runs its
 * stamp build and writes 8 u64 per wave (grid x 8 waves x 8) into buf: cycles in the DMA wait,
 * barrier, prologue, MFMA block and epilogue, K-steps, tiles, K-steps per tile (tools/stamp_psplit.py).
 * buf = NULL turns it off. */
int dg_debug_stamps(void* buf, int64_t bytes);
/* test hook: 1/0 force the persistent pipelined conv forward on/off, -1 = DGVCC_PERSIST default */
int dg_set_persist(int mode);
/* f32 GEMM arithmetic of the DG_F32 convolutions: 0 = v_mfma_f32_16x16x4_f32;
 * 1 = exact 3-way bf16 split of both operands (x = h0 + h1 + h2), six
 * v_mfma_f32_16x16x32_bf16 products per block, f32 accumulation (the truncated parts
 * drop terms up to ~2^-20 |x*y|, typically ~2^-22, one-sided; see dg_common.h).  Default from DGVCC_F32_MATH (exact | split | h16), else 2. */
int dg_set_f32_math(int mode);
/* mode 2 (the default since ABI 3; DGVCC_F32_MATH=split selects 1) = 1 with the "f16 x3"
 * arithmetic where a kernel has it (the pre-split forward/dgrad, the 3-tap Cout = 64 forward,
 * the split weight gradients):
 * each f32 operand scaled by a power of two into f16 range and cut into two f16 parts by
 * nearest rounding, three v_mfma_f32_16x16x32_f16 products per block (hi*hi + hi*lo + lo*hi),
 * f32 accumulation, exact rescale (dropped terms <= ~2^-21 |x*y|, two-sided; dg_common.h). */
int dg_get_f32_math(void);
#define DGVCC_ABI_VERSION 8 /* 8: dg_pack_weight_flip; 7: dg_bn_apply_pair / dg_bn_apply_pool_pair / dg_bn_bwd_pair / dg_bn_bwd_pool_pair write the f16 x3 pair image of their f32 output and dg_conv_fwd_pair reads it (dg_bn_workspace grew for the backward ones); 6: operand maxima with channels ([1 + C] floats, rounded up to 4, for f32 producers, dg_amax and the f32 dg_softmax_head_bwd; the f16 x3 weight gradients take per-channel scales from them); 5: amax (max |gL_1|, |gL_2|) on dg_softmax_head_bwd; 4: amax on dg_bn_add_apply / dg_instnorm_apply / dg_instnorm_bwd, operand maxima on dg_conv2d_wgrad; 3: xamax on the f32 conv entries, dg_amax; 2: dg_conv_fwd_bnbwd takes (workspace, ws_bytes) */

/* ---- convolution (implicit GEMM on MFMA) --------------------------------
 * Replaces nn.Conv2d forward/backward inside vgg16_bn.features
 * (models/models.py:35-38), ConvBlock (models/models.py:8-21) and the cls head
 * (models/models.py:238-243).  Stride 1, "same" padding (2*pad == R-1).
 * x: [N,H,W,C] (pixel stride ldx), w: [Cout][R][S][C] packed (dg_pack_weight),
 * y: [N,H,W,Cout] (pixel stride ldy).  C % 64 == 0 (bf16) / C % 32 == 0 (f32),
 * Cout % 64 == 0.  bias (f32 [Cout]) may be NULL.  accumulate != 0 adds into y. */
int dg_conv_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C,
                const void* w, int Cout, int R, int S, int pad, const float* bias,
                void* y, int64_t ldy, int accumulate, void* stream);

/* dX = conv_transpose(dY, W): dy [N,H,W,Cout] (lddy), wflip workspace of
 * R*S*C*Cout elements of dtype (caller-allocated), dx [N,H,W,C] (lddx). */
int dg_conv_dgrad(int dtype, const void* dy, int64_t lddy, int N, int H, int W, int Cout,
                  const void* w, int C, int R, int S, int pad, void* wflip,
                  void* dx, int64_t lddx, int accumulate, void* stream);

/* Forward conv (bf16, pipelined kernels) with the BatchNorm2d statistics of the stored
 * output computed in the epilogue: part[dg_conv_stats_rows][3][Cout] = (n, mean, M2) per
 * 256-pixel tile, for dg_bn_part_finalize (replaces the statistics pass over y).
 * Returns DG_ERR_UNSUPPORTED (nothing launched) where only the register-staged kernel
 * serves the shape; the caller then runs dg_conv_fwd + dg_bn_fwd_train. */
int64_t dg_conv_stats_rows(int N, int H, int W);
/* rows of (n, mean, M2) BN partials a dg_conv_fwd_ex launch of this shape writes: one per
 * tile of 256 output pixels; on the pre-split f32 kernel (DG_F32, split math) one per tile of
 * 192 pixels, or of 256 where the 256-channel launch takes 256-pixel tiles (DGVCC_PSPLIT_TALL) */
int64_t dg_conv_stats_rows_ex(int dtype, int N, int H, int W, int C, int64_t ldx, int Cout, int R, int S);
/* rows of the BN-backward partials part[rows][3][C] that dg_conv_fwd_bnbwd writes for an
 * output-gradient shape (N, H, W, C = the gradient's channels) and Cout = the consumer's input
 * channels (the dgrad-epilogue launches never take the 256-pixel tiles) */
int64_t dg_conv_bnpart_rows_ex(int dtype, int N, int H, int W, int C, int64_t ldx, int Cout, int R, int S);
int dg_conv_fwd_stats(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C,
                      const void* w, int Cout, int R, int S, int pad, const float* bias,
                      void* y, int64_t ldy, float* part, void* stream);
/* Workspace (bytes, 0 = none needed) of dg_conv_fwd_ex / dg_conv_fwd_bn_eval /
 * dg_conv_fwd_bnbwd: 16-bit, the split-K partials of a shape whose tile grid cannot fill the
 * GPU (deep layers at small batch); DG_F32, the pre-split filter planes of the split-math
 * kernels (Cout*R*S*C*6 bytes) and, after them (256-B aligned), room for the f16 x3 pixel
 * operand pre-split once per launch (N*H*W*C*4 bytes; used by 3x3 launches whose Cout spans
 * several output-channel tiles).  With less (or none, as dg_conv_fwd passes) an f32 launch
 * splits in-kernel (planes but no pixel room) or takes a kernel that splits the filter per
 * wave (no planes); the statistics row counts of dg_conv_stats_rows_ex assume the planes. */
int64_t dg_conv_fwd_workspace(int dtype, int N, int H, int W, int C, int Cout, int R, int S);
/* dg_conv_fwd + dg_conv_fwd_stats in one entry: part may be NULL; with a workspace of
 * dg_conv_fwd_workspace bytes the K loop is split over blocks and reduced deterministically
 * (bias, accumulate and the statistics partials in the reduce pass). */
int dg_conv_fwd_ex(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                   int Cout, int R, int S, int pad, const float* bias, void* y, int64_t ldy,
                   int accumulate, float* part, void* workspace, int64_t ws_bytes, const float* xamax,
                   void* stream);
/* dg_conv_fwd_ex (DG_F32) whose input x also comes as xpair, the f16 x3 pair image its producer wrote
 * (dg_bn_apply_pair / dg_bn_apply_pool_pair), with xbound the producer's *pbound: the f16 x3 pre-split
 * forward reads the pair (no pass over x to split it, no split in the kernel) with its scale from
 * xbound; launches on the other kernels read x and xamax as dg_conv_fwd_ex.  xpair = xbound = NULL:
 * dg_conv_fwd_ex.  Same statistics rows and workspace as dg_conv_fwd_ex. */
int dg_conv_fwd_pair(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                     int Cout, int R, int S, int pad, const float* bias, void* y, int64_t ldy,
                     int accumulate, float* part, void* workspace, int64_t ws_bytes, const float* xamax,
                     const void* xpair, const float* xbound, void* stream);
/* xamax (f32 entries, f16 x3 arithmetic): NULL, or operand maxima of x (dg_amax, or the kernel that
 * produced x): word 0 >= max |x| over the operand, and -- for the weight-gradient entries, which
 * scale per channel -- words 1 .. C >= max |x| over each channel (channel c of the slice x points
 * at in word 1 + c).  The forward / dgrad entries read word 0 only.  NULL makes the library take
 * one read pass over x for them.  A maximum below the true one is undefined behaviour (f16
 * overflow). */
/* out[0 .. C] (device f32): out[0] = max |x| over the M x C f32 rows of pixel stride ldx, out[1 + c]
 * = max over channel c (C % 4 == 0, C <= 2048).  Every operand-maxima buffer the library writes
 * (here and the producers' amax) holds 1 + C words rounded up to a multiple of 4: the zeroing
 * before the pass writes them all. */
int dg_amax(int dtype, const void* x, int64_t ldx, int64_t M, int C, float* out, void* stream);
/* y = (relu_out > 0) ? conv1x1(x, w) + y : 0: the accumulating dgrad of a bottleneck's conv1 (w
 * flipped, dg_flip_weight) whose input relu_out is the previous block's ReLU output
 * (models/SW/backbones/resnet.py:77 Bottleneck.forward's final relu, autograd's ReLU backward),
 * so that ReLU's backward needs no pass of its own; equals dg_conv_fwd_ex(accumulate = 1)
 * followed by dg_relu_bwd on y bit for bit.  relu_out: y's dtype and rows (ldr elements).
 * Workspace as dg_conv_fwd_ex; DG_ERR_UNSUPPORTED (nothing launched) for the 16-bit shapes that
 * launch splits over K with this workspace. */
int dg_conv_fwd_acc_relu(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                         int Cout, const void* relu_out, int64_t ldr, void* y, int64_t ldy, void* workspace,
                         int64_t ws_bytes, const float* xamax, void* stream);
/* Eval-mode Conv + BatchNorm(running stats) [+ ReLU]: y = act((conv(x) + bias) * scale + shift)
 * with scale = gamma/sqrt(running_var+eps), shift = beta - running_mean*scale applied in the conv
 * epilogue (z never stored);
 * f32 results equal dg_conv_fwd + dg_bn_apply bit for bit.  Workspace as dg_conv_fwd_ex. */
int dg_conv_fwd_bn_eval(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                        int Cout, int R, int S, int pad, const float* bias, const float* scale,
                        const float* shift, int act, void* y, int64_t ldy, void* workspace, int64_t ws_bytes,
                        const float* xamax, void* stream);
/* bf16 forward (used for dgrad: flipped filters) that also emits the BatchNorm-backward
 * partial sums of the layer whose output gradient y is, from the epilogue:
 * bpart[dg_conv_stats_rows][3][Cout] for dg_bn_bwd_from_part (replaces dg_bn_bwd's
 * partial pass over g and z).  z, scale/shift/mean/invstd, act, drop, HW: that layer's
 * dg_bn_bwd arguments.  DG_ERR_UNSUPPORTED (nothing launched) when the shape is not served
 * in one pipelined pass. */
int dg_conv_fwd_bnbwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, const void* w,
                      int Cout, int R, int S, int pad, void* y, int64_t ldy, const void* z, int64_t ldz,
                      const float* scale, const float* shift, const float* mean, const float* invstd,
                      int act, const float* drop, int HW, float* bpart, void* workspace, int64_t ws_bytes,
                      const float* xamax, void* stream);

/* wflip[C][R][S][Cout] = w[Cout][R-1-r][S-1-s][C] (packed filters of dtype). */
int dg_flip_weight(int dtype, const void* w, int Cout, int C, int R, int S, void* wflip, void* stream);

/* dW[Cout][C][R][S] (f32, torch layout) = sum_pixels dY (x) X (split-K over
 * pixels, deterministic slab reduce).  `accumulate` adds into dw. */
int64_t dg_conv_wgrad_workspace(int dtype, int N, int H, int W, int C, int Cout, int R, int S);
int dg_conv_wgrad(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C,
                  const void* dy, int64_t lddy, int Cout, int R, int S, int pad,
                  float* dw, void* workspace, int64_t ws_bytes, int accumulate, const float* xamax,
                  const float* dyamax, void* stream);
/* xamax / dyamax: operand maxima of x and dy with channels ([1 + C] and [1 + Cout] floats, as
 * dg_amax writes; f32, f16 x3 arithmetic): each channel of x and of dy is scaled by its own power of
 * two, and each dW element scaled back by 2^-(e_dy[co] + e_x[c]), so a channel far below its
 * tensor's largest magnitude keeps f32-grade relative precision.  NULL: one read pass each. */

/* torch [Cout][C][R][S] f32 -> packed rows out[Cout][row_len] of dtype holding
 * [R][S][Cpad] (zero-padded C, zero tail up to row_len). Cpad=3,row_len=64 gives
 * the im2col filter of the first layer. */
int dg_pack_weight(int dtype, const float* w, int Cout, int C, int R, int S, int Cpad,
                   int row_len, void* out, void* stream);
/* dg_pack_weight's default layout (Cpad = C, row_len = R*S*C) into out and dg_flip_weight of it into
 * wflip, in one launch (a training step's filter prep: the forward's packed filter and the dgrad's
 * flipped one); both outputs identical to the two-call sequence.  Cout*C*R*S < 2^31. */
int dg_pack_weight_flip(int dtype, const float* w, int Cout, int C, int R, int S, void* out, void* wflip,
                        void* stream);

/* First VGG layer (Cin=3): NCHW f32 image -> im2col rows [N*H*W][64] (27 taps,
 * zero padded to 64) so conv1_1 runs on the same MFMA GEMM (models/models.py:36). */
int dg_im2col3x3_c3(int dtype, const float* img, int N, int H, int W, void* out, void* stream);
/* dW for the im2col'd first layer: col-layout grad [Cout][64] -> torch [Cout][3][3][3]. */
int dg_unpack_c3_grad(const float* dwcol, int Cout, float* dw, int accumulate, void* stream);

/* ---- general convolution (ResNet-50 trunks of IBN-Net / ISW / SW) ------------
 * Replaces the strided nn.Conv2d of models/ibnnet/resnet_ibn.py:65-107,
 * models/ISW/Resnet.py:137-216,395-495 and models/SW/backbones/resnet.py:75-212.
 * Any R x S, stride, pad; output P = (H+2pad-R)/stride+1.  Whole-tensor buffer
 * addressing: the gathered tensor must be < 2 GiB. */
int dg_conv2d_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C,
                  const void* w, int Cout, int R, int S, int stride, int pad, const float* bias,
                  void* y, int64_t ldy, int accumulate, void* stream);
/* wt[C][R][S][Cout] = w[Cout][R][S][C] (packed filters, no flip) */
int dg_transpose_weight(int dtype, const void* w, int Cout, int C, int R, int S, void* wt, void* stream);
/* dX [N,H,W,C] from dY [N,P,Q,Cout] and wt (transposed gather: taps whose
 * (p + pad - r) is a multiple of stride). */
int dg_conv2d_dgrad(int dtype, const void* dy, int64_t lddy, int N, int P, int Q, int Cout,
                    const void* wt, int C, int H, int W, int R, int S, int stride, int pad,
                    void* dx, int64_t lddx, int accumulate, void* stream);
int64_t dg_conv2d_wgrad_workspace(int dtype, int N, int P, int Q, int C, int Cout, int R, int S);
int dg_conv2d_wgrad(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C,
                    const void* dy, int64_t lddy, int Cout, int R, int S, int stride, int pad,
                    float* dw, void* workspace, int64_t ws_bytes, int accumulate, const float* xamax,
                    const float* dyamax, void* stream);
/* Cin=3 stems (7x7/2 of the ResNets): NCHW f32 -> im2col [N*P*Q][Kpad], k=(r*S+s)*3+c */
int dg_im2col_c3(int dtype, const float* img, int N, int H, int W, int R, int S, int stride,
                 int pad, int Kpad, void* out, void* stream);
/* col-layout filter grad [Cout][Kpad] -> torch [Cout][3][R][S] */
int dg_unpack_c3(const float* dwcol, int Cout, int R, int S, int Kpad, float* dw, int accumulate,
                 void* stream);

/* ---- batch norm (training statistics) + activation -------------------------
 * Replaces nn.BatchNorm2d(train) + nn.ReLU (vgg16_bn, ConvBlock bn=True).
 * Stats are per channel over N*H*W pixels; running stats use momentum and the
 * unbiased variance exactly as torch.nn.BatchNorm2d. */
int64_t dg_bn_workspace(int M, int C);
int dg_bn_fwd_train(int dtype, const void* z, int64_t ldz, int M, int C,
                    const float* gamma, const float* beta, float* running_mean,
                    float* running_var, float momentum, float eps,
                    float* save_mean, float* save_invstd, float* scale, float* shift,
                    void* workspace, void* stream);
/* y = act(z*scale + shift) * drop[n][c]; act: 0 none, 1 relu. drop may be NULL
 * (Dropout2d mask already scaled by 1/(1-p), models/models.py:55-58). HW = pixels per image. */
int dg_bn_apply(int dtype, const void* z, int64_t ldz, int M, int C, const float* scale,
                const float* shift, int act, const float* drop, int HW, void* y, int64_t ldy,
                float* amax, void* stream);
/* dg_bn_apply (f32, train-mode statistics, no dropout) that also writes pair: the f16 x3 image of y
 * the following conv's pre-split forward reads (dg_conv_fwd_pair), [M][C / 32][32 x f16 hi | 32 x f16
 * lo] of y * 2^e (the split of y as stored; 4 * M * C bytes, C % 32 == 0), and *pbound, the bound e
 * came from (>= max |y|): |scale_c| sqrt(count) / invstd_c + |shift_c + mean_c scale_c| maximised over c
 * (= |gamma_c| sqrt(count) + |beta_c|, since |z - mean| <= sqrt(count) sigma for statistics over count
 * pixels; mean / invstd the batch statistics y was normalised with).  No read pass over y, but a
 * scale up to the bound's slack looser than one from max |y|.  y, amax: as dg_bn_apply. */
int dg_bn_apply_pair(const float* z, int64_t ldz, int M, int C, const float* scale, const float* shift,
                     const float* mean, const float* invstd, double count, int act, float* y, int64_t ldy,
                     float* amax, void* pair, float* pbound, void* stream);
/* amax (here and on the BN-backward / pooled / join / InstanceNorm entries below; may be NULL):
 * the operand maxima of the pass's output (the written activation or dz; the pooled entries: over
 * the un-pooled values, >= max |yp|) -- the xamax a following f32 conv can take instead of a read
 * pass of its own.  f32: [1 + C] floats, word 0 the tensor's max and word 1 + c channel c's
 * (C <= 2048); 16-bit: word 0 only.  Zeroed by the entry before its launch. */
/* Backward: g = dL/dy (pixel stride ldg).  Produces dz (lddz), dgamma, dbeta
 * (written, not accumulated) and dbias_conv (sum dz, may be NULL).
 * save_mean = save_invstd = NULL: no normalisation (a biased conv + activation, e.g. the
 * counter heads' Conv+ReLU, models/ibnnet/__init__.py:17-23): dz = act'(z)*g, where z is
 * the pre-activation and scale/shift (NULL = identity) map it as in the forward;
 * dbeta = dbias = sum dz. */
int dg_bn_bwd(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
              const float* gamma, const float* save_mean, const float* save_invstd,
              const float* scale, const float* shift, int act, const float* drop, int HW,
              void* dz, int64_t lddz, float* dgamma, float* dbeta, float* dbias,
              void* workspace, float* amax, void* stream);
/* dg_bn_bwd (f32, train-mode statistics over count pixels, no dropout) that also writes pair, the f16
 * x3 image of dz the dgrad that follows reads (dg_conv_fwd_pair; layout as dg_bn_apply_pair), and
 * *pbound: the partial pass also keeps max |g'| per channel, and the scale comes from
 * max_c |k1_c| max |g'_c| + |k2_c| sqrt(count) + |k3_c| >= max |dz| (dz = k1 g' - k2 xhat - k3,
 * |xhat| <= sqrt(count)).  Workspace: dg_bn_workspace(M, C). */
int dg_bn_bwd_pair(const float* g, int64_t ldg, const float* z, int64_t ldz, int M, int C,
                   const float* gamma, const float* save_mean, const float* save_invstd,
                   const float* scale, const float* shift, int act, double count, float* dz,
                   int64_t lddz, float* dgamma, float* dbeta, float* dbias, void* workspace,
                   float* amax, void* pair, float* pbound, void* stream);
/* BN-backward finalize on caller-made partial sums part[nblk][3][C] = (sum g', sum g' xhat,
 * sum xhat): coef[3][C] (dz = k1 g' - k2 xhat - k3) and dgamma/dbeta/dbias (may be NULL). */
int dg_bn_bwd_finalize_part(const float* part, int nblk, int M, int C, const float* gamma,
                            const float* save_invstd, float* dgamma, float* dbeta, float* dbias,
                            float* coef, void* stream);
/* dg_bn_bwd from precomputed partial sums part[nblk][3][C] (dg_conv_fwd_bnbwd): finalize +
 * apply; coef: caller workspace of 3*C floats. */
int dg_bn_bwd_from_part(int dtype, const float* part, int nblk, const void* g, int64_t ldg, const void* z,
                        int64_t ldz, int M, int C, const float* gamma, const float* save_mean,
                        const float* save_invstd, const float* scale, const float* shift, int act,
                        const float* drop, int HW, void* dz, int64_t lddz, float* dgamma, float* dbeta,
                        float* dbias, float* coef, float* amax, void* stream);

/* BN(+ReLU) fused with the following MaxPool2d(2,2) (vgg16_bn.features[5:7] etc.,
 * models/models.py:35-38).  Apply: y = act(z*scale+shift)*drop (written only when y != NULL,
 * e.g. x1/x2 that also feed the decoder) and yp [N,H/2,W/2,C] = first-max of each 2x2 window
 * of y (ATen rule).  Backward: gp = dL/dyp, gd = direct dL/dy (NULL = none); the pooled
 * gradient is routed to the recomputed argmax, then the BN/ReLU backward as dg_bn_bwd.
 * H, W even; workspace of dg_bn_workspace(N*H*W, C) bytes. */
int dg_bn_apply_pool(int dtype, const void* z, int64_t ldz, int N, int H, int W, int C,
                     const float* scale, const float* shift, int act, const float* drop, void* y,
                     int64_t ldy, void* yp, int64_t ldyp, float* amax, void* stream);
/* dg_bn_apply_pool (f32, train-mode statistics, no dropout) with the pair image of the pooled yp
 * ([N * H/2 * W/2][C / 32][hi | lo], the bound of the un-pooled y): as dg_bn_apply_pair. */
int dg_bn_apply_pool_pair(const float* z, int64_t ldz, int N, int H, int W, int C, const float* scale,
                          const float* shift, const float* mean, const float* invstd, double count, int act,
                          float* y, int64_t ldy, float* yp, int64_t ldyp, float* amax, void* pair,
                          float* pbound, void* stream);
int dg_bn_bwd_pool(int dtype, const void* gp, int64_t ldgp, const void* gd, int64_t ldgd,
                   const void* z, int64_t ldz, int N, int H, int W, int C, const float* gamma,
                   const float* save_mean, const float* save_invstd, const float* scale,
                   const float* shift, int act, const float* drop, void* dz, int64_t lddz,
                   float* dgamma, float* dbeta, float* dbias, void* workspace, float* amax, void* stream);
/* dg_bn_bwd_pool (f32, no dropout) with the pair image of dz, as dg_bn_bwd_pair */
int dg_bn_bwd_pool_pair(const float* gp, int64_t ldgp, const float* gd, int64_t ldgd, const float* z,
                        int64_t ldz, int N, int H, int W, int C, const float* gamma, const float* save_mean,
                        const float* save_invstd, const float* scale, const float* shift, int act,
                        double count, float* dz, int64_t lddz, float* dgamma, float* dbeta, float* dbias,
                        void* workspace, float* amax, void* pair, float* pbound, void* stream);

/* Coefficients of the BN backward without the dz pass: coef[3][C] = (k1, k2, k3) with
 * dz = k1*act'(g) - k2*xhat - k3 (the bn_bwd_apply arithmetic), plus dgamma/dbeta/dbias.
 * For fused consumers (dg_stem_bwd). */
int dg_bn_bwd_coef(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
                   const float* gamma, const float* save_mean, const float* save_invstd,
                   const float* scale, const float* shift, int act, const float* drop, int HW,
                   float* coef, float* dgamma, float* dbeta, float* dbias, void* workspace,
                   void* stream);

/* Merge per-block BN partials part[nblk][3][C] = (n, mean, M2) (Chan, double) into the
 * batch statistics: same outputs and running-stat update as dg_bn_fwd_train. */
int64_t dg_bn_part_workspace(int nblk, int C);
int dg_bn_part_finalize(const float* part, int nblk, int C, const float* gamma, const float* beta,
                        float* running_mean, float* running_var, float momentum, float eps,
                        float* save_mean, float* save_invstd, float* scale, float* shift,
                        void* workspace, void* stream);

/* ---- SyncBatchNorm phases (nn.SyncBatchNorm over data-parallel ranks; the reference's ISW
 * Norm2d, models/ISW/mynn.py:8-14, and convert_sync_batchnorm'd DGModel_* BN layers).  The host
 * exchanges the per-rank rows between the phases (dgvcc_amd/syncbn.py):
 *   forward:  a rank's (n, mean, M2) row [3][C] (dg_bn_stats_row from z, or dg_bn_part_row from
 *             epilogue partials) -> all-gather [world][3][C] -> dg_bn_part_finalize(nblk = world):
 *             the global batch statistics and running-stat update, as one BN over the global batch;
 *   backward: a rank's sums [3][C] = (sum g', sum g' xhat, sum xhat) (dg_bn_bwd_sums,
 *             dg_bn_bwd_pool_sums, or dg_bn_part_sums of dgrad-epilogue partials) -> all-reduce ->
 *             dg_bn_bwd_finalize_sync (dz coefficients from the global sums over M_global pixels, or,
 *             with M_global <= 0, over the count all-reduced as a fourth row of the sums [4][C]:
 *             sums[3][0] + sums[3][1], hi and lo parts of this rank's pixel count;
 *             dgamma / dbeta and the conv-bias gradient from this rank's, as torch SyncBatchNorm)
 *             -> dg_bn_bwd_apply_coef / dg_bn_bwd_pool_apply_coef.
 * Workspaces: dg_bn_workspace(M, C) (stats_row, bwd_sums), dg_bn_workspace(N*H*W, C)
 * (bwd_pool_sums), dg_bn_part_workspace(nblk, C) (part_row). */
int dg_bn_stats_row(int dtype, const void* z, int64_t ldz, int M, int C, float* row, void* workspace,
                    void* stream);
int dg_bn_part_row(const float* part, int nblk, int C, float* row, void* workspace, void* stream);
int dg_bn_part_sums(const float* part, int nblk, int C, float* sums, void* stream);
int dg_bn_bwd_sums(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
                   const float* save_mean, const float* save_invstd, const float* scale, const float* shift,
                   int act, const float* drop, int HW, float* sums, void* workspace, void* stream);
int dg_bn_bwd_pool_sums(int dtype, const void* gp, int64_t ldgp, const void* gd, int64_t ldgd, const void* z,
                        int64_t ldz, int N, int H, int W, int C, const float* save_mean,
                        const float* save_invstd, const float* scale, const float* shift, int act,
                        const float* drop, float* sums, void* workspace, void* stream);
int dg_bn_bwd_finalize_sync(const float* sums_local, const float* sums_global, int M_local, int64_t M_global,
                            int C, const float* gamma, const float* save_invstd, float* dgamma, float* dbeta,
                            float* dbias, float* coef, void* stream);
int dg_bn_bwd_apply_coef(int dtype, const void* g, int64_t ldg, const void* z, int64_t ldz, int M, int C,
                         const float* save_mean, const float* save_invstd, const float* scale,
                         const float* shift, int act, const float* drop, int HW, const float* coef, void* dz,
                         int64_t lddz, float* amax, void* stream);
int dg_bn_bwd_pool_apply_coef(int dtype, const void* gp, int64_t ldgp, const void* gd, int64_t ldgd,
                              const void* z, int64_t ldz, int N, int H, int W, int C, const float* save_mean,
                              const float* save_invstd, const float* scale, const float* shift, int act,
                              const float* drop, const float* coef, void* dz, int64_t lddz, float* amax,
                              void* stream);

/* ---- fused first layer (bf16): Conv2d(3,64,3,pad 1) of vgg16_bn.features[0]
 * (models/models.py:35-36) read straight from the NCHW f32 image (no im2col buffer).
 * dg_stem_fwd: z[N,H,W,64] (pixel stride ldz, bf16) = conv + bias, and the BN statistics
 * partials part[dg_stem_part_rows][3][64] for dg_bn_part_finalize.  wpack: bf16 [64][32]
 * (dg_pack_weight Cpad=3, row_len=32: k = (r*3+s)*3+c).  N*H*W % 64 == 0.
 * dg_stem_bwd: dW [64][3][3][3] f32 (torch layout) of the conv from the BN+ReLU
 * backward (g = dL/dy, z, the forward statistics and dg_bn_bwd_coef's coef), dz never
 * materialised. */
int64_t dg_stem_part_rows(int N, int H, int W);
int dg_stem_fwd(const float* img, int N, int H, int W, const void* wpack, const float* bias,
                void* z, int64_t ldz, float* part, void* stream);
/* dg_stem_fwd_f32: the fp32 first layer forward (exact f32 FMAs): z f32 (pixel stride ldz,
 * ldz % 4 == 0) = conv + bias and the same BN partials; wk: f32 [27][64], k = (c*3+r)*3+s
 * (torch weight [co][c][r][s] permuted to [c][r][s][co]).  W % 64 == 0. */
int dg_stem_fwd_f32(const float* img, int N, int H, int W, const float* wk, const float* bias,
                    float* z, int64_t ldz, float* part, void* stream);
/* dg_stem_bwd_f32: fp32 counterpart of dg_stem_bwd with z stored (g, z f32, ldg/ldz % 4 == 0,
 * W % 32 == 0; dg_stem_bwd_workspace bytes): dW [64][3][3][3] f32 on f32 MFMA, dz and the im2col
 * never materialised. */
int dg_stem_bwd_f32(const float* img, int N, int H, int W, const float* g, int64_t ldg, const float* z,
                    int64_t ldz, const float* save_mean, const float* save_invstd, const float* scale,
                    const float* shift, const float* coef, float* dw, void* workspace, int64_t ws_bytes,
                    int accumulate, void* stream);
int64_t dg_stem_bwd_workspace(int N, int H, int W);
int dg_stem_bwd(const float* img, int N, int H, int W, const void* g, int64_t ldg, const void* z,
                int64_t ldz, const float* save_mean, const float* save_invstd, const float* scale,
                const float* shift, const float* coef, float* dw, void* workspace, int64_t ws_bytes,
                int accumulate, const void* wpack, const float* bias, void* stream);
/* z-free stem (z = conv(img) + bias is recomputed where needed instead of stored; 27 MACs
 * per output against 128 B of HBM traffic per pixel per pass): dg_stem_stats (BN statistics
 * partials only, rows = dg_stem_part_rows), dg_stem_apply (y = relu(scale z + shift), equal
 * bit for bit to dg_stem_fwd + dg_bn_apply), dg_stem_bwd_coef (BN-backward coefficients
 * from g with z recomputed; part: dg_stem_part_rows x 3 x 64 floats), and dg_stem_bwd with
 * z = NULL (wpack/bias given). */
int dg_stem_stats(const float* img, int N, int H, int W, const void* wpack, const float* bias, float* part,
                  void* stream);
int dg_stem_apply(const float* img, int N, int H, int W, const void* wpack, const float* bias,
                  const float* scale, const float* shift, void* y, int64_t ldy, void* stream);
int dg_stem_bwd_coef(const float* img, int N, int H, int W, const void* wpack, const float* bias,
                     const void* g, int64_t ldg, const float* gamma, const float* save_mean,
                     const float* save_invstd, const float* scale, const float* shift, float* coef,
                     float* dgamma, float* dbeta, float* dbias, float* part, void* stream);

/* ---- ResNet bottleneck joins and InstanceNorm (IBN-b / ISW / SW trunks) --------
 * Residual join out = act(bn3(z1) + bn_ds(z2) | z2) of Bottleneck.forward
 * (models/ibnnet/resnet_ibn.py:96-107, models/ISW/Resnet.py:187-216,
 * models/SW/backbones/resnet.py:100-118). scale2/shift2 NULL = identity shortcut. */
int dg_bn_add_apply(int dtype, const void* z1, int64_t ld1, int M, int C, const float* scale1,
                    const float* shift1, const void* z2, int64_t ld2, const float* scale2,
                    const float* shift2, int act, void* y, int64_t ldy, float* amax, void* stream);
/* nn.ReLU backward from the saved output: out = g * (y > 0) (out may alias g). */
int dg_relu_bwd(int dtype, const void* g, int64_t ldg, const void* y, int64_t ldy, int M, int C,
                void* out, int64_t ldo, void* stream);
/* nn.InstanceNorm2d(affine) with statistics from dg_instnorm_stats:
 * y = act((x-mean[n,c])*invstd[n,c]*gamma[c]+beta[c]); gamma/beta NULL = affine=False
 * (IBN-b IN, resnet_ibn.py:77,115,159; ISW InstanceWhitening, instance_whitening.py:5-16). */
int dg_instnorm_apply(int dtype, const void* x, int64_t ldx, int N, int HW, int C,
                      const float* mean, const float* invstd, const float* gamma,
                      const float* beta, int act, void* y, int64_t ldy, float* amax, void* stream);
/* Backward of the above (g already masked by any following ReLU): dx (+)=, dgamma/dbeta
 * written (sum over n), either may be NULL. */
int64_t dg_instnorm_bwd_workspace(int N, int HW, int C);
int dg_instnorm_bwd(int dtype, const void* g, int64_t ldg, const void* x, int64_t ldx, int N,
                    int HW, int C, const float* mean, const float* invstd, const float* gamma,
                    void* dx, int64_t lddx, int accumulate, float* dgamma, float* dbeta,
                    void* workspace, float* amax, void* stream);

/* ---- instance / switchable whitening ------------------------------------------
 * ISW (models/ISW/instance_whitening.py:19-39, models/ISW/__init__.py:93-120):
 * fraw [B][C][C] = per-instance sum_p w_p w_p^T (dg_conv2d_wgrad of w with itself);
 * f = fraw*inv_hw1 + eps*I.  loss (+)= out_scale * mean_b sum|f o mask|/ns (ns = device
 * scalar); gsym[b] (may be NULL) = d loss/d fraw symmetrised and scaled by inv_hw1, so
 * dL/dw_b = w_b gsym[b] (a 1x1 conv).  grad_coef: device scalar upstream grad (NULL = 1). */
int64_t dg_iw_loss_workspace(int B, int C);
int dg_iw_loss(const float* fraw, int B, int C, float inv_hw1, float eps, const float* mask,
               const float* num_sensitive, const float* grad_coef, float out_scale, int accumulate,
               float* loss, float* gsym, void* workspace, void* stream);
/* cal_covstat: var[C][C] (+)= unbiased variance over B of f_ij*[j>i]. */
int dg_iw_cov_var(const float* fraw, int B, int C, float inv_hw1, float* var, int accumulate,
                  void* stream);
/* SwitchWhiten2d sw_type 2 (BW+IW), 16 channels per group, C <= 256
 * (models/SW/ops/switchwhiten.py:84-183).  mean_w/var_w: raw sw_mean_weight /
 * sw_var_weight (softmax inside).  running_mean [G][16], running_cov [G][16][16] updated
 * with `momentum` when training.  y = act(gamma*W(x-mean)+beta); `save`
 * (dg_sw_save_size bytes) holds the statistics for dg_sw_bwd. */
int64_t dg_sw_save_size(int N, int C);
int64_t dg_sw_workspace(int N, int HW, int C);
int dg_sw_fwd(int dtype, const void* x, int64_t ldx, int N, int HW, int C, int T, float eps,
              float momentum, const float* mean_w, const float* var_w, const float* gamma,
              const float* beta, float* running_mean, float* running_cov, int training, int act,
              float* save, void* y, int64_t ldy, void* workspace, void* stream);
/* Split phases for SyncSwitchWhiten2d (models/SW/ops/sync_switchwhiten.py:9-56): the batch
 * moments moments[G][272] (doubles: sum_n mu_n | sum_n cov_n + mu_n mu_n^T) are the only
 * cross-instance quantities, so a caller can all-reduce them between the phases; `count` =
 * images over all ranks.  dg_sw_fwd == stats + finish(count = N).  `workspace` (dg_sw_workspace
 * bytes) must be the same buffer across a stats/finish pair. */
int64_t dg_sw_moments_size(int C);
int dg_sw_fwd_stats(int dtype, const void* x, int64_t ldx, int N, int HW, int C, float* save,
                    double* moments, void* workspace, void* stream);
int dg_sw_fwd_finish(int dtype, const void* x, int64_t ldx, int N, int HW, int C, int T, float eps,
                     float momentum, const float* mean_w, const float* var_w, const float* gamma,
                     const float* beta, float* running_mean, float* running_cov, int training, int act,
                     int64_t count, const double* moments, float* save, void* y, int64_t ldy,
                     void* stream);
/* Backward phases: bmoments[G][272] = (dL/dmu_bn | dL/dcov_bn) of this rank, summed over ranks
 * by the caller (SyncMeanCov.backward all-reduces grad_mean/grad_cov) before finish. */
int dg_sw_bwd_stats(int dtype, const void* gy, int64_t ldg, const void* y, int64_t ldy, const void* x,
                    int64_t ldx, int N, int HW, int C, int T, float eps, const float* mean_w,
                    const float* var_w, const float* gamma, int act, const float* save, double* bmoments,
                    float* dgamma, float* dbeta, void* workspace, void* stream);
int dg_sw_bwd_finish(int dtype, const void* gy, int64_t ldg, const void* y, int64_t ldy, const void* x,
                     int64_t ldx, int N, int HW, int C, int act, const float* mean_w, const float* var_w,
                     const float* save, int64_t count, const double* bmoments, void* dx, int64_t lddx,
                     int accumulate, float* dmean_w, float* dvar_w, void* workspace, void* stream);
/* Exact adjoint (batch statistics, Newton-Schulz iterations recomputed). y = forward
 * output (ReLU mask when act == 1). Any of dgamma/dbeta/dmean_w/dvar_w may be NULL. */
int dg_sw_bwd(int dtype, const void* gy, int64_t ldg, const void* y, int64_t ldy, const void* x,
              int64_t ldx, int N, int HW, int C, int T, float eps, const float* mean_w,
              const float* var_w, const float* gamma, int act, const float* save, void* dx,
              int64_t lddx, int accumulate, float* dgamma, float* dbeta, float* dmean_w,
              float* dvar_w, void* workspace, void* stream);

/* ---- pooling / resampling ---------------------------------------------------
 * nn.MaxPool2d(2,2) (vgg16_bn features 6,13,23,33) and F.interpolate
 * (models/models.py:23-27).  Bilinear supports align_corners 0/1, nearest. */
int dg_maxpool2_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C,
                    void* y, int64_t ldy, void* stream);
int dg_maxpool2_bwd(int dtype, const void* x, int64_t ldx, const void* gy, int64_t ldgy,
                    int N, int H, int W, int C, void* gx, int64_t ldgx, int accumulate,
                    void* stream);
/* nn.MaxPool2d(k, stride, pad) of the ResNet stems (models/ibnnet/resnet_ibn.py:161,
 * models/ISW/Resnet.py:288, models/SW/backbones/resnet.py:153): -inf padding, first
 * maximum wins, NaN propagates (ATen). Output P = (H+2pad-k)/stride+1. */
int dg_maxpool_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, int k,
                   int stride, int pad, void* y, int64_t ldy, void* stream);
int dg_maxpool_bwd(int dtype, const void* x, int64_t ldx, const void* gy, int64_t ldgy, int N,
                   int H, int W, int C, int k, int stride, int pad, void* gx, int64_t ldgx,
                   int accumulate, void* stream);
/* The same pool recording the argmax: idx [N,P,Q,C] uint8 = r*k + s of each window's first
 * maximum (k <= 15); the backward gathers (idx, gy) pairs instead of re-scanning windows. */
int dg_maxpool_fwd_idx(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, int k,
                       int stride, int pad, void* y, int64_t ldy, unsigned char* idx, void* stream);
int dg_maxpool_bwd_idx(int dtype, const unsigned char* idx, const void* gy, int64_t ldgy, int N,
                       int H, int W, int C, int k, int stride, int pad, void* gx, int64_t ldgx,
                       int accumulate, void* stream);
/* mode: 0 bilinear(align_corners=False), 1 bilinear(align_corners=True), 2 nearest */
int dg_upsample_fwd(int dtype, const void* x, int64_t ldx, int N, int H, int W, int C, int scale,
                    int mode, void* y, int64_t ldy, void* stream);
/* gx (+)= U^T (gy + gy2); gy2 may be NULL (two consumers of one upsample). */
int dg_upsample_bwd(int dtype, const void* gy, int64_t ldgy, const void* gy2, int64_t ldgy2,
                    int N, int H, int W, int C, int scale, int mode, void* gx, int64_t ldgx,
                    int accumulate, void* stream);

/* den_dec on the decomposed decoder concatenation (models/models.py:84,89-90):
 * conv1x1(cat[y1, up2(y2), up4(y3)]) = z1 + up2(z2) + up4(z3) with zk = conv1x1(yk; W[:, slice k]).
 * z [N,H,W,C] = z1 + up2(z2 [N,H/2,W/2,C]) + up4(z3 [N,H/4,W/4,C]) + bias (bilinear,
 * align_corners=False), stored in dtype; part (may be NULL) receives the BN statistics
 * partials [dg_cat_combine_part_rows][3][C] = (n, mean, M2) of the stored z for
 * dg_bn_part_finalize.  z may alias z1. */
int64_t dg_cat_combine_part_rows(int N, int H, int W);
int dg_cat_combine(int dtype, const void* z1, int64_t ldz1, const void* z2, int64_t ldz2,
                   const void* z3, int64_t ldz3, int N, int H, int W, int C, const float* bias,
                   void* z, int64_t ldz, float* part, void* stream);

/* ---- device-side training augmentation (DenClsDataset, datasets/den_cls_dataset.py:29-35,
 * 77-158) -------------------------------------------------------------------------------
 * imgs: B uint8 RGB crops [B][H][W][3] (HBM-resident); params: [B][16] f32 per-sample
 * decisions drawn on the host in the reference's RNG order (dgvcc_amd/datasets/augment.py):
 * grey, hflip, ColorJitter (applied, op order, factors, uint8 hue shift), GaussianBlur
 * (applied, 1-D weights), RandomAdjustSharpness (applied, factor).
 * img1 = Normalize(ToTensor(grey/flip(img))), img2 = Normalize(ToTensor(more_transform(...)))
 * as NCHW f32 [B][3][H][W], bit-identical to the PIL/torchvision host pipeline (see augment.hip).
 * dg_block_map: bmap [B][h/16][w/16] = (16x16 block sums of dmap [B][h][w] > 0). */
int64_t dg_augment_workspace(int B, int H, int W);
int dg_augment_den_cls(const unsigned char* imgs, int B, int H, int W, const float* params,
                       float* img1, float* img2, void* workspace, int64_t ws_bytes, void* stream);
int dg_block_map(const float* dmap, int B, int h, int w, float* bmap, void* stream);

/* ---- density head: 1x1 conv C->1 (+ReLU) --------------------------------------
 * den_head (models/models.py:60-62) / cls_head tail (models/models.py:241-242). */
int dg_head_fwd(int dtype, const void* x, int64_t ldx, int M, int C, const float* w,
                const float* bias, int act, float* y, void* stream);
/* act: 0 none, 1 relu, 2 sigmoid (y is the saved output) */
int64_t dg_head_workspace(int M, int C);
int dg_head_bwd(int dtype, const void* x, int64_t ldx, int M, int C, const float* w, int act,
                const float* y, const float* gy, void* gx, int64_t ldgx, int accumulate_gx,
                float* gw, float* gbias, void* workspace, void* stream);

/* ---- two-view consistency + memory read ----------------------------------------
 * DGModel_memadd/final.forward_train (models/models.py:147-184, 298-335) and
 * forward_mem (models/models.py:116-125).  The memory GEMMs run on dg_conv_fwd /
 * dg_conv_wgrad as 1x1 convolutions; these are the non-GEMM pieces. */
int64_t dg_instnorm_workspace(int N, int HW, int C);
/* F.instance_norm statistics (biased variance) per (n, c) over HW pixels. */
int dg_instnorm_stats(int dtype, const void* x, int64_t ldx, int N, int HW, int C, float eps,
                      float* mean, float* invstd, void* workspace, void* stream);
/* e = |IN(y1) - IN(y2)| < thr (bytes, [N*HW][C]); m_v = y_v * e * drop_v[n][c] (dense). */
int dg_emask_fwd(int dtype, const void* y1, const void* y2, int64_t ld, int N, int HW, int C,
                 const float* mu1, const float* is1, const float* mu2, const float* is2, float thr,
                 const float* drop1, const float* drop2, void* m1, void* m2, unsigned char* mask,
                 void* stream);
int dg_emask_bwd(int dtype, const void* gm1, const void* gm2, int N, int HW, int C,
                 const unsigned char* mask, const float* drop1, const float* drop2, void* gy1,
                 void* gy2, int64_t ldgy, void* stream);
/* softmax over the C (1024) memory slots of each pixel row, both views, plus
 * loss_con = mean((P1-P2)^2) (the `jsd`, models/models.py:286-296). */
int64_t dg_softmax_workspace(int M);
int dg_softmax_pair_fwd(int dtype, const void* L1, const void* L2, int M, int C, void* P1, void* P2,
                        float* loss_con, void* workspace, void* stream);
/* dL_v = P_v (g_v' - <P_v, g_v'>), g_1' = g_1 + k(P1-P2), g_2' = g_2 - k(P1-P2),
 * k = 2*coef[0]/(M*C) with coef a device scalar (upstream grad of loss_con; may be NULL). */
int dg_softmax_pair_bwd(int dtype, const void* P1, const void* P2, const void* G1, const void* G2,
                        int M, int C, const float* coef, void* GL1, void* GL2, void* stream);
int dg_softmax_fwd(int dtype, const void* L, int M, int C, void* P, void* stream);
int dg_softmax_bwd(int dtype, const void* P, const void* G, int M, int C, void* GL, void* stream);
/* class maps (models/models.py:196-207, 323-327): nearest x`scale` of thresholded
 * c1/c2 and of c_gt; two-view: c_resized = clamp(gt + |c1b - c2b|, 0, 1), c_err;
 * single view (c2 NULL): c_resized = cgt ? up(cgt) : up(c1 >= thr). */
int dg_cls_combine(const float* c1, const float* c2, const float* cgt, int N, int h, int w, int scale,
                   float thr, float* c_resized, float* c_err, void* stream);
int dg_mul_f32(const float* a, const float* b, int64_t n, float* out, void* stream);
/* models2.DensityRegressorM.forward_train (models/models2.py:326-346): the two slot
 * softmaxes plus loss_kl = 0.5/HW (KL(p1||pm) + KL(p2||pm)) batchmean, pm = (p1+p2)/2;
 * backward adds k (p_v (A - <p_v, A> + 1) - pm), A = log pm - (log p1 + log p2)/2,
 * k = coef[0] / (2M), to the readout's softmax backward. */
int dg_softmax_jsd_fwd(int dtype, const void* L1, const void* L2, int M, int C, void* P1, void* P2,
                       float* loss_kl, void* workspace, void* stream);
int dg_softmax_jsd_bwd(int dtype, const void* P1, const void* P2, const void* G1, const void* G2,
                       int M, int C, const float* coef, void* GL1, void* GL2, void* stream);
/* Memory read + density head fused (models/models.py:116-125 forward_mem feeding den_head
 * :112-114; models2.py DensityRegressorM): y_new = mem P only feeds the 1x1 k->1 head, so
 * d = act(v . P + b) with v = mem^T w (dg_mem_head_vec, [S] f32 from the f32 master mem [k][S]).
 * dg_softmax_head_fwd: slot softmax of nviews (1|2) logit rows + head output yh_v [M] f32 +
 *   loss (0 none, 1 mean((P1-P2)^2) as dg_softmax_pair_fwd, 2 KL-JSD as dg_softmax_jsd_fwd; nviews 2).
 *   P_v may be NULL (no backward: eval).  workspace: dg_mem_head_workspace(M, C) bytes.
 * dg_softmax_head_bwd: gL_v = P_v (gP_v - <P_v, gP_v>), gP_v = gpre_v v + loss term, gpre_v =
 *   act'(yh_v) gyh_v (gyh_v NULL = 0); GL NULL = head gradients only.  Leaves per-block
 *   partials of u = sum_px gpre P and sum gpre in the workspace for
 * dg_mem_head_grads: dmem[k][S] = w u^T (the readout's mem gradient; NULL = skip), gw[k] = mem u,
 *   gb = sum gpre (NULL = skip); fixed-order (deterministic) reductions. */
int64_t dg_mem_head_workspace(int M, int C);
int dg_mem_head_vec(const float* mem, const float* w, int k, int S, float* v, void* stream);
int dg_softmax_head_fwd(int dtype, int nviews, int loss, const void* L1, const void* L2, int M, int C,
                        const float* v, const float* bias, int act, void* P1, void* P2, float* yh1,
                        float* yh2, float* loss_out, void* workspace, void* stream);
int dg_softmax_head_bwd(int dtype, int nviews, int loss, const void* P1, const void* P2, int M, int C,
                        const float* v, int act, const float* yh1, const float* yh2, const float* gyh1,
                        const float* gyh2, const float* coef, void* GL1, void* GL2, void* workspace,
                        float* amax, void* stream);
/* amax (may be NULL): f32, the logit gradients' operand maxima with channels, view v at
 * v * words (words = 1 + C rounded up to a multiple of 4; word 0 max |gL_v|, word 1 + s slot s's);
 * 16-bit, amax[v] = max |gL_v|. */
int dg_mem_head_grads(void* workspace, int M, int C, const float* mem, const float* w, int k,
                      float* dmem, float* gw, float* gb, void* stream);
/* loss_err = F.l1_loss(IN(y1), IN(y2)) (models/models2.py:334) from the instance-norm
 * statistics; backward writes g_IN1 = coef[0] sgn(IN1 - IN2)/(N HW C) and g_IN2 = -g_IN1
 * (dense [N*HW][C]) for dg_instnorm_bwd. */
int64_t dg_in_l1_workspace(int N, int HW, int C);
int dg_in_l1_fwd(int dtype, const void* y1, const void* y2, int64_t ld, int N, int HW, int C,
                 const float* mu1, const float* is1, const float* mu2, const float* is2, float* loss,
                 void* workspace, void* stream);
int dg_in_l1_bwd(int dtype, const void* y1, const void* y2, int64_t ld, int N, int HW, int C,
                 const float* mu1, const float* is1, const float* mu2, const float* is2,
                 const float* coef, void* g1, void* g2, void* stream);
/* nn.Tanh of models2.Generator/Generator0 (models/models2.py:50,85): y = tanh(x);
 * backward gx (+)= gy (1 - y^2) from the saved output. */
int dg_tanh_fwd(const float* x, int64_t n, float* y, void* stream);
int dg_tanh_bwd(const float* y, const float* gy, int64_t n, float* gx, int accumulate, void* stream);

/* ---- losses ------------------------------------------------------------------
 * nn.MSELoss()(pred, gt*log_para) (trainers/dgtrainer.py:57): loss (f32 scalar
 * on device) and optionally dpred = coef*2*(pred-gt*scale)/n. */
int dg_mse_loss(const float* pred, const float* gt, float gt_scale, int64_t n, float* loss,
                float* dpred, float grad_coef, void* workspace, void* stream);
int64_t dg_reduce_workspace(int64_t n);
/* F.binary_cross_entropy(pred, target) mean (trainers/dgtrainer.py:178,188) and
 * dpred = coef * dBCE/dpred (ATen clamps: log >= -100, denominator >= 1e-12). */
int dg_bce_loss(const float* pred, const float* target, int64_t n, float* loss, float* dpred,
                float grad_coef, void* workspace, void* stream);

/* ---- Bayesian loss (losses/bl.py:5-91) ------------------------------------------
 * points [total][2] (x, y) concatenated over images with offsets[B+1] (device
 * int64); st_sizes[B]; targets [total]; density [B][G][G] (G = c_size/stride).
 * loss (device scalar) = BL(points, st_sizes, targets, density); ddensity (may be
 * NULL) = grad_coef[0] (device scalar, NULL = 1) * dloss/ddensity. */
int64_t dg_bl_workspace(int B, int G, int64_t total_points);
int dg_bl_loss(const float* points, const int64_t* offsets, int64_t total_points,
               const float* st_sizes, const float* targets, const float* density, int B, int G,
               float stride, float sigma, float bg_ratio, int use_bg, float* loss, float* ddensity,
               const float* grad_coef, void* workspace, void* stream);
/* Post_Prob posterior rows (n_b [+1 background]) x G^2 per image at prob + row_offsets[b]*G^2. */
int dg_bl_prob(const float* points, const int64_t* offsets, int64_t total_points,
               const float* st_sizes, int B, int G, float stride, float sigma, float bg_ratio,
               int use_bg, const int64_t* row_offsets, float* prob, void* workspace, void* stream);

/* ---- optimizer -----------------------------------------------------------------
 * torch.optim.AdamW step over one flat f32 buffer (main.py:85-86). */
int dg_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, float lr,
                  float beta1, float beta2, float eps, float weight_decay, int step,
                  void* stream);
/* fp16 mode dynamic loss scaling (torch.cuda.amp.GradScaler semantics): g *= inv_scale in
 * place over the flat gradient; *nonfinite (device int) = 1 if any element was inf/NaN. */
int dg_grad_unscale(float* g, int64_t n, float inv_scale, int* nonfinite, void* stream);
/* Gather `count` tensors (ptrs[i], sizes[i]; device arrays) into a flat buffer. */
int dg_gather_flat(const float* const* ptrs, const int64_t* offsets, int count,
                   int64_t total, float* flat, void* stream);

/* ---- Gaussian density-map scatter (utils/dmap_gen.py:53-81) --------------------
 * points: [npts][2] f32 (x=col, y=row) per image, concatenated; offsets[N+1]
 * (device int64) delimit images.  dmap: [N][H][W] f32, overwritten.  sigma=4,
 * radius 7 (15x15 normalized separable Gaussian, constant-0 borders). */
int dg_dmap_fixed(const float* points, const int64_t* offsets, int N, int H, int W,
                  float sigma, int radius, float* dmap, void* stream);

/* Deterministic dg_dmap_fixed (no atomics on the map), one launch: one block per 64x64 tile
 * forms the 1-D weights and walks its image's points in order (hits compacted in point order), so every
 * pixel sums its stamp values in the reference's f32 accumulation order: bit-identical to
 * gaussian_filter_density_fixed and run to run.  dmap fully written (no memset needed).
 * npoints = offsets[N] (host value); workspace: dg_dmap_fixed_tiled_workspace bytes (now 0:
 * NULL is accepted; points may be NULL when npoints == 0). */
int64_t dg_dmap_fixed_tiled_workspace(int N, int H, int W, int radius, int64_t npoints);
int dg_dmap_fixed_tiled(const float* points, const int64_t* offsets, int N, int H, int W,
                        float sigma, int radius, int64_t npoints, void* workspace, float* dmap, void* stream);

/* gaussian_filter_density (utils/dmap_gen.py:14-51): per-point sigma from the
 * 3 nearest neighbours (0.1 * sum; 15 when <= 3 points), truncate 4.
 * sigma_ws: caller workspace of total-points doubles (receives the sigmas). */
int dg_dmap_adaptive(const float* points, const int64_t* offsets, int N, int H, int W,
                     double* sigma_ws, float* dmap, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DGVCC_H */
