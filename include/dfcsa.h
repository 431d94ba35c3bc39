/* libdfcsa -- MI355X (gfx950) kernels for the DFC-SA-Res U-Net training step.
 *
 * C ABI: plain pointers (device pointers unless stated), int sizes, a hipStream_t passed as
 * void*.  Every entry point only enqueues work on that stream: it never allocates, never
 * synchronises and never throws; it returns 0 on success, DFCSA_EINVAL for a shape/argument
 * error, or -hipError_t for a launch error.  Scratch memory ("slabs") is owned by the caller
 * (the PyTorch caching allocator on the Python side); sizes follow from the documented shapes.
 *
 * Layouts: activations are NHWC ("[M][C]" with M = B*H*W pixels), element type selected by
 * `dtype` (DFCSA_DT_F32 = 0 or DFCSA_DT_BF16 = 1); all statistics, accumulators, parameters,
 * gradients and optimizer state are fp32.  Channel counts of NHWC tensors are multiples of 8.
 *
 * The reference (YukiHataRin/DFC-SA-UNet) has no native boundary: every function below
 * replaces PyTorch/ATen calls made by the reference's Python modules; the replaced call sites
 * are cited per entry point (file:line in the reference checkout).
 */
#ifndef DFCSA_H_
#define DFCSA_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DFCSA_DT_F32 0
#define DFCSA_DT_BF16 1
#define DFCSA_MAX_SEG 32
#define DFCSA_EINVAL (-10000)

/* ------------------------------------------------------------------------------------------
 * Implicit-GEMM convolution (MFMA).  Replaces nn.Conv2d / nn.ConvTranspose2d forward and the
 * data-gradient half of their backward, plus torch.cat of the block inputs:
 *   models/unet_dfc_sa_res.py:58-59 (3x3), :66, :74, :81, :88 (1x1), :147-156 (ConvTranspose),
 *   :102, :109, :182-200 (cat).
 * C[m][n] = sum_k A[m][k] * weight[n][k] (+ bias[n]); A is gathered on the fly:
 *   A[m][s*Cseg + c] = seg_ptr[s][b, oh*stride + seg_dh[s], ow*stride + seg_dw[s], c]
 * over an output grid of Ho x Wo pixels (m = (b*Ho + oh)*Wo + ow), sources Hi x Wi.
 * weight: [N][Kpad] of dtype, Kpad >= nseg*Cseg, multiple of 64 (bf16) / 32 (f32), zero-padded.
 * mode PLAIN: columns [d*Nd, (d+1)*Nd) go to dest[d] ([M][Nd]).  mode SHUFFLE2 (ConvTranspose
 * k2 s2): column n = (2i + j)*Nd + co goes to dest[0][b, 2oh+i, 2ow+j, co] of Hout x Wout.
 * accumulate: dest += C.  stats (optional): one row per workgroup M tile t of the kernel the call
 * picks (64..256 rows, or the tiles a persistent streaming workgroup visits), stats[t][0][n] = sum
 * of the fp32 accumulator (without bias) over its valid rows, stats[t][1][n] = sum of squares;
 * dfcsa_conv_stats_rows gives the number of rows the call writes.
 *
 * Slab capacities: every entry point that writes a per-workgroup partial slab (the stats above,
 * `partial`, `bias_partial`, `stats3/4`) also takes that slab's size in floats (`*_floats`), and
 * returns DFCSA_EINVAL without launching when its grid would write past it.
 * ---------------------------------------------------------------------------------------- */
#define CONV_STORE_PLAIN 0
#define CONV_STORE_SHUFFLE2 1
typedef struct {
  int dtype;
  int M, N, Kpad, Cseg, nseg;
  const void* seg_ptr[DFCSA_MAX_SEG];
  int seg_dh[DFCSA_MAX_SEG];
  int seg_dw[DFCSA_MAX_SEG];
  int Ho, Wo, Hi, Wi, stride;
  const void* weight;
  const float* bias;
  int mode, ndest;
  void* dest[3];
  int Nd, accumulate;
  float* stats;
  int Hout, Wout;
  int64_t stats_floats; /* capacity of stats in floats: >= dfcsa_conv_stats_rows(d)*2*N (<= ceil(M/64)*2*N) */
  float* work;          /* split-K workspace (optional): a bf16 launch with few 128x128 tiles and a long K */
  int64_t work_floats;  /* splits its K range over workgroups when work holds dfcsa_conv_work_floats(d) */
} dfcsa_conv_desc;
int dfcsa_conv_gemm(const dfcsa_conv_desc* d, void* stream);
/* The conv of *d (stats required) followed by the train-mode BatchNorm finalisation of its first C
 * output columns -- the result of dfcsa_conv_gemm + dfcsa_bn_finalize(training = 1) over the
 * launch's statistics rows (scale/shift/mean/invstd, running statistics, num_batches_tracked).  When
 * the picked kernel's epilogue can (the tile kernels) the finalisation runs in the launch's own tail:
 * its last workgroups reduce the statistics rows in two fixed-order ticket levels (no finalize
 * launch, reference models/unet_dfc_sa_res.py:58-59 + nn.BatchNorm2d); otherwise the finalize is
 * launched after the conv. */
typedef struct {
  int C;                      /* channels finalised: output columns [0, C) (C <= N) */
  int count;                  /* elements per channel (M) */
  const float* conv_bias;     /* optional: the conv bias, added to the batch mean (stats exclude it) */
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  int64_t* num_batches_tracked;   /* optional */
  float momentum, eps;
  float* scale;
  float* shift;
  float* mean;
  float* invstd;
} dfcsa_bn_fold;
int dfcsa_conv_gemm_bn(const dfcsa_conv_desc* d, const dfcsa_bn_fold* f, void* stream);
int dfcsa_conv_gemm_mtile(int N); /* rows per stats tile of the row-tile kernels */
/* statistics rows the launch of *d writes (and dfcsa_bn_finalize reads as ntiles): one per M tile
 * of the row-tile kernels (ceil(M / BM), BM = 64..256), one per workgroup of the persistent 1x1
 * streaming kernel, one per 2-D tile of the bf16 3x3 halo-tile kernel */
int dfcsa_conv_stats_rows(const dfcsa_conv_desc* d);
/* fp32 workspace the launch of *d splits its K range into (fixed-order partial-tile reduction in a
 * second launch that also runs the epilogue); 0 when it does not split.  A caller that passes no
 * workspace (work == NULL) gets the unsplit kernel. */
int64_t dfcsa_conv_work_floats(const dfcsa_conv_desc* d);

/* ------------------------------------------------------------------------------------------
 * Weight gradient (MFMA, reduction over pixels).  Replaces the weight half of
 * convolution_backward for every conv of the block (unet_dfc_sa_res.py:58,66,74,81,88) and
 * of ConvTranspose2d (:147-156).
 * partial[s][i][j] = sum over pixels m in chunk s of G[m][i] * X[m][j], where G = concat of
 * ng tensors [M][Cg] (i = src*Cg + c) and X is gathered like dfcsa_conv_desc's A (j = seg*Cseg+c),
 * NI = ng*Cg, NJ = nseg*Cseg; splits/mchunk/slab size from dfcsa_wgrad_plan.
 * ndst == 0: slab = [splits][NI][NJ] fp32, reduced by the caller (dfcsa_wgrad_reduce).
 * ndst > 0: the launch also reduces the partials and adds them to dst[] in `layout` (the mapping
 *   of dfcsa_wgrad_reduce), by a fixed-order reduction launch after the wgrad kernel; or, with
 *   splits <= dfcsa_wgrad_fuse_max() (0 by default, tuning knob 13), inside the wgrad kernel:
 *   every workgroup publishes its fp32 partial tile (write-through stores), takes a ticket on its
 *   output tile, and the LAST arriving workgroup of the tile sums the partials in split order
 *   0..splits-1 and adds the sum to dst (deterministic, no float atomics, no second launch).
 *   slab must hold *slab_floats floats either way.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  int dtype;
  int M;
  int ng, Cg;
  const void* g_ptr[3];
  int nseg, Cseg;
  const void* seg_ptr[DFCSA_MAX_SEG];
  int seg_dh[DFCSA_MAX_SEG];
  int seg_dw[DFCSA_MAX_SEG];
  int Ho, Wo, Hi, Wi, stride;
  float* slab;
  int splits, mchunk;
  int layout, ntaps, Ctot, Creal, ndst;
  float* dst[3];
  int64_t slab_floats;  /* capacity of slab in floats (checked against the launch) */
  /* layout 2 (stacked q/k/v 1x1 rows) with ndst == 3: bias_dst[0] != NULL also adds the pixel sums
   * of G (sum_m G[m][i], the three biases' gradients) into bias_dst[0..2] with the row mapping of
   * the weights -- in the weight-gradient launch where the kernel allows it, else by one column-sum
   * launch after it (the result of dfcsa_slab_colsum3 on G either way) */
  float* bias_dst[3];
} dfcsa_wgrad_desc;
int dfcsa_wgrad_plan(int M, int NI, int NJ, int dtype, int* splits, int* mchunk, int64_t* slab_floats);
/* the plan of the launch dfcsa_conv_wgrad will make for *d (segments, shapes, layout filled in):
 * a bf16 3x3 weight gradient (layout 0, one dY tensor, M >= 32768) runs on 2-D halo tiles with its
 * own pixel-range split count; everything else as dfcsa_wgrad_plan */
int dfcsa_wgrad_plan_desc(const dfcsa_wgrad_desc* d, int* splits, int* mchunk, int64_t* slab_floats);
int dfcsa_wgrad_fuse_max(void);
/* Split-K weight gradients whose grid fits on the device at once reduce their partials INSIDE the
 * launch (cooperative: every split reduces one slice of its tile over all splits, in split order;
 * tuning knob 31 = 0 selects the separate dfcsa_wgrad_reduce launch).  A wait that exceeded its
 * bound (never in a correct launch) is recorded instead of hanging: returns the sticky error flag
 * (0 = none) and clears it when reset != 0.  Synchronous (reads a device word). */
int dfcsa_wgrad_coop_errors(int reset);
int dfcsa_conv_wgrad(const dfcsa_wgrad_desc* d, void* stream);
/* dfcsa_conv_wgrad(d) plus the input gradient of a 1x1 conv from the same G (ng = 1):
 * dx[m][n] = sum_i G[m][i] * wt[n * kpad + i] for n < N (wt: the transposed weight, the
 * dfcsa_conv_gemm operand of that dgrad), in ONE launch when both fit the small fp32 kernels
 * (M <= 4096, 1x1, fp32, one split); otherwise the two calls in order.  The LightSelfAttention
 * projection backward (dW_q/k/v, db_q/k/v, dpooled) is one launch this way. */
int dfcsa_conv_wgrad_dgrad1x1(const dfcsa_wgrad_desc* d, const float* wt, int kpad, int N, float* dx, void* stream);
/* dfcsa_conv_wgrad_dgrad1x1 for the LightSelfAttention backward of a DFC block, whose dx is dpooled
 * [B][P*P][N]: the same launch also writes the attention entry's pool-backward BatchNorm sums as
 * ceil(M/16) extra partial rows of [2][N] (rows[t][0][c] = sum over its 16 pooled positions of
 * dpooled/area * R, rows[t][1][c] = the same of dpooled/area * invstd*(Y - mean*R); R, Y: the
 * window sums of dfcsa_lsa_pooled_ws), so that dfcsa_bn_bwd_finalize over the dattn rows of
 * dfcsa_bwd_relu_bn plus these rows gives the entry's coefficients.  Small fp32 path only (M <=
 * 4096); DFCSA_EINVAL otherwise. */
typedef struct {
  const float* wsum;     /* [B][P*P][2][N] */
  const float* mean;     /* [N] */
  const float* invstd;   /* [N] */
  float* rows;           /* ceil(M/16) x [2][N] */
  int H, W, P;
} dfcsa_pool_contract;
int dfcsa_conv_wgrad_dgrad1x1_pool(const dfcsa_wgrad_desc* d, const float* wt, int kpad, int N, float* dx,
                                   const dfcsa_pool_contract* pc, void* stream);
/* grad += sum_s slab[s] (slab [splits][NI][NJ]) mapped to the reference weight layout.
 *  layout 0 (Conv2d): rows split over ndst tensors of NI/ndst rows; column j = tap*Ctot + cin
 *     -> dst[row][cin][tap] (Conv2d weight [Cout][Cin][kh][kw]); cin >= Creal skipped.
 *  layout 1 (ConvTranspose2d): row = ci, column j = ij*Cout + co -> dst[ci][co][ij].
 *  layout 2 (stacked 1x1 q/k/v): rows [0,Ctot) -> dst[0], [Ctot,2Ctot) -> dst[1],
 *     [2Ctot, 2Ctot+Creal) -> dst[2], later rows (GEMM padding) dropped; dst[d][row - base][j]
 *     with NJ columns (ndst must be 3).
 *  layout 3 (two 1x1 convs over shared trailing inputs: the DFC block's fusion conv over
 *           [fused | local | attn] and gate conv over [local | attn], one GEMM with G = [dy4 | dy3]):
 *           rows [0,Ctot) -> dst[0][i][j] over all NJ columns; rows [Ctot,2Ctot) -> dst[1][i-Ctot][j-Ctot]
 *           for j >= Ctot (the [dy3 x fused] block is discarded); ndst must be 2. */
int dfcsa_wgrad_reduce(const float* slab, int splits, int NI, int NJ, int layout, int ntaps,
                       int Ctot, int Creal, int ndst, float* const* dst, void* stream);

/* ------------------------------------------------------------------------------------------
 * Weight packing (fp32 reference layouts -> dtype GEMM operands).  Runs every forward
 * (weights change every step).
 * ---------------------------------------------------------------------------------------- */
/* out[row0 + co][tap*Cpad + ci] = w[co][ci][tap] (ci < Cin), zero elsewhere in the row;
 * out has row stride Kpad; w is [Cout][Cin][ntaps] fp32.  */
int dfcsa_pack_conv_w(int dtype, const float* w, int Cout, int Cin, int ntaps, int Cpad,
                      int Kpad, int row0, void* out, void* stream);
/* transposed (dgrad) packing: out[ci][col0 + tap*Cout + co] = w[co][ci][tap] (row stride Kpad) */
int dfcsa_pack_conv_w_t(int dtype, const float* w, int Cout, int Cin, int ntaps, int Kpad,
                        int col0, void* out, void* stream);
/* transposed packing of up to three weights side by side, full rows (zeros elsewhere):
 * out[ci][off_s + tap*Cout_s + co] = w_s[co][ci][tap] for s = 0..2 (off_0 = 0, off_{s+1} = off_s +
 * ntaps_s*Cout_s), rows ci < Cin, row stride Kpad; the weights have wcin input channels (rows
 * ci >= wcin are zero).  w_s may be NULL (segment absent, Cout_s = 0) or, for s = 2 with
 * identity2 != 0, the identity (out[ci][off_2 + co] = (ci == co)). */
int dfcsa_pack_t3(int dtype, int Cin, int Kpad, int wcin, const float* w0, int cout0, int ntaps0, const float* w1,
                  int cout1, int ntaps1, const float* w2, int cout2, int ntaps2, int identity2, void* out,
                  void* stream);
/* ConvTranspose2d weight [Cin][Cout][2][2]: fwd [4*Cout][Cin] (row ij*Cout+co), bwd [Cin][4*Cout],
 * bias4[ij*Cout+co] = bias[co]. */
int dfcsa_pack_convT_w(int dtype, const float* w, const float* bias, int Cin, int Cout, void* out_fwd,
                       void* out_bwd, float* bias4, void* stream);
/* One-launch weight packing for a whole model.  A device table of entries (built once; the
 * parameter and packed-buffer pointers are stable) is processed by one launch of `total`
 * workgroups: entry e owns workgroup tasks [start, start + count) (entries sorted by start).
 * kinds (a* = integer args):
 *  PACK_ROWS      0: out[(a5 + co)*a4 + tap*a3 + ci] = w0[co][ci][tap] (fp32 source) for ci < a1;
 *                    a0 = Cout, a1 = Cin, a2 = ntaps, a3 = Cpad, a4 = Kpad, a5 = row0,
 *                    a6 = rows per task; count = ceil(Cout / a6).  Padding is not written.
 *  PACK_TRANSPOSE 1: out[c*a3 + r] = w0[r*a2 + c] for r < a0, c < a1 (both of `dtype`), in
 *                    64x64 tiles; a4 = ceil(a1 / 64); count = ceil(a0 / 64) * a4.  w0 / out point
 *                    at the first element of the sub-matrices.
 *  PACK_CONCAT    4: fp32 out[i] = w0[i] (i < a0), w1[i - a0] (< a0 + a1), w2[...] (< a0+a1+a2),
 *                    else 0, up to a3; count 1
 *  PACK_BIAS4     5: fp32 out[ij*a0 + co] = w0[co], ij < 4; count 1
 * dtype: element type of `out` (ROWS) / of both operands (TRANSPOSE).  A transpose that reads
 * a ROWS output must run in a later launch (the host splits the plan into two tables).
 * Replaces the per-step weight casts/permutations ATen performs inside every conv call of
 * models/unet_dfc_sa_res.py:58-88, :147-156. */
#define DFCSA_PACK_ROWS 0
#define DFCSA_PACK_TRANSPOSE 1
#define DFCSA_PACK_CONCAT 4
#define DFCSA_PACK_BIAS4 5
typedef struct {
  int64_t start, count;
  int kind, dtype;
  const float* w0;
  const float* w1;
  const float* w2;
  void* out;
  int a[8];
} dfcsa_pack_entry;
int dfcsa_pack_plan(const dfcsa_pack_entry* table_dev, int n, int64_t total, void* stream);

/* zero-fill (used for padded weight rows) */
int dfcsa_zero(void* p, int64_t bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * BatchNorm2d (train: batch statistics, biased variance for normalising, unbiased for
 * running_var, momentum 0.1, eps 1e-5; eval: running statistics).  Replaces
 * native_batch_norm at unet_dfc_sa_res.py:60, :67, :75, :82.
 * finalize: from the conv epilogue slab (sums of the accumulator without bias) and the conv
 * bias, produce per-channel scale/shift (y_bn = y*scale + shift), mean, invstd; update the
 * running statistics and num_batches_tracked in place (training only).  stats rows are
 * ld floats long (stats[t][k][c] at (t*2 + k)*ld + c), so a slice of a wider GEMM works.
 * ---------------------------------------------------------------------------------------- */
int dfcsa_bn_finalize(const float* stats, int ntiles, int C, int ld, int count, const float* conv_bias,
                      const float* gamma, const float* beta, float* running_mean, float* running_var,
                      int64_t* num_batches_tracked, float momentum, float eps, int training,
                      float* scale, float* shift, float* mean, float* invstd, void* stream);
/* out = act(y*scale + shift): act 0 none, 1 relu, 2 sigmoid */
int dfcsa_bn_act(int dtype, int M, int C, const void* y, const float* scale, const float* shift,
                 int act, void* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * DFC block elementwise stages (forward).  unet_dfc_sa_res.py:97-114, :36-38.
 * ---------------------------------------------------------------------------------------- */
/* local = relu(bn1(y1)); attn = gamma * bilinear(o -> H x W) + act(bn2(y2)), act = relu when
 * relu != 0 else identity (standalone LightSelfAttention).  y1 may be NULL (no local output).
 * o: fp32 [B][P][P][C]; gamma: device scalar. */
int dfcsa_block_local_attn(int dtype, int B, int H, int W, int C, const void* y1, const float* sc1,
                           const float* sh1, const void* y2, const float* sc2, const float* sh2,
                           const float* o, int P, const float* gamma, int relu, void* local, void* attn,
                           void* stream);
/* fused = g*local + (1-g)*attn, g = sigmoid(bn3(y3)) */
int dfcsa_gate_fuse(int dtype, int M, int C, const void* y3, const float* sc3, const float* sh3,
                    const void* local, const void* attn, void* fused, void* stream);
/* out = relu(bn4(y4)) + res_scale * res */
int dfcsa_block_out(int dtype, int M, int C, const void* y4, const float* sc4, const float* sh4,
                    const void* res, const float* res_scale, void* out, void* stream);

/* encoder block output fused with the 2x2 max-pool after it (even H, W): out = relu(bn4(y4)) +
 * res_scale*res (stored: the decoder skip) and pooled = MaxPool2d(2,2)(out) (first maximum, NaN
 * wins) in one pass (reference models/unet_dfc_sa_res.py:113-114, :165-172) */
int dfcsa_block_out_pool(int dtype, int B, int H, int W, int C, const void* y4, const float* sc4,
                         const float* sh4, const void* res, const float* res_scale, void* out, void* pooled,
                         void* stream);
/* ------------------------------------------------------------------------------------------
 * Backward elementwise + per-channel reductions.  Partial slabs: [ntiles][nsum][C] fp32 with
 * ntiles = dfcsa_ew_ntiles(M, C); dz = gradient at the BatchNorm output, xh = normalised input.
 * ---------------------------------------------------------------------------------------- */
int dfcsa_ew_ntiles(int M, int C);
/* block output: dz4 = dout*(y4*sc4+sh4 > 0); dres = res_scale*dout;
 * sums: [sum dz4, sum dz4*xh4, sum dout*res] */
int dfcsa_bwd_block_out(int dtype, int M, int C, const void* dout, const void* y4, const float* sc4,
                        const float* sh4, const float* mean4, const float* invstd4, const void* res,
                        const float* res_scale, void* dz4, void* dres, float* partial, int64_t partial_floats, void* stream);
/* its backward: dout = dskip (NULL: 0) + maxpool_bwd(dpooled) routed by the saved `out`, stored,
 * then dfcsa_bwd_block_out on it (dres = res_scale*dout; sums [dz4, dz4*xh4, dout*res]) in one
 * pass; partial [dfcsa_bwd_block_out_pool_ntiles(B, H, W, C)][3][C] */
int dfcsa_bwd_block_out_pool_ntiles(int B, int H, int W, int C);
int dfcsa_bwd_block_out_pool(int dtype, int B, int H, int W, int C, const void* dskip, const void* out,
                             const void* dpooled, const void* y4, const float* sc4, const float* sh4,
                             const float* mean4, const float* invstd4, const void* res, const float* res_scale,
                             void* dout, void* dres, float* partial, int64_t partial_floats, void* stream);
/* dz = dact * (y*sc+sh > 0); sums [sum dz, sum dz*xh] */
int dfcsa_bwd_relu_bn(int dtype, int M, int C, const void* dact, const void* y, const float* sc,
                      const float* sh, const float* mean, const float* invstd, void* dz,
                      float* partial, int64_t partial_floats, void* stream);
/* two dfcsa_bwd_relu_bn statistics passes (dz not stored) of the same shape in one launch:
 * (dact0, y0, bn 0) -> partial0 and (dact1, y1, bn 1) -> partial1, each of dfcsa_ew_ntiles(M, C) rows
 * of [2][C] (partial_floats: the capacity of each) -- a DFC block's local-branch and attention-entry
 * BatchNorm-backward sums */
int dfcsa_bwd_relu_bn_pair(int dtype, int M, int C, const void* dact0, const void* y0, const float* sc0,
                           const float* sh0, const float* mean0, const float* invstd0, float* partial0,
                           const void* dact1, const void* y1, const float* sc1, const float* sh1,
                           const float* mean1, const float* invstd1, float* partial1, int64_t partial_floats,
                           void* stream);
/* gate: g = sigmoid(y3*sc3+sh3); dz3 = dfused*(local-attn)*g*(1-g); dlocal += dfused*g;
 * dattn += dfused*(1-g); sums [sum dz3, sum dz3*xh3] */
int dfcsa_bwd_gate(int dtype, int M, int C, const void* dfused, const void* y3, const float* sc3,
                   const float* sh3, const float* mean3, const float* invstd3, const void* local,
                   const void* attn, void* dlocal, void* dattn, void* dz3, float* partial, int64_t partial_floats,
                   void* stream);
/* fusion-conv input gradient with the gate backward in the epilogue (bf16, C % 64 == 0,
 * C <= 256): [dfused | dlocal | dattn] = dy4 . W4t (W4t = dfcsa_conv_gemm's [3C][Kpad] dgrad
 * operand of the fusion conv), each rounded to bf16 as the unfused GEMM stores them, then
 * dfcsa_bwd_gate's arithmetic on them: dlocal/dattn written (not accumulated), dz3 written,
 * dfused never stored.  Sums [sum dz3, sum dz3*xh3] per workgroup row: partial
 * [dfcsa_dgrad_gate_parts(M, C)][2][C].  Replaces the dgrad GEMM + dfcsa_bwd_gate pair
 * (reference models/unet_dfc_sa_res.py:102-110 backward). */
int dfcsa_dgrad_gate_parts(int M, int C);
int dfcsa_dgrad_gate(int M, int C, const void* dy4, const void* w4t, int Kpad, const void* y3,
                     const float* sc3, const float* sh3, const float* mean3, const float* invstd3,
                     const void* local, const void* attn, void* dlocal, void* dattn, void* dz3,
                     float* partial, int64_t partial_floats, void* stream);
/* fusion conv forward with the gate fusion in its A-operand prologue (bf16, C == 64 or 128, Kpad == 3C):
 * fused = g*local + (1-g)*attn, g = sigmoid(y3*sc3+sh3) (dfcsa_gate_fuse's arithmetic), stored;
 * y4 = [fused | local | attn] . w4^T + b4 (w4 = the fusion conv's [C][3C] forward operand) with
 * BatchNorm partial statistics (stats4 [parts][2][C], see below).  Replaces the
 * dfcsa_gate_fuse + dfcsa_conv_gemm pair (reference models/unet_dfc_sa_res.py:102-110).
 * The statistics slab holds ONE row per workgroup (rows [0, dfcsa_fwd_pro_parts(M, C, 0))), the
 * sums of that workgroup's 64-row tiles: dfcsa_bn_finalize takes that row count as ntiles. */
int dfcsa_fwd_pro_parts(int M, int C, int pro);
int dfcsa_gate_fusion_fwd(int M, int C, const void* y3, const float* sc3, const float* sh3, const void* local,
                          const void* attn, const void* w4, int Kpad, const float* b4, void* fused, void* y4,
                          float* stats4, int64_t stats4_floats, void* stream);
/* gate conv forward with the local/attention merge in its A-operand prologue (bf16, C == 64 or 128
 * (round 4), Kpad == 2C, relu): local = relu(y1*sc1+sh1), attn = gamma*bilinear(o) + relu(y2*sc2+sh2)
 * (dfcsa_block_local_attn's arithmetic; o fp32 [B][P][P][C]), both stored; y3 = [local | attn] .
 * w3^T + b3 with BatchNorm partial statistics (one row per workgroup: dfcsa_fwd_pro_parts(M, C, 1) rows).  Replaces the
 * dfcsa_block_local_attn + dfcsa_conv_gemm pair (reference models/unet_dfc_sa_res.py:36-38, 97-102). */
int dfcsa_local_attn_gate_fwd(int B, int H, int W, int C, const void* y1, const float* sc1, const float* sh1,
                              const void* y2, const float* sc2, const float* sh2, const float* o, int P,
                              const float* gamma, const void* w3, int Kpad, const float* b3, void* local,
                              void* attn, void* y3, float* stats3, int64_t stats3_floats, void* stream);
/* The two prologue GEMMs above with their BatchNorm finalised in the launch's tail (round 5; the
 * fold of dfcsa_conv_gemm_bn: f->C == C, the statistics rows are the workgroups).  With the fold
 * off (tuning knob 39) or no ticket space they launch dfcsa_bn_finalize after the GEMM instead.
 * Outputs f->scale/shift/mean/invstd and the running statistics as dfcsa_bn_finalize (training). */
int dfcsa_gate_fusion_fwd_bn(int M, int C, const void* y3, const float* sc3, const float* sh3, const void* local,
                             const void* attn, const void* w4, int Kpad, const float* b4, void* fused, void* y4,
                             float* stats4, int64_t stats4_floats, const dfcsa_bn_fold* f, void* stream);
int dfcsa_local_attn_gate_fwd_bn(int B, int H, int W, int C, const void* y1, const float* sc1, const float* sh1,
                                 const void* y2, const float* sc2, const float* sh2, const float* o, int P,
                                 const float* gamma, const void* w3, int Kpad, const float* b3, void* local,
                                 void* attn, void* y3, float* stats3, int64_t stats3_floats,
                                 const dfcsa_bn_fold* f, void* stream);
/* dfcsa_dgrad_gate / dfcsa_dgrad_acc_relu_bn at C == 64 with the BatchNorm-backward apply of their
 * A operand in a prologue: dy4 = gamma4*invstd4*(dz4 - coef4[0] - xh4*coef4[1]) with dz4 =
 * dout*(y4*sc4+sh4 > 0) (dfcsa_bn_bwd_apply_relu; sc4 = sh4 = NULL: dz4 = dout) and dy3 likewise from
 * dz3 (dfcsa_bn_bwd_apply), formed in LDS from the DMA'd [dout | y4] / [dz3 | y3] image, stored
 * once (dy4, dy3: the weight gradients read them) and multiplied.  The conv-bias gradient is the
 * analytic zero (no bias sums).  partial rows: dfcsa_dgrad_apply_parts(M, 0 = gate / 1 = acc). */
int dfcsa_dgrad_apply_parts(int M, int epi);
int dfcsa_dgrad_gate_apply(int M, const void* dout, const void* y4, const float* gamma4, const float* coef4,
                           const float* mean4, const float* invstd4, const float* sc4, const float* sh4, void* dy4,
                           const void* w4t, const void* y3, const float* sc3, const float* sh3, const float* mean3,
                           const float* invstd3, const void* local, const void* attn, void* dlocal, void* dattn,
                           void* dz3, float* partial, int64_t partial_floats, void* stream);
int dfcsa_dgrad_acc_relu_bn_apply(int M, const void* dz3, const void* y3, const float* gamma3, const float* coef3,
                                  const float* mean3, const float* invstd3, void* dy3, const void* w3t,
                                  const void* y1, const float* sc1, const float* sh1, const float* mean1,
                                  const float* invstd1, void* dlocal, void* dattn, float* partial, int64_t partial_floats, void* stream);
/* gate-conv input gradient added into [dlocal | dattn] (bf16, C % 64 == 0, C <= 256): dlocal +=
 * (dy3 . W3t)[:, :C], dattn += (dy3 . W3t)[:, C:] (W3t = the [2C][Kpad] dgrad operand of the gate
 * conv; same bf16 roundings as dfcsa_conv_gemm's accumulate mode), and on the final dlocal the
 * sums of dfcsa_bwd_relu_bn (dz1 = dlocal*(y1*sc1+sh1 > 0): [sum dz1, sum dz1*xh1]) per
 * workgroup row: partial [dfcsa_dgrad_acc_relu_bn_parts(M, C)][2][C].  Replaces the accumulate
 * GEMM + dfcsa_bwd_relu_bn pair (reference models/unet_dfc_sa_res.py:57-62, :73-77 backward). */
int dfcsa_dgrad_acc_relu_bn_parts(int M, int C);
int dfcsa_dgrad_acc_relu_bn(int M, int C, const void* dy3, const void* w3t, int Kpad, const void* y1,
                            const float* sc1, const float* sh1, const float* mean1, const float* invstd1,
                            void* dlocal, void* dattn, float* partial, int64_t partial_floats, void* stream);
/* attention entry: dz2 = (dattn + adaptive_pool^T(dpooled)) * (y2*sc2+sh2 > 0) (mask only when
 * relu != 0); dpooled fp32 [B][P][P][C]; sums [sum dz2, sum dz2*xh2] */
int dfcsa_bwd_attn_entry(int dtype, int B, int H, int W, int C, const void* dattn, const float* dpooled,
                         int P, const void* y2, const float* sc2, const float* sh2, const float* mean2,
                         const float* invstd2, int relu, void* dz2, float* partial, int64_t partial_floats, void* stream);
/* from partial sums: coef[0][c] = mean dz, coef[1][c] = mean dz*xh; dgamma += sum dz*xh,
 * dbeta += sum dz; nsum == 3: coef holds [3][C] floats and coef[2][c] = the third sum, and with
 * extra != null the launch also adds sum over c of it to *extra (round 5: with extra == null the
 * caller may sum coef[2][.] itself, e.g. dfcsa_sum_into on another stream). */
int dfcsa_bn_bwd_finalize(const float* partial, int ntiles, int nsum, int C, int count,
                          float* coef, float* dgamma, float* dbeta, float* extra, void* stream);
/* dfcsa_bn_bwd_finalize (nsum = 2) for a DFC block's attention entry: `partial` holds the sums of
 * dfcsa_bwd_relu_bn over dattn alone, and the launch adds the pool-backward part from the forward
 * pool's window sums (dfcsa_lsa_pooled_ws: wsum [B][P*P][2][C]) and dpooled [B][P*P][C]:
 *   sum r*pb = sum_{b,n} dpooled/area_n * R,  sum r*pb*xhat = sum dpooled/area_n * invstd*(Y - mean*R)
 * -- the same coefficients as dfcsa_bwd_attn_entry's statistics, without its full-resolution pass
 * after the attention backward (adaptive windows of an H x W map pooled to P x P). */
int dfcsa_bn_bwd_finalize_pool(const float* partial, int ntiles, int C, int count, float* coef, float* dgamma,
                               float* dbeta, const float* dpooled, const float* wsum, int B, int H, int W, int P,
                               const float* mean, const float* invstd, void* stream);
/* dy = gamma*invstd*(dz - coef0 - xh*coef1); partial column sums of dy -> bias_partial
 * [ntiles][C] (conv bias gradient; NULL = not computed: for a conv feeding a train-mode
 * BatchNorm it is exactly zero, sum_m dy = gamma*invstd*(sum dz - M*coef0 - coef1*sum xh) = 0) */
int dfcsa_bn_bwd_apply(int dtype, int M, int C, const void* dz, const void* y, const float* mean,
                       const float* invstd, const float* gamma, const float* coef, void* dy,
                       float* bias_partial, int64_t bias_partial_floats, void* stream);
/* dfcsa_bn_bwd_apply with dz recomputed from the activation's output gradient instead of read
 * from a dz tensor (the producing stage -- dfcsa_bwd_relu_bn / dfcsa_bwd_block_out with dz = NULL
 * -- then only emits its partial sums): dz = (y*sc + sh > 0) ? dact : 0.  Replaces the BN/ReLU
 * backward of reference models/unet_dfc_sa_res.py:57-62, :65-69, :80-84 (autograd). */
int dfcsa_bn_bwd_apply_relu(int dtype, int M, int C, const void* dact, const void* y, const float* sc,
                            const float* sh, const float* mean, const float* invstd, const float* gamma,
                            const float* coef, void* dy, float* bias_partial, int64_t bias_partial_floats, void* stream);
/* the same for the attention entry a = relu(bn2 y2) (reference :65-69 + the adaptive-avg-pool of
 * :24 and the residual of :38): dz = act'(bn y) * (dattn + pool_backward(dpooled)); pairs with
 * dfcsa_bwd_attn_entry(dz2 = NULL). */
int dfcsa_bn_bwd_apply_entry(int dtype, int B, int H, int W, int C, const void* dattn, const float* dpooled, int P,
                             const void* y, const float* sc, const float* sh, const float* mean,
                             const float* invstd, int relu, const float* gamma, const float* coef, void* dy,
                             float* bias_partial, int64_t bias_partial_floats, void* stream);
/* the same with dpooled in bf16 (the bf16 flash layers' projection dgrad output as it is; 16-B aligned) */
int dfcsa_bn_bwd_apply_entry16(int dtype, int B, int H, int W, int C, const void* dattn, const void* dpooled16, int P,
                               const void* y, const float* sc, const float* sh, const float* mean,
                               const float* invstd, int relu, const float* gamma, const float* coef, void* dy,
                               float* bias_partial, int64_t bias_partial_floats, void* stream);
/* Two-stage reduction helper for per-tile slabs: dst[g][j] = sum of rows t in group g of
 * src[t][j] (T rows of rowlen floats, G groups of ceil(T/G) consecutive rows).  The finalize
 * entry points then reduce G rows instead of T.  dst: [G][rowlen] fp32 (caller scratch). */
int dfcsa_rows_reduce(const float* src, int T, int rowlen, float* dst, int G, void* stream);
/* out[c] += sum_t slab[t][c]  (ntiles x C); fp64 accumulation */
int dfcsa_slab_colsum(const float* slab, int ntiles, int C, float* out, void* stream);
/* as dfcsa_slab_colsum with columns [0,n0) -> d0, [n0,n0+n1) -> d1, [n0+n1,C) -> d2 */
int dfcsa_slab_colsum3(const float* slab, int ntiles, int C, int n0, int n1, float* d0, float* d1, float* d2,
                       void* stream);
/* per-channel partial sums of an NHWC tensor -> partial [ntiles][C] */
int dfcsa_channel_sum(int dtype, int M, int C, const void* x, float* partial, int64_t partial_floats, void* stream);

/* ------------------------------------------------------------------------------------------
 * LightSelfAttention on the pooled map (unet_dfc_sa_res.py:20-39).  Pooled tensors are fp32
 * [B][N][C], N = P*P (n = pi*P + pj); qkv = [B][N][2*Cq + C] (q | k | v).
 * ---------------------------------------------------------------------------------------- */
int dfcsa_lsa_pool_splits(int H, int P);
/* partial[b][n][s][c] = sum over the s-th row slice of window n of act(y2*sc2+sh2) */
int dfcsa_lsa_pool(int dtype, int B, int H, int W, int C, const void* y2, const float* sc2,
                   const float* sh2, int P, int relu, float* partial, void* stream);
/* pooled = partial sums / window area  ([B][N][C] fp32) */
int dfcsa_lsa_pooled(int B, int H, int W, int C, int P, const float* partial, float* pooled, void* stream);
/* dfcsa_lsa_pool / dfcsa_lsa_pooled that also form the window sums of the relu mask of the pooled
 * activation, r = [y*sc + sh > 0] (r = 1 without relu): wpart [B][N][S][2][C] (S =
 * dfcsa_lsa_pool_splits) holds per-slice sum r and sum r*y, and the pooled launch reduces them into
 * wsum [B][N][2][C].  The attention-entry backward then needs no full-resolution statistics pass of
 * its own (dfcsa_bn_bwd_finalize_pool). */
int dfcsa_lsa_pool_ws(int dtype, int B, int H, int W, int C, const void* y2, const float* sc2,
                      const float* sh2, int P, int relu, float* partial, float* wpart, void* stream);
int dfcsa_lsa_pooled_ws(int B, int H, int W, int C, int P, const float* partial, float* pooled,
                        const float* wpart, float* wsum, void* stream);
/* Large pools or small windows (P >= 16, or P >= 8 with windows of <= 8 x 8 pixels; C / 8 a power of two or a multiple
 * of 64: dfcsa_lsa_pool_direct_ok): the pool in
 * ONE launch, one wave per window -- pooled [B][N][C] fp32 = window mean of act(y2*sc2+sh2); pooled16
 * (bf16 [B][N][C]) the same values rounded (either may be NULL, not both); wsum (optional, [B][N][2][C]) the window sums of
 * dfcsa_lsa_pooled_ws.  Replaces dfcsa_lsa_pool_ws + dfcsa_lsa_pooled_ws (+ the bf16 cast) there. */
int dfcsa_lsa_pool_direct_ok(int C, int P, int H, int W);
int dfcsa_lsa_pool_direct(int dtype, int B, int H, int W, int C, const void* y2, const float* sc2,
                          const float* sh2, int P, int relu, float* pooled, void* pooled16, float* wsum,
                          void* stream);
/* pooled = partial sums / window area; qkv = pooled @ wT + b  (wT: [C][2Cq+C] fp32) */
int dfcsa_lsa_qkv(int B, int H, int W, int C, int Cq, int P, const float* partial, const float* wT,
                  const float* bias, float* pooled, float* qkv, void* stream);
/* A = softmax_rows(q k^T) [B][N][N]; o[n][c] = sum_m A[n][m] v[m][c]  [B][N][C] */
int dfcsa_lsa_attn(int B, int N, int C, int Cq, const float* qkv, float* A, float* o, void* stream);
/* Pooled attention for large pools (P >= 8: configs/config_dfc-sa-res-block-p16.yaml / -p32.yaml,
 * N = 256 / 1024 tokens; replaces the bmm -> softmax -> bmm of unet_dfc_sa_res.py:30-33 and their
 * autograd backward) on the flash kernels of fra.hip with gamma = 1: nothing N x N is stored.
 *   fwd: o [B][N][C] fp32 = softmax_rows(q k^T) v, lse [B*N] = log-sum-exp of each score row.
 *   bwd: dqkv [B][N][ldq] (the dtype of qkv) from dO [B][N][C] fp32 (= gamma * U^T dattn) and the
 *        saved o / lse; work: dfcsa_lsa_flash_bwd_bytes bytes of device scratch (16-byte aligned).
 * qkv [B][N][ldq], ldq = 2Cq + C, C <= 1024, is fp32 (dtype DFCSA_DT_F32: the generic fp32 kernels)
 * or bf16 (DFCSA_DT_BF16: bf16 MFMA kernels, only where dfcsa_lsa_flash_path(C, Cq, ldq) returns 1:
 * C % 64 == 0, Cq a power of two in [8, 128]; the q/k/v projections then run as bf16 GEMMs too, as
 * the reference's 1x1 convs do under bf16 autocast). */
int dfcsa_lsa_flash_path(int C, int Cq, int ldq);
int dfcsa_lsa_flash_fwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, float* o, float* lse,
                        void* stream);
int dfcsa_lsa_flash_bwd_bytes(int dtype, int B, int N, int C, int Cq, int ldq, int64_t* bytes);
int dfcsa_lsa_flash_bwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const float* dO,
                        const float* o, const float* lse, void* dqkv, void* work, int64_t work_bytes, void* stream);
/* The attention entry's pool-backward BatchNorm sums as ceil(BN/16) partial rows [row][2][C] (the rows
 * dfcsa_conv_wgrad_dgrad1x1_pool's epilogue adds for the fp32 projections), from dpooled [BN][C] (dtype:
 * fp32, or bf16 -- the flash layers' projection dgrad output as it is) and the forward's window sums
 * wsum [BN][2][C]: for the bf16 projections of the flash layers.  rows_floats: capacity of rows in floats. */
int dfcsa_lsa_pool_rows(int dtype, int BN, int C, int P, int H, int W, const void* dpooled, const float* wsum,
                        const float* mean, const float* invstd, float* rows, int64_t rows_floats, void* stream);
/* bf16 flash layers: dfcsa_lsa_up_bwd_cols (gamma_grad NULL) + dfcsa_lsa_flash_bwd in one call, the
 * column pass writing the flash backward's bf16 dO and r itself (one wave per token; the fp32 dO is never
 * formed): rows [B][H][P][C] (dfcsa_lsa_up_bwd_rows), o [B][N][C] fp32, qkv16 / lse / dqkv16 / work as
 * dfcsa_lsa_flash_bwd (work sized by dfcsa_lsa_flash_bwd_bytes with dtype bf16), gpart [B*N] the
 * per-token dgamma partials (sum them: dfcsa_sum_to_scalar).  H <= 29 P; knob 49 = 0 refuses. */
int dfcsa_lsa_flash_bwd_up(int B, int H, int C, int Cq, int P, const float* rows, const float* o,
                           const float* gamma, const void* qkv16, const float* lse, void* dqkv16,
                           float* gpart, void* work, int64_t work_bytes, void* stream);
/* dst[i] = src[i] (bf16 -> fp32), n % 8 == 0, 16-byte aligned pointers */
int dfcsa_bf16_to_f32(int64_t n, const void* src, float* dst, void* stream);
/* backward through the bilinear upsample: rows[b][h][pj][c] = sum_w wx(pj,w) dattn[b,h,w,c] */
int dfcsa_lsa_up_bwd_rows(int dtype, int B, int H, int W, int C, const void* dattn, int P, float* rows,
                          void* stream);
/* du[b][pi][pj][c] = sum_h wy(pi,h) rows[b][h][pj][c]; do = gamma*du; gpart[b*P*P + n] = sum_c o*du;
 * gamma_grad != NULL: *gamma_grad += sum of gpart (fixed order, by the last workgroup: no extra
 * launch); ngpart != NULL receives the gpart count B*P*P */
int dfcsa_lsa_up_bwd_cols(int B, int H, int C, int P, const float* rows, const float* o,
                          const float* gamma, float* dO, float* gpart, int* ngpart, float* gamma_grad,
                          void* stream);
/* attention core backward -> dqkv [B][N][2Cq+C]; dE scratch [B][N][N] */
/* P <= 4, C <= 1024, C % 8 == 0, Cq even: dfcsa_lsa_up_bwd_cols + dfcsa_lsa_attn_bwd in one launch (one
 * workgroup per token and image; the image's last workgroup forms dk / dv): dqkv [B][N][2Cq+C];
 * dO [B][N][C], dE [B][N][N], gpart [B*N] scratch; dgamma added to *gamma_grad (last workgroup). */
int dfcsa_lsa_core_bwd(int B, int H, int C, int Cq, int P, const float* rows, const float* o, const float* gamma,
                       const float* qkv, const float* A, float* dqkv, float* dO, float* dE, float* gpart,
                       float* gamma_grad, void* stream);
int dfcsa_lsa_attn_bwd(int B, int N, int C, int Cq, const float* qkv, const float* A, const float* dO,
                       float* dE, float* dqkv, void* stream);
/* projection backward: dW[j][c] += sum_bn dqkv[bn][j]*pooled[bn][c] (w layout [2Cq+C][C]);
 * db[j] += sum_bn dqkv[bn][j]; dpooled[bn][c] = sum_j dqkv[bn][j] * w[j][c] */
int dfcsa_lsa_proj_bwd(int B, int N, int C, int Cq, const float* dqkv, const float* pooled,
                       const float* w, float* dWq, float* dWk, float* dWv, float* dbq, float* dbk,
                       float* dbv, float* dpooled, void* stream);
/* out += sum of n floats (single workgroup, fp64) */
int dfcsa_sum_to_scalar(const float* x, int n, float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * U-Net plumbing: MaxPool2d(2,2) (unet_dfc_sa_res.py:132-141), input layout conversion,
 * the bilinear shape fix (:180-199), final 1x1 head (:159, :203).
 * ---------------------------------------------------------------------------------------- */
int dfcsa_maxpool2_fwd(int dtype, int B, int H, int W, int C, const void* x, void* out, void* stream);
/* dx += scatter of dout to the first maximum of each 2x2 window (PyTorch tie/NaN order) */
int dfcsa_maxpool2_bwd(int dtype, int B, int H, int W, int C, const void* x, const void* dout, void* dx,
                       void* stream);
/* NCHW fp32 [B][Cin][H][W] -> NHWC dtype [B][H][W][Cpad] (zero channels Cin..Cpad-1) */
int dfcsa_pack_input(int dtype, int B, int Cin, int H, int W, const float* x, int Cpad, void* out,
                     void* stream);
/* NHWC [B][Hi][Wi][C] -> [B][Ho][Wo][C], bilinear, align_corners=False */
int dfcsa_resize_bilinear(int dtype, int B, int C, int Hi, int Wi, int Ho, int Wo, const void* x,
                          void* out, void* stream);
/* dx (fp32 accumulation buffer [B][Hi][Wi][C], must be zeroed) += resize^T(dout) */
int dfcsa_resize_bilinear_bwd(int dtype, int B, int C, int Hi, int Wi, int Ho, int Wo, const void* dout,
                              float* dx32, void* stream);
/* fp32 buffer -> dtype tensor (out = x, or out += x when accumulate) */
int dfcsa_cast_f32(int dtype, int64_t n, const float* x, void* out, int accumulate, void* stream);
/* logits NCHW fp32 [B][Cout][HW] = x[M][C] @ w^T + b   (w fp32 [Cout][C]) */
int dfcsa_head_fwd(int dtype, int B, int HW, int C, int Cout, const void* x, const float* w,
                   const float* b, float* logits, void* stream);
/* dx[M][C] = dlogit @ w; partial_w [ntiles][Cout][C], partial_b [ntiles][Cout] */
int dfcsa_head_bwd(int dtype, int B, int HW, int C, int Cout, const void* x, const float* w,
                   const float* dlogit, void* dx, float* partial_w, float* partial_b, int* ntiles,
                   void* stream);

/* ------------------------------------------------------------------------------------------
 * Loss and metrics: torch.sigmoid (utils/trainer.py:124) + calculate_metrics('bce_dice')
 * (utils/metrics.py:211-264 -> BCEDiceLoss :52-78 -> BCELoss + dice_loss :6-24).
 * stats (fp32[8]): [loss, bce_sum, sum p*t, sum p, sum t, sum b*t, sum b, finite(1/0)],
 * b = (p > 0.5).
 * ---------------------------------------------------------------------------------------- */
int dfcsa_sigmoid(int64_t n, const float* x, float* y, void* stream);
int dfcsa_sigmoid_bwd(int64_t n, const float* y, const float* dy, float* dx, void* stream);
int dfcsa_bce_dice_partial_count(int64_t n);
int dfcsa_bce_dice_fwd(int64_t n, const float* p, const float* t, float* partial, float wbce, float wdice,
                       float* stats, void* stream);
/* dp = dloss * (wbce*(p-t)/max(p(1-p),1e-12)/n + wdice*d(1-dice)/dp) */
int dfcsa_bce_dice_bwd(int64_t n, const float* p, const float* t, const float* stats, float wbce,
                       float wdice, const float* dloss, float* dp, void* stream);

/* ------------------------------------------------------------------------------------------
 * clip_grad_norm_(max_norm) + SGD(momentum, weight_decay) over one flat fp32 parameter
 * buffer (utils/trainer.py:149-151, train.py:73-78).  grad_scale multiplies the gradient
 * first (1/world_size after an all-reduce sum).  If *skip_if_nan is NaN the step is skipped on
 * the device (the reference's NaN-loss `continue`, trainer.py:134-139; an inf loss still steps).
 * A NaN total norm gives a NaN clip coefficient (torch's clip_grad_norm_).  partial: nparts fp64
 * per-block sums of squares.
 * *mom_init == 0 -> momentum buffer = d (torch's first step), then set to 1.
 * ---------------------------------------------------------------------------------------- */
int dfcsa_sumsq_nparts(int64_t n);
int dfcsa_sumsq_partial(int64_t n, const float* g, double* partial, void* stream);
int dfcsa_clip_sgd(int64_t n, float* w, float* g, float* buf, const double* partial, int nparts,
                   float max_norm, float grad_scale, float lr, float momentum, float weight_decay,
                   int* mom_init, const float* skip_if_nan, float* norm_out, void* stream);
/* dfcsa_clip_sgd with a momentum buffer that starts at zero instead of a first-step flag
 * (buf = momentum * 0 + d == d exactly: torch's first step, one launch instead of two);
 * zero_grad != 0 writes zeros to g instead of the clipped gradient (also on a skipped step), so
 * the caller's next zero_grad needs no memset pass. */
int dfcsa_clip_sgd2(int64_t n, float* w, float* g, float* buf, const double* partial, int nparts,
                    float max_norm, float grad_scale, float lr, float momentum, float weight_decay,
                    int zero_grad, const float* skip_if_nan, float* norm_out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Full-resolution self-attention (models/unet_dfc_sa_ablation_attention.py:15-26, the attention
 * of FullResAttnDFCBlock / UNet_FullResAttention, config_ablation3_full_res_attn.yaml), flash-style:
 * the N x N score matrix is never stored.  Per image (N = H*W tokens) qkv is NHWC [B][N][ldq] with
 * q at columns [0,Cq), k at [Cq,2Cq), v at [2Cq,2Cq+C) (the 1x1 projections, done by
 * dfcsa_conv_gemm); A = softmax_rows(q k^T) (no scale), O = A v.
 * fwd: o = O [B][N][C], y = gamma*O + x [B][N][C] (dtype), lse [B*N] fp32 = log-sum-exp of each
 *      score row (saved for the backward).
 * bwd_prep: r[row] = sum_c dy*o (dgamma = sum r; delta = gamma*r).
 * bwd: dqkv [B][N][ldq] = gradients of q, k, v for dy at y (padding columns zeroed); P is
 *      recomputed from lse.
 * path: 1 if the bf16 MFMA kernels serve this shape (fwd: C % 64 == 0, Cq in {8..128} powers of 2;
 *      bwd: C in {64, 128, 256}, Cq in {8, 16, 32}), 2 (bwd only: bf16, C > 256, C % 128 == 0 --
 *      the 64^2 / 32^2 levels) = dfcsa_fra_bwd_wide, 0 = the generic kernels (fp32, other shapes).
 * bwd_wide: the same MFMA kernels over value-column chunks of 128 (dP = dy V^T is a sum over value
 *      columns and dS is linear in dP, so dQ / dK are exact sums of per-chunk shares, kept as fp32
 *      partials in `work` and summed in fixed chunk order; dV columns are written per chunk).
 *      work: dfcsa_fra_bwd_wide_bytes(B, N, C, Cq) bytes of device memory.
 * ---------------------------------------------------------------------------------------- */
int dfcsa_fra_path(int dtype, int C, int Cq, int ldq, int backward);
int dfcsa_fra_fwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const void* x,
                  const float* gamma, void* o, void* y, float* lse, void* stream);
int dfcsa_fra_bwd_prep(int dtype, int rows, int C, const void* dy, const void* o, float* r, void* stream);
int dfcsa_fra_bwd(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const void* dy,
                  const float* gamma, const float* lse, const float* r, void* dqkv, void* stream);
int dfcsa_fra_bwd_wide_bytes(int B, int N, int C, int Cq, int64_t* bytes);
int dfcsa_fra_bwd_wide(int dtype, int B, int N, int C, int Cq, int ldq, const void* qkv, const void* dy,
                       const float* gamma, const float* lse, const float* r, void* dqkv, float* work, void* stream);

/* ------------------------------------------------------------------------------------------
 * Plain U-Net (models/unet.py, BASELINE config 1): MaxPool2d(2, ceil_mode=True) (:26) and the
 * crop-to-match of Up.forward (:47-55), NHWC, C % 8 == 0.
 * ---------------------------------------------------------------------------------------- */
/* out [B][ceil(H/2)][ceil(W/2)][C] = max over the in-bounds pixels of each 2x2 window
 * (first maximum in window order, NaN propagates, as ATen) */
int dfcsa_maxpool2_ceil_fwd(int dtype, int B, int H, int W, int C, const void* x, void* out, void* stream);
/* dx (every element written) = dout at the window's first maximum, 0 elsewhere */
int dfcsa_maxpool2_ceil_bwd(int dtype, int B, int H, int W, int C, const void* x, const void* dout, void* dx,
                            void* stream);
/* dst [B][Hd][Wd][C]: dst[b][h][w][c] = src[b][h + oy][w + ox][c] inside src [B][Hs][Ws][C], else 0
 * (a crop for oy, ox >= 0; its backward with -oy, -ox) */
int dfcsa_window_copy(int dtype, int B, int C, int Hs, int Ws, const void* src, int Hd, int Wd, void* dst, int oy,
                      int ox, void* stream);

/* ------------------------------------------------------------------------------------------
 * TransUNet R50-ViT-B/16 (models/transformer_unet.py, BASELINE config 4).  Convolutions and
 * Linear layers run on dfcsa_conv_gemm / dfcsa_conv_wgrad; these are the remaining operations.
 * ---------------------------------------------------------------------------------------- */
/* StdConv2d weight standardisation (transformer_unet.py:21-27), one launch for a table of convs:
 * rows [row0, row0 + rows) of the table's global row space belong to entry e (sorted by row0);
 * fwd: what[r][k] = (w[r][k] - mean_r)/sqrt(var_r + 1e-5) (biased variance over K), rstd[r] saved;
 * bwd: dw[r][k] += rstd_r*(g - mean(g) - what*mean(g*what)) with g = dL/dwhat. */
typedef struct {
  const float* w;
  float* what;
  float* rstd;
  const float* g;
  float* dw;
  int K, rows, row0, pad;
} dfcsa_wstd_entry;
int dfcsa_wstd_fwd(const dfcsa_wstd_entry* tab, int n, int total_rows, void* stream);
int dfcsa_wstd_bwd(const dfcsa_wstd_entry* tab, int n, int total_rows, void* stream);
/* root conv operand (ResNetV2 root, :77): out[m][tap*Cin + ci] = x[b][ci % Csrc][oh*s-p+kh][ow*s-p+kw]
 * for an NCHW fp32 image (Csrc = 1 repeats the channel, :363-364), zero outside / past k*k*Cin;
 * out [B*Ho*Wo][Kpad] dtype */
int dfcsa_im2col_input(int dtype, int B, int Csrc, int Cin, int H, int W, int k, int s, int p, const float* x,
                       int Kpad, void* out, void* stream);
/* GroupNorm (nn.GroupNorm, :46-67, :78): per image b and group g of C/G channels over HW pixels.
 * stats: partial [B][S][2][C] (S = dfcsa_gn_nslices pixel slices); finalize: mean_rstd [B][2][G],
 * scale_shift [B][2][C] (y*scale + shift = gamma*xhat + beta); apply: out = act(y*scale + shift +
 * r), r = res*res_scale + res_shift (res_scale_shift given) or res (or none); act 1 = ReLU.
 * bwd: dz = dout*(mask > 0) (mask NULL: dz = dout); reduce -> partial [B][S][2][C] (sum dz, sum
 * dz*xhat); finalize -> coef [B][2][G], dgamma/dbeta += ; apply -> dy (and dz_out = dz if given). */
int dfcsa_gn_nslices(int HW, int C);
int dfcsa_gn_stats(int dtype, int B, int HW, int C, int S, const void* y, float* partial, void* stream);
int dfcsa_gn_finalize(int B, int HW, int C, int G, int S, const float* partial, const float* gamma,
                      const float* beta, float eps, float* mean_rstd, float* scale_shift, void* stream);
int dfcsa_gn_apply(int dtype, int B, int HW, int C, const void* y, const float* scale_shift, const void* res,
                   const float* res_scale_shift, int act, void* out, void* stream);
int dfcsa_gn_bwd_reduce(int dtype, int B, int HW, int C, int G, int S, const void* dout, const void* mask,
                        const void* y, const float* mean_rstd, float* partial, void* stream);
int dfcsa_gn_bwd_finalize(int B, int HW, int C, int G, int S, const float* partial, const float* gamma,
                          float* coef, float* dgamma, float* dbeta, void* stream);
int dfcsa_gn_bwd_apply(int dtype, int B, int HW, int C, int G, const void* dout, const void* mask, const void* y,
                       const float* mean_rstd, const float* gamma, const float* coef, void* dy, void* dz_out,
                       void* stream);
/* GroupNorm with the reductions finished inside the launch (round 5; replaces stats + finalize and
 * bwd_reduce + bwd_finalize, same outputs, C <= 1024, G <= 256): grid (S, B, C / CW), S =
 * dfcsa_gn_nslices_fused(B, HW, C), CW = 128 channels (whole groups) for C > 128, else C (round 6);
 * rows: B * S * 2C floats of hand-off scratch; the last workgroup of each (image, chunk) finalises it.  bwd: work [B][2][C] doubles (the images' channel sums,
 * summed in image order by the last image into dgamma / dbeta). */
int dfcsa_gn_nslices_fused(int B, int HW, int C);
int dfcsa_gn_stats_fused(int dtype, int B, int HW, int C, int G, int S, const void* y, float* rows,
                         const float* gamma, const float* beta, float eps, float* mean_rstd, float* scale_shift,
                         void* stream);
int dfcsa_gn_bwd_reduce_fused(int dtype, int B, int HW, int C, int G, int S, const void* dout, const void* mask,
                              const void* y, const float* mean_rstd, const float* gamma, float* rows, double* work,
                              float* coef, float* dgamma, float* dbeta, void* stream);
/* MaxPool2d(kernel 3, stride 2, padding 1) (:101): out [B][Ho][Wo][C], Ho = (H-1)/2 + 1; idx
 * uint8 [B][Ho][Wo][C] = tap (kh*3 + kw) of the first maximum; bwd writes every dx element. */
int dfcsa_maxpool3s2_fwd(int dtype, int B, int H, int W, int C, const void* x, void* out, void* idx, void* stream);
int dfcsa_maxpool3s2_bwd(int dtype, int B, int H, int W, int C, const void* idx, const void* dout, void* dx,
                         void* stream);
/* data gradient of a k x k / stride s / pad p conv from the column gradient dcols [B*Ho*Wo][k*k*C]
 * (= dY @ W, one GEMM): dx [B][H][W][C] (+)= the sum over taps landing on each input pixel */
int dfcsa_col2im(int dtype, int B, int H, int W, int C, int Ho, int Wo, int k, int s, int p, const void* dcols,
                 void* dx, int accumulate, void* stream);
/* LayerNorm over the last dim (:206-207, :226): x fp32 [rows][C] -> y dtype, mean_rstd [rows][2].
 * bwd: dx (fp32) = LN backward + dres (dres fp32 or NULL; may alias dx); partial
 * [dfcsa_ln_bwd_ntiles(rows)][2][C] = (sum dy*xhat, sum dy) for dgamma / dbeta. */
int dfcsa_ln_fwd(int dtype, int rows, int C, const float* x, const float* gamma, const float* beta, float eps,
                 void* y, float* mean_rstd, void* stream);
int dfcsa_ln_bwd_ntiles(int rows);
int dfcsa_ln_bwd(int dtype, int rows, int C, const void* dy, const float* x, const float* mean_rstd,
                 const float* gamma, const float* dres, float* dx, float* partial, void* stream);
/* Dropout (p) with a counter-based mask keyed by the device state rng[2] (seed, step), the call
 * site and the element index (the backward regenerates it; rng_advance moves to a new mask):
 * drop_add_fwd: out (fp32) = drop(a + pos[i % L]) + res  (pos, res fp32, optional) -- patch
 * embeddings + position embeddings (:195-199) and the two residual adds of Block (:215, :219);
 * drop_bwd: da = dout*keep/(1-p);  gelu_drop: out = drop(gelu(x)) (erf GELU, :114, :169-170). */
int dfcsa_drop_add_fwd(int dtype, int64_t n, const void* a, const float* pos, int64_t L, const float* res, float p,
                       const int64_t* rng, int site, float* out, void* stream);
int dfcsa_drop_bwd(int dtype, int64_t n, const float* dout, float p, const int64_t* rng, int site, void* da,
                   void* stream);
int dfcsa_gelu_drop_fwd(int dtype, int64_t n, const void* x, float p, const int64_t* rng, int site, void* out,
                        void* stream);
int dfcsa_gelu_drop_bwd(int dtype, int64_t n, const void* x, const void* dout, float p, const int64_t* rng, int site,
                        void* dx, void* stream);
/* dfcsa_drop_bwd / dfcsa_gelu_drop_bwd over [M][C] (C % 8 == 0) that also write the column sums of
 * their output per 16-row tile: partial [dfcsa_cs_ntiles(M)][C] (capacity partial_floats), reduced by
 * dfcsa_slab_colsum3 -- the Linear bias gradient of the GEMM whose dY the output is, without a
 * dfcsa_colsum_partial pass (round 5).  The outputs equal the flat kernels'. */
int dfcsa_cs_ntiles(int64_t M);   /* ceil(M / 16): partial rows of the *_cs passes */
int dfcsa_drop_bwd_cs(int dtype, int64_t M, int C, const float* dout, float p, const int64_t* rng, int site,
                      void* da, float* partial, int64_t partial_floats, void* stream);
int dfcsa_gelu_drop_bwd_cs(int dtype, int64_t M, int C, const void* x, const void* dout, float p,
                           const int64_t* rng, int site, void* dx, float* partial, int64_t partial_floats,
                           void* stream);
/* out[j] += sum_b x[b*L + j] (position-embedding gradient) */
int dfcsa_batch_sum(int dtype, int B, int64_t L, const void* x, float* out, void* stream);
int dfcsa_rng_advance(int64_t* state, void* stream);
/* Multi-head self-attention core (Attention.forward :137-157): qkv [B*N][ldq] = [q | k | v] of
 * heads*dh columns each; ctx [B*N][heads*dh] = softmax(q k^T * scale) v per head; lse [B][heads][N].
 * bwd: dqkv [B*N][ldq] (q, k, v columns written), dvec [B][heads][N] scratch. dh in {16, 32, 64}. */
/* bf16 relayout between token-major [B*N][nparts*heads*dh] (part p, head h at columns
 * p*heads*dh + h*dh) and head-major [heads*B][N][nparts*dh]; unpack = 0: token -> head-major.
 * Part 0 is multiplied by scale0.  Lets the bf16 MFMA flash-attention kernels (dfcsa_fra_*,
 * gamma = 1, x = 0) run the ViT's multi-head attention with q pre-scaled by 1/sqrt(dh). */
int dfcsa_heads_relayout(int unpack, int B, int N, int heads, int dh, int nparts, float scale0, const void* src,
                         void* dst, void* stream);
/* dfcsa_heads_relayout(unpack = 1) (bf16) that also writes the column sums of the token-major output
 * per 16-row tile: partial [dfcsa_cs_ntiles(B*N)][nparts*heads*dh] for dfcsa_slab_colsum3 (the q / k / v
 * bias gradients; round 5). */
int dfcsa_heads_unpack_cs(int B, int N, int heads, int dh, int nparts, float scale0, const void* src, void* dst,
                          float* partial, int64_t partial_floats, void* stream);
int dfcsa_mha_fwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv, void* ctx,
                  float* lse, void* stream);
int dfcsa_mha_bwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv,
                  const void* ctx, const void* dctx, const float* lse, float* dvec, void* dqkv, void* stream);
/* The same core with attention-probability dropout (attn_dropout, :147-151, attention_dropout_rate
 * = p > 0 in training): ctx = (keep * softmax(q k^T * scale) / (1 - p)) v, keep from the
 * counter-based dropout key (rng, site) of element (bh*N + n)*N + m.  probs [B*heads][N][N] fp32
 * receives the undropped probabilities (the backward's input); dscores [B*heads][N][N] fp32 is
 * backward scratch.  Any dh; N <= 8192 (one workgroup per query / key row, materialised scores). */
int dfcsa_mha_drop_fwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv, float p,
                       const int64_t* rng, int site, float* probs, void* ctx, void* stream);
int dfcsa_mha_drop_bwd(int dtype, int B, int N, int heads, int dh, int ldq, float scale, const void* qkv,
                       const void* dctx, const float* probs, float p, const int64_t* rng, int site, float* dscores,
                       void* dqkv, void* stream);
/* nn.UpsamplingBilinear2d(scale_factor=2) (align_corners=True, :262): [B][Hi][Wi][C] -> [B][2Hi][2Wi][C];
 * bwd is a deterministic gather into dx [B][Hi][Wi][C] */
int dfcsa_upsample2_ac(int dtype, int B, int C, int Hi, int Wi, const void* x, void* out, void* stream);
int dfcsa_upsample2_ac_bwd(int dtype, int B, int C, int Hi, int Wi, const void* dout, void* dx, void* stream);
/* nn.UpsamplingBilinear2d(scale_factor) (align_corners=True) on fp32 NCHW planes [planes][Hi][Wi] ->
 * [planes][Ho][Wo], Ho = floor(Hi * s): SegmentationHead(upsampling > 1) (reference
 * models/transformer_unet.py:272-276) after the head conv.  The backward gathers (deterministic). */
int dfcsa_upsample_ac_f32(int64_t planes, int Hi, int Wi, int Ho, int Wo, const float* x, float* out, void* stream);
int dfcsa_upsample_ac_f32_bwd(int64_t planes, int Hi, int Wi, int Ho, int Wo, const float* dout, float* dx,
                              void* stream);
/* dst[m][j] (+)= src[m][j], j < ncols (row strides ld_src / ld_dst): channel concat / split */
int dfcsa_copy_cols(int dtype, int64_t M, int ncols, const void* src, int ld_src, void* dst, int ld_dst,
                    int accumulate, void* stream);
/* column sums of x [M][C] per 64-row tile: partial [dfcsa_colsum_ntiles(M)][C] (Linear bias gradients,
 * any C % 8 == 0) */
int dfcsa_colsum_ntiles(int64_t M);
int dfcsa_colsum_partial(int dtype, int64_t M, int C, const void* x, float* partial, void* stream);
/* the same sums reduced inside the launch (last workgroup per 2048-column block, row order) and
 * added into d0 [0, n0), d1 [n0, n0 + n1), d2 [n0 + n1, C) -- colsum_partial + slab_colsum3 in one
 * launch; partial: [dfcsa_colsum_ntiles(M)][C] floats of hand-off scratch */
int dfcsa_colsum_fused(int dtype, int64_t M, int C, const void* x, float* partial, int n0, int n1, float* d0,
                       float* d1, float* d2, void* stream);
/* SegmentationHead 3x3 conv + bias (:272-276): logits NCHW fp32 [B][Cout][H][W] from x NHWC
 * [B][H][W][C] (C <= 64, Cout <= 4), w fp32 [Cout][C][3][3]; bwd: dx, partial_w
 * [ntiles][Cout*C*9], partial_b [ntiles][Cout], ntiles = dfcsa_head3_ntiles */
int dfcsa_head3_fwd(int dtype, int B, int H, int W, int C, int Cout, const void* x, const float* w,
                    const float* bias, float* logits, void* stream);
int dfcsa_head3_ntiles(int B, int H, int W);
int dfcsa_head3_bwd(int dtype, int B, int H, int W, int C, int Cout, const void* x, const float* w,
                    const float* dlogits, void* dx, float* partial_w, float* partial_b, void* stream);

/* ------------------------------------------------------------------------------------------
 * Ablation-zoo block outputs (reference unet_dfc_sa_ablation_branches.py:62-70, :93-101,
 * unet_dfc_sa_ablation_fusion.py:35-49, :86-100): out = a (+ b) + res_scale * res; backward:
 * dres = res_scale * dout (dres may be NULL), partial [ntiles][C] of dout * res (ntiles =
 * dfcsa_ew_ntiles(M, C)); dfcsa_sum_into: *out += sum of x[0..n).
 * ---------------------------------------------------------------------------------------- */
int dfcsa_sum_out(int dtype, int M, int C, const void* a, const void* b, const void* res, const float* res_scale,
                  void* out, void* stream);
int dfcsa_bwd_sum_out(int dtype, int M, int C, const void* dout, const void* res, const float* res_scale, void* dres,
                      float* partial, int64_t partial_floats, void* stream);
int dfcsa_sum_into(const float* x, int n, float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Sliding-window inference (reference inference.py:104-153 predict_large_image, :73-91
 * calculate_segmentation_metrics).  Tiles are th x tw; the grid is ys[ny] x xs[nx] with tile
 * t = iy*nx + ix (the reference's y-major loop order).
 * ---------------------------------------------------------------------------------------- */
/* img uint8 [H][W][C] -> out fp32 [T*variants][C][th][tw] for the T tiles with origins
 * (ty[t], tx[t]): (v/255 - mean[c]) / std[c] (mean_std: HOST array of 2*C floats, :116-119).
 * variants 3 appends the h-flipped and the v-flipped tile (TTA, :136-139). */
int dfcsa_tiles_gather(const uint8_t* img, int H, int W, int C, const int* ty, const int* tx, int T, int th, int tw,
                       int variants, const float* mean_std, float* out, void* stream);
/* logits fp32 [ny*nx*variants][th][tw] -> canvas fp32 [H][W]: mean over the covering tiles of
 * sigmoid (variants 3: (p + unflip(p_h) + unflip(p_v)) / 3), sums in tile order (:132-151). */
int dfcsa_tiles_accumulate(const float* logits, const int* ys, int ny, const int* xs, int nx, int th, int tw,
                           int variants, int H, int W, float* canvas, void* stream);
/* counts[0..2] = TP, FP, FN of (prob > thr) against (gray(gt) > gt_thr); gt uint8 [n][gt_channels]
 * (3 channels: OpenCV RGB2GRAY fixed point, :300-305).  counts: device, 4 x uint64, zeroed here. */
int dfcsa_seg_counts(const float* prob, int64_t n, float thr, const uint8_t* gt, int gt_channels, int gt_thr,
                     unsigned long long* counts, void* stream);

/* ------------------------------------------------------------------------------------------
 * Paired image/mask transforms on the GPU (reference utils/data_loader.py:25-73, :119-135:
 * ExtResize, ExtRandomRotation, ExtRandomHorizontalFlip, ExtToTensor, ExtNormalize), bit-exact with
 * the Pillow calls the reference makes.  The random draws stay on the host, in the reference's
 * order; decoding stays on the host.
 * ---------------------------------------------------------------------------------------- */
/* one pass of Image.resize(BILINEAR) for one sample: out[o] = clamp((2^21 + sum_t kk[o][t] *
 * src[bounds[o][0] + t]) >> 22, 0, 255) along `axis` (1: along a row, 0: down a column) */
typedef struct {
  const uint8_t* src;     /* rows of src_pitch bytes; the horizontal pass reads rows row0.. */
  uint8_t* dst;           /* rows of dst_pitch bytes */
  const int* bounds;      /* [n_out][2]: first tap, tap count */
  const int* kk;          /* [n_out][ksize] 22-bit fixed-point coefficients */
  int n_out, n_lines, ksize, axis;
  int src_pitch, dst_pitch, row0, pad;
} dfcsa_resample_desc;
/* descs_dev: n descriptors in device memory; max_work >= n_out * n_lines of every descriptor */
int dfcsa_aug_resample(const dfcsa_resample_desc* descs_dev, int n, int max_work, int C, void* stream);
/* rotation (rotate: 0 none, 1 affine, 2 ROTATE_180, 3 ROTATE_90, 4 ROTATE_270), flip, ToTensor,
 * Normalize of the resized image img [H][W][3]; the mask is sampled from the source mask
 * [.][mask_w] through the resize(NEAREST) tables xtab[W] / ytab[H] (-1: 0). */
typedef struct {
  const uint8_t* img;
  const uint8_t* mask;
  const int* xtab;
  const int* ytab;
  double m[6];            /* Image.rotate's inverse affine matrix (bilinear image sampling) */
  int fix[6];             /* the same matrix in 16.16 fixed point, Geometry.c affine_fixed (mask) */
  int rotate, flip, mask_w, pad;
} dfcsa_aug_desc;
/* images fp32 [n][3][H][W], masks fp32 [n][1][H][W]; mean_std: HOST array of 6 floats */
int dfcsa_aug_finish(const dfcsa_aug_desc* descs_dev, int n, int H, int W, const float* mean_std, int normalize,
                     float* images, float* masks, void* stream);

/* ------------------------------------------------------------------------------------------
 * Profiling hook: when enabled for a kernel class, every launch of that class is bracketed by
 * hipEvents on its own stream; dfcsa_prof_read returns the summed elapsed milliseconds and
 * the launch count since the last reset (synchronises on the recorded events).
 * ---------------------------------------------------------------------------------------- */
#define DFCSA_PROF_CONV_GEMM 1
#define DFCSA_PROF_WGRAD 2
#define DFCSA_PROF_ATTN 3
#define DFCSA_PROF_CONV_STREAM 4   /* 1x1 streaming GEMMs; the "flops" slot carries algorithmic bytes */
int dfcsa_prof_enable(int kernel_class, int enable);
int dfcsa_prof_read(int kernel_class, double* total_ms, int64_t* launches, double* flops);

/* Tuning knobs (benchmarking/autotuning only; 0 = automatic choice).
 * knob 1: conv_gemm tile configuration (see conv_gemm.hip, launch_t).
 * knob 2: target workgroups per weight-gradient launch (split-K count = target / tiles).
 * knob 3: workgroups per CU of the persistent 1x1 streaming GEMM (0 = occupancy limit).
 * knob 4: 1 = print kernel selection decisions to stderr.
 * knob 5: 1 = use the 1x1 streaming GEMM whenever it applies (coverage tests).
 * knob 6: waves per weight-gradient workgroup (4 or 8; 0 = automatic).
 * knob 7: 1 = register-staged bf16 weight gradient instead of the LDS-DMA kernel.
 * knob 8: 0 = allow the 64x256 weight-gradient tile for 64-row problems (default 1: off).
 * knob 9: 1 = generic (non-MFMA) full-resolution attention kernels (coverage tests).
 * knob 19: smallest M routed to the 2-D halo-tile 3x3 conv kernel (0 = never).
 * knob 20: 1 = 3x3 weight gradients on the 2-D halo-tile kernel, 0 = row tiles.
 * knob 21: 1 = divide-per-stage X addressing in the weight-gradient tile kernel.
 * knob 22: halo-tile conv variant (0 = by N, 1 = BN 64 always).
 * knob 23: 1 = element-order weight-gradient split reduction for every split count.
 * knob 24: LDS-DMA ring depth of the 64-row weight-gradient tiles (0 = follow knob 14).
 * knob 25: 0 = never split K in the forward / dgrad implicit GEMM.
 * knob 26: 0 = pointer-DMA weight-gradient kernel instead of the buffer-descriptor one.
 * knob 27: 0 = 4-wave small fp32 GEMM tiles (LightSelfAttention projections).
 * knob 28: 1 = item-owner LightSelfAttention upsample-backward row kernel.
 * knob 30: 0 = no streaming kernel for shifted-segment (3x3, 9 * Cin <= 256) convs.
 * knob 31: 1 = cooperative in-launch split-K weight-gradient reduction.
 * knob 33: smallest M the 1x1 streaming GEMM takes (default 65536).
 * knob 34: 0 = ConvTranspose2d forward GEMMs on the tile kernels instead of the streaming one.
 * knob 35: threads of the LightSelfAttention upsample-backward column kernel at C <= 128.
 * knob 36: 0 = one slot-sized grid per column block in the fused gate dgrad kernels (default 1:
 *          the C / 64 column blocks share the resident slots, grid.x = slots / (C / 64)).
 * knob 37: fewest 64-deep K stages a split-K conv launch may have (default 24).
 * knob 38: workgroups a split-K conv launch aims for (default 600).
 * knob 39: 0 = dfcsa_conv_gemm_bn always launches the separate finalize (no epilogue fold).
 * knob 40: 1 = stream-K decomposition of the 256x256 ping-pong conv tile (default 0: measured slower).
 * knob 42: LDS-DMA ring depth of the buffer-descriptor weight-gradient kernel (2 = default, 3, 4).
 * knob 43: 1 = single-buffer C = 128 forward prologue GEMMs (two workgroups per CU; default 1).
 * knob 44: 1 = single-buffer KP = 256 fused gate dgrad kernels (two workgroups per CU).
 * knob 45: (removed in round 6: several pool windows per workgroup, measured slower).
 * knob 46: 0 = LightSelfAttention pool windows of <= 8 rows split into row slices too (default 1: one slice).
 * knob 47: 0 = large pools (P >= 16) on the sliced pool + pooled launches (default 1: dfcsa_lsa_pool_direct).
 * knob 48: 0 = uncentred dQ in the bf16 pooled-attention backward (default 1: dQ = sum_k dS (K_k - mean key)).
 * knob 49: 0 = the bf16 flash layers' column pass + separate prep (default 1: dfcsa_lsa_flash_bwd_up).
 * knob 50: 0 = one channel chunk in the fused GroupNorm reductions (default 1: 128-channel chunks for C > 128).
 * dfcsa_get_tuning returns a knob's current value (DFCSA_EINVAL for an unknown knob). */
int dfcsa_set_tuning(int knob, int value);
int dfcsa_get_tuning(int knob);

const char* dfcsa_version(void);

#ifdef __cplusplus
}
#endif
#endif /* DFCSA_H_ */
