/*
 * dvie.h — C ABI of the MI355X-native frame-synthesis hot path
 * (deep_video_interpolation_extrapolation, HIP/CDNA4, gfx950).
 *
 * One shared library (libdvie.so) exports these entry points.  Every entry point takes
 * raw device pointers, plain integer shapes/strides and a hipStream_t (passed as void*),
 * launches asynchronously on that stream, never allocates, and returns an int status
 * (DVIE_OK = 0, DVIE_EINVAL = argument validation failure, otherwise a hipError_t).
 *
 * Activations are NHWC ("channels_last"): element (n, y, x, c) of a tensor with pixel
 * stride `ld` (elements) lives at base[((n*H + y)*W + x)*ld + c].  A channel slice of a
 * wider buffer is addressed by offsetting `base` and keeping the wider `ld`.
 *
 * The reference has no native code: every entry point replaces a PyTorch/cuDNN op that
 * the reference calls from Python.  The reference call site each one replaces is cited
 * next to it (paths relative to the reference repository root).
 */
#ifndef DVIE_H
#define DVIE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DVIE_OK 0
#define DVIE_EINVAL 1001

/* element types */
#define DVIE_F32 0
#define DVIE_BF16 1

/* activations (forward) and activation derivatives (backward, computed from the
 * activation's OUTPUT z: lrelu'(z) = z > 0 ? 1 : alpha, elu'(z) = z > 0 ? 1 : z + 1,
 * relu'(z) = z > 0) */
#define DVIE_ACT_NONE 0
#define DVIE_ACT_LRELU 1 /* nn.LeakyReLU(0.2)  nets/HRNet.py:22,59,107 */
#define DVIE_ACT_ELU 2   /* nn.ELU()           nets/HRNet.py:360,362    */
#define DVIE_ACT_RELU 3  /* VGG19 ReLU         nets/vgg.py:11-54         */
#define DVIE_ACT_TANH 4  /* F.tanh RGB head    nets/UNet.py:151, nets/SepUNet.py:65 (tanh'(z) = 1 - z^2) */

/*
 * Implicit-GEMM convolution (forward, and data-gradient as a forward conv over the
 * output gradient with re-packed weights).  Replaces nn.Conv2d forward/backward-data:
 *   3x3 s1 / 3x3 s2 / 1x1 convs of nets/HRNet.py:9-12,52-57,127-129,166-194,367-371,
 *   410-441,444-477; seg encoder nets/HRNet.py:358-364; VGG19 convs nets/vgg.py:11-54.
 *
 * GEMM view: rows = output channels (cout), columns = output pixels of the grid
 * (n, oy, ox) in [0,n)x[0,oh)x[0,ow), reduction over K = taps * c:
 *   acc[co][pix] = sum_{t,ci} w[co][t*c + ci] * x[n][oy*sy + dy(t)][ox*sx + dx(t)][ci]
 * with taps on a th x tw grid, dy(i,j) = dy0 + i*ddy, dx(i,j) = dx0 + j*ddx and
 * t = i*tw + j; out-of-image taps read zero.  w is packed [cout][kpad] (kpad a multiple
 * of 64 elements, zero-filled past taps*c).
 * The result for pixel (n,oy,ox) lands at output position
 *   (n, oy*osy + ory, ox*osx + orx) of a yh x yw image with pixel stride y_ld,
 * which is how the stride-2 data gradient writes its 4 phases.
 * Epilogue, in order: v = acc; v += bias[co]; v += res; v += y_old (beta=1);
 *   v = act(v) (forward activation); v *= act'(z) (dact, derivative from output z);
 *   y = v.
 * Constraints: c % (16/sizeof(elem)) == 0, cout % 4 == 0, every ld % 4 == 0, pointers
 * 16-byte aligned for x/w and 8-byte aligned (bf16) / 16-byte (f32) for y/res/z.
 * Size: one input image and the packed weights must each stay below 4 GiB; a larger
 * batch runs internally as batch chunks whose input span fits (the kernels use 32-bit
 * buffer offsets), so e.g. 448-channel bf16 activations at 1024x2048 work at any n.
 */
typedef struct dvie_conv_desc {
  const void* x;
  const void* w;
  void* y;
  const float* bias; /* [cout] fp32 or NULL */
  const void* res;   /* residual at output placement or NULL (same elem type as y) */
  const void* z;     /* activation output for dact (elem type = dtype) or NULL */
  long long x_ld, y_ld, res_ld, z_ld;
  int n, ih, iw, c;
  int kpad, cout;
  int oh, ow, sy, sx;
  int th, tw, dy0, dx0, ddy, ddx;
  int yh, yw, osy, osx, ory, orx;
  int act, dact, beta, dtype;
  int out_f32; /* 1: y (and res) are fp32, 0: y has elem type dtype */
  float alpha; /* activation slope / parameter */
  int phc;     /* 0, or the stride-2 data gradient of a 3x3 pad-1 conv (nets/HRNet.py:181-194,
                  466-474) in ONE launch: cout = 4*phc output channels are the four output
                  phases, blocks of phc channels in the order (a,b) = (0,0), (1,1), (0,1), (1,0);
                  channel q*phc + ci of grid pixel (oy, ox) lands at channel ci of output pixel
                  (2*oy + a, 2*ox + b) (osy = osx = 2, ory = orx = 0; pixels outside yh x yw are
                  skipped).  Taps 2 x 2 at dy0 = dx0 = 0; tap (i, j) carries weight row
                  kh = a + 1 - 2i, kw = b + 1 - 2j of the forward kernel, so a phase with a = 0
                  (b = 0) has no i = 1 (j = 1) taps: those MFMAs are skipped, not multiplied by
                  zero.  bf16, phc % 32 == 0, no bias / fp32 output. */
  int pad1;
} dvie_conv_desc;

int dvie_conv2d_fwd(const dvie_conv_desc* d, void* stream);

/*
 * Weight gradient of the convolution above (replaces nn.Conv2d backward-weight):
 *   part[s][co][t*c + ci] = sum_{pix in split s} g[pix][co] * x[pix + tap t][ci]
 * g is the pre-activation output gradient on the (n, oh, ow) grid (pixel stride g_ld),
 * x the forward input.  The pixel range is cut into `splits` contiguous chunks; fp32
 * partials go to `ws` ([splits][cout][taps*c]).  dvie_wgrad_reduce then sums them.
 */
typedef struct dvie_wgrad_desc {
  const void* g;
  const void* x;
  float* ws;
  long long g_ld, x_ld;
  int n, oh, ow, cout;
  int ih, iw, c, sy;
  int sx, th, tw, dy0;
  int dx0, ddy, ddx, splits;
  int dtype;
  int tmap;   /* with ws_taps > 0: tap t of this launch's th x tw grid (t = i*tw + j) is column
                 block (tmap >> 4t) & 15 of the slab rows */
  float* bws; /* NULL, or the bias-gradient partials: bws[slab][cout] = column sums of g over
                 the slab's pixels (dvie_wgrad_bias_slabs slabs; reduce them with
                 dvie_wgrad_reduce, ws_k = 1).  The halo weight-gradient kernels sum g while
                 they hold it for the MFMAs (no second pass over g); other launches run a
                 column-sum pass.  Replaces the separate nn.Conv2d bias backward. */
  int ws_taps; /* 0: slab rows hold th*tw*c values, tap t at column t*c.  > 0: rows hold
                  ws_taps*c values and this launch writes only its taps' column blocks (tmap),
                  so several launches fill one slab set: the stride-2 weight gradient
                  (nets/HRNet.py:181-194, 466-474) runs as its four input phases, each a
                  stride-1 weight gradient over a phase view of x (x + (a*W + b)*ld, x_ld =
                  2*ld, ih = H/2, iw = W as the row pitch: the halo kernels, which then read
                  only columns < ow, require ow % 64 == 0), into the 9 tap columns of one
                  [splits][cout][9*c] slab set reduced by one dvie_wgrad_reduce. */
  int pad1;
} dvie_wgrad_desc;

int dvie_conv2d_wgrad(const dvie_wgrad_desc* d, void* stream);

/* Number of bias partial slabs dvie_conv2d_wgrad writes to d->bws. */
int dvie_wgrad_bias_slabs(const dvie_wgrad_desc* d);

/* Split count the library prefers for this weight gradient (0: no preference).  bf16
 * stride-1 1x1/3x3 convs with c and cout multiples of 64 run a halo-tile kernel that
 * assigns contiguous ranges of 64-pixel-wide output tiles to splits. */
int dvie_wgrad_splits_hint(const dvie_wgrad_desc* d);

/* Number of partial slabs ([slabs][cout][taps*c] fp32) dvie_conv2d_wgrad writes for d
 * (d->splits, or 4*d->splits for the halo kernel's 1x1 case); size `ws` and pass this as
 * dvie_wreduce_desc.splits. */
int dvie_wgrad_slabs(const dvie_wgrad_desc* d);

/*
 * dw[co][cmap[j]][kh][kw] (+)= sum_s part[s][co_off + co][t*c + j]  for every packed
 * position j in [0, c) whose source channel cmap[j] >= 0 (identity when cmap is NULL),
 * t = kh*kw_n + kw, writing an OIHW fp32 parameter gradient of cout_p x cin_p x kh_n x kw_n.
 * Rows co_off .. ws_rows-1 of the slabs are scanned (ws_rows*ws_k and co_off*ws_k multiples
 * of 4), rows co < cout_p written.  Threads walk the partial slabs in memory order
 * (16-byte coalesced), 8 split-lanes per column.  Also used for bias gradients
 * (kh_n = kw_n = 1, cin_p = 1, c = 1, ws_k = 1).
 */
typedef struct dvie_wreduce_desc {
  const float* ws;
  float* dw;
  const int* cmap;
  int splits, ws_rows, ws_k, co_off;
  int cout_p, cin_p, kh_n, kw_n;
  int c, beta;
} dvie_wreduce_desc;

int dvie_wgrad_reduce(const dvie_wreduce_desc* d, void* stream);

/*
 * Several slab reductions in ONE launch (replaces as many dvie_wgrad_reduce launches; the
 * engine batches the weight lane's reductions, each weight gradient of a batch writing its
 * own slab region).  descs: a HOST array of n descriptors, read at launch time, so the caller
 * may re-point their dw / beta between launches.  A flat grid: each descriptor owns a
 * contiguous block range.  Same results as n dvie_wgrad_reduce calls.
 */
int dvie_wgrad_reduce_multi(const dvie_wreduce_desc* descs, int n, void* stream);
typedef struct dvie_wreduce_multi_desc {
  const dvie_wreduce_desc* descs; /* host array */
  int n, pad;
} dvie_wreduce_multi_desc;

/* Bias gradient partials: part[s][co] = sum_{pix in split s} g[pix][co]. */
typedef struct dvie_colsum_desc {
  const void* g;
  float* ws;
  long long g_ld;
  long long rows;
  int c, splits, dtype, pad0;
} dvie_colsum_desc;

int dvie_colsum(const dvie_colsum_desc* d, void* stream);

/*
 * Weight packing: fp32 OIHW parameter -> packed GEMM operand rows (elem type dtype).
 * mode 0 (forward):   dst[r][t*c + j] = src[r][cmap[j]][kh(t)][kw(t)], r < cout_s
 * mode 1 (transpose): dst[r][t*c + j] = src[j][cmap[r]][kh(t)][kw(t)], j < cout_s
 * with kh(t) = kh0 + (t / tw)*dkh, kw(t) = kw0 + (t % tw)*dkw; entries whose source is
 * out of range (cmap < 0, r/j past the source extent, k >= taps*c) are zero.
 * `n` descriptors are processed by one launch (descs points to DEVICE memory) over a flat
 * grid of `blocks` workgroups: descriptor i owns blocks [blk0_i, blk0_i + nb_i), the blk0
 * increasing with i (the caller fills them; `blocks` is the sum), with nb = rows (mode 0,
 * kpad >= 64 and kpad % 4 == 0, cin_s*kh_s*kw_s <= 8192: one packed row per block),
 * ceil(rows / 8) * ceil(c / 64) (mode 1, the same kpad, kh_s*kw_s <= 16, c % 4 == 0: 8 rows x
 * 64 columns per block), else ceil(rows * kpad / 1024) (1024 elements per block).
 */
typedef struct dvie_pack_desc {
  const float* src;
  void* dst;
  const int* cmap; /* device int array or NULL (identity) */
  int rows, kpad, c, mode;
  int th, tw, kh0, kw0;
  int dkh, dkw, cout_s, cin_s;
  int kh_s, kw_s, dtype, blk0; /* blk0: first flat-grid block of this descriptor */
} dvie_pack_desc;

int dvie_pack_weights(const dvie_pack_desc* descs_dev, int n, int blocks, void* stream);

/* Number of flat-grid blocks dvie_pack_weights gives descriptor d (host memory): the blk0 of
 * the next descriptor is d->blk0 plus this, and `blocks` is the sum over all descriptors. */
int dvie_pack_blocks(const dvie_pack_desc* d);

/*
 * Pointwise NHWC family (4 channels per thread).  op selects:
 *  DVIE_EW_FUSE   y = act( sum_i up_i(src_i) ) — HighResolutionModule fuse sum
 *                 (nets/HRNet.py:212-225) and the final bilinear upsample into the
 *                 448-channel concat (nets/HRNet.py:576-582).  up_i is bilinear from
 *                 (src_h, src_w) to (h, w), identity when equal; align_corners=False, or
 *                 True when `align` is set (nn.Upsample of nets/UNet.py:70).
 *  DVIE_EW_UPT    y = up^T(src_0) — adjoint of the bilinear upsample (gather form,
 *                 deterministic, no atomics); src_0 is the fine grid (src_h x src_w);
 *                 `align` as for FUSE.
 *  DVIE_EW_POOL   y = avgpool2x2(src_0) (nets/vgg.py:9 AvgPool2d(2,2)).
 *  DVIE_EW_POOLT  y = adjoint of avgpool2x2 applied to src_0 (coarse grid).
 *  DVIE_EW_COPY   y = src_0 (same grid).
 *  DVIE_EW_L1SIGN y = scale * sign(src_0 - src_1) (VGG feature-L1 gradient, losses.py:178-179)
 *  DVIE_EW_NCHW   y = ext (fp32, arbitrary NCHW strides sn,sc,sh,sw; channels >= ext_c
 *                 read as zero), optionally (ext - mean[c]) / std[c]
 *                 (preprocess_norm, utils/net_utils.py:11-23).  With src1 set, channels
 *                 [sh1, ext_c) come from the fp32 tensor src1 (channel c - sh1, same
 *                 strides): two frames read in place instead of torch.cat
 *                 (runners/InterTrainer.py:373-374 of the reference).
 *  DVIE_EW_TONCHW ext (+)= channels [0, ext_c) of src_0 as fp32 with NCHW strides,
 *                 divided by std[c] when std is set (adjoint of the normalisation);
 *                 beta selects accumulate; the NHWC epilogue is not applied.
 *  DVIE_EW_MASK   y = src_0 * m or src_0 * (1 - m) (ext_c = 0 / 1), m = ext[n, 0, y, x]
 *                 (fp32, NCHW strides): the fg/bg split of nets/SepUNet.py:45-46 (its own
 *                 adjoint with respect to src_0).
 *  DVIE_EW_IM2COL y[n,y,x][t*ext_c + ch] = src_0[n, y + sh1 + ty*sh2, x + sw1 + tx*sw2][ch]
 *                 for tap t = ty*sw0 + tx of an sh0 x sw0 tap grid; zero outside the (h, w)
 *                 image and for t >= sh0*sw0 (ext_c % 8 == 0).  Lowers a stride-1 conv whose
 *                 input has few channels (the data gradient of HRNet's 3x3 448->3 / 448->20
 *                 heads) to a 1x1 GEMM over K = taps*ext_c instead of taps*64.
 * then the shared epilogue: v += res; v += y_old (beta); v = act(v); v *= act'(z); y = v.
 * Channels c % 4 == 0; all lds % 4 == 0.
 */
#define DVIE_EW_FUSE 0
#define DVIE_EW_UPT 1
#define DVIE_EW_POOL 2
#define DVIE_EW_POOLT 3
#define DVIE_EW_COPY 4
#define DVIE_EW_L1SIGN 5
#define DVIE_EW_NCHW 6
#define DVIE_EW_TONCHW 7
#define DVIE_EW_MASK 8
#define DVIE_EW_IM2COL 9

typedef struct dvie_ew_desc {
  void* y;
  const void* src0;
  const void* src1;
  const void* src2;
  const void* res;
  const void* z;
  float* ext;
  const float* mean;
  const float* std;
  long long y_ld, src_ld0, src_ld1, src_ld2, res_ld, z_ld;
  long long sn, sc, sh, sw;
  int op, n, h, w;
  int c, nsrc, sh0, sw0;
  int sh1, sw1, sh2, sw2;
  int act, dact, beta, dtype;
  int ext_c, align;
  float alpha, scale;
} dvie_ew_desc;

int dvie_ew(const dvie_ew_desc* d, void* stream);

/*
 * Loss reductions on fp32 NCHW-strided (B, C, H, W) images (pred a, target b).
 * Every loss writes its partial sums to `partial` (double[nblocks]) and the final
 * scalar (fp32) to `out`, and — when `grad` is non-NULL — the gradient of `weight *
 * loss` with respect to a in NCHW-contiguous fp32 layout ([B][C][H][W]), overwritten
 * (beta=0) or accumulated (beta=1).
 *  L1   : mean|a-b|                                   nn.L1Loss (losses.py:224)
 *  GDL  : (mean|dx a - dx b| + mean|dy a - dy b|)/2   GDLLoss (losses.py:137-151)
 *  SSIM : 1 - mean ssim_map (11x11 gaussian, sigma 1.5, zero pad 5, C1=1e-4, C2=9e-4)
 *                                                      SSIM/_ssim (losses.py:18-48,63-87)
 *  MSE  : per-sample mean((a-b)^2) -> out[b] (PSNR, losses.py:103-116)
 *  CE   : mean_pix( logsumexp(a[:,.]) - a[label] ), label = argmax_c b[:, c]
 *         (nn.CrossEntropyLoss(a, argmax(b,1)), runners/InterTrainer.py:75,414)
 */
#define DVIE_LOSS_L1 0
#define DVIE_LOSS_GDL 1
#define DVIE_LOSS_SSIM 2
#define DVIE_LOSS_MSE 3
#define DVIE_LOSS_CE 4
#define DVIE_LOSS_L1NHWC 5 /* mean|a-b| over NHWC tensors of elem type dtype (VGG features) */
/* validation metrics (no gradient; `grad` must be NULL):
 *  COSNHWC    : weight * mean_pix( sum_c a.b / (|a| |b|) ) over (B, C=ch, H, W) tensors of
 *               elem type dtype, channel stride a_sc/b_sc (VGGCosineLoss, losses.py:182-207;
 *               NaN for an all-zero feature vector, as the reference's 0/0)
 *  IOU        : mean_pix( a == b ) of int64 label maps (B, H, W), strides a_sn/a_sh/a_sw
 *               (IoU, losses.py:122-131)
 *  ARGMAX_IOU : IOU of argmax_c a and argmax_c b, fp32 (B, C, H, W) scores (first maximum,
 *               as torch.argmax; InterTrainer.validate, runners/InterTrainer.py:615-624) */
#define DVIE_LOSS_COSNHWC 6
#define DVIE_LOSS_IOU 7
#define DVIE_LOSS_ARGMAX_IOU 8

/*
 * grad (L1, GDL, SSIM, CE): d(weight * loss)/d(a), NCHW-contiguous fp32; beta = 1 adds it
 * to what grad holds (several losses of one prediction write one gradient buffer).
 * out: the loss value times out_scale, taken as given (a weight-0 term reports 0; builders
 * set 1.0 for the plain value); out_acc = 1 adds it to *out instead of storing it (the five
 * VGG feature levels into one scalar).  weight scales the gradient only (COSNHWC: the value).
 */
typedef struct dvie_loss_desc {
  const void* a;
  const void* b;
  float* grad;
  float* out;
  double* partial;
  float* ws; /* SSIM gradient scratch: 3*B*C*H*W floats (dvie_loss_ws_floats) */
  long long a_sn, a_sc, a_sh, a_sw;
  long long b_sn, b_sc, b_sh, b_sw;
  int kind, bsz, ch, h;
  int w, beta, dtype, out_acc;
  float weight, out_scale;
} dvie_loss_desc;

int dvie_loss(const dvie_loss_desc* d, void* stream);

/* out[0] = sum of x[0 .. n-1] in index order, one workgroup (the training step's loss_all
 * from its weighted terms; replaces the Python sum at runners/InterTrainer.py:426-430 of
 * the reference) */
int dvie_sum_f32(const float* x, int n, float* out, void* stream);
size_t dvie_loss_partial_count(const dvie_loss_desc* d);
size_t dvie_loss_ws_floats(const dvie_loss_desc* d);

/*
 * Bilinear flow warp (FlowWrapper, utils/net_utils.py:89-114; F.grid_sample bilinear,
 * zeros padding, align_corners=True as in the pinned torch 1.0.1):
 *   gx = linspace(-1,1,W)[x] - flow[n,0,y,x],  gy = linspace(-1,1,H)[y] - flow[n,1,y,x]
 *   out[n,c,y,x] = bilinear(img[n,c], (gx+1)/2*(W-1), (gy+1)/2*(H-1))
 * fp32, NCHW contiguous.  Backward: dimg and dflow (both overwritten), given dout.  Three
 * launches: per sample its source position (ix, iy) into `ws` and dflow; per dimg pixel the
 * samples of a 3x3 window around c minus its displacement (the side chosen by the fractional
 * part) gathered as a plain store, plus the per-sample check that appends samples a corner's
 * window misses to a far list in `ws`; global atomics for the listed samples.  dimg = NULL
 * computes dflow only (ws may be NULL).  `ws` holds dvie_warp_ws_floats(d) floats.
 */
typedef struct dvie_warp_desc {
  const float* img;
  const float* flow;
  float* out;
  const float* dout;
  float* dimg;
  float* dflow;
  float* ws;
  int n, c, h, w;
  int align_corners, pad0;
} dvie_warp_desc;

int dvie_warp_fwd(const dvie_warp_desc* d, void* stream);
int dvie_warp_bwd(const dvie_warp_desc* d, void* stream);
size_t dvie_warp_ws_floats(const dvie_warp_desc* d);

/*
 * Fused Adamax step over a flat fp32 buffer (torch.optim.Adamax semantics,
 * runners/InterTrainer.py:79): m = lerp(m, g, 1-b1); u = max(u*b2, |g|+eps);
 * p -= clr * m / u with clr = lr / (1 - b1^step) (computed by the caller);
 * weight decay applied as g += wd*p first.
 */
int dvie_adamax(float* p, const float* g, float* m, float* u, long long n, float clr,
                float b1, float b2, float eps, float wd, void* stream);

/*
 * Graph-capturable variants (the step count lives on the device, so a captured step
 * replays with the right bias correction): dvie_step_inc adds 1 to *step; dvie_adamax_dev
 * computes clr = lr / (1 - b1^(*step)) on the device in double from the double lr / b1 a
 * host would use, then updates as dvie_adamax (elementwise math in float, as there).
 */
int dvie_step_inc(float* step, void* stream);
int dvie_adamax_dev(float* p, const float* g, float* m, float* u, long long n, double lr, double b1, double b2,
                    double eps, double wd, const float* step, void* stream);

/* scale a flat fp32 buffer in place (used for the 1/W gradient factor) */
int dvie_scale(float* p, long long n, float s, void* stream);

/*
 * Measurement only (bench.py): `blocks` workgroups of 4 waves, each wave issuing
 * 8 * iters back-to-back v_mfma_f32_32x32x16_bf16 on pseudo-random operands in registers
 * (32768 FLOP each); out[blocks * 256] receives per-lane sums.  Its rate is the dense bf16
 * MFMA ceiling at the clock the chip holds under that load on this box.
 */
int dvie_mfma_probe(float* out, int blocks, int iters, void* stream);

/*
 * Measurement only (bench.py): `blocks` workgroups of `threads` threads of an empty kernel --
 * the dispatch / ramp / drain floor of a launch of that shape (the warp forward's grid at
 * 256x512 is a ~7 us launch, where this floor is a large part).
 */
int dvie_launch_probe(int blocks, int threads, void* stream);

/*
 * BatchNorm2d over NHWC rows (rows = N*H*W pixels, c channels), fused with the following
 * activation (nets/FrameDisc.py:45-46, nets/VidDisc.py:45-50, nets/HRNet.py:726-789).
 * training = 1: batch statistics (biased variance for the normalisation; running_mean /
 * running_var, if non-NULL, updated with `momentum` and the unbiased variance, as
 * nn.BatchNorm2d.train()); training = 0: running statistics.
 *   forward : y = act(gamma * (x - mean) * invstd + beta)
 *   backward: g = dL/d(pre-activation output) (the engine applies act' upstream);
 *             dgamma (+)= sum g*xhat, dbeta (+)= sum g (accumulate selects +=);
 *             dx (+)= gamma*invstd*(g - mean(g) - xhat*mean(g*xhat)) (beta_dx selects +=).
 * partial: double [splits][2][c] workspace (splits = dvie_bn_partial_splits); stats: fp32
 * [8][c] per-call state written by the forward and read by the backward.
 * Constraints: c % 4 == 0, c <= 1024, lds % 4 == 0.
 */
typedef struct dvie_bn_desc {
  const void* x;
  void* y;
  const void* g;
  void* dx;
  const float* gamma;
  const float* beta;
  float* dgamma;
  float* dbeta;
  float* running_mean;
  float* running_var;
  double* partial;
  float* stats;
  long long x_ld, y_ld, g_ld, dx_ld;
  long long rows;
  int c, splits, act, training;
  int dtype, accumulate, beta_dx, x_f32; /* x_f32: x is fp32 (y, g, dx have elem type dtype) */
  float alpha, eps, momentum, pad1;
} dvie_bn_desc;

int dvie_bn_fwd(const dvie_bn_desc* d, void* stream);
int dvie_bn_bwd(const dvie_bn_desc* d, void* stream);
int dvie_bn_partial_splits(const dvie_bn_desc* d);

/*
 * Discriminator head: AvgPool2d(pool) of an NHWC (n, h, w, c) map, then
 * view(-1, c).mean(1) over the NCHW-flat pooled tensor (nets/FrameDisc.py:66,74;
 * nets/VidDisc.py:77,83): out[r] = mean(pooled_nchw[r*c : (r+1)*c]), r < n*(h/pool)*(w/pool).
 * pooled: fp32 workspace of n*c*(h/pool)*(w/pool).  Backward: gx (+)= the adjoint applied
 * to gout (pixels past the floor(h/pool)*pool crop get 0).
 */
typedef struct dvie_head_desc {
  const void* x;
  void* gx;
  const float* gout;
  float* out;
  float* pooled;
  long long x_ld, gx_ld;
  int n, h, w, c;
  int pool, dtype, beta, pad0;
} dvie_head_desc;

int dvie_head_fwd(const dvie_head_desc* d, void* stream);
int dvie_head_bwd(const dvie_head_desc* d, void* stream);

/*
 * Channel softmax (F.softmax(seg, dim=1), nets/InterGANNet.py:40), fp32: x with NCHW
 * strides (sn, sc, sh, sw) in elements, y contiguous NCHW.  Backward (gy, y contiguous):
 * gx (+)= y * (gy - sum_c gy*y).
 */
typedef struct dvie_softmax_desc {
  const float* x;
  float* y;
  const float* gy;
  float* gx;
  long long sn, sc, sh, sw;
  int n, c, h, w;
  int beta, pad0;
} dvie_softmax_desc;

int dvie_softmax_fwd(const dvie_softmax_desc* d, void* stream);
int dvie_softmax_bwd(const dvie_softmax_desc* d, void* stream);

/*
 * Fused Adam over a flat fp32 buffer, torch 1.0.1 update form (the discriminator
 * optimizers, runners/InterGANTrainer.py:110-112): m = b1*m + (1-b1)*g;
 * v = b2*v + (1-b2)*g^2; p -= step_size * m / (sqrt(v) + eps) with
 * step_size = lr*sqrt(1-b2^t)/(1-b1^t) computed by the caller; weight decay g += wd*p first.
 */
int dvie_adam(float* p, const float* g, float* m, float* v, long long n, float step_size, float b1, float b2,
              float eps, float wd, void* stream);
/* the same with step_size computed on the device from lr and *step (graph-captured steps) */
int dvie_adam_dev(float* p, const float* g, float* m, float* v, long long n, double lr, double b1, double b2,
                  double eps, double wd, const float* step, void* stream);

/*
 * SpectralNorm (reference nets/SpectralNorm.py:10-68), fp32, one workgroup per layer.
 * W_bar is the (h, width) row-major view of the OIHW weight (width = cin*kh*kw).
 * Forward (SpectralNorm._update_u_v, l.23-35), `power_iterations` times:
 *   v = l2normalize(W_bar^T u); u = l2normalize(W_bar v)      (l2normalize: x / (|x| + 1e-12))
 * then sigma = u . (W_bar v) and w_eff = W_bar / sigma.  u and v are updated in place; the
 * values used ([sigma, u(h), v(width)]) are saved at state + state_off for the backward.
 * Backward (autograd of `w / sigma` with sigma = u.dot(W_bar.mv(v))),
 * g_sigma = -sum(g_eff * W_bar) / sigma^2:
 *   g_bar (+)= g_eff / sigma + g_sigma * u v^T
 *   g_u   (+)= g_sigma * (W_bar v),  g_v (+)= g_sigma * (W_bar^T u)   (only if non-null: u and v
 *   become trainable in the reference once set_net_grad(True) ran, nets/InterGANNet.py:81)
 * beta = 1 accumulates into g_bar / g_u / g_v.  u, v here are the values the forward saved.
 * Replaces: SpectralNorm.forward's _update_u_v (l.66-68) and its autograd backward.
 * `n` layers (host array, any count), one workgroup each.
 */
typedef struct dvie_sn_layer {
  const float* w_bar;
  float* u;
  float* v;
  float* w_eff;
  const float* g_eff;
  float* g_bar;
  float* g_u;
  float* g_v;
  long long state_off;
  int h, width, power_iterations, beta;
} dvie_sn_layer;

int dvie_sn_fwd(const dvie_sn_layer* layers, int n, float* state, void* stream);
int dvie_sn_bwd(const dvie_sn_layer* layers, int n, const float* state, void* stream);

/*
 * VAEHRNet reparameterisation (reference nets/HRNet.py:960-966), fp32, n elements:
 *   forward  z = eps * exp(0.5 * logvar) + mu
 *   backward gmu (+)= gz; glogvar (+)= gz * eps * 0.5 * exp(0.5 * logvar)   (beta: accumulate)
 * eps is the caller's standard-normal draw (std.new(std.size()).normal_()).
 */
int dvie_reparam_fwd(const float* mu, const float* logvar, const float* eps, float* z, long long n, void* stream);
int dvie_reparam_bwd(const float* logvar, const float* eps, const float* gz, float* gmu, float* glogvar, long long n,
                     int beta, void* stream);

/*
 * Local-window attention ops of the second-stage refinement nets (MSResAttnRefine,
 * nets/refine_nets.py:138-399; corrmap l.253-287, weight_neighbors_by_probmap l.313-323,
 * weight_neighbors_by_low_probmap l.289-311).  NHWC tensors of elem type dtype on an
 * (n, h, w) grid; window entry k of a (wh x ww) window (both odd) is the neighbour at
 * offset (k / ww - wh/2, k % ww - ww/2); the window weights of map m occupy channels
 * [m*K, (m+1)*K), K = wh*ww; out-of-image neighbours read zero.
 *   L2NORM      y[p, :c] = a[p, :c] / |a[p, :c]|                          (x / x.norm(dim=1))
 *   L2NORM_BWD  y = (a - b0 <b0, a>) / |b1|      a = dL/dxn, b0 = xn, b1 = x
 *   CORR        y[p, m*K + k] = <a[p, :c], b_m[p + o_k, :c]>, m < nhalf    (b_0 = b0, b_1 = b1;
 *               a NULL map's entries are written as 0)
 *   GATHER      y[p, :c] = sum_m sum_k a[p, (half0+m)*K + k] * b_m[p + o_k, :c]   (m < 1 + !!b1)
 *   GATHER_T    y[q, :c] = sum_k a[q - o_k, half0*K + k] * b0[q - o_k, :c]  (adjoint in b)
 *   SOFTMAX     y[p, :J] = softmax(a[p, :J]), J = nhalf*K
 *   SOFTMAX_BWD y = b0 * (a - <b0, a>)           a = dL/dprob, b0 = prob
 *   WNORM       per map: y = a / sum_k a
 *   WNORM_BWD   per map: y = (a - <a, b0>) / sum_k b1     a = dL/dWn, b0 = Wn, b1 = W
 *   POOL        y[p, :c] = mean of a over the in-image part of the centred (wh x ww) window
 *               (F.avg_pool2d(k=(wh,ww), stride 1, pad (wh/2, ww/2), count_include_pad=False))
 *   POOL_T      adjoint of POOL
 * Then the common epilogue: v += res; v += y_old (beta); v = act(v); v *= act'(z) (dact).
 * Vector ops (GATHER*, POOL*) need c, every ld % 4 == 0.
 */
#define DVIE_ATTN_L2NORM 0
#define DVIE_ATTN_L2NORM_BWD 1
#define DVIE_ATTN_CORR 2
#define DVIE_ATTN_GATHER 3
#define DVIE_ATTN_GATHER_T 4
#define DVIE_ATTN_SOFTMAX 5
#define DVIE_ATTN_SOFTMAX_BWD 6
#define DVIE_ATTN_WNORM 7
#define DVIE_ATTN_WNORM_BWD 8
#define DVIE_ATTN_POOL 9
#define DVIE_ATTN_POOL_T 10

typedef struct dvie_attn_desc {
  const void* a;
  const void* b0;
  const void* b1;
  void* y;
  const void* res;
  const void* z;
  long long a_ld, b_ld, y_ld, res_ld, z_ld;
  int op, n, h, w;
  int c, wh, ww, nhalf;
  int half0, act, dact, beta;
  int dtype, pad0;
  float alpha, pad1;
} dvie_attn_desc;

int dvie_attn(const dvie_attn_desc* d, void* stream);

/*
 * Fused backward of a narrow-output 3x3 stride-1 conv over a LeakyReLU-activated map: the
 * HRNet output heads rgb_layer[2] / seg_layer[2] (448 -> 3 / 448 -> 20, reference
 * nets/HRNet.py:410-442, 584-588), whose backward is nn.Conv2d backward-data + the preceding
 * LeakyReLU's derivative + nn.Conv2d backward-weight.  One pass over the hidden map h:
 *   dh[p][ci]  = act'(h[p][ci]) * sum_{t, o} wd[ci][t * cout + o] * g[p + (dy0 + i_t, dx0 + j_t)][o]
 *   ws[s][o][(8 - t) * c + ci] = sum_{p in split s} g[p + (dy0 + i_t, dx0 + j_t)][o] * h[p][ci]
 * (t = 3 i_t + j_t the data-gradient tap; 8 - t the forward tap of the same weight), so
 * h is read once and the dh map written once; the weight-gradient partial slabs have the
 * dvie_conv2d_wgrad layout (reduce them with dvie_wgrad_reduce, ws_k = 9 * c).
 * g: (n, h, w, cout) bf16 NHWC output gradient (cout 8 or 24, padded channels zero);
 * h: the conv input (bf16 NHWC, c channels, a multiple of 64); wd: the packed data-gradient
 * weights [c][kpad] (dvie_pack_weights mode 1: wd[ci][t * cout + o] = w[o][ci][2 - i_t][2 - j_t]);
 * dh: bf16 NHWC, written (not accumulated); dact: DVIE_ACT_LRELU (alpha) or DVIE_ACT_NONE.
 * splits: weight-gradient slabs (grid = (c / 64) * splits workgroups); bf16 only.
 */
typedef struct dvie_head3_bwd_desc {
  const void* g;
  const void* h;
  const void* wd;
  void* dh;
  float* ws;
  long long g_ld, h_ld, dh_ld;
  int n, hgt, wid, c;
  int cout, kpad, dy0, dx0;
  int splits, dact;
  float alpha, pad0;
} dvie_head3_bwd_desc;

int dvie_head3_bwd(const dvie_head3_bwd_desc* d, void* stream);

/*
 * Fused forward of HRNet's segmentation encoder (reference nets/HRNet.py:358-364, applied at
 * l.533-537): e1 = ELU(conv3x3(in) + b0) (24 -> 32 channels; the 20 classes padded to 24),
 * e2 = ELU(conv3x3(e1) + b2) (32 -> 32), out = conv3x3(e2) + b4 (32 -> 8: the 4 encoder
 * channels + 4 zero-weight pads), stride 1, zero padding, bf16 NHWC.  e1 and e2 are written
 * (the backward reads them); out may be a channel slice of a wider buffer (out_ld).  w0 / w2 /
 * w4: the forward-packed weights [cout][kpad] (dvie_pack_weights mode 0: w[co][t * cin + ci]),
 * b0 / b2 / b4: fp32 biases (32, 32, 8).
 */
typedef struct dvie_segenc_desc {
  const void* in;
  void* e1;
  void* e2;
  void* out;
  const void* w0;
  const void* w2;
  const void* w4;
  const float* b0;
  const float* b2;
  const float* b4;
  long long in_ld, e1_ld, e2_ld, out_ld;
  int n, h, w, kpad0;
  int kpad2, kpad4;
} dvie_segenc_desc;

int dvie_segenc_fwd(const dvie_segenc_desc* d, void* stream);

/*
 * Fused backward of the same encoder (the encoder input needs no gradient): from dout (the
 * gradient of the 8-channel output, bf16 NHWC, e.g. a slice of the stem buffer's gradient)
 * and the forward's e2 / e1 / in, the weight- and bias-gradient partial slabs of the three
 * convs; d_e2 = ELU'(e2) conv4^T(dout) and d_e1 = ELU'(e1) conv2^T(d_e2) stay on chip.
 * w4d / w2d: the packed data-gradient weights of conv4 [32][kpad4 >= 80] and conv2
 * [32][kpad2 >= 288] (dvie_pack_weights mode 1).  Slabs (one per workgroup, `slabs` of them):
 * dw4 [slabs][8][288], dw2 [slabs][32][288], dw0 [slabs][32][216] (dvie_conv2d_wgrad layout,
 * reduce with dvie_wgrad_reduce), db4 [slabs][8], db2 / db0 [slabs][32].
 */
typedef struct dvie_segenc_bwd_desc {
  const void* dout;
  const void* e2;
  const void* e1;
  const void* in;
  const void* w4d;
  const void* w2d;
  float* dw4;
  float* dw2;
  float* dw0;
  float* db4;
  float* db2;
  float* db0;
  long long dout_ld, e2_ld, e1_ld, in_ld;
  int n, h, w, kpad4;
  int kpad2, slabs;
} dvie_segenc_bwd_desc;

int dvie_segenc_bwd(const dvie_segenc_bwd_desc* d, void* stream);

/*
 * Op-list executor: runs n descriptors in order with a single host call (the per-step
 * forward and backward plans of the HRNet / VGG executors).  dvie_op.lane picks the stream:
 *   0     the caller's stream;
 *   1     the weight lane (a library side stream of the current device and host thread):
 *         work off the critical path (weight gradients and their reductions).  A run of
 *         lane-1 ops first waits for everything issued so far on the caller's stream (the
 *         lane-0 ops that produced its inputs), so lane-1 ops read only finished data.
 * The call ends with the caller's stream waiting for the side stream if it was used, so the
 * call as a whole is ordered on the caller's stream and capturable (the wait is a graph
 * edge).  DVIE_OP_LANES=0 runs every op on the caller's stream.
 */
#define DVIE_OP_CONV 1
#define DVIE_OP_WGRAD 2
#define DVIE_OP_WREDUCE 3
#define DVIE_OP_COLSUM 4
#define DVIE_OP_EW 5
#define DVIE_OP_LOSS 6
#define DVIE_OP_PACK 7
#define DVIE_OP_BN_FWD 8
#define DVIE_OP_BN_BWD 9
#define DVIE_OP_HEAD_FWD 10
#define DVIE_OP_HEAD_BWD 11
#define DVIE_OP_ATTN 12
#define DVIE_OP_HEAD3_BWD 13
#define DVIE_OP_SEGENC_FWD 14
#define DVIE_OP_SEGENC_BWD 15
#define DVIE_OP_WREDUCE_MULTI 16

typedef struct dvie_pack_list {
  const dvie_pack_desc* descs_dev;
  int n, blocks; /* dvie_pack_weights arguments */
} dvie_pack_list;

typedef struct dvie_op {
  int kind;
  int lane; /* 0: caller's stream, 1: weight lane (see above) */
  union {
    dvie_conv_desc conv;
    dvie_wgrad_desc wgrad;
    dvie_wreduce_desc wreduce;
    dvie_colsum_desc colsum;
    dvie_ew_desc ew;
    dvie_loss_desc loss;
    dvie_pack_list pack;
    dvie_bn_desc bn;
    dvie_head_desc head;
    dvie_attn_desc attn;
    dvie_head3_bwd_desc head3;
    dvie_segenc_desc segenc;
    dvie_segenc_bwd_desc segenc_bwd;
    dvie_wreduce_multi_desc wreduce_multi;
  } u;
} dvie_op;

/*
 * Cityscapes clip preparation on the device (reference folder.py:225-247 train branch and
 * l.248-261 val branch; crop parameters folder.py:125-149, flip l.211).  Replaces the
 * DataLoader worker's PIL flip / crop, to_tensor, normalize((.5,.5,.5),(.5,.5,.5)) and
 * np.eye(20)[seg] one-hot.  For clip b (dataset clip idx[b]) and frame t with
 * params[(b*T+t)*3 + {0,1,2}] = {flip, h1, w1}:
 *   src_x = flip ? W0-1-(w1+x) : w1+x,  src_y = h1+y      (flip the full frame, then crop)
 *   frames[t][b][c][y][x] = (img[idx[b]][t][src_y][src_x][c] / 255 - 0.5) / 0.5   (fp32)
 *   segs[t][b][k][y][x]   = (seg[idx[b]][t][src_y][src_x] == k)                      (fp32)
 * img: uint8 (N, T, H0, W0, 3) RGB as decoded, seg: uint8 (N, T, H0, W0) class ids (NULL:
 * no segs), both HBM-resident.  A label >= n_classes (np.eye raises IndexError there)
 * gives an all-zero one-hot and is counted into *bad (optional, accumulated).  idx = NULL
 * means clip b = b.  Every read must stay inside the frame: h1 + hc <= h0, w1 + wc <= w0
 * (the caller's crop generator guarantees it; not re-checked per pixel).
 */
typedef struct dvie_clip_desc {
  const uint8_t* img;
  const uint8_t* seg;
  const int* idx;
  const int* params;
  float* frames;
  float* segs;
  int* bad;
  int b, t, h0, w0, hc, wc, n_classes, pad0;
} dvie_clip_desc;

int dvie_clip_prep(const dvie_clip_desc* d, void* stream);

int dvie_run_ops(const dvie_op* ops, int n, void* stream);

/* ABI self-check: sizeof of each descriptor, indexed by DVIE_OP_* (0 = dvie_op). */
size_t dvie_abi_sizeof(int which);
/* library version string */
const char* dvie_version(void);
/* last error text of the calling thread (argument validation) */
const char* dvie_last_error(void);

/* Diagnostics (tests, profiling): launch trace of the calling thread.  dvie_trace_kernels(1)
 * starts recording the kernels every entry point of this thread launches (0 stops; both clear
 * the record; returns the previous state).  dvie_traced_kernels() returns the demangled names
 * of the kernels launched since the last call, ';'-separated in launch order, and clears the
 * record (the text stays valid until the thread's next call). */
int dvie_trace_kernels(int on);
const char* dvie_traced_kernels(void);

#ifdef __cplusplus
}
#endif

#endif /* DVIE_H */
