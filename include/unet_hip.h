/*
 * unet_hip.h — C-ABI of the MI355X (gfx950) Attention-U-Net hot path.
 *
 * The drop-in boundary of this build.  The reference (seagochen/unet-segment-pytorch) is pure Python
 * and has no FFI: its device work is implicit ATen calls made from `nn.Module.forward`s.  Each entry
 * point below replaces one of those call sites (or a fused group of them); the reference line it
 * replaces is cited on each declaration.  The Python host (`unet/_hip/lib.py`) binds this header
 * with ctypes — see INTEGRATION.md.
 *
 * Conventions
 *  - Plain pointers + sizes only.  Activations are NHWC (channels innermost), element type chosen by
 *    `dtype` (UNET_F32, UNET_BF16 or UNET_F16); BN statistics, gradients and parameters are fp32.
 *  - `stream` is a hipStream_t passed as void* (0 = legacy default stream).  No entry point
 *    synchronises, allocates, or reads device memory from the host.
 *  - Every entry point returns 0 on success or a hipError_t / UNET_ERR_* code; unet_last_error()
 *    returns a static message describing the last failure on the calling thread.
 *  - Workspace sizes are queried with the matching *_workspace() call and allocated by the caller.
 */
#ifndef UNET_HIP_H
#define UNET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* unet_version() of a library built from this header.  110: unet_conv_desc gained `workspace` (round 5);
 * a caller built against an older header must not pass its (shorter) descriptors to this library */
#define UNET_ABI_VERSION 110

enum { UNET_F32 = 0, UNET_BF16 = 1, UNET_F16 = 2 };  /* operand (activation / weight) type */
enum { UNET_ERR_ARG = 1001, UNET_ERR_UNSUPPORTED = 1002 };

/* How a convolution input channel range is produced from a stored tensor ("virtual activation").
 * The conv kernels apply these transforms while staging input tiles into LDS, so BN-apply, ReLU,
 * zero-pad, the concat and the attention multiply are never materialised.  The network plan does
 * write two derived maps once per step with unet_materialize / unet_materialize_pool (the 2x2
 * max-pooled input of each Down block and the bilinear x2 upsample of each Up block's decoder
 * input), because a 4-corner gather inside the MFMA kernels measured slower; the POOL_ACT / UP_ACT
 * kinds remain for standalone module calls and those materialise kernels. */
enum {
  UNET_SRC_PLAIN = 0,    /* x[n,h,w,c] as stored                                                  */
  UNET_SRC_ACT = 1,      /* relu?(x*scale[c]+shift[c]) (train/eval BN apply + ReLU), optional gate  */
  UNET_SRC_POOL_ACT = 2, /* max over 2x2 of ACT(x) at (2h+i, 2w+j)           — layers.py:56        */
  UNET_SRC_UP_ACT = 3,   /* bilinear(align_corners) of ACT(x), placed with pad — layers.py:78,183  */
  UNET_SRC_NCHW_F32 = 4, /* fp32 NCHW model input (no transform)             — unet.py:75/177    */
  UNET_SRC_UP_PLAIN = 5  /* PLAIN placed with pad offsets (ConvTranspose2d output, layers.py:101)  */
};

typedef struct unet_src {
  int kind;             /* UNET_SRC_*                                                            */
  int C;                /* channels contributed by this source                                   */
  int H, W;             /* stored tensor spatial size                                            */
  const void* data;     /* stored tensor (op dtype; fp32 for NCHW_F32)                           */
  const float* scale;   /* ACT kinds: per-channel scale (gamma*invstd)                           */
  const float* shift;   /* ACT kinds: per-channel shift (beta-mean*scale)                        */
  int relu;             /* ACT kinds: apply ReLU after the affine                                */
  int up_h, up_w;       /* UP kinds: interpolated size (before pad) / placed size for UP_PLAIN   */
  int pad_t, pad_l;     /* UP kinds: placement of the interpolated map in the conv input         */
  float sh, sw;         /* UP_ACT: align_corners source scales (H-1)/(up_h-1), (W-1)/(up_w-1)   */
  const float* gate_p;  /* ACT only, optional: psi pre-activation p[n,h,w]; value *= sigmoid(...)  */
  const float* gate_ab; /* ACT only: psi BN affine {scale, shift} (2 floats, device)              */
} unet_src;

/* Output modes of the implicit-GEMM convolution */
enum {
  UNET_OUT_Y = 0,         /* store y (op dtype, NHWC) + per-tile BN partial sums                  */
  UNET_OUT_F32 = 1,       /* fp32 NHWC; split channels [0,split) -> out, [split,Cout) -> out2      */
  UNET_OUT_POOL_BWD = 2,  /* route to the 2x2 argmax of pool_src (ACT), add into out (fp32)        */
  UNET_OUT_SHUFFLE2 = 3,  /* ConvTranspose2d(k=2, s=2) as a 1x1 conv with Cout = 4*Ct: output channel
                             (2a+b)*Ct + c of pixel (y, x) -> out[n, 2y+a, 2x+b, c] + bias[c]
                             (op dtype [N,2H,2W,Ct])                         — layers.py:81,218   */
  UNET_OUT_F32_GATED = 4  /* the attention gate's W_x input gradient with the x*s term fused in
                             (layers.py:171-192): out[px][c] (+)= sigmoid(pool_src.gate_p[px] *
                             pool_src.gate_ab[0] + gate_ab[1]) * pool_src.data[px][c] + (W^T dy)[px][c];
                             pool_src.data = d(x*s), fp32 NHWC [N,H,W,Cout]; split == Cout; `accum` as
                             F32.  Served by the bf16 1x1 path only (unet_conv_variant "pw_conv_kernel")*/
};

typedef struct unet_conv_desc {
  int dtype;              /* UNET_F32 / UNET_BF16 — operand type of x/weights                     */
  int N, H, W;            /* conv input == output spatial size (stride 1, 'same' padding)        */
  int Cin, Cout;
  int ksize;              /* 1 or 3                                                               */
  int nsrc;               /* 1 or 2 (channel concat, src[0] first — layers.py:105,254)            */
  unet_src src[2];
  const void* weight;     /* packed by unet_pack_weight (fragment-major, see below)               */
  int out_mode;           /* UNET_OUT_*                                                           */
  void* out;              /* Y: op dtype [N,H,W,Cout]; F32: fp32 [N,H,W,split]                     */
  void* out2;             /* F32 split: fp32 [N,H,W,Cout-split]                                   */
  int split;              /* F32: channel split point (== Cout for no split)                       */
  int accum, accum2;      /* F32: add into out / out2 instead of storing                          */
  float* stats;           /* Y: [2][Cout][mtiles] partial sum / sum of squares (may be NULL)       */
  unet_src pool_src;      /* POOL_BWD: the pre-pool activation (kind ACT, H=2H', W=2W')           */
  const float* bias;      /* SHUFFLE2: fp32 [Ct] (may be NULL)                                     */
  const uint8_t* pool_code; /* POOL_BWD, optional: 2x2 argmax (0..3, row-major) per pooled element and
                             channel [N,H,W,Cout], as written by unet_materialize_pool             */
  /* Y mode, optional — the BatchNorm backward reduction of the activation whose gradient this conv
   * writes (a dgrad with a single consumer; replaces the Σ passes of BatchNorm2d's backward,
   * layers.py:33-37): with g = out (as stored) where relu?(bnb_y*bnb_scale+bnb_shift) > 0, else 0,
   * bnb_stats[r][Cout] = Σ g and bnb_stats[rows + r][Cout] = Σ g·(bnb_y − bnb_mean)·bnb_invstd over the
   * r-th of rows = unet_conv_stats_rows(d) pixel tiles (ask with bnb_y set; reduce the two
   * [rows][Cout] arrays with unet_bn_bwd_finalize).                                                 */
  const void* bnb_y;      /* op dtype [N,H,W,Cout]: the activation's stored conv output            */
  const float* bnb_scale; /* its BN affine (scale, shift), ReLU flag and batch statistics          */
  const float* bnb_shift;
  int bnb_relu;
  const float* bnb_mean;
  const float* bnb_invstd;
  float* bnb_stats;       /* NULL: no reduction                                                    */
  /* Y mode, optional (unet_conv_act_out_ok): src[0]'s values as the conv reads them (BN-apply, ReLU,
   * attention gate, layers.py:33-34,192), op dtype [N,H,W,src[0].C], written once — the weight
   * gradient of this conv then reads a stored map instead of re-applying the transform               */
  void* act_out;
  /* scratch of unet_conv_workspace(d) bytes (device), or NULL: the split-K form of the 3x3 conv on maps
   * too small to fill the chip keeps its fp32 partial sums there.  Optional: with NULL, unet_conv runs
   * the unsplit form (slower on those maps, same contract).  unet_conv_stats_rows depends on it: ask
   * with the workspace pointer you will launch with                                                   */
  void* workspace;
} unet_conv_desc;

typedef struct unet_wgrad_desc {
  int dtype;
  int N, H, W, Cin, Cout, ksize, nsrc;
  unet_src src[2];        /* conv input, same description as the forward                          */
  const void* dy;         /* op dtype NHWC [N,H,W,Cout] — gradient at the conv output             */
  float* dw;              /* fp32 OIHW [Cout][Cin][k][k] — output (overwritten, or += if accum)     */
  int accum;
  void* workspace;        /* unet_wgrad_workspace() bytes                                          */
} unet_wgrad_desc;

/* ---- misc ---------------------------------------------------------------------------------- */
const char* unet_last_error(void);
int unet_version(void);   /* == UNET_ABI_VERSION */
/* number of M tiles (8x16 output pixels) of a conv with this geometry: rows of the stats buffer  */
int unet_conv_mtiles(int N, int H, int W);
/* rows of the BN partial-sum buffer (stats = float[2][Cout][rows]) unet_conv will write for d    */
int unet_conv_stats_rows(const unet_conv_desc* d);
/* name of the kernel instantiation unet_conv dispatches d to (for profiling / roofline probes)   */
int unet_conv_variant(const unet_conv_desc* d, char* buf, int len);
/* bytes of d->workspace the split-K form of d needs (0: d has no split-K form); independent of
 * d->workspace itself                                                                             */
size_t unet_conv_workspace(const unet_conv_desc* d);
/* does unet_conv write d->act_out for this descriptor (else the caller keeps the activation source)? */
int unet_conv_act_out_ok(const unet_conv_desc* d);
/* name of the weight-gradient kernel unet_conv_wgrad dispatches d to (profiling / tests)          */
int unet_wgrad_variant(const unet_wgrad_desc* d, char* buf, int len);

/* ---- weights (nn.Conv2d weight OIHW fp32 -> packed operand) -------------------------------- */
/* replaces the implicit weight read of nn.Conv2d — layers.py:32,35,120,152,158,164            */
/* fragment-major [Rpad/16][Kpad/KC][k*k][64 lanes][16 B], KC = 32 (bf16) / 16 (fp32), Rpad = R
 * rounded up to 128.  transpose=0: rows R = Cout, reduction K = Cin (forward);
 * transpose=1 (dgrad): rows R = Cin, reduction K = Cout, taps flipped 180 degrees               */
int unet_pack_weight(int dtype, const float* w_oihw, void* packed, int Cout, int Cin, int ksize,
                     int transpose, void* stream);
int unet_packed_weight_elems(int dtype, int Cout, int Cin, int ksize, int transpose);
/* many weights in one launch (all convs of a network forward, or all dgrad packs of a backward) */
#define UNET_PACK_MAX_JOBS 64
typedef struct unet_pack_job {
  const float* w;         /* OIHW fp32                                                            */
  void* packed;           /* unet_packed_weight_elems(dtype, Cout, Cin, ksize, transpose) elements   */
  int Cout, Cin, ksize, transpose;
} unet_pack_job;
int unet_pack_weights(int dtype, int count, const unet_pack_job* jobs, void* stream);

/* ---- convolution (fwd / dgrad) ------------------------------------------------------------- */
/* replaces nn.Conv2d.forward (3x3 pad1 / 1x1, no bias) on a transformed input — layers.py:31-38,
 * 55-58, 95-106, 151-160, 183-188, 241-255; and its input-gradient (convolution_backward dgrad) */
int unet_conv(const unet_conv_desc* d, void* stream);

/* ---- convolution weight gradient ----------------------------------------------------------- */
size_t unet_wgrad_workspace(const unet_wgrad_desc* d);
int unet_conv_wgrad(const unet_wgrad_desc* d, void* stream);

/* ---- BatchNorm2d (train: batch stats; eval: running stats) — layers.py:33,36,153,159,165 ---- */
/* reduce conv partial sums -> mean/invstd/scale/shift; update running stats in place (momentum<0:
 * cumulative average as nn.BatchNorm2d(momentum=None)); ++num_batches_tracked                    */
int unet_bn_finalize(const float* stats, int rows, int C, long long count, const float* gamma,
                     const float* beta, float* running_mean, float* running_var,
                     long long* num_batches_tracked, float momentum, float eps,
                     float* mean, float* invstd, float* scale, float* shift, void* stream);
/* eval mode: scale/shift from the running statistics; mean / invstd (optional, may be NULL) receive
 * running_mean and 1/sqrt(running_var + eps) for the backward of an eval-mode forward             */
int unet_bn_eval_affine(int C, const float* gamma, const float* beta, const float* running_mean,
                        const float* running_var, float eps, float* scale, float* shift, float* mean,
                        float* invstd, void* stream);
/* backward: g = da * [scale*y+shift > 0] (relu!=0) ; partial sums of g and g*xhat              */
int unet_bn_bwd_reduce_rows(long long P, int C);
/* da: gradient w.r.t. the activation, fp32 (da_dtype UNET_F32) or bf16 (UNET_BF16, with dtype UNET_BF16) */
int unet_bn_bwd_reduce(int dtype, int da_dtype, long long P, int C, const void* da, const void* y,
                       const float* scale, const float* shift, int relu, const float* mean,
                       const float* invstd, float* partial, void* stream);
/* -> dgamma, dbeta (fp32 [C], stored or accumulated) and coef[3][C] with dy = A*g + B*y + Cc.
 * count = the batch-statistics pixel count; count == 0: eval mode (running statistics, which the
 * backward treats as constants): A = gamma*invstd, B = Cc = 0                                      */
int unet_bn_bwd_finalize(const float* sum_g, const float* sum_gx, int rows, int C, long long count,
                         const float* gamma, const float* mean, const float* invstd, float* dgamma,
                         float* dbeta, int accum, float* coef, void* stream);
/* column sums of a [rows][C] fp32 partial table (fp64 accumulation): out (+)= sum_r part[r][:]    */
int unet_colsum(const float* part, int rows, int C, float* out, int accum, void* stream);
/* Several independent finalizes in ONE launch (round 5: the attention gate's W_g / W_x BatchNorms,
 * whose statistics are ready together).  Each job has exactly the arguments (and results) of one
 * unet_bn_finalize / unet_bn_bwd_finalize call; a backward job with gamma == NULL and coef == NULL is
 * a column sum into dbeta (unet_colsum).  count <= UNET_BN_MULTI_MAX.                                 */
#define UNET_BN_MULTI_MAX 4
typedef struct unet_bn_finalize_job {
  const float* stats; int rows, C; long long count; const float* gamma; const float* beta;
  float* running_mean; float* running_var; long long* num_batches_tracked; float momentum, eps;
  float* mean; float* invstd; float* scale; float* shift;
} unet_bn_finalize_job;
int unet_bn_finalize_multi(int count, const unet_bn_finalize_job* jobs, void* stream);
typedef struct unet_bn_bwd_finalize_job {
  const float* sum_g; const float* sum_gx; int rows, C; long long count; const float* gamma;
  const float* mean; const float* invstd; float* dgamma; float* dbeta; int accum; float* coef;
} unet_bn_bwd_finalize_job;
int unet_bn_bwd_finalize_multi(int count, const unet_bn_bwd_finalize_job* jobs, void* stream);
/* dy (op dtype) = A*g + B*y + Cc                                                                */
int unet_bn_bwd_apply(int dtype, int da_dtype, long long P, int C, const void* da, const void* y,
                      const float* scale, const float* shift, int relu, const float* coef, void* dy, void* stream);
/* the same two passes for a Down block's input activation (N, H, W, C; C % 8 == 0, C/8 a power of two),
 * whose MaxPool2d(2) backward (layers.py:56) is folded in: g = da (fp32, NULL = no other consumer) +
 * g2[n][h/2][w/2][c] where code[n][h/2][w/2][c] == 2*(h&1) + (w&1) (g2: fp32 [N][ph][pw][C], the Down
 * conv's dgrad; code: unet_materialize_pool's argmax codes).  Replaces the pool-routing dgrad epilogue's
 * read-modify-write of the full-resolution gradient.                                             */
int unet_bn_bwd_reduce_pool(int dtype, long long N, int H, int W, int C, const float* da, const float* g2,
                            const uint8_t* code, int ph, int pw, const void* y, const float* scale,
                            const float* shift, int relu, const float* mean, const float* invstd, float* partial,
                            void* stream);
int unet_bn_bwd_apply_pool(int dtype, long long N, int H, int W, int C, const float* da, const float* g2,
                           const uint8_t* code, int ph, int pw, const void* y, const float* scale, const float* shift,
                           int relu, const float* coef, void* dy, void* stream);

/* ---- attention gate (AttentionGate.forward/backward) — layers.py:171-192 ---------------------- */
/* p = sum_c wpsi_c * relu(sg*gw+bg + sx*xw+bx) ; partial sums of p                               */
int unet_gate_psi_rows(long long P);
int unet_gate_psi(int dtype, long long P, int Ci, const void* gw, const void* xw, const float* gab,
                  const float* xab, const float* wpsi, float* p, float* partial, void* stream);
/* eval mode in one pass (scripts/predict.py): p = sum_c wpsi_c * relu(sg*(W_g.g)+bg + sx*(W_x.x)+bx)
 * straight from g (stored, at x's size) and x = relu?(y*xs+xb), W_g / W_x packed (transpose=0);
 * gab / xab: [2][Ci] eval BN affines.  16-bit operands, Cg, Cx, Ci divisible by 32               */
int unet_gate_psi_eval(int dtype, long long P, int Cg, int Cx, int Ci, const void* g, const void* x,
                       const float* xs, const float* xb, int xrelu, const void* wg_packed,
                       const void* wx_packed, const float* gab, const float* xab, const float* wpsi,
                       float* p, void* stream);
/* backward 1: x = ACT(y_x); s = sigmoid(psi BN(p)); ds = sum_c d_c x_c; dx (+)= d*s; dq = ds s (1-s)
 * (dx may be NULL: the d*s term then goes through the W_x dgrad, UNET_OUT_F32_GATED)             */
int unet_gate_bwd1(int dtype, long long P, int Cx, const float* dxs, const void* yx, const float* sx,
                   const float* bx, int relu, const float* p, const float* psi_ab, const float* psi_mean,
                   const float* psi_invstd, float* dx, int dx_accum, float* dq, float* partial, void* stream);
/* backward 2 (reduce): dz = dp*wpsi*[a>0]; partial sums (dz, dz*ghat, dz*xhat, dp*a)             */
int unet_gate_bwd2_rows(long long P, int Ci);
int unet_gate_bwd2(int dtype, long long P, int Ci, const void* gw, const void* xw, const float* gab,
                   const float* xab, const float* g_mean, const float* g_invstd, const float* x_mean,
                   const float* x_invstd, const float* wpsi, const float* dq, const float* p,
                   const float* psi_coef, float* partial, void* stream);
/* finalize of bwd2: two unet_bn_bwd_finalize calls (partial rows 0/1 and 0/2) + unet_colsum (row 3)  */
/* backward 3 (apply): dgw, dxw (op dtype)                                                        */
int unet_gate_bwd3(int dtype, long long P, int Ci, const void* gw, const void* xw, const float* gab,
                   const float* xab, const float* wpsi, const float* dq, const float* p,
                   const float* psi_coef, const float* gcoef, const float* xcoef, void* dgw, void* dxw,
                   void* stream);

/* ---- bilinear resampling (align_corners=True) — layers.py:78,183 ; unet.py:206-208 ---------- */
/* backward of UP: gather-form adjoint of the interpolation (deterministic).  d_up is fp32 NHWC
 * [N,Hp,Wp,C] (the padded map), result fp32 NHWC [N,Hs,Ws,C] stored or accumulated             */
int unet_upsample_bwd(long long N, int C, int Hs, int Ws, int up_h, int up_w, int pad_t, int pad_l,
                      int Hp, int Wp, float sh, float sw, const float* d_up, float* dx, int accum,
                      void* stream);
/* generic fp32 NCHW bilinear resize (deep-supervision heads) fwd and bwd                         */
int unet_resize_nchw(long long NC, int Hi, int Wi, int Ho, int Wo, float sh, float sw, const float* x,
                     float* y, void* stream);
int unet_resize_nchw_bwd(long long NC, int Hi, int Wi, int Ho, int Wo, float sh, float sw,
                         const float* dy, float* dx, int accum, void* stream);

/* ---- ConvTranspose2d(k=2, s=2) backward helper — layers.py:81,218 ------------------------------ */
/* d_up: fp32 NHWC [N,Hp,Wp,Ct] gradient at the padded up map (the transposed conv output sits at
 * rows pad_t.., cols pad_l..).  Writes dy_s2d (op dtype [N,h,w,4*Ct], channel (2a+b)*Ct + c =
 * d_up[n, pad_t+2y+a, pad_l+2x+b, c]) — the gradient of the equivalent 1x1 conv — and per-block
 * bias partial sums partial[rows][Ct] (finish with unet_colsum).                                  */
int unet_convt_bwd_rows(long long P);
int unet_convt_bwd_prep(int dtype, long long N, int h, int w, int Ct, int Hp, int Wp, int pad_t, int pad_l,
                        const float* d_up, void* dy_s2d, float* partial, void* stream);

/* ---- OutConv (1x1 conv + bias, few classes) — layers.py:109-123 ------------------------------ */
int unet_outconv_rows(long long P);
int unet_outconv_fwd(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                     const float* shift, int relu, const float* w, const float* b, float* logits_nchw,
                     void* stream);
int unet_outconv_bwd(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                     const float* shift, int relu, const float* w, const float* dlogits_nchw, float* da,
                     int da_accum, float* partial, void* stream);
/* OutConv backward fused with the BatchNorm backward of its input (the last DoubleConv's output, whose only
 * consumer is OutConv — unet.py:92, 203; layers.py:120 + 33-37): from y and the logit gradient dl (fp32 NCHW,
 * n_classes == 2) accumulates OutConv's partials (as unet_outconv_bwd) and the BN-backward sums
 * bn_partial[2][rows][C] (Σ g_m, Σ g_m·x̂; rows = unet_outconv_rows(P), for unet_bn_bwd_finalize) without storing
 * the activation gradient g = W^T dl                                                                      */
int unet_outconv_bwd_bn(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                        const float* shift, int relu, const float* w, const float* dl, const float* mean,
                        const float* invstd, float* partial, float* bn_partial, void* stream);
/* the matching BN-backward apply: dy = coef0·g_m + coef1·y + coef2 with g recomputed from dl          */
int unet_bn_bwd_apply_oc(int dtype, long long N, int H, int W, int C, int K, const void* y, const float* scale,
                         const float* shift, int relu, const float* w, const float* dl, const float* coef, void* dy,
                         void* stream);
int unet_outconv_bwd_finalize(const float* partial, int rows, int C, int K, float* dw, float* db,
                              int accum, void* stream);

/* ---- layout ---------------------------------------------------------------------------------- */
/* NCHW fp32 <-> NHWC (op dtype / fp32) for standalone module calls                                */
int unet_nchw_to_nhwc(int dtype, long long N, int C, int H, int W, const float* x, void* y, void* stream);
int unet_nhwc_to_nchw(int dtype, long long N, int C, int H, int W, const void* x, const float* scale,
                      const float* shift, int relu, float* y, void* stream);
/* x*sigmoid(psi BN(p)) of an ACT tensor as NCHW fp32 (standalone AttentionGate output)           */
int unet_gated_to_nchw(int dtype, long long N, int C, int H, int W, const void* x, const float* scale,
                       const float* shift, int relu, const float* p, const float* psi_ab, float* y, void* stream);
int unet_fill_f32(float* x, long long n, float v, void* stream);
/* write the virtual source `src` (as a conv with an N x H x W input would read it: pool, bilinear-up
 * + pad, BN-apply/ReLU, attention gate) as a plain NHWC tensor of op dtype [N,H,W,src->C]          */
int unet_materialize(int dtype, const unet_src* src, long long N, int H, int W, void* out, void* stream);
/* MaxPool2d(2) of an ACT source (kind POOL_ACT) as a plain tensor plus its argmax codes (0..3 in
 * the window's row-major order, first maximum wins as in ATen; uint8 [N,H,W,C]) — layers.py:56   */
int unet_materialize_pool(int dtype, const unet_src* src, long long N, int H, int W, void* out, uint8_t* code,
                          void* stream);

/* ---- segmentation metrics — SegmentationMetrics.update, metrics.py:55-84 ----------------------- */
/* confusion[t][p] += #pixels with target t, predicted class p (argmax over the C fp32 NCHW logit
 * channels — C may differ from K, as the reference's argmax-then-count allows — or the int64 labels
 * when logits == NULL); pixels with t == ignore_index (has_ignore != 0) or a t or p outside [0, K) are
 * skipped (metrics.py:68-84).  confusion: int64 [K][K] on the device, accumulated (never cleared).  */
int unet_confusion_matrix(long long N, int C, int K, long long HW, const float* logits, const int64_t* labels,
                          const int64_t* targets, long long ignore_index, int has_ignore, int64_t* confusion,
                          void* stream);
/* compute_iou / compute_dice, metrics.py:160-231: a (K+1) x (K+1) matrix (int64, accumulated) whose
 * row / column K counts targets / predictions outside [0, K), so every pixel lands once and
 * |pred == c| / |target == c| are the column / row sums; logits have C channels (C may differ from K). */
int unet_confusion_matrix_ext(long long N, int C, int K, long long HW, const float* logits, const int64_t* labels,
                              const int64_t* targets, int64_t* confusion, void* stream);

/* ---- DiceBCE / Dice / BalancedCE loss + grad — loss.py:18-191 ------------------------------- */
int unet_loss_rows(long long HW);
/* pass 1: per-image partial sums (fp32 NCHW logits, int64 targets)                               */
int unet_loss_reduce(long long N, int K, long long HW, const float* z, const int64_t* t, float* partial,
                     void* stream);
/* finalize: loss scalar(s) + per-(n,c) gradient coefficients                                    */
int unet_loss_finalize(const float* partial, int rows, long long N, int K, float ce_w, float dice_w,
                       float class_w, float ce_smooth, float dice_smooth, int ignore_bg, int reduction,
                       float* loss, float* coef, void* stream);
/* pass 2: dz = gout * d loss / dz                                                                 */
int unet_loss_grad(long long N, int K, long long HW, const float* z, const int64_t* t, const float* coef,
                   const float* gout, int gout_per_elem, int ignore_bg, float* dz, void* stream);

/* ---- DeepSupervisionLoss(base) over S <= 4 logit sets — loss.py:194-229 ----------------------
 * The sets [main, ds1, ds2, ds3] (same shape, shared targets; unet.py:204-209) go through ONE launch
 * of each pass: partial [S][N][rows][4+3K], coef [S][N][2+2K] (scaled by set_weights[s]),
 * loss = sum_s set_weights[s] * base_loss_s (host arrays z / dz / set_weights of S entries).       */
int unet_loss_reduce_multi(int S, long long N, int K, long long HW, const float* const* z, const int64_t* t,
                           float* partial, void* stream);
int unet_loss_finalize_multi(const float* partial, int rows, int S, const float* set_weights, long long N, int K,
                             float ce_w, float dice_w, float class_w, float ce_smooth, float dice_smooth,
                             int ignore_bg, int reduction, float* loss, float* coef, void* stream);
int unet_loss_grad_multi(int S, long long N, int K, long long HW, const float* const* z, const int64_t* t,
                         const float* coef, const float* gout, int gout_per_elem, int ignore_bg, float* const* dz,
                         void* stream);

/* ---- device input pipeline and inference post-processing (csrc/infer.hip) ------------------- */
/* One separable pass of PIL's 8-bit Image.resize(BILINEAR) (Resample.c) over a (N, inH, inW) uint8
 * batch: axis 1 = horizontal (out (N, inH, out_len)), axis 0 = vertical (out (N, out_len, inW)).
 * bounds int32 [out_len][2] (first source index, count) and coeffs int32 [out_len][ksize] are
 * Pillow's fixed-point tables (unet/utils/pil_tables.py).  roundtrip != 0 first maps each source
 * byte u -> uint8(float32(u / 255) * 255) (the float round trip of augmentations.py:150).           */
int unet_resample_u8(int axis, long long N, int inH, int inW, int out_len, const uint8_t* in, int roundtrip,
                     const int32_t* bounds, const int32_t* coeffs, int ksize, uint8_t* out, void* stream);
/* apply_basic_transforms tail (augmentations.py:153-171) + mask binarisation (dataset.py:148-149):
 * out_img fp32 (N,1,H,W) = (uint8 img [after the optional round trip] / 255 - mean) / std, flipped
 * left-right where flip[n] != 0 (flip may be NULL); if mask != NULL: out_mask int64 (N,H,W) =
 * (mask[n][ytab[y]][xtab[x']] > 127) with PIL NEAREST tables ytab[H], xtab[W] (mask is mask_h x mask_w). */
int unet_slice_finish(long long N, int H, int W, const uint8_t* img, int roundtrip, int mask_h, int mask_w,
                      const uint8_t* mask, const int32_t* ytab, const int32_t* xtab, const uint8_t* flip, float mean,
                      float stdv, float* out_img, int64_t* out_mask, void* stream);
/* postprocess_mask of scripts/predict.py:138-165: out uint8 (N,outH,outW) = 255 where
 * softmax(logits[n, :, ytab[y], xtab[x]])[cls] > threshold, else 0 (PIL NEAREST tables).           */
int unet_postprocess_mask(long long N, int K, int H, int W, const float* logits, int cls, float threshold, int outH,
                          int outW, const int32_t* ytab, const int32_t* xtab, uint8_t* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UNET_HIP_H */
