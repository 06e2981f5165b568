// bn.hip — training-mode BatchNorm2d statistics and backward for NHWC activations.
//
// Reference: nn.BatchNorm2d in unet/models/layers.py:33,36,153,159,165 (train mode: biased batch
// variance to normalise, unbiased variance into running_var, momentum 0.1, eps 1e-5).  The forward
// statistics come from the conv epilogue's per-tile partial sums; they are reduced here in a fixed
// order in fp64 (deterministic, like the CPU path's double accumulation).  The backward is
//   g    = da * [scale*y + shift > 0]                       (ReLU, layers.py:34,37)
//   dβ   = Σ g,  dγ = Σ g·x̂,  dy = γ·invstd·(g − dβ/M − x̂·dγ/M)
// as two streaming passes (reduce, apply) around a per-channel finalize.
#include "common.h"

namespace unet {

__device__ __forceinline__ double block_sum_d(double v, double* sh) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((tid & 63) == 0) sh[tid >> 6] = v;
  __syncthreads();
  double r = 0;
  if (tid == 0) {
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r += sh[w];
    sh[0] = r;
  }
  __syncthreads();
  r = sh[0];
  __syncthreads();
  return r;
}


// the (sum, sum) pair of a block in one LDS round (fixed order: waves in index order)
__device__ __forceinline__ void block_sum2_d(double& a, double& b, double* sh) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
  if ((tid & 63) == 0) { sh[2 * (tid >> 6)] = a; sh[2 * (tid >> 6) + 1] = b; }
  __syncthreads();
  a = 0; b = 0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { a += sh[2 * w]; b += sh[2 * w + 1]; }
}

// finalize blocks: one trip of 4 loads per thread for up to 4096 partial rows (the kernels are a few
// dependent memory round trips long; fewer trips = shorter kernels)
static inline int fin_threads(int rows) {
  int t = ((rows + 3) / 4 + 63) / 64 * 64;
  return t < 64 ? 64 : (t > 1024 ? 1024 : t);
}

// one block per channel (the body shared by the single and the batched launch)
__device__ __forceinline__ void bn_finalize_body(const float* stats, int rows, int C, long long count,
                                                 const float* gamma, const float* beta, float* rmean, float* rvar,
                                                 long long* nbt, float momentum, float eps, float* mean, float* invstd,
                                                 float* scale, float* shift, int c, double* sh2) {
  // the per-channel operands of the epilogue, loaded before the partial rows (in flight together: the kernel is
  // a chain of dependent memory round trips, and these need not be one of them)
  float g_ = 0.f, b_ = 0.f, rm_ = 0.f, rv_ = 0.f;
  long long nb_ = 0;
  if (threadIdx.x == 0) {
    g_ = gamma[c];
    b_ = beta[c];
    if (rmean && rvar) { rm_ = rmean[c]; rv_ = rvar[c]; }
    if (nbt && momentum < 0) nb_ = *nbt;
  }
  double s = 0, ss = 0;
  const float* s0 = stats + (size_t)c * rows;         // [2][C][rows]: contiguous over r
  const float* s1 = stats + ((size_t)C + c) * rows;
  const int B = blockDim.x;
  int r = threadIdx.x;
  // 4 rows per trip: the loads of a trip are independent (issued together), the fp64 adds stay in
  // row order per thread (deterministic)
  for (; r + 3 * B < rows; r += 4 * B) {
    const float a0 = s0[r], a1 = s0[r + B], a2 = s0[r + 2 * B], a3 = s0[r + 3 * B];
    const float b0 = s1[r], b1 = s1[r + B], b2 = s1[r + 2 * B], b3 = s1[r + 3 * B];
    s += a0; s += a1; s += a2; s += a3;
    ss += b0; ss += b1; ss += b2; ss += b3;
  }
  for (; r < rows; r += B) {
    s += s0[r];
    ss += s1[r];
  }
  block_sum2_d(s, ss, sh2);
  if (threadIdx.x == 0) {
    const double m = s / (double)count;
    double var = ss / (double)count - m * m;
    if (var < 0) var = 0;
    const double is = 1.0 / sqrt(var + (double)eps);
    mean[c] = (float)m;
    invstd[c] = (float)is;
    const float sc = (float)((double)g_ * is);
    scale[c] = sc;
    shift[c] = (float)((double)b_ - m * (double)g_ * is);
    if (rmean && rvar) {
      double f = momentum;
      if (momentum < 0) f = nbt ? 1.0 / (double)(nb_ + 1) : 1.0;  // momentum=None: cumulative average
      const double unb = count > 1 ? var * (double)count / (double)(count - 1) : var;
      rmean[c] = (float)((1.0 - f) * (double)rm_ + f * m);
      rvar[c] = (float)((1.0 - f) * (double)rv_ + f * unb);
    }
    // momentum=None reads *nbt in every block, so block 0 must not increment it in the same launch (a block
    // scheduled after it would use 1/(nbt+2)): that case increments in a follow-up launch (bn_nbt_inc_kernel)
    if (c == 0 && nbt && momentum >= 0) *nbt += 1;
  }
}

// ++num_batches_tracked of the momentum=None finalizes, after every block of the finalize has read the old value
struct BnNbtList {
  long long* p[UNET_BN_MULTI_MAX];
  int n;
};
__global__ void bn_nbt_inc_kernel(const BnNbtList l) {
  if (threadIdx.x < (unsigned)l.n) *l.p[threadIdx.x] += 1;
}

__global__ void bn_finalize_kernel(const float* stats, int rows, int C, long long count, const float* gamma,
                                   const float* beta, float* rmean, float* rvar, long long* nbt, float momentum,
                                   float eps, float* mean, float* invstd, float* scale, float* shift) {
  __shared__ double sh2[32];
  bn_finalize_body(stats, rows, C, count, gamma, beta, rmean, rvar, nbt, momentum, eps, mean, invstd, scale, shift,
                   (int)blockIdx.x, sh2);
}

// the batched form: blocks [c0[k], c0[k+1]) serve job k (block-uniform)
struct BnFinJobs {
  unet_bn_finalize_job j[UNET_BN_MULTI_MAX];
  int c0[UNET_BN_MULTI_MAX + 1];
  int n;
};
__global__ void bn_finalize_multi_kernel(const BnFinJobs js) {
  __shared__ double sh2[32];
  int k = 0;
  while (k + 1 < js.n && (int)blockIdx.x >= js.c0[k + 1]) ++k;
  const unet_bn_finalize_job& jb = js.j[k];
  bn_finalize_body(jb.stats, jb.rows, jb.C, jb.count, jb.gamma, jb.beta, jb.running_mean, jb.running_var,
                   jb.num_batches_tracked, jb.momentum, jb.eps, jb.mean, jb.invstd, jb.scale, jb.shift,
                   (int)blockIdx.x - js.c0[k], sh2);
}

// eval mode: the running-statistics affine; mean / invstd (optional) are what the backward of an eval-mode
// forward normalises with (x̂ = (y - running_mean) * invstd)
__global__ void bn_eval_kernel(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                               float* scale, float* shift, float* mean, float* invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = 1.0f / sqrtf(rv[c] + eps);
  const float sc = gamma[c] * is;
  scale[c] = sc;
  shift[c] = beta[c] - rm[c] * sc;
  if (mean) mean[c] = rm[c];
  if (invstd) invstd[c] = is;
}

// 2-D layout: CL channel lanes x (256/CL) pixel rows; grid (ceil(C/CL), rows)
static inline int chan_lanes(int C) {
  int cl = 1;
  while (cl < C && cl < 64) cl <<= 1;
  return cl;
}
static inline int reduce_rows(long long P, int C) {
  const int cl = chan_lanes(C);
  const int cblocks = (C + cl - 1) / cl;
  const char* e = getenv("UNET_BN_ROWS");   // A/B of the partial-row count (default 2048 blocks)
  const long long want = e && atoll(e) > 0 ? atoll(e) : 2048;
  long long r = (want + cblocks - 1) / cblocks;
  const long long maxr = (P + 63) / 64;  // at least 64 pixels per block
  if (r > maxr) r = maxr;
  if (r < 1) r = 1;
  return (int)r;
}

template <typename T, typename G>
__global__ void bn_bwd_reduce_kernel(long long P, int C, int CL, const G* da, const T* y, const float* scale,
                                     const float* shift, int relu, const float* mean, const float* invstd, float* part,
                                     int rows) {
  __shared__ float sh[2][256];
  const int tid = threadIdx.x;
  const int cx = tid % CL, py = tid / CL, R = blockDim.x / CL;
  const int c = blockIdx.x * CL + cx;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.y * per, p1 = min(P, p0 + per);
  float sg = 0.f, sgx = 0.f;
  if (c < C) {
    const float sc = scale[c], sf = shift[c], mu = mean[c], is = invstd[c];
    for (long long p = p0 + py; p < p1; p += R) {
      const float yv = to_f(y[p * C + c]);
      float g = to_f(da[p * C + c]);
      if (relu && !(__builtin_fmaf(yv, sc, sf) > 0.f)) g = 0.f;
      sg += g;
      sgx += g * (yv - mu) * is;
    }
  }
  sh[0][tid] = sg;
  sh[1][tid] = sgx;
  __syncthreads();
  if (py == 0 && c < C) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < R; ++r) { a += sh[0][r * CL + cx]; b += sh[1][r * CL + cx]; }
    part[(size_t)blockIdx.y * C + c] = a;
    part[((size_t)rows + blockIdx.y) * C + c] = b;
  }
}

// 8 gradient values (fp32: two 16-byte loads; bf16: one)
template <typename G> __device__ __forceinline__ void load8(const G* p, float* v) {
  load_vec<G>(p, v);
  if constexpr (sizeof(G) == 4) load_vec<G>(p + 4, v + 4);
}

// The MaxPool2d(2) backward of a Down block's input, left at the pooled resolution: the Down's first-conv
// dgrad writes g2 (fp32 [N][ph][pw][C], plain stores) and the materialised pool's argmax codes (uint8, same
// shape, q = 2*dy + dx in the window) route it here.  Full-resolution element (n, h, w, c) receives
// g2[n][h/2][w/2][c] where code == 2*(h&1) + (w&1) (rows / columns past 2*ph, 2*pw: none), added after the
// other consumers' sum `da` — the order and values of the RMW the pool-routing dgrad epilogue did
// (layers.py:56, MaxPool2d backward), without that epilogue's read-modify-write of the full map.
struct PoolG {
  const float* g2;
  const uint8_t* code;
  int H, W, ph, pw;
};

// (32-bit index math: the host admits N*H*W < 2^31; a 64-bit division here cost half the bandwidth)
__device__ __forceinline__ void pool_add8(const PoolG& pg, int C, long long p, int c0, float* g) {
  const unsigned pu = (unsigned)p, W = (unsigned)pg.W, H = (unsigned)pg.H;
  const unsigned t = pu / W, w = pu - t * W;
  const unsigned n = t / H, h = t - n * H;
  const unsigned hh = h >> 1, ww = w >> 1;
  if (hh >= (unsigned)pg.ph || ww >= (unsigned)pg.pw) return;
  const size_t o = (size_t)((n * (unsigned)pg.ph + hh) * (unsigned)pg.pw + ww) * C + c0;
  const uint2 cw = *reinterpret_cast<const uint2*>(pg.code + o);
  const float4 a = *reinterpret_cast<const float4*>(pg.g2 + o);
  const float4 b = *reinterpret_cast<const float4*>(pg.g2 + o + 4);
  const unsigned q = (unsigned)((h & 1) * 2 + (w & 1));
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned cj = ((j < 4 ? cw.x : cw.y) >> (8 * (j & 3))) & 0xffu;
    if (cj == q) g[j] += v[j];
  }
}

// a pixel's (n, h, w), advanced in place by a fixed pixel step (no per-pixel division): the routed pooled
// gradient of a thread's pixel sequence p, p + S, p + 2S, ...
struct PixCur {
  unsigned n, h, w;
};
__device__ __forceinline__ PixCur pix_cur(const PoolG& pg, unsigned p) {
  const unsigned W = (unsigned)pg.W, H = (unsigned)pg.H;
  const unsigned t = p / W, w = p - t * W;
  const unsigned n = t / H;
  return PixCur{n, t - n * H, w};
}
// step = sq * W + sr (sr < W), split once by the caller
__device__ __forceinline__ void pix_adv(PixCur& c, const PoolG& pg, unsigned sq, unsigned sr) {
  c.w += sr;
  unsigned h = c.h + sq;
  if (c.w >= (unsigned)pg.W) { c.w -= (unsigned)pg.W; ++h; }
  while (h >= (unsigned)pg.H) { h -= (unsigned)pg.H; ++c.n; }
  c.h = h;
}
__device__ __forceinline__ void pool_add8c(const PoolG& pg, int C, const PixCur& pc, int c0, float* g) {
  const unsigned hh = pc.h >> 1, ww = pc.w >> 1;
  if (hh >= (unsigned)pg.ph || ww >= (unsigned)pg.pw) return;
  const size_t o = (size_t)((pc.n * (unsigned)pg.ph + hh) * (unsigned)pg.pw + ww) * C + c0;
  const uint2 cw = *reinterpret_cast<const uint2*>(pg.code + o);
  const float4 a = *reinterpret_cast<const float4*>(pg.g2 + o);
  const float4 b = *reinterpret_cast<const float4*>(pg.g2 + o + 4);
  const unsigned q = (pc.h & 1) * 2 + (pc.w & 1);
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const unsigned cj = ((j < 4 ? cw.x : cw.y) >> (8 * (j & 3))) & 0xffu;
    if (cj == q) g[j] += v[j];
  }
}

// vectorised forms (C % 8 == 0): a thread owns 8 channels (16-byte y, 2 x 16-byte da) of one pixel;
// the block covers 256 / (C/8) pixels per iteration with a fixed channel vector per thread.
// POOL: + the pooled gradient (PoolG); da may then be null (no other consumer)
template <typename T, typename G, bool POOL = false>
__global__ __launch_bounds__(256) void bn_bwd_reduce_vec_kernel(long long P, int C, const G* __restrict__ da,
                                                                const T* __restrict__ y,
                                                                const float* scale, const float* shift, int relu,
                                                                const float* mean, const float* invstd, float* part,
                                                                int rows, PoolG pg = PoolG{}) {
  __shared__ float sh[2][256 * 8 / 8];
  const int CV = C / 8, tid = threadIdx.x;
  const int cv = tid % CV, py = tid / CV, R = 256 / CV;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float sc[8], sf[8], mu[8], is[8], sg[8], sgx[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cv * 8 + j;
    sc[j] = scale[c]; sf[j] = shift[c]; mu[j] = mean[c]; is[j] = invstd[c];
    sg[j] = 0.f; sgx[j] = 0.f;
  }
  // 4 pixels per trip without the pooled gradient (17.6 -> 15.7 us per launch); with it the extra registers
  // cost more than the overlap gains (59 -> 64 us), so one.  The pooled gradient's pixel coordinates advance
  // by the fixed step R (pix_adv) instead of two 32-bit divisions per pixel
  // (the pooled form must stay at one pixel per trip: its cursor pc only tracks p while p < p1)
  constexpr int BNR_U = POOL ? 1 : 4;
  PixCur pc{0, 0, 0};
  const unsigned sq = POOL ? (unsigned)R / (unsigned)(pg.W > 0 ? pg.W : 1) : 0u, sr = POOL ? (unsigned)R - sq * (unsigned)pg.W : 0u;
  if (POOL && py < R && p0 + py < p1) pc = pix_cur(pg, (unsigned)(p0 + py));
  if (py < R) {
    // BNR_U pixels per trip, all their loads issued before the sums (one memory round trip per trip, not
    // per pixel); the sums still run over p, p + R, p + 2R, ... in order (bit-identical to one per trip)
    for (long long p = p0 + py; p < p1; p += BNR_U * (long long)R) {
      float yv[BNR_U][8], g[BNR_U][8];
      bool ok[BNR_U];
#pragma unroll
      for (int u = 0; u < BNR_U; ++u) {
        ok[u] = p + u * R < p1;
        const long long q = ok[u] ? p + u * R : p;
        load_vec<T>(y + q * C + cv * 8, yv[u]);
        if constexpr (sizeof(T) == 4) load_vec<T>(y + q * C + cv * 8 + 4, yv[u] + 4);
        if (!POOL || da) {
          load8<G>(da + q * C + cv * 8, g[u]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) g[u][j] = 0.f;
        }
        if constexpr (POOL) {
          pool_add8c(pg, C, pc, cv * 8, g[u]);
          pix_adv(pc, pg, sq, sr);
        }
      }
#pragma unroll
      for (int u = 0; u < BNR_U; ++u) {
        if (!ok[u]) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float gj = (relu && !(__builtin_fmaf(yv[u][j], sc[j], sf[j]) > 0.f)) ? 0.f : g[u][j];
          sg[j] += gj;
          sgx[j] += gj * (yv[u][j] - mu[j]) * is[j];
        }
      }
    }
  }
  // reduce over the R pixel rows of each channel vector (fixed order)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][tid] = sg[j];
    sh[1][tid] = sgx[j];
    __syncthreads();
    if (tid < CV) {
      float a = 0.f, b = 0.f;
      for (int r = 0; r < R; ++r) { a += sh[0][r * CV + tid]; b += sh[1][r * CV + tid]; }
      part[(size_t)blockIdx.x * C + tid * 8 + j] = a;
      part[((size_t)rows + blockIdx.x) * C + tid * 8 + j] = b;
    }
    __syncthreads();
  }
}

template <typename T, typename G, bool POOL = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_vec_kernel(long long P, int C, const G* da, const T* y,
                                                               const float* scale, const float* shift, int relu,
                                                               const float* coef, T* dy, PoolG pg = PoolG{}) {
  const int CV = C / 8;
  const long long total = P * CV;
  const long long stride = (long long)gridDim.x * blockDim.x;
  long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const int cv = (int)(e % CV);  // fixed: the stride is a multiple of CV (power of two <= 256)
  float sc[8], sf[8], A[8], B[8], Cc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cv * 8 + j;
    sc[j] = scale[c]; sf[j] = shift[c]; A[j] = coef[c]; B[j] = coef[C + c]; Cc[j] = coef[2 * C + c];
  }
  const int cvs = __builtin_ctz(CV);  // CV is a power of two (bn_vec_ok)
  // 2 pixels per trip, every load issued before the stores (dy may alias the loads as far as the compiler
  // knows, which serialised one memory round trip per pixel); elementwise, so the results are unchanged
  constexpr int U = 2;
  for (; e < total; e += U * stride) {
    float yv[U][8], g[U][8];
    long long pu[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ok[u] = e + u * stride < total;
      pu[u] = (ok[u] ? e + u * stride : e) >> cvs;
      const long long p = pu[u];
      load_vec<T>(y + p * C + cv * 8, yv[u]);
      if constexpr (sizeof(T) == 4) load_vec<T>(y + p * C + cv * 8 + 4, yv[u] + 4);
      if (!POOL || da) {
        load8<G>(da + p * C + cv * 8, g[u]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[u][j] = 0.f;
      }
      if constexpr (POOL) pool_add8(pg, C, p, cv * 8, g[u]);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) break;
      const long long p = pu[u];
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float gj = (relu && !(__builtin_fmaf(yv[u][j], sc[j], sf[j]) > 0.f)) ? 0.f : g[u][j];
        // explicit fma order, here and in the pre-activation y * scale + shift of the ReLU masks (the compiler's
        // contraction choice moved with the code's shape in round 6: fused and unfused paths must round alike);
        // the OutConv and attention-gate forms (misc.hip, gate.hip) round the same way
        o[j] = f32_rounded(__builtin_fmaf(A[j], gj, __builtin_fmaf(B[j], yv[u][j], Cc[j])));
      }
      if constexpr (sizeof(T) == 2) {
        store_vec<T>(dy + p * C + cv * 8, o);
      } else {
        store_vec<T>(dy + p * C + cv * 8, o);
        store_vec<T>(dy + p * C + cv * 8 + 4, o + 4);
      }
    }
  }
}

static inline bool bn_vec_ok(int C) {
  const int cv = C / 8;
  return C % 8 == 0 && cv <= 256 && (cv & (cv - 1)) == 0;
}
static inline int reduce_rows_vec(long long P, int C) {
  const int R = 256 / (C / 8);
  long long r = (P + 8LL * R - 1) / (8LL * R);  // >= 8 pixel iterations per thread
  const char* e = getenv("UNET_BN_ROWS");        // A/B of the partial-row cap (default 2048 blocks)
  const long long cap = e && atoll(e) > 0 ? atoll(e) : 2048;
  if (r > cap) r = cap;
  if (r < 1) r = 1;
  return (int)r;
}

// one block per channel: sums over rows in fp64.  count == 0: eval mode (running statistics are constants
// of the forward), so dy = γ·invstd·g: coef = (γ·invstd, 0, 0).  (The body shared by the single and the
// batched launch; with coef == NULL and dgamma == NULL it is a column sum of sum_g into dbeta.)
__device__ __forceinline__ void bn_bwd_finalize_body(const float* sum_g, const float* sum_gx, int rows, int C,
                                                     long long count, const float* gamma, const float* mean,
                                                     const float* invstd, float* dgamma, float* dbeta, int accum,
                                                     float* coef, int c, double* sh2) {
  // the epilogue's per-channel operands, in flight with the partial rows (as bn_finalize_body)
  float g_ = 0.f, is_ = 0.f, mu_ = 0.f, dg_ = 0.f, db_ = 0.f;
  if (threadIdx.x == 0) {
    if (coef) {
      g_ = gamma[c];
      is_ = invstd[c];
      if (count > 0) mu_ = mean[c];
    }
    if (accum) {
      if (dgamma) dg_ = dgamma[c];
      if (dbeta) db_ = dbeta[c];
    }
  }
  const bool two = sum_gx && (dgamma || coef);   // a column-sum job reads one table
  double a = 0, b = 0;
  const int B = blockDim.x;
  int r = threadIdx.x;
  for (; r + 3 * B < rows; r += 4 * B) {  // 4 independent loads per trip, adds in row order
    const float g0 = sum_g[(size_t)r * C + c], g1 = sum_g[(size_t)(r + B) * C + c];
    const float g2 = sum_g[(size_t)(r + 2 * B) * C + c], g3 = sum_g[(size_t)(r + 3 * B) * C + c];
    a += g0; a += g1; a += g2; a += g3;
    if (two) {
      const float x0 = sum_gx[(size_t)r * C + c], x1 = sum_gx[(size_t)(r + B) * C + c];
      const float x2 = sum_gx[(size_t)(r + 2 * B) * C + c], x3 = sum_gx[(size_t)(r + 3 * B) * C + c];
      b += x0; b += x1; b += x2; b += x3;
    }
  }
  for (; r < rows; r += B) {
    a += sum_g[(size_t)r * C + c];
    if (two) b += sum_gx[(size_t)r * C + c];
  }
  block_sum2_d(a, b, sh2);
  if (threadIdx.x == 0) {
    if (dbeta) dbeta[c] = accum ? db_ + (float)a : (float)a;
    if (dgamma) dgamma[c] = accum ? dg_ + (float)b : (float)b;
    if (coef) {
      const double k = (double)g_ * is_;
      coef[c] = (float)k;
      if (count > 0) {
        const double M = (double)count;
        const double B = -k * (double)is_ * b / M;
        coef[C + c] = (float)B;
        coef[2 * C + c] = (float)(-k * a / M - B * (double)mu_);
      } else {
        coef[C + c] = 0.f;
        coef[2 * C + c] = 0.f;
      }
    }
  }
}

__global__ void bn_bwd_finalize_kernel(const float* sum_g, const float* sum_gx, int rows, int C, long long count,
                                       const float* gamma, const float* mean, const float* invstd, float* dgamma,
                                       float* dbeta, int accum, float* coef) {
  __shared__ double sh2[32];
  bn_bwd_finalize_body(sum_g, sum_gx, rows, C, count, gamma, mean, invstd, dgamma, dbeta, accum, coef,
                       (int)blockIdx.x, sh2);
}

struct BnBwdFinJobs {
  unet_bn_bwd_finalize_job j[UNET_BN_MULTI_MAX];
  int c0[UNET_BN_MULTI_MAX + 1];
  int n;
};
__global__ void bn_bwd_finalize_multi_kernel(const BnBwdFinJobs js) {
  __shared__ double sh2[32];
  int k = 0;
  while (k + 1 < js.n && (int)blockIdx.x >= js.c0[k + 1]) ++k;
  const unet_bn_bwd_finalize_job& jb = js.j[k];
  bn_bwd_finalize_body(jb.sum_g, jb.sum_gx, jb.rows, jb.C, jb.count, jb.gamma, jb.mean, jb.invstd, jb.dgamma,
                       jb.dbeta, jb.accum, jb.coef, (int)blockIdx.x - js.c0[k], sh2);
}

template <typename T, typename G>
__global__ void bn_bwd_apply_kernel(long long P, int C, int CL, const G* da, const T* y, const float* scale,
                                    const float* shift, int relu, const float* coef, T* dy, int rows) {
  const int tid = threadIdx.x;
  const int cx = tid % CL, py = tid / CL, R = blockDim.x / CL;
  const int c = blockIdx.x * CL + cx;
  if (c >= C) return;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.y * per, p1 = min(P, p0 + per);
  const float sc = scale[c], sf = shift[c], A = coef[c], B = coef[C + c], Cc = coef[2 * C + c];
  for (long long p = p0 + py; p < p1; p += R) {
    const float yv = to_f(y[p * C + c]);
    float g = to_f(da[p * C + c]);
    if (relu && !(__builtin_fmaf(yv, sc, sf) > 0.f)) g = 0.f;
    dy[p * C + c] = from_f<T>(f32_rounded(__builtin_fmaf(A, g, __builtin_fmaf(B, yv, Cc))));
  }
}

// column sums over rows (fp64): out[c] (+)= sum_r part[r][c]
__global__ void colsum_kernel(const float* part, int rows, int C, float* out, int accum) {
  __shared__ double sh[16];
  const int c = blockIdx.x;
  double a = 0;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) a += part[(size_t)r * C + c];
  a = block_sum_d(a, sh);
  if (threadIdx.x == 0) out[c] = accum ? out[c] + (float)a : (float)a;
}

}  // namespace unet

using namespace unet;

extern "C" {

int unet_bn_finalize(const float* stats, int rows, int C, long long count, const float* gamma, const float* beta,
                     float* running_mean, float* running_var, long long* nbt, float momentum, float eps, float* mean,
                     float* invstd, float* scale, float* shift, void* stream) {
  if (!stats || rows <= 0 || C <= 0 || count <= 0 || !gamma || !beta || !mean || !invstd || !scale || !shift) {
    set_error("unet_bn_finalize: bad args");
    return UNET_ERR_ARG;
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(fin_threads(rows)), 0, (hipStream_t)stream, stats, rows, C, count, gamma,
                     beta, running_mean, running_var, nbt, momentum, eps, mean, invstd, scale, shift);
  if (int e = check_launch("bn_finalize")) return e;
  if (nbt && momentum < 0) {
    BnNbtList l{};
    l.p[0] = nbt;
    l.n = 1;
    hipLaunchKernelGGL(bn_nbt_inc_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, l);
    return check_launch("bn_finalize nbt");
  }
  return 0;
}

int unet_bn_finalize_multi(int count, const unet_bn_finalize_job* jobs, void* stream) {
  if (count < 1 || count > UNET_BN_MULTI_MAX || !jobs) {
    set_error("unet_bn_finalize_multi: 1..UNET_BN_MULTI_MAX jobs");
    return UNET_ERR_ARG;
  }
  BnFinJobs js{};
  js.n = count;
  int rows_max = 1;
  js.c0[0] = 0;
  for (int k = 0; k < count; ++k) {
    const unet_bn_finalize_job& j = jobs[k];
    if (!j.stats || j.rows <= 0 || j.C <= 0 || j.count <= 0 || !j.gamma || !j.beta || !j.mean || !j.invstd || !j.scale ||
        !j.shift) {
      set_error("unet_bn_finalize_multi: bad job");
      return UNET_ERR_ARG;
    }
    js.j[k] = j;
    js.c0[k + 1] = js.c0[k] + j.C;
    rows_max = j.rows > rows_max ? j.rows : rows_max;
  }
  hipLaunchKernelGGL(bn_finalize_multi_kernel, dim3(js.c0[count]), dim3(fin_threads(rows_max)), 0, (hipStream_t)stream, js);
  if (int e = check_launch("bn_finalize_multi")) return e;
  BnNbtList l{};
  for (int k = 0; k < count; ++k) {
    const unet_bn_finalize_job& j = jobs[k];
    if (j.num_batches_tracked && j.momentum < 0) l.p[l.n++] = j.num_batches_tracked;
  }
  if (l.n) {
    hipLaunchKernelGGL(bn_nbt_inc_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, l);
    return check_launch("bn_finalize_multi nbt");
  }
  return 0;
}

int unet_bn_bwd_finalize_multi(int count, const unet_bn_bwd_finalize_job* jobs, void* stream) {
  if (count < 1 || count > UNET_BN_MULTI_MAX || !jobs) {
    set_error("unet_bn_bwd_finalize_multi: 1..UNET_BN_MULTI_MAX jobs");
    return UNET_ERR_ARG;
  }
  BnBwdFinJobs js{};
  js.n = count;
  int rows_max = 1;
  js.c0[0] = 0;
  for (int k = 0; k < count; ++k) {
    const unet_bn_bwd_finalize_job& j = jobs[k];
    const bool colsum = !j.coef && !j.dgamma;
    if (!j.sum_g || j.rows <= 0 || j.C <= 0 || j.count < 0 || (!colsum && !j.sum_gx) ||
        (j.coef && (!j.gamma || !j.invstd || (j.count > 0 && !j.mean))) || (colsum && !j.dbeta)) {
      set_error("unet_bn_bwd_finalize_multi: bad job");
      return UNET_ERR_ARG;
    }
    js.j[k] = j;
    js.c0[k + 1] = js.c0[k] + j.C;
    rows_max = j.rows > rows_max ? j.rows : rows_max;
  }
  hipLaunchKernelGGL(bn_bwd_finalize_multi_kernel, dim3(js.c0[count]), dim3(fin_threads(rows_max)), 0, (hipStream_t)stream,
                     js);
  return check_launch("bn_bwd_finalize_multi");
}

int unet_bn_eval_affine(int C, const float* gamma, const float* beta, const float* rm, const float* rv, float eps,
                        float* scale, float* shift, float* mean, float* invstd, void* stream) {
  if (C <= 0 || !gamma || !beta || !rm || !rv || !scale || !shift) {
    set_error("unet_bn_eval_affine: bad args");
    return UNET_ERR_ARG;
  }
  hipLaunchKernelGGL(bn_eval_kernel, dim3(cdiv(C, 256)), dim3(256), 0, (hipStream_t)stream, C, gamma, beta, rm, rv,
                     eps, scale, shift, mean, invstd);
  return check_launch("bn_eval_affine");
}

int unet_bn_bwd_reduce_rows(long long P, int C) { return bn_vec_ok(C) ? reduce_rows_vec(P, C) : reduce_rows(P, C); }

int unet_bn_bwd_reduce(int dtype, int da_dtype, long long P, int C, const void* da, const void* y, const float* scale,
                       const float* shift, int relu, const float* mean, const float* invstd, float* partial,
                       void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (da_dtype != UNET_F32 && da_dtype != dtype) { set_error("unet_bn_bwd_reduce: a 16-bit gradient needs y of the same type"); return UNET_ERR_ARG; }
  if (bn_vec_ok(C)) {
    const int rows = reduce_rows_vec(P, C);
    if (dtype == UNET_F16 && da_dtype == UNET_F16)
      hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<f16, f16>), dim3(rows), dim3(256), 0, st, P, C, (const f16*)da,
                         (const f16*)y, scale, shift, relu, mean, invstd, partial, rows);
    else if (dtype == UNET_BF16 && da_dtype == UNET_BF16)
      hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<bf16, bf16>), dim3(rows), dim3(256), 0, st, P, C, (const bf16*)da,
                         (const bf16*)y, scale, shift, relu, mean, invstd, partial, rows);
    else if (dtype == UNET_F16)
      hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<f16, float>), dim3(rows), dim3(256), 0, st, P, C, (const float*)da,
                         (const f16*)y, scale, shift, relu, mean, invstd, partial, rows);
    else if (dtype == UNET_BF16)
      hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<bf16, float>), dim3(rows), dim3(256), 0, st, P, C, (const float*)da,
                         (const bf16*)y, scale, shift, relu, mean, invstd, partial, rows);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<float, float>), dim3(rows), dim3(256), 0, st, P, C, (const float*)da,
                         (const float*)y, scale, shift, relu, mean, invstd, partial, rows);
    return check_launch("bn_bwd_reduce");
  }
  const int cl = chan_lanes(C), rows = reduce_rows(P, C);
  dim3 grid(cdiv(C, cl), rows);
  if (dtype == UNET_F16 && da_dtype == UNET_F16)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<f16, f16>), grid, dim3(256), 0, st, P, C, cl, (const f16*)da,
                       (const f16*)y, scale, shift, relu, mean, invstd, partial, rows);
  else if (dtype == UNET_BF16 && da_dtype == UNET_BF16)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<bf16, bf16>), grid, dim3(256), 0, st, P, C, cl, (const bf16*)da,
                       (const bf16*)y, scale, shift, relu, mean, invstd, partial, rows);
  else if (dtype == UNET_F16)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<f16, float>), grid, dim3(256), 0, st, P, C, cl, (const float*)da,
                       (const f16*)y, scale, shift, relu, mean, invstd, partial, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<bf16, float>), grid, dim3(256), 0, st, P, C, cl, (const float*)da,
                       (const bf16*)y, scale, shift, relu, mean, invstd, partial, rows);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_kernel<float, float>), grid, dim3(256), 0, st, P, C, cl, (const float*)da,
                       (const float*)y, scale, shift, relu, mean, invstd, partial, rows);
  return check_launch("bn_bwd_reduce");
}

int unet_bn_bwd_finalize(const float* sum_g, const float* sum_gx, int rows, int C, long long count, const float* gamma,
                         const float* mean, const float* invstd, float* dgamma, float* dbeta, int accum, float* coef,
                         void* stream) {
  if (!sum_g || !sum_gx || rows <= 0 || C <= 0 || count < 0 || (coef && (!gamma || !invstd || (count > 0 && !mean)))) {
    set_error("unet_bn_bwd_finalize: bad args");
    return UNET_ERR_ARG;
  }
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(fin_threads(rows)), 0, (hipStream_t)stream, sum_g, sum_gx, rows, C, count,
                     gamma, mean, invstd, dgamma, dbeta, accum, coef);
  return check_launch("bn_bwd_finalize");
}

int unet_bn_bwd_apply(int dtype, int da_dtype, long long P, int C, const void* da, const void* y, const float* scale,
                      const float* shift, int relu, const float* coef, void* dy, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (da_dtype != UNET_F32 && da_dtype != dtype) { set_error("unet_bn_bwd_apply: a 16-bit gradient needs y of the same type"); return UNET_ERR_ARG; }
  if (bn_vec_ok(C)) {
    long long b = (P * (C / 8) + 255) / 256;
    if (b > 8192) b = 8192;
    if (dtype == UNET_F16 && da_dtype == UNET_F16)
      hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<f16, f16>), dim3((int)b), dim3(256), 0, st, P, C, (const f16*)da,
                         (const f16*)y, scale, shift, relu, coef, (f16*)dy);
    else if (dtype == UNET_BF16 && da_dtype == UNET_BF16)
      hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<bf16, bf16>), dim3((int)b), dim3(256), 0, st, P, C, (const bf16*)da,
                         (const bf16*)y, scale, shift, relu, coef, (bf16*)dy);
    else if (dtype == UNET_F16)
      hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<f16, float>), dim3((int)b), dim3(256), 0, st, P, C, (const float*)da,
                         (const f16*)y, scale, shift, relu, coef, (f16*)dy);
    else if (dtype == UNET_BF16)
      hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<bf16, float>), dim3((int)b), dim3(256), 0, st, P, C, (const float*)da,
                         (const bf16*)y, scale, shift, relu, coef, (bf16*)dy);
    else
      hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<float, float>), dim3((int)b), dim3(256), 0, st, P, C, (const float*)da,
                         (const float*)y, scale, shift, relu, coef, (float*)dy);
    return check_launch("bn_bwd_apply");
  }
  const int cl = chan_lanes(C), rows = reduce_rows(P, C);
  dim3 grid(cdiv(C, cl), rows);
  if (dtype == UNET_F16 && da_dtype == UNET_F16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<f16, f16>), grid, dim3(256), 0, st, P, C, cl, (const f16*)da,
                       (const f16*)y, scale, shift, relu, coef, (f16*)dy, rows);
  else if (dtype == UNET_BF16 && da_dtype == UNET_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16, bf16>), grid, dim3(256), 0, st, P, C, cl, (const bf16*)da,
                       (const bf16*)y, scale, shift, relu, coef, (bf16*)dy, rows);
  else if (dtype == UNET_F16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<f16, float>), grid, dim3(256), 0, st, P, C, cl, (const float*)da,
                       (const f16*)y, scale, shift, relu, coef, (f16*)dy, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16, float>), grid, dim3(256), 0, st, P, C, cl, (const float*)da,
                       (const bf16*)y, scale, shift, relu, coef, (bf16*)dy, rows);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<float, float>), grid, dim3(256), 0, st, P, C, cl, (const float*)da,
                       (const float*)y, scale, shift, relu, coef, (float*)dy, rows);
  return check_launch("bn_bwd_apply");
}

// BN backward of a Down block's input activation with the pooled gradient folded in (PoolG above)
int unet_bn_bwd_reduce_pool(int dtype, long long N, int H, int W, int C, const float* da, const float* g2,
                            const uint8_t* code, int ph, int pw, const void* y, const float* scale,
                            const float* shift, int relu, const float* mean, const float* invstd, float* partial,
                            void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long long P = N * H * W;
  if (!bn_vec_ok(C) || !g2 || !code || P <= 0 || P >= (1LL << 31) || ph > (H >> 1) || pw > (W >> 1) || ph < 0 ||
      pw < 0) {
    set_error("unet_bn_bwd_reduce_pool: bad arguments (C % 8 == 0, C/8 a power of two <= 256)");
    return UNET_ERR_ARG;
  }
  const PoolG pg{g2, code, H, W, ph, pw};
  const int rows = reduce_rows_vec(P, C);
  if (dtype == UNET_F16)
    hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<f16, float, true>), dim3(rows), dim3(256), 0, st, P, C, da,
                       (const f16*)y, scale, shift, relu, mean, invstd, partial, rows, pg);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<bf16, float, true>), dim3(rows), dim3(256), 0, st, P, C, da,
                       (const bf16*)y, scale, shift, relu, mean, invstd, partial, rows, pg);
  else
    hipLaunchKernelGGL((bn_bwd_reduce_vec_kernel<float, float, true>), dim3(rows), dim3(256), 0, st, P, C, da,
                       (const float*)y, scale, shift, relu, mean, invstd, partial, rows, pg);
  return check_launch("bn_bwd_reduce_pool");
}

int unet_bn_bwd_apply_pool(int dtype, long long N, int H, int W, int C, const float* da, const float* g2,
                           const uint8_t* code, int ph, int pw, const void* y, const float* scale, const float* shift,
                           int relu, const float* coef, void* dy, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long long P = N * H * W;
  if (!bn_vec_ok(C) || !g2 || !code || P <= 0 || P >= (1LL << 31) || ph > (H >> 1) || pw > (W >> 1) || ph < 0 ||
      pw < 0) {
    set_error("unet_bn_bwd_apply_pool: bad arguments (C % 8 == 0, C/8 a power of two <= 256)");
    return UNET_ERR_ARG;
  }
  const PoolG pg{g2, code, H, W, ph, pw};
  long long b = (P * (C / 8) + 255) / 256;
  if (b > 8192) b = 8192;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<f16, float, true>), dim3((int)b), dim3(256), 0, st, P, C, da,
                       (const f16*)y, scale, shift, relu, coef, (f16*)dy, pg);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<bf16, float, true>), dim3((int)b), dim3(256), 0, st, P, C, da,
                       (const bf16*)y, scale, shift, relu, coef, (bf16*)dy, pg);
  else
    hipLaunchKernelGGL((bn_bwd_apply_vec_kernel<float, float, true>), dim3((int)b), dim3(256), 0, st, P, C, da,
                       (const float*)y, scale, shift, relu, coef, (float*)dy, pg);
  return check_launch("bn_bwd_apply_pool");
}

int unet_colsum(const float* part, int rows, int C, float* out, int accum, void* stream) {
  hipLaunchKernelGGL(colsum_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, part, rows, C, out, accum);
  return check_launch("colsum");
}

}  // extern "C"
