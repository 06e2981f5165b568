// loss.hip — fused DiceBCE / Dice / BalancedCE loss and gradient (unet/utils/loss.py:18-191).
//
// Pass 1 (reduce): per image n and 256-pixel-range block, softmax + cross entropy per pixel and the
//   sums  n0 = #[t=0], n1 = #[t=1], S0 = Σ_{t=0} ce, S1 = Σ_{t=1} ce, and per class c:
//   I_c = Σ p_c [t=c], P_c = Σ p_c, T_c = #[t=c].           (loss.py:63-73 and 129-148)
// Finalize (one block): loss scalar and per-(n, c) gradient coefficients, in fp64.
// Pass 2 (grad): dz_k = gout · ( w_t (p_k − [k=t]) + G_k p_k [k∈D] − p_k Σ_{c∈D} G_c p_c ),
//   G_c = gA_nc [t=c] + gB_nc,  w_t = BalancedCE per-pixel weight (labels 0/1 only, loss.py:136-145).
// The per-image Python loop with boolean-mask indexing of the reference (loss.py:134-145) becomes
// these device reductions: no host synchronisation.
// Deep supervision (DeepSupervisionLoss, loss.py:194-229; unet.py:204-209): the S = 4 logit sets
// [main, ds1, ds2, ds3] share the targets, so one launch of each pass covers all of them (blockIdx.z /
// the grid-stride index select the set) and the finalize forms Σ_s w_s · loss_s and per-set
// coefficients already scaled by w_s.
#include "common.h"

namespace unet {

constexpr int LMAXK = 16;
constexpr int LMAXS = 4;   // logit sets per launch (deep supervision: main + 3 heads)

struct LossSets {
  const float* z[LMAXS];
  float* dz[LMAXS];
  float w[LMAXS];
};

// partial rows per image: 1024 pixels each (4 per thread; round 5 — 4096-pixel rows left the bs-4 512^2 reduce
// on 256 blocks, 16 dependent pixel iterations per thread: 19 us for 16 MB)
static inline int loss_rows(long long HW) {
  long long r = (HW + 1023) / 1024;
  if (r > 1024) r = 1024;
  if (r < 1) r = 1;
  return (int)r;
}

template <int KT>
__global__ void loss_reduce_kernel(long long N, int K_, long long HW, const LossSets sets, const int64_t* t, float* part,
                                   int rows) {
  __shared__ float sh[8];
  const int K = KT ? KT : K_;
  const int F = 4 + 3 * K;
  const long long n = blockIdx.y;
  const float* z = sets.z[blockIdx.z];
  part += (size_t)blockIdx.z * N * rows * F;
  const long long per = (HW + rows - 1) / rows;
  const long long q0 = blockIdx.x * per, q1 = min(HW, q0 + per);
  float acc[4 + 3 * (KT ? KT : LMAXK)];
#pragma unroll
  for (int f = 0; f < 4 + 3 * (KT ? KT : LMAXK); ++f) acc[f] = 0.f;
  for (long long q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
    const float* zp = z + n * K * HW + q;
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < (KT ? KT : LMAXK); ++k) if (k < K) m = fmaxf(m, zp[k * HW]);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < (KT ? KT : LMAXK); ++k) if (k < K) se += __expf(zp[k * HW] - m);
    const float lse = m + __logf(se);
    int tv = (int)t[n * HW + q];
    if (tv < 0 || tv >= K) tv = -1;  // out-of-range label (the reference raises): contributes nothing
    const float ce = tv >= 0 ? lse - zp[tv * HW] : 0.f;
    if (tv == 0) { acc[0] += 1.f; acc[2] += ce; }
    if (tv == 1) { acc[1] += 1.f; acc[3] += ce; }
    const float inv = 1.f / se;
#pragma unroll
    for (int k = 0; k < (KT ? KT : LMAXK); ++k) {
      if (k >= K) break;
      const float pk = __expf(zp[k * HW] - m) * inv;
      acc[4 + 3 * k + 1] += pk;
      if (tv == k) { acc[4 + 3 * k] += pk; acc[4 + 3 * k + 2] += 1.f; }
    }
  }
#pragma unroll
  for (int f = 0; f < 4 + 3 * (KT ? KT : LMAXK); ++f) {
    if (f >= F) break;
    float v = wave_sum(acc[f]);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      float s = 0.f;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sh[w];
      part[((size_t)n * rows + blockIdx.x) * F + f] = s;
    }
    __syncthreads();
  }
}

// one block: per set s (1) one wave per (image, field) pair sums the partial rows in fp64 (fixed order
// per lane, then a fixed shuffle tree); (2) one thread per image forms its terms; (3) thread 0 combines.
// coef layout [S][N][2 + 2K]: w0, w1, gA[K], gB[K] (already scaled by the set weight); loss: Σ_s w_s loss_s
__global__ void loss_finalize_kernel(const float* part, int rows, int S, const LossSets sets, long long N, int K,
                                     float ce_w, float dice_w, float class_w, float ce_smooth, float dice_smooth,
                                     int ignore_bg, int reduction, float* loss, float* coef) {
  extern __shared__ double dsh[];  // [N] ce terms, [N*K] dice terms, [N*F] field sums
  const int F = 4 + 3 * K;
  const int c_lo = (ignore_bg && K > 1) ? 1 : 0;
  const int nd = K - c_lo;
  const double wred = reduction == 0 ? 1.0 / ((double)N * nd) : 1.0;  // mean / sum / none(=1, gout per elem)
  double* fs = dsh + N + N * K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  double total = 0;
  for (int si = 0; si < S; ++si) {
    const float* ps = part + (size_t)si * N * rows * F;
    const double ws = sets.w[si];
    for (long long pf = wave; pf < N * F; pf += nw) {
      const long long n = pf / F;
      const int f = (int)(pf % F);
      double a = 0;
      for (int r = lane; r < rows; r += 64) a += ps[((size_t)n * rows + r) * F + f];
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o, 64);
      if (lane == 0) fs[pf] = a;
    }
    __syncthreads();
    for (long long n = threadIdx.x; n < N; n += blockDim.x) {
      const double* s = fs + n * F;
      const double n0 = (double)(float)(s[0]) + ce_smooth, n1 = (double)(float)(s[1]) + ce_smooth;
      const double w0 = (1.0 - class_w) / n0, w1 = class_w / n1;
      dsh[n] = w0 * s[2] + w1 * s[3];
      float* cf = coef + ((size_t)si * N + n) * (2 + 2 * K);
      cf[0] = (float)(ws * ce_w * w0 / (double)N);
      cf[1] = (float)(ws * ce_w * w1 / (double)N);
      for (int c = 0; c < K; ++c) {
        const double I = s[4 + 3 * c], P = s[4 + 3 * c + 1], T = s[4 + 3 * c + 2];
        const double U = P + T + dice_smooth;
        const double D = (2.0 * I + dice_smooth) / U;
        double gA = 0, gB = 0;
        if (c >= c_lo) {
          gA = -2.0 * ws * dice_w * wred / U;
          gB = ws * dice_w * wred * (2.0 * I + dice_smooth) / (U * U);
        }
        cf[2 + c] = (float)gA;
        cf[2 + K + c] = (float)gB;
        dsh[N + n * K + c] = D;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (reduction == 2) {  // DiceLoss(reduction='none'): per-(n, c) 1 - D (single set)
        for (long long n = 0; n < N; ++n)
          for (int c = c_lo; c < K; ++c) loss[n * nd + (c - c_lo)] = (float)(1.0 - dsh[N + n * K + c]);
      } else {
        double ce = 0, dsum = 0;
        for (long long n = 0; n < N; ++n) {
          ce += dsh[n];
          for (int c = c_lo; c < K; ++c) dsum += dsh[N + n * K + c];
        }
        ce /= (double)N;
        const double dl = reduction == 0 ? 1.0 - dsum / ((double)N * nd) : (double)N * nd - dsum;
        total += ws * (ce_w * ce + dice_w * dl);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && reduction != 2) loss[0] = (float)total;
}

template <int KT>
__global__ void loss_grad_kernel(int S, long long N, int K_, long long HW, const LossSets sets, const int64_t* t,
                                 const float* coef, const float* gout, int gout_per_elem, int c_lo) {
  constexpr int KM = KT ? KT : LMAXK;
  const int K = KT ? KT : K_;
  const long long total = N * HW;
  const int nd = K - c_lo;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total * S;
       e += (long long)gridDim.x * blockDim.x) {
    const int si = (int)(e / total);
    const long long en = e - (long long)si * total;
    const long long n = en / HW, q = en % HW;
    const float* zp = sets.z[si] + n * K * HW + q;
    float* dz = sets.dz[si];
    const float* cf = coef + ((size_t)si * N + n) * (2 + 2 * K);
    float p[KM];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < KM; ++k) if (k < K) m = fmaxf(m, zp[k * HW]);
    float se = 0.f;
#pragma unroll
    for (int k = 0; k < KM; ++k) { p[k] = (k < K) ? __expf(zp[k * HW] - m) : 0.f; se += p[k]; }
    const float inv = 1.f / se;
#pragma unroll
    for (int k = 0; k < KM; ++k) p[k] *= inv;
    int tv = (int)t[n * HW + q];
    if (tv < 0 || tv >= K) tv = -1;
    const float wt = tv == 0 ? cf[0] : (tv == 1 ? cf[1] : 0.f);
    float G[KM];
    float sgp = 0.f;
#pragma unroll
    for (int c = 0; c < KM; ++c) {
      float g = 0.f;
      if (c < K && c >= c_lo) {
        g = (tv == c ? cf[2 + c] : 0.f) + cf[2 + K + c];
        if (gout_per_elem) g *= gout[n * nd + c - c_lo];
      }
      G[c] = g;
      sgp += g * p[c];
    }
    const float go = gout_per_elem ? 1.f : gout[0];
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      if (k >= K) break;
      const float ce = wt * (p[k] - (k == tv ? 1.f : 0.f));
      dz[n * K * HW + k * HW + q] = go * (ce + G[k] * p[k] - p[k] * sgp);
    }
  }
}

}  // namespace unet

using namespace unet;

extern "C" {

int unet_loss_rows(long long HW) { return loss_rows(HW); }

static int load_sets(int S, const float* const* z, float* const* dz, const float* w, LossSets& ls) {
  if (S < 1 || S > LMAXS || !z) { set_error("unet_loss: 1 to 4 logit sets"); return UNET_ERR_ARG; }
  for (int i = 0; i < LMAXS; ++i) {
    ls.z[i] = i < S ? z[i] : nullptr;
    ls.dz[i] = (i < S && dz) ? dz[i] : nullptr;
    ls.w[i] = i < S ? (w ? w[i] : 1.f) : 0.f;
  }
  return 0;
}

int unet_loss_reduce_multi(int S, long long N, int K, long long HW, const float* const* z, const int64_t* t,
                           float* partial, void* stream) {
  if (K < 1 || K > LMAXK) { set_error("unet_loss_reduce: n_classes must be in [1, 16]"); return UNET_ERR_UNSUPPORTED; }
  LossSets ls;
  if (int rc = load_sets(S, z, nullptr, nullptr, ls)) return rc;
  const int rows = loss_rows(HW);
  if (K == 2)
    hipLaunchKernelGGL(loss_reduce_kernel<2>, dim3(rows, N, S), dim3(256), 0, (hipStream_t)stream, N, K, HW, ls, t,
                       partial, rows);
  else
    hipLaunchKernelGGL(loss_reduce_kernel<0>, dim3(rows, N, S), dim3(256), 0, (hipStream_t)stream, N, K, HW, ls, t,
                       partial, rows);
  return check_launch("loss_reduce");
}

int unet_loss_reduce(long long N, int K, long long HW, const float* z, const int64_t* t, float* partial, void* stream) {
  return unet_loss_reduce_multi(1, N, K, HW, &z, t, partial, stream);
}

int unet_loss_finalize_multi(const float* partial, int rows, int S, const float* set_weights, long long N, int K,
                             float ce_w, float dice_w, float class_w, float ce_smooth, float dice_smooth, int ignore_bg,
                             int reduction, float* loss, float* coef, void* stream) {
  LossSets ls;
  const float* zs[LMAXS] = {nullptr, nullptr, nullptr, nullptr};
  if (S < 1 || S > LMAXS || (S > 1 && reduction == 2)) {
    set_error("unet_loss_finalize: 1 to 4 sets, reduction 'none' only for one set");
    return UNET_ERR_ARG;
  }
  load_sets(S, zs, nullptr, set_weights, ls);
  const size_t shm = (size_t)(N + N * K + N * (4 + 3 * K)) * sizeof(double);
  if (shm > 60000) { set_error("unet_loss_finalize: batch too large"); return UNET_ERR_UNSUPPORTED; }
  // 16 waves: the (image, field) row sums are one memory round trip each, spread over more waves
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(1024), shm, (hipStream_t)stream, partial, rows, S, ls, N, K,
                     ce_w, dice_w, class_w, ce_smooth, dice_smooth, ignore_bg, reduction, loss, coef);
  return check_launch("loss_finalize");
}

int unet_loss_finalize(const float* partial, int rows, long long N, int K, float ce_w, float dice_w, float class_w,
                       float ce_smooth, float dice_smooth, int ignore_bg, int reduction, float* loss, float* coef,
                       void* stream) {
  return unet_loss_finalize_multi(partial, rows, 1, nullptr, N, K, ce_w, dice_w, class_w, ce_smooth, dice_smooth,
                                  ignore_bg, reduction, loss, coef, stream);
}

int unet_loss_grad_multi(int S, long long N, int K, long long HW, const float* const* z, const int64_t* t,
                         const float* coef, const float* gout, int gout_per_elem, int ignore_bg, float* const* dz,
                         void* stream) {
  LossSets ls;
  if (!dz) { set_error("unet_loss_grad: no outputs"); return UNET_ERR_ARG; }
  if (int rc = load_sets(S, z, dz, nullptr, ls)) return rc;
  long long b = (S * N * HW + 255) / 256;
  if (b > 8192) b = 8192;
  const int c_lo = (ignore_bg && K > 1) ? 1 : 0;
  if (K == 2)
    hipLaunchKernelGGL(loss_grad_kernel<2>, dim3((int)b), dim3(256), 0, (hipStream_t)stream, S, N, K, HW, ls, t, coef,
                       gout, gout_per_elem, c_lo);
  else
    hipLaunchKernelGGL(loss_grad_kernel<0>, dim3((int)b), dim3(256), 0, (hipStream_t)stream, S, N, K, HW, ls, t, coef,
                       gout, gout_per_elem, c_lo);
  return check_launch("loss_grad");
}

int unet_loss_grad(long long N, int K, long long HW, const float* z, const int64_t* t, const float* coef,
                   const float* gout, int gout_per_elem, int ignore_bg, float* dz, void* stream) {
  return unet_loss_grad_multi(1, N, K, HW, &z, t, coef, gout, gout_per_elem, ignore_bg, &dz, stream);
}

}  // extern "C"
