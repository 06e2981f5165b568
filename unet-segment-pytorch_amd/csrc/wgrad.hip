// wgrad.hip — convolution weight gradient on MFMA (gfx950).
//
// dW[co][tap][ci] = Σ_pix dy[pix][co] · X[pix + tap][ci]  (the weight half of convolution_backward for
// nn.Conv2d in unet/models/layers.py:32,35,152,158).  X is the conv input exactly as the forward saw it:
// the same unet_src descriptors re-gather BN+ReLU / pool / upsample / pad / concat / gate on the fly.
// K = pixels: both operands are read from LDS with the CDNA4 transposed read ds_read_b64_tr_b16 (bf16)
// so the [pixel][channel] tiles need no explicit transpose.  Split-K over pixel tiles into fp32 slabs,
// reduced afterwards in a fixed order (deterministic).
#include "conv_common.h"

namespace unet {

constexpr int TH = 8, TW = 16, BM = TH * TW, NTHR = 256;

// ------------------------------------------------------------------------------------------------
// weight gradient: dW[co][tap][ci] = sum_pix dy[pix][co] * X[pix + tap][ci]
// Split-K over pixel tiles; each block writes an fp32 slab, reduced in a fixed order afterwards.
// ------------------------------------------------------------------------------------------------
constexpr int WG_BCO = 64;

template <typename T> struct WgFrag {
  // A/B operand with K on the LDS ROW axis (pixels) and M/N on the column axis (channels):
  // two ds_read_b64_tr_b16 per operand (CDNA4 hardware transpose read).
  static constexpr int KSTEP = 32;
  typedef typename Mma<T>::frag frag;
  __device__ static __forceinline__ frag tr_load(const T* row_q, const T* row_q4) {
    i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(row_q));
    i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(row_q4));
    typedef __attribute__((ext_vector_type(8))) short i16x8;
    i16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(frag, r);
  }
};

template <typename T, int KS>
__global__ __launch_bounds__(NTHR) void wgrad_kernel(const unet_wgrad_desc d, int tiles_w, int tiles_h, int mtiles,
                                                      int per_split, float* ws) {
  using M = Mma<T>;
  constexpr int KC = M::KC, VEC = Vec<T>::N, NV = KC / VEC;
  constexpr int BCI = 2 * KC;                     // 64 (bf16) / 32 (f32) input channels per block
  constexpr int HALO = (KS == 3) ? 1 : 0;
  constexpr int HWID = TW + 2 * HALO, HHGT = TH + 2 * HALO, HP = HWID * HHGT;
  constexpr int RSX = BCI + 16 / (int)sizeof(T);
  constexpr int RSD = WG_BCO + 16 / (int)sizeof(T);
  constexpr int TAPS = KS * KS;
  constexpr int NTN = BCI / 32;                   // n-tiles (ci) per wave
  constexpr int KSTEP = M::KSTEP;                 // pixels per MFMA
  __shared__ __attribute__((aligned(16))) T lds[HP * RSX + BM * RSD];
  T* lds_x = lds;
  T* lds_d = lds + HP * RSX;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave >> 1, wci = wave & 1;
  const int split = blockIdx.x;
  const int ci0 = blockIdx.y * BCI;
  const int co0 = blockIdx.z * WG_BCO;

  f32x4 acc[TAPS][2][NTN];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int mt_begin = split * per_split;
  const int mt_end = min(mtiles, mt_begin + per_split);
  const T* dy = (const T*)d.dy;
  for (int mt = mt_begin; mt < mt_end; ++mt) {
    const int tw_i = mt % tiles_w;
    const int t2 = mt / tiles_w;
    const int th_i = t2 % tiles_h;
    const long long n = t2 / tiles_h;
    const int h0 = th_i * TH, w0 = tw_i * TW;
    // dy tile [BM][WG_BCO]
    constexpr int DV = WG_BCO / VEC;
    for (int it = tid; it < BM * DV; it += NTHR) {
      const int p = it / DV, v = it % DV;
      const int oh = h0 + p / TW, ow = w0 + p % TW;
      const int co = co0 + v * VEC;
      float vals[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) vals[j] = 0.f;
      if (oh < d.H && ow < d.W && co < d.Cout) {
        const T* src = dy + ((n * d.H + oh) * (long long)d.W + ow) * d.Cout + co;
        if (co + VEC <= d.Cout && (d.Cout % VEC) == 0) {
          load_vec<T>(src, vals);
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j) vals[j] = (co + j < d.Cout) ? to_f(src[j]) : 0.f;
        }
      }
      store_vec<T>(lds_d + p * RSD + v * VEC, vals);
    }
    // input halo [HP][BCI]
    for (int it = tid; it < HP * 2 * NV; it += NTHR) {
      const int hp = it / (2 * NV), v = it % (2 * NV);
      const int hy = h0 + hp / HWID - HALO, hx = w0 + hp % HWID - HALO;
      float vals[VEC];
      src_gather<T>(d.src, d.nsrc, d.Cin, d.H, d.W, n, hy, hx, ci0 + v * VEC, vals);
      store_vec<T>(lds_x + hp * RSX + v * VEC, vals);
    }
    __syncthreads();
#pragma unroll 1
    for (int k0 = 0; k0 < BM; k0 += KSTEP) {
      typename M::frag a[2];
      if constexpr (sizeof(T) == 2) {
        const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = (i16 & 3) * 4;
        const int pr = k0 + 8 * g + q;  // pixel row of the tr-read block (and +4)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int m0 = wco * 32 + i * 16 + p4;
          a[i] = WgFrag<T>::tr_load(lds_d + pr * RSD + m0, lds_d + (pr + 4) * RSD + m0);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = M::load(lds_d + (k0 + (lane >> 4)) * RSD + wco * 32 + i * 16 + (lane & 15));
      }
#pragma unroll
      for (int tap = 0; tap < TAPS; ++tap) {
        const int dy_ = tap / KS, dx_ = tap % KS;
        typename M::frag b[NTN];
        if constexpr (sizeof(T) == 2) {
          const int g = lane >> 4, i16 = lane & 15, q = i16 >> 2, p4 = (i16 & 3) * 4;
          const int p0 = k0 + 8 * g + q, p1 = p0 + 4;
          const int hp0 = (p0 / TW + dy_) * HWID + p0 % TW + dx_;
          const int hp1 = (p1 / TW + dy_) * HWID + p1 % TW + dx_;
#pragma unroll
          for (int j = 0; j < NTN; ++j) {
            const int n0 = wci * (BCI / 2) + j * 16 + p4;
            b[j] = WgFrag<T>::tr_load(lds_x + hp0 * RSX + n0, lds_x + hp1 * RSX + n0);
          }
        } else {
          const int p = k0 + (lane >> 4);
          const int hp = (p / TW + dy_) * HWID + p % TW + dx_;
#pragma unroll
          for (int j = 0; j < NTN; ++j) b[j] = M::load(lds_x + hp * RSX + wci * (BCI / 2) + j * 16 + (lane & 15));
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NTN; ++j) acc[tap][i][j] = M::mma(a[i], b[j], acc[tap][i][j]);
      }
    }
    __syncthreads();
  }
  // slab write: ws[split][co][tap][ci]  (C layout: row = co = 4*(l>>4)+r, col = ci = l&15)
  float* slab = ws + (size_t)split * d.Cout * TAPS * d.Cin;
#pragma unroll
  for (int tap = 0; tap < TAPS; ++tap)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        const int ci = ci0 + wci * (BCI / 2) + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + wco * 32 + i * 16 + 4 * (lane >> 4) + r;
          if (co < d.Cout && ci < d.Cin) slab[((size_t)co * TAPS + tap) * d.Cin + ci] = acc[tap][i][j][r];
        }
      }
}

// dw[co][ci][kh][kw] (+)= sum_s ws[s][co][tap][ci]
__global__ void wgrad_reduce_kernel(const float* ws, int splits, int Cout, int Cin, int taps, float* dw, int accum) {
  const long long total = (long long)Cout * Cin * taps;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int tap = e % taps;
    const long long t = e / taps;
    const int ci = t % Cin;
    const int co = t / Cin;
    const size_t src = ((size_t)co * taps + tap) * Cin + ci;
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += ws[(size_t)k * Cout * taps * Cin + src];
    dw[e] = accum ? dw[e] + s : s;
  }
}

struct WgPlan {
  int tiles_w, tiles_h, mtiles, splits, per_split, ci_tiles, co_tiles;
  size_t ws_bytes;
};

static WgPlan wg_plan(const unet_wgrad_desc* d) {
  WgPlan p;
  const int kc = d->dtype != UNET_F32 ? 32 : 16;
  p.tiles_w = cdiv(d->W, TW);
  p.tiles_h = cdiv(d->H, TH);
  p.mtiles = d->N * p.tiles_w * p.tiles_h;
  p.ci_tiles = cdiv(d->Cin, 2 * kc);
  p.co_tiles = cdiv(d->Cout, WG_BCO);
  const int taps = d->ksize * d->ksize;
  const size_t slab = (size_t)d->Cout * taps * d->Cin * sizeof(float);
  const int tiles = p.ci_tiles * p.co_tiles;
  int want = cdiv(1024, tiles);
  const size_t cap = (size_t)160 << 20;
  int by_ws = (int)(cap / (slab ? slab : 1));
  if (by_ws < 1) by_ws = 1;
  int s = want < by_ws ? want : by_ws;
  if (s > p.mtiles) s = p.mtiles;
  if (s < 1) s = 1;
  p.per_split = cdiv(p.mtiles, s);
  p.splits = cdiv(p.mtiles, p.per_split);
  p.ws_bytes = slab * p.splits;
  return p;
}

template <typename T, int KS>
static int launch_wgrad(const unet_wgrad_desc* d, hipStream_t st) {
  WgPlan p = wg_plan(d);
  float* ws = (float*)d->workspace;
  dim3 grid(p.splits, p.ci_tiles, p.co_tiles);
  hipLaunchKernelGGL((wgrad_kernel<T, KS>), grid, dim3(NTHR), 0, st, *d, p.tiles_w, p.tiles_h, p.mtiles,
                     p.per_split, ws);
  int e = check_launch("wgrad");
  if (e) return e;
  const long long total = (long long)d->Cout * d->Cin * KS * KS;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, ws, p.splits, d->Cout, d->Cin, KS * KS,
                     d->dw, d->accum);
  return check_launch("wgrad_reduce");
}

bool wgrad2_eligible(const unet_wgrad_desc* d, size_t* ws_bytes);  // wgrad2.hip
int wgrad2_run(const unet_wgrad_desc* d, hipStream_t st);
bool wgrad5_eligible(const unet_wgrad_desc* d, size_t* ws_bytes);  // wgrad5.hip
int wgrad5_run(const unet_wgrad_desc* d, hipStream_t st);
bool smallcin_wgrad_ok(const unet_wgrad_desc* d);  // smallcin.hip
bool pw_wgrad_ok(const unet_wgrad_desc* d);        // pw.hip
size_t pw_wgrad_ws(const unet_wgrad_desc* d);
int pw_wgrad(const unet_wgrad_desc* d, hipStream_t st);
size_t smallcin_wgrad_ws(const unet_wgrad_desc* d);
bool smallcin_wgrad_is_mfma(const unet_wgrad_desc* d);
int smallcin_wgrad(const unet_wgrad_desc* d, hipStream_t st);

}  // namespace unet

using namespace unet;

extern "C" {

static int validate_src_w(const unet_src& s) {
  if (s.kind < 0 || s.kind > UNET_SRC_UP_PLAIN || !s.data || s.C <= 0) return 0;
  if ((s.kind == UNET_SRC_ACT || s.kind == UNET_SRC_POOL_ACT || s.kind == UNET_SRC_UP_ACT) && (!s.scale || !s.shift))
    return 0;
  if (s.gate_p && !s.gate_ab) return 0;
  return 1;
}

size_t unet_wgrad_workspace(const unet_wgrad_desc* d) {
  size_t b = 0;
  if (unet::smallcin_wgrad_ok(d)) return unet::smallcin_wgrad_ws(d);
  if (unet::pw_wgrad_ok(d)) return unet::pw_wgrad_ws(d);
  if (unet::wgrad5_eligible(d, &b)) return b;
  if (unet::wgrad2_eligible(d, &b)) return b;
  return wg_plan(d).ws_bytes;
}

int unet_wgrad_variant(const unet_wgrad_desc* d, char* buf, int len) {
  if (!d || !buf || len <= 0) return UNET_ERR_ARG;
  const char* tn = d->dtype == UNET_F16 ? "fp16" : d->dtype == UNET_BF16 ? "bf16" : "fp32";
  if (unet::smallcin_wgrad_ok(d))
    snprintf(buf, len, unet::smallcin_wgrad_is_mfma(d) ? "smallcin_wgrad_mfma_kernel<%s>" : "smallcin_wgrad_kernel<%s>", tn);
  else if (unet::pw_wgrad_ok(d)) snprintf(buf, len, "pw_wgrad_kernel<%s>", tn);
  else if (unet::wgrad5_eligible(d, nullptr)) snprintf(buf, len, "wgrad5_kernel<%s>", tn);
  else if (unet::wgrad2_eligible(d, nullptr)) snprintf(buf, len, "wgrad2_kernel<%s,%d>", tn, d->ksize);
  else snprintf(buf, len, "wgrad_kernel<%s,%d>", tn, d->ksize);
  return 0;
}

int unet_conv_wgrad(const unet_wgrad_desc* d, void* stream) {
  if (!d || d->N <= 0 || d->H <= 0 || d->W <= 0 || d->Cin <= 0 || d->Cout <= 0 || !d->dy || !d->dw ||
      !d->workspace || (d->ksize != 1 && d->ksize != 3) || d->nsrc < 1 || d->nsrc > 2) {
    set_error("unet_conv_wgrad: bad descriptor");
    return UNET_ERR_ARG;
  }
  int csum = 0;
  for (int i = 0; i < d->nsrc; ++i) {
    if (!validate_src_w(d->src[i])) { set_error("unet_conv_wgrad: bad source"); return UNET_ERR_ARG; }
    csum += d->src[i].C;
  }
  if (csum != d->Cin) { set_error("unet_conv_wgrad: source channels != Cin"); return UNET_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  if (unet::smallcin_wgrad_ok(d)) return unet::smallcin_wgrad(d, st);
  if (unet::pw_wgrad_ok(d)) return unet::pw_wgrad(d, st);
  if (unet::wgrad5_eligible(d, nullptr)) return unet::wgrad5_run(d, st);
  if (unet::wgrad2_eligible(d, nullptr)) return unet::wgrad2_run(d, st);
  if (d->dtype == UNET_BF16) return d->ksize == 3 ? launch_wgrad<bf16, 3>(d, st) : launch_wgrad<bf16, 1>(d, st);
  if (d->dtype == UNET_F16) return d->ksize == 3 ? launch_wgrad<f16, 3>(d, st) : launch_wgrad<f16, 1>(d, st);
  if (d->dtype == UNET_F32) return d->ksize == 3 ? launch_wgrad<float, 3>(d, st) : launch_wgrad<float, 1>(d, st);
  set_error("unet_conv_wgrad: bad dtype");
  return UNET_ERR_ARG;
}

}  // extern "C"
