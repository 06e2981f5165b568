// conv.hip — LDS-tiled direct convolution on MFMA for gfx950 (fwd + dgrad), weight packing.
//
// Replaces nn.Conv2d(k=3, pad=1, bias=False) / nn.Conv2d(k=1, bias=False) of
// unet/models/layers.py:32,35,152,158 and their input-gradient.  One workgroup computes an
// 8x16-pixel x BN-channel output tile of one image:
//   * the (8+2)x(16+2) input halo for a 64-byte channel chunk is gathered ONCE into LDS through
//     src_gather() (BN-apply+ReLU, max-pool, bilinear-up, pad, concat and attention multiply are
//     applied on the way in), and re-used by all 9 taps;
//   * the packed weights of the chunk ([tap][co][ci], 64-B rows) are staged next to it;
//   * 4 waves (2 x 2) run v_mfma_f32_16x16x32_bf16 (bf16) or v_mfma_f32_16x16x4_f32 (exact fp32
//     parity mode) over taps x chunk;
//   * the epilogue stores y NHWC and per-tile BN partial sums (train-mode BatchNorm stats), or, for
//     dgrad, fp32 gradients (optionally split across a channel concat, or routed through the 2x2
//     max-pool argmax).
#include "src_gather.h"

namespace unet {

constexpr int TH = 8, TW = 16, BM = TH * TW, NTHR = 256;

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static constexpr int KC = 32;     // channels per staged chunk (64 bytes)
  static constexpr int KSTEP = 32;  // K of one MFMA
  static constexpr int E = 8;       // operand elements per lane
  typedef bf16x8 frag;
  __device__ static __forceinline__ frag load(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
  __device__ static __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static constexpr int KC = 16;
  static constexpr int KSTEP = 4;
  static constexpr int E = 1;
  typedef float frag;
  __device__ static __forceinline__ frag load(const float* p) { return *p; }
  __device__ static __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
};

template <typename T> __host__ __device__ constexpr int kc_of() { return sizeof(T) == 2 ? 32 : 16; }
static inline int round_up(int a, int b) { return (a + b - 1) / b * b; }
__device__ __forceinline__ int round_up_d(int a, int b) { return (a + b - 1) / b * b; }

// ------------------------------------------------------------------------------------------------
// forward / dgrad kernel
// ------------------------------------------------------------------------------------------------
template <typename T, int KS, int BN>
__global__ __launch_bounds__(NTHR) void conv_kernel(const unet_conv_desc d, int tiles_w, int tiles_h, int mtiles) {
  using M = Mma<T>;
  constexpr int KC = M::KC, VEC = Vec<T>::N, NV = KC / VEC;
  constexpr int HALO = (KS == 3) ? 1 : 0;
  constexpr int HWID = TW + 2 * HALO, HHGT = TH + 2 * HALO, HP = HWID * HHGT;
  constexpr int RS = KC + 16 / (int)sizeof(T);  // padded LDS row (elements): 80 bytes
  constexpr int TAPS = KS * KS;
  constexpr int NTN = BN / 32;                  // 16-wide n-tiles per wave (2 waves along N)
  __shared__ __attribute__((aligned(16))) T lds[(HP + TAPS * BN) * RS];
  T* lds_x = lds;
  T* lds_w = lds + HP * RS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int mt = blockIdx.x;
  const int tw_i = mt % tiles_w;
  const int t2 = mt / tiles_w;
  const int th_i = t2 % tiles_h;
  const long long n = t2 / tiles_h;
  const int h0 = th_i * TH, w0 = tw_i * TW;
  const int co0 = blockIdx.y * BN;
  const int Cin_pad = round_up_d(d.Cin, KC);

  f32x4 acc[4][NTN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c0 = 0; c0 < d.Cin; c0 += KC) {
    // ---- stage the input halo (transformed) ----
    for (int it = tid; it < HP * NV; it += NTHR) {
      const int hp = it / NV, v = it % NV;
      const int hy = h0 + hp / HWID - HALO, hx = w0 + hp % HWID - HALO;
      float vals[VEC];
      src_gather<T>(d.src, d.nsrc, d.Cin, d.H, d.W, n, hy, hx, c0 + v * VEC, vals);
      store_vec<T>(lds_x + hp * RS + v * VEC, vals);
    }
    // ---- stage the packed weights of this chunk ----
    for (int it = tid; it < TAPS * BN * NV; it += NTHR) {
      const int row = it / NV, v = it % NV;
      const int tap = row / BN, col = row % BN;
      const int co = co0 + col;
      uint4 q = make_uint4(0, 0, 0, 0);
      if (co < d.Cout)
        q = *reinterpret_cast<const uint4*>((const T*)d.weight + ((size_t)co * TAPS + tap) * Cin_pad + c0 + v * VEC);
      *reinterpret_cast<uint4*>(lds_w + (tap * BN + col) * RS + v * VEC) = q;
    }
    __syncthreads();
#pragma unroll
    for (int tap = 0; tap < TAPS; ++tap) {
      const int dy = tap / KS, dx = tap % KS;
#pragma unroll
      for (int ks = 0; ks < KC / M::KSTEP; ++ks) {
        const int kofs = ks * M::KSTEP + (lane >> 4) * M::E;
        typename M::frag a[4], b[NTN];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = M::load(lds_x + ((wm * 4 + i + dy) * HWID + (lane & 15) + dx) * RS + kofs);
#pragma unroll
        for (int j = 0; j < NTN; ++j) b[j] = M::load(lds_w + (tap * BN + wn * (BN / 2) + j * 16 + (lane & 15)) * RS + kofs);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NTN; ++j) acc[i][j] = M::mma(a[i], b[j], acc[i][j]);
      }
    }
    __syncthreads();
  }

  // ---- epilogue ----
  // acc[i][j][r] (lane l): pixel (h0 + 4*wm + i, w0 + 4*(l>>4) + r), channel co0 + wn*BN/2 + 16j + (l&15)
  const int ow_base = w0 + 4 * (lane >> 4);
  if (d.out_mode == UNET_OUT_Y) {
    T* y = (T*)d.out;
    float s[NTN], ss[NTN];
#pragma unroll
    for (int j = 0; j < NTN; ++j) { s[j] = 0.f; ss[j] = 0.f; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oh = h0 + wm * 4 + i;
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) {
            const float v = acc[i][j][r];
            const T tv = from_f<T>(v);
            y[((n * d.H + oh) * (long long)d.W + ow) * d.Cout + co] = tv;
            s[j] += v;
            ss[j] += v * v;
          }
        }
      }
    }
    if (d.stats) {
      float* red = reinterpret_cast<float*>(lds);  // [2 wm][BN][2]
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        s[j] += __shfl_xor(s[j], 16, 64);
        s[j] += __shfl_xor(s[j], 32, 64);
        ss[j] += __shfl_xor(ss[j], 16, 64);
        ss[j] += __shfl_xor(ss[j], 32, 64);
        if (lane < 16) {
          const int col = wn * (BN / 2) + j * 16 + lane;
          red[(wm * BN + col) * 2 + 0] = s[j];
          red[(wm * BN + col) * 2 + 1] = ss[j];
        }
      }
      __syncthreads();
      if (tid < BN) {
        const int co = co0 + tid;
        if (co < d.Cout) {
          d.stats[(size_t)mt * d.Cout + co] = red[tid * 2] + red[(BN + tid) * 2];
          d.stats[((size_t)mtiles + mt) * d.Cout + co] = red[tid * 2 + 1] + red[(BN + tid) * 2 + 1];
        }
      }
    }
  } else if (d.out_mode == UNET_OUT_F32) {
    float* o1 = (float*)d.out;
    float* o2 = (float*)d.out2;
    const int c2 = d.Cout - d.split;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oh = h0 + wm * 4 + i;
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) {
            const long long pix = (n * d.H + oh) * (long long)d.W + ow;
            const float v = acc[i][j][r];
            if (co < d.split) {
              float* p = o1 + pix * d.split + co;
              *p = d.accum ? *p + v : v;
            } else {
              float* p = o2 + pix * c2 + (co - d.split);
              *p = d.accum2 ? *p + v : v;
            }
          }
        }
      }
    }
  } else {  // UNET_OUT_POOL_BWD: gradient w.r.t. the pooled map -> 2x2 argmax of ACT(pool_src)
    const unet_src& ps = d.pool_src;
    float* da = (float*)d.out;
    const T* ysrc = (const T*)ps.data;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oh = h0 + wm * 4 + i;
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) {
            const float sc = ps.scale[co], sf = ps.shift[co];
            float best = -INFINITY;
            int bq = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const long long sp = (n * ps.H + 2 * oh + (q >> 1)) * (long long)ps.W + 2 * ow + (q & 1);
              float a = to_f(ysrc[sp * d.Cout + co]) * sc + sf;
              if (ps.relu) a = fmaxf(a, 0.f);
              if (a > best || a != a) { best = a; bq = q; }
            }
            const long long sp = (n * ps.H + 2 * oh + (bq >> 1)) * (long long)ps.W + 2 * ow + (bq & 1);
            da[sp * d.Cout + co] += acc[i][j][r];
          }
        }
      }
    }
  }
}

template <typename T, int KS, int BN>
static int launch_conv(const unet_conv_desc* d, hipStream_t st) {
  const int tw = cdiv(d->W, TW), th = cdiv(d->H, TH);
  const int mt = d->N * tw * th;
  dim3 grid(mt, cdiv(d->Cout, BN));
  hipLaunchKernelGGL((conv_kernel<T, KS, BN>), grid, dim3(NTHR), 0, st, *d, tw, th, mt);
  return check_launch("conv");
}

template <typename T>
static int dispatch_conv(const unet_conv_desc* d, hipStream_t st) {
  if (d->ksize == 3) {
    if (d->Cout <= 32) return launch_conv<T, 3, 32>(d, st);
    return launch_conv<T, 3, 64>(d, st);
  }
  if (d->Cout <= 32) return launch_conv<T, 1, 32>(d, st);
  return launch_conv<T, 1, 64>(d, st);
}

// ------------------------------------------------------------------------------------------------
// weight gradient: dW[co][tap][ci] = sum_pix dy[pix][co] * X[pix + tap][ci]
// Split-K over pixel tiles; each block writes an fp32 slab, reduced in a fixed order afterwards.
// ------------------------------------------------------------------------------------------------
constexpr int WG_BCO = 64;

template <typename T> struct WgFrag;
template <> struct WgFrag<bf16> {
  // A/B operand with K on the LDS ROW axis (pixels) and M/N on the column axis (channels):
  // two ds_read_b64_tr_b16 per operand (CDNA4 hardware transpose read).
  static constexpr int KSTEP = 32;
  typedef bf16x8 frag;
  __device__ static __forceinline__ frag tr_load(const bf16* row_q, const bf16* row_q4) {
    i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(row_q));
    i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(row_q4));
    typedef __attribute__((ext_vector_type(8))) short i16x8;
    i16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, r);
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
          a[i] = WgFrag<bf16>::tr_load(lds_d + pr * RSD + m0, lds_d + (pr + 4) * RSD + m0);
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
            b[j] = WgFrag<bf16>::tr_load(lds_x + hp0 * RSX + n0, lds_x + hp1 * RSX + n0);
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
  const int kc = d->dtype == UNET_BF16 ? 32 : 16;
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

// ------------------------------------------------------------------------------------------------
// weight packing: OIHW fp32 -> [Cout][k*k][Cin_pad] (fwd) or [Cin][k*k flipped][Cout_pad] (dgrad)
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void pack_kernel(const float* w, T* out, int Cout, int Cin, int ks, int transpose, int kc) {
  const int taps = ks * ks;
  const int rows = transpose ? Cin : Cout;      // output-channel axis of the packed operand
  const int cols = transpose ? Cout : Cin;      // reduction-channel axis
  const int cols_pad = (cols + kc - 1) / kc * kc;
  const long long total = (long long)rows * taps * cols_pad;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int c = e % cols_pad;
    const long long t = e / cols_pad;
    const int tap = t % taps;
    const int r = t / taps;
    float v = 0.f;
    if (c < cols) {
      if (!transpose) {
        v = w[((long long)r * Cin + c) * taps + tap];                      // w[co=r][ci=c][tap]
      } else {
        const int ftap = taps - 1 - tap;                                 // 180-degree flip
        v = w[((long long)c * Cin + r) * taps + ftap];                     // w[co=c][ci=r][flip(tap)]
      }
    }
    out[e] = from_f<T>(v);
  }
}

}  // namespace unet

using namespace unet;

extern "C" {

int unet_conv_mtiles(int N, int H, int W) { return N * cdiv(W, TW) * cdiv(H, TH); }

int unet_packed_weight_elems(int dtype, int Cout, int Cin, int ksize, int transpose) {
  const int kc = dtype == UNET_BF16 ? 32 : 16;
  const int rows = transpose ? Cin : Cout, cols = transpose ? Cout : Cin;
  return rows * ksize * ksize * round_up(cols, kc);
}

int unet_pack_weight(int dtype, const float* w, void* packed, int Cout, int Cin, int ksize, int transpose,
                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const long long total = unet_packed_weight_elems(dtype, Cout, Cin, ksize, transpose);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (dtype == UNET_BF16)
    hipLaunchKernelGGL(pack_kernel<bf16>, dim3(blocks), dim3(256), 0, st, w, (bf16*)packed, Cout, Cin, ksize,
                       transpose, 32);
  else
    hipLaunchKernelGGL(pack_kernel<float>, dim3(blocks), dim3(256), 0, st, w, (float*)packed, Cout, Cin, ksize,
                       transpose, 16);
  return check_launch("pack_weight");
}

static int validate_src(const unet_src& s) {
  if (s.kind < 0 || s.kind > UNET_SRC_UP_PLAIN || !s.data || s.C <= 0) return 0;
  if ((s.kind == UNET_SRC_ACT || s.kind == UNET_SRC_POOL_ACT || s.kind == UNET_SRC_UP_ACT) && (!s.scale || !s.shift))
    return 0;
  if (s.gate_p && !s.gate_ab) return 0;
  return 1;
}

int unet_conv(const unet_conv_desc* d, void* stream) {
  if (!d || d->N <= 0 || d->H <= 0 || d->W <= 0 || d->Cin <= 0 || d->Cout <= 0 || !d->weight || !d->out ||
      (d->ksize != 1 && d->ksize != 3) || d->nsrc < 1 || d->nsrc > 2) {
    set_error("unet_conv: bad descriptor");
    return UNET_ERR_ARG;
  }
  int csum = 0;
  for (int i = 0; i < d->nsrc; ++i) {
    if (!validate_src(d->src[i])) { set_error("unet_conv: bad source"); return UNET_ERR_ARG; }
    csum += d->src[i].C;
  }
  if (csum != d->Cin) { set_error("unet_conv: source channels != Cin"); return UNET_ERR_ARG; }
  if (d->out_mode == UNET_OUT_F32 && (d->split < 0 || d->split > d->Cout || (d->split < d->Cout && !d->out2))) {
    set_error("unet_conv: bad split");
    return UNET_ERR_ARG;
  }
  if (d->out_mode == UNET_OUT_POOL_BWD &&
      (!validate_src(d->pool_src) || d->pool_src.H < 2 * d->H || d->pool_src.W < 2 * d->W || d->pool_src.C != d->Cout)) {
    set_error("unet_conv: bad pool_src");
    return UNET_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  if (d->dtype == UNET_BF16) return dispatch_conv<bf16>(d, st);
  if (d->dtype == UNET_F32) return dispatch_conv<float>(d, st);
  set_error("unet_conv: bad dtype");
  return UNET_ERR_ARG;
}

size_t unet_wgrad_workspace(const unet_wgrad_desc* d) { return wg_plan(d).ws_bytes; }

int unet_conv_wgrad(const unet_wgrad_desc* d, void* stream) {
  if (!d || d->N <= 0 || d->H <= 0 || d->W <= 0 || d->Cin <= 0 || d->Cout <= 0 || !d->dy || !d->dw ||
      !d->workspace || (d->ksize != 1 && d->ksize != 3) || d->nsrc < 1 || d->nsrc > 2) {
    set_error("unet_conv_wgrad: bad descriptor");
    return UNET_ERR_ARG;
  }
  int csum = 0;
  for (int i = 0; i < d->nsrc; ++i) {
    if (!validate_src(d->src[i])) { set_error("unet_conv_wgrad: bad source"); return UNET_ERR_ARG; }
    csum += d->src[i].C;
  }
  if (csum != d->Cin) { set_error("unet_conv_wgrad: source channels != Cin"); return UNET_ERR_ARG; }
  hipStream_t st = (hipStream_t)stream;
  if (d->dtype == UNET_BF16) return d->ksize == 3 ? launch_wgrad<bf16, 3>(d, st) : launch_wgrad<bf16, 1>(d, st);
  if (d->dtype == UNET_F32) return d->ksize == 3 ? launch_wgrad<float, 3>(d, st) : launch_wgrad<float, 1>(d, st);
  set_error("unet_conv_wgrad: bad dtype");
  return UNET_ERR_ARG;
}

}  // extern "C"
