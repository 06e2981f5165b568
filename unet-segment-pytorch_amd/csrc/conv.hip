// conv.hip — LDS-halo direct convolution on MFMA for gfx950 (fwd + dgrad) and weight packing.
//
// Replaces nn.Conv2d(k=3, pad=1, bias=False) / nn.Conv2d(k=1, bias=False) of
// unet/models/layers.py:32,35,152,158 and the input-gradient half of their convolution_backward.
//
// One workgroup (WM x WN waves) computes a TH x 16-pixel x BN-channel output tile of one image.
//  * Input ("A"): per 64-byte channel chunk, the (TH+2) x 18 halo is gathered ONCE into LDS and
//    re-used by all 9 taps.  The gather applies the virtual-activation transform of the source
//    (BN-apply+ReLU, 2x2 max-pool, bilinear-up + pad, concat, attention multiply; src_gather.h), and
//    is software-pipelined: the raw loads of chunk c+1 are issued before chunk c's MFMAs and only
//    transformed + written to the second LDS buffer after them (one barrier per chunk).
//  * Weights ("B"): packed fragment-major ([n-tile][chunk][tap][lane][16 B]) so each MFMA operand is
//    one coalesced 1 KiB wave load straight from L2 into VGPRs, prefetched two taps ahead; no LDS.
//  * MFMA: v_mfma_f32_16x16x32_bf16 (bf16) or v_mfma_f32_16x16x4_f32 (exact fp32 parity mode).
//  * Epilogue: y (NHWC) + per-tile BN partial sums, or fp32 gradients (channel split for the concat,
//    or routed through the 2x2 max-pool argmax).
#include <stdio.h>
#include "conv_src16.h"

namespace unet {

constexpr int CTW = 16;          // tile width in pixels

// ------------------------------------------------------------------------------------------------
// epilogue shared by conv2 / conv3.  acc[i][j][r] (lane l): pixel (h0 + MI*wm + i, w0 + 4*(l>>4) + r),
// channel co0 + (wn*NTN + j)*16 + (l&15).  Modes: y + BN partial sums, fp32 (split across the concat,
// optionally accumulated), ConvTranspose2d shuffle, max-pool backward routing.
// OM: the output mode when known at compile time (-1: dispatch on d.out_mode at run time)
template <typename T, int WM, int WN, int NTN, int MI = 4, int OM = -1>
__device__ __forceinline__ void conv_epilogue(const unet_conv_desc& d, f32x4 (&acc)[MI][NTN], T* lds, int tid,
                                              int lane, int wm, int wn, long long n, int h0, int w0, int co0,
                                              int mt, int mtiles) {
  constexpr int BN = WN * NTN * 16;
  // acc[i][j][r] (lane l): pixel (h0 + MI*wm + i, w0 + 4*(l>>4) + r), channel co0 + (wn*NTN + j)*16 + (l&15)
  const int ow_base = w0 + 4 * (lane >> 4);
  auto is = [&](int m) { return OM < 0 ? d.out_mode == m : OM == m; };
  if (is(UNET_OUT_Y)) {
    T* y = (T*)d.out;
    float s[NTN], ss[NTN];
#pragma unroll
    for (int j = 0; j < NTN; ++j) { s[j] = 0.f; ss[j] = 0.f; }
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      const int oh = h0 + wm * MI + i;
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + (wn * NTN + j) * 16 + (lane & 15);
#pragma unroll 4
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) {
            const float val = acc[i][j][r];
            y[((n * d.H + oh) * (long long)d.W + ow) * d.Cout + co] = from_f<T>(val);
            s[j] += val;
            ss[j] += val * val;
          }
        }
      }
    }
    if (d.stats) {
      float* red = reinterpret_cast<float*>(lds);  // [WM][BN][2]
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j) {
        s[j] += __shfl_xor(s[j], 16, 64);
        s[j] += __shfl_xor(s[j], 32, 64);
        ss[j] += __shfl_xor(ss[j], 16, 64);
        ss[j] += __shfl_xor(ss[j], 32, 64);
        if (lane < 16) {
          const int col = (wn * NTN + j) * 16 + lane;
          red[(wm * BN + col) * 2 + 0] = s[j];
          red[(wm * BN + col) * 2 + 1] = ss[j];
        }
      }
      __syncthreads();
      if (tid < BN) {
        const int co = co0 + tid;
        if (co < d.Cout) {
          float a = 0.f, b = 0.f;
#pragma unroll
          for (int w = 0; w < WM; ++w) { a += red[(w * BN + tid) * 2]; b += red[(w * BN + tid) * 2 + 1]; }
          d.stats[(size_t)co * mtiles + mt] = a;
          d.stats[((size_t)d.Cout + co) * mtiles + mt] = b;
        }
      }
    }
  } else if (is(UNET_OUT_F32) && (d.Cout % 4) == 0 && (d.split % 4) == 0) {
    // fp32 gradients: each row of the wave's tile is transposed through a wave-private LDS slice so a
    // lane stores (or read-modify-writes) 4 consecutive channels of one pixel as one 16-byte access,
    // instead of 4-byte accesses strided by the pixel pitch
    float* o1 = (float*)d.out;
    float* o2 = (float*)d.out2;
    const int c2 = d.Cout - d.split;
    constexpr int SW = NTN * 16 + 4;  // staged row pitch in floats (the +4 keeps the writes conflict-free)
    float* stg = reinterpret_cast<float*>(lds) + (wm * WN + wn) * 16 * SW;
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      const int oh = h0 + wm * MI + i;
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j)
#pragma unroll 4
        for (int r = 0; r < 4; ++r) stg[(4 * (lane >> 4) + r) * SW + j * 16 + (lane & 15)] = acc[i][j][r];
#pragma unroll
      for (int k = 0; k < NTN; ++k) {
        const int f = lane + 64 * k;
        const int px = f / (4 * NTN), c4 = f % (4 * NTN);
        const float4 v = *reinterpret_cast<const float4*>(stg + px * SW + c4 * 4);
        const int ow = w0 + px, co = co0 + wn * NTN * 16 + c4 * 4;
        if (oh < d.H && ow < d.W && co < d.Cout) {
          const long long pix = (n * d.H + oh) * (long long)d.W + ow;
          float4* p;
          int acc_in;
          if (co < d.split) { p = reinterpret_cast<float4*>(o1 + pix * d.split + co); acc_in = d.accum; }
          else { p = reinterpret_cast<float4*>(o2 + pix * c2 + (co - d.split)); acc_in = d.accum2; }
          float4 w = v;
          if (acc_in) {
            const float4 a = *p;
            w.x += a.x; w.y += a.y; w.z += a.z; w.w += a.w;
          }
          *p = w;
        }
      }
    }
  } else if (is(UNET_OUT_POOL_BWD) && d.pool_code && (d.Cout % 4) == 0) {
    // max-pool backward through the argmax codes of unet_materialize_pool: the row is transposed through
    // a wave-private LDS slice as in the fp32 path, so a lane owns 4 consecutive channels of one pooled
    // pixel (one 4-byte code load) and adds each channel into the 2x2 source position it selected: all four
    // positions are read-modify-written as 16-byte accesses with per-channel selects (no divergence; the
    // cache lines are touched either way), instead of 4-byte scattered accesses per channel
    const unet_src& ps = d.pool_src;
    float* da = (float*)d.out;
    constexpr int SW = NTN * 16 + 4;
    float* stg = reinterpret_cast<float*>(lds) + (wm * WN + wn) * 16 * SW;
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      const int oh = h0 + wm * MI + i;
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j)
#pragma unroll 4
        for (int r = 0; r < 4; ++r) stg[(4 * (lane >> 4) + r) * SW + j * 16 + (lane & 15)] = acc[i][j][r];
#pragma unroll
      for (int k = 0; k < NTN; ++k) {
        const int f = lane + 64 * k;
        const int px = f / (4 * NTN), c4 = f % (4 * NTN);
        const float4 v = *reinterpret_cast<const float4*>(stg + px * SW + c4 * 4);
        const int ow = w0 + px, co = co0 + wn * NTN * 16 + c4 * 4;
        if (oh < d.H && ow < d.W && co < d.Cout) {
          const long long pix = (n * d.H + oh) * (long long)d.W + ow;
          const unsigned code = *reinterpret_cast<const unsigned*>(d.pool_code + pix * d.Cout + co);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const bool s0 = (code & 0xffu) == (unsigned)q, s1 = ((code >> 8) & 0xffu) == (unsigned)q;
            const bool s2 = ((code >> 16) & 0xffu) == (unsigned)q, s3 = (code >> 24) == (unsigned)q;
            const long long sp = (n * ps.H + 2 * oh + (q >> 1)) * (long long)ps.W + 2 * ow + (q & 1);
            float4* p = reinterpret_cast<float4*>(da + sp * d.Cout + co);
            float4 a = *p;
            a.x = s0 ? a.x + v.x : a.x;
            a.y = s1 ? a.y + v.y : a.y;
            a.z = s2 ? a.z + v.z : a.z;
            a.w = s3 ? a.w + v.w : a.w;
            *p = a;
          }
        }
      }
    }
  } else if (is(UNET_OUT_F32)) {
    float* o1 = (float*)d.out;
    float* o2 = (float*)d.out2;
    const int c2 = d.Cout - d.split;
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      const int oh = h0 + wm * MI + i;
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + (wn * NTN + j) * 16 + (lane & 15);
#pragma unroll 4
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) {
            const long long pix = (n * d.H + oh) * (long long)d.W + ow;
            const float val = acc[i][j][r];
            if (co < d.split) {
              float* p = o1 + pix * d.split + co;
              *p = d.accum ? *p + val : val;
            } else {
              float* p = o2 + pix * c2 + (co - d.split);
              *p = d.accum2 ? *p + val : val;
            }
          }
        }
      }
    }
  } else if (is(UNET_OUT_SHUFFLE2)) {
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      const int oh = h0 + wm * MI + i;
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + (wn * NTN + j) * 16 + (lane & 15);
#pragma unroll 4
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) store_shuffle2<T>(d, n, oh, ow, co, acc[i][j][r]);
        }
      }
    }
  } else if (!is(UNET_OUT_POOL_BWD)) {
  } else if (d.pool_code) {  // UNET_OUT_POOL_BWD with the argmax recorded by unet_materialize_pool
    const unet_src& ps = d.pool_src;
    float* da = (float*)d.out;
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      const int oh = h0 + wm * MI + i;
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + (wn * NTN + j) * 16 + (lane & 15);
#pragma unroll 4
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) {
            const int bq = d.pool_code[((n * d.H + oh) * (long long)d.W + ow) * d.Cout + co];
            const long long sp = (n * ps.H + 2 * oh + (bq >> 1)) * (long long)ps.W + 2 * ow + (bq & 1);
            da[sp * d.Cout + co] += acc[i][j][r];
          }
        }
      }
    }
  } else {  // UNET_OUT_POOL_BWD
    const unet_src& ps = d.pool_src;
    float* da = (float*)d.out;
    const T* ysrc = (const T*)ps.data;
#pragma unroll MI
    for (int i = 0; i < MI; ++i) {
      const int oh = h0 + wm * MI + i;
#pragma unroll NTN
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + (wn * NTN + j) * 16 + (lane & 15);
#pragma unroll 4
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) {
            const float scv = ps.scale[co], sfv = ps.shift[co];
            float best = -INFINITY;
            int bq = 0;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const long long sp = (n * ps.H + 2 * oh + (q >> 1)) * (long long)ps.W + 2 * ow + (q & 1);
              float a = to_f(ysrc[sp * d.Cout + co]) * scv + sfv;
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

// ------------------------------------------------------------------------------------------------
template <typename T, int KS, int WM, int WN, int NTN, int RAW>
__global__ __launch_bounds__(64 * WM * WN) void conv2_kernel(const unet_conv_desc d, int tiles_w, int tiles_h,
                                                             int mtiles, int nchunks) {
  using M = Mma<T>;
  constexpr int NT = 64 * WM * WN;
  constexpr int KC = M::KC, VEC = Vec<T>::N, NV = KC / VEC;
  constexpr int TH = 4 * WM, BN = WN * NTN * 16;
  constexpr int HALO = (KS == 3) ? 1 : 0;
  constexpr int HWID = CTW + 2 * HALO, HHGT = TH + 2 * HALO, HP = HWID * HHGT;
  // 96-byte LDS rows (24 dwords): the 16 lanes of a ds_read_b128 phase (4 rows x 4 k-groups) hit
  // distinct bank quads for any row base, so the A reads are conflict-free
  constexpr int RS = KC + 32 / (int)sizeof(T);
  constexpr int TAPS = KS * KS;
  constexpr int ITEMS = (HP * NV + NT - 1) / NT;
  constexpr int E16 = 16 / (int)sizeof(T);
  static_assert(NT % NV == 0, "thread->channel-vector mapping must be fixed");
  __shared__ __attribute__((aligned(16))) T lds[2 * HP * RS];
  static_assert(2 * HP * RS * sizeof(T) >= (size_t)(WM * WN) * 16 * (NTN * 16 + 4) * 4, "fp32 epilogue staging");

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int mt = blockIdx.x;
  const int tw_i = mt % tiles_w;
  const int t2 = mt / tiles_w;
  const int th_i = t2 % tiles_h;
  const long long n = t2 / tiles_h;
  const int h0 = th_i * TH, w0 = tw_i * CTW;
  const int co0 = blockIdx.y * BN;

  // this thread's halo items: item k covers halo vector (tid + k*NT); its channel vector v is the same
  // for every k and every chunk (NT % NV == 0)
  const int v = tid % NV;
  auto item_hp = [&](int k) { return (tid + k * NT) / NV; };
  auto item_y = [&](int k) { return h0 + item_hp(k) / HWID - HALO; };
  auto item_x = [&](int k) { return w0 + item_hp(k) % HWID - HALO; };

  // weight fragments: [ntile][chunk][tap][lane][16B]
  // (uniform byte base of this wave's first n-tile) + (uniform 32-bit offset) + lane * 16
  const int ntile0 = co0 / 16 + wn * NTN;
  const char* wsb = reinterpret_cast<const char*>(d.weight) + (size_t)ntile0 * nchunks * TAPS * 1024;
  const unsigned jstride = (unsigned)nchunks * TAPS * 1024u;
  const unsigned lane16 = (unsigned)lane * 16u;
  auto bptr = [&](int j, int c, int t) -> const uint4* {
    return reinterpret_cast<const uint4*>(wsb + (j * jstride + (unsigned)(c * TAPS + t) * 1024u + lane16));
  };

  f32x4 acc[4][NTN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NTN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  SrcView sv;
  float sc[VEC], sf[VEC];
  Item<RAW> item;

  // ---- prologue: chunk 0 into buffer 0 ----
  make_view<T>(d, v * VEC, sv, sc, sf);
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int hp = item_hp(k);
    if (hp < HP) {
      item_issue<T, RAW>(sv, d.H, d.W, n, item_y(k), item_x(k), 1, item);
      float vals[VEC];
      item_finish<T, RAW>(d, sv, sc, sf, n, item_y(k), item_x(k), v * VEC, item, vals);
      store_vec<T>(lds + hp * RS + v * VEC, vals);
    }
  }
  uint4 B[2][NTN];
#pragma unroll
  for (int j = 0; j < NTN; ++j) B[0][j] = *bptr(j, 0, 0);
  __syncthreads();

  for (int c = 0; c < nchunks; ++c) {
    const T* xb = lds + (c & 1) * HP * RS;
    T* xn = lds + ((c & 1) ^ 1) * HP * RS;
    const bool has_next = c + 1 < nchunks;
    const int cn = (c + 1) * KC + v * VEC;
    if (has_next) make_view<T>(d, cn, sv, sc, sf);
#pragma unroll
    for (int t = 0; t < TAPS; ++t) {
      // B fragments one tap ahead (crossing into the next chunk)
      const int tt = t + 1;
      if (tt < TAPS) {
#pragma unroll
        for (int j = 0; j < NTN; ++j) B[tt & 1][j] = *bptr(j, c, tt);
      } else if (has_next) {
#pragma unroll
        for (int j = 0; j < NTN; ++j) B[tt & 1][j] = *bptr(j, c + 1, tt - TAPS);
      }
      // next chunk's halo: item k issued at tap 3k, finished (transform + LDS write) at tap 3k+2
      if constexpr (TAPS == 9) {
        if (has_next && t % 3 == 0 && t / 3 < ITEMS) {
          const int k = t / 3;
          item_issue<T, RAW>(sv, d.H, d.W, n, item_y(k), item_x(k), item_hp(k) < HP, item);
        }
      }
      const int dy = t / KS, dx = t % KS;
#pragma unroll
      for (int ks = 0; ks < KC / M::KSTEP; ++ks) {
        typename M::frag a[4];
        const int kofs = ks * M::KSTEP + (lane >> 4) * M::E;
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = M::load(xb + ((wm * 4 + i + dy) * HWID + (lane & 15) + dx) * RS + kofs);
#pragma unroll
        for (int j = 0; j < NTN; ++j) {
          typename M::frag b;
          const uint4 q = B[t & 1][j];
          if constexpr (sizeof(T) == 2) b = __builtin_bit_cast(typename M::frag, q);
          else b = __uint_as_float(ks == 0 ? q.x : ks == 1 ? q.y : ks == 2 ? q.z : q.w);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = M::mma(a[i], b, acc[i][j]);
        }
      }
      if constexpr (TAPS == 9) {
        if (has_next && t % 3 == 2 && t / 3 < ITEMS) {
          const int k = t / 3;
          const int hp = item_hp(k);
          if (hp < HP) {
            float vals[VEC];
            item_finish<T, RAW>(d, sv, sc, sf, n, item_y(k), item_x(k), cn, item, vals);
            store_vec<T>(xn + hp * RS + v * VEC, vals);
          }
        }
      }
    }
    // TAPS is odd: the next chunk's tap-0 fragments were prefetched into slot 1
    if (has_next) {
#pragma unroll
      for (int j = 0; j < NTN; ++j) B[0][j] = B[1][j];
    }
    if constexpr (TAPS == 1) {
      if (has_next) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
          const int hp = item_hp(k);
          if (hp < HP) {
            item_issue<T, RAW>(sv, d.H, d.W, n, item_y(k), item_x(k), 1, item);
            float vals[VEC];
            item_finish<T, RAW>(d, sv, sc, sf, n, item_y(k), item_x(k), cn, item, vals);
            store_vec<T>(xn + hp * RS + v * VEC, vals);
          }
        }
      }
    }
    __syncthreads();
  }

  conv_epilogue<T, WM, WN, NTN>(d, acc, lds, tid, lane, wm, wn, n, h0, w0, co0, mt, mtiles);
}

// ------------------------------------------------------------------------------------------------
// configuration choice (host)
// ------------------------------------------------------------------------------------------------
struct ConvCfg {
  int wm, wn, ntn, raw;
  const char* name;
  int w4;  // bf16 3x3, plain/act sources: 4-wave 8-row conv3 tile with 8-row waves (two workgroups per CU)
};

// UNET_CONV3_TILE=16 restores the 8-wave 16-row conv3 tiles (one workgroup per CU) for comparison
static bool conv3_w4_enabled() {
  static const int v = [] {
    const char* e = getenv("UNET_CONV3_TILE");
    return (e && atoi(e) == 16) ? 0 : 1;
  }();
  return v != 0;
}

static ConvCfg pick_cfg(const unet_conv_desc* d) {
  ConvCfg c;
  c.raw = 1;
  for (int i = 0; i < d->nsrc; ++i)
    if (d->src[i].kind == UNET_SRC_POOL_ACT || d->src[i].kind == UNET_SRC_UP_ACT) c.raw = 4;
  c.w4 = 0;
  const long long tiles16 = (long long)d->N * cdiv(d->H, 16) * cdiv(d->W, CTW);
  // 8-row 4-wave conv3 tiles: same 8-row x 16-px x 8-rows-per-wave MFMA work per wave as the 16-row
  // 8-wave tile, but two independent workgroups share a CU, so one's barrier / staging / epilogue runs
  // under the other's MFMAs
  // (measured: faster for the y epilogue; the fp32 dgrad and pool-routing epilogues spill in the 4-wave
  // tile and keep the 16-row one)
  const bool w4 = conv3_w4_enabled() && d->dtype != UNET_F32 && d->ksize == 3 && c.raw == 1 &&
                  d->out_mode == UNET_OUT_Y;
  if (d->Cout <= 32) {
    c.wm = 2; c.wn = 2; c.ntn = 1;
  } else if (d->Cout <= 64) {
    if (tiles16 >= 256 && w4) { c.wm = 2; c.wn = 2; c.ntn = 2; c.w4 = 1; }
    else if (tiles16 >= 256) { c.wm = 4; c.wn = 2; c.ntn = 2; }
    else { c.wm = 2; c.wn = 2; c.ntn = 2; }
  } else {
    if (c.raw == 1 && tiles16 * cdiv(d->Cout, 128) >= 256 && w4) { c.wm = 2; c.wn = 2; c.ntn = 4; c.w4 = 1; }
    else if (c.raw == 1 && tiles16 * cdiv(d->Cout, 128) >= 256) { c.wm = 4; c.wn = 2; c.ntn = 4; }
    else if ((long long)d->N * cdiv(d->H, 8) * cdiv(d->W, CTW) * cdiv(d->Cout, 128) < 256) {
      c.wm = 2; c.wn = 2; c.ntn = 2;  // small maps (32^2 x bs4): 64-channel tiles, twice the workgroups
    }
    else { c.wm = 2; c.wn = 4; c.ntn = 2; }
  }
  return c;
}

template <typename T, int KS, int WM, int WN, int NTN, int RAW>
static int launch_conv2(const unet_conv_desc* d, hipStream_t st) {
  constexpr int TH = 4 * WM, BN = WN * NTN * 16;
  const int tw = cdiv(d->W, CTW), th = cdiv(d->H, TH);
  const int mt = d->N * tw * th;
  const int kc = Mma<T>::KC;
  dim3 grid(mt, cdiv(d->Cout, BN));
  hipLaunchKernelGGL((conv2_kernel<T, KS, WM, WN, NTN, RAW>), grid, dim3(64 * WM * WN), 0, st, *d, tw, th, mt,
                     cdiv(d->Cin, kc));
  return check_launch("conv");
}

template <typename T, int KS, int RAW>
static int dispatch_cfg(const unet_conv_desc* d, const ConvCfg& c, hipStream_t st) {
  if (c.wm == 2 && c.wn == 2 && c.ntn == 1) return launch_conv2<T, KS, 2, 2, 1, RAW>(d, st);
  if (c.wm == 4 && c.wn == 2 && c.ntn == 2) return launch_conv2<T, KS, 4, 2, 2, RAW>(d, st);
  if (c.wm == 2 && c.wn == 2 && c.ntn == 2) return launch_conv2<T, KS, 2, 2, 2, RAW>(d, st);
  if (c.wm == 4 && c.wn == 2 && c.ntn == 4) return launch_conv2<T, KS, 4, 2, 4, RAW>(d, st);
  return launch_conv2<T, KS, 2, 4, 2, RAW>(d, st);
}

#include "conv3_body.inc"

template <typename T> int dispatch_generic(const unet_conv_desc* d, hipStream_t st);
bool conv5_eligible(const unet_conv_desc* d);   // conv5.hip: the LDS-DMA 3x3 path
bool conv5_serves(const unet_conv_desc* d);     // conv5.hip: eligible, or small enough for its split-K form
size_t conv5_workspace(const unet_conv_desc* d);
bool conv5_act_out_ok(const unet_conv_desc* d);
int pack_tiles_launch(int dtype, int count, const unet_pack_job* jobs, hipStream_t st);   // pack.hip
int conv5_run(const unet_conv_desc* d, hipStream_t st);
int conv5_stats_rows(const unet_conv_desc* d);
int conv5_variant(const unet_conv_desc* d, char* buf, int len);
bool smallcin_conv_ok(const unet_conv_desc* d);  // smallcin.hip
bool pw_conv_ok(const unet_conv_desc* d);        // pw.hip
int pw_conv_rows(const unet_conv_desc* d);
int pw_conv(const unet_conv_desc* d, hipStream_t st);
int pw_conv_variant(const unet_conv_desc* d, char* buf, int len);
int smallcin_rows(long long P);
int smallcin_stats_rows(const unet_conv_desc* d);
bool smallcin_is_mfma(const unet_conv_desc* d);
int smallcin_conv(const unet_conv_desc* d, hipStream_t st);

// the pipelined kernel needs every source channel vector to be one aligned 16-byte load, and every
// source tensor addressable with 32-bit byte offsets
static bool fast_eligible(const unet_conv_desc* d) {
  const int vec = d->dtype != UNET_F32 ? 8 : 4;
  const int es = d->dtype != UNET_F32 ? 2 : 4;
  for (int i = 0; i < d->nsrc; ++i) {
    const unet_src& s = d->src[i];
    if (s.kind == UNET_SRC_NCHW_F32 || s.C % vec) return false;
    if ((double)d->N * s.H * s.W * s.C * es >= 4294967296.0) return false;
  }
  return true;
}

template <typename T>
static int dispatch_conv(const unet_conv_desc* d, hipStream_t st) {
  if (!fast_eligible(d)) return dispatch_generic<T>(d, st);
  if constexpr (sizeof(T) == 2) {
    if (conv5_serves(d)) return conv5_run(d, st);
  }
  const ConvCfg c = pick_cfg(d);
  if constexpr (sizeof(T) == 2) {
    if (conv3_eligible(d)) return dispatch_conv3<T>(d, c, st);
  }
  if (d->ksize == 3) return c.raw == 4 ? dispatch_cfg<T, 3, 4>(d, c, st) : dispatch_cfg<T, 3, 1>(d, c, st);
  return c.raw == 4 ? dispatch_cfg<T, 1, 4>(d, c, st) : dispatch_cfg<T, 1, 1>(d, c, st);
}

// ------------------------------------------------------------------------------------------------
// weight packing: OIHW fp32 -> fragment-major [Npad/16][nchunks][taps][64][16 B]
//   transpose=0: rows = Cout, reduction = Cin (forward);
//   transpose=1: rows = Cin, reduction = Cout, taps flipped 180 degrees (dgrad)
// ------------------------------------------------------------------------------------------------
// one 16-byte unit of the packed layout (E16 consecutive K elements of one lane's fragment) per thread:
// the E16 source values are gathered (L2-resident OIHW rows) and written with a single vector store
template <typename T>
__device__ __forceinline__ void pack_unit(const float* w, T* out, int Cout, int Cin, int taps, int transpose,
                                          int nchunks, long long u) {
  constexpr int KC = Mma<T>::KC, E16 = 16 / (int)sizeof(T);
  const int rows = transpose ? Cin : Cout;
  const int cols = transpose ? Cout : Cin;
  const int lane = (int)(u % 64);
  long long t = u / 64;
  const int tap = (int)(t % taps);
  t /= taps;
  const int chunk = (int)(t % nchunks);
  const int ntile = (int)(t / nchunks);
  const int r = ntile * 16 + (lane & 15);
  float v[E16];
#pragma unroll
  for (int el = 0; el < E16; ++el) {
    const int k = (sizeof(T) == 2) ? 8 * (lane >> 4) + el : 4 * el + (lane >> 4);
    const int cc = chunk * KC + k;
    v[el] = 0.f;
    if (r < rows && cc < cols)
      v[el] = !transpose ? w[((long long)r * Cin + cc) * taps + tap] : w[((long long)cc * Cin + r) * taps + (taps - 1 - tap)];
  }
  store_vec<T>(out + u * E16, v);
}

template <typename T>
__global__ void pack_kernel(const float* w, T* out, int Cout, int Cin, int ks, int transpose, int rows_pad,
                            int nchunks) {
  constexpr int KC = Mma<T>::KC, E16 = 16 / (int)sizeof(T);
  const int taps = ks * ks;
  const long long units = (long long)rows_pad * nchunks * KC * taps / E16;
  for (long long u = blockIdx.x * (long long)blockDim.x + threadIdx.x; u < units; u += (long long)gridDim.x * blockDim.x)
    pack_unit<T>(w, out, Cout, Cin, taps, transpose, nchunks, u);
}

// many weights in one launch: job table passed by value in the kernel arguments; blockIdx.y = job
struct PackJobs {
  unet_pack_job j[UNET_PACK_MAX_JOBS];
};

template <typename T>
__global__ void pack_many_kernel(const PackJobs jobs) {
  const unet_pack_job& jb = jobs.j[blockIdx.y];
  constexpr int KC = Mma<T>::KC, E16 = 16 / (int)sizeof(T);
  const int taps = jb.ksize * jb.ksize;
  const int rows = jb.transpose ? jb.Cin : jb.Cout;
  const int cols = jb.transpose ? jb.Cout : jb.Cin;
  const int rows_pad = (rows + PACK_NPAD - 1) / PACK_NPAD * PACK_NPAD;
  const int nchunks = (cols + KC - 1) / KC;
  const long long units = (long long)rows_pad * nchunks * KC * taps / E16;
  for (long long u = blockIdx.x * (long long)blockDim.x + threadIdx.x; u < units; u += (long long)gridDim.x * blockDim.x)
    pack_unit<T>(jb.w, (T*)jb.packed, jb.Cout, jb.Cin, taps, jb.transpose, nchunks, u);
}

static int packed_rows(int Cout, int Cin, int transpose) {
  return round_up(transpose ? Cin : Cout, PACK_NPAD);
}

}  // namespace unet

using namespace unet;

extern "C" {

static const char* tname(int dtype) { return dtype == UNET_BF16 ? "bf16" : dtype == UNET_F16 ? "fp16" : "fp32"; }

int unet_conv_mtiles(int N, int H, int W) { return N * cdiv(W, CTW) * cdiv(H, 8); }

// does unet_conv reduce d's bnb_* sums in the conv epilogue (rows = the conv's M tiles)?
static bool bnb_in_epilogue(const unet_conv_desc* d) {
  if (smallcin_conv_ok(d) || pw_conv_ok(d) || !fast_eligible(d) || d->dtype == UNET_F32) return false;
  if (conv5_serves(d)) return true;
  return conv3_bnb_tile(d, pick_cfg(d));
}

int unet_conv_stats_rows(const unet_conv_desc* d) {
  if (d->bnb_y && !bnb_in_epilogue(d)) return unet_bn_bwd_reduce_rows((long long)d->N * d->H * d->W, d->Cout);
  if (smallcin_conv_ok(d)) return smallcin_stats_rows(d);
  if (pw_conv_ok(d)) return pw_conv_rows(d);
  if (!fast_eligible(d)) return d->N * cdiv(d->W, CTW) * cdiv(d->H, 8);
  if (d->dtype != UNET_F32 && conv5_serves(d)) return conv5_stats_rows(d);
  const ConvCfg c = pick_cfg(d);
  return d->N * cdiv(d->W, CTW) * cdiv(d->H, 4 * c.wm);
}

size_t unet_conv_workspace(const unet_conv_desc* d) {
  if (!d || smallcin_conv_ok(d) || pw_conv_ok(d) || !fast_eligible(d) || d->dtype == UNET_F32) return 0;
  return conv5_workspace(d);
}

int unet_conv_act_out_ok(const unet_conv_desc* d) { return d && conv5_act_out_ok(d) ? 1 : 0; }

int unet_conv_variant(const unet_conv_desc* d, char* buf, int len) {
  if (smallcin_conv_ok(d)) {
    snprintf(buf, len, smallcin_is_mfma(d) ? "smallcin_fwd_mfma_kernel<%s>" : "smallcin_fwd_kernel<%s>", tname(d->dtype));
    return 0;
  }
  if (pw_conv_ok(d)) return pw_conv_variant(d, buf, len);
  if (!fast_eligible(d)) {
    snprintf(buf, len, "conv_generic_kernel<%s,%d,%d>", tname(d->dtype), d->ksize,
             d->Cout <= 32 ? 32 : 64);
    return 0;
  }
  if (d->dtype != UNET_F32 && conv5_serves(d)) return conv5_variant(d, buf, len);
  const ConvCfg c = pick_cfg(d);
  if (conv3_eligible(d)) {
    // the (wm, wn, ntn) block tile of pick_cfg; 16-row tiles run as MI=8 waves (dispatch_conv3)
    if (c.w4) {
      snprintf(buf, len, "conv3_kernel<%s,3,1,4,%d,8,1>", tname(d->dtype), c.ntn / 2);
      return 0;
    }
    const bool mi8 = c.raw == 1 && c.wm == 4 && (c.ntn == 4 || c.ntn == 2);
    snprintf(buf, len, "conv3_kernel<%s,3,%d,%d,%d,%d,%d>", tname(d->dtype), mi8 ? 2 : c.wm, mi8 ? 4 : c.wn, mi8 ? c.ntn / 2 : c.ntn,
             mi8 ? 8 : 4, c.raw);
    return 0;
  }
  snprintf(buf, len, "conv2_kernel<%s,%d,%d,%d,%d,%d>", tname(d->dtype), d->ksize, c.wm, c.wn,
           c.ntn, c.raw);
  return 0;
}

int unet_pack_weights(int dtype, int count, const unet_pack_job* jobs, void* stream) {
  if (count < 0 || count > UNET_PACK_MAX_JOBS || (count && !jobs)) {
    set_error("unet_pack_weights: bad job count");
    return UNET_ERR_ARG;
  }
  if (count == 0) return 0;
  PackJobs pj;
  long long maxe = 0;
  for (int i = 0; i < count; ++i) {
    pj.j[i] = jobs[i];
    const unet_pack_job& j = jobs[i];
    if (!j.w || !j.packed || j.Cout <= 0 || j.Cin <= 0 || (j.ksize != 1 && j.ksize != 3)) {
      set_error("unet_pack_weights: bad job");
      return UNET_ERR_ARG;
    }
    const long long e = unet_packed_weight_elems(dtype, j.Cout, j.Cin, j.ksize, j.transpose);
    if (e > maxe) maxe = e;
  }
  if (dtype != UNET_F32) return pack_tiles_launch(dtype, count, jobs, (hipStream_t)stream);   // pack.hip
  const long long maxu = maxe / (dtype != UNET_F32 ? 8 : 4);   // 16-byte units
  int blocks = (int)((maxu + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(pack_many_kernel<f16>, dim3(blocks, count), dim3(256), 0, st, pj);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(pack_many_kernel<bf16>, dim3(blocks, count), dim3(256), 0, st, pj);
  else
    hipLaunchKernelGGL(pack_many_kernel<float>, dim3(blocks, count), dim3(256), 0, st, pj);
  return check_launch("pack_weights");
}

int unet_packed_weight_elems(int dtype, int Cout, int Cin, int ksize, int transpose) {
  const int kc = dtype != UNET_F32 ? 32 : 16;
  const int cols = transpose ? Cout : Cin;
  return packed_rows(Cout, Cin, transpose) * ksize * ksize * round_up(cols, kc);
}

int unet_pack_weight(int dtype, const float* w, void* packed, int Cout, int Cin, int ksize, int transpose,
                     void* stream) {
  hipStream_t st = (hipStream_t)stream;
  const int kc = dtype != UNET_F32 ? 32 : 16;
  const int rows_pad = packed_rows(Cout, Cin, transpose);
  const int nchunks = cdiv(transpose ? Cout : Cin, kc);
  const long long total = (long long)rows_pad * nchunks * kc * ksize * ksize / (dtype != UNET_F32 ? 8 : 4);
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(pack_kernel<f16>, dim3(blocks), dim3(256), 0, st, w, (f16*)packed, Cout, Cin, ksize,
                       transpose, rows_pad, nchunks);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(pack_kernel<bf16>, dim3(blocks), dim3(256), 0, st, w, (bf16*)packed, Cout, Cin, ksize,
                       transpose, rows_pad, nchunks);
  else
    hipLaunchKernelGGL(pack_kernel<float>, dim3(blocks), dim3(256), 0, st, w, (float*)packed, Cout, Cin, ksize,
                       transpose, rows_pad, nchunks);
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
  if (d->out_mode == UNET_OUT_F32_GATED) {
    if (!d->pool_src.data || !d->pool_src.gate_p || !d->pool_src.gate_ab || d->split != d->Cout) {
      set_error("unet_conv: F32_GATED needs pool_src.data / gate_p / gate_ab and split == Cout");
      return UNET_ERR_ARG;
    }
    if (!pw_conv_ok(d)) {
      set_error("unet_conv: F32_GATED is served by the bf16 1x1 path only");
      return UNET_ERR_UNSUPPORTED;
    }
  } else if (d->out_mode < UNET_OUT_Y || d->out_mode > UNET_OUT_SHUFFLE2 ||
      (d->out_mode == UNET_OUT_SHUFFLE2 && (d->Cout % 4 || d->ksize != 1))) {
    set_error("unet_conv: bad out_mode");
    return UNET_ERR_ARG;
  }
  if (d->out_mode == UNET_OUT_POOL_BWD &&
      (!validate_src(d->pool_src) || d->pool_src.H < 2 * d->H || d->pool_src.W < 2 * d->W || d->pool_src.C != d->Cout)) {
    set_error("unet_conv: bad pool_src");
    return UNET_ERR_ARG;
  }
  if (d->bnb_stats && (d->out_mode != UNET_OUT_Y || d->stats || !d->bnb_y || !d->bnb_scale || !d->bnb_shift ||
                       !d->bnb_mean || !d->bnb_invstd)) {
    set_error("unet_conv: bnb_stats needs the y mode, no forward stats and every bnb_* pointer");
    return UNET_ERR_ARG;
  }
  if (d->dtype != UNET_BF16 && d->dtype != UNET_F16 && d->dtype != UNET_F32) {
    set_error("unet_conv: bad dtype");
    return UNET_ERR_ARG;
  }
  if (d->act_out && !conv5_act_out_ok(d)) {
    set_error("unet_conv: act_out is served for y-mode BN-activation sources on the conv5 path only "
              "(ask unet_conv_act_out_ok)");
    return UNET_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if (smallcin_conv_ok(d)) rc = smallcin_conv(d, st);
  else if (pw_conv_ok(d)) rc = pw_conv(d, st);
  else rc = UNET_DISPATCH_T(d->dtype, dispatch_conv<T>(d, st));
  if (rc || !d->bnb_stats || bnb_in_epilogue(d)) return rc;
  // the other paths: the separate BatchNorm-backward reduction over the stored gradient
  return unet_bn_bwd_reduce(d->dtype, d->dtype, (long long)d->N * d->H * d->W, d->Cout, d->out, d->bnb_y,
                            d->bnb_scale, d->bnb_shift, d->bnb_relu, d->bnb_mean, d->bnb_invstd, d->bnb_stats,
                            stream);
}

}  // extern "C"
