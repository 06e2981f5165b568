// conv_generic.hip — fallback convolution for inputs the pipelined kernel (conv.hip) does not take:
// the fp32 NCHW model input (inc.0, Cin = 1 or 3) and channel counts that are not a multiple of the
// 16-byte vector.  Same math and epilogues as conv2_kernel, simpler structure: the (8+2)x18 halo
// and the chunk's weights are staged in LDS through src_gather(), one barrier pair per chunk.
#include "conv_common.h"

namespace unet {

constexpr int TH = 8, TW = 16, BM = TH * TW, NTHR = 256;

template <typename T, int KS, int BN>
__global__ __launch_bounds__(NTHR) void conv_generic_kernel(const unet_conv_desc d, int tiles_w, int tiles_h, int mtiles) {
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
  const int nchunks = (d.Cin + KC - 1) / KC;
  constexpr int E16 = 16 / (int)sizeof(T);

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
      // fragment-major packed weights (conv.hip pack_kernel): gather the KC-slice of row co
      T vals[VEC];
      const int chunk = c0 / KC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const int k = v * VEC + j;  // channel inside the chunk
        const int lanep = (sizeof(T) == 2) ? (k / 8) * 16 + (co & 15) : (k % 4) * 16 + (co & 15);
        const int el = (sizeof(T) == 2) ? k % 8 : k / 4;
        vals[j] = ((const T*)d.weight)[((((size_t)(co / 16) * nchunks + chunk) * TAPS + tap) * 64 + lanep) * E16 + el];
      }
      *reinterpret_cast<uint4*>(lds_w + (tap * BN + col) * RS + v * VEC) = *reinterpret_cast<const uint4*>(vals);
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
          d.stats[(size_t)co * mtiles + mt] = red[tid * 2] + red[(BN + tid) * 2];
          d.stats[((size_t)d.Cout + co) * mtiles + mt] = red[tid * 2 + 1] + red[(BN + tid) * 2 + 1];
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
  } else if (d.out_mode == UNET_OUT_SHUFFLE2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oh = h0 + wm * 4 + i;
#pragma unroll
      for (int j = 0; j < NTN; ++j) {
        const int co = co0 + wn * (BN / 2) + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ow = ow_base + r;
          if (oh < d.H && ow < d.W && co < d.Cout) store_shuffle2<T>(d, n, oh, ow, co, acc[i][j][r]);
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
              float a = __builtin_fmaf(to_f(ysrc[sp * d.Cout + co]), sc, sf);
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
static int launch_generic(const unet_conv_desc* d, hipStream_t st) {
  const int tw = cdiv(d->W, TW), th = cdiv(d->H, TH);
  const int mt = d->N * tw * th;
  dim3 grid(mt, cdiv(d->Cout, BN));
  hipLaunchKernelGGL((conv_generic_kernel<T, KS, BN>), grid, dim3(NTHR), 0, st, *d, tw, th, mt);
  return check_launch("conv");
}

template <typename T>
int dispatch_generic(const unet_conv_desc* d, hipStream_t st) {
  if (d->ksize == 3) {
    if (d->Cout <= 32) return launch_generic<T, 3, 32>(d, st);
    return launch_generic<T, 3, 64>(d, st);
  }
  if (d->Cout <= 32) return launch_generic<T, 1, 32>(d, st);
  return launch_generic<T, 1, 64>(d, st);
}

template int dispatch_generic<bf16>(const unet_conv_desc*, hipStream_t);
template int dispatch_generic<f16>(const unet_conv_desc*, hipStream_t);
template int dispatch_generic<float>(const unet_conv_desc*, hipStream_t);

}  // namespace unet
