// smallcin.hip — the network's first convolution (inc.0: nn.Conv2d(n_channels<=4 -> 64, 3x3),
// unet/models/layers.py:32 via unet.py:152) reading the fp32 NCHW model input directly.
//
// With 1-3 input channels the layer is pure streaming (K = 9..27): a 64-wide MFMA tile would be >90 %
// zero padding.  Forward: one thread computes 8 output channels of one pixel with VALU FMAs from
// L1-cached input taps and writes them as one 16-byte vector, plus BN partial sums.  Weight
// gradient: per-thread 8 x (9*Cin) partial sums over a pixel range, reduced across the block, one
// fp32 row per block; unet_colsum finishes (fixed order).
#include "common.h"

namespace unet {

constexpr int SC_ROWS_MAX = 1024;
constexpr int SC_MAXK = 36;  // 9 taps x 4 channels
constexpr int SC_U = 4;      // pixels per trip of the 1-channel forward loop

int smallcin_rows(long long P) {
  long long r = (P + 1023) / 1024;
  if (r > SC_ROWS_MAX) r = SC_ROWS_MAX;
  if (r < 1) r = 1;
  return (int)r;
}

bool smallcin_conv_ok(const unet_conv_desc* d) {
  return d->nsrc == 1 && d->src[0].kind == UNET_SRC_NCHW_F32 && d->Cin <= 4 && d->ksize == 3 &&
         (double)d->N * d->H * d->W < 2147483648.0 &&
         d->out_mode == UNET_OUT_Y && (d->Cout % 8) == 0;
}
bool smallcin_wgrad_ok(const unet_wgrad_desc* d) {
  return d->nsrc == 1 && d->src[0].kind == UNET_SRC_NCHW_F32 && d->Cin <= 4 && d->ksize == 3 && (d->Cout % 8) == 0 &&
         (double)d->N * d->H * d->W < 2147483648.0;
}

// packed-weight element (co, ci, tap) of the fragment-major layout written by conv.hip pack_kernel
template <typename T>
__device__ __forceinline__ float packed_w(const T* wp, int co, int ci, int tap, int nchunks) {
  constexpr int KC = sizeof(T) == 2 ? 32 : 16, E16 = 16 / (int)sizeof(T);
  const int k = ci;  // chunk 0
  const int lane = (sizeof(T) == 2) ? (k / 8) * 16 + (co & 15) : (k % 4) * 16 + (co & 15);
  const int el = (sizeof(T) == 2) ? k % 8 : k / 4;
  (void)KC;
  return to_f(wp[((((size_t)(co / 16) * nchunks) * 9 + tap) * 64 + lane) * E16 + el]);
}

__device__ __forceinline__ void load_taps(const float* x, long long n, int C, int H, int W, int y0, int x0, int cin,
                                          float* v) {
  const long long plane = (long long)H * W;
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int yy = y0 + t / 3 - 1, xx = x0 + t % 3 - 1;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    v[t] = ok ? x[(n * C + cin) * plane + (long long)yy * W + xx] : 0.f;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void smallcin_fwd_kernel(const unet_conv_desc d, int rows) {
  __shared__ float ws[64 * SC_MAXK];      // [co][ci*9+tap] for up to 64 output channels per pass
  __shared__ float red[2][256];
  const unet_src& s = d.src[0];
  const float* x = (const float*)s.data;
  const int G = d.Cout / 8;
  const int tid = threadIdx.x;
  const int g = tid % G;               // co group (8 channels)
  const int pl = tid / G, PPB = 256 / G;  // pixel lane within a block iteration
  const int KK = 9 * d.Cin;
  const int nchunks = 1;
  const T* wp = (const T*)d.weight;
  for (int i = tid; i < d.Cout * KK; i += 256) {
    const int co = i / KK, r = i % KK;
    ws[i] = packed_w<T>(wp, co, r / 9, r % 9, nchunks);
  }
  __syncthreads();
  const long long P = (long long)d.N * d.H * d.W;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { s1[j] = 0.f; s2[j] = 0.f; }
  // single input channel (the model's 1-channel slices): the 72 weights of this thread's 8 output
  // channels live in registers instead of being re-read from LDS for every pixel
  float w1[8][9];
  if (d.Cin == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int t = 0; t < 9; ++t) w1[j][t] = ws[(g * 8 + j) * KK + t];
  }
  if (pl < PPB && d.Cin == 1 && (d.W % 2) == 0 && (per % 2) == 0) {
    // 1-channel input, two horizontally adjacent pixels per lane and trip: their 3x4 tap window is 12
    // loads instead of 18, the index / bounds math is shared, and the two accumulators form one packed
    // fp32 pair (the kernel is VALU-issue bound, profiles/r01_smallcin_pmc.txt)
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int per_i = (int)(p1 - p0);
    const long long plane = (long long)d.H * d.W;
    for (int b = 2 * pl; b < per_i; b += 2 * PPB) {
      const unsigned q = (unsigned)(p0 + b);
      const int xx = (int)(q % (unsigned)d.W);
      const unsigned t2 = q / (unsigned)d.W;
      const int yy = (int)(t2 % (unsigned)d.H), n = (int)(t2 / (unsigned)d.H);
      const float* xn = x + (long long)n * s.C * plane;
      float v[3][4];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int y2 = yy + r - 1;
        const bool rok = y2 >= 0 && y2 < d.H;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int x2 = xx + c - 1;
          v[r][c] = (rok && x2 >= 0 && x2 < d.W) ? xn[(long long)y2 * d.W + x2] : 0.f;
        }
      }
      f2 acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[j] = f2{0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const f2 tv = {v[t / 3][t % 3], v[t / 3][t % 3 + 1]};
          acc[j] += f2{w1[j][t], w1[j][t]} * tv;
        }
      }
      float a0[8], a1[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { a0[j] = acc[j].x; a1[j] = acc[j].y; }
      const long long p = p0 + b;
      T* o = (T*)d.out + p * d.Cout + g * 8;
      store_vec<T>(o, a0);
      store_vec<T>(o + d.Cout, a1);
      if constexpr (sizeof(T) == 4) {
        store_vec<T>(o + 4, a0 + 4);
        store_vec<T>(o + d.Cout + 4, a1 + 4);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s1[j] += a0[j]; s2[j] += a0[j] * a0[j];
        s1[j] += a1[j]; s2[j] += a1[j] * a1[j];
      }
    }
  } else if (pl < PPB && d.Cin == 1) {
    // 1-channel input: SC_U pixels per trip with all their tap loads issued before the FMAs (the loop
    // is load-latency bound at 4 waves per SIMD).  Pixels and stats keep the one-pixel loop's order.
    const int per_i = (int)(p1 - p0);
    for (int b = pl; b < per_i; b += SC_U * PPB) {
      float v[SC_U][9];
#pragma unroll
      for (int u = 0; u < SC_U; ++u) {
        const int lp = b + u * PPB;
        const unsigned q = (unsigned)(p0 + (lp < per_i ? lp : per_i - 1));
        const int xx = (int)(q % (unsigned)d.W);
        const unsigned t2 = q / (unsigned)d.W;
        load_taps(x, (int)(t2 / (unsigned)d.H), s.C, d.H, d.W, (int)(t2 % (unsigned)d.H), xx, 0, v[u]);
      }
#pragma unroll
      for (int u = 0; u < SC_U; ++u) {
        const int lp = b + u * PPB;
        if (lp < per_i) {
          float acc[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            acc[j] = 0.f;
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[j] += w1[j][t] * v[u][t];
          }
          const long long p = p0 + lp;
          store_vec<T>((T*)d.out + p * d.Cout + g * 8, acc);
          if constexpr (sizeof(T) == 4) store_vec<T>((T*)d.out + p * d.Cout + g * 8 + 4, acc + 4);
#pragma unroll
          for (int j = 0; j < 8; ++j) { s1[j] += acc[j]; s2[j] += acc[j] * acc[j]; }
        }
      }
    }
  } else if (pl < PPB) {
    // pixel index math in 32 bits (host-checked P < 2^31); the column advances by PPB per step
    unsigned q = (unsigned)(p0 + pl);
    int xx = (int)(q % (unsigned)d.W);
    unsigned t2 = q / (unsigned)d.W;
    int yy = (int)(t2 % (unsigned)d.H);
    int n = (int)(t2 / (unsigned)d.H);
    for (long long p = p0 + pl; p < p1; p += PPB) {
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      for (int ci = 0; ci < d.Cin; ++ci) {
        float v[9];
        load_taps(x, n, s.C, d.H, d.W, yy, xx, ci, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float* wr = ws + (g * 8 + j) * KK + ci * 9;
#pragma unroll
          for (int t = 0; t < 9; ++t) acc[j] += wr[t] * v[t];
        }
      }
      xx += PPB;
      while (xx >= d.W) {
        xx -= d.W;
        if (++yy == d.H) { yy = 0; ++n; }
      }
      store_vec<T>((T*)d.out + p * d.Cout + g * 8, acc);
      if constexpr (sizeof(T) == 4) store_vec<T>((T*)d.out + p * d.Cout + g * 8 + 4, acc + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) { s1[j] += acc[j]; s2[j] += acc[j] * acc[j]; }
    }
  }
  if (!d.stats) return;
  // reduce the 8 channel sums over the PPB pixel lanes of each co group
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][tid] = s1[j];
    red[1][tid] = s2[j];
    __syncthreads();
    if (tid < G) {
      float a = 0.f, b = 0.f;
      for (int q = 0; q < PPB; ++q) { a += red[0][q * G + tid]; b += red[1][q * G + tid]; }
      const int co = tid * 8 + j;
      d.stats[(size_t)co * rows + blockIdx.x] = a;
      d.stats[((size_t)d.Cout + co) * rows + blockIdx.x] = b;
    }
    __syncthreads();
  }
}

// dW partial rows: part[row][co*Cin*9 + ci*9 + tap]
template <typename T>
__global__ __launch_bounds__(256) void smallcin_wgrad_kernel(const unet_wgrad_desc d, int rows, float* part) {
  __shared__ float red[4][8 * 9];
  const unet_src& s = d.src[0];
  const float* x = (const float*)s.data;
  const T* dy = (const T*)d.dy;
  const int G = d.Cout / 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // every wave covers all G co groups: lane -> (pixel slot, group)
  const int lanes_per_px = G <= 64 ? G : 64;
  const int g0 = lane % lanes_per_px, ps = lane / lanes_per_px, PPW = 64 / lanes_per_px;
  const long long P = (long long)d.N * d.H * d.W;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  const int KK = 9 * d.Cin;
  for (int gbase = 0; gbase < G; gbase += lanes_per_px) {
    const int g = gbase + g0;
    for (int ci = 0; ci < d.Cin; ++ci) {
      float acc[8][9];
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int t = 0; t < 9; ++t) acc[j][t] = 0.f;
      if (g < G) {
        const unsigned q0 = (unsigned)(p0 + wave * PPW + ps);
        int xx = (int)(q0 % (unsigned)d.W);
        const unsigned t2 = q0 / (unsigned)d.W;
        int yy = (int)(t2 % (unsigned)d.H);
        int n = (int)(t2 / (unsigned)d.H);
        for (long long p = p0 + wave * PPW + ps; p < p1; p += 4 * PPW) {
          float v[9], gy[8];
          load_taps(x, n, s.C, d.H, d.W, yy, xx, ci, v);
          load_vec<T>(dy + p * d.Cout + g * 8, gy);
          if constexpr (sizeof(T) == 4) load_vec<T>(dy + p * d.Cout + g * 8 + 4, gy + 4);
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) acc[j][t] += gy[j] * v[t];
          xx += 4 * PPW;
          while (xx >= d.W) {
            xx -= d.W;
            if (++yy == d.H) { yy = 0; ++n; }
          }
        }
      }
      // reduce over the PPW pixel slots of the wave (lanes with equal g0), then over the 4 waves
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          float a = acc[j][t];
          for (int o = lanes_per_px; o < 64; o <<= 1) a += __shfl_xor(a, o, 64);
          acc[j][t] = a;
        }
      for (int gg = 0; gg < lanes_per_px; ++gg) {
        if (ps == 0 && g0 == gg) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int t = 0; t < 9; ++t) red[wave][j * 9 + t] = acc[j][t];
        }
        __syncthreads();
        const int gq = gbase + gg;
        if (tid < 72 && gq < G) {
          const float a = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
          const int j = tid / 9, t = tid % 9;
          part[(size_t)blockIdx.x * d.Cout * KK + (gq * 8 + j) * KK + ci * 9 + t] = a;
        }
        __syncthreads();
      }
    }
  }
}

int smallcin_conv(const unet_conv_desc* d, hipStream_t st) {
  if (d->Cout > 64) { set_error("smallcin: Cout > 64"); return UNET_ERR_UNSUPPORTED; }
  const int rows = smallcin_rows((long long)d->N * d->H * d->W);
  if (d->dtype == UNET_BF16)
    hipLaunchKernelGGL(smallcin_fwd_kernel<bf16>, dim3(rows), dim3(256), 0, st, *d, rows);
  else if (d->dtype == UNET_F16)
    hipLaunchKernelGGL(smallcin_fwd_kernel<f16>, dim3(rows), dim3(256), 0, st, *d, rows);
  else
    hipLaunchKernelGGL(smallcin_fwd_kernel<float>, dim3(rows), dim3(256), 0, st, *d, rows);
  return check_launch("smallcin_fwd");
}

size_t smallcin_wgrad_ws(const unet_wgrad_desc* d) {
  return (size_t)smallcin_rows((long long)d->N * d->H * d->W) * d->Cout * d->Cin * 9 * sizeof(float);
}

int smallcin_wgrad(const unet_wgrad_desc* d, hipStream_t st) {
  const int rows = smallcin_rows((long long)d->N * d->H * d->W);
  float* part = (float*)d->workspace;
  if (d->dtype == UNET_BF16)
    hipLaunchKernelGGL(smallcin_wgrad_kernel<bf16>, dim3(rows), dim3(256), 0, st, *d, rows, part);
  else if (d->dtype == UNET_F16)
    hipLaunchKernelGGL(smallcin_wgrad_kernel<f16>, dim3(rows), dim3(256), 0, st, *d, rows, part);
  else
    hipLaunchKernelGGL(smallcin_wgrad_kernel<float>, dim3(rows), dim3(256), 0, st, *d, rows, part);
  int e = check_launch("smallcin_wgrad");
  if (e) return e;
  return unet_colsum(part, rows, d->Cout * d->Cin * 9, d->dw, d->accum, (void*)st);
}

}  // namespace unet
