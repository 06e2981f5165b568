// smallcin.hip — the network's first convolution (inc.0: nn.Conv2d(n_channels<=4 -> 64, 3x3),
// unet/models/layers.py:32 via unet.py:152) reading the fp32 NCHW model input directly.
//
// With 1-3 input channels the layer is pure streaming (K = 9..27): a 64-wide MFMA tile would be >90 %
// zero padding.  Forward: one thread computes 8 output channels of one pixel with VALU FMAs from
// L1-cached input taps and writes them as one 16-byte vector, plus BN partial sums.  Weight
// gradient: per-thread 8 x (9*Cin) partial sums over a pixel range, reduced across the block, one
// fp32 row per block; unet_colsum finishes (fixed order).
#include "conv_src16.h"

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

// 16-bit output, Cout = 64, Cin <= 3: the layer on MFMA.  y[co][px] = Σ_k W[co][k] X[k][px] with
// K = [the 9 Cin taps of x_hi | the same taps of x_lo] (x = x_hi + x_lo, both 16-bit, so the fp32 input keeps
// ~17 mantissa bits; weights are the 16-bit packed ones), padded to 32 / 64 with zeros: one or two
// v_mfma_f32_16x16x32 per 16 output channels x 16 pixels.  The fp32 NCHW input tile (+ halo) is staged in LDS
// by coalesced loads; a wave owns 16 pixels of each tile row and writes 4 channels x 16 bit per lane and
// fragment; BN partial sums of the fp32 accumulators per wave.  The VALU kernel above is issue-bound at
// ~4x the HBM time of its 67 MB output (profiles/r01_smallcin_pmc.txt).
template <typename T> struct SCElem;
template <> struct SCElem<bf16> { typedef __bf16 type; };
template <> struct SCElem<f16> { typedef _Float16 type; };
constexpr int SCM_TR = 8, SCM_TW = 64, SCM_HW = SCM_TW + 2;
constexpr int SCM_GRID = 512;     // persistent blocks; stats rows = 4 per block

template <typename T>
__global__ __launch_bounds__(256) void smallcin_fwd_mfma_kernel(const unet_conv_desc d, int ntiles) {
  using F = typename Mma<T>::frag;
  __shared__ float xt[4 * (SCM_TR + 2) * SCM_HW];   // [ci][row][col] fp32 input tile with halo
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15;
  const int Cin = d.Cin, K9 = 9 * Cin, nks = (2 * K9 + 31) / 32;
  const int tiles_w = (d.W + SCM_TW - 1) / SCM_TW, tiles_h = (d.H + SCM_TR - 1) / SCM_TR;
  const float* x = (const float*)d.src[0].data;
  const int Cs = d.src[0].C;
  const T* wp = (const T*)d.weight;
  // A fragments (weights): lane holds W[co = 16 f + c16][k = 32 ks + 8 g + e]; B operand offsets: the LDS
  // element of k = 32 ks + 8 g + e relative to the lane's pixel (-1: zero), and whether it is the low half
  F a[2][4];
  int off[2][8];
  unsigned lomask = 0;
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 32 * ks + 8 * g + e;
      const bool real = k < 2 * K9;
      const int kk = k < K9 ? k : k - K9;
      const int ci = kk / 9, tap = kk % 9;
      off[ks][e] = real ? ci * (SCM_TR + 2) * SCM_HW + (tap / 3) * SCM_HW + tap % 3 : -1;
      if (real && k >= K9) lomask |= 1u << (8 * ks + e);
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const float wv = real ? packed_w<T>(wp, 16 * f + c16, ci, tap, 1) : 0.f;
        a[ks][f][e] = (typename SCElem<T>::type)wv;
      }
    }
  float s1[4][4], s2[4][4];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) { s1[f][r] = 0.f; s2[f][r] = 0.f; }
  T* y = (T*)d.out;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int tw = tile % tiles_w, t2 = tile / tiles_w;
    const int h0 = (t2 % tiles_h) * SCM_TR, w0 = tw * SCM_TW, n = t2 / tiles_h;
    __syncthreads();
    const int nel = Cin * (SCM_TR + 2) * SCM_HW;
    for (int i = tid; i < nel; i += 256) {
      const int ci = i / ((SCM_TR + 2) * SCM_HW), rem = i % ((SCM_TR + 2) * SCM_HW);
      const int yy = h0 - 1 + rem / SCM_HW, xx = w0 - 1 + rem % SCM_HW;
      xt[i] = ((unsigned)yy < (unsigned)d.H && (unsigned)xx < (unsigned)d.W)
                  ? x[(((size_t)n * Cs + ci) * d.H + yy) * d.W + xx] : 0.f;
    }
    __syncthreads();
    const int ow = w0 + 16 * wave + c16;
    for (int r = 0; r < SCM_TR && h0 + r < d.H; ++r) {
      f32x4 acc[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* xr = xt + r * SCM_HW + 16 * wave + c16;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if (ks < nks) {
          F b;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = off[ks][e] >= 0 ? xr[off[ks][e] < 0 ? 0 : off[ks][e]] : 0.f;
            const float hi = (float)(typename SCElem<T>::type)v;
            b[e] = (typename SCElem<T>::type)(((lomask >> (8 * ks + e)) & 1) ? v - hi : v);
          }
#pragma unroll
          for (int f = 0; f < 4; ++f) acc[f] = Mma<T>::mma(a[ks][f], b, acc[f]);
        }
      }
      // lane (c16, g) holds channels 16 f + 4 g .. + 3 of pixel ow for f = 0..3.  v_permlane16_swap of the
      // packed (f, f + 1) pairs (odd rows of the first with even rows of the second) leaves row g with the
      // 8 contiguous channels 16 (f + (g & 1)) + 8 (g >> 1) .. + 7: two 16-byte stores per lane and row
      // instead of four 8-byte ones (all lanes take part in the swaps; the stores are masked)
      unsigned px_[4], py_[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        px_[f] = pack2_16<T>(acc[f][0], acc[f][1]);
        py_[f] = pack2_16<T>(acc[f][2], acc[f][3]);
      }
      const size_t pix = ((size_t)n * d.H + h0 + r) * d.W + ow;
#pragma unroll
      for (int f = 0; f < 4; f += 2) {
        const auto sx = __builtin_amdgcn_permlane16_swap(px_[f], px_[f + 1], false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(py_[f], py_[f + 1], false, false);
        if (ow < d.W)
          *reinterpret_cast<uint4*>(y + pix * 64 + 16 * (f + (g & 1)) + 8 * (g >> 1)) =
              make_uint4(sx[0], sy[0], sx[1], sy[1]);
      }
      if (ow < d.W) {
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            s1[f][q] += acc[f][q];
            s2[f][q] = __builtin_fmaf(acc[f][q], acc[f][q], s2[f][q]);
          }
      }
    }
  }
  if (!d.stats) return;
  const int rows = gridDim.x * 4, row = blockIdx.x * 4 + wave;
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float a1 = row16_sum(s1[f][q]), a2 = row16_sum(s2[f][q]);
      if (c16 == 0) {
        const int co = 16 * f + 4 * g + q;
        d.stats[(size_t)co * rows + row] = a1;
        d.stats[((size_t)64 + co) * rows + row] = a2;
      }
    }
}

static bool smallcin_mfma_ok(const unet_conv_desc* d) {
  const char* e = getenv("UNET_SMALLCIN_MFMA");
  if (e && !atoi(e)) return false;
  return (d->dtype == UNET_BF16 || d->dtype == UNET_F16) && d->Cout == 64 && d->Cin <= 3;
}

static int smallcin_mfma_tiles(const unet_conv_desc* d) {
  return d->N * cdiv(d->H, SCM_TR) * cdiv(d->W, SCM_TW);
}

int smallcin_stats_rows(const unet_conv_desc* d) {
  if (smallcin_mfma_ok(d)) {
    const int t = smallcin_mfma_tiles(d);
    return 4 * (t < SCM_GRID ? t : SCM_GRID);
  }
  return smallcin_rows((long long)d->N * d->H * d->W);
}

bool smallcin_is_mfma(const unet_conv_desc* d) { return smallcin_mfma_ok(d); }

int smallcin_conv(const unet_conv_desc* d, hipStream_t st) {
  if (smallcin_mfma_ok(d)) {
    const int t = smallcin_mfma_tiles(d);
    const int grid = t < SCM_GRID ? t : SCM_GRID;
    if (d->dtype == UNET_BF16)
      hipLaunchKernelGGL(smallcin_fwd_mfma_kernel<bf16>, dim3(grid), dim3(256), 0, st, *d, t);
    else
      hipLaunchKernelGGL(smallcin_fwd_mfma_kernel<f16>, dim3(grid), dim3(256), 0, st, *d, t);
    return check_launch("smallcin_fwd_mfma");
  }
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

// weight gradient on MFMA (16-bit dy, Cout = 64, Cin <= 3): D[co][k] = Σ_px dy[px][co] X[px][k], K = the
// pixels (32 per v_mfma_f32_16x16x32, one tile-row half), k = [the 9 Cin taps of x_hi | the same of x_lo]
// (16 per fragment); dW[co][ci][tap] = D[co][k] + D[co][k + 9 Cin] (smallcin_fold).  A wave stages the dy of
// its 32 pixels (4 KB, one coalesced 16-byte load per lane x 4, prefetched one step ahead) in its own LDS
// slice, swizzled for the conflict-free transposed reads (ds_read_b64_tr_b16) that turn NHWC pixel rows into
// K-major fragments; the fp32 input tile is shared by the block.  Per-wave partial D rows, fixed-order sums.
template <typename T>
__global__ __launch_bounds__(256) void smallcin_wgrad_mfma_kernel(const unet_wgrad_desc d, int ntiles, float* part) {
  using F = typename Mma<T>::frag;
  __shared__ float xt[4 * (SCM_TR + 2) * SCM_HW];
  __shared__ __attribute__((aligned(16))) unsigned char dyl[4][32 * 128];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, c16 = lane & 15, q = (lane >> 2) & 3, pp = lane & 3;
  const int Cin = d.Cin, K9 = 9 * Cin, NJ = (2 * K9 + 15) / 16;
  const int tiles_w = (d.W + SCM_TW - 1) / SCM_TW, tiles_h = (d.H + SCM_TR - 1) / SCM_TR;
  const float* x = (const float*)d.src[0].data;
  const int Cs = d.src[0].C;
  const rsrc_t rdy = mk_rsrc(d.dy, (unsigned)((long long)d.N * d.H * d.W * 128));
  // B operand: lane's k = 16 j + c16 -> LDS element offset of its tap (-1: zero column) and hi / lo half
  int boff[4];
  unsigned lom = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 16 * j + c16;
    const bool real = k < 2 * K9;
    const int kk = k < K9 ? k : k - K9;
    const int ci = kk / 9, tap = kk % 9;
    boff[j] = real ? ci * (SCM_TR + 2) * SCM_HW + (tap / 3) * SCM_HW + tap % 3 : -1;
    if (real && k >= K9) lom |= 1u << j;
  }
  // A operand (dy, 16 co x 32 px): transposed-read addresses in the wave's swizzled dy slice
  // (pixel px = 128 B = 8 units of 8 channels, unit u stored at u ^ swz(px), swz as wgrad5's UPP = 8)
  auto swz = [](int px) { return 2 * ((px >> 1) & 1) + 4 * ((px >> 3) & 1); };
  unsigned aoff[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int px = 8 * g + 4 * h + q, u = 2 * f + (pp >> 1);
      aoff[h][f] = (unsigned)(px * 128 + ((u ^ swz(px)) * 16) + 8 * (pp & 1));
    }
  // this lane's 4 staged dy units: pixel 8 k + (lane >> 3), unit lane & 7
  unsigned woff[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int px = 8 * k + (lane >> 3), u = lane & 7;
    woff[k] = (unsigned)(px * 128 + ((u ^ swz(px)) * 16));
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned char* dw_ = dyl[wave];
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int tw = tile % tiles_w, t2 = tile / tiles_w;
    const int h0 = (t2 % tiles_h) * SCM_TR, w0 = tw * SCM_TW, n = t2 / tiles_h;
    __syncthreads();
    const int nel = Cin * (SCM_TR + 2) * SCM_HW;
    for (int i = tid; i < nel; i += 256) {
      const int ci = i / ((SCM_TR + 2) * SCM_HW), rem = i % ((SCM_TR + 2) * SCM_HW);
      const int yy = h0 - 1 + rem / SCM_HW, xx = w0 - 1 + rem % SCM_HW;
      xt[i] = ((unsigned)yy < (unsigned)d.H && (unsigned)xx < (unsigned)d.W)
                  ? x[(((size_t)n * Cs + ci) * d.H + yy) * d.W + xx] : 0.f;
    }
    __syncthreads();
    // K steps of this wave: rows wave, wave + 4; two 32-pixel halves each
    uint4 nx[4];
    auto load_dy = [&](int st) {
      const int r = wave + 4 * (st >> 1), c0 = 32 * (st & 1);
      const int oh = h0 + r;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ow = w0 + c0 + 8 * k + (lane >> 3);
        const bool ok = oh < d.H && ow < d.W;
        const unsigned pix = ((unsigned)n * d.H + oh) * (unsigned)d.W + ow;
        nx[k] = bld(rdy, ok ? pix * 128u + (unsigned)(lane & 7) * 16u : OOB, 0);
      }
    };
    load_dy(0);
#pragma unroll 1
    for (int st = 0; st < 4; ++st) {
#pragma unroll
      for (int k = 0; k < 4; ++k) *reinterpret_cast<uint4*>(dw_ + woff[k]) = nx[k];
      if (st + 1 < 4) load_dy(st + 1);
      F a[4];
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const i16x4 lo4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(dw_ + aoff[0][f]));
        const i16x4 hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(dw_ + aoff[1][f]));
        a[f] = __builtin_bit_cast(F, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      const int r = wave + 4 * (st >> 1), c0 = 32 * (st & 1);
      const float* xr = xt + r * SCM_HW + c0 + 8 * g;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (j < NJ) {
          F b;
          const int o = boff[j] < 0 ? 0 : boff[j];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = boff[j] >= 0 ? xr[o + e] : 0.f;
            const float hi = (float)(typename SCElem<T>::type)v;
            b[e] = (typename SCElem<T>::type)(((lom >> j) & 1) ? v - hi : v);
          }
#pragma unroll
          for (int f = 0; f < 4; ++f) acc[f][j] = Mma<T>::mma(a[f], b, acc[f][j]);
        }
      }
    }
  }
  // partial D of this wave: part[row][co][k] (k < 2 K9), row = 4 * block + wave
  const int row = blockIdx.x * 4 + wave, K2 = 2 * K9;
  float* pr = part + (size_t)row * 64 * K2;
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = 16 * j + c16;
      if (j < NJ && k < K2) {
#pragma unroll
        for (int r = 0; r < 4; ++r) pr[(16 * f + 4 * g + r) * K2 + k] = acc[f][j][r];
      }
    }
}

// dW[co][kk] (+)= Σ_rows part[row][co][kk] + part[row][co][kk + K9]  (fixed order), in two coalesced passes
// over the [rows][W = Cout·2·K9] partial table: pass 1 — block b sums its SCF_R consecutive rows for every column
// (consecutive threads, consecutive columns), pass 2 — one thread per output column adds the blocks' sums in
// block order and folds the x_hi / x_lo halves.  (Round 5: the one-pass fold, one block per output column or
// per output channel, read one column of the 2048-row table at a 4.6 KB stride per row: 18-20 us per step.)
constexpr int SCF_R = 8;     // rows per pass-1 block (2048 rows: 256 blocks)
constexpr int SCF_KL = 32;   // pass 2: lanes over the pass-1 blocks (x 8 output columns per block)
template <int CIN>
__global__ __launch_bounds__(256) void smallcin_fold1_kernel(const float* part, int rows, float* sums) {
  constexpr int W = 64 * 18 * CIN, NC = (W + 255) / 256;
  const int r0 = blockIdx.x * SCF_R;
  float v[NC][SCF_R];
#pragma unroll
  for (int j = 0; j < NC; ++j)
#pragma unroll
    for (int i = 0; i < SCF_R; ++i) {   // every load of the thread issued first (one memory round trip)
      const int c = threadIdx.x + 256 * j, r = r0 + i;
      v[j][i] = (c < W && r < rows) ? part[(size_t)r * W + c] : 0.f;
    }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int c = threadIdx.x + 256 * j;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < SCF_R; ++i) s += v[j][i];   // row order
    if (c < W) sums[(size_t)blockIdx.x * W + c] = s;
  }
}
template <int CIN>
__global__ __launch_bounds__(256) void smallcin_fold2_kernel(const float* sums, int nb, float* dw, int accum) {
  constexpr int K9 = 9 * CIN, W = 64 * 2 * K9;
  __shared__ float red[2][SCF_KL][8];
  const int cl = threadIdx.x & 7, kl = threadIdx.x >> 3;   // 8 output columns x 32 block lanes
  const int col = blockIdx.x * 8 + cl;                    // output column (co, kk) of 64 * K9
  const bool ok = col < 64 * K9;
  const int co = ok ? col / K9 : 0, kk = ok ? col % K9 : 0;
  const float* p = sums + (size_t)co * 2 * K9 + kk;
  float a = 0.f, b = 0.f;
  for (int k0 = kl; k0 < nb; k0 += 4 * SCF_KL) {   // 4 block rows per trip, loads first
    float va[4], vb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = k0 + u * SCF_KL;
      va[u] = (ok && k < nb) ? p[(size_t)k * W] : 0.f;
      vb[u] = (ok && k < nb) ? p[(size_t)k * W + K9] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) { a += va[u]; b += vb[u]; }
  }
  red[0][kl][cl] = a;
  red[1][kl][cl] = b;
  __syncthreads();
  if (kl == 0 && ok) {
    float sa = 0.f, sb = 0.f;
    for (int k = 0; k < SCF_KL; ++k) { sa += red[0][k][cl]; sb += red[1][k][cl]; }   // lane order
    const float v = sa + sb;
    dw[col] = accum ? dw[col] + v : v;
  }
}

static bool smallcin_wgrad_mfma_ok(const unet_wgrad_desc* d) {
  const char* e = getenv("UNET_SMALLCIN_MFMA");
  if (e && !atoi(e)) return false;
  return (d->dtype == UNET_BF16 || d->dtype == UNET_F16) && d->Cout == 64 && d->Cin <= 3 &&
         (double)d->N * d->H * d->W * 128 < (double)OOB;
}

static int smallcin_wgrad_grid(const unet_wgrad_desc* d, int* tiles) {
  const int t = d->N * cdiv(d->H, SCM_TR) * cdiv(d->W, SCM_TW);
  if (tiles) *tiles = t;
  return t < SCM_GRID ? t : SCM_GRID;
}

bool smallcin_wgrad_is_mfma(const unet_wgrad_desc* d) { return smallcin_wgrad_mfma_ok(d); }

size_t smallcin_wgrad_ws(const unet_wgrad_desc* d) {
  if (smallcin_wgrad_mfma_ok(d)) {   // the partial table [4·grid][64·2·9·Cin] + the fold's block sums
    const int rows = 4 * smallcin_wgrad_grid(d, nullptr);
    return (size_t)(rows + cdiv(rows, SCF_R)) * 64 * (2 * 9 * d->Cin) * sizeof(float);
  }
  return (size_t)smallcin_rows((long long)d->N * d->H * d->W) * d->Cout * d->Cin * 9 * sizeof(float);
}

int smallcin_wgrad(const unet_wgrad_desc* d, hipStream_t st) {
  if (smallcin_wgrad_mfma_ok(d)) {
    int t;
    const int grid = smallcin_wgrad_grid(d, &t);
    float* part = (float*)d->workspace;
    if (d->dtype == UNET_BF16)
      hipLaunchKernelGGL(smallcin_wgrad_mfma_kernel<bf16>, dim3(grid), dim3(256), 0, st, *d, t, part);
    else
      hipLaunchKernelGGL(smallcin_wgrad_mfma_kernel<f16>, dim3(grid), dim3(256), 0, st, *d, t, part);
    int e = check_launch("smallcin_wgrad_mfma");
    if (e) return e;
    const int rows = 4 * grid, W = 64 * 2 * 9 * d->Cin, nb = cdiv(rows, SCF_R);
    float* sums = part + (size_t)rows * W;   // after the partial table (smallcin_wgrad_ws)
    const dim3 g2(cdiv(64 * 9 * d->Cin, 8));
#define SCF_LAUNCH(CI)                                                                                          \
  do {                                                                                                        \
    hipLaunchKernelGGL(smallcin_fold1_kernel<CI>, dim3(nb), dim3(256), 0, st, part, rows, sums);             \
    hipLaunchKernelGGL(smallcin_fold2_kernel<CI>, g2, dim3(256), 0, st, sums, nb, d->dw, d->accum);          \
  } while (0)
    if (d->Cin == 1) SCF_LAUNCH(1);
    else if (d->Cin == 2) SCF_LAUNCH(2);
    else SCF_LAUNCH(3);
#undef SCF_LAUNCH
    return check_launch("smallcin_fold");
  }
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
