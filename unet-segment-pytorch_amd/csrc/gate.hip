// gate.hip — AttentionGate (unet/models/layers.py:126-192) element/reduction passes.
//
// Forward:  gw = W_g·g_up and xw = W_x·x are produced by the 1x1 conv kernel (with BN partials).
//           psi pass (here): a = relu(bn_g(gw) + bn_x(xw)); p = wpsi·a; partial Σp, Σp²   (:186-189)
//           s = sigmoid(bn_psi(p)) is never stored: the next conv's loader evaluates it (:192).
// Backward: bwd1  (per pixel)   ds = Σ_c d(x·s)_c x_c ; dx (+)= d·s ; dq = ds·s(1−s) ; Σdq, Σdq·p̂
//           bwd2  (per channel) dz = dp·wpsi·[a>0] ; Σdz, Σdz·ĝ, Σdz·x̂, Σdp·a
//           bwd3  (apply)       dgw, dxw = BN-backward(dz)  -> 1x1 conv dgrad/wgrad
#include "common.h"

namespace unet {

static inline int chan_lanes_g(int C) {
  int cl = 1;
  while (cl < C && cl < 64) cl <<= 1;
  return cl;
}
static inline int rows_for(long long P, int C) {
  const int cl = chan_lanes_g(C);
  const int cblocks = (C + cl - 1) / cl;
  long long r = (2048 + cblocks - 1) / cblocks;
  const long long maxr = (P + 15) / 16;   // >= 16 pixels per block (the 64^2 maps: 1024 blocks, not 256)
  if (r > maxr) r = maxr;
  if (r < 1) r = 1;
  return (int)r;
}
// blocks (= partial rows) of the per-pixel passes: >= 32 pixels per block, so the small maps (64^2: 16 K
// pixels) still spread over 512 blocks — with 256 pixels per block that map ran on 64 blocks, a quarter
// of the CUs (gate pass 1 at 64^2: 62 us for 84 MB, round-4 layerprof)
static inline int pix_rows(long long P) {
  long long r = (P + 31) / 32;
  if (r > 2048) r = 2048;
  if (r < 1) r = 1;
  return (int)r;
}

__device__ __forceinline__ float block_sum_f(float v, float* sh) {
  const int tid = threadIdx.x;
  v = wave_sum(v);
  if ((tid & 63) == 0) sh[tid >> 6] = v;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r += sh[w];
  __syncthreads();
  return r;
}

// one thread per pixel; grid-stride over a contiguous pixel range per block (deterministic partials)
template <typename T>
__global__ void psi_kernel(long long P, int Ci, const T* gw, const T* xw, const float* gab, const float* xab,
                           const float* wpsi, float* p, float* part, int rows) {
  __shared__ float sh[8];
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float s = 0.f, ss = 0.f;
  for (long long q = p0 + threadIdx.x; q < p1; q += blockDim.x) {
    const T* g = gw + q * Ci;
    const T* x = xw + q * Ci;
    float acc = 0.f;
    for (int c = 0; c < Ci; ++c) {
      const float a = fmaxf(to_f(g[c]) * gab[c] + gab[Ci + c] + to_f(x[c]) * xab[c] + xab[Ci + c], 0.f);
      acc += wpsi[c] * a;
    }
    p[q] = acc;
    s += acc;
    ss += acc * acc;
  }
  s = block_sum_f(s, sh);
  ss = block_sum_f(ss, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s;
    part[rows + blockIdx.x] = ss;
  }
}

template <typename T>
__global__ void gate_bwd1_kernel(long long P, int Cx, const float* dxs, const T* yx, const float* sx, const float* bx,
                                 int relu, const float* pp, const float* psi_ab, const float* psi_mean,
                                 const float* psi_inv, float* dx, int dx_accum, float* dq, float* part, int rows) {
  __shared__ float sh[8];
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  const float pa = psi_ab[0], pb = psi_ab[1], pm = psi_mean[0], pi = psi_inv[0];
  float s1 = 0.f, s2 = 0.f;
  for (long long q = p0 + threadIdx.x; q < p1; q += blockDim.x) {
    const float pv = pp[q];
    const float sg = sigmoidf_(pv * pa + pb);
    const float* d = dxs + q * Cx;
    const T* y = yx + q * Cx;
    float* o = dx ? dx + q * Cx : nullptr;
    float ds = 0.f;
    for (int c = 0; c < Cx; ++c) {
      float xv = __builtin_fmaf(to_f(y[c]), sx[c], bx[c]);
      if (relu) xv = fmaxf(xv, 0.f);
      const float dv = d[c];
      ds += dv * xv;
      if (dx) {
        o[c] = dx_accum ? __builtin_fmaf(dv, sg, o[c]) : dv * sg;
      }
    }
    const float dqv = ds * sg * (1.f - sg);
    dq[q] = dqv;
    s1 += dqv;
    s2 += dqv * (pv - pm) * pi;
  }
  s1 = block_sum_f(s1, sh);
  s2 = block_sum_f(s2, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s1;
    part[rows + blockIdx.x] = s2;
  }
}

// ---- coalesced variants: a group of G = C/8 lanes owns one pixel (8 channels per lane); per-pixel
// channel sums by xor-shuffles inside the group.  Used when C % 8 == 0 and C/8 is a power of two <= 64.
__device__ __forceinline__ float group_sum(float v, int G) {
  for (int o = G >> 1; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    load_vec<T>(p, v);
  } else {
    load_vec<float>((const float*)p, v);
    load_vec<float>((const float*)p + 4, v + 4);
  }
}

constexpr int GV_U = 4;    // pixels per lane per trip of the vectorised psi pass (loads in flight)
constexpr int GV_U2 = 2;   // the same for gate passes 2 / 3 (4 measured slower there: 162 VGPRs, 28.4 -> 30.5 us)

template <typename T>
__global__ void psi_vec_kernel(long long P, int Ci, int G, const T* __restrict__ gw, const T* __restrict__ xw,
                               const float* gab, const float* xab, const float* wpsi, float* __restrict__ p, float* part,
                               int rows) {
  __shared__ float sh[8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int sub = lane % G, ppw = 64 / G;
  const int c0 = sub * 8;
  float gs[8], gb[8], xs[8], xb[8], w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    gs[j] = gab[c0 + j]; gb[j] = gab[Ci + c0 + j]; xs[j] = xab[c0 + j]; xb[j] = xab[Ci + c0 + j]; w[j] = wpsi[c0 + j];
  }
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float s = 0.f, ss = 0.f;
  // GV_U pixels per lane per trip, every load issued first (one pixel per trip serialised a memory round
  // trip per pixel); the pixels are then reduced in the one-pixel loop's order, so s / ss are unchanged
  const long long S = (long long)nw * ppw;
  for (long long q = p0 + wave * ppw + lane / G; q < p1; q += GV_U * S) {
    float g[GV_U][8], x[GV_U][8];
#pragma unroll
    for (int u = 0; u < GV_U; ++u) {
      const long long qq = q + u * S < p1 ? q + u * S : q;
      load8<T>(gw + qq * Ci + c0, g[u]);
      load8<T>(xw + qq * Ci + c0, x[u]);
    }
#pragma unroll
    for (int u = 0; u < GV_U; ++u) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += w[j] * fmaxf(g[u][j] * gs[j] + gb[j] + x[u][j] * xs[j] + xb[j], 0.f);
      acc = group_sum(acc, G);
      if (sub == 0 && q + u * S < p1) {
        p[q + u * S] = acc;
        s += acc;
        ss += acc * acc;
      }
    }
  }
  s = block_sum_f(s, sh);
  ss = block_sum_f(ss, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s;
    part[rows + blockIdx.x] = ss;
  }
}

constexpr int GB1_U = 4;   // pixels per lane per trip (loads in flight)

template <typename T>
__global__ void gate_bwd1_vec_kernel(long long P, int Cx, int G, const float* __restrict__ dxs,
                                     const T* __restrict__ yx, const float* sx, const float* bx, int relu,
                                     const float* __restrict__ pp, const float* psi_ab, const float* psi_mean,
                                     const float* psi_inv, float* __restrict__ dx, int dx_accum,
                                     float* __restrict__ dq, float* part, int rows) {
  __shared__ float sh[8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int sub = lane % G, ppw = 64 / G;
  const int c0 = sub * 8;
  float sc[8], sf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = sx[c0 + j]; sf[j] = bx[c0 + j]; }
  const float pa = psi_ab[0], pb = psi_ab[1], pm = psi_mean[0], pi = psi_inv[0];
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float s1 = 0.f, s2 = 0.f;
  // GB1_U pixels per trip with every load issued before the stores (the stores to dx may alias the loads
  // as far as the compiler knows, so a one-pixel loop serialises a full memory round trip per pixel);
  // s1 / s2 keep the one-pixel loop's pixel order
  const long long S = (long long)nw * ppw;
  for (long long q = p0 + wave * ppw + lane / G; q < p1; q += GB1_U * S) {
    float d[GB1_U][8], y[GB1_U][8], g[GB1_U][8], pv[GB1_U];
    bool ok[GB1_U];
#pragma unroll
    for (int u = 0; u < GB1_U; ++u) {
      ok[u] = q + u * S < p1;
      const long long qq = ok[u] ? q + u * S : q;
      load_vec<float>(dxs + qq * Cx + c0, d[u]);
      load_vec<float>(dxs + qq * Cx + c0 + 4, d[u] + 4);
      load8<T>(yx + qq * Cx + c0, y[u]);
      pv[u] = pp[qq];
      if (dx && dx_accum) {
        load_vec<float>(dx + qq * Cx + c0, g[u]);
        load_vec<float>(dx + qq * Cx + c0 + 4, g[u] + 4);
      }
    }
#pragma unroll
    for (int u = 0; u < GB1_U; ++u) {
      const float sg = sigmoidf_(pv[u] * pa + pb);
      float ds = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float xv = __builtin_fmaf(y[u][j], sc[j], sf[j]);
        if (relu) xv = fmaxf(xv, 0.f);
        ds += d[u][j] * xv;
      }
      if (dx_accum) {  // one rounding (explicit fmaf), the operation the gated W_x dgrad epilogue uses
#pragma unroll
        for (int j = 0; j < 8; ++j) g[u][j] = __builtin_fmaf(d[u][j], sg, g[u][j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) g[u][j] = d[u][j] * sg;
      }
      ds = group_sum(ds, G);
      if (ok[u]) {
        const long long qq = q + u * S;
        if (dx) {  // null: the x*s term is added by the W_x dgrad (UNET_OUT_F32_GATED)
          float* o = dx + qq * Cx + c0;
          store_vec<float>(o, g[u]);
          store_vec<float>(o + 4, g[u] + 4);
        }
        if (sub == 0) {
          const float dqv = ds * sg * (1.f - sg);
          dq[qq] = dqv;
          s1 += dqv;
          s2 += dqv * (pv[u] - pm) * pi;
        }
      }
    }
  }
  s1 = block_sum_f(s1, sh);
  s2 = block_sum_f(s2, sh);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = s1;
    part[rows + blockIdx.x] = s2;
  }
}

static inline int vec_group(int C) {
  if (C % 8) return 0;
  const int g = C / 8;
  if (g > 64 || (g & (g - 1))) return 0;
  return g;
}

// channel lanes x pixel rows
template <typename T>
__global__ void gate_bwd2_kernel(long long P, int Ci, int CL, const T* gw, const T* xw, const float* gab,
                                 const float* xab, const float* gm, const float* gi, const float* xm, const float* xi,
                                 const float* wpsi, const float* dq, const float* pp, const float* pc, float* part,
                                 int rows) {
  __shared__ float sh[4][256];
  const int tid = threadIdx.x;
  const int cx = tid % CL, py = tid / CL, R = blockDim.x / CL;
  const int c = blockIdx.x * CL + cx;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.y * per, p1 = min(P, p0 + per);
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < Ci) {
    const float gs = gab[c], gb = gab[Ci + c], xs = xab[c], xb = xab[Ci + c];
    const float gmu = gm[c], giv = gi[c], xmu = xm[c], xiv = xi[c], w = wpsi[c];
    const float A = pc[0], B = pc[1], Cc = pc[2];
    for (long long q = p0 + py; q < p1; q += R) {
      const float g = to_f(gw[q * Ci + c]), x = to_f(xw[q * Ci + c]);
      const float a = fmaxf(g * gs + gb + x * xs + xb, 0.f);
      const float dp = A * dq[q] + B * pp[q] + Cc;
      const float dz = a > 0.f ? dp * w : 0.f;
      a0 += dz;
      a1 += dz * (g - gmu) * giv;
      a2 += dz * (x - xmu) * xiv;
      a3 += dp * a;
    }
  }
  sh[0][tid] = a0;
  sh[1][tid] = a1;
  sh[2][tid] = a2;
  sh[3][tid] = a3;
  __syncthreads();
  if (py == 0 && c < Ci) {
    float r[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < R; ++k)
#pragma unroll
      for (int f = 0; f < 4; ++f) r[f] += sh[f][k * CL + cx];
#pragma unroll
    for (int f = 0; f < 4; ++f) part[((size_t)f * rows + blockIdx.y) * Ci + c] = r[f];
  }
}

template <typename T>
__global__ void gate_bwd3_kernel(long long P, int Ci, int CL, const T* gw, const T* xw, const float* gab,
                                 const float* xab, const float* wpsi, const float* dq, const float* pp, const float* pc,
                                 const float* gcoef, const float* xcoef, T* dgw, T* dxw, int rows) {
  const int tid = threadIdx.x;
  const int cx = tid % CL, py = tid / CL, R = blockDim.x / CL;
  const int c = blockIdx.x * CL + cx;
  if (c >= Ci) return;
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.y * per, p1 = min(P, p0 + per);
  const float gs = gab[c], gb = gab[Ci + c], xs = xab[c], xb = xab[Ci + c], w = wpsi[c];
  const float A = pc[0], B = pc[1], Cc = pc[2];
  const float gA = gcoef[c], gB = gcoef[Ci + c], gC = gcoef[2 * Ci + c];
  const float xA = xcoef[c], xB = xcoef[Ci + c], xC = xcoef[2 * Ci + c];
  for (long long q = p0 + py; q < p1; q += R) {
    const float g = to_f(gw[q * Ci + c]), x = to_f(xw[q * Ci + c]);
    const float a = fmaxf(g * gs + gb + x * xs + xb, 0.f);
    const float dp = A * dq[q] + B * pp[q] + Cc;
    const float dz = a > 0.f ? dp * w : 0.f;
    dgw[q * Ci + c] = from_f<T>(f32_rounded(__builtin_fmaf(gA, dz, __builtin_fmaf(gB, g, gC))));   // bn.hip's rounding
    dxw[q * Ci + c] = from_f<T>(f32_rounded(__builtin_fmaf(xA, dz, __builtin_fmaf(xB, x, xC))));
  }
}

// ---- coalesced gate passes 2 / 3 (Ci % 8 == 0, G = Ci/8 a power of two <= 64): a group of G lanes owns a
// pixel, 8 channels per lane, so every load / store is one 16-byte vector (the per-channel forms above move
// 2 bytes per lane).  Pass 2's four per-channel sums: per lane over its pixels, then xor-shuffles over the
// lanes of a wave that hold the same channels, then the 4 waves in order through LDS — a fixed order
// (deterministic), into the same [4][rows][Ci] partial layout, so unet_bn_bwd_finalize / unet_colsum are
// unchanged.  Pass 3 evaluates the same per-element expressions as gate_bwd3_kernel (bit-identical).
template <typename T>
__device__ __forceinline__ void store8(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    store_vec<T>(p, v);
  } else {
    store_vec<float>((float*)p, v);
    store_vec<float>((float*)p + 4, v + 4);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gate_bwd2_vec_kernel(long long P, int Ci, int G, const T* gw, const T* xw,
                                                            const float* gab, const float* xab, const float* gm,
                                                            const float* gi, const float* xm, const float* xi,
                                                            const float* wpsi, const float* dq, const float* pp,
                                                            const float* pc, float* part, int rows) {
  __shared__ float sh[4][4][256];   // [wave][sum][channel], Ci <= 256 (G <= 32 for the partial width)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = lane % G, c0 = sub * 8, slots = 256 / G;
  float gs[8], gb[8], xs[8], xb[8], gmu[8], giv[8], xmu[8], xiv[8], w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    gs[j] = gab[c]; gb[j] = gab[Ci + c]; xs[j] = xab[c]; xb[j] = xab[Ci + c];
    gmu[j] = gm[c]; giv[j] = gi[c]; xmu[j] = xm[c]; xiv[j] = xi[c]; w[j] = wpsi[c];
  }
  const float A = pc[0], B = pc[1], Cc = pc[2];
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  float a0[8], a1[8], a2[8], a3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { a0[j] = 0.f; a1[j] = 0.f; a2[j] = 0.f; a3[j] = 0.f; }
  // GV_U2 pixels per trip, loads first, summed in the one-pixel loop's order (bit-identical sums)
  for (long long q = p0 + tid / G; q < p1; q += GV_U2 * slots) {
    float g[GV_U2][8], x[GV_U2][8], dqv[GV_U2], ppv[GV_U2];
#pragma unroll
    for (int u = 0; u < GV_U2; ++u) {
      const long long qq = q + u * slots < p1 ? q + u * slots : q;
      load8<T>(gw + qq * Ci + c0, g[u]);
      load8<T>(xw + qq * Ci + c0, x[u]);
      dqv[u] = dq[qq];
      ppv[u] = pp[qq];
    }
#pragma unroll
    for (int u = 0; u < GV_U2; ++u) {
      if (q + u * slots >= p1) break;
      const float dp = A * dqv[u] + B * ppv[u] + Cc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = fmaxf(g[u][j] * gs[j] + gb[j] + x[u][j] * xs[j] + xb[j], 0.f);
        const float dz = a > 0.f ? dp * w[j] : 0.f;
        a0[j] += dz;
        a1[j] += dz * (g[u][j] - gmu[j]) * giv[j];
        a2[j] += dz * (x[u][j] - xmu[j]) * xiv[j];
        a3[j] += dp * a;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    for (int o = G; o < 64; o <<= 1) {
      a0[j] += __shfl_xor(a0[j], o, 64);
      a1[j] += __shfl_xor(a1[j], o, 64);
      a2[j] += __shfl_xor(a2[j], o, 64);
      a3[j] += __shfl_xor(a3[j], o, 64);
    }
    if (lane < G) {
      sh[wave][0][c0 + j] = a0[j];
      sh[wave][1][c0 + j] = a1[j];
      sh[wave][2][c0 + j] = a2[j];
      sh[wave][3][c0 + j] = a3[j];
    }
  }
  __syncthreads();
  if (tid < Ci) {
#pragma unroll
    for (int f = 0; f < 4; ++f)
      part[((size_t)f * rows + blockIdx.x) * Ci + tid] = ((sh[0][f][tid] + sh[1][f][tid]) + sh[2][f][tid]) + sh[3][f][tid];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void gate_bwd3_vec_kernel(long long P, int Ci, int G, const T* __restrict__ gw, const T* __restrict__ xw,
                                                            const float* gab, const float* xab, const float* wpsi,
                                                            const float* __restrict__ dq, const float* __restrict__ pp, const float* pc,
                                                            const float* gcoef, const float* xcoef, T* __restrict__ dgw, T* __restrict__ dxw,
                                                            int rows) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int sub = lane % G, c0 = sub * 8, slots = 256 / G;
  float gs[8], gb[8], xs[8], xb[8], w[8], gA[8], gB[8], gC[8], xA[8], xB[8], xC[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    gs[j] = gab[c]; gb[j] = gab[Ci + c]; xs[j] = xab[c]; xb[j] = xab[Ci + c]; w[j] = wpsi[c];
    gA[j] = gcoef[c]; gB[j] = gcoef[Ci + c]; gC[j] = gcoef[2 * Ci + c];
    xA[j] = xcoef[c]; xB[j] = xcoef[Ci + c]; xC[j] = xcoef[2 * Ci + c];
  }
  const float A = pc[0], B = pc[1], Cc = pc[2];
  const long long per = (P + rows - 1) / rows;
  const long long p0 = blockIdx.x * per, p1 = min(P, p0 + per);
  for (long long q = p0 + tid / G; q < p1; q += GV_U2 * slots) {
    float g[GV_U2][8], x[GV_U2][8], dqv[GV_U2], ppv[GV_U2];
#pragma unroll
    for (int u = 0; u < GV_U2; ++u) {
      const long long qq = q + u * slots < p1 ? q + u * slots : q;
      load8<T>(gw + qq * Ci + c0, g[u]);
      load8<T>(xw + qq * Ci + c0, x[u]);
      dqv[u] = dq[qq];
      ppv[u] = pp[qq];
    }
#pragma unroll
    for (int u = 0; u < GV_U2; ++u) {
      const long long qq = q + u * slots;
      if (qq >= p1) break;
      float og[8], ox[8];
      const float dp = A * dqv[u] + B * ppv[u] + Cc;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = fmaxf(g[u][j] * gs[j] + gb[j] + x[u][j] * xs[j] + xb[j], 0.f);
        const float dz = a > 0.f ? dp * w[j] : 0.f;
        og[j] = f32_rounded(__builtin_fmaf(gA[j], dz, __builtin_fmaf(gB[j], g[u][j], gC[j])));   // bn.hip's rounding
        ox[j] = f32_rounded(__builtin_fmaf(xA[j], dz, __builtin_fmaf(xB[j], x[u][j], xC[j])));
      }
      store8<T>(dgw + qq * Ci + c0, og);
      store8<T>(dxw + qq * Ci + c0, ox);
    }
  }
}

static bool gate_vec_ok(int Ci) {
  const int G = vec_group(Ci);
  return G && G <= 32 && !getenv("UNET_NO_GATE_VEC");
}

}  // namespace unet

using namespace unet;

extern "C" {

int unet_gate_psi_rows(long long P) { return pix_rows(P); }

int unet_gate_psi(int dtype, long long P, int Ci, const void* gw, const void* xw, const float* gab, const float* xab,
                  const float* wpsi, float* p, float* partial, void* stream) {
  const int rows = pix_rows(P);
  const int G = vec_group(Ci);
  if (G) {
    if (dtype == UNET_F16)
      hipLaunchKernelGGL(psi_vec_kernel<f16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, G,
                         (const f16*)gw, (const f16*)xw, gab, xab, wpsi, p, partial, rows);
    else if (dtype == UNET_BF16)
      hipLaunchKernelGGL(psi_vec_kernel<bf16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, G,
                         (const bf16*)gw, (const bf16*)xw, gab, xab, wpsi, p, partial, rows);
    else
      hipLaunchKernelGGL(psi_vec_kernel<float>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, G,
                         (const float*)gw, (const float*)xw, gab, xab, wpsi, p, partial, rows);
    return check_launch("gate_psi");
  }
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(psi_kernel<f16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, (const f16*)gw,
                       (const f16*)xw, gab, xab, wpsi, p, partial, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(psi_kernel<bf16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, (const bf16*)gw,
                       (const bf16*)xw, gab, xab, wpsi, p, partial, rows);
  else
    hipLaunchKernelGGL(psi_kernel<float>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, (const float*)gw,
                       (const float*)xw, gab, xab, wpsi, p, partial, rows);
  return check_launch("gate_psi");
}

int unet_gate_bwd1(int dtype, long long P, int Cx, const float* dxs, const void* yx, const float* sx, const float* bx,
                   int relu, const float* p, const float* psi_ab, const float* psi_mean, const float* psi_invstd, float* dx,
                   int dx_accum, float* dq, float* partial, void* stream) {
  const int rows = pix_rows(P);
  const int G = vec_group(Cx);
  if (G) {
    if (dtype == UNET_F16)
      hipLaunchKernelGGL(gate_bwd1_vec_kernel<f16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Cx, G, dxs,
                         (const f16*)yx, sx, bx, relu, p, psi_ab, psi_mean, psi_invstd, dx, dx_accum, dq, partial,
                         rows);
    else if (dtype == UNET_BF16)
      hipLaunchKernelGGL(gate_bwd1_vec_kernel<bf16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Cx, G, dxs,
                         (const bf16*)yx, sx, bx, relu, p, psi_ab, psi_mean, psi_invstd, dx, dx_accum, dq, partial,
                         rows);
    else
      hipLaunchKernelGGL(gate_bwd1_vec_kernel<float>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Cx, G, dxs,
                         (const float*)yx, sx, bx, relu, p, psi_ab, psi_mean, psi_invstd, dx, dx_accum, dq, partial,
                         rows);
    return check_launch("gate_bwd1");
  }
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(gate_bwd1_kernel<f16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Cx, dxs,
                       (const f16*)yx, sx, bx, relu, p, psi_ab, psi_mean, psi_invstd, dx, dx_accum, dq, partial, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(gate_bwd1_kernel<bf16>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Cx, dxs,
                       (const bf16*)yx, sx, bx, relu, p, psi_ab, psi_mean, psi_invstd, dx, dx_accum, dq, partial, rows);
  else
    hipLaunchKernelGGL(gate_bwd1_kernel<float>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Cx, dxs,
                       (const float*)yx, sx, bx, relu, p, psi_ab, psi_mean, psi_invstd, dx, dx_accum, dq, partial, rows);
  return check_launch("gate_bwd1");
}

int unet_gate_bwd2_rows(long long P, int Ci) { return rows_for(P, Ci); }

int unet_gate_bwd2(int dtype, long long P, int Ci, const void* gw, const void* xw, const float* gab, const float* xab,
                   const float* g_mean, const float* g_invstd, const float* x_mean, const float* x_invstd,
                   const float* wpsi, const float* dq, const float* p, const float* psi_coef, float* partial,
                   void* stream) {
  const int cl = chan_lanes_g(Ci), rows = rows_for(P, Ci);
  if (gate_vec_ok(Ci)) {
    const int G = vec_group(Ci);
#define UNET_G2V(TT)                                                                                                \
  hipLaunchKernelGGL(gate_bwd2_vec_kernel<TT>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, G, (const TT*)gw, \
                     (const TT*)xw, gab, xab, g_mean, g_invstd, x_mean, x_invstd, wpsi, dq, p, psi_coef, partial, rows)
    if (dtype == UNET_F16) UNET_G2V(f16);
    else if (dtype == UNET_BF16) UNET_G2V(bf16);
    else UNET_G2V(float);
#undef UNET_G2V
    return check_launch("gate_bwd2");
  }
  dim3 grid(cdiv(Ci, cl), rows);
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(gate_bwd2_kernel<f16>, grid, dim3(256), 0, (hipStream_t)stream, P, Ci, cl, (const f16*)gw,
                       (const f16*)xw, gab, xab, g_mean, g_invstd, x_mean, x_invstd, wpsi, dq, p, psi_coef, partial,
                       rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(gate_bwd2_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, P, Ci, cl, (const bf16*)gw,
                       (const bf16*)xw, gab, xab, g_mean, g_invstd, x_mean, x_invstd, wpsi, dq, p, psi_coef, partial,
                       rows);
  else
    hipLaunchKernelGGL(gate_bwd2_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, P, Ci, cl, (const float*)gw,
                       (const float*)xw, gab, xab, g_mean, g_invstd, x_mean, x_invstd, wpsi, dq, p, psi_coef, partial,
                       rows);
  return check_launch("gate_bwd2");
}

int unet_gate_bwd3(int dtype, long long P, int Ci, const void* gw, const void* xw, const float* gab, const float* xab,
                   const float* wpsi, const float* dq, const float* p, const float* psi_coef, const float* gcoef,
                   const float* xcoef, void* dgw, void* dxw, void* stream) {
  const int cl = chan_lanes_g(Ci), rows = rows_for(P, Ci);
  if (gate_vec_ok(Ci)) {
    const int G = vec_group(Ci);
#define UNET_G3V(TT)                                                                                                \
  hipLaunchKernelGGL(gate_bwd3_vec_kernel<TT>, dim3(rows), dim3(256), 0, (hipStream_t)stream, P, Ci, G, (const TT*)gw, \
                     (const TT*)xw, gab, xab, wpsi, dq, p, psi_coef, gcoef, xcoef, (TT*)dgw, (TT*)dxw, rows)
    if (dtype == UNET_F16) UNET_G3V(f16);
    else if (dtype == UNET_BF16) UNET_G3V(bf16);
    else UNET_G3V(float);
#undef UNET_G3V
    return check_launch("gate_bwd3");
  }
  dim3 grid(cdiv(Ci, cl), rows);
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(gate_bwd3_kernel<f16>, grid, dim3(256), 0, (hipStream_t)stream, P, Ci, cl, (const f16*)gw,
                       (const f16*)xw, gab, xab, wpsi, dq, p, psi_coef, gcoef, xcoef, (f16*)dgw, (f16*)dxw, rows);
  else if (dtype == UNET_BF16)
    hipLaunchKernelGGL(gate_bwd3_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, P, Ci, cl, (const bf16*)gw,
                       (const bf16*)xw, gab, xab, wpsi, dq, p, psi_coef, gcoef, xcoef, (bf16*)dgw, (bf16*)dxw, rows);
  else
    hipLaunchKernelGGL(gate_bwd3_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, P, Ci, cl, (const float*)gw,
                       (const float*)xw, gab, xab, wpsi, dq, p, psi_coef, gcoef, xcoef, (float*)dgw, (float*)dxw,
                       rows);
  return check_launch("gate_bwd3");
}

}  // extern "C"
