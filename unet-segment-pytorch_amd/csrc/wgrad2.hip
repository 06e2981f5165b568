// wgrad2.hip — pipelined bf16 weight gradient on MFMA (gfx950).
//
// dW[co][ci][tap] = Σ_pix dy[pix][co] · X[pix + off(tap)][ci]   (weight half of convolution_backward of
// nn.Conv2d, unet/models/layers.py:32,35,152,158; X = the conv input re-gathered through its unet_src
// descriptors exactly as the forward saw it).
//
// GEMM view: M = co, N = (tap, ci), K = pixels.  One workgroup = 4 waves (one per SIMD, up to 512
// VGPRs each) owns a BCO x BCI x 9 output block and walks a range of 8x16-pixel tiles (split-K):
//  * the dy tile [128 px][BCO] and the input halo [(8+2) x 18][BCI] are double-buffered in LDS; the
//    next tile's raw loads are issued before this tile's MFMAs and transformed/stored after them;
//  * each wave holds 64 co x 16 ci x 9 taps of fp32 accumulators (36 MFMA tiles); per 32-pixel K step
//    it reads 4 dy fragments (re-used by all 9 taps) and 9 halo fragments, all with the CDNA4
//    transposed LDS read ds_read_b64_tr_b16 (K runs along LDS rows);
//  * partial sums go to an fp32 slab per split in OIHW order; wgrad_reduce2 sums the slabs in a fixed
//    order (deterministic) with 16-byte accesses.
#include "halo_items.h"

namespace unet {

constexpr int W2_TH = 8, W2_TW = 16, W2_BM = 128;
constexpr int W2_RG = 32, W2_RG_MIN = 32;  // two-pass slab reduction above W2_RG_MIN splits
int slab_reduce_two_pass(const float* ws, int splits, long long total, float* scratch, float* dw, int accum,
                         hipStream_t st);  // pw.hip (W2_RG == PW_RG partial slabs)

template <typename T>
__device__ __forceinline__ typename Mma<T>::frag tr8(const T* r0, const T* r1) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(r0));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(r1));
  // one vector concatenation (lets the two reads land in the halves of one register quad; an element-wise
  // initialiser compiled to v_mov copies)
  return __builtin_bit_cast(typename Mma<T>::frag, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// compile-time source kinds of the conv input (as conv3's SK): W2_ANY switches per halo item at run time;
// W2_PLAIN: stored map(s) only; W2_ACT: BN(+ReLU)(+gate) source(s) and stored ones, decided per thread
// (a thread's channel vector has one source).  Known kinds keep only that staging code: a plain vector
// goes to LDS as loaded, an activated one is unpacked, transformed and packed once.
enum { W2_ANY = 0, W2_PLAIN = 1, W2_ACT = 2 };

template <typename T, int KS, int WCO, int WCI, int MI, int RAW, int SK = W2_ANY>
__global__ __launch_bounds__(64 * WCO * WCI) void wgrad2_kernel(const unet_wgrad_desc d, int tiles_w, int tiles_h, int mtiles,
                                                      int per_split, float* ws) {
  constexpr int W2_NT = 64 * WCO * WCI;
  constexpr int VEC = 8;
  constexpr int BCO = WCO * 16 * MI, BCI = WCI * 16;
  constexpr int HALO = (KS == 3) ? 1 : 0;
  constexpr int HWID = W2_TW + 2 * HALO, HHGT = W2_TH + 2 * HALO, HP = HWID * HHGT;
  // LDS row strides are odd multiples of 32 B (16 bf16): the 4 rows a 16-lane group reads in one
  // ds_read_b64_tr_b16 land on distinct 8-bank octets, and lane groups g = 1, 3 (which start 8 rows /
  // pixels further, i.e. a multiple of 64 banks) read their "+4" half first (see the main loop), so the
  // two groups served together hit disjoint octets: conflict-free
  constexpr int RSX = BCI + (BCI % 32 == 0 ? 16 : 32), RSD = BCO + 16;
  static_assert((RSX / 16) % 2 == 1 && (RSD / 16) % 2 == 1, "strides must be odd multiples of 32 B");
  constexpr int TAPS = KS * KS;
  constexpr int NVX = BCI / VEC, NVD = BCO / VEC;
  constexpr int IX = (HP * NVX + W2_NT - 1) / W2_NT;
  constexpr int ID = (W2_BM * NVD + W2_NT - 1) / W2_NT;
  constexpr int BUF = HP * RSX + W2_BM * RSD;
  static_assert(W2_NT % NVX == 0 && W2_NT % NVD == 0, "fixed channel vector per thread");
  __shared__ __attribute__((aligned(16))) T lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave / WCI, wci = wave % WCI;
  const int split = blockIdx.x;
  const int ci0 = blockIdx.y * BCI;
  const int co0 = blockIdx.z * BCO;
  const int mt_begin = split * per_split;
  const int mt_end = min(mtiles, mt_begin + per_split);

  // fixed per-thread channel vectors
  const int vx = tid % NVX, vd = tid % NVD;
  SrcView sv;
  float sc[VEC], sf[VEC];
  make_view<T>(d, ci0 + vx * VEC, sv, sc, sf);
  const int cod = co0 + vd * VEC;
  const bool dy_ok = cod < d.Cout;
  const char* dyb = (const char*)d.dy + (size_t)cod * sizeof(T);  // 32-bit offsets from here (host-checked)
  const unsigned dy_pixb = (unsigned)d.Cout * sizeof(T);

  auto tile_nhw = [&](int mt, long long& n, int& h0, int& w0) {
    const int tw_i = mt % tiles_w;
    const int t2 = mt / tiles_w;
    h0 = (t2 % tiles_h) * W2_TH;
    w0 = tw_i * W2_TW;
    n = t2 / tiles_h;
  };

  // staging of a tile, split into pieces so that only a few raw loads are in flight at once:
  //   dy vectors: issued at K-step 0, stored after K-step 1; halo item k: issued at K-step
  //   (3k / IX), stored after the following K-step (see the main loop)
  Item<SK == W2_ANY ? RAW : 1> xi[SK == W2_ANY ? IX : 1];
  uint4 dq[ID];
  // SK != W2_ANY: raw 16-byte vectors (zero outside the map), the gate pre-activation per item
  const bool act_src = SK == W2_ACT && (sv.kind == UNET_SRC_ACT);
  uint4 xq[IX];
  float xg[IX];
  auto issue_x = [&](long long n, int h0, int w0, int k) {
    const int hp = (tid + k * W2_NT) / NVX;
    const int y = h0 + hp / HWID - HALO, x = w0 + hp % HWID - HALO;
    if constexpr (SK == W2_ANY) {
      item_issue<T, RAW>(sv, d.H, d.W, n, y, x, hp < HP, xi[k]);
    } else {
      xq[k] = make_uint4(0, 0, 0, 0);
      xg[k] = 0.f;
      if (hp < HP && sv.fast && y >= 0 && y < d.H && x >= 0 && x < d.W) {
        const unsigned px = ((unsigned)n * d.H + y) * d.W + x;
        xq[k] = ld16b(sv.base, px * sv.pixb);
        if (act_src && sv.gate_p) xg[k] = sv.gate_p[px];
      }
    }
  };
  auto finish_x = [&](long long n, int h0, int w0, int k, T* buf) {
    const int hp = (tid + k * W2_NT) / NVX;
    if (hp < HP) {
      if constexpr (SK == W2_ANY) {
        float vals[VEC];
        item_finish<T, RAW>(d, sv, sc, sf, n, h0 + hp / HWID - HALO, w0 + hp % HWID - HALO, ci0 + vx * VEC, xi[k],
                            vals);
        store_vec<T>(buf + hp * RSX + vx * VEC, vals);
      } else {
        uint4 o = xq[k];
        if (act_src) {
          // zero-padding positions stay zero (the conv pads the activation, not y)
          const int y = h0 + hp / HWID - HALO, x = w0 + hp % HWID - HALO;
          const bool inb = sv.fast && y >= 0 && y < d.H && x >= 0 && x < d.W;
          float v[VEC];
          unpack16<T>(o, v);
          const float lo = sv.relu ? 0.f : -INFINITY;
          const float gm = sv.gate_p ? sigmoidf_(xg[k] * sv.gate_ab[0] + sv.gate_ab[1]) : 1.f;
#pragma unroll
          for (int j = 0; j < VEC; ++j) v[j] = inb ? fmaxf(__builtin_fmaf(v[j], sc[j], sf[j]), lo) * gm : 0.f;
          o = pack8_16<T>(v);
        }
        *reinterpret_cast<uint4*>(buf + hp * RSX + vx * VEC) = o;
      }
    }
  };
  auto issue_d = [&](long long n, int h0, int w0) {
#pragma unroll
    for (int k = 0; k < ID; ++k) {
      const int p = (tid + k * W2_NT) / NVD;
      const int oh = h0 + p / W2_TW, ow = w0 + p % W2_TW;
      dq[k] = make_uint4(0, 0, 0, 0);
      if (dy_ok && p < W2_BM && oh < d.H && ow < d.W)
        dq[k] = ld16b(dyb, (((unsigned)n * d.H + oh) * d.W + ow) * dy_pixb);
    }
  };
  auto finish_d = [&](T* buf) {
    T* bd = buf + HP * RSX;
#pragma unroll
    for (int k = 0; k < ID; ++k) {
      const int p = (tid + k * W2_NT) / NVD;
      // pixels of odd 8-blocks swap their 4-halves (the K permutation the halo reads apply, see below)
      if (p < W2_BM) *reinterpret_cast<uint4*>(bd + (p ^ ((p & 8) >> 1)) * RSD + vd * VEC) = dq[k];
    }
  };
  auto issue = [&](long long n, int h0, int w0) {
#pragma unroll
    for (int k = 0; k < IX; ++k) issue_x(n, h0, w0, k);
    issue_d(n, h0, w0);
  };
  auto finish = [&](long long n, int h0, int w0, T* buf) {
#pragma unroll
    for (int k = 0; k < IX; ++k) finish_x(n, h0, w0, k, buf);
    finish_d(buf);
  };

  f32x4 acc[TAPS][MI];
#pragma unroll
  for (int t = 0; t < TAPS; ++t)
#pragma unroll
    for (int i = 0; i < MI; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (mt_begin < mt_end) {
    long long n;
    int h0, w0;
    tile_nhw(mt_begin, n, h0, w0);
    issue(n, h0, w0);
    finish(n, h0, w0, lds);
  }
  __syncthreads();

  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
  for (int mt = mt_begin; mt < mt_end; ++mt) {
    const int cur = (mt - mt_begin) & 1;
    const T* bx = lds + cur * BUF;
    const T* bd = bx + HP * RSX;
    const bool has_next = mt + 1 < mt_end;
    T* nb = lds + (cur ^ 1) * BUF;
    long long nn = 0;   // the next tile's coordinates, once per tile
    int nh0 = 0, nw0 = 0;
    if (has_next) tile_nhw(mt + 1, nn, nh0, nw0);
#pragma unroll
    for (int k0 = 0; k0 < W2_BM; k0 += 32) {
      const int s = k0 / 32;  // K step 0..3
      // next tile's raw loads: all issued at K-step 0 (x) / 1 (dy) and consumed after K-steps 2-3,
      // so two to three K-steps of MFMAs cover their latency
      // (RAW=4 sources keep the shorter one-K-step window: their 4-corner loads and max/bilinear
      // transforms measured faster spread over all four K-steps)
      if (has_next) {
        if constexpr (RAW == 1) {
          if (s == 0) {
#pragma unroll
            for (int k = 0; k < IX; ++k) issue_x(nn, nh0, nw0, k);
          }
          if (s == 1) issue_d(nn, nh0, nw0);
        } else {
          if (s == 0) issue_d(nn, nh0, nw0);
#pragma unroll
          for (int k = 0; k < IX; ++k)
            if ((3 * k) / IX == s) issue_x(nn, nh0, nw0, k);
        }
      }
      // lane bases + compile-time offsets (so every LDS read is base + immediate): this lane addresses
      // pixel rows pa = k0 + 8g + q and pa + 4; pixel pa sits at tile row 2s + (g>>1), column 8(g&1) + q.
      // Odd lane groups take the pa + 4 half as fragment elements 0..3 (bank spread, see RSX/RSD); A and
      // B use the same K permutation (for dy it is built into the LDS row order by finish_d), so the
      // products summed by the MFMA are unchanged.
      const int sw = (g & 1) * 4;
      const T* dl = bd + (8 * g + q) * RSD + wco * 16 * MI + p4;
      const T* xl0 = bx + ((g >> 1) * HWID + 8 * (g & 1) + q + sw) * RSX + wci * 16 + p4;
      const T* xl1 = bx + ((g >> 1) * HWID + 8 * (g & 1) + q + 4 - sw) * RSX + wci * 16 + p4;
      typename Mma<T>::frag a[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = tr8(dl + k0 * RSD + i * 16, dl + (k0 + 4) * RSD + i * 16);
#pragma unroll
      for (int t = 0; t < TAPS; ++t) {
        const int dy = t / KS, dx = t % KS;
        const int off = ((2 * s + dy) * HWID + dx) * RSX;
        const typename Mma<T>::frag b = tr8(xl0 + off, xl1 + off);
#pragma unroll
        for (int i = 0; i < MI; ++i) acc[t][i] = Mma<T>::mma(a[i], b, acc[t][i]);
      }
      if (has_next) {
        if constexpr (RAW == 1) {
#pragma unroll
          for (int k = 0; k < IX; ++k)
            if (s == 2 + (k * 2) / IX) finish_x(nn, nh0, nw0, k, nb);
          if (s == 3) finish_d(nb);
        } else {
          if (s == 1) finish_d(nb);
#pragma unroll
          for (int k = 0; k < IX; ++k)
            if ((3 * k) / IX + 1 == s) finish_x(nn, nh0, nw0, k, nb);
        }
      }
    }
    __syncthreads();
  }

  // slab (OIHW order): ws[split][co][ci][tap]; C layout: row (co) = 4*(l>>4)+r, col (ci) = l&15
  float* slab = ws + (size_t)split * d.Cout * d.Cin * TAPS;
  const int ci = ci0 + wci * 16 + (lane & 15);
  const int cob = co0 + wco * 16 * MI + 4 * (lane >> 4);
  const unsigned row = (unsigned)d.Cin * TAPS;   // slab elements per output channel
  const unsigned base = ((unsigned)cob * d.Cin + ci) * TAPS;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = cob + i * 16 + r;
      if (co < d.Cout && ci < d.Cin) {
        float* o = slab + base + (unsigned)(i * 16 + r) * row;
#pragma unroll
        for (int t = 0; t < TAPS; ++t) o[t] = acc[t][i][r];
      }
    }
}

// dw (+)= Σ_s ws[s]   (fixed order; 16-byte accesses when the size allows)
__global__ void wgrad_reduce2_kernel(const float* ws, int splits, long long total, float* dw, int accum) {
  if ((total & 3) == 0) {
    const long long n4 = total / 4;
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n4; e += (long long)gridDim.x * blockDim.x) {
      float4 s = reinterpret_cast<const float4*>(ws)[e];
      // 4 slabs per trip, loads first, adds in slab order (the same sums): a one-slab loop was a memory round
      // trip per slab (8 slabs: 11.7 us per launch, round-5 trace)
      int k = 1;
      for (; k + 3 < splits; k += 4) {
        const float4 v0 = reinterpret_cast<const float4*>(ws + (size_t)k * total)[e];
        const float4 v1 = reinterpret_cast<const float4*>(ws + (size_t)(k + 1) * total)[e];
        const float4 v2 = reinterpret_cast<const float4*>(ws + (size_t)(k + 2) * total)[e];
        const float4 v3 = reinterpret_cast<const float4*>(ws + (size_t)(k + 3) * total)[e];
        s.x += v0.x; s.y += v0.y; s.z += v0.z; s.w += v0.w;
        s.x += v1.x; s.y += v1.y; s.z += v1.z; s.w += v1.w;
        s.x += v2.x; s.y += v2.y; s.z += v2.z; s.w += v2.w;
        s.x += v3.x; s.y += v3.y; s.z += v3.z; s.w += v3.w;
      }
      for (; k < splits; ++k) {
        const float4 v = reinterpret_cast<const float4*>(ws + (size_t)k * total)[e];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      float4* o = reinterpret_cast<float4*>(dw) + e;
      if (accum) {
        const float4 a = *o;
        s.x += a.x; s.y += a.y; s.z += a.z; s.w += a.w;
      }
      *o = s;
    }
  } else {
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
      float s = ws[e];
      for (int k = 1; k < splits; ++k) s += ws[(size_t)k * total + e];
      dw[e] = accum ? dw[e] + s : s;
    }
  }
}

// dw (+)= the fixed-order sum of `splits` slabs of `total` floats
int wgrad_reduce2_launch(const float* ws, int splits, long long total, float* dw, int accum, hipStream_t st) {
  long long blocks = (total / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(wgrad_reduce2_kernel, dim3((int)blocks), dim3(256), 0, st, ws, splits, total, dw, accum);
  return check_launch("wgrad_reduce2");
}

struct W2Plan {
  bool ok;
  int wco, wci, mi, raw, tiles_w, tiles_h, mtiles, splits, per_split;
  size_t ws_bytes;
};

W2Plan wgrad2_plan(const unet_wgrad_desc* d) {
  W2Plan p{};
  p.ok = d->dtype != UNET_F32 && (d->Cout % 8) == 0;
  p.raw = 1;
  for (int i = 0; i < d->nsrc; ++i) {
    const unet_src& s = d->src[i];
    if (s.kind == UNET_SRC_NCHW_F32 || (s.C % 8)) p.ok = false;
    if ((double)d->N * s.H * s.W * s.C * 2 >= 4294967296.0) p.ok = false;  // 32-bit byte offsets
    if (s.kind == UNET_SRC_POOL_ACT || s.kind == UNET_SRC_UP_ACT) p.raw = 4;
  }
  if ((double)d->N * d->H * d->W * d->Cout * 2 >= 4294967296.0) p.ok = false;
  if (!p.ok) return p;
  // 8 waves (2 per SIMD: one wave's staging VALU runs beside the other's MFMAs) when Cin fills BCI=64
  // wave tile = (16*MI co) x 16 ci x k*k taps.  3x3, Cout > 64: 8 waves of 32co (2 per SIMD, so one
  // wave's staging VALU runs beside the other's MFMAs; 72 accumulators fit the 256-VGPR budget)
  // (RAW=4 sources keep 4 waves: their staging registers do not fit beside 72 accumulators at 2/SIMD)
  if (d->Cout <= 64 && d->ksize == 3 && p.raw == 1) { p.wco = 2; p.wci = 4; p.mi = 2; }
  else if (d->Cout <= 64) { p.wco = 1; p.wci = 4; p.mi = 4; }
  else if (d->ksize == 3 && p.raw == 1) { p.wco = 4; p.wci = 2; p.mi = 2; }
  else if (d->Cin >= 64) { p.wco = 2; p.wci = 4; p.mi = 4; }
  else { p.wco = 2; p.wci = 2; p.mi = 4; }
  const int bco = p.wco * 16 * p.mi, bci = p.wci * 16;
  p.tiles_w = cdiv(d->W, W2_TW);
  p.tiles_h = cdiv(d->H, W2_TH);
  p.mtiles = d->N * p.tiles_w * p.tiles_h;
  const long long tiles_out = (long long)cdiv(d->Cout, bco) * cdiv(d->Cin, bci);
  const size_t slab = (size_t)d->Cout * d->Cin * d->ksize * d->ksize * sizeof(float);
  // one resident workgroup per CU (LDS 98-131 KB): aim for at least one wave of 256 blocks; the slab
  // traffic (written once, read once by wgrad_reduce2, ~25 us per 150 MB) is capped at 160 MB
  long long s = (256 + tiles_out - 1) / tiles_out;
  const long long cap = (long long)(((size_t)160 << 20) / (slab ? slab : 1));
  if (s > cap) s = cap;
  if (s > p.mtiles) s = p.mtiles;
  if (s < 1) s = 1;
  p.per_split = cdiv(p.mtiles, s);
  p.splits = cdiv(p.mtiles, p.per_split);
  // + room for the partial slabs of the two-pass reduction (many splits of a small weight tensor)
  p.ws_bytes = slab * (p.splits + (p.splits > W2_RG_MIN ? W2_RG : 0));
  return p;
}

template <typename T, int KS, int WCO, int WCI, int MI, int RAW, int SK = W2_ANY>
static int launch_w2(const unet_wgrad_desc* d, const W2Plan& p, hipStream_t st) {
  dim3 grid(p.splits, cdiv(d->Cin, WCI * 16), cdiv(d->Cout, WCO * 16 * MI));
  hipLaunchKernelGGL((wgrad2_kernel<T, KS, WCO, WCI, MI, RAW, SK>), grid, dim3(64 * WCO * WCI), 0, st, *d, p.tiles_w, p.tiles_h, p.mtiles,
                     p.per_split, (float*)d->workspace);
  return check_launch("wgrad2");
}

// the W2 source-kind specialisation a raw-1 descriptor can use
static int w2_source_kinds(const unet_wgrad_desc* d) {
  bool plain = true, ok = true;
  for (int i = 0; i < d->nsrc; ++i) {
    const unet_src& s = d->src[i];
    if (s.kind == UNET_SRC_ACT) plain = false;
    else if (s.kind != UNET_SRC_PLAIN || s.gate_p) ok = false;
  }
  return !ok ? W2_ANY : (plain ? W2_PLAIN : W2_ACT);
}

template <typename T, int KS, int RAW>
static int launch_w2_cfg(const unet_wgrad_desc* d, const W2Plan& p, hipStream_t st) {
  if (p.wco == 1) return launch_w2<T, KS, 1, 4, 4, RAW>(d, p, st);
  if constexpr (KS == 3 && RAW == 1) {
    const int sk = w2_source_kinds(d);
    if (p.wco == 4) {
      if (sk == W2_PLAIN) return launch_w2<T, KS, 4, 2, 2, RAW, W2_PLAIN>(d, p, st);
      if (sk == W2_ACT) return launch_w2<T, KS, 4, 2, 2, RAW, W2_ACT>(d, p, st);
      return launch_w2<T, KS, 4, 2, 2, RAW>(d, p, st);
    }
    if (p.wco == 2 && p.mi == 2) {
      if (sk == W2_PLAIN) return launch_w2<T, KS, 2, 4, 2, RAW, W2_PLAIN>(d, p, st);
      if (sk == W2_ACT) return launch_w2<T, KS, 2, 4, 2, RAW, W2_ACT>(d, p, st);
      return launch_w2<T, KS, 2, 4, 2, RAW>(d, p, st);
    }
  }
  if constexpr (KS == 1) {
    if (p.wci == 4) return launch_w2<T, KS, 2, 4, 4, RAW>(d, p, st);
  }
  return launch_w2<T, KS, 2, 2, 4, RAW>(d, p, st);
}

int launch_wgrad2(const unet_wgrad_desc* d, const W2Plan& p, hipStream_t st) {
  int e;
  if (d->dtype == UNET_F16) {
    if (d->ksize == 3) e = p.raw == 4 ? launch_w2_cfg<f16, 3, 4>(d, p, st) : launch_w2_cfg<f16, 3, 1>(d, p, st);
    else e = p.raw == 4 ? launch_w2_cfg<f16, 1, 4>(d, p, st) : launch_w2_cfg<f16, 1, 1>(d, p, st);
  } else {
    if (d->ksize == 3) e = p.raw == 4 ? launch_w2_cfg<bf16, 3, 4>(d, p, st) : launch_w2_cfg<bf16, 3, 1>(d, p, st);
    else e = p.raw == 4 ? launch_w2_cfg<bf16, 1, 4>(d, p, st) : launch_w2_cfg<bf16, 1, 1>(d, p, st);
  }
  if (e) return e;
  const long long total = (long long)d->Cout * d->Cin * d->ksize * d->ksize;
  if (p.splits > W2_RG_MIN && (total & 3) == 0) {
    // two fixed-order passes (splits -> W2_RG groups -> 1): one serial loop of hundreds of slabs per
    // 16-byte column would leave the reduction latency-bound for small weights (e.g. 64x64x3x3)
    return slab_reduce_two_pass((const float*)d->workspace, p.splits, total,
                                (float*)d->workspace + (size_t)p.splits * total, d->dw, d->accum, st);
  }
  return wgrad_reduce2_launch((const float*)d->workspace, p.splits, total, d->dw, d->accum, st);
}

// entry points used by wgrad.hip (which keeps the generic kernel for fp32 / odd channel counts)
bool wgrad2_eligible(const unet_wgrad_desc* d, size_t* ws_bytes) {
  const W2Plan p = wgrad2_plan(d);
  if (p.ok && ws_bytes) *ws_bytes = p.ws_bytes;
  return p.ok;
}
int wgrad2_run(const unet_wgrad_desc* d, hipStream_t st) { return launch_wgrad2(d, wgrad2_plan(d), st); }

}  // namespace unet
