// wgrad5.hip — 3x3 weight gradient (bf16 / fp16) for gfx950 with an LDS-DMA operand pipeline.
//
// dW[co][ci][tap] = Σ_pix dy[pix][co] · X[pix + off(tap)][ci]   (the weight half of convolution_backward of
// nn.Conv2d(k=3, pad=1), unet/models/layers.py:32,35; X = the conv input rebuilt from its unet_src
// descriptors exactly as the forward saw it: BN-apply + ReLU (+ attention gate) of a stored pre-BN map, or
// the stored map itself, the up-block concat as two sources).
//
// Why: wgrad2 stages its operands through registers (global load -> VGPR -> transform -> ds_write) one tile
// ahead; its dominant instantiations spend 36 % of their wave cycles parked on s_waitcnt / barriers and 11 %
// on LDS issue (profiles/r02_end_conv3_wgrad2_pmc.txt).  Here, as in conv5.hip, every operand reaches LDS by
// buffer_load ... lds, issued TWO pixel stages ahead, with one hand-counted vmcnt wait and one barrier per
// stage:
//  * stage = TH=2 rows x 32 pixels of dy (the GEMM's K) and the (TH+2) x 34 input halo those rows need;
//  * GEMM: M = co, N = (tap, ci), K = pixels, on v_mfma_f32_16x16x32 (K = one 32-pixel row); wave tile
//    64 co x 16 ci x 9 taps (36 accumulators of 4 fp32): per K step 4 dy fragments and 9 halo fragments,
//    each two ds_read_b64_tr_b16 (the transposed read turns the NHWC pixel rows into K-major fragments);
//  * LDS images: one pixel = BCO/8 (dy) or BCI/8 (halo) 16-byte channel units, permuted within the pixel by
//    an XOR of the pixel's column (w5_swz), which makes every transposed read bank-conflict free (a half-wave
//    reads columns x0 + {0..3, 8..11} of one row, two adjacent units each) while keeping the row offset a
//    compile-time constant;
//  * a BN-activation source lands in a raw ring and is transformed (BN-apply, ReLU, gate, zero padding)
//    slot for slot by the lane that loaded it one stage ahead (conv5's scheme);
//  * persistent split-K: a block walks a contiguous range of stages and writes one fp32 slab; the slabs are
//    summed in a fixed order afterwards (deterministic, as wgrad2).
// Block = 8 waves = WCO (64-co groups) x WCI (16-ci groups) x WK (K halves: the rows of a stage); with
// WK = 2 the two halves' accumulators are summed through LDS before the slab store.
#include "conv_src16.h"
#include "lds_dma.h"

namespace unet {

constexpr int W5_TW = 32, W5_HW = 34, W5_NW = 8, W5_NT = 512;
int slab_reduce_two_pass(const float* ws, int splits, long long total, float* scratch, float* dw, int accum,
                         hipStream_t st);                                                   // pw.hip
int wgrad_reduce2_launch(const float* ws, int splits, long long total, float* dw, int accum, hipStream_t st);  // wgrad2.hip
constexpr int W5_RG = 32, W5_RG_MIN = 32;   // as wgrad2: slab reduction scratch above 32 splits
constexpr int W5_ACT_NG = 4;   // SK value of wgrad5 only: BN-activation source without the attention gate

// XOR permutation of the 16-byte channel units of a pixel in column x (UPP units per pixel): the 8 columns a
// half-wave's transposed read touches (x0 + {0..3, 8..11}) x 2 adjacent units land on 16 distinct bank
// quads.  UPP = 16: bank quad = unit ^ swz; UPP = 8: two pixels share the 16 quads, x & 1 picks the half.
template <int UPP>
__device__ __forceinline__ int w5_swz(int x) {
  static_assert(UPP == 8 || UPP == 16, "8 or 16 units per pixel");
  if constexpr (UPP == 16) return 2 * ((x & 3) | ((x >> 1) & 4));
  else return 2 * ((x >> 1) & 1) + 4 * ((x >> 3) & 1);
}

template <int TH, int UPPD, int UPPX, bool ACT, bool GT = ACT>
struct W5Layout {
  static constexpr int DUN = TH * W5_TW * UPPD;        // dy image: 16-byte units
  static constexpr int NID = DUN / 64;                     // DMA instructions per dy image (exact)
  static constexpr int XPIX = (TH + 2) * W5_HW;
  static constexpr int XUN = XPIX * UPPX;
  static constexpr int NIX = (XUN + 63) / 64;
  static constexpr int DPWD = (NID + W5_NW - 1) / W5_NW, DPWX = (NIX + W5_NW - 1) / W5_NW;
  static constexpr int DIMG = NID * 1024, XIMG = NIX * 1024;
  static constexpr int NCX = ACT ? 2 : 3;                  // compute-image ring of the halo
  // gate pre-activations: per wave one 64-lane DMA of the (<= 8 per instruction) pixels its halo slots cover
  static constexpr int GATE = W5_NW * 256;
  static constexpr int OFF_D = 0;
  static constexpr int OFF_X = OFF_D + 3 * DIMG;
  static constexpr int OFF_RAW = OFF_X + NCX * XIMG;
  static constexpr int OFF_GATE = OFF_RAW + (ACT ? 2 * XIMG : 0);
  static constexpr int OFF_TAB = OFF_GATE + (GT ? 2 * GATE : 0);
  static constexpr int OFF_JUNK = OFF_TAB + (ACT ? 2 * UPPX * 8 * 4 : 0);
  static constexpr int BYTES = OFF_JUNK + 1024;
  static_assert(BYTES <= 160 * 1024, "LDS");
};

template <typename T>
__device__ __forceinline__ typename Mma<T>::frag w5_tr8(const unsigned char* r0, const unsigned char* r1) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(r0));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(r1));
  return __builtin_bit_cast(typename Mma<T>::frag, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// SK: SK_PLAIN (every source stored), SK_ACT (src0 a BN activation, optionally gated; src1 stored) or W5_ACT_NG
// (an ungated BN activation: no gate ring in LDS)
template <typename T, int WCO, int WK, int SK, int TH>
__global__ __launch_bounds__(W5_NT, 1) void wgrad5_kernel(const unet_wgrad_desc d, int mtiles, int per_split,
                                                         float* ws) {
  constexpr int WCI = W5_NW / (WCO * WK);
  constexpr int BCO = 64 * WCO, BCI = 16 * WCI;
  constexpr int UPPD = BCO / 8, UPPX = BCI / 8;
  constexpr bool ACT = SK != SK_PLAIN, GT = SK == SK_ACT;
  using Lay = W5Layout<TH, UPPD, UPPX, ACT, GT>;
  constexpr int NID = Lay::NID, NIX = Lay::NIX, DPWD = Lay::DPWD, DPWX = Lay::DPWX;
  constexpr int KPW = TH / WK;            // K steps (rows) per wave per stage
  constexpr int ND0 = DPWD + DPWX;           // DMA instructions per wave per stage (+ DPWX gate loads)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[Lay::BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave % WK, wci = (wave / WK) % WCI, wco = wave / (WK * WCI);
  const int ci0 = blockIdx.y * BCI, co0 = blockIdx.z * BCO;
  const int mt0 = blockIdx.x * per_split;
  const int ntl = min(mtiles, mt0 + per_split) - mt0;     // stages of this block (host: >= 1)

  // ---- the block's input channels: one source (the concat's sources hold multiples of BCI channels) ----
  const unet_src& s0 = d.src[0];
  const unet_src& s1 = d.src[1];
  const int C0 = s0.C;
  const bool in1 = d.nsrc > 1 && ci0 >= C0;
  const int cl0 = in1 ? ci0 - C0 : ci0;
  const int Cs = in1 ? s1.C : C0;
  const bool xact = ACT && !in1;
  const bool gated = GT && xact && s0.gate_p != nullptr;
  const long long npix = (long long)d.N * d.H * d.W;
  const rsrc4_t rsx = mk_rsrc4(in1 ? s1.data : s0.data, (unsigned)(npix * Cs * 2));
  const rsrc4_t rsd = mk_rsrc4(d.dy, (unsigned)(npix * d.Cout * 2));
  const rsrc4_t rsg = mk_rsrc4(gated ? (const void*)s0.gate_p : d.dy, (unsigned)(npix * 4));
  float ga = 0.f, gb = 0.f;
  if (gated) { ga = s0.gate_ab[0]; gb = s0.gate_ab[1]; }
  if constexpr (ACT) {
    // scale / shift of the block's BCI channels (ordinary loads, before any DMA is in flight)
    float* tab = reinterpret_cast<float*>(lds + Lay::OFF_TAB);
    if (tid < BCI) {
      tab[tid] = xact ? s0.scale[cl0 + tid] : 1.f;
      tab[BCI + tid] = xact ? s0.shift[cl0 + tid] : 0.f;
    }
  }

  // ---- this lane's DMA slots (instruction i = wave + k * 8 covers units 64 i .. 64 i + 63 of an image):
  // row / column of the unit's pixel relative to the stage origin and its channel offset.  Every wave issues
  // the same compile-time number of DMAs per stage; instructions past an image go to a junk slot and units
  // past it load out of range (zeros), so each wait is an immediate vmcnt.
  int drow[DPWD], dcol[DPWD], dch[DPWD];
#pragma unroll
  for (int k = 0; k < DPWD; ++k) {
    const int u = (wave + k * W5_NW) * 64 + lane;
    const int p = u / UPPD, x = p % W5_TW;
    drow[k] = u < Lay::DUN ? p / W5_TW : -(1 << 16);
    dcol[k] = x;
    dch[k] = 8 * ((u % UPPD) ^ w5_swz<UPPD>(x));
  }
  int xrow[DPWX], xcol[DPWX], xch[DPWX];
#pragma unroll
  for (int k = 0; k < DPWX; ++k) {
    const int u = (wave + k * W5_NW) * 64 + lane;
    const int hp = u / UPPX, hx = hp % W5_HW;
    xrow[k] = u < Lay::XUN ? hp / W5_HW - 1 : -(1 << 16);
    xcol[k] = hx - 1;
    xch[k] = 8 * ((u % UPPX) ^ w5_swz<UPPX>(hx));
  }

  // the gate DMA lane: lane 8k + p loads the pre-activation of pixel p of this wave's k-th halo instruction
  // (instruction i = wave + 8k covers units 64 i .. 64 i + 63, i.e. pixels 8 i .. 8 i + 7 at 8 units per pixel)
  static_assert(!GT || UPPX == 8, "gate layout assumes 8 units per halo pixel");
  int grow, gcol;
  {
    const int k = lane >> 3, i = wave + k * W5_NW, hp = 8 * i + (lane & 7);
    const bool v = k < DPWX && i < NIX && hp < Lay::XPIX;
    grow = v ? hp / W5_HW - 1 : -(1 << 16);
    gcol = hp % W5_HW - 1;
  }

  // ---- transposed-read addresses (bytes inside an image; + row * row stride as an immediate) ----
  // lane 4q+p of 16-lane group g supplies row q (pixel column 8g + q, + 4 for the second read) and channels
  // 4p .. 4p+3 of the fragment's 16: unit (p >> 1), byte 8 (p & 1) inside it
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  unsigned aoff[2][4], boff[2][3];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int x = 8 * g + 4 * h + q;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int u = wco * 8 + 2 * f + (pp >> 1);
      aoff[h][f] = (unsigned)(x * UPPD + (u ^ w5_swz<UPPD>(x))) * 16u + 8u * (pp & 1);
    }
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int hx = x + dx;
      const int u = wci * 2 + (pp >> 1);
      boff[h][dx] = (unsigned)(hx * UPPX + (u ^ w5_swz<UPPX>(hx))) * 16u + 8u * (pp & 1);
    }
  }
  constexpr unsigned DROW = W5_TW * UPPD * 16, XROW = W5_HW * UPPX * 16;

  const unsigned l32 = lds_addr(lds);
  const unsigned junk = l32 + Lay::OFF_JUNK;

  // a stage cursor: origin (n, h0, w0) and ring slots (chunk % 3, chunk & 1)
  struct Cur {
    int t, n, h0, w0, s3, s2;
  };
  auto cur_init = [&](Cur& c) {
    const int mt = mt0;
    const int tiles_w = (d.W + W5_TW - 1) / W5_TW, tiles_h = (d.H + TH - 1) / TH;
    c.t = 0; c.s3 = 0; c.s2 = 0;
    c.w0 = (mt % tiles_w) * W5_TW;
    const int t2 = mt / tiles_w;
    c.h0 = (t2 % tiles_h) * TH;
    c.n = t2 / tiles_h;
  };
  auto cur_next = [&](Cur& c) {
    ++c.t;
    c.s3 = c.s3 == 2 ? 0 : c.s3 + 1;
    c.s2 ^= 1;
    c.w0 += W5_TW;
    if (c.w0 >= d.W) {
      c.w0 = 0;
      c.h0 += TH;
      if (c.h0 >= d.H) { c.h0 = 0; ++c.n; }
    }
  };

  // DMAs of the stage at cursor c: dy rows, halo (+ the gate pre-activation of each halo slot's pixel)
  auto issue = [&](const Cur& c) {
    const unsigned pb = ((unsigned)c.n * d.H + c.h0) * d.W + c.w0;
    const unsigned dimg = l32 + Lay::OFF_D + c.s3 * Lay::DIMG;
#pragma unroll
    for (int k = 0; k < DPWD; ++k) {
      const int i = wave + k * W5_NW;
      const int y = c.h0 + drow[k], x = c.w0 + dcol[k];
      const bool ok = ((unsigned)y < (unsigned)d.H) & (x < d.W);
      const unsigned pix = pb + (unsigned)(drow[k] * d.W + dcol[k]);
      dma16(rsd, i < NID ? dimg + i * 1024 : junk, ok ? (pix * (unsigned)d.Cout + (unsigned)(co0 + dch[k])) * 2u : OOB);
    }
    const unsigned ximg = l32 + (ACT ? Lay::OFF_RAW + c.s2 * Lay::XIMG : Lay::OFF_X + c.s3 * Lay::XIMG);
#pragma unroll
    for (int k = 0; k < DPWX; ++k) {
      const int i = wave + k * W5_NW;
      const int y = c.h0 + xrow[k], x = c.w0 + xcol[k];
      const bool ok = ((unsigned)y < (unsigned)d.H) & ((unsigned)x < (unsigned)d.W);
      const unsigned pix = pb + (unsigned)(xrow[k] * d.W + xcol[k]);
      dma16(rsx, i < NIX ? ximg + i * 1024 : junk, ok ? (pix * (unsigned)Cs + (unsigned)(cl0 + xch[k])) * 2u : OOB);
    }
    if (gated) {
      const int y = c.h0 + grow, x = c.w0 + gcol;
      const bool ok = ((unsigned)y < (unsigned)d.H) & ((unsigned)x < (unsigned)d.W);
      const unsigned pix = pb + (unsigned)(grow * d.W + gcol);
      dma4(rsg, l32 + Lay::OFF_GATE + c.s2 * Lay::GATE + wave * 256, ok ? pix * 4u : OOB);
    }
  };

  // BN-activation (+gate) transform of the halo at cursor c, raw -> compute image, this lane's own slots
  // (zero padding and the image's tail come out 0; a block on the stored concat source copies).  Packed as in
  // conv5.hip: v_pk_fma_f32 / v_pk_mul_f32 on channel pairs, ReLU as v_pk_max_i16 against 0 after the 16-bit
  // rounding (the same bits up to the sign of zero); slots past the image use the junk region (no branch)
  typedef __attribute__((ext_vector_type(2))) float f2_t;
  typedef __attribute__((ext_vector_type(2))) short s2_t;
  const s2_t lo2 = s0.relu ? s2_t{0, 0} : s2_t{-32768, -32768};
  auto transform = [&](const Cur& c) {
    const unsigned char* rb = lds + Lay::OFF_RAW + c.s2 * Lay::XIMG;
    unsigned char* cb = lds + Lay::OFF_X + c.s2 * Lay::XIMG;
    const float* tab = reinterpret_cast<const float*>(lds + Lay::OFF_TAB);
#pragma unroll
    for (int k = 0; k < DPWX; ++k) {
      const int i = wave + k * W5_NW;
      const bool live = i < NIX;
      const int s = i * 64 + lane;
      const unsigned so = live ? (unsigned)s * 16u : (unsigned)(Lay::OFF_JUNK + lane * 16);
      uint4 q4 = *reinterpret_cast<const uint4*>((live ? rb : lds) + so);
      if (xact) {
        const int y = c.h0 + xrow[k], x = c.w0 + xcol[k];
        const bool ok = ((unsigned)y < (unsigned)d.H) & ((unsigned)x < (unsigned)d.W);
        const int cc = xch[k];
        const float4 a0 = *reinterpret_cast<const float4*>(tab + cc);
        const float4 a1 = *reinterpret_cast<const float4*>(tab + cc + 4);
        const float4 b0 = *reinterpret_cast<const float4*>(tab + BCI + cc);
        const float4 b1 = *reinterpret_cast<const float4*>(tab + BCI + cc + 4);
        const f2_t sc[4] = {{a0.x, a0.y}, {a0.z, a0.w}, {a1.x, a1.y}, {a1.z, a1.w}};
        const f2_t sf[4] = {{b0.x, b0.y}, {b0.z, b0.w}, {b1.x, b1.y}, {b1.z, b1.w}};
        float gm = ok ? 1.f : 0.f;
        if (gated) {
          const float pv = *reinterpret_cast<const float*>(lds + Lay::OFF_GATE + c.s2 * Lay::GATE + wave * 256 +
                                                           (k * 8 + (lane >> 3)) * 4);
          gm = ok ? sigmoidf_(pv * ga + gb) : 0.f;
        }
        const f2_t g2 = {gm, gm};
        float v[8];
        unpack8_16<T>(q4, v);
        unsigned u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f2_t x2 = {v[2 * j], v[2 * j + 1]};
          const f2_t t2 = __builtin_elementwise_fma(x2, sc[j], sf[j]) * g2;
          u[j] = __builtin_bit_cast(unsigned, __builtin_elementwise_max(
                                                  __builtin_bit_cast(s2_t, pack2_16<T>(t2.x, t2.y)), lo2));
        }
        q4 = make_uint4(u[0], u[1], u[2], u[3]);
      }
      *reinterpret_cast<uint4*>((live ? cb : lds) + so) = q4;
    }
  };

  // ---- prologue: stages 0-2 in flight, stage 0 ready ----
  Cur I, X, K;
  cur_init(I);
  cur_init(K);
  issue(I);
  cur_next(I);
  if (ntl > 1) {
    issue(I);
    cur_next(I);
    if (gated) wait_vm<ND0 + 1>(); else wait_vm<ND0>();
  } else {
    wait_vm<0>();
  }
  if constexpr (ACT) {
    lds_barrier();            // the scale / shift table
    cur_init(X);
    transform(X);
    cur_next(X);
  }
  if (ntl > 2) {
    issue(I);
    cur_next(I);
  }
  lds_barrier();

  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[t][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one K step: row r of the stage at K (4 dy fragments, then the 9 taps' halo fragments)
  auto kstep = [&](const unsigned char* db, const unsigned char* xb, int r) {
    typename Mma<T>::frag a[4];
#pragma unroll
    for (int f = 0; f < 4; ++f) a[f] = w5_tr8<T>(db + aoff[0][f] + r * DROW, db + aoff[1][f] + r * DROW);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ty = t / 3, tx = t % 3;
      const typename Mma<T>::frag b =
          w5_tr8<T>(xb + boff[0][tx] + (r + ty) * XROW, xb + boff[1][tx] + (r + ty) * XROW);
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[t][f] = Mma<T>::mma(a[f], b, acc[t][f]);
    }
  };
  // this wave's DMAs of the stage after K have landed (only the youngest stage's may still be in flight)
  auto wait_next = [&](int t) {
    if (t + 2 < ntl) {
      if (gated) wait_vm<ND0 + 1>(); else wait_vm<ND0>();
    } else {
      wait_vm<0>();
    }
  };

#pragma unroll 1
  for (int t = 0; t < ntl; ++t) {
    const unsigned char* db = lds + Lay::OFF_D + K.s3 * Lay::DIMG;
    const unsigned char* xb = lds + Lay::OFF_X + (ACT ? K.s2 : K.s3) * Lay::XIMG;
    // K steps of this wave: rows wk, wk + WK, ...; the next stage's wait + transform after the first
    kstep(db, xb, wk);
    wait_next(t);
    if constexpr (ACT) {
      if (X.t < ntl) {
        transform(X);
        cur_next(X);
      }
    }
#pragma unroll
    for (int kk = 1; kk < KPW; ++kk) kstep(db, xb, wk + kk * WK);
    lds_barrier();
    // every wave has finished reading stage K: the DMA of stage K+3 reuses its ring slots
    if (I.t < ntl) {
      issue(I);
      cur_next(I);
    }
    cur_next(K);
  }

  // ---- the K halves' sums (WK = 2), then the block's slab: ws[split][co][ci][tap] (OIHW) ----
  if constexpr (WK > 1) {
    // the ring is free (last barrier passed, no DMA in flight); rounds of RE accumulator registers per lane
    constexpr int NPAIR = W5_NW / WK;
    constexpr int RE = (Lay::BYTES / (NPAIR * 64 * 4)) / 4 * 4 >= 144 ? 144 : (Lay::BYTES / (NPAIR * 64 * 4)) / 4 * 4;
    float* red = reinterpret_cast<float*>(lds);
    const int pair = wave / WK;
#pragma unroll
    for (int e0 = 0; e0 < 144; e0 += RE) {
      if (wk == 1) {
#pragma unroll
        for (int e = 0; e < RE; ++e)
          if (e0 + e < 144) red[((pair * RE) + e) * 64 + lane] = acc[(e0 + e) / 16][((e0 + e) / 4) % 4][(e0 + e) % 4];
      }
      __syncthreads();
      if (wk == 0) {
#pragma unroll
        for (int e = 0; e < RE; ++e)
          if (e0 + e < 144) acc[(e0 + e) / 16][((e0 + e) / 4) % 4][(e0 + e) % 4] += red[((pair * RE) + e) * 64 + lane];
      }
      __syncthreads();
    }
    if (wk != 0) return;
  }
  float* slab = ws + (size_t)blockIdx.x * d.Cout * d.Cin * 9;
  const int ci = ci0 + wci * 16 + (lane & 15);
  const int cob = co0 + wco * 64 + 4 * (lane >> 4);
  const unsigned row = (unsigned)d.Cin * 9u;
  const unsigned base = ((unsigned)cob * d.Cin + ci) * 9u;
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float* o = slab + base + (unsigned)(16 * f + r) * row;
#pragma unroll
      for (int t = 0; t < 9; ++t) o[t] = acc[t][f][r];
    }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
struct W5Plan {
  bool ok;
  int wco, wk, th, mtiles, splits, per_split;
  size_t ws_bytes;
};

// UNET_WGRAD5: unset = the default policy (below), 0 = never (wgrad2 everywhere), 1 = every eligible wgrad
static int wgrad5_mode() {
  const char* e = getenv("UNET_WGRAD5");
  return e ? (atoi(e) ? 1 : 0) : 2;
}

static W5Plan wgrad5_plan(const unet_wgrad_desc* d) {
  W5Plan p{};
  p.ok = (d->dtype == UNET_BF16 || d->dtype == UNET_F16) && d->ksize == 3 && d->Cout % 64 == 0 && d->Cin % 64 == 0;
  if (!p.ok) return p;
  const unet_src& s0 = d->src[0];
  if (s0.kind != UNET_SRC_PLAIN && s0.kind != UNET_SRC_ACT) p.ok = false;
  if (s0.kind == UNET_SRC_PLAIN && s0.gate_p) p.ok = false;
  if (d->nsrc > 1 && (s0.C % 64 || d->src[1].kind != UNET_SRC_PLAIN || d->src[1].gate_p)) p.ok = false;
  for (int i = 0; i < d->nsrc; ++i) {
    const unet_src& s = d->src[i];
    if (s.H != d->H || s.W != d->W) p.ok = false;
    if ((double)d->N * s.H * s.W * s.C * 2 >= (double)OOB) p.ok = false;
  }
  if ((double)d->N * d->H * d->W * d->Cout * 2 >= (double)OOB) p.ok = false;
  if ((double)d->N * d->H * d->W * 4 >= (double)OOB) p.ok = false;
  if (!p.ok) return p;
  // 64-output-channel blocks everywhere (round 5): twice the channel tiles of the former 128-channel blocks for
  // Cout >= 128, so half the splits — and half the fp32 slab traffic (every split writes a whole weight-sized
  // slab that the reduction reads back): 10-15 % per layer, 73-120 us per step (profiles/r05_wgrad5_wco_ab.txt).
  // UNET_W5_WCO2=1: the 128-channel blocks for Cout >= 128 (A/B)
  const char* wco2 = getenv("UNET_W5_WCO2");
  const bool wide = wco2 && atoi(wco2) && d->Cout >= 128;
  p.wco = wide ? 2 : 1;
  p.wk = wide ? 1 : 2;
  const int bco = 64 * p.wco, bci = 64;
  // 4-row stages where the LDS allows (stored sources, 64-channel output blocks): the halo rows cost 6/4
  // instead of 4/2 of a stage's rows and each wave runs two K steps per stage
  p.th = p.wco == 1 ? 4 : 2;
  p.mtiles = d->N * cdiv(d->W, W5_TW) * cdiv(d->H, p.th);
  const long long tiles_out = (long long)(d->Cout / bco) * (d->Cin / bci);
  const size_t slab = (size_t)d->Cout * d->Cin * 9 * sizeof(float);
  // one resident block per CU: at least 256 blocks, the split count a multiple of 8 (the blocks of one
  // split — same pixels, other channel blocks — then share an XCD and its L2); slabs capped at 160 MB
  long long s = (256 + tiles_out - 1) / tiles_out;
  // (a layer whose channel tiles alone fill >= 32 of the CUs keeps its few splits: rounding 4 up to 8 doubled
  // the slab traffic of the 1024 -> 512 weight gradient at 64^2, 151 instead of 75 MB; UNET_W5_SPLIT8=1: old rule)
  if (s > 8 || getenv("UNET_W5_SPLIT8")) s = (s + 7) / 8 * 8;
  const long long cap = (long long)(((size_t)160 << 20) / slab);
  if (s > cap) s = cap;
  if (s > p.mtiles) s = p.mtiles;
  if (s < 1) s = 1;
  p.per_split = cdiv(p.mtiles, (int)s);
  p.splits = cdiv(p.mtiles, p.per_split);
  p.ws_bytes = slab * (p.splits + (p.splits > W5_RG_MIN ? W5_RG : 0));
  return p;
}

bool wgrad5_eligible(const unet_wgrad_desc* d, size_t* ws_bytes) {
  const int mode = wgrad5_mode();
  if (mode == 0) return false;
  const W5Plan p = wgrad5_plan(d);
  if (!p.ok) return false;
  // default: pipelines of >= 6 stages per block (short ones are prologue-bound; wgrad2 keeps those)
  if (mode == 2 && p.per_split < 6) return false;
  if (ws_bytes) *ws_bytes = p.ws_bytes;
  return true;
}

template <typename T, int WCO, int WK, int SK, int TH>
static int launch5w(const unet_wgrad_desc* d, const W5Plan& p, hipStream_t st) {
  dim3 grid(p.splits, d->Cin / 64, d->Cout / (64 * WCO));
  hipLaunchKernelGGL((wgrad5_kernel<T, WCO, WK, SK, TH>), grid, dim3(W5_NT), 0, st, *d, p.mtiles, p.per_split,
                     (float*)d->workspace);
  return check_launch("wgrad5");
}

template <typename T>
static int dispatch5w(const unet_wgrad_desc* d, const W5Plan& p, hipStream_t st) {
  const bool act = d->src[0].kind == UNET_SRC_ACT;
  if (p.wco == 2) return act ? launch5w<T, 2, 1, SK_ACT, 2>(d, p, st) : launch5w<T, 2, 1, SK_PLAIN, 2>(d, p, st);
  if (!act) return launch5w<T, 1, 2, SK_PLAIN, 4>(d, p, st);
  return d->src[0].gate_p ? launch5w<T, 1, 2, SK_ACT, 4>(d, p, st) : launch5w<T, 1, 2, W5_ACT_NG, 4>(d, p, st);
}

int wgrad5_run(const unet_wgrad_desc* d, hipStream_t st) {
  const W5Plan p = wgrad5_plan(d);
  const int e = d->dtype == UNET_F16 ? dispatch5w<f16>(d, p, st) : dispatch5w<bf16>(d, p, st);
  if (e) return e;
  const long long total = (long long)d->Cout * d->Cin * 9;
  if (p.splits > W5_RG_MIN) {
    return slab_reduce_two_pass((const float*)d->workspace, p.splits, total,
                                (float*)d->workspace + (size_t)p.splits * total, d->dw, d->accum, st);
  }
  return wgrad_reduce2_launch((const float*)d->workspace, p.splits, total, d->dw, d->accum, st);
}

}  // namespace unet
