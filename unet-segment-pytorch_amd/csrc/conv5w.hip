// conv5w.hip — the wide form of conv5 (round 6): 3x3 convolution, 128 output channels per workgroup.
//
// Replaces nn.Conv2d(k=3, pad=1, bias=False) of unet/models/layers.py:32,35 (the DoubleConv halves with >= 128
// output channels: Down blocks down1-down2, the Up blocks' conv0 over the [skip, up] concat, up2's conv3) and the
// input-gradient half of its convolution_backward into >= 128 channels, on maps whose 16 x 32 x 128 tiles fill
// the chip.
//
// Why a second form: conv5 gives each 8-wave workgroup 16 rows x 32 px x 64 output
// channels, so every halo chunk a workgroup DMAs, BN-transforms and reads from LDS feeds 64 channels' MFMAs, and
// a layer with 128+ output channels stages and transforms each input chunk twice or more.  Here a workgroup owns
// 16 rows x 32 px x 128 channels: 2 row groups x 4 channel quarters of 8-row x 32-px x 32-channel wave tiles
// (v_mfma_f32_32x32x16, D[co][px] = W[co][k] X[k][px], 8 accumulators = 128 registers).  Per 16-channel chunk
// the workgroup issues twice the MFMAs (576) for the same halo (18 x 34 pixels), so per MFMA:
//  * the halo DMA, the BN-activation transform and the per-chunk barrier / cursor work are halved;
//  * B-operand LDS reads drop from 9 to 6.5 per 12 MFMAs: a wave reads 10 halo rows + 3 weight fragments per
//    tap column for 24 MFMAs (each halo row feeds the 1-3 MFMAs of its dy taps, read two rows ahead, so only
//    three row fragments are live);
//  * the input is read from L2 / HBM once per 128 output channels instead of once per 64.
// Register budget (2 waves per SIMD, <= 256): 128 accumulators, 32 BN partial sums, ~36 operand registers.
//
// Layout changes against conv5, each for the register budget:
//  * halo image swizzle by the pixel's COLUMN (x >> 3 & 1 flips the two 16-byte channel halves of a pixel),
//    not by its image index: a halo row is then a fixed 1088-byte stride, so one base register per tap column
//    and an immediate offset per row address every B fragment (conv5: 18 offset registers).  Brute-force
//    checked bank-conflict free for every row, tap column and ds_read_b128 lane group (as conv5's);
//  * BN-activation sources land in ONE raw image (not two): each lane transforms its own slots, so the DMA of
//    chunk g+2 can reuse the raw slots right after that lane's transform of chunk g+1, one chunk (576 MFMAs per
//    workgroup, as long as two of conv5's) ahead of its use;
//  * the weight fragments of a chunk (36 KB) go to a 2-deep ring, issued one chunk ahead (the L2-resident
//    weights need less lead than the halo);
//  * the attention gate's sigmoid is taken once per tile and slot (the zero-padding multiplier carries it).
// Epilogues: y (16-bit) + BatchNorm partial sums (+ act_out, as conv5), fp32 gradient with counted stores (split
// across two outputs, no accumulation).  Not served: the BN-backward-sums epilogue (its y1 loads would need 64
// more registers), accumulating fp32 gradients, ragged channel counts.
#include "conv_mfma32.h"
#include "lds_dma.h"

namespace unet {

constexpr int W5_WM = 2;                    // wave row groups
constexpr int W5_W = 32, W5_HW = 34;        // tile / halo width (pixels)
constexpr int W5_BN = 128;                  // output channels per workgroup (4 quarters of 32)
constexpr int W5_ROWB = 2 * W5_HW * 16;     // bytes per halo row of an image (1088)
// MI: wave-tile rows — 8 (16-row workgroup tiles), or 4 (8-row tiles: twice the tiles, for the 64^2 maps)
template <int MI>
struct W5Geo {
  static constexpr int TH = W5_WM * MI;                 // tile rows
  static constexpr int NS = 2 * W5_HW * (TH + 2);       // 16-byte slots per image (MI 8: 1224)
  static constexpr int NI = (NS + 63) / 64;             // DMA instructions per image (20)
  static constexpr int DPW = (NI + 7) / 8;              // per wave (3)
  static constexpr int IMG = NI * 1024;
};
constexpr int W5_NWF = 9 * 4;               // weight fragments per chunk (9 taps x 4 quarters)
constexpr int W5_WPW = (W5_NWF + 7) / 8;    // per wave (5; 4 of the 40 go to the junk slot)
constexpr int W5_WIMG = W5_NWF * 1024;
constexpr int W5_CMAX = 1024;               // largest BN-activation source
constexpr int W5_TABS = W5_CMAX + 8;        // scale / shift table stride (each half zero-padded)
constexpr int W5_OM_Y = 0, W5_OM_F32 = 1, W5_OM_BNB = 2;
constexpr int W5_SK_PLAIN1 = 4;             // = conv5.hip's SK5_PLAIN1: one stored source, C % 16 == 0

template <int MI, bool ACT, bool GATED, bool BNB>
struct W5Lay {
  static constexpr int W5_IMG = W5Geo<MI>::IMG, W5_NI = W5Geo<MI>::NI;
  static constexpr int NCOMP = ACT ? 2 : 3;
  static constexpr int OFF_COMP = 0;
  static constexpr int OFF_RAW = OFF_COMP + NCOMP * W5_IMG;
  static constexpr int OFF_W = OFF_RAW + (ACT ? W5_IMG : 0);
  static constexpr int OFF_GATE = OFF_W + 2 * W5_WIMG;
  static constexpr int OFF_TAB = OFF_GATE + (GATED ? W5_NI * 256 : 0);
  static constexpr int OFF_BTAB = OFF_TAB + (ACT ? 2 * W5_TABS * 4 : 0);   // BNB: the block's BN affine
  static constexpr int OFF_JUNK = OFF_BTAB + (BNB ? 2 * W5_BN * 4 : 0);
  static constexpr int BYTES = OFF_JUNK + 1024;
  static_assert(BYTES <= 160 * 1024, "conv5w LDS");
};

// SK: W5_SK_PLAIN1 (stored, one source), SK_ACT (one BN activation, GATE: attention-gated) or SK_ACT_PLAIN
// (src0 BN activation (+gate), src1 stored: the up-block concat); OM: W5_OM_Y, W5_OM_F32 or W5_OM_BNB (y + the
// BN-backward sums of the activation whose gradient this dgrad writes; the last two with PLAIN1 only)
template <typename T, int OM, int SK, int GATE, int MI = 8>
__global__ __launch_bounds__(512, 1) void conv5w_kernel(const unet_conv_desc d, int tiles_w, int tiles_h, int mtiles,
                                                        int nch, int prio) {
  using F = typename Mma32<T>::frag;
  constexpr bool ACT = SK != W5_SK_PLAIN1;
  constexpr bool ONE = SK != SK_ACT_PLAIN;
  constexpr bool GATED = ACT && GATE;
  using Lay = W5Lay<MI, ACT, GATED, OM == W5_OM_BNB>;
  using Geo = W5Geo<MI>;
  constexpr int TH = Geo::TH, NI = Geo::NI, DPW = Geo::DPW, WPW = W5_WPW, NS = Geo::NS, W5_IMG = Geo::IMG;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[Lay::BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;     // waves w and w + 4 share a SIMD: same quarter, other rows
  const int cw0 = (int)blockIdx.y * W5_BN + wn * 32;
  const int ntl = (mtiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int G = ntl * nch;
  const int dW = (int)(gridDim.x % (unsigned)tiles_w), dT = (int)(gridDim.x / (unsigned)tiles_w);
  const int dH = dT % tiles_h, dN = dT / tiles_h;

  // ---- sources ----
  const unet_src& s0 = d.src[0];
  const unet_src& s1 = d.src[1];
  const int C0 = s0.C, C1 = ONE ? C0 : s1.C;
  const long long npix = (long long)d.N * d.H * d.W;
  const rsrc4_t rs0 = mk_rsrc4(s0.data, (unsigned)(npix * C0 * 2));
  const rsrc4_t rs1 = ONE ? rs0 : mk_rsrc4(s1.data, (unsigned)(npix * C1 * 2));
  const rsrc4_t rsg = mk_rsrc4(GATED ? (const void*)s0.gate_p : s0.data, (unsigned)(npix * 4));
  float ga = 0.f, gb = 0.f;
  if constexpr (GATED) { ga = s0.gate_ab[0]; gb = s0.gate_ab[1]; }

  // ---- weights: the 32 x 16 A fragments of conv3's fragment-major packing (conv5's addressing) ----
  const int nch32 = (nch + 1) >> 1;
  const unsigned jstride = (unsigned)nch32 * 9u * 1024u;
  const unsigned ntiles16 = (unsigned)((d.Cout + PACK_NPAD - 1) / PACK_NPAD * (PACK_NPAD / 16));
  const rsrc4_t rw = mk_rsrc4(d.weight, ntiles16 * jstride);
  const unsigned lanew = (unsigned)((lane >> 4) & 1) * jstride + (unsigned)(16 * (lane >> 5) + (lane & 15)) * 16u;

  // ---- this lane's halo slots: instruction i = wave + 8k lands slots 64 i .. 64 i + 63; slot s holds pixel s >> 1
  // of the (TH + 2) x 34 halo, channel half (s & 1) ^ swz(column) in the compute image; a BN-activation source
  // lands unswizzled (half s & 1 = lane & 1: one scale / shift read per chunk) and its transform writes slot
  // s ^ swz(column) ----
  int soy[DPW], sox[DPW], hbit[DPW];
  unsigned cso[DPW];
#pragma unroll
  for (int k = 0; k < DPW; ++k) {
    const int i = wave + 8 * k, s = i * 64 + lane, hp = s >> 1;
    const int x = hp % W5_HW, sw = (x >> 3) & 1;
    soy[k] = s < NS ? hp / W5_HW - 1 : -(1 << 20);
    sox[k] = x - 1;
    hbit[k] = ACT ? (lane & 1) : ((s & 1) ^ sw);
    cso[k] = (unsigned)(s ^ sw) * 16u;
  }
  const unsigned l32 = lds_addr(lds);
  const unsigned junk = l32 + Lay::OFF_JUNK;

  struct Cur {
    int ti, c, n, h0, w0, s3, s2, tw, th;
  };
  auto cur_init = [&](Cur& q) {
    q.ti = 0; q.c = 0; q.s3 = 0; q.s2 = 0;
    const unsigned t = blockIdx.x, t2 = t / (unsigned)tiles_w;
    q.tw = (int)(t - t2 * (unsigned)tiles_w);
    q.th = (int)(t2 % (unsigned)tiles_h);
    q.n = (int)(t2 / (unsigned)tiles_h);
    q.h0 = q.th * TH;
    q.w0 = q.tw * W5_W;
  };
  auto cur_next = [&](Cur& q) {
    q.s3 = q.s3 == 2 ? 0 : q.s3 + 1;
    q.s2 ^= 1;
    if (++q.c == nch) {
      q.c = 0;
      if (++q.ti < ntl) {
        q.tw += dW;
        int cy = q.tw >= tiles_w;
        q.tw -= cy ? tiles_w : 0;
        q.th += dH + cy;
        cy = q.th >= tiles_h;
        q.th -= cy ? tiles_h : 0;
        q.n += dN + cy;
        q.h0 = q.th * TH;
        q.w0 = q.tw * W5_W;
      }
    }
  };

  // per-tile DMA offsets of the slots (>= OOB for zero padding and dead slots)
  unsigned ib0[DPW], ib1[ONE ? 1 : DPW];
  auto tile_slots = [&](const Cur& q) {
    const unsigned pbase = ((unsigned)q.n * d.H + q.h0) * d.W + q.w0;
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const int y = q.h0 + soy[k], x = q.w0 + sox[k];
      const bool ok = ((unsigned)y < (unsigned)d.H) & ((unsigned)x < (unsigned)d.W);
      const unsigned pix = pbase + (unsigned)(soy[k] * d.W + sox[k]);
      ib0[k] = ok ? (pix * (unsigned)C0 + 8u * hbit[k]) * 2u : OOB;
      if constexpr (!ONE) ib1[k] = ok ? (pix * (unsigned)C1 + 8u * hbit[k]) * 2u : OOB;
    }
  };
  // halo DMA of chunk q (ACT: the raw image; plain: compute image q.s3); at a gated tile's first chunk also the
  // gate pre-activations of the slots.  Returns whether those went out (the batch then counts 2 DPW)
  auto issue_h = [&](const Cur& q) -> bool {
    if (q.c == 0) tile_slots(q);
    const int cn0 = q.c * 16;
    const bool s1sel = !ONE && cn0 >= C0;
    const unsigned cl = (unsigned)(s1sel ? cn0 - C0 : cn0) * 2u;
    const unsigned img = l32 + (ACT ? Lay::OFF_RAW : Lay::OFF_COMP + q.s3 * W5_IMG);
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const int i = wave + 8 * k;
      unsigned vo;
      if constexpr (ONE) vo = ib0[k] + cl;
      else vo = (s1sel ? ib1[k] : ib0[k]) + cl;
      dma16(s1sel ? rs1 : rs0, i < NI ? img + i * 1024 : junk, vo);
    }
    const bool gl = GATED && q.c == 0;
    if (gl) {
      const unsigned pbase = ((unsigned)q.n * d.H + q.h0) * d.W + q.w0;
#pragma unroll
      for (int k = 0; k < DPW; ++k) {
        const int i = wave + 8 * k;
        const unsigned pix = pbase + (unsigned)(soy[k] * d.W + sox[k]);
        dma4(rsg, i < NI ? l32 + Lay::OFF_GATE + i * 256 : junk, ib0[k] < OOB ? pix * 4u : OOB);
      }
    }
    return gl;
  };
  // weight DMA of chunk q into ring slot q.s2 (fragment j = tap * 4 + quarter); the weight cursor carries only
  // the chunk index and ring slot (SGPR budget)
  struct WCur {
    int c, s2;
  };
  auto wcur_next = [&](WCur& q) {
    q.s2 ^= 1;
    if (++q.c == nch) q.c = 0;
  };
  auto issue_w = [&](const WCur& q) {
    const unsigned wd = l32 + Lay::OFF_W + q.s2 * W5_WIMG;
    const unsigned wofs = (unsigned)((q.c >> 1) * 9) * 1024u + (unsigned)(q.c & 1) * 512u;
#pragma unroll
    for (int k = 0; k < WPW; ++k) {
      const int j = wave + 8 * k;
      const int tap = j >> 2, qq = j & 3;
      const unsigned nt0 = (unsigned)(((int)blockIdx.y * W5_BN + qq * 32) / 16);
      const unsigned vo = lanew + nt0 * jstride + (unsigned)tap * 1024u + wofs;
      dma16(rw, j < W5_NWF ? wd + j * 1024 : junk, j < W5_NWF ? vo : OOB);
    }
  };

  // ---- BN-activation transform (raw -> compute image), this lane's own slots ----
  T* const aout = (ACT && OM == W5_OM_Y && blockIdx.y == 0) ? (T*)d.act_out : nullptr;
  const rsrc_t rao = mk_rsrc(aout ? (const void*)aout : d.out, (unsigned)(aout ? npix * C0 * 2 : 0));
  float xg[ACT ? DPW : 1];      // zero-padding multiplier x attention gate of the slot, per tile
  unsigned xao[ACT ? DPW : 1];  // act_out byte offset of the slot (interior pixels only, else OOB)
  typedef __attribute__((ext_vector_type(2))) float f2_t;
  typedef __attribute__((ext_vector_type(2))) short s2_t;
  const s2_t lo2 = s0.relu ? s2_t{0, 0} : s2_t{-32768, -32768};
  auto transform = [&](const Cur& q) {
    if (q.c == 0) {
      const unsigned pbase = ((unsigned)q.n * d.H + q.h0) * d.W + q.w0;
#pragma unroll
      for (int k = 0; k < DPW; ++k) {
        const int i = wave + 8 * k;
        const int y = q.h0 + soy[k], x = q.w0 + sox[k];
        const bool ok = ((unsigned)y < (unsigned)d.H) & ((unsigned)x < (unsigned)d.W);
        float g = ok ? 1.f : 0.f;
        if constexpr (GATED) {
          // (padding slots loaded zeros: a finite sigmoid times 0; dead slots read the junk slot, never used)
          const float pv = *reinterpret_cast<const float*>(lds + (i < NI ? Lay::OFF_GATE + i * 256 : Lay::OFF_JUNK) + lane * 4);
          g *= sigmoidf_(pv * ga + gb);
        }
        xg[k] = g;
        const bool in = ok && (unsigned)soy[k] < (unsigned)TH && (unsigned)sox[k] < (unsigned)W5_W && i < NI;
        const unsigned pix = pbase + (unsigned)(soy[k] * d.W + sox[k]);
        xao[k] = in ? (pix * (unsigned)C0 + 8u * (unsigned)(lane & 1)) * 2u : OOB;
      }
    }
    const int cn0 = q.c * 16;
    const bool act = ONE || cn0 < C0;
    f2_t sc[4], sf[4];
    if (act) {
      const float* tab = reinterpret_cast<const float*>(lds + Lay::OFF_TAB);
      const int ch = cn0 + 8 * (lane & 1);
      const float4 a0 = *reinterpret_cast<const float4*>(tab + ch);
      const float4 a1 = *reinterpret_cast<const float4*>(tab + ch + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(tab + W5_TABS + ch);
      const float4 b1 = *reinterpret_cast<const float4*>(tab + W5_TABS + ch + 4);
      sc[0] = f2_t{a0.x, a0.y}; sc[1] = f2_t{a0.z, a0.w}; sc[2] = f2_t{a1.x, a1.y}; sc[3] = f2_t{a1.z, a1.w};
      sf[0] = f2_t{b0.x, b0.y}; sf[1] = f2_t{b0.z, b0.w}; sf[2] = f2_t{b1.x, b1.y}; sf[3] = f2_t{b1.z, b1.w};
    }
    const unsigned cbase = Lay::OFF_COMP + (unsigned)q.s2 * W5_IMG;
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const int i = wave + 8 * k;
      const bool live = i < NI;
      uint4 q4 = *reinterpret_cast<const uint4*>(lds + (live ? Lay::OFF_RAW + (unsigned)(i * 64 + lane) * 16u
                                                             : Lay::OFF_JUNK + lane * 16));
      if (act) {
        const f2_t g2 = {xg[k], xg[k]};
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
      if constexpr (OM == W5_OM_Y) {
        // act_out: every transform issues exactly DPW stores (out of range where nothing is written)
        typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
        const unsigned vo = act ? xao[k] + (unsigned)cn0 * 2u : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, q4), rao, (int)vo, 0, 0);
      }
      *reinterpret_cast<uint4*>(lds + (live ? cbase + cso[k] : Lay::OFF_JUNK + lane * 16)) = q4;
    }
  };

  // ---- B fragment base offsets (per tap column; halo row r of the wave adds r * 1088, an immediate) ----
  unsigned boff[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int x = (lane & 31) + dx;
    boff[dx] = (unsigned)(wm * MI * W5_ROWB + 32 * x + 16 * ((lane >> 5) ^ ((x >> 3) & 1)));
  }
  const unsigned wlane = (unsigned)(wn * 1024 + lane * 16);

  // ---- prologue ----
  if constexpr (ACT) {
    float* tab = reinterpret_cast<float*>(lds + Lay::OFF_TAB);
    for (int c = tid; c < C0; c += 512) { tab[c] = s0.scale[c]; tab[W5_TABS + c] = s0.shift[c]; }
    if (tid < 8) { tab[C0 + tid] = 0.f; tab[W5_TABS + C0 + tid] = 0.f; }
  }
  if constexpr (OM == W5_OM_BNB) {
    // the BN affine of the activation whose gradient this dgrad writes (its ReLU mask), the block's channels
    float* bt = reinterpret_cast<float*>(lds + Lay::OFF_BTAB);
    if (tid < W5_BN) {
      const int co = (int)blockIdx.y * W5_BN + tid;
      const bool ok = co < d.Cout && d.bnb_relu;
      bt[tid] = ok ? d.bnb_scale[co] : 0.f;
      bt[W5_BN + tid] = ok ? d.bnb_shift[co] : 0.f;
    }
  }
  Cur I, K;   // I: next chunk to DMA (halo); K: chunk being computed
  cur_init(I);
  cur_init(K);
  WCur IW = {0, 0};   // next chunk whose weights to DMA
  if constexpr (ACT) {
    Cur X = I;
    issue_h(I);
    cur_next(I);
    issue_w(IW);
    wcur_next(IW);
    wait_vm<0>();
    lds_barrier();            // the scale / shift table (and nothing else is shared yet)
    transform(X);             // chunk 0 -> compute image 0 (+ DPW act_out stores)
    issue_h(I);               // chunk 1 (nch >= 2: never a tile's first chunk)
    cur_next(I);
    issue_w(IW);              // chunk 1
    wcur_next(IW);
    lds_barrier();            // compute image 0 written by every wave (chunk 0's weights landed: vmcnt(0) above)
  } else {
    issue_h(I); cur_next(I);     // 0
    issue_w(IW); wcur_next(IW);   // 0
    issue_h(I); cur_next(I);     // 1
    issue_w(IW); wcur_next(IW);   // 1
    if (G > 2) {
      issue_h(I); cur_next(I);   // 2 (never a first chunk: plain sources carry no gate)
      wait_vm<2 * DPW + WPW>();
    } else {
      wait_vm<DPW + WPW>();
    }
    lds_barrier();
  }
  if (prio && wave >= 4) __builtin_amdgcn_s_setprio(1);

  // BatchNorm partial sums of this lane's pixel column over the block's tiles (y mode)
  float sA[16], sB[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) { sA[r] = 0.f; sB[r] = 0.f; }
  f32x16 acc[MI];

  // MFMAs of one chunk: 3 tap columns x 10 halo rows; row r of column dx feeds acc[r - dy] with tap (dy, dx).
  // The row fragments are read two rows ahead (3 live), the next column's 3 weight fragments during the
  // current column; sched_group_barrier pins one LDS read between MFMAs
  auto chunk_mma = [&](unsigned cb, unsigned wb) {
    const unsigned char* xb = lds + cb;
    const unsigned char* wp = lds + wb + wlane;
    F w[2][3], x[3];
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) w[0][dy] = *reinterpret_cast<const F*>(wp + (dy * 3) * 4096);
    x[0] = *reinterpret_cast<const F*>(xb + boff[0]);
    x[1] = *reinterpret_cast<const F*>(xb + boff[0] + W5_ROWB);
    constexpr int R = MI + 2, NSTEP = 3 * R;   // halo rows per tap column, row steps per chunk
#pragma unroll
    for (int t = 0; t < NSTEP; ++t) {
      const int dx = t / R, r = t % R;
      // prefetch: the row two steps ahead (possibly the next column's), the next column's weights at rows 2-4
      if (t + 2 < NSTEP) {
        const int dx2 = (t + 2) / R, r2 = (t + 2) % R;
        x[(t + 2) % 3] = *reinterpret_cast<const F*>(xb + boff[dx2] + r2 * W5_ROWB);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      if (dx < 2 && r >= 2 && r <= 4) {
        w[(dx + 1) & 1][r - 2] = *reinterpret_cast<const F*>(wp + ((r - 2) * 3 + dx + 1) * 4096);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int dy = 2; dy >= 0; --dy) {
        const int i = r - dy;
        if (i >= 0 && i < MI) {
          acc[i] = Mma32<T>::mma(w[dx & 1][dy], x[t % 3], acc[i]);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
      }
      // nothing crosses a row step: hipcc otherwise sinks the prefetches next to their MFMAs (one live row
      // fragment, an lgkmcnt(0) per row in the last tap column)
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // the vmcnt waits: what may stay in flight is counted from the issue order (file header)
  constexpr int NST = OM == W5_OM_F32 ? 4 * MI : 2 * MI;   // epilogue stores per tile
  // BNB: the tile's last DMA batch is issued after its epilogue (behind the y1 loads' wait), so the epilogue's
  // stores are older than the next wait's batch: none of them may stay in flight there
  constexpr int NSTW = OM == W5_OM_BNB ? 0 : NST;
  constexpr int NSA = (ACT && OM == W5_OM_Y) ? DPW : 0;  // act_out stores per transform
  bool st = false;   // the previous chunk ended a tile: its NST epilogue stores are the youngest
  int g = 0;
  const bool f32c = OM == W5_OM_F32;
  const rsrc_t ry = mk_rsrc(d.out, (unsigned)(OM != W5_OM_F32 ? npix * d.Cout * 2 : 0));
  const rsrc_t ry1 = mk_rsrc(OM == W5_OM_BNB ? d.bnb_y : d.out, (unsigned)(OM == W5_OM_BNB ? npix * d.Cout * 2 : 0));
  bool pend_w = false, pend_h = false;   // BNB: the deferred DMA issues of a tile's last chunk
  const rsrc_t rf1 = mk_rsrc(d.out, (unsigned)(f32c ? npix * d.split * 4 : 0));
  const rsrc_t rf2 = mk_rsrc(d.out2 ? d.out2 : d.out, (unsigned)(f32c ? npix * (d.Cout - d.split) * 4 : 0));
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  Cur X = K;   // ACT: the next chunk to transform (chunk 1)
  if constexpr (ACT) cur_next(X);

  for (int ti = 0; ti < ntl; ++ti) {
    const int tn = K.n, th0 = K.h0, tw0 = K.w0;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll 1
    for (int c = 0; c < nch; ++c, ++g) {
      const unsigned cb = Lay::OFF_COMP + (unsigned)(ACT ? K.s2 : K.s3) * W5_IMG;
      const unsigned wb = Lay::OFF_W + (unsigned)K.s2 * W5_WIMG;
      chunk_mma(cb, wb);
      const bool w1 = g + 1 < G, h2 = g + 2 < G;
      if constexpr (ACT) {
        // raw chunk g+1 landed (W(g+1) and the previous tile's epilogue stores may stay in flight)
        if (st) { if (w1) wait_vm<WPW + NST>(); else wait_vm<NST>(); }
        else { if (w1) wait_vm<WPW>(); else wait_vm<0>(); }
        bool gl = false;
        if (w1) {
          transform(X);
          cur_next(X);
          if (h2) {
            gl = issue_h(I);
            cur_next(I);
          }
        }
        // W(g+1) landed: the epilogue stores, the act_out stores and H(g+2) may stay in flight
        const int sh = st ? 1 : 0;
        if (h2) {
          if (gl) { if (sh) wait_vm<NST + NSA + 2 * DPW>(); else wait_vm<NSA + 2 * DPW>(); }
          else { if (sh) wait_vm<NST + NSA + DPW>(); else wait_vm<NSA + DPW>(); }
        } else if (w1) {
          if (sh) wait_vm<NST + NSA>(); else wait_vm<NSA>();
        } else {
          if (sh) wait_vm<NST>(); else wait_vm<0>();
        }
        lds_barrier();
        if (h2) {
          issue_w(IW);
          wcur_next(IW);
        }
      } else {
        // H(g+1) and W(g+1) landed: H(g+2) (issued with W(g+1)) and the epilogue stores may stay in flight
        if (st && NSTW) { if (h2) wait_vm<NSTW + DPW>(); else wait_vm<NSTW>(); }
        else { if (h2) wait_vm<DPW>(); else wait_vm<0>(); }
        lds_barrier();
        const bool h3 = g + 3 < G;
        if (OM == W5_OM_BNB && c == nch - 1) {
          pend_w = h2;
          pend_h = h3;
        } else {
          if (h2) {
            issue_w(IW);
            wcur_next(IW);
          }
          if (h3) {
            issue_h(I);
            cur_next(I);
          }
        }
      }
      st = false;
      cur_next(K);
    }

    // ---------------- epilogue of tile ti ----------------
    const int pxl = lane & 31, hh = lane >> 5;
    const int ow = tw0 + pxl;
    const bool colok = ow < d.W;
    const int oh0 = th0 + wm * MI;
    int rows = d.H - oh0;
    rows = rows < 0 ? 0 : (rows > MI ? MI : rows);
    const unsigned pix0 = ((unsigned)tn * d.H + oh0) * (unsigned)d.W + ow;
    if constexpr (OM == W5_OM_Y) {
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bool ok = colok && i < rows;
        const unsigned pix = pix0 + (unsigned)i * d.W;
        unsigned px_[4], py_[4];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          px_[gq] = pack2_16<T>(acc[i][4 * gq], acc[i][4 * gq + 1]);
          py_[gq] = pack2_16<T>(acc[i][4 * gq + 2], acc[i][4 * gq + 3]);
        }
#pragma unroll
        for (int kp = 0; kp < 4; kp += 2) {
          const auto sx = __builtin_amdgcn_permlane32_swap(px_[kp], px_[kp + 1], false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(py_[kp], py_[kp + 1], false, false);
          const int co = cw0 + 8 * kp + 8 * hh;
          const unsigned vo = (ok && co < d.Cout) ? (pix * (unsigned)d.Cout + (unsigned)co) * 2u : OOB;
          const u32x4_t v4 = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v4, ry, (int)vo, 0, 0);
        }
      }
      if (d.stats) {
        typedef __attribute__((ext_vector_type(2))) float f2s;
        const bool full = rows == MI && tw0 + W5_W <= d.W;
#pragma unroll
        for (int r = 0; r < 16; r += 2) {
          f2s a2 = {sA[r], sA[r + 1]}, b2 = {sB[r], sB[r + 1]};
          if (full) {
#pragma unroll
            for (int i = 0; i < MI; ++i) {
              const f2s x2 = {acc[i][r], acc[i][r + 1]};
              a2 += x2;
              b2 = __builtin_elementwise_fma(x2, x2, b2);
            }
          } else {
#pragma unroll
            for (int i = 0; i < MI; ++i) {
              const bool ok = colok && i < rows;
              const f2s x2 = {ok ? acc[i][r] : 0.f, ok ? acc[i][r + 1] : 0.f};
              a2 += x2;
              b2 = __builtin_elementwise_fma(x2, x2, b2);
            }
          }
          sA[r] = a2.x; sA[r + 1] = a2.y;
          sB[r] = b2.x; sB[r + 1] = b2.y;
        }
      }
    } else if constexpr (OM == W5_OM_BNB) {
      // per 16-channel half h: y1 of this wave's pixels, 16-byte loads in the layout of the swapped g stores
      // (lanes 0-31 channels 16h + 0..7 of their pixel, lanes 32-63 16h + 8..15; one half at a time: 32
      // registers); the compiler's wait for them also covers the older DMAs, all issued a chunk or more ago
      const float* btab = reinterpret_cast<const float*>(lds + Lay::OFF_BTAB);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int co = cw0 + 16 * h + 8 * hh;
        const bool cok = co < d.Cout;
        const int cb = co - (int)blockIdx.y * W5_BN;
        uint4 yv[MI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const bool ok = colok && i < rows && cok;
          const unsigned vo = ok ? ((pix0 + (unsigned)i * d.W) * (unsigned)d.Cout + (unsigned)co) * 2u : OOB;
          yv[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ry1, (int)vo, 0, 0));
        }
        float sc8[8], sf8[8];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float4 a4 = *reinterpret_cast<const float4*>(btab + cb + 4 * q);
          const float4 b4 = *reinterpret_cast<const float4*>(btab + W5_BN + cb + 4 * q);
          sc8[4 * q] = a4.x; sc8[4 * q + 1] = a4.y; sc8[4 * q + 2] = a4.z; sc8[4 * q + 3] = a4.w;
          sf8[4 * q] = b4.x; sf8[4 * q + 1] = b4.y; sf8[4 * q + 2] = b4.z; sf8[4 * q + 3] = b4.w;
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const unsigned pix = pix0 + (unsigned)i * d.W;
          const bool ok = colok && i < rows && cok;
          const int g0 = 2 * h;
          const unsigned pxa = pack2_16<T>(acc[i][4 * g0], acc[i][4 * g0 + 1]);
          const unsigned pxb = pack2_16<T>(acc[i][4 * g0 + 4], acc[i][4 * g0 + 5]);
          const unsigned pya = pack2_16<T>(acc[i][4 * g0 + 2], acc[i][4 * g0 + 3]);
          const unsigned pyb = pack2_16<T>(acc[i][4 * g0 + 6], acc[i][4 * g0 + 7]);
          const auto sx = __builtin_amdgcn_permlane32_swap(pxa, pxb, false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(pya, pyb, false, false);
          const unsigned vo = ok ? (pix * (unsigned)d.Cout + (unsigned)co) * 2u : OOB;
          const u32x4_t v4 = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v4, ry, (int)vo, 0, 0);
          if (ok) {
            float gv[8], yy[8];
            unpack4_16<T>(make_uint2(v4[0], v4[1]), gv);
            unpack4_16<T>(make_uint2(v4[2], v4[3]), gv + 4);
            unpack4_16<T>(make_uint2(yv[i].x, yv[i].y), yy);
            unpack4_16<T>(make_uint2(yv[i].z, yv[i].w), yy + 4);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              const float gg = (d.bnb_relu && !(yy[r] * sc8[r] + sf8[r] > 0.f)) ? 0.f : gv[r];
              sA[8 * h + r] += gg;
              sB[8 * h + r] = __builtin_fmaf(gg, yy[r], sB[8 * h + r]);
            }
          }
        }
      }
      if (pend_w) {
        issue_w(IW);
        wcur_next(IW);
      }
      if (pend_h) {
        issue_h(I);
        cur_next(I);
      }
      pend_w = pend_h = false;
    } else {   // fp32 gradient, counted buffer stores (no accumulation: host-checked), split at d.split
      const int c2 = d.Cout - d.split;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const unsigned pix = pix0 + (unsigned)i * d.W;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int co = cw0 + 8 * gq + 4 * hh;
          const bool to1 = cw0 + 8 * gq < d.split;      // wave-uniform (split % 8 == 0)
          const bool ok = colok && i < rows && co < d.Cout;
          const unsigned vo = !ok ? OOB : to1 ? (pix * (unsigned)d.split + (unsigned)co) * 4u
                                             : (pix * (unsigned)c2 + (unsigned)(co - d.split)) * 4u;
          typedef __attribute__((ext_vector_type(4))) float f32x4v;
          const f32x4v w = {acc[i][4 * gq], acc[i][4 * gq + 1], acc[i][4 * gq + 2], acc[i][4 * gq + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, w), to1 ? rf1 : rf2, (int)vo, 0, 0);
        }
      }
    }
    st = true;
  }

  // ---- the workgroup's BatchNorm sums: one partial row per wave row group ----
  if constexpr (OM == W5_OM_Y) {
    if (d.stats) {
      const int hh = lane >> 5;
      const int srow = blockIdx.x * W5_WM + wm, srows = gridDim.x * W5_WM;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float a = half32_sum(sA[r]), b = half32_sum(sB[r]);
        const int co = cw0 + 8 * (r >> 2) + 4 * hh + (r & 3);
        if ((lane & 31) == 0 && co < d.Cout) {
          d.stats[(size_t)co * srows + srow] = a;
          d.stats[((size_t)d.Cout + co) * srows + srow] = b;
        }
      }
    }
  } else if constexpr (OM == W5_OM_BNB) {
    // one [rows][Cout] partial row per wave row group; sum slot 8h + r is channel cw0 + 16h + 8hh + r
    const int hh = lane >> 5;
    const int srow = blockIdx.x * W5_WM + wm, srows = gridDim.x * W5_WM;
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      const int co = cw0 + 16 * (gq >> 1) + 8 * hh + 4 * (gq & 1);
      float a[4], b[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = half32_sum(sA[4 * gq + r]);
        b[r] = half32_sum(sB[4 * gq + r]);
      }
      if ((lane & 31) == 0 && co < d.Cout) {
        const float4 m4 = *reinterpret_cast<const float4*>(d.bnb_mean + co);
        const float4 i4 = *reinterpret_cast<const float4*>(d.bnb_invstd + co);
        const float mu[4] = {m4.x, m4.y, m4.z, m4.w}, is[4] = {i4.x, i4.y, i4.z, i4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) b[r] = is[r] * (b[r] - mu[r] * a[r]);
        *reinterpret_cast<float4*>(d.bnb_stats + (size_t)srow * d.Cout + co) = make_float4(a[0], a[1], a[2], a[3]);
        *reinterpret_cast<float4*>(d.bnb_stats + ((size_t)srows + srow) * d.Cout + co) = make_float4(b[0], b[1], b[2], b[3]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
static long long w5_mtiles(const unet_conv_desc* d, int mi) {
  return (long long)d->N * cdiv(d->W, W5_W) * cdiv(d->H, W5_WM * mi);
}
// MI of a descriptor: 8 (16-row tiles) where those fill the chip, else 4 (8-row tiles), else none (0)
static int w5_mi(const unet_conv_desc* d) {
  if (w5_mtiles(d, 8) * (d->Cout / W5_BN) >= 256) return 8;
  if (w5_mtiles(d, 4) * (d->Cout / W5_BN) >= 256) return 4;
  return 0;
}

// UNET_CONV5W: unset = the measured default (below), 0 = never, 1 = every descriptor it can serve (tests, A/B);
// read per call so tests can flip it
static int conv5w_mode() {
  const char* e = getenv("UNET_CONV5W");
  return e ? (atoi(e) ? 1 : 0) : 2;
}

bool conv5w_ok(const unet_conv_desc* d) {
  const int mode = conv5w_mode();
  if (mode == 0) return false;
  // default: the BN-activation forwards with >= 256 input channels (the gated [skip, up] concats, down2.3):
  // -5 to -23 us per layer against conv5, which stages and transforms every chunk twice there.  Measured
  // slower (round 6, profiles/r06_layerprof_conv5w*.txt): the BNB dgrads (+10 to +28 us: its y1 loads cannot
  // be issued during the last chunk, so the tile's next DMAs wait behind them), the stored-source forwards and
  // any layer with few chunk steps per workgroup (+2 to +5 us: a chunk of this form is twice conv5's, so the
  // pipeline's fill and drain cost twice as much), and the fp32 dgrads (even with conv3)
  if (mode == 2 && (d->out_mode != UNET_OUT_Y || d->bnb_stats || d->src[0].kind != UNET_SRC_ACT || d->Cin < 256))
    return false;
  if ((d->dtype != UNET_BF16 && d->dtype != UNET_F16) || d->ksize != 3) return false;
  if (d->Cout % W5_BN || d->Cin < 32 || d->Cin % 16) return false;
  if (d->bnb_stats && (d->out_mode != UNET_OUT_Y || d->nsrc != 1 || d->src[0].kind != UNET_SRC_PLAIN || !d->bnb_y))
    return false;
  const unet_src& s0 = d->src[0];
  if (d->nsrc < 1 || d->nsrc > 2) return false;
  if (s0.kind != UNET_SRC_PLAIN && s0.kind != UNET_SRC_ACT) return false;
  if (s0.C % 16 || (s0.kind == UNET_SRC_PLAIN && s0.gate_p)) return false;
  if (s0.kind == UNET_SRC_ACT && s0.C > W5_CMAX) return false;
  if (d->nsrc == 2) {
    const unet_src& s1 = d->src[1];
    if (s0.kind != UNET_SRC_ACT || s1.kind != UNET_SRC_PLAIN || s1.gate_p || s1.C % 16) return false;
  } else if (s0.kind == UNET_SRC_PLAIN && s0.C != d->Cin) {
    return false;
  }
  if (d->out_mode == UNET_OUT_F32) {
    if (s0.kind != UNET_SRC_PLAIN || d->nsrc != 1 || d->accum || d->accum2 || d->split % 8) return false;
    if (d->split < d->Cout && !d->out2) return false;
    if ((double)d->N * d->H * d->W * d->Cout * 4 >= (double)OOB) return false;
  } else if (d->out_mode != UNET_OUT_Y) {
    return false;
  }
  for (int i = 0; i < d->nsrc; ++i) {
    const unet_src& s = d->src[i];
    if (s.H != d->H || s.W != d->W) return false;
    if ((double)d->N * s.H * s.W * s.C * 2 >= (double)OOB) return false;
  }
  if ((double)d->N * d->H * d->W * 4 >= (double)OOB) return false;
  if ((double)d->N * d->H * d->W * d->Cout * 2 >= (double)OOB) return false;
  // enough 16 x 32 x 128 tiles to fill the chip, or (BN-activation y outputs only) 8 x 32 x 128 ones
  const int mi = w5_mi(d);
  return mi == 8 || (mi == 4 && d->out_mode == UNET_OUT_Y && !d->bnb_stats && s0.kind == UNET_SRC_ACT);
}

static int w5_gx(const unet_conv_desc* d) {
  const long long mt = w5_mtiles(d, w5_mi(d));
  long long gx = cdiv(256, d->Cout / W5_BN);   // one 8-wave workgroup per CU (LDS), persistent
  if (gx > mt) gx = mt;
  return (int)(gx < 1 ? 1 : gx);
}

int conv5w_stats_rows(const unet_conv_desc* d) { return w5_gx(d) * W5_WM; }

int conv5w_variant(const unet_conv_desc* d, char* buf, int len) {
  if (w5_mi(d) == 4) snprintf(buf, len, "conv5w_kernel<%s,4>", d->dtype == UNET_F16 ? "fp16" : "bf16");
  else snprintf(buf, len, "conv5w_kernel<%s>", d->dtype == UNET_F16 ? "fp16" : "bf16");
  return 0;
}

template <typename T, int OM, int SK, int GATE, int MI = 8>
static int launch5w(const unet_conv_desc* d, int prio, hipStream_t st) {
  if constexpr (MI == 8 && OM == W5_OM_Y && SK != W5_SK_PLAIN1) {
    if (w5_mi(d) == 4) return launch5w<T, OM, SK, GATE, 4>(d, prio, st);
  }
  const int tw = cdiv(d->W, W5_W), th = cdiv(d->H, W5_WM * MI);
  const int mt = d->N * tw * th;
  const int gy = d->Cout / W5_BN, gx = w5_gx(d);
  const int nch = d->Cin / 16;
  hipLaunchKernelGGL((conv5w_kernel<T, OM, SK, GATE, MI>), dim3(gx, gy), dim3(512), 0, st, *d, tw, th, mt, nch, prio);
  return check_launch("conv5w");
}

template <typename T>
static int dispatch5w(const unet_conv_desc* d, int prio, hipStream_t st) {
  const unet_src& s0 = d->src[0];
  if (d->out_mode == UNET_OUT_F32) return launch5w<T, W5_OM_F32, W5_SK_PLAIN1, 0>(d, prio, st);
  if (d->bnb_stats) return launch5w<T, W5_OM_BNB, W5_SK_PLAIN1, 0>(d, prio, st);
  if (s0.kind == UNET_SRC_PLAIN) return launch5w<T, W5_OM_Y, W5_SK_PLAIN1, 0>(d, prio, st);
  const bool g = s0.gate_p != nullptr;
  if (d->nsrc == 1) return g ? launch5w<T, W5_OM_Y, SK_ACT, 1>(d, prio, st) : launch5w<T, W5_OM_Y, SK_ACT, 0>(d, prio, st);
  return g ? launch5w<T, W5_OM_Y, SK_ACT_PLAIN, 1>(d, prio, st) : launch5w<T, W5_OM_Y, SK_ACT_PLAIN, 0>(d, prio, st);
}

int conv5w_run(const unet_conv_desc* d, int prio, hipStream_t st) {
  return d->dtype == UNET_F16 ? dispatch5w<f16>(d, prio, st) : dispatch5w<bf16>(d, prio, st);
}

}  // namespace unet
