// conv5.hip — 3x3 convolution (forward and dgrad) for gfx950 with an LDS-DMA operand pipeline.
//
// Replaces nn.Conv2d(k=3, pad=1, bias=False) of unet/models/layers.py:32,35 (every DoubleConv half) and the
// input-gradient half of its convolution_backward, on maps large enough to fill the chip.
//
// Why: register-staged kernels spend most of their time waiting, not computing.  The round-3 ablations of a
// register-staged 32x32x16 kernel (since removed; 64->64 @ 4x512^2): 142 us full; 54 us with the halo staging, the
// in-loop weight loads and the epilogue removed, i.e. the MFMA + LDS loop alone runs at 57 % of the bf16 peak.
// The halo staging cost 39 us: its loads were issued 6 taps (~0.6 us) before use, less than the load
// latency under full-chip streaming, and held registers while in flight.  Here every operand reaches LDS by
// buffer_load ... lds (LDS DMA: no VGPRs, no VALU), issued TWO 16-channel chunks ahead:
//  * input halo of chunk g+2: (TH+2) x 34 pixels x 16 channels, 16-byte slots in lane order; a plain source
//    (dgrad dy, materialised pool / upsample) lands directly in the compute image (3-deep ring); a BN
//    activation (+ attention gate) source lands in a raw ring and is transformed slot for slot by the lane
//    that loaded it (BN-apply, ReLU, gate, zero padding) one chunk ahead — only that lane's vmcnt orders it,
//    no barrier; scale / shift come from an LDS table, the gate pre-activation from per-lane DMA slots;
//  * weights of chunk g+2: the 18 KB of 32x16 A fragments of the block's 64 output channels x 9 taps, read
//    from conv3's fragment-major packing by per-lane addresses into a 3-deep ring (one 1 KB fragment per
//    DMA instruction, ds_read_b128 in lane order: conflict free) — shared by the block's 8 waves instead of
//    8 L2 streams;
//  * one hand-counted s_waitcnt vmcnt(D) per chunk (D = this wave's DMAs for chunk g+2) and one raw
//    s_barrier per chunk; no ordinary global load inside the chunk loop (hipcc would drain the DMA queue
//    with vmcnt(0) in front of its first use).
// The compute image is swizzled ((pixel >> 3) & 1 flips the two 16-byte channel halves of a pixel), which
// makes the B-fragment ds_read_b128 (32 pixels x 2 halves per wave) bank-conflict free for every row and tap
// (brute-force checked over the lane groups of MI355X_MICROARCH.md's LDS table).
//
// Tile: 16 rows x 32 px x 64 output channels per workgroup of 8 waves (4 row groups x 2 channel halves);
// wave tile MI=4 rows x 32 px x 32 channels on v_mfma_f32_32x32x16 (D[co][px] = W[co][k] X[k][px]),
// persistent over M tiles.  Epilogues: y (16-bit) + BatchNorm partial sums, y + BatchNorm-backward
// sums (bnb_*), fp32 gradient (split / accumulate); the sums are per lane across the workgroup's tiles and
// reduced once (one partial row per wave row group: [.. gridDim.x * 4 ..]).
#include "conv_mfma32.h"
#include "lds_dma.h"

namespace unet {

// conv5w.hip: the 128-output-channel form (round 6), preferred wherever it serves
bool conv5w_ok(const unet_conv_desc* d);
int conv5w_stats_rows(const unet_conv_desc* d);
int conv5w_variant(const unet_conv_desc* d, char* buf, int len);
int conv5w_run(const unet_conv_desc* d, int prio, hipStream_t st);

constexpr int C5_W = 32, C5_HW = 34;     // tile width, halo width (pixels)
constexpr int C5_WM = 4;                 // wave row groups of a workgroup tile
constexpr int C5_WH = 2;                 // 32-channel halves of the block's 64 output channels
constexpr int C5_BN = 64;                // output channels per workgroup
constexpr int C5_CMAX = 1024;            // largest BN-activation source (scale / shift table)
constexpr int C5_TABS = C5_CMAX + 8;     // table stride: each half carries its own 8-float zero pad
constexpr int C5_NPAD = PACK_NPAD;       // packed weight rows are padded to this (conv_common.h)
constexpr int OM5_Y = 0, OM5_F32 = 1, OM5_BNB = 2;
// conv5's own source kind beside conv_src16.h's: one stored source whose channel count is a multiple of 16 (the
// dgrads' dy, the Down blocks' pooled map).  Like SK_ACT (one BN activation, host-checked C % 16 == 0), it lets
// the chunk DMA and transform drop the per-chunk source selection and ragged-chunk masks (round 5)
constexpr int SK5_PLAIN1 = 4;

template <int MI, bool ACT, int NWV>
struct C5Layout {
  static constexpr int TH = C5_WM * MI;
  static constexpr int HP = C5_HW * (TH + 2);       // halo pixels
  static constexpr int NS = 2 * HP;                 // 16-byte slots per chunk image
  static constexpr int NI = (NS + 63) / 64;         // DMA instructions per image
  static constexpr int DPW = (NI + NWV - 1) / NWV;
  static constexpr int IMG = NI * 1024;             // padded: the last instruction's tail lanes land inside
  static constexpr int NCOMP = ACT ? 2 : 3;
  static constexpr int WIMG = 9 * C5_WH * 1024;     // weight fragments of one chunk
  static constexpr int WPW = (9 * C5_WH + NWV - 1) / NWV;
  static constexpr int OFF_COMP = 0;
  static constexpr int OFF_RAW = OFF_COMP + NCOMP * IMG;
  static constexpr int OFF_W = OFF_RAW + (ACT ? 2 * IMG : 0);
  static constexpr int OFF_GATE = OFF_W + 3 * WIMG;
  static constexpr int GATE = NI * 256;             // per-lane gate pre-activations of one tile
  static constexpr int OFF_TAB = OFF_GATE + (ACT ? 2 * GATE : 0);
  static constexpr int OFF_BTAB = OFF_TAB + (ACT ? 2 * C5_TABS * 4 : 0);   // BNB: the block's BN affine
  static constexpr int OFF_JUNK = OFF_BTAB + 2 * C5_BN * 4;                   // target of the filler DMAs
  static constexpr int BYTES = OFF_JUNK + 1024;
};

// wave tile: MI rows x 32 px x 32 channels; SK: SK_PLAIN (every source stored as is), SK_ACT (one source, a BN
// activation) or SK_ACT_PLAIN (src0 a BN activation, src1 — if any — stored); GATE: src0 carries the attention
// gate (compile-time, so the transform is one straight-line block).  ABL (diagnostic ablations,
// unet_diag_conv5_ablate; 0 in the product): 1 no in-loop halo DMA, 2 no in-loop weight DMA, 4 no epilogue,
// 8 no per-chunk barrier, 16 no BN transform
// NWV: waves per workgroup.  8 = 4 row groups x 2 channel halves (two waves per SIMD, each 32 output
// channels); 4 = 4 row groups, each wave all 64 channels (one wave per SIMD with the whole 512-register file:
// every halo fragment it reads from LDS feeds twice the MFMAs — 12 reads per 24 MFMAs per tap column instead
// of 9 per 12 — and the two accumulator halves and both operand columns fit without spills)
// SPLIT (round 5, maps too small to fill the chip): blockIdx.z owns the 16-channel chunks [z*nch, (z+1)*nch) of
// the nch_all in the reduction and writes its fp32 partial sums to slab z of d.out ([S][N*H*W][Cout], OM5_F32,
// split == Cout, no accumulation: the host's descriptor); conv5_splitk_finish_kernel sums the slabs in order
template <typename T, int MI, int OM, int SK, int GATE, int ABL = 0, int PIPE = 1, int NWV = 8, bool SPLIT = false>
__global__ __launch_bounds__(64 * NWV, 1) void conv5_kernel(const unet_conv_desc d, int tiles_w, int tiles_h,
                                                           int mtiles, int nch, int nch_all, int prio) {
  using F = typename Mma32<T>::frag;
  constexpr bool ACT = SK != SK_PLAIN && SK != SK5_PLAIN1;
  constexpr bool ONE = SK == SK_ACT || SK == SK5_PLAIN1;   // one source, no ragged 16-channel chunk
  constexpr int WN = NWV / C5_WM, NJ = C5_WH / WN, NT = 64 * NWV;
  using Lay = C5Layout<MI, ACT, NWV>;
  constexpr int TH = Lay::TH, NS = Lay::NS, NI = Lay::NI, DPW = Lay::DPW, WPW = Lay::WPW;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[Lay::BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = WN == 2 ? wave >> 1 : wave, wn = WN == 2 ? (wave & 1) : 0;
  const int cw0 = blockIdx.y * C5_BN + wn * 32;     // this wave's first output channel (NJ blocks of 32)
  const int ntl = (mtiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;   // tiles of this block
  const int G = ntl * nch;                          // chunk steps of this block
  // a block's tiles are blockIdx.x + ti * gridDim.x: the first one by division, each next one by adding the
  // grid stride's (image, tile row, tile column) decomposition with carries (round 5: the signed divisions at
  // every tile change of three cursors were ~120 SALU per tile, paid over as few as 4 chunks on 64-channel maps)
  const int dW = (int)(gridDim.x % (unsigned)tiles_w), dT = (int)(gridDim.x / (unsigned)tiles_w);
  const int dH = dT % tiles_h, dN = dT / tiles_h;

  // ---- sources ----
  const unet_src& s0 = d.src[0];
  const unet_src& s1 = d.src[1];
  const int C0 = s0.C;
  const long long npix = (long long)d.N * d.H * d.W;
  const rsrc4_t rs0 = mk_rsrc4(s0.data, (unsigned)(npix * C0 * 2));
  const rsrc4_t rs1 = d.nsrc > 1 ? mk_rsrc4(s1.data, (unsigned)(npix * s1.C * 2)) : rs0;
  constexpr bool gated = ACT && GATE;
  const rsrc4_t rsg = mk_rsrc4(gated ? (const void*)s0.gate_p : s0.data, (unsigned)(npix * 4));
  float ga = 0.f, gb = 0.f;
  if (gated) { ga = s0.gate_ab[0]; gb = s0.gate_ab[1]; }
  const float lo = s0.relu ? 0.f : -INFINITY;

  // ---- weights: A fragment (32 output channels x 16 k) of the 16x16x32 fragment-major packing ----
  const int nch32 = (nch_all + 1) >> 1;
  const int kc0 = SPLIT ? (int)blockIdx.z * nch : 0;   // this block's first chunk of the reduction
  const unsigned jstride = (unsigned)nch32 * 9u * 1024u;
  const unsigned ntiles16 = (unsigned)((d.Cout + C5_NPAD - 1) / C5_NPAD * (C5_NPAD / 16));
  const rsrc4_t rw = mk_rsrc4(d.weight, ntiles16 * jstride);
  const rsrc_t ry = mk_rsrc(d.out, (unsigned)(npix * d.Cout * 2));   // y output (OM5_Y)
  const unsigned lanew = (unsigned)((lane >> 4) & 1) * jstride + (unsigned)(16 * (lane >> 5) + (lane & 15)) * 16u;

  // ---- this lane's halo DMA slots: instruction i = wave + k*NW covers slots 64 i .. 64 i + 63 ----
  // Every wave issues the same, compile-time number of DMA instructions per chunk (ND; + DPW gate loads at
  // a gated tile's first chunk), with no per-lane branch: instructions past the image go to a junk slot,
  // lanes past it (the last instruction's tail, inside the 1 KB-padded image) and zero-padding pixels load
  // out of range (zeros).  So the per-chunk wait is an immediate vmcnt and the chunk loop carries almost no
  // scalar work — the scalar unit is shared by the CU's 8 waves, and a version with per-slot exec branches,
  // divisions for the tile geometry and a switch over the wait count issued ~360 SALU per 36 MFMAs per
  // wave (SQ_INSTS_SALU), which paced the loop
  // Round 6: the compute image's swizzle is by the pixel's halo COLUMN x (x >> 3 & 1 flips the two 16-byte
  // channel halves), not by its image index, so a halo row is a fixed 1088-byte stride and the B fragments are
  // addressed by one base register per tap column plus an immediate per row (round 5: 18 offset registers and a
  // v_add per ds_read).  A plain source DMAs each slot's swizzled half directly; a BN-activation source lands
  // unswizzled (half = lane & 1: one scale / shift read per chunk) and its transform stores slot s ^ swz
  int hbit[DPW];        // channel half this lane's slot loads
  int soy[DPW], sox[DPW];   // the slot's pixel offset from the tile origin (halo: -1 .. TH, -1 .. 32)
  unsigned cso[ACT ? DPW : 1];   // ACT: the transformed slot's byte offset in the compute image
#pragma unroll
  for (int k = 0; k < DPW; ++k) {
    const int i = wave + k * NWV, s = i * 64 + lane;
    const int hp = s >> 1, x = hp % C5_HW, sw = (x >> 3) & 1;
    hbit[k] = ACT ? (lane & 1) : ((s & 1) ^ sw);
    if constexpr (ACT) cso[k] = (unsigned)(s ^ sw) * 16u;
    soy[k] = s < NS ? hp / C5_HW - 1 : -(1 << 20);    // past the image: never a valid row
    sox[k] = x - 1;
  }
  constexpr int ND = DPW + WPW;   // DMA instructions per wave per chunk (without gate loads)

  // B-fragment byte offsets in a compute image: tap column dx, row wm*MI (row rr adds rr * 1088, an immediate)
  unsigned boff[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int x = (lane & 31) + dx;
    boff[dx] = (unsigned)(wm * MI * 2 * C5_HW * 16 + 32 * x + 16 * ((lane >> 5) ^ ((x >> 3) & 1)));
  }

  // ring slots: compute images (PLAIN: 3 = chunk % 3; ACT: 2 = chunk & 1), raw images (ACT: chunk & 1),
  // weights (chunk % 3), gate pre-activations (tile & 1)
  auto comp_buf = [&](int slot) -> unsigned char* { return lds + Lay::OFF_COMP + slot * Lay::IMG; };
  auto raw_buf = [&](int slot) -> unsigned char* { return lds + Lay::OFF_RAW + slot * Lay::IMG; };
  auto w_buf = [&](int slot) -> unsigned char* { return lds + Lay::OFF_W + slot * Lay::WIMG; };
  auto gate_buf = [&](int ti) -> unsigned char* { return lds + Lay::OFF_GATE + (ti & 1) * Lay::GATE; };
  // the same regions as LDS byte addresses (scalars) for the DMAs' M0
  const unsigned l32 = lds_addr(lds);
  const unsigned junk = l32 + Lay::OFF_JUNK;

  // a chunk cursor: tile ti (origin n, h0, w0), 16-channel chunk c, ring slots of chunk index g
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
    q.w0 = q.tw * C5_W;
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
        q.w0 = q.tw * C5_W;
      }
    }
  };

  // Per-tile slot offsets, recomputed at a tile's first chunk (a wave-uniform branch), so that a chunk's DMA
  // and transform cost one add per slot: ib0 / ib1 = byte offset of the slot's pixel in src0 / src1 plus its
  // channel half (>= OOB for zero-padding pixels and slots past the image); xok / xao for the transform
  // cursor: the slot's pixel inside the image / its act_out byte offset (interior pixels only, else >= OOB)
  unsigned ib0[DPW], ib1[DPW], xao[DPW];
  bool xok[DPW];
  float xg[DPW];   // xok as a 0 / 1 multiplier (ONE: the zero-padding multiply without a per-chunk select)
  auto tile_slots = [&](const Cur& q, unsigned (&o0)[DPW], unsigned (&o1)[DPW]) {
    const unsigned pbase = ((unsigned)q.n * d.H + q.h0) * d.W + q.w0;
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const int y = q.h0 + soy[k], x = q.w0 + sox[k];
      const bool ok = ((unsigned)y < (unsigned)d.H) & ((unsigned)x < (unsigned)d.W);
      const unsigned pix = pbase + (unsigned)(soy[k] * d.W + sox[k]);
      o0[k] = ok ? (pix * (unsigned)C0 + 8u * hbit[k]) * 2u : OOB;
      o1[k] = ok ? (pix * (unsigned)(d.nsrc > 1 ? s1.C : C0) + 8u * hbit[k]) * 2u : OOB;
    }
  };

  // DMA of the chunk at cursor q: halo slots, weight fragments, and at a gated tile's first chunk the gate
  // pre-activations of this lane's slots (returns whether those went out: the chunk counts ND + DPW)
  auto issue = [&](const Cur& q, bool prologue) -> bool {
    if (q.c == 0) tile_slots(q, ib0, ib1);
    const int ca = q.c + kc0;                       // the chunk's index in the whole reduction
    const int cn0 = ca * 16;
    const bool s1sel = !ONE && d.nsrc > 1 && cn0 >= C0;
    const int cl = s1sel ? cn0 - C0 : cn0;
    const int Cs = s1sel ? s1.C : C0;
    const bool rag = !ONE && cl + 16 > Cs;          // the chunk's upper channel half is past the source
    const rsrc4_t rs = s1sel ? rs1 : rs0;
    const unsigned img = l32 + (ACT ? Lay::OFF_RAW + q.s2 * Lay::IMG : Lay::OFF_COMP + q.s3 * Lay::IMG);
    if (!(ABL & 1) || prologue) {
#pragma unroll
      for (int k = 0; k < DPW; ++k) {
        const int i = wave + k * NWV;
        unsigned vo = (s1sel ? ib1[k] : ib0[k]) + (unsigned)cl * 2u;   // stays >= OOB when the base is
        if (rag && hbit[k]) vo = OOB;
        dma16(rs, i < NI ? img + i * 1024 : junk, vo);
      }
    }
    if (!(ABL & 2) || prologue) {
      const unsigned wd = l32 + Lay::OFF_W + q.s3 * Lay::WIMG;
      const unsigned wofs = (unsigned)((ca >> 1) * 9) * 1024u + (unsigned)(ca & 1) * 512u;
#pragma unroll
      for (int k = 0; k < WPW; ++k) {
        const int j = wave + k * NWV;
        const int tap = j >> 1, wj = j & 1;
        const unsigned nt0 = (unsigned)((blockIdx.y * C5_BN + wj * 32) / 16);
        const unsigned vo = lanew + nt0 * jstride + (unsigned)tap * 1024u + wofs;
        dma16(rw, j < 9 * C5_WH ? wd + j * 1024 : junk, j < 9 * C5_WH ? vo : OOB);
      }
    }
    const bool gl = gated && q.c == 0;
    if (gl) {
      const unsigned gd = l32 + Lay::OFF_GATE + (q.ti & 1) * Lay::GATE;
      const unsigned pbase = ((unsigned)q.n * d.H + q.h0) * d.W + q.w0;
#pragma unroll
      for (int k = 0; k < DPW; ++k) {
        const int i = wave + k * NWV;
        const unsigned pix = pbase + (unsigned)(soy[k] * d.W + sox[k]);
        dma4(rsg, i < NI ? gd + i * 256 : junk, ib0[k] < OOB ? pix * 4u : OOB);
      }
    }
    return gl;
  };

  // BN-activation (+gate) transform of the chunk at cursor q, raw -> compute image, this lane's own slots
  // (zero-padding pixels and the image's tail slots come out 0).  Two channels per VALU op: v_pk_fma_f32 for
  // the affine (fp32, as before: the same roundings), the gate / zero-padding multiply as v_pk_mul_f32, and
  // ReLU after the 16-bit rounding as v_pk_max_i16 against 0 (a 16-bit float is negative iff its sign bit is
  // set; rounding is monotone and maps 0 to 0, and the multiplier is >= 0, so max(round(t*g), 0) equals
  // round(max(t, 0)*g) — the same bits up to the sign of zero)
  T* const aout = (ACT && OM == OM5_Y && blockIdx.y == 0) ? (T*)d.act_out : nullptr;
  const rsrc_t rao = mk_rsrc(aout ? (const void*)aout : d.out, (unsigned)(aout ? npix * C0 * 2 : 0));
  bool ns_prev = false;   // the last transform issued DPW act_out stores (after the DMA batch the next wait needs)
  typedef __attribute__((ext_vector_type(2))) float f2_t;
  typedef __attribute__((ext_vector_type(2))) short s2_t;
  const s2_t lo2 = s0.relu ? s2_t{0, 0} : s2_t{-32768, -32768};   // ReLU as a 16-bit integer max (no-op: -32768)
  auto transform = [&](const Cur& q) {
    if (q.c == 0) {
      const unsigned pbase = ((unsigned)q.n * d.H + q.h0) * d.W + q.w0;
#pragma unroll
      for (int k = 0; k < DPW; ++k) {
        const int y = q.h0 + soy[k], x = q.w0 + sox[k];
        xok[k] = ((unsigned)y < (unsigned)d.H) & ((unsigned)x < (unsigned)d.W);
        xg[k] = xok[k] ? 1.f : 0.f;
        const bool in = xok[k] && (unsigned)soy[k] < (unsigned)TH && (unsigned)sox[k] < (unsigned)C5_W &&
                        wave + k * NWV < NI;    // (dead slots: OOB here, so the store offset needs no select)
        const unsigned pix = pbase + (unsigned)(soy[k] * d.W + sox[k]);
        xao[k] = in ? (pix * (unsigned)C0 + 8u * hbit[k]) * 2u : OOB;
      }
    }
    const int cn0 = (q.c + kc0) * 16;
    // src0 (activation) or, for SK_ACT_PLAIN, src1 (stored: copied)
    const bool act = SK == SK_ACT || !(d.nsrc > 1 && cn0 >= C0);
    const bool rag = !ONE && cn0 + 16 > C0;
    const unsigned char* rb = raw_buf(q.s2);
    unsigned char* cb = comp_buf(q.s2);
    const float* tab = reinterpret_cast<const float*>(lds + Lay::OFF_TAB);
    // this lane's 8 channels' scale / shift, read once per chunk (an activation source's slots all load the
    // lane's half lane & 1; the compiler would re-read them per slot: the stores may alias the table)
    f2_t sc[4], sf[4];
    if (act) {
      const int ch = cn0 + 8 * hbit[0];             // < C0 + 8: the table is zero-padded there
      const float4 a0 = *reinterpret_cast<const float4*>(tab + ch);
      const float4 a1 = *reinterpret_cast<const float4*>(tab + ch + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(tab + C5_TABS + ch);
      const float4 b1 = *reinterpret_cast<const float4*>(tab + C5_TABS + ch + 4);
      sc[0] = f2_t{a0.x, a0.y}; sc[1] = f2_t{a0.z, a0.w}; sc[2] = f2_t{a1.x, a1.y}; sc[3] = f2_t{a1.z, a1.w};
      sf[0] = f2_t{b0.x, b0.y}; sf[1] = f2_t{b0.z, b0.w}; sf[2] = f2_t{b1.x, b1.y}; sf[3] = f2_t{b1.z, b1.w};
    }
#pragma unroll
    for (int k = 0; k < DPW; ++k) {
      const int i = wave + k * NWV;
      const bool live = i < NI;                      // slots past the image: the junk region (no branch)
      const int s = i * 64 + lane;
      const unsigned so = live ? (unsigned)s * 16u : (unsigned)(Lay::OFF_JUNK + lane * 16);
      uint4 q4 = *reinterpret_cast<const uint4*>((live ? rb : lds) + so);
      if (act) {
        const bool ok = xok[k] && !(rag && hbit[k]);   // ONE: rag is false
        float gm = ONE ? xg[k] : (ok ? 1.f : 0.f);
        if constexpr (gated) {
          // (a padding or dead slot's gate value is a zero load: sigmoid stays finite, times xg = 0)
          const float pv = *reinterpret_cast<const float*>(gate_buf(q.ti) + (live ? i : 0) * 256 + lane * 4);
          gm = ONE ? xg[k] * sigmoidf_(pv * ga + gb) : (ok ? sigmoidf_(pv * ga + gb) : 0.f);
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
        // act_out: the first output-channel block writes the transformed interior once (the weight
        // gradient then reads it as a stored map) — a buffer store per slot, out-of-range for halo, padding
        // and dead slots and in the other blocks (zero-size resource), so every transform of an activation
        // chunk issues exactly DPW (ns_prev: the next chunk's wait leaves them in flight)
        if constexpr (OM == OM5_Y) {
          const unsigned vo = (ONE || !(rag && hbit[k])) ? xao[k] + (unsigned)cn0 * 2u : OOB;
          typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, q4), rao, (int)vo, 0, 0);
        }
      }
      if constexpr (ACT) *reinterpret_cast<uint4*>(live ? cb + cso[k] : lds + so) = q4;
    }
    if constexpr (OM == OM5_Y) ns_prev = act;
  };

  // ---- prologue: scale/shift table, chunks 0-2 in flight, chunk 0 ready ----
  if constexpr (ACT) {
    float* tab = reinterpret_cast<float*>(lds + Lay::OFF_TAB);
    for (int c = tid; c < C0; c += NT) { tab[c] = s0.scale[c]; tab[C5_TABS + c] = s0.shift[c]; }
    if (tid < 8) { tab[C0 + tid] = 0.f; tab[C5_TABS + C0 + tid] = 0.f; }   // C0 <= C5_CMAX: inside each half
  }
  if constexpr (OM == OM5_BNB) {
    // the BN affine of the activation whose gradient this dgrad writes (its ReLU mask), the block's channels
    float* bt = reinterpret_cast<float*>(lds + Lay::OFF_BTAB);
    if (tid < C5_BN) {
      const int co = (int)blockIdx.y * C5_BN + tid;
      const bool ok = co < d.Cout && d.bnb_relu;
      bt[tid] = ok ? d.bnb_scale[co] : 0.f;
      bt[C5_BN + tid] = ok ? d.bnb_shift[co] : 0.f;
    }
  }
  // cursors: I = the next chunk to DMA, X = the next chunk to transform (ACT), K = the chunk being computed.
  // G >= 2 (nch >= 2).  The youngest DMA'd chunk's instruction count decides each wait: ND, ND + DPW (gate
  // loads went out with it) or none in flight (0).
  Cur I, X, K;
  cur_init(I);
  cur_init(K);
  issue(I, true);
  cur_next(I);
  issue(I, true);           // chunk 1: never a tile's first chunk (nch >= 2)
  cur_next(I);
  wait_vm<ND>();            // chunk 0 landed
  if constexpr (ACT) {
    lds_barrier();          // the scale/shift table
    cur_init(X);
    transform(X);           // chunk 0; then chunk 2 may reuse its raw slot
    cur_next(X);
  }
  bool y_live = G > 2, y_big = false;
  if (y_live) {
    y_big = issue(I, true);
    cur_next(I);
  }
  lds_barrier();

  // BatchNorm sums of this lane's pixel column over the block's tiles (reduced once, after the last tile)
  constexpr bool SUMS = OM == OM5_Y || OM == OM5_BNB;
  float sA[NJ][16], sB[NJ][16];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) { sA[j][r] = 0.f; sB[j][r] = 0.f; }
  f32x16 acc[MI][NJ];

  // operand fragments of one tap column dx of the chunk at K: MI+2 halo rows (B) and the 3 taps' weights (A)
  auto load_col = [&](const Cur& q, int dx, F (&x)[MI + 2], F (&w)[3][NJ]) {
    const unsigned char* xb = comp_buf(ACT ? q.s2 : q.s3);
    const unsigned char* wb = w_buf(q.s3) + wn * NJ * 1024 + lane * 16;
#pragma unroll
    for (int rr = 0; rr < MI + 2; ++rr) x[rr] = *reinterpret_cast<const F*>(xb + boff[dx] + rr * (2 * C5_HW * 16));
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int j = 0; j < NJ; ++j) w[dy][j] = *reinterpret_cast<const F*>(wb + j * 1024 + (dy * 3 + dx) * 2048);
  };
  auto mma_col = [&](const F (&x)[MI + 2], const F (&w)[3][NJ]) {
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < MI; ++i) acc[i][j] = Mma32<T>::mma(w[dy][j], x[i + dy], acc[i][j]);
  };
  // this wave's DMAs of the chunk after K have landed: only the youngest chunk's may still be in flight
  // (the y epilogue's NST stores sit between DMA batches for the two chunks after it: sw counts them down)
  // (BNB: the epilogue's 2 MI 16-byte g stores likewise; and the tile's NYL y1 loads, issued at the start of
  // its last chunk — after the two in-flight DMA batches — are counted by that chunk's wait: yl)
  constexpr int NST = NJ * (OM == OM5_Y || OM == OM5_BNB ? 2 * MI : (OM == OM5_F32 ? 4 * MI : 0));
  typedef __attribute__((ext_vector_type(4))) unsigned u32x4_t;
  // F32 without accumulation: counted buffer stores (no RMW loads, whose compiler waits drain the DMA queue)
  const bool f32_counted = OM == OM5_F32 && !d.accum && !d.accum2 && (d.split % 8) == 0 &&
                           (double)npix * d.Cout * 4 < (double)OOB;
  const rsrc_t rf1 = mk_rsrc(SPLIT ? (const void*)((const char*)d.out + (size_t)blockIdx.z * (size_t)npix * d.Cout * 4) : d.out,
                             (unsigned)(f32_counted ? npix * d.split * 4 : 0));
  const rsrc_t rf2 = mk_rsrc(d.out2 ? d.out2 : d.out, (unsigned)(f32_counted ? npix * (d.Cout - d.split) * 4 : 0));
  constexpr int NYL = OM == OM5_BNB ? 2 * MI * NJ : 0;
  int sw = 0;
  auto wait_next = [&](bool yl) {
    const bool st = NST && sw > 0;
    if (!y_live) wait_vm<0>();
    else if (NYL && yl) {
      if (y_big) wait_vm<ND + DPW + NYL>();
      else wait_vm<ND + NYL>();
    } else if (st && ns_prev) {
      if (y_big) wait_vm<ND + DPW + NST + DPW>();
      else wait_vm<ND + NST + DPW>();
    } else if (st) {
      if (y_big) wait_vm<ND + DPW + NST>();
      else wait_vm<ND + NST>();
    } else if (ns_prev) {
      if (y_big) wait_vm<ND + DPW + DPW>();
      else wait_vm<ND + DPW>();
    } else {
      if (y_big) wait_vm<ND + DPW>();
      else wait_vm<ND>();
    }
    if (st) --sw;
  };
  auto issue_next = [&]() {
    // called right after a chunk's barrier: every wave has finished reading chunk K, whose ring slots
    // the DMA of chunk K+3 (the cursor I) reuses
    y_live = I.ti < ntl;
    if (y_live) {
      y_big = issue(I, false);
      cur_next(I);
    }
  };

  F xA[MI + 2], wA[3][NJ], xB[MI + 2], wB[3][NJ];
  // PIPE 1: the operands of tap column dx+1 are read from LDS while the MFMAs of column dx run (pinned
  // one ds_read per MFMA by sched_group_barrier), and column 0 of the next chunk right after the barrier.
  // hipcc's own schedule (PIPE 0) reads every fragment just before its MFMA with an lgkmcnt(0) in between;
  // PIPE 1 measured 5-9 % faster per layer for the y / fp32 epilogues (launch5)
  auto pin_col = [&]() {
    if constexpr (PIPE) {
      constexpr int NDS = MI + 2 + 3 * NJ, NMF = 3 * MI * NJ;   // reads of the next column, MFMAs of this one
      constexpr int NP = NDS < NMF ? NDS : NMF;
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      }
      if constexpr (NMF > NP) __builtin_amdgcn_sched_group_barrier(0x008, NMF - NP, 0);
      if constexpr (NDS > NP) __builtin_amdgcn_sched_group_barrier(0x100, NDS - NP, 0);   // (MI = 2: 7 reads, 6 MFMAs)
    }
  };
  if constexpr (PIPE) load_col(K, 0, xA, wA);
  // static priority for the second-dispatched half (MI355X_MICROARCH.md, two waves per SIMD, item 4): waves 4-7
  // share their SIMDs with waves 0-3 and lose every issue arbitration by age
  if (prio && wave >= NWV / 2) __builtin_amdgcn_s_setprio(1);
  // BNB: the activation y1 of this wave's tile pixels (buffer loads, out-of-range offsets for masked lanes:
  // a fixed count), loaded during the tile's last chunk so that the epilogue's wait for them does not drain
  // the next chunks' DMAs (their issue follows the epilogue).  16-byte loads in the layout of the epilogue's
  // swapped g stores: lanes 0-31 channels 16h+0..7 of their pixel, lanes 32-63 channels 16h+8..15
  uint4 yv[OM == OM5_BNB ? MI : 1][NJ][2];
  const rsrc_t ry1 = mk_rsrc(OM == OM5_BNB ? d.bnb_y : d.out, (unsigned)(npix * d.Cout * 2));
  auto load_y1 = [&](const Cur& q) {   // K's tile (its last chunk)
    const int n = q.n, h0 = q.h0, w0 = q.w0;
    const int ow = w0 + (lane & 31), oh0 = h0 + wm * MI;
    const unsigned pix0 = ((unsigned)n * d.H + oh0) * (unsigned)d.W + ow;
#pragma unroll
    for (int i = 0; i < (OM == OM5_BNB ? MI : 0); ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int co = cw0 + 32 * j + 16 * h + 8 * (lane >> 5);
          const bool ok = ow < d.W && oh0 + i < d.H && co < d.Cout;
          const unsigned vo = ok ? ((pix0 + (unsigned)i * d.W) * (unsigned)d.Cout + (unsigned)co) * 2u : OOB;
          yv[i][j][h] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ry1, (int)vo, 0, 0));
        }
  };
  for (int ti = 0; ti < ntl; ++ti) {
    const int tn = K.n, th0 = K.h0, tw0 = K.w0;     // this tile's origin (K is at its first chunk)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
      // one tap column at a time; the barrier ends the chunk (after it: chunk K's slots are free and the
      // next chunk is readable by every wave)
      const bool last = c == nch - 1;
      if constexpr (OM == OM5_BNB) {
        if (last) load_y1(K);
      }
      if constexpr (PIPE) {
        load_col(K, 1, xB, wB);
        mma_col(xA, wA);
        pin_col();
        load_col(K, 2, xA, wA);
        mma_col(xB, wB);
        pin_col();
      } else {
        load_col(K, 0, xA, wA);
        mma_col(xA, wA);
        load_col(K, 1, xB, wB);
        mma_col(xB, wB);
      }
      wait_next(last);
      if constexpr (ACT && !(ABL & 16)) {
        if (X.ti < ntl) {
          transform(X);
          cur_next(X);
        }
      }
      if constexpr (!PIPE) load_col(K, 2, xA, wA);
      mma_col(xA, wA);
      if constexpr (!(ABL & 8)) lds_barrier();
      if (OM != OM5_BNB || !last) issue_next();
      cur_next(K);
      // the next chunk's column 0 (past the block's last chunk: harmless reads of stale LDS)
      if constexpr (PIPE) load_col(K, 0, xA, wA);
    }

    // ---------------- epilogue of tile ti ----------------
    if constexpr (ABL & 4) {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) sum += acc[i][0][0] + acc[i][NJ - 1][7] + acc[i][0][15];
      if (sum == 12345.f) ((float*)d.out)[tid] = sum;
      continue;
    }
    const int n = tn, h0 = th0, w0 = tw0;
    const int pxl = lane & 31, hh = lane >> 5;
    const int ow = w0 + pxl;
    const bool colok = ow < d.W;
    const int oh0 = h0 + wm * MI;
    int rows = d.H - oh0;
    rows = rows < 0 ? 0 : (rows > MI ? MI : rows);
    const unsigned pix0 = ((unsigned)n * d.H + oh0) * (unsigned)d.W + ow;
    if constexpr (OM == OM5_Y) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bool ok = colok && i < rows;
        const unsigned pix = pix0 + (unsigned)i * d.W;
        // lane l < 32 holds channels 8gq+0..3 of pixel l, lane l+32 channels 8gq+4..7 of the same pixel:
        // v_permlane32_swap of the packed groups (gq, gq+1) leaves lanes 0-31 with channels 8gq..8gq+7 and
        // lanes 32-63 with 8gq+8..8gq+15 — one 16-byte store per pair instead of two 8-byte ones
        // Buffer stores with out-of-range offsets for the masked lanes: every wave issues exactly NST stores
        // per tile (no exec branch), which the next chunks' vmcnt waits count (wait_next)
        unsigned px_[4], py_[4];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          px_[gq] = pack2_16<T>(acc[i][j][4 * gq], acc[i][j][4 * gq + 1]);
          py_[gq] = pack2_16<T>(acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
        }
#pragma unroll
        for (int kp = 0; kp < 4; kp += 2) {
          const auto sx = __builtin_amdgcn_permlane32_swap(px_[kp], px_[kp + 1], false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(py_[kp], py_[kp + 1], false, false);
          const int co = cw0 + 32 * j + 8 * kp + 8 * hh;
          const unsigned vo = (ok && co < d.Cout) ? (pix * (unsigned)d.Cout + (unsigned)co) * 2u : OOB;
          typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
          const u32x4 v4 = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v4, ry, (int)vo, 0, 0);
        }
      }
      sw = 2;
      if (d.stats) {
        // channel pairs on v_pk_add_f32 / v_pk_fma_f32 (each element's sum in the same order); the masks only
        // on a tile that crosses the map's bottom or right edge (wave-uniform)
        typedef __attribute__((ext_vector_type(2))) float f2s;
        const bool full = rows == MI && w0 + C5_W <= d.W;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int r = 0; r < 16; r += 2) {
            f2s a2 = {sA[j][r], sA[j][r + 1]}, b2 = {sB[j][r], sB[j][r + 1]};
            if (full) {
#pragma unroll
              for (int i = 0; i < MI; ++i) {
                const f2s x2 = {acc[i][j][r], acc[i][j][r + 1]};
                a2 += x2;
                b2 = __builtin_elementwise_fma(x2, x2, b2);
              }
            } else {
#pragma unroll
              for (int i = 0; i < MI; ++i) {
                const bool ok = colok && i < rows;
                const f2s x2 = {ok ? acc[i][j][r] : 0.f, ok ? acc[i][j][r + 1] : 0.f};
                a2 += x2;
                b2 = __builtin_elementwise_fma(x2, x2, b2);
              }
            }
            sA[j][r] = a2.x; sA[j][r + 1] = a2.y;
            sB[j][r] = b2.x; sB[j][r + 1] = b2.y;
          }
      }
    } else if constexpr (OM == OM5_BNB) {
      // g stored as buffer stores (fixed count NST, out-of-range offsets mask lanes); the BN affine of the
      // block's channels from the LDS table the prologue filled; y1 from the loads of the last chunk
      const float* btab = reinterpret_cast<const float*>(lds + Lay::OFF_BTAB);
      const rsrc_t rg = mk_rsrc(d.out, (unsigned)(npix * d.Cout * 2));
      // g packed and v_permlane32_swap'ed as the y epilogue (one 16-byte store per 8 channels): this lane then
      // holds channels co..co+7 (co = cw0 + 32j + 16h + 8hh) of its pixel — sum slot 8h + r is channel co + r
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int co = cw0 + 32 * j + 16 * h + 8 * hh;
        const bool cok = co < d.Cout;
        const int cb = co - (int)blockIdx.y * C5_BN;
        float sc8[8], sf8[8];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float4 a4 = *reinterpret_cast<const float4*>(btab + cb + 4 * q);
          const float4 b4 = *reinterpret_cast<const float4*>(btab + C5_BN + cb + 4 * q);
          sc8[4 * q] = a4.x; sc8[4 * q + 1] = a4.y; sc8[4 * q + 2] = a4.z; sc8[4 * q + 3] = a4.w;
          sf8[4 * q] = b4.x; sf8[4 * q + 1] = b4.y; sf8[4 * q + 2] = b4.z; sf8[4 * q + 3] = b4.w;
        }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const unsigned pix = pix0 + (unsigned)i * d.W;
          const bool ok = colok && i < rows && cok;
          const int g0 = 2 * h;
          const unsigned pxa = pack2_16<T>(acc[i][j][4 * g0], acc[i][j][4 * g0 + 1]);
          const unsigned pxb = pack2_16<T>(acc[i][j][4 * g0 + 4], acc[i][j][4 * g0 + 5]);
          const unsigned pya = pack2_16<T>(acc[i][j][4 * g0 + 2], acc[i][j][4 * g0 + 3]);
          const unsigned pyb = pack2_16<T>(acc[i][j][4 * g0 + 6], acc[i][j][4 * g0 + 7]);
          const auto sx = __builtin_amdgcn_permlane32_swap(pxa, pxb, false, false);
          const auto sy = __builtin_amdgcn_permlane32_swap(pya, pyb, false, false);
          const unsigned vo = ok ? (pix * (unsigned)d.Cout + (unsigned)co) * 2u : OOB;
          const u32x4_t v4 = {sx[0], sy[0], sx[1], sy[1]};
          __builtin_amdgcn_raw_buffer_store_b128(v4, rg, (int)vo, 0, 0);
          if (ok) {
            float gv[8], yy[8];
            unpack4_16<T>(make_uint2(v4[0], v4[1]), gv);
            unpack4_16<T>(make_uint2(v4[2], v4[3]), gv + 4);
            unpack4_16<T>(make_uint2(yv[i][j][h].x, yv[i][j][h].y), yy);
            unpack4_16<T>(make_uint2(yv[i][j][h].z, yv[i][j][h].w), yy + 4);
#pragma unroll
            for (int r = 0; r < 8; ++r) {
              const float gg = (d.bnb_relu && !(yy[r] * sc8[r] + sf8[r] > 0.f)) ? 0.f : gv[r];
              sA[j][8 * h + r] += gg;
              sB[j][8 * h + r] = __builtin_fmaf(gg, yy[r], sB[j][8 * h + r]);
            }
          }
        }
      }
      issue_next();     // the last chunk's DMA, deferred behind the y1 wait
      sw = 1;           // the next chunk's wait leaves the NST stores (older than that DMA) in flight
    } else if (f32_counted) {  // OM5_F32, plain stores: buffer stores, fixed count NST (sw as the y epilogue)
      const int c2 = d.Cout - d.split;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const unsigned pix = pix0 + (unsigned)i * d.W;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int co = cw0 + 32 * j + 8 * gq + 4 * hh;
          const bool to1 = cw0 + 32 * j + 8 * gq < d.split;     // wave-uniform (split % 8 == 0)
          const bool ok = colok && i < rows && co < d.Cout;
          const unsigned vo = !ok ? OOB : to1 ? (pix * (unsigned)d.split + (unsigned)co) * 4u
                                             : (pix * (unsigned)c2 + (unsigned)(co - d.split)) * 4u;
          typedef __attribute__((ext_vector_type(4))) float f32x4v;
          const f32x4v w = {acc[i][j][4 * gq], acc[i][j][4 * gq + 1], acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, w), to1 ? rf1 : rf2, (int)vo, 0, 0);
        }
      }
      sw = 2;
    } else if constexpr (!SPLIT) {  // OM5_F32 with read-modify-write (accumulating into an existing gradient;
      // never a split-K slab: launch5_split_mi's descriptors always take the counted stores above)
      float* o1 = (float*)d.out;
      float* o2 = (float*)d.out2;
      const int c2 = d.Cout - d.split;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if (!(colok && i < rows)) continue;
        const unsigned pix = pix0 + (unsigned)i * d.W;
        float4* pp[4];
        float4 old[4];
        bool acc_in[4];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int co = cw0 + 32 * j + 8 * gq + 4 * hh;
          if (co < d.split) {
            pp[gq] = reinterpret_cast<float4*>(o1 + (size_t)pix * d.split + co);
            acc_in[gq] = d.accum;
          } else {
            pp[gq] = reinterpret_cast<float4*>(o2 + (size_t)pix * c2 + (co - d.split));
            acc_in[gq] = d.accum2;
          }
          old[gq] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (co < d.Cout && acc_in[gq]) old[gq] = *pp[gq];
        }
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int co = cw0 + 32 * j + 8 * gq + 4 * hh;
          if (co < d.Cout) {
            float4 w = make_float4(acc[i][j][4 * gq], acc[i][j][4 * gq + 1], acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
            if (acc_in[gq]) { w.x += old[gq].x; w.y += old[gq].y; w.z += old[gq].z; w.w += old[gq].w; }
            *pp[gq] = w;
          }
        }
      }
    }
  }

  // ---- the workgroup's BatchNorm sums: one partial row per wave row group ----
  if constexpr (SUMS) {
    const int hh = lane >> 5;
    const int srow = blockIdx.x * C5_WM + wm, srows = gridDim.x * C5_WM;
    if constexpr (OM == OM5_Y) {
      if (d.stats) {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float a = half32_sum(sA[j][r]), b = half32_sum(sB[j][r]);
          const int co = cw0 + 32 * j + 8 * (r >> 2) + 4 * hh + (r & 3);
          if ((lane & 31) == 0 && co < d.Cout) {
            d.stats[(size_t)co * srows + srow] = a;
            d.stats[((size_t)d.Cout + co) * srows + srow] = b;
          }
        }
      }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {   // slot 8h + r: channel cw0 + 32j + 16h + 8hh + r (the BNB epilogue)
        const int co = cw0 + 32 * j + 16 * (gq >> 1) + 8 * hh + 4 * (gq & 1);
        float a[4], b[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          a[r] = half32_sum(sA[j][4 * gq + r]);
          b[r] = half32_sum(sB[j][4 * gq + r]);
        }
        if ((lane & 31) == 0 && co < d.Cout) {
          const float4 m4 = *reinterpret_cast<const float4*>(d.bnb_mean + co);
          const float4 i4 = *reinterpret_cast<const float4*>(d.bnb_invstd + co);
          const float mu[4] = {m4.x, m4.y, m4.z, m4.w}, is[4] = {i4.x, i4.y, i4.z, i4.w};
#pragma unroll
          for (int r = 0; r < 4; ++r) b[r] = is[r] * (b[r] - mu[r] * a[r]);
          *reinterpret_cast<float4*>(d.bnb_stats + (size_t)srow * d.Cout + co) = make_float4(a[0], a[1], a[2], a[3]);
          *reinterpret_cast<float4*>(d.bnb_stats + ((size_t)srows + srow) * d.Cout + co) =
              make_float4(b[0], b[1], b[2], b[3]);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// split-K finisher: out = sum over the S slabs of ws ([S][npix][Cout] fp32, in slab order) through the conv's
// real epilogue.  Block = CV = Cout/4 channel vectors x R = 256/CV pixel lanes over a contiguous pixel range
// (one partial-sum row per block, like one conv5 workgroup row).  MODE 0: y (op dtype) + the BN partial sums of
// the fp32 sums (stats[2][Cout][rows], as conv5's y epilogue sums its accumulators); 1: y + the BatchNorm-backward
// sums of the stored gradient (bnb_stats[2][rows][Cout], conv5's OM5_BNB); 2: fp32, split across out / out2,
// optionally accumulating
// ------------------------------------------------------------------------------------------------
constexpr int FIN_TRIPS = 8;   // pixels per lane of a finisher block (fin_rows)
template <typename T, int MODE, int S>
__global__ __launch_bounds__(256) void conv5_splitk_finish_kernel(const unet_conv_desc d, const float* __restrict__ ws,
                                                                  int rows) {
  __shared__ float4 red[2][256];
  const int CV = d.Cout >> 2, R = 256 / CV, tid = threadIdx.x;
  const int cv = tid % CV, r = tid / CV, co = cv * 4;
  const long long npix = (long long)d.N * d.H * d.W;
  const long long per = (npix + rows - 1) / rows;
  const long long p0 = (long long)blockIdx.x * per, p1 = min(npix, p0 + per);
  const size_t slab = (size_t)npix * d.Cout;
  float4 sa = make_float4(0.f, 0.f, 0.f, 0.f), sb = sa;
  float4 sc = sa, sf = sa;
  if constexpr (MODE == 1) {
    if (d.bnb_relu) {
      sc = *reinterpret_cast<const float4*>(d.bnb_scale + co);
      sf = *reinterpret_cast<const float4*>(d.bnb_shift + co);
    }
  }
  // FIN_TRIPS pixels per lane at once: every slab load (and the BNB y1 loads) of a lane issued before the first
  // add — one memory round trip per batch instead of one per pixel (the loop was latency-bound: 10-17 us for a
  // 4 x 32^2 x 512 finish, profiles/r05_conv5_split_ablate.txt).  Per element the slabs still add in slab order
  // and each lane's BN sums in pixel order: the same results as one pixel at a time.
  constexpr int U = FIN_TRIPS;
  for (long long pb = p0 + r; pb < p1; pb += (long long)R * U) {
    float4 v[U];
    uint2 yb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long p = pb + (long long)u * R;
      const long long pc = p < p1 ? p : p1 - 1;     // clamped: loads unconditional, results unused past p1
      v[u] = *reinterpret_cast<const float4*>(ws + (size_t)pc * d.Cout + co);
      if constexpr (MODE == 1) yb[u] = *reinterpret_cast<const uint2*>((const T*)d.bnb_y + (size_t)pc * d.Cout + co);
    }
#pragma unroll
    for (int z = 1; z < S; ++z)
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long p = pb + (long long)u * R;
        const long long pc = p < p1 ? p : p1 - 1;
        const float4 q = *reinterpret_cast<const float4*>(ws + (size_t)z * slab + (size_t)pc * d.Cout + co);
        v[u].x += q.x; v[u].y += q.y; v[u].z += q.z; v[u].w += q.w;
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long p = pb + (long long)u * R;
      if (p >= p1) break;
      const float4 vv = v[u];
      if constexpr (MODE == 0 || MODE == 1) {
        uint2 pk;
        pk.x = pack2_16<T>(vv.x, vv.y);
        pk.y = pack2_16<T>(vv.z, vv.w);
        *reinterpret_cast<uint2*>((T*)d.out + (size_t)p * d.Cout + co) = pk;
        if constexpr (MODE == 0) {
          sa.x += vv.x; sa.y += vv.y; sa.z += vv.z; sa.w += vv.w;
          sb.x = __builtin_fmaf(vv.x, vv.x, sb.x); sb.y = __builtin_fmaf(vv.y, vv.y, sb.y);
          sb.z = __builtin_fmaf(vv.z, vv.z, sb.z); sb.w = __builtin_fmaf(vv.w, vv.w, sb.w);
        } else {
          float g[4], y[4];
          unpack4_16<T>(pk, g);
          unpack4_16<T>(yb[u], y);
          const float scv[4] = {sc.x, sc.y, sc.z, sc.w}, sfv[4] = {sf.x, sf.y, sf.z, sf.w};
          float gg[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) gg[k] = (d.bnb_relu && !(y[k] * scv[k] + sfv[k] > 0.f)) ? 0.f : g[k];
          sa.x += gg[0]; sa.y += gg[1]; sa.z += gg[2]; sa.w += gg[3];
          sb.x = __builtin_fmaf(gg[0], y[0], sb.x); sb.y = __builtin_fmaf(gg[1], y[1], sb.y);
          sb.z = __builtin_fmaf(gg[2], y[2], sb.z); sb.w = __builtin_fmaf(gg[3], y[3], sb.w);
        }
      } else {
        float4* o;
        int acc;
        if (co < d.split) { o = reinterpret_cast<float4*>((float*)d.out + (size_t)p * d.split + co); acc = d.accum; }
        else { o = reinterpret_cast<float4*>((float*)d.out2 + (size_t)p * (d.Cout - d.split) + (co - d.split)); acc = d.accum2; }
        float4 w = vv;
        if (acc) {
          const float4 b2 = *o;
          w.x += b2.x; w.y += b2.y; w.z += b2.z; w.w += b2.w;
        }
        *o = w;
      }
    }
  }
  if constexpr (MODE == 0 || MODE == 1) {
    if (MODE == 0 && !d.stats) return;
    red[0][tid] = sa;
    red[1][tid] = sb;
    __syncthreads();
    if (r == 0) {
      float4 a = red[0][cv], b = red[1][cv];
      for (int k = 1; k < R; ++k) {
        const float4 x = red[0][k * CV + cv], y = red[1][k * CV + cv];
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
        b.x += y.x; b.y += y.y; b.z += y.z; b.w += y.w;
      }
      if constexpr (MODE == 0) {
        const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          d.stats[(size_t)(co + k) * rows + blockIdx.x] = av[k];
          d.stats[(size_t)(d.Cout + co + k) * rows + blockIdx.x] = bv[k];
        }
      } else {
        const float4 m4 = *reinterpret_cast<const float4*>(d.bnb_mean + co);
        const float4 i4 = *reinterpret_cast<const float4*>(d.bnb_invstd + co);
        b = make_float4(i4.x * (b.x - m4.x * a.x), i4.y * (b.y - m4.y * a.y), i4.z * (b.z - m4.z * a.z),
                        i4.w * (b.w - m4.w * a.w));
        *reinterpret_cast<float4*>(d.bnb_stats + (size_t)blockIdx.x * d.Cout + co) = a;
        *reinterpret_cast<float4*>(d.bnb_stats + ((size_t)rows + blockIdx.x) * d.Cout + co) = b;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
constexpr int C5_MI = 4;      // wave-tile rows of the large maps (16-row workgroup tiles)
constexpr int C5_MI_S = 2;    // and of the small ones (8-row tiles: twice the tiles, round 5)

// UNET_CONV5: unset = the measured default (below), 0 = never (conv3 everywhere), 1 = every eligible conv
// (tests, ablations); read per call so tests can flip it
static int conv5_mode() {
  const char* e = getenv("UNET_CONV5");
  return e ? (atoi(e) ? 1 : 0) : 2;
}

// UNET_C5_PRIO=1: s_setprio 1 for waves 4-7 (A/B; read per call)
static int conv5_prio() {
  const char* e = getenv("UNET_C5_PRIO");
  return e ? atoi(e) : 0;
}

static long long conv5_mtiles(const unet_conv_desc* d, int mi) {
  return (long long)d->N * cdiv(d->W, C5_W) * cdiv(d->H, C5_WM * mi);
}

// MI of a descriptor: 4 where its 16 x 32 x 64 tiles fill the chip (>= 256 workgroups), else 2 — 8 x 32 x 64
// tiles, twice as many (the 64^2 layers then need no split-K, the 32^2 ones half the splits).  The 2-row wave
// tile reads 7 LDS fragments per 6 MFMAs per tap column instead of 9 per 12 (LDS-bound nearer the MFMA peak)
// but drops the split slabs' HBM round trip and the finisher.  UNET_CONV5_MI2=0: MI = 4 everywhere (A/B).
static int conv5_mi(const unet_conv_desc* d) {
  const char* e = getenv("UNET_CONV5_MI2");   // read per call
  if (e && !atoi(e)) return C5_MI;
  if (e && atoi(e) == 2) return C5_MI_S;      // (diagnostic: 8-row tiles everywhere)
  return conv5_mtiles(d, C5_MI) * cdiv(d->Cout, C5_BN) >= 256 ? C5_MI : C5_MI_S;
}

static int conv5_gx(const unet_conv_desc* d, int mi) {
  const long long mt = conv5_mtiles(d, mi);
  const int gy = cdiv(d->Cout, C5_BN);
  long long gx = cdiv(256, gy);                     // one 8-wave workgroup per CU (LDS), persistent
  if (gx > mt) gx = mt;
  if (gx < 1) gx = 1;
  return (int)gx;
}

// 16-bit 3x3; stored or BN-activation sources (src0 may be gated, src1 stored; the network's pooled and
// upsampled maps are materialised), Cin > 16 (two chunks in flight), a BN activation of <= 1024 channels,
// y / y + BN-backward sums / fp32 epilogues, enough 16 x 32 tiles to fill the chip
static bool conv5_shape_ok(const unet_conv_desc* d) {
  if ((d->dtype != UNET_BF16 && d->dtype != UNET_F16) || d->ksize != 3) return false;
  if (d->out_mode != UNET_OUT_Y && d->out_mode != UNET_OUT_F32) return false;
  if (d->Cout % 8 || (d->out_mode == UNET_OUT_F32 && d->split % 4)) return false;   // 16-byte y stores
  if (d->Cin <= 16) return false;
  if (d->nsrc > 1 && (d->src[0].C % 16 || d->src[1].kind != UNET_SRC_PLAIN || d->src[1].gate_p)) return false;
  const unet_src& s0 = d->src[0];
  if (s0.kind != UNET_SRC_PLAIN && s0.kind != UNET_SRC_ACT) return false;
  if (s0.kind == UNET_SRC_PLAIN && s0.gate_p) return false;
  if (s0.kind == UNET_SRC_ACT && s0.C > C5_CMAX) return false;
  for (int i = 0; i < d->nsrc; ++i) {
    const unet_src& s = d->src[i];
    if (s.C % 8) return false;
    if ((double)d->N * s.H * s.W * s.C * 2 >= (double)OOB) return false;
    if (s.H != d->H || s.W != d->W) return false;
  }
  if ((double)d->N * d->H * d->W * 4 >= (double)OOB) return false;
  if ((double)d->N * d->H * d->W * d->Cout * 2 >= (double)OOB) return false;   // y stores: OOB masks lanes
  return true;
}

bool conv5_eligible(const unet_conv_desc* d) {
  const int mode = conv5_mode();
  if (mode == 0) return false;
  // default: every 16-bit y output (forward and the middle-activation dgrads) and the fp32 dgrads of <= 64
  // channels — per layer conv5 measured 0-31 % faster there (the 512^2 64-channel layers 14-31 %); the
  // wider fp32 dgrads stay on conv3, whose tiles measured 5-20 % faster (profiles/r03_layerprof_*.txt)
  // (the small maps' MI = 2 form serves the wide fp32 dgrads too: conv3 there is a 64- or 128-workgroup launch)
  if (!conv5_shape_ok(d)) return false;
  const int mi = conv5_mi(d);
  if (mode == 2 && d->out_mode == UNET_OUT_F32 && d->Cout > C5_BN && mi == C5_MI) return false;
  const long long work = conv5_mtiles(d, mi) * cdiv(d->Cout, C5_BN);
  return work >= 256;
}

// ---- split-K over the input channels for maps whose 16 x 32 x 64 tiles do not fill the chip (round 5,
// the 32^2 512 -> 512 down4 layers ran on conv3 at 12-15 % of peak with 64 tiles of work):
// S = the smallest power of two with tiles x S >= 256 (<= 8), each split >= 2 chunks; the partial sums go to
// S fp32 slabs in d->workspace and conv5_splitk_finish_kernel adds them in slab order (deterministic) and applies
// the real epilogue (y + BN partial sums, y + BN-backward sums, or fp32 with split / accumulation).
// UNET_CONV5_SPLIT=0 turns it off (A/B).
// the split count of d's shape (unet_conv_workspace sizes the slabs from it, whatever d->workspace holds)
static int conv5_splitk_shape(const unet_conv_desc* d) {
  const char* e = getenv("UNET_CONV5_SPLIT");   // read per call (tests flip it)
  const int on = e ? atoi(e) : 1;
  if (!on || conv5_mode() == 0 || d->act_out || !conv5_shape_ok(d) || conv5w_ok(d)) return 1;
  if (d->Cout > 1024 || (d->Cout & (d->Cout - 1))) return 1;     // the finisher's channel-vector layout
  // a slab is addressed by one buffer resource (32-bit range): the kernel's counted fp32 stores need it
  if ((double)d->N * d->H * d->W * d->Cout * 4 >= (double)OOB) return 1;
  const long long work = conv5_mtiles(d, conv5_mi(d)) * cdiv(d->Cout, C5_BN);
  if (work >= 256) return 1;
  const int nch = cdiv(d->Cin, 16);
  int S = 1;
  while (work * S < 256 && S < 8 && nch % (2 * S) == 0 && nch / (2 * S) >= 2) S *= 2;
  return S;
}

// the split count unet_conv runs d with: the shape's, if the caller passed a workspace (a
// descriptor without one — e.g. zero-initialised by a C caller — runs the unsplit form, as before round 5)
int conv5_splitk(const unet_conv_desc* d) { return d->workspace ? conv5_splitk_shape(d) : 1; }

bool conv5_serves(const unet_conv_desc* d) {
  return (conv5_mode() != 0 && conv5w_ok(d)) || conv5_eligible(d) || conv5_splitk(d) > 1;
}

size_t conv5_workspace(const unet_conv_desc* d) {
  const int S = conv5_eligible(d) ? 1 : conv5_splitk_shape(d);
  return S > 1 ? (size_t)S * d->N * d->H * d->W * d->Cout * sizeof(float) : 0;
}

// the finisher: 256 threads = CV channel vectors (4 channels) x R pixel lanes, FIN_TRIPS pixels per lane
static int fin_rows(const unet_conv_desc* d) {
  const int R = 256 / (d->Cout / 4);
  const long long npix = (long long)d->N * d->H * d->W;
  long long rows = (npix + (long long)R * FIN_TRIPS - 1) / ((long long)R * FIN_TRIPS);
  return (int)(rows < 1 ? 1 : rows);
}

int conv5_stats_rows(const unet_conv_desc* d) {
  if (conv5_mode() != 0 && conv5w_ok(d)) return conv5w_stats_rows(d);
  if (!conv5_eligible(d) && conv5_splitk(d) > 1) return fin_rows(d);
  return conv5_gx(d, conv5_mi(d)) * C5_WM;
}

// can the forward write src[0]'s transformed input to act_out (the y-mode BN-activation kernel serves d)?
bool conv5_act_out_ok(const unet_conv_desc* d) {
  if (conv5_mode() != 0 && conv5w_ok(d))
    return d->out_mode == UNET_OUT_Y && !d->bnb_stats && d->src[0].kind == UNET_SRC_ACT;
  return conv5_eligible(d) && d->out_mode == UNET_OUT_Y && !d->bnb_stats && d->src[0].kind == UNET_SRC_ACT &&
         d->src[0].C % 16 == 0;
}

int conv5_variant(const unet_conv_desc* d, char* buf, int len) {
  if (conv5_mode() != 0 && conv5w_ok(d)) return conv5w_variant(d, buf, len);
  const int S = conv5_eligible(d) ? 1 : conv5_splitk(d);
  const int mi = conv5_mi(d);
  if (S > 1) snprintf(buf, len, "conv5_kernel<%s,%d>+splitk%d", d->dtype == UNET_F16 ? "fp16" : "bf16", mi, S);
  else snprintf(buf, len, "conv5_kernel<%s,%d>", d->dtype == UNET_F16 ? "fp16" : "bf16", mi);
  return 0;
}

// PIPE: the column-ahead operand reads (per layer 5-9 % faster: 117 -> 108 us on the 512^2 64->64 forward,
// profiles/r04_layerprof_conv5_pipe{0,1}.txt).  The BN-backward-sums epilogue of a stored source (the dgrads'
// dy) has it too since round 5's register cuts (245-251 VGPRs, no spills); with a BN-activation source
// (SK_ACT_PLAIN) both operand columns plus its 32 y1 registers still run out of VGPRs (256 + 28-36 bytes of
// scratch), so that form keeps the compiler's schedule (round 4: 14-30 % slower with the spills)
// The 8-wave form (NWV 8).  The one-wave-per-SIMD form (NWV 4: 64 channels per wave, 12 LDS reads per 24 MFMAs
// per tap column, 462-502 registers, no spills) measured 10-25 % slower on every layer
// (profiles/r04_layerprof_conv5_{8,4}waves.txt): one wave cannot cover its own LDS and DMA latencies.
template <typename T, int OM, int SK, int GATE, int ABL, int PIPE_, int MI>
static int launch5_mi(const unet_conv_desc* d, hipStream_t st) {
  constexpr int TH = C5_WM * MI;
  constexpr int PIPE = PIPE_ >= 0 ? PIPE_ : (OM == OM5_BNB && SK != SK_PLAIN && SK != SK5_PLAIN1) ? 0 : 1;
  const int tw = cdiv(d->W, C5_W), th = cdiv(d->H, TH);
  const int mt = d->N * tw * th;
  const int gy = cdiv(d->Cout, C5_BN);
  const int gx = conv5_gx(d, MI);
  const int nch = cdiv(d->Cin, 16);
  hipLaunchKernelGGL((conv5_kernel<T, MI, OM, SK, GATE, ABL, PIPE, 8>), dim3(gx, gy), dim3(512), 0, st, *d, tw, th,
                     mt, nch, nch, conv5_prio());
  return check_launch("conv5");
}
template <typename T, int OM, int SK, int GATE, int ABL = 0, int PIPE_ = -1>
static int launch5(const unet_conv_desc* d, hipStream_t st) {
  if constexpr (ABL == 0) {
    if (conv5_mi(d) == C5_MI_S) return launch5_mi<T, OM, SK, GATE, 0, PIPE_, C5_MI_S>(d, st);
  }
  return launch5_mi<T, OM, SK, GATE, ABL, PIPE_, C5_MI>(d, st);
}

template <typename T, int MODE>
static void launch5_finish_m(const unet_conv_desc* d, int S, hipStream_t st) {
  const int rows = fin_rows(d);
  const float* ws = (const float*)d->workspace;
  if (S == 2) hipLaunchKernelGGL((conv5_splitk_finish_kernel<T, MODE, 2>), dim3(rows), dim3(256), 0, st, *d, ws, rows);
  else if (S == 4) hipLaunchKernelGGL((conv5_splitk_finish_kernel<T, MODE, 4>), dim3(rows), dim3(256), 0, st, *d, ws, rows);
  else hipLaunchKernelGGL((conv5_splitk_finish_kernel<T, MODE, 8>), dim3(rows), dim3(256), 0, st, *d, ws, rows);
}
// the finisher of a split-K conv (S in {2, 4, 8}: conv5_splitk)
template <typename T>
static int launch5_finish(const unet_conv_desc* d, int S, hipStream_t st) {
  if (d->out_mode == UNET_OUT_F32) launch5_finish_m<T, 2>(d, S, st);
  else if (d->bnb_stats) launch5_finish_m<T, 1>(d, S, st);
  else launch5_finish_m<T, 0>(d, S, st);
  return check_launch("conv5 split finish");
}

// split-K: the conv into S fp32 slabs (one workgroup per tile and split), then the finisher
template <typename T, int SK, int GATE, int MI>
static int launch5_split_mi(const unet_conv_desc* d, int S, hipStream_t st) {
  constexpr int TH = C5_WM * MI;
  if (!d->workspace || S < 2 || (double)d->N * d->H * d->W * d->Cout * 4 >= (double)OOB) {   // (conv5_splitk)
    set_error("unet_conv: split-K without a workspace or past a slab's 32-bit range");
    return UNET_ERR_ARG;
  }
  const int tw = cdiv(d->W, C5_W), th = cdiv(d->H, TH);
  const int mt = d->N * tw * th;
  const int gy = cdiv(d->Cout, C5_BN);
  const int nch = cdiv(d->Cin, 16);
  unet_conv_desc k = *d;
  k.out_mode = UNET_OUT_F32;
  k.out = d->workspace;
  k.out2 = nullptr;
  k.split = d->Cout;
  k.accum = k.accum2 = 0;
  k.stats = nullptr;
  k.bnb_stats = nullptr;
  k.act_out = nullptr;
  hipLaunchKernelGGL((conv5_kernel<T, MI, OM5_F32, SK, GATE, 0, 1, 8, true>), dim3(mt, gy, S), dim3(512), 0, st, k,
                     tw, th, mt, nch / S, nch, conv5_prio());
  if (int e = check_launch("conv5 split")) return e;
  return launch5_finish<T>(d, S, st);
}
template <typename T, int SK, int GATE>
static int launch5_split(const unet_conv_desc* d, int S, hipStream_t st) {
  return conv5_mi(d) == C5_MI_S ? launch5_split_mi<T, SK, GATE, C5_MI_S>(d, S, st) : launch5_split_mi<T, SK, GATE, C5_MI>(d, S, st);
}

// source kind of a descriptor: plain, one BN activation (gated or not), or a BN activation + a stored map.
// The gradient epilogues (whose network sources are the stored dy) get the generic activation form only.
template <typename T, int OM>
static int dispatch5_om(const unet_conv_desc* d, hipStream_t st) {
  const unet_src& s0 = d->src[0];
  const bool one = d->nsrc == 1 && s0.C % 16 == 0;
  if constexpr (OM == OM5_BNB) {   // UNET_C5_BNB_PIPE=0: the round-4 schedule of the dy dgrads (A/B)
    const char* e = getenv("UNET_C5_BNB_PIPE");
    if (one && s0.kind != UNET_SRC_ACT && e && !atoi(e)) return launch5<T, OM, SK5_PLAIN1, 0, 0, 0>(d, st);
  }
  if (s0.kind != UNET_SRC_ACT) return one ? launch5<T, OM, SK5_PLAIN1, 0>(d, st) : launch5<T, OM, SK_PLAIN, 0>(d, st);
  const bool g = s0.gate_p != nullptr;
  if constexpr (OM == OM5_Y) {
    if (one) return g ? launch5<T, OM, SK_ACT, 1>(d, st) : launch5<T, OM, SK_ACT, 0>(d, st);
  }
  return g ? launch5<T, OM, SK_ACT_PLAIN, 1>(d, st) : launch5<T, OM, SK_ACT_PLAIN, 0>(d, st);
}

template <typename T>
static int dispatch5(const unet_conv_desc* d, hipStream_t st) {
  if (!conv5_eligible(d)) {
    const int S = conv5_splitk(d);
    const unet_src& s0 = d->src[0];
    const bool one = d->nsrc == 1 && s0.C % 16 == 0;
    if (s0.kind != UNET_SRC_ACT)
      return one ? launch5_split<T, SK5_PLAIN1, 0>(d, S, st) : launch5_split<T, SK_PLAIN, 0>(d, S, st);
    if (one) return s0.gate_p ? launch5_split<T, SK_ACT, 1>(d, S, st) : launch5_split<T, SK_ACT, 0>(d, S, st);
    return s0.gate_p ? launch5_split<T, SK_ACT_PLAIN, 1>(d, S, st) : launch5_split<T, SK_ACT_PLAIN, 0>(d, S, st);
  }
  if (d->out_mode == UNET_OUT_F32) return dispatch5_om<T, OM5_F32>(d, st);
  if (d->bnb_stats) return dispatch5_om<T, OM5_BNB>(d, st);
  return dispatch5_om<T, OM5_Y>(d, st);
}

int conv5_run(const unet_conv_desc* d, hipStream_t st) {
  if (conv5_mode() != 0 && conv5w_ok(d)) return conv5w_run(d, conv5_prio(), st);
  return d->dtype == UNET_F16 ? dispatch5<f16>(d, st) : dispatch5<bf16>(d, st);
}

template <int SK, int GATE>
static int abl5(const unet_conv_desc* d, int abl, hipStream_t st) {
  switch (abl) {
    case 0: return launch5<bf16, OM5_Y, SK, GATE, 0>(d, st);
    case 1: return launch5<bf16, OM5_Y, SK, GATE, 1>(d, st);
    case 2: return launch5<bf16, OM5_Y, SK, GATE, 2>(d, st);
    case 3: return launch5<bf16, OM5_Y, SK, GATE, 3>(d, st);
    case 4: return launch5<bf16, OM5_Y, SK, GATE, 4>(d, st);
    case 8: return launch5<bf16, OM5_Y, SK, GATE, 8>(d, st);
    case 7: return launch5<bf16, OM5_Y, SK, GATE, 7>(d, st);
    case 15: return launch5<bf16, OM5_Y, SK, GATE, 15>(d, st);
    case 16: return launch5<bf16, OM5_Y, SK, GATE, 16>(d, st);
    case 31: return launch5<bf16, OM5_Y, SK, GATE, 31>(d, st);
  }
  return UNET_ERR_ARG;
}

// split-K ablations: the split kernel alone (ABL bits as above) or, abl < 0, the y + BN-stats finisher alone
template <int SK, int MI>
static int abl5_split_mi(const unet_conv_desc* d, int abl, hipStream_t st) {
  constexpr int TH = C5_WM * MI;
  const int S = conv5_splitk(d);
  const int tw = cdiv(d->W, C5_W), th = cdiv(d->H, TH), mt = d->N * tw * th, gy = cdiv(d->Cout, C5_BN);
  const int nch = cdiv(d->Cin, 16);
  if (S < 2 || !d->workspace) return UNET_ERR_ARG;
  if (abl < 0) {
    launch5_finish_m<bf16, 0>(d, S, st);
    return check_launch("conv5 split finish (diag)");
  }
  unet_conv_desc k = *d;
  k.out_mode = UNET_OUT_F32;
  k.out = d->workspace;
  k.out2 = nullptr;
  k.split = d->Cout;
  k.accum = k.accum2 = 0;
  k.stats = nullptr;
  k.bnb_stats = nullptr;
  k.act_out = nullptr;
  const dim3 grid(mt, gy, S);
#define C5SA(A) hipLaunchKernelGGL((conv5_kernel<bf16, MI, OM5_F32, SK, 0, A, 1, 8, true>), grid, dim3(512), 0, st, k, tw, th, mt, nch / S, nch, 0)
  switch (abl) {
    case 0: C5SA(0); break;
    case 1: C5SA(1); break;
    case 2: C5SA(2); break;
    case 3: C5SA(3); break;
    case 4: C5SA(4); break;
    case 8: C5SA(8); break;
    case 16: C5SA(16); break;
    case 31: C5SA(31); break;
    default: return UNET_ERR_ARG;
  }
#undef C5SA
  return check_launch("conv5 split (diag)");
}
template <int SK>
static int abl5_split(const unet_conv_desc* d, int abl, hipStream_t st) {
  return conv5_mi(d) == C5_MI_S ? abl5_split_mi<SK, C5_MI_S>(d, abl, st) : abl5_split_mi<SK, C5_MI>(d, abl, st);
}

}  // namespace unet

// diagnostic (not part of the C ABI header): the split-K form's ablations (abl5_split) on a one-source plain or
// BN-activation bf16 y-mode descriptor whose map is small enough for split-K (d->workspace set); tools/conv5_ablate.py
extern "C" int unet_diag_conv5_split_ablate(const unet_conv_desc* d, int abl, void* stream) {
  using namespace unet;
  if (conv5_eligible(d) || d->nsrc != 1 || d->out_mode != UNET_OUT_Y || d->dtype != UNET_BF16 || d->src[0].C % 16)
    return UNET_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  return d->src[0].kind == UNET_SRC_PLAIN ? abl5_split<SK5_PLAIN1>(d, abl, st) : abl5_split<SK_ACT>(d, abl, st);
}

// diagnostic (not part of the C ABI header): conv5 ablations of the bf16 y-mode kernel (ABL bits above) on a
// one-source plain or BN-activation descriptor; tools/conv5_ablate.py
extern "C" int unet_diag_conv5_ablate(const unet_conv_desc* d, int abl, void* stream) {
  using namespace unet;
  if (!conv5_eligible(d) || d->nsrc != 1 || d->out_mode != UNET_OUT_Y || d->dtype != UNET_BF16) return UNET_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (d->src[0].C % 16) return UNET_ERR_ARG;
  return d->src[0].kind == UNET_SRC_PLAIN ? abl5<SK5_PLAIN1, 0>(d, abl, st) : abl5<SK_ACT, 0>(d, abl, st);
}
