// conv4.hip — 3x3 convolution (forward and dgrad) on v_mfma_f32_32x32x16_{bf16,f16} for gfx950.
//
// Replaces nn.Conv2d(k=3, pad=1, bias=False) of unet/models/layers.py:32,35 (every DoubleConv half) and the
// input-gradient half of its convolution_backward, on maps large enough to fill the chip with 32-pixel-wide
// tiles.  Why a second 3x3 kernel beside conv3 (16x16x32 MFMAs): a 16x16x32 MFMA holds the SIMD's vector
// issue for 8 of its 16 cycles, leaving room for ~2 VALU instructions per MFMA, while the halo transform
// (BN-apply + ReLU + gate of the previous layer), the epilogue (16-bit pack, BatchNorm partial sums) and the
// per-tile set-up of the 64-channel layers need 5.5-7.4 per MFMA (profiles/r02_end_conv3_wgrad2_pmc.txt).
// A 32x32x16 MFMA does the same FLOPs in 32 cycles and leaves 24 of them for vector work: three times the
// VALU headroom per FLOP.  The wave tile is also larger (MI rows x 32 px x 32*NJ channels), so the per-tile
// set-up and the halo are amortised over more MFMAs.
//
//  * Implicit GEMM, D[co][px] = W[co][k] * X[k][px]: the weights are the A operand (32 output channels x 16
//    k), the staged input the B operand (16 k x 32 pixels of one row, shifted by the tap).  A lane owns one
//    pixel and four runs of 4 consecutive channels, so every output mode stores 8 bytes (16-bit y) or 16
//    bytes (fp32 gradient) per run without an LDS transpose.
//  * Input: per 16-channel chunk the (TH+2) x 34 halo is staged once into LDS (48-byte pixel rows: the
//    ds_read_b128 B-fragment reads are bank-conflict free) through conv_src16.h's buffer-load gather, which
//    applies the virtual-activation transform; chunk c+1 is issued under taps 0-2 and stored under taps 6-8
//    of chunk c into the other buffer: one barrier per chunk.  Taps run dx-major so the MI+2 rows read for one
//    dx serve its three taps.
//  * Weights: conv3's fragment-major packing ([Npad/16][Cin/32][9][64 lanes][16 B], unet_pack_weights) read
//    in place: the 32x16 A fragment of channels co..co+31, k-half s of a 32-channel chunk is four 256-byte
//    runs of it (lane-constant offset), prefetched two taps ahead into a 3-slot VGPR ring; no repacking.
//  * Persistent over M tiles with the next tile's chunk 0 staged under the last chunk, as conv3.
//  * Epilogues: y (16-bit) + BatchNorm partial sums; y + the BatchNorm-backward sums of the activation it is
//    the gradient of (unet_conv_desc.bnb_*); fp32 gradient (concat split, accumulate).  The sums are kept per
//    lane across all the tiles a workgroup visits (2 VALU per value per tile) and reduced across lanes once,
//    at the end: one partial row per wave of the persistent grid, so the finalize kernels read ~1k rows
//    instead of one per tile.
#include "conv_mfma32.h"

namespace unet {

constexpr int C4W = 32;          // tile width in pixels (the MFMA's N)
constexpr int C4_NPAD = 128;     // packed weight rows are padded to this (conv.hip PACK_NPAD)
constexpr int OM4_Y = 0, OM4_F32 = 1, OM4_BNB = 2;

// wave tile: MI rows x 32 px x (32*NJ) channels; block: WM x WN waves -> (MI*WM) rows x 32 px x (32*NJ*WN) ch.
// ABL (diagnostic ablations, unet_diag_conv4_ablate; 0 in the product): 1 no next-chunk halo staging, 2 no
// weight loads inside the chunk loop, 4 no epilogue stores / sums, 8 no per-chunk barrier
template <typename T, int WM, int WN, int NJ, int MI, int OM, int SK, int ABL = 0>
__global__ __launch_bounds__(64 * WM * WN, (WM * WN <= 4) ? 2 : 1) void conv4_kernel(const unet_conv_desc d, int tiles_w,
                                                                                   int tiles_h, int mtiles, int nch16) {
  using F = typename Mma32<T>::frag;
  constexpr int NT = 64 * WM * WN;
  constexpr int NV = 2;                       // 16-byte vectors per pixel of a 16-channel chunk
  constexpr int TH = MI * WM;
  constexpr int HWID = C4W + 2, HP = HWID * (TH + 2);
  constexpr int RS = 24;                      // 48-byte LDS pixel rows (conflict-free ds_read_b128)
  constexpr int ITEMS = (HP * NV + NT - 1) / NT;
  constexpr int IPT = (ITEMS + 2) / 3;        // items issued per tap (taps 0-2) and finished per tap (6-8)
  constexpr int BNW = 32 * NJ;                // output channels per wave
  static_assert(ITEMS <= 9, "halo items per thread");
  __shared__ __attribute__((aligned(16))) T lds[2 * HP * RS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int cw0 = blockIdx.y * (WN * BNW) + wn * BNW;   // first output channel of this wave
  const int v = tid % NV;
  auto tile_of = [&](int t, int& n_, int& h0_, int& w0_) {
    const int tw_i = t % tiles_w;
    const int t2 = t / tiles_w;
    h0_ = (t2 % tiles_h) * TH;
    w0_ = tw_i * C4W;
    n_ = t2 / tiles_h;
  };
  int mt = blockIdx.x;
  if (mt >= mtiles) return;
  int n, h0, w0;
  tile_of(mt, n, h0, w0);

  // A fragment (weights) of output channels cw0 + 32 nb + (l & 31), k = 16 c16 + 8 (l >> 5) + j, tap t, from
  // the 16x16x32 fragment-major packing: 16-row tile 2 (cw0/32 + nb) + ((l >> 4) & 1), 32-channel chunk
  // c16 / 2, packed lane 16 (2 (c16 & 1) + (l >> 5)) + (l & 15)
  const int nch32 = (nch16 + 1) >> 1;
  const unsigned jstride = (unsigned)nch32 * 9u * 1024u;
  const unsigned ntiles = (unsigned)((d.Cout + C4_NPAD - 1) / C4_NPAD * (C4_NPAD / 16));
  const rsrc_t wr = mk_rsrc(d.weight, ntiles * jstride);
  const unsigned lanew = (unsigned)((lane >> 4) & 1) * jstride + (unsigned)(16 * (lane >> 5) + (lane & 15)) * 16u;
  const unsigned wbase = (unsigned)(cw0 / 16) * jstride;
  auto afrag = [&](int nb, int c16, int t) -> uint4 {
    return bld(wr, lanew,
               wbase + (unsigned)nb * 2u * jstride + (unsigned)((c16 >> 1) * 9 + t) * 1024u + (unsigned)(c16 & 1) * 512u);
  };
  auto tap_of = [](int s) { return (s % 3) * 3 + s / 3; };   // step s: dx = s / 3, dy = s % 3

  f32x16 acc[MI][NJ];
  Geo<1> geo[ITEMS];
  uint4 q[ITEMS][1];
  ChunkV cv;
  const int c0 = d.src[0].C;
  int cur_si = 0;
  conv3_geo<1, HWID, 1, HP, NT, NV, ITEMS, SK>(d, d.src[0], n, h0, w0, tid, geo);

  // ---- prologue: chunk 0 of the first tile -> LDS buffer 0, weights of steps 0 and 1 ----
  conv3_view<1, 0, SK>(d, 0, 0, v, cv);
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) conv3_issue<1, SK>(cv, geo[k], q[k]);
#pragma unroll
  for (int k = 0; k < ITEMS; ++k) {
    const int hp = (tid + k * NT) / NV;
    if (hp < HP) *reinterpret_cast<uint4*>(lds + hp * RS + v * 8) = conv3_finish<T, 1, 0, SK>(cv, geo[k], q[k]);
  }
  uint4 B[3][NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) { B[0][j] = afrag(j, 0, tap_of(0)); B[1][j] = afrag(j, 0, tap_of(1)); }
  __syncthreads();

  // BatchNorm sums (y: Σy, Σy²; BNB: Σg, Σg·y1) of this lane's pixel column and 16*NJ channels, accumulated
  // over every tile the workgroup visits and reduced across lanes / written once at the end (one partial
  // row per wave: [2][Cout][gridDim.x * WM] for y, [2][gridDim.x * WM][Cout] for BNB)
  constexpr bool SUMS = OM == OM4_Y || OM == OM4_BNB;
  float sA[SUMS ? NJ : 1][16], sB[SUMS ? NJ : 1][16];
#pragma unroll
  for (int j = 0; j < (SUMS ? NJ : 1); ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) { sA[j][r] = 0.f; sB[j][r] = 0.f; }

  int buf = 0;
  for (;;) {
    const int mt_next = mt + (int)gridDim.x;
    const bool tile_next = mt_next < mtiles;
    int nn = n, nh0 = h0, nw0 = w0;
    if (tile_next) tile_of(mt_next, nn, nh0, nw0);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

#pragma unroll 1
    for (int c = 0; c < nch16; ++c) {
      const T* xb = lds + buf * HP * RS;
      T* xn = lds + (buf ^ 1) * HP * RS;
      const bool more = c + 1 < nch16;
      const bool has_next = more || tile_next;
      const int cw = more ? c + 1 : 0;
      if (more) {
        const int cn0 = (c + 1) * 16;
        const int si = (d.nsrc > 1 && cn0 >= c0) ? 1 : 0;
        if (si != cur_si) {
          conv3_geo<1, HWID, 1, HP, NT, NV, ITEMS, SK>(d, d.src[si], n, h0, w0, tid, geo);
          cur_si = si;
        }
        conv3_view<1, 0, SK>(d, si, cn0 - (si ? c0 : 0), v, cv);
      } else if (tile_next) {
        conv3_geo<1, HWID, 1, HP, NT, NV, ITEMS, SK>(d, d.src[0], nn, nh0, nw0, tid, geo);
        cur_si = 0;
        conv3_view<1, 0, SK>(d, 0, 0, v, cv);
      }
      F xr[MI + 2];
#pragma unroll
      for (int st = 0; st < 9; ++st) {
        const int dx = st / 3, dy = st % 3;
        if constexpr (!(ABL & 2)) {
          const int s2 = st + 2;
          if (s2 < 9) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) B[s2 % 3][j] = afrag(j, c, tap_of(s2));
          } else if (more) {   // the next tile's first weights are loaded after the epilogue
#pragma unroll
            for (int j = 0; j < NJ; ++j) B[s2 % 3][j] = afrag(j, cw, tap_of(s2 - 9));
          }
        }
        if (st < 3 && has_next && !(ABL & 1)) {
#pragma unroll
          for (int u = 0; u < IPT; ++u)
            if (st * IPT + u < ITEMS) conv3_issue<1, SK>(cv, geo[st * IPT + u], q[st * IPT + u]);
        }
        if (dy == 0) {
#pragma unroll
          for (int r = 0; r < MI + 2; ++r)
            xr[r] = *reinterpret_cast<const F*>(xb + ((wm * MI + r) * HWID + (lane & 31) + dx) * RS + (lane >> 5) * 8);
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const F a = __builtin_bit_cast(F, B[st % 3][j]);
#pragma unroll
          for (int i = 0; i < MI; ++i) acc[i][j] = Mma32<T>::mma(a, xr[i + dy], acc[i][j]);
        }
        if (st >= 6 && has_next && !(ABL & 1)) {
#pragma unroll
          for (int u = 0; u < IPT; ++u) {
            const int k = (st - 6) * IPT + u;
            if (k < ITEMS) {
              const int hp = (tid + k * NT) / NV;
              const uint4 val = conv3_finish<T, 1, 0, SK>(cv, geo[k], q[k]);
              if (hp < HP) *reinterpret_cast<uint4*>(xn + hp * RS + v * 8) = val;
            }
          }
        }
        if (dy == 2) __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (!(ABL & 8)) __syncthreads();
      buf ^= 1;
    }

    // ---------------- epilogue ----------------
    if constexpr (ABL & 4) {
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) sum += acc[i][j][0] + acc[i][j][5] + acc[i][j][10] + acc[i][j][15];
      if (sum == 12345.f) ((float*)d.out)[tid] = sum;
    } else {
      const int px = lane & 31, hh = lane >> 5;
      const int ow = w0 + px;
      const bool colok = ow < d.W;
      const int oh0 = h0 + wm * MI;
      int rows = d.H - oh0;
      rows = rows < 0 ? 0 : (rows > MI ? MI : rows);
      const unsigned pix0 = ((unsigned)n * d.H + oh0) * (unsigned)d.W + ow;   // < 2^30 (conv4_eligible)
      if constexpr (OM == OM4_Y) {
        T* y = (T*)d.out;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const bool ok = colok && i < rows;
          const unsigned pix = pix0 + (unsigned)i * d.W;
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int co = cw0 + 32 * j + 8 * g + 4 * hh;
              if (ok && co < d.Cout) {
                uint2 pk;
                pk.x = pack2_16<T>(acc[i][j][4 * g], acc[i][j][4 * g + 1]);
                pk.y = pack2_16<T>(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
                *reinterpret_cast<uint2*>(y + (size_t)pix * d.Cout + co) = pk;
              }
            }
        }
        if (d.stats) {
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
#pragma unroll
              for (int i = 0; i < MI; ++i) {
                const float x = (colok && i < rows) ? acc[i][j][r] : 0.f;
                sA[j][r] += x;
                sB[j][r] = __builtin_fmaf(x, x, sB[j][r]);
              }
        }
      } else if constexpr (OM == OM4_BNB) {
        // y (the gradient of a single-consumer activation, 16-bit) + that activation's BatchNorm backward
        // sums: g = the value as stored where relu?(y1 * scale + shift) > 0; Σg and Σg·y1 per lane here,
        // Σg·(y1 - mean)·invstd = invstd·(Σg·y1 - mean·Σg) formed once per channel at the end
        T* y = (T*)d.out;
        const T* y1 = (const T*)d.bnb_y;
        uint2 yv[MI][NJ][4];
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int co = cw0 + 32 * j + 8 * g + 4 * hh;
              yv[i][j][g] = make_uint2(0u, 0u);
              if (colok && i < rows && co < d.Cout)
                yv[i][j][g] = *reinterpret_cast<const uint2*>(y1 + (size_t)(pix0 + (unsigned)i * d.W) * d.Cout + co);
            }
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int co = cw0 + 32 * j + 8 * g + 4 * hh;
            const bool cok = co < d.Cout;
            float sc4[4] = {0.f, 0.f, 0.f, 0.f}, sf4[4] = {0.f, 0.f, 0.f, 0.f};
            if (cok && d.bnb_relu) {
              const float4 a4 = *reinterpret_cast<const float4*>(d.bnb_scale + co);
              const float4 b4 = *reinterpret_cast<const float4*>(d.bnb_shift + co);
              sc4[0] = a4.x; sc4[1] = a4.y; sc4[2] = a4.z; sc4[3] = a4.w;
              sf4[0] = b4.x; sf4[1] = b4.y; sf4[2] = b4.z; sf4[3] = b4.w;
            }
#pragma unroll
            for (int i = 0; i < MI; ++i) {
              const unsigned pix = pix0 + (unsigned)i * d.W;
              const bool ok = colok && i < rows && cok;
              uint2 pk;
              pk.x = pack2_16<T>(acc[i][j][4 * g], acc[i][j][4 * g + 1]);
              pk.y = pack2_16<T>(acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
              if (ok) {
                *reinterpret_cast<uint2*>(y + (size_t)pix * d.Cout + co) = pk;
                float gv[4], yy[4];
                unpack4_16<T>(pk, gv);
                unpack4_16<T>(yv[i][j][g], yy);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const float gg = (d.bnb_relu && !(yy[r] * sc4[r] + sf4[r] > 0.f)) ? 0.f : gv[r];
                  sA[j][4 * g + r] += gg;
                  sB[j][4 * g + r] = __builtin_fmaf(gg, yy[r], sB[j][4 * g + r]);
                }
              }
            }
          }
      } else {  // OM4_F32: fp32 gradient, channels [0, split) -> out, [split, Cout) -> out2, optionally accumulated
        float* o1 = (float*)d.out;
        float* o2 = (float*)d.out2;
        const int c2 = d.Cout - d.split;
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          if (!(colok && i < rows)) continue;
          const unsigned pix = pix0 + (unsigned)i * d.W;
          float4* p[NJ][4];
          float4 old[NJ][4];
          bool acc_in[NJ][4];
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int co = cw0 + 32 * j + 8 * g + 4 * hh;
              if (co < d.split) {
                p[j][g] = reinterpret_cast<float4*>(o1 + (size_t)pix * d.split + co);
                acc_in[j][g] = d.accum;
              } else {
                p[j][g] = reinterpret_cast<float4*>(o2 + (size_t)pix * c2 + (co - d.split));
                acc_in[j][g] = d.accum2;
              }
              old[j][g] = make_float4(0.f, 0.f, 0.f, 0.f);
              if (co < d.Cout && acc_in[j][g]) old[j][g] = *p[j][g];
            }
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int co = cw0 + 32 * j + 8 * g + 4 * hh;
              if (co < d.Cout) {
                float4 w = make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
                if (acc_in[j][g]) { w.x += old[j][g].x; w.y += old[j][g].y; w.z += old[j][g].z; w.w += old[j][g].w; }
                *p[j][g] = w;
              }
            }
        }
      }
    }

    if (!tile_next) break;
    mt = mt_next;
    n = nn;
    h0 = nh0;
    w0 = nw0;
    cur_si = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) { B[0][j] = afrag(j, 0, tap_of(0)); B[1][j] = afrag(j, 0, tap_of(1)); }
  }

  // ---- the workgroup's BatchNorm sums: over the 32 pixel columns of each half-wave, one row per wave ----
  if constexpr (SUMS) {
    const int hh = lane >> 5;
    const int srow = blockIdx.x * WM + wm, srows = gridDim.x * WM;
    if constexpr (OM == OM4_Y) {
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
        for (int g = 0; g < 4; ++g) {
          const int co = cw0 + 32 * j + 8 * g + 4 * hh;
          float a[4], b[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            a[r] = half32_sum(sA[j][4 * g + r]);
            b[r] = half32_sum(sB[j][4 * g + r]);
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
// host side
// ------------------------------------------------------------------------------------------------
struct Cfg4 {
  int wm, wn, nj, mi;
};

// UNET_CONV4=1 routes the eligible convs to conv4 (off by default until it beats conv3 on every layer it
// takes; read per call so tests can flip it)
static bool conv4_enabled() {
  const char* e = getenv("UNET_CONV4");
  return e && atoi(e) != 0;
}

static Cfg4 conv4_cfg(const unet_conv_desc* d) {
  if (d->Cout <= 64) return {4, 2, 1, 4};   // 16 rows x 32 px x 64 ch, 8 waves of 4 rows x 32 ch
  return {2, 4, 1, 4};                      // 8 rows x 32 px x 128 ch, 8 waves of 4 rows x 32 ch
}

static long long conv4_mtiles(const unet_conv_desc* d, const Cfg4& c) {
  return (long long)d->N * cdiv(d->W, C4W) * cdiv(d->H, c.wm * c.mi);
}

// 16-bit 3x3, plain / BN-activation sources (the network's pooled and upsampled maps are materialised),
// y / y+BN-backward-sums / fp32 epilogues, and enough 32-pixel tiles to fill the chip
bool conv4_eligible(const unet_conv_desc* d) {
  if (!conv4_enabled()) return false;
  if ((d->dtype != UNET_BF16 && d->dtype != UNET_F16) || d->ksize != 3) return false;
  if (d->out_mode != UNET_OUT_Y && d->out_mode != UNET_OUT_F32) return false;
  if (d->Cout % 4 || (d->out_mode == UNET_OUT_F32 && d->split % 4)) return false;
  if (d->nsrc > 1 && d->src[0].C % 16) return false;
  for (int i = 0; i < d->nsrc; ++i) {
    const unet_src& s = d->src[i];
    if (s.kind != UNET_SRC_PLAIN && s.kind != UNET_SRC_ACT) return false;
    if (s.C % 8) return false;
    if ((double)d->N * s.H * s.W * s.C * 2 >= (double)OOB) return false;
    if (s.gate_p && s.kind != UNET_SRC_ACT) return false;
  }
  if ((double)d->N * d->H * d->W >= (double)(1u << 30)) return false;
  const Cfg4 c = conv4_cfg(d);
  const long long work = conv4_mtiles(d, c) * cdiv(d->Cout, 32 * c.nj * c.wn);
  return work >= 512;
}

// persistent grid: about two (4-wave) workgroups per CU or one 8-wave workgroup, never more than the tiles
static int conv4_gx(const unet_conv_desc* d, const Cfg4& c) {
  const long long mt = conv4_mtiles(d, c);
  const int gy = cdiv(d->Cout, 32 * c.nj * c.wn);
  long long gx = cdiv(c.wm * c.wn <= 4 ? 512 : 256, gy);
  if (gx > mt) gx = mt;
  if (gx < 1) gx = 1;
  return (int)gx;
}

// partial-sum rows: one per wave row of the persistent grid (conv4_kernel's SUMS)
int conv4_stats_rows(const unet_conv_desc* d) {
  const Cfg4 c = conv4_cfg(d);
  return conv4_gx(d, c) * c.wm;
}

int conv4_variant(const unet_conv_desc* d, char* buf, int len) {
  const Cfg4 c = conv4_cfg(d);
  snprintf(buf, len, "conv4_kernel<%s,%d,%d,%d,%d>", d->dtype == UNET_F16 ? "fp16" : "bf16", c.wm, c.wn, c.nj, c.mi);
  return 0;
}

template <typename T, int WM, int WN, int NJ, int MI, int OM, int SK, int ABL = 0>
static int launch4(const unet_conv_desc* d, hipStream_t st) {
  constexpr int TH = MI * WM, BN = WN * NJ * 32;
  const int tw = cdiv(d->W, C4W), th = cdiv(d->H, TH);
  const int mt = d->N * tw * th;
  const int gy = cdiv(d->Cout, BN);
  const int gx = conv4_gx(d, Cfg4{WM, WN, NJ, MI});
  hipLaunchKernelGGL((conv4_kernel<T, WM, WN, NJ, MI, OM, SK, ABL>), dim3(gx, gy), dim3(64 * WM * WN), 0, st, *d, tw, th, mt,
                     cdiv(d->Cin, 16));
  return check_launch("conv4");
}

template <typename T, int WM, int WN, int NJ, int MI>
static int dispatch4_cfg(const unet_conv_desc* d, hipStream_t st) {
  if (d->out_mode == UNET_OUT_F32) {
    if (d->nsrc == 1 && d->src[0].kind == UNET_SRC_PLAIN) return launch4<T, WM, WN, NJ, MI, OM4_F32, SK_PLAIN>(d, st);
    return launch4<T, WM, WN, NJ, MI, OM4_F32, SK_ANY>(d, st);
  }
  if (d->bnb_stats) {
    if (d->nsrc == 1 && d->src[0].kind == UNET_SRC_PLAIN) return launch4<T, WM, WN, NJ, MI, OM4_BNB, SK_PLAIN>(d, st);
    return launch4<T, WM, WN, NJ, MI, OM4_BNB, SK_ANY>(d, st);
  }
  const unet_src &s0 = d->src[0], &s1 = d->src[1];
  const bool p0 = s0.kind == UNET_SRC_PLAIN && !s0.gate_p, a0 = s0.kind == UNET_SRC_ACT;
  const bool p1 = d->nsrc > 1 && s1.kind == UNET_SRC_PLAIN && !s1.gate_p;
  if ((d->nsrc == 1 && p0) || (p0 && p1)) return launch4<T, WM, WN, NJ, MI, OM4_Y, SK_PLAIN>(d, st);
  if (d->nsrc == 1 && a0) return launch4<T, WM, WN, NJ, MI, OM4_Y, SK_ACT>(d, st);
  if (a0 && p1) return launch4<T, WM, WN, NJ, MI, OM4_Y, SK_ACT_PLAIN>(d, st);
  return launch4<T, WM, WN, NJ, MI, OM4_Y, SK_ANY>(d, st);
}

template <typename T>
static int dispatch4(const unet_conv_desc* d, hipStream_t st) {
  const Cfg4 c = conv4_cfg(d);
  if (c.wm == 4) return dispatch4_cfg<T, 4, 2, 1, 4>(d, st);
  return dispatch4_cfg<T, 2, 4, 1, 4>(d, st);
}

int conv4_run(const unet_conv_desc* d, hipStream_t st) {
  return d->dtype == UNET_F16 ? dispatch4<f16>(d, st) : dispatch4<bf16>(d, st);
}

template <int SK, int ABL>
static int abl4(const unet_conv_desc* d, hipStream_t st) {
  if (d->Cout <= 64) return launch4<bf16, 4, 2, 1, 4, OM4_Y, SK, ABL>(d, st);
  return launch4<bf16, 2, 4, 1, 4, OM4_Y, SK, ABL>(d, st);
}
template <int SK>
static int abl4_modes(const unet_conv_desc* d, int abl, hipStream_t st) {
  switch (abl) {
    case 0: return abl4<SK, 0>(d, st);
    case 1: return abl4<SK, 1>(d, st);
    case 2: return abl4<SK, 2>(d, st);
    case 3: return abl4<SK, 3>(d, st);
    case 4: return abl4<SK, 4>(d, st);
    case 8: return abl4<SK, 8>(d, st);
    case 7: return abl4<SK, 7>(d, st);
    case 15: return abl4<SK, 15>(d, st);
  }
  return UNET_ERR_ARG;
}

}  // namespace unet

// diagnostic (not part of the C ABI header): conv4 ablations of the bf16 y-mode kernel (ABL bits above) on
// a one-source plain or BN-activation descriptor; tools/conv_ablate.py
extern "C" int unet_diag_conv4_ablate(const unet_conv_desc* d, int abl, void* stream) {
  using namespace unet;
  if (!conv4_eligible(d) || d->nsrc != 1 || d->out_mode != UNET_OUT_Y || d->dtype != UNET_BF16) return UNET_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  return d->src[0].kind == UNET_SRC_PLAIN ? abl4_modes<SK_PLAIN>(d, abl, st) : abl4_modes<SK_ACT>(d, abl, st);
}
