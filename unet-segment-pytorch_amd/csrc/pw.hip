// pw.hip — pointwise (1x1) convolution fwd / dgrad / wgrad on MFMA for the attention-gate projections.
//
// Reference: AttentionGate W_g / W_x (nn.Conv2d(k=1, bias=False) + BN, unet/models/layers.py:151-160,
// applied at :186-187) and their convolution_backward.  These are HBM-bound GEMMs (AI 21-169 FLOP/B
// at bs 4, SURVEY §8(a) gate rows): the work is to stream the NHWC operands once at full width, so the
// 1x1 case drops the 3x3 machinery (halo, LDS, per-chunk barriers) entirely:
//  * fwd / dgrad: a 1x1 conv is a GEMM over the flattened pixel index, so a wave computes
//    D[co][px] = W[co][ci] . X[ci][px] with the weight fragment as the MFMA A operand (the packed
//    fragment-major layout, L2-resident) and the activation as the B operand, which is exactly one
//    16-byte NHWC load per lane (8 channels of one pixel) — no LDS.  The virtual-activation transform
//    (BN-apply + ReLU, x sigmoid(psi)) is applied in registers.  The accumulator lane then holds 4
//    consecutive channels of one pixel: 8-byte bf16 stores (y) or 16-byte fp32 stores / read-modify-
//    writes (dgrad), and the BN partial sums reduce over the 16 pixel lanes with shuffles;
//  * wgrad: dW[co][ci] = sum_px dy[px][co] X[px][ci]: 64-pixel tiles of dy and X are staged in LDS
//    (double-buffered, one barrier per tile) and read with the CDNA4 transposed read
//    ds_read_b64_tr_b16 so the pixel index runs along K; split-K partial slabs are summed in a fixed
//    order by wgrad_reduce2 (deterministic).
#include "conv_common.h"

namespace unet {

constexpr unsigned PW_OOB = 0x40000000u;  // >= every tensor byte size admitted below (< 1 GiB)
typedef __amdgpu_buffer_rsrc_t pw_rsrc_t;

__device__ __forceinline__ pw_rsrc_t pw_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 pw_ld(pw_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}
// 8 channels (one lane's 16-byte vector of the 16-bit operand type T) through the source transform
template <typename T>
__device__ __forceinline__ typename Mma<T>::frag pw_act(uint4 q, bool act, const float* sc, const float* sf, float lo,
                                                        float gmul) {
  typedef typename Mma<T>::frag F;
  if (!act && gmul == 1.f) return __builtin_bit_cast(F, q);
  float v[8];
  unpack8_16<T>(q, v);
  if (act) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fmaxf(__builtin_fmaf(v[j], sc[j], sf[j]), lo);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] *= gmul;
  return __builtin_bit_cast(F, pack8_16<T>(v));
}

// ------------------------------------------------------------------------------------------------
// fwd / dgrad.  Block = 4 waves; wave = 16*NB pixels x 16*NA output channels; grid (P / (64*NB), Cout / (16*NA))
// ------------------------------------------------------------------------------------------------
// OMK: the output mode at compile time (0: y + BN partial sums, 1: fp32 gradient, 2: UNET_OUT_F32_GATED — the
// attention gate's W_x input gradient, with the x*s term of the same gradient added here instead of by
// gate_bwd1: d(x*s) and s = sigmoid(psi) are loaded ahead of the MFMAs).  Distinct instantiations also keep
// the forward and the dgrads apart in kernel traces and PMC passes (tools/traffic.py)
// XD (round 6): the x vectors are loaded XD chunk steps ahead (a ring of XD register sets; XD divides nchunks, so
// a tile's last steps prefetch the next tile's first XD chunks into the same ring slots).  With one step ahead,
// a wave had ~2 KB of x in flight per memory round trip: the small maps (one or two 32-pixel tiles per wave,
// 8-16 chunks each) ran latency-bound at 0.8-1.5 TB/s.  The weights and scale / shift (L2-resident) stay one
// step ahead.
template <typename T, int NA, int NB, int OMK, int XD>
__global__ __launch_bounds__(256, 2) void pw_conv_kernel(const unet_conv_desc d, long long P, int nchunks) {
  constexpr bool GATED = OMK == 2;
  typedef typename Mma<T>::frag F;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int co0 = blockIdx.y * (16 * NA);
  const unet_src& s = d.src[0];
  const bool act = s.kind == UNET_SRC_ACT;
  const float lo = s.relu ? 0.f : -INFINITY;
  const unsigned pixb = (unsigned)d.Cin * 2u;
  const pw_rsrc_t xr = pw_rsrc(s.data, (unsigned)(P * pixb));
  // packed weights [ntile][chunk][64 lanes][16 B] (1x1: one tap)
  const pw_rsrc_t wr = pw_rsrc(d.weight, (unsigned)((d.Cout + 127) / 128 * 8) * (unsigned)nchunks * 1024u);
  // persistent over pixel tiles (16 NB pixels per wave tile, wave tiles grid-strided so that the waves in
  // flight read neighbouring pixels): the set-up, the BN-sum reduction and the partial-row store are paid once
  // per wave instead of once per tile, and the next tile's first loads are issued before this tile's epilogue
  const long long ntiles = (P + 16 * NB - 1) / (16 * NB);
  const long long tstride = (long long)gridDim.x * 4;
  long long tile = (long long)blockIdx.x * 4 + wave;

  // this lane's pixels (one per px tile) and their gate pre-activations; pixels past P read as 0 (OOB) and
  // are forced to 0 after the transform.  Every (tile, chunk) step's operands — the x vectors, the weight
  // fragments and the BN scale / shift of the chunk — are loaded one step ahead, across tile boundaries too
  // (round 5: the weights and scale / shift were loaded by the step that used them, and a tile's first x
  // chunk at its start: ~3 memory round trips per 64-pixel tile, 5.8 us per tile per wave at 512^2)
  const bool gate = act && s.gate_p != nullptr;
  unsigned xoff[NB], xoffn[NB];
  float gp[NB], gok[NB], gm[NB], gpn[NB], gokn[NB];
  // a tile's pixel offsets / validity / gate pre-activations (no x loads)
  auto setup = [&](long long t, unsigned (&xo)[NB], float (&go)[NB], float (&gq)[NB]) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const long long p = t * (16 * NB) + 16 * b + i16;
      const bool ok = t < ntiles && p < P;
      xo[b] = ok ? (unsigned)p * pixb + (unsigned)g * 16u : PW_OOB;
      go[b] = ok ? 1.f : 0.f;
      gq[b] = (ok && gate) ? s.gate_p[p] : 0.f;
    }
  };
  auto stage = [&](int c, uint4 (&wv)[NA], float4 (&scv)[2], float4 (&sfv)[2]) {
#pragma unroll
    for (int a = 0; a < NA; ++a)
      wv[a] = pw_ld(wr, (unsigned)lane * 16u, ((unsigned)(co0 / 16 + a) * nchunks + c) * 1024u);
    if (act) {
      const int ch = c * 32 + g * 8;
      scv[0] = *reinterpret_cast<const float4*>(s.scale + ch);
      scv[1] = *reinterpret_cast<const float4*>(s.scale + ch + 4);
      sfv[0] = *reinterpret_cast<const float4*>(s.shift + ch);
      sfv[1] = *reinterpret_cast<const float4*>(s.shift + ch + 4);
    }
  };
  uint4 xq[XD][NB], wq[NA];
  float4 scq[2], sfq[2];
  setup(tile, xoff, gok, gp);
#pragma unroll
  for (int u = 0; u < XD; ++u)
#pragma unroll
    for (int b = 0; b < NB; ++b) xq[u][b] = pw_ld(xr, xoff[b], (unsigned)u * 64u);   // XD <= nchunks
  stage(0, wq, scq, sfq);

  float sm[NA][4], sq[NA][4];   // OMK 0: BN partial sums over all of this wave's tiles (pixels past P add 0)
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int r = 0; r < 4; ++r) { sm[a][r] = 0.f; sq[a][r] = 0.f; }

  for (; tile < ntiles; tile += tstride) {
    const long long pw0 = tile * (16 * NB);
#pragma unroll
    for (int b = 0; b < NB; ++b) gm[b] = gate ? gok[b] * sigmoidf_(gp[b] * s.gate_ab[0] + s.gate_ab[1]) : gok[b];
    f32x4 acc[NA][NB];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < NB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    // fp32 gradient epilogue that accumulates: the old values are loaded here, ahead of the MFMAs (the
    // compiler cannot hoist them over the stores, which it must assume alias; loaded in the epilogue, each
    // read-modify-write was a full memory round trip per 16-byte column)
    float4 old[NB][NA];
    const bool rmw = OMK == 1 && (d.accum || d.accum2);
    float4 gxs[GATED ? NB : 1][GATED ? NA : 1];
    float gsv[GATED ? NB : 1];
    if constexpr (GATED) {
      const float* dxs = (const float*)d.pool_src.data;
      const float ga = d.pool_src.gate_ab[0], gb = d.pool_src.gate_ab[1];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const long long p = pw0 + 16 * b + i16;
        gsv[b] = p < P ? sigmoidf_(d.pool_src.gate_p[p] * ga + gb) : 0.f;
#pragma unroll
        for (int a = 0; a < NA; ++a)
          gxs[b][a] = p < P ? *reinterpret_cast<const float4*>(dxs + p * d.Cout + co0 + 16 * a + 4 * g)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (rmw) {
      const int c2 = d.Cout - d.split;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const long long p = pw0 + 16 * b + i16;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          const int co = co0 + 16 * a + 4 * g;
          const bool first = co < d.split;
          const int acc_in = first ? d.accum : d.accum2;
          old[b][a] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (p < P && acc_in)
            old[b][a] = first ? *reinterpret_cast<const float4*>((const float*)d.out + p * d.split + co)
                              : *reinterpret_cast<const float4*>((const float*)d.out2 + p * c2 + (co - d.split));
        }
      }
    }
    setup(tile + tstride, xoffn, gokn, gpn);   // the next tile's offsets: its first XD chunks load during this one
    for (int c0 = 0; c0 < nchunks; c0 += XD) {
#pragma unroll
      for (int u = 0; u < XD; ++u) {
        const int c = c0 + u;
        const float sc[8] = {scq[0].x, scq[0].y, scq[0].z, scq[0].w, scq[1].x, scq[1].y, scq[1].z, scq[1].w};
        const float sf[8] = {sfq[0].x, sfq[0].y, sfq[0].z, sfq[0].w, sfq[1].x, sfq[1].y, sfq[1].z, sfq[1].w};
        F xb[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) xb[b] = pw_act<T>(xq[u][b], act, sc, sf, lo, gm[b]);
        // ring slot u: chunk c + XD (of this tile, or of the next one)
        const int cn = c + XD;
        if (cn < nchunks) {
#pragma unroll
          for (int b = 0; b < NB; ++b) xq[u][b] = pw_ld(xr, xoff[b], (unsigned)cn * 64u);
        } else {
#pragma unroll
          for (int b = 0; b < NB; ++b) xq[u][b] = pw_ld(xr, xoffn[b], (unsigned)(cn - nchunks) * 64u);
        }
        // the next step's weights and scale / shift
        uint4 wn[NA];
        float4 scn[2], sfn[2];
        stage(c + 1 < nchunks ? c + 1 : 0, wn, scn, sfn);
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          const F wa = __builtin_bit_cast(F, wq[a]);
#pragma unroll
          for (int b = 0; b < NB; ++b) acc[a][b] = Mma<T>::mma(wa, xb[b], acc[a][b]);
        }
#pragma unroll
        for (int a = 0; a < NA; ++a) wq[a] = wn[a];
        scq[0] = scn[0]; scq[1] = scn[1]; sfq[0] = sfn[0]; sfq[1] = sfn[1];
      }
    }

    // epilogue: acc[a][b][r] = out[px = pw0 + 16b + i16][co = co0 + 16a + 4g + r]
    if constexpr (OMK == 0) {
      T* y = (T*)d.out;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const long long p = pw0 + 16 * b + i16;
        if constexpr (NA % 2 == 0) {
          // lane (i16, g) holds channels 16 a + 4 g .. + 3 of pixel p: v_permlane16_swap of the packed (a, a + 1)
          // pairs leaves row g with the 8 contiguous channels 16 (a + (g & 1)) + 8 (g >> 1) .. + 7, stored as one
          // 16-byte vector (smallcin.hip's epilogue); every lane takes part in the swaps, the stores are masked
#pragma unroll
          for (int a = 0; a < NA; a += 2) {
            const f32x4 v0 = acc[a][b], v1 = acc[a + 1][b];
            const auto sx = __builtin_amdgcn_permlane16_swap(pack2_16<T>(v0[0], v0[1]), pack2_16<T>(v1[0], v1[1]),
                                                             false, false);
            const auto sy = __builtin_amdgcn_permlane16_swap(pack2_16<T>(v0[2], v0[3]), pack2_16<T>(v1[2], v1[3]),
                                                             false, false);
            if (p < P)
              *reinterpret_cast<uint4*>(y + p * d.Cout + co0 + 16 * (a + (g & 1)) + 8 * (g >> 1)) =
                  make_uint4(sx[0], sy[0], sx[1], sy[1]);
          }
        } else {
#pragma unroll
          for (int a = 0; a < NA; ++a) {
            const int co = co0 + 16 * a + 4 * g;
            if (p < P) {
              const f32x4 v = acc[a][b];
              *reinterpret_cast<uint2*>(y + p * d.Cout + co) = make_uint2(pack2_16<T>(v[0], v[1]), pack2_16<T>(v[2], v[3]));
            }
          }
        }
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
          for (int r = 0; r < 4; ++r) {  // pixels past P accumulated exact zeros
            sm[a][r] += acc[a][b][r];
            sq[a][r] += acc[a][b][r] * acc[a][b][r];
          }
      }
    } else {  // UNET_OUT_F32 (host-checked: split % 4 == 0)
      float* o1 = (float*)d.out;
      float* o2 = (float*)d.out2;
      const int c2 = d.Cout - d.split;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const long long p = pw0 + 16 * b + i16;
        if (p >= P) continue;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          const int co = co0 + 16 * a + 4 * g;
          float4* q = co < d.split ? reinterpret_cast<float4*>(o1 + p * d.split + co)
                                   : reinterpret_cast<float4*>(o2 + p * c2 + (co - d.split));
          float4 v = make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
          if constexpr (GATED) {
            // the x*s term as gate_bwd1 formed it (old + d*s, or d*s), then + W_x^T dy as the separate
            // accumulating dgrad added it: the same fp32 operations in the same order
            const float4 x = gxs[b][a];
            const float sg = gsv[b];
            float4 t;
            if (d.accum) {
              const float4 o = *q;
              t = make_float4(__builtin_fmaf(x.x, sg, o.x), __builtin_fmaf(x.y, sg, o.y), __builtin_fmaf(x.z, sg, o.z),
                              __builtin_fmaf(x.w, sg, o.w));
            } else {
              t = make_float4(x.x * sg, x.y * sg, x.z * sg, x.w * sg);
            }
            v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
          } else if (rmw && (co < d.split ? d.accum : d.accum2)) {
            const float4 o = old[b][a];
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *q = v;
        }
      }
    }
#pragma unroll
    for (int b = 0; b < NB; ++b) { xoff[b] = xoffn[b]; gok[b] = gokn[b]; gp[b] = gpn[b]; }
  }
  if constexpr (OMK == 0) {
    if (d.stats) {
      __shared__ float red[4][NA * 16][2];
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float u = sm[a][r], w = sq[a][r];
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) { u += __shfl_xor(u, o, 64); w += __shfl_xor(w, o, 64); }
          if (i16 == 0) { red[wave][16 * a + 4 * g + r][0] = u; red[wave][16 * a + 4 * g + r][1] = w; }
        }
      __syncthreads();
      if (tid < NA * 16) {
        const int co = co0 + tid;
        const float u = red[0][tid][0] + red[1][tid][0] + red[2][tid][0] + red[3][tid][0];
        const float w = red[0][tid][1] + red[1][tid][1] + red[2][tid][1] + red[3][tid][1];
        d.stats[(size_t)co * gridDim.x + blockIdx.x] = u;
        d.stats[((size_t)d.Cout + co) * gridDim.x + blockIdx.x] = w;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// wgrad.  Block = 4 waves owns dW[co0 .. co0+16*MA)[ci0 .. ci0+64*MB); wave w owns ci tiles
// [w*MB, (w+1)*MB).  blockIdx.x = split (a contiguous range of 64-pixel tiles).
// ------------------------------------------------------------------------------------------------
constexpr int PW_KP = 64;  // pixels per staged tile

template <typename T>
__device__ __forceinline__ typename Mma<T>::frag pw_tr8(const T* r0, const T* r1) {
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(r0));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) i16x4*)(r1));
  typedef __attribute__((ext_vector_type(8))) short i16x8;
  const i16x8 r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(typename Mma<T>::frag, r);
}

template <typename T, int MA, int MB, bool GATED>
__global__ __launch_bounds__(256, 2) void pw_wgrad_kernel(const unet_wgrad_desc d, long long P, int per_split, float* ws) {
  typedef typename Mma<T>::frag F;
  constexpr int BCO = 16 * MA, BCI = 64 * MB;
  // LDS row strides: odd multiples of 32 B (see wgrad2.hip) so the tr reads are conflict-free
  constexpr int RSD = BCO + (BCO % 32 == 0 ? 16 : 32 - BCO % 32 + 16);
  constexpr int RSX = BCI + 16;
  static_assert((RSD / 16) % 2 == 1 && (RSX / 16) % 2 == 1, "odd multiples of 32 B");
  constexpr int NVD = BCO / 8, NVX = BCI / 8;              // 16-byte vectors per pixel row
  constexpr int ID = (PW_KP * NVD + 255) / 256, IX = (PW_KP * NVX + 255) / 256;
  constexpr int BUF = PW_KP * (RSD + RSX);
  __shared__ __attribute__((aligned(16))) T lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int co0 = blockIdx.z * BCO, ci0 = blockIdx.y * BCI;
  const long long ntiles = (P + PW_KP - 1) / PW_KP;
  const long long t_begin = (long long)blockIdx.x * per_split;
  const long long t_end = t_begin + per_split < ntiles ? t_begin + per_split : ntiles;
  const unet_src& s = d.src[0];
  const bool act = s.kind == UNET_SRC_ACT;
  const float lo = s.relu ? 0.f : -INFINITY;
  const unsigned xpix = (unsigned)d.Cin * 2u, dpix = (unsigned)d.Cout * 2u;
  const pw_rsrc_t xr = pw_rsrc(s.data, (unsigned)(P * xpix));
  const pw_rsrc_t dr = pw_rsrc(d.dy, (unsigned)(P * dpix));
  const pw_rsrc_t gr_ = pw_rsrc(GATED ? (const void*)s.gate_p : s.data, (unsigned)(GATED ? P * 4 : 0));
  float ga = 0.f, gb = 0.f;
  if (GATED) { ga = s.gate_ab[0]; gb = s.gate_ab[1]; }

  // fixed per-thread channel vectors (NVX, NVD divide 256)
  const int vx = tid % NVX, vd = tid % NVD;
  const int cx = ci0 + vx * 8, cd = co0 + vd * 8;
  const bool cx_ok = cx < d.Cin, cd_ok = cd < d.Cout;
  float sc[8], sf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = 1.f; sf[j] = 0.f; }
  if (act && cx_ok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = s.scale[cx + j]; sf[j] = s.shift[cx + j]; }
  }
  // NQ register sets of staged loads: tiles t+1 .. t+NQ in flight while tile t is computed from LDS.  The loop
  // is a memory round trip per NQ tiles: with 2 sets the 512^2 1x1 weight gradients ran at ~1.7 TB/s (round 5,
  // profiles/r05_*), i.e. latency-bound; the gate pre-activation is loaded with the tile and turned into its
  // sigmoid when the tile is written to LDS (a sigmoid at issue time waited for its load right there)
  constexpr int NQ = 4;
  uint4 qx[NQ][IX], qd[NQ][ID];
  float gv[NQ][IX], gp[NQ][IX];
  auto issue = [&](int b, long long t) {
    const long long pbase = t * PW_KP;
#pragma unroll
    for (int k = 0; k < IX; ++k) {
      const int pr = (tid + 256 * k) / NVX;
      const long long p = pbase + pr;
      const bool ok = t < t_end && pr < PW_KP && p < P && cx_ok;
      qx[b][k] = pw_ld(xr, ok ? (unsigned)p * xpix + (unsigned)cx * 2u : PW_OOB, 0);
      gv[b][k] = ok ? 1.f : 0.f;
      if constexpr (GATED)
        gp[b][k] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(gr_, ok ? (int)((unsigned)p * 4u) : (int)PW_OOB, 0, 0));
    }
#pragma unroll
    for (int k = 0; k < ID; ++k) {
      const int pr = (tid + 256 * k) / NVD;
      const long long p = pbase + pr;
      const bool ok = t < t_end && pr < PW_KP && p < P && cd_ok;
      qd[b][k] = pw_ld(dr, ok ? (unsigned)p * dpix + (unsigned)cd * 2u : PW_OOB, 0);
    }
  };
  auto finish = [&](int b, T* buf) {
    T* bd = buf;
    T* bx = buf + PW_KP * RSD;
#pragma unroll
    for (int k = 0; k < IX; ++k) {
      const int pr = (tid + 256 * k) / NVX;
      float gm = gv[b][k];
      if constexpr (GATED) gm = gm * sigmoidf_(gp[b][k] * ga + gb);
      if (pr < PW_KP) *reinterpret_cast<F*>(bx + pr * RSX + vx * 8) = pw_act<T>(qx[b][k], act, sc, sf, lo, gm);
    }
#pragma unroll
    for (int k = 0; k < ID; ++k) {
      const int pr = (tid + 256 * k) / NVD;
      if (pr < PW_KP) *reinterpret_cast<uint4*>(bd + pr * RSD + vd * 8) = qd[b][k];
    }
  };

  f32x4 acc[MA][MB];
#pragma unroll
  for (int a = 0; a < MA; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // tr-read lane geometry: group g reads pixel rows k0 + 8g + q (+4); odd groups take the +4 half first
  // (bank spread) — A and B apply the same K permutation, so the MFMA sums are unchanged
  const int g = lane >> 4, q = (lane & 15) >> 2, p4 = (lane & 3) * 4;
  const int sw = (g & 1) * 4;
  auto compute = [&](const T* bd) {
    const T* bx = bd + PW_KP * RSD;
#pragma unroll
    for (int k0 = 0; k0 < PW_KP; k0 += 32) {
      const int r0 = k0 + 8 * g + q + sw, r1 = k0 + 8 * g + q + 4 - sw;
      F av[MA];
#pragma unroll
      for (int a = 0; a < MA; ++a) av[a] = pw_tr8<T>(bd + r0 * RSD + 16 * a + p4, bd + r1 * RSD + 16 * a + p4);
#pragma unroll
      for (int b = 0; b < MB; ++b) {
        const int col = 16 * (wave * MB + b) + p4;
        const F bv = pw_tr8<T>(bx + r0 * RSX + col, bx + r1 * RSX + col);
#pragma unroll
        for (int a = 0; a < MA; ++a) acc[a][b] = Mma<T>::mma(av[a], bv, acc[a][b]);
      }
    }
  };

  if (t_begin < t_end) {
#pragma unroll
    for (int b = 0; b < NQ; ++b) issue(b, t_begin + b);
    finish(0, lds);
  }
  __syncthreads();
  // tile t: register set (t - t_begin) % NQ, LDS buffer (t - t_begin) & 1; a set is re-issued (tile t + NQ) as
  // soon as its tile is in LDS; tiles past t_end load nothing (zeros, never finished)
  for (long long t = t_begin; t < t_end; t += NQ) {
#pragma unroll
    for (int j = 0; j < NQ; ++j) {
      const long long tj = t + j;
      if (tj >= t_end) break;
      issue(j, tj + NQ);
      compute(lds + (j & 1) * BUF);
      if (tj + 1 < t_end) finish((j + 1) % NQ, lds + ((j + 1) & 1) * BUF);
      __syncthreads();
    }
  }

  // slab ws[split][co][ci]; C layout: row (co) = 4*(l>>4)+r, col (ci) = l&15
  float* slab = ws + (size_t)blockIdx.x * d.Cout * d.Cin;
#pragma unroll
  for (int a = 0; a < MA; ++a)
#pragma unroll
    for (int b = 0; b < MB; ++b) {
      const int ci = ci0 + 16 * (wave * MB + b) + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + 16 * a + 4 * (lane >> 4) + r;
        if (co < d.Cout && ci < d.Cin) slab[(size_t)co * d.Cin + ci] = acc[a][b][r];
      }
    }
}

// out[g][e] (+)= sum over slabs s in [g*per, min(splits, (g+1)*per)) of ws[s][e], in slab order (deterministic).
// One thread per (16-byte column, group): a split-K reduction of many slabs of a small weight gradient
// runs as two such passes (splits -> PW_RG groups -> 1) instead of one long serial loop per column.
constexpr int PW_RG = 32;
__global__ void pw_slab_reduce_kernel(const float* ws, int splits, int per, long long total4, float* out, int accum) {
  const long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const int g = blockIdx.y;
  if (e >= total4) return;
  const int s0 = g * per, s1 = min(splits, s0 + per);
  const float4* w = reinterpret_cast<const float4*>(ws);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  int s = s0;
  for (; s + 4 <= s1; s += 4) {
    const float4 v0 = w[(size_t)s * total4 + e], v1 = w[(size_t)(s + 1) * total4 + e];
    const float4 v2 = w[(size_t)(s + 2) * total4 + e], v3 = w[(size_t)(s + 3) * total4 + e];
    a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
    a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
    a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
    a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
  }
  for (; s < s1; ++s) {
    const float4 v = w[(size_t)s * total4 + e];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  float4* o = reinterpret_cast<float4*>(out) + (size_t)g * total4 + e;
  if (accum) {
    const float4 b = *o;
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  }
  *o = a;
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
// dw (+)= Σ_s ws[s] over `splits` slabs of `total` floats (total % 4 == 0) in two fixed-order passes
// through PW_RG partial slabs at `scratch` (PW_RG * total floats)
// one launch for many slabs: a block owns 64 float4 columns; its 4 waves sum contiguous quarters of the splits
// (4 independent loads in flight per trip), then the quarters are added in wave order — a fixed order, so
// the weight gradient is deterministic (it replaced a two-launch splits -> 32 -> 1 reduction: 2 x ~7 us of
// mostly launch latency per weight gradient)
__global__ __launch_bounds__(256) void slab_reduce_q_kernel(const float* ws, int splits, long long total4, float* out,
                                                            int accum) {
  __shared__ float4 part[4][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const long long e = blockIdx.x * 64LL + lane;
  const int per = (splits + 3) / 4, s0 = q * per, s1 = min(splits, s0 + per);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < total4) {
    const float4* w = reinterpret_cast<const float4*>(ws);
    int s = s0;
    for (; s + 4 <= s1; s += 4) {
      const float4 v0 = w[(size_t)s * total4 + e], v1 = w[(size_t)(s + 1) * total4 + e];
      const float4 v2 = w[(size_t)(s + 2) * total4 + e], v3 = w[(size_t)(s + 3) * total4 + e];
      a.x += v0.x; a.y += v0.y; a.z += v0.z; a.w += v0.w;
      a.x += v1.x; a.y += v1.y; a.z += v1.z; a.w += v1.w;
      a.x += v2.x; a.y += v2.y; a.z += v2.z; a.w += v2.w;
      a.x += v3.x; a.y += v3.y; a.z += v3.z; a.w += v3.w;
    }
    for (; s < s1; ++s) {
      const float4 v = w[(size_t)s * total4 + e];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  part[q][lane] = a;
  __syncthreads();
  if (q == 0 && e < total4) {
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 b = part[k][lane];
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float4* o = reinterpret_cast<float4*>(out) + e;
    if (accum) {
      const float4 b = *o;
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    *o = a;
  }
}

int slab_reduce_two_pass(const float* ws, int splits, long long total, float* scratch, float* dw, int accum,
                         hipStream_t st) {
  const long long total4 = total / 4;
  if (total4 >= 8192) {
    hipLaunchKernelGGL(slab_reduce_q_kernel, dim3((unsigned)((total4 + 63) / 64)), dim3(256), 0, st, ws, splits, total4,
                       dw, accum);
    return check_launch("slab_reduce");
  }
  // small weights (the attention gate's 1x1 projections): too few columns for one launch to fill the chip —
  // splits -> PW_RG groups -> 1, still a fixed order
  const int per = cdiv(splits, PW_RG), groups = cdiv(splits, per);
  hipLaunchKernelGGL(pw_slab_reduce_kernel, dim3(cdiv(total4, 256), groups), dim3(256), 0, st, ws, splits, per, total4,
                     scratch, 0);
  hipLaunchKernelGGL(pw_slab_reduce_kernel, dim3(cdiv(total4, 256), 1), dim3(256), 0, st, (const float*)scratch, groups,
                     groups, total4, dw, accum);
  return check_launch("slab_reduce");
}
static bool pw_src_ok(const unet_src& s, int C) {
  return (s.kind == UNET_SRC_PLAIN || s.kind == UNET_SRC_ACT) && s.C == C && !(s.gate_p && s.kind != UNET_SRC_ACT);
}

// the 1x1 convs of the attention-gate projections at 64^2..512^2 (P >= 16384 pixels at bs 4).  Round 6: the 64^2
// ones moved here from the tiled conv2 (the x prefetch ring made the difference: 33 -> 23 us fwd, 37 -> 28 us
// dgrad, profiles/r06_layerprof_pw_*.txt); UNET_PW_WIDE=0 restores the round-5 cut (P >= 32768, Cin <= 256)
bool pw_conv_ok(const unet_conv_desc* d) {
  const long long P = (long long)d->N * d->H * d->W;
  if ((d->dtype != UNET_BF16 && d->dtype != UNET_F16) || d->ksize != 1 || d->nsrc != 1 ||
      !pw_src_ok(d->src[0], d->Cin))
    return false;
  static const int wide = [] { const char* e = getenv("UNET_PW_WIDE"); return e ? atoi(e) : 1; }();
  if (d->Cin % 32 || d->Cout % 16) return false;
  if (wide ? (d->Cin > 512 || P < 16384) : (d->Cin > 256 || P < 32768)) return false;
  if (d->out_mode == UNET_OUT_F32) { if (d->split % 4) return false; }
  else if (d->out_mode == UNET_OUT_F32_GATED) { if (d->split != d->Cout) return false; }
  else if (d->out_mode != UNET_OUT_Y) return false;
  return (double)P * d->Cin * 2 < (double)PW_OOB;
}

// NA = 4 (64 output channels per wave) with 32-pixel wave tiles: the 64-pixel ones needed 268-292 registers, one
// wave per SIMD (round 5); every instantiation is bounded to 256 (two waves per SIMD, __launch_bounds__(256, 2))
static void pw_conv_geom(const unet_conv_desc* d, int& na, int& nb) {
  na = d->Cout % 64 == 0 ? 4 : (d->Cout % 32 == 0 ? 2 : 1);
  nb = na == 4 ? 2 : 4;
}

// blocks along the pixels: the pw_conv_kernel waves are persistent over wave tiles (16 NB pixels each); up to
// PW_BLOCKS blocks of 4 waves, i.e. 8 tiles per wave on the 512^2 maps (UNET_PW_BLOCKS: A/B override).  Round-4
// layer sweep (tools/gpu_r04.sh lp): one tile per wave 797 us/step for the 1x1 fwd + dgrads, 1024 blocks 758,
// 512 blocks 739 (profiles/r04_pw_persistent_sweep.txt)
constexpr long long PW_BLOCKS = 512;
static int pw_blocks(const unet_conv_desc* d, int nb) {
  const long long P = (long long)d->N * d->H * d->W;
  const long long tiles = cdiv(P, 16 * nb);
  const char* e = getenv("UNET_PW_BLOCKS");
  const long long cap = e && atoll(e) > 0 ? atoll(e) : PW_BLOCKS;
  long long b = cdiv(tiles, 4);
  return (int)(b < cap ? b : cap);
}

int pw_conv_rows(const unet_conv_desc* d) {
  int na, nb;
  pw_conv_geom(d, na, nb);
  return pw_blocks(d, nb);
}

template <typename T, int NA, int NB, int XD>
static void launch_pw_xd(const unet_conv_desc* d, hipStream_t st) {
  const long long P = (long long)d->N * d->H * d->W;
  dim3 grid(pw_blocks(d, NB), d->Cout / (16 * NA));
  if (d->out_mode == UNET_OUT_F32_GATED)
    hipLaunchKernelGGL((pw_conv_kernel<T, NA, NB, 2, XD>), grid, dim3(256), 0, st, *d, P, d->Cin / 32);
  else if (d->out_mode == UNET_OUT_F32)
    hipLaunchKernelGGL((pw_conv_kernel<T, NA, NB, 1, XD>), grid, dim3(256), 0, st, *d, P, d->Cin / 32);
  else
    hipLaunchKernelGGL((pw_conv_kernel<T, NA, NB, 0, XD>), grid, dim3(256), 0, st, *d, P, d->Cin / 32);
}
// x prefetch depth: 4 chunks where the chunk count allows (NB = 2: 8 registers per ring slot), else 2 or 1
// (UNET_PW_XD: A/B cap, read per call)
template <typename T, int NA, int NB>
static int launch_pw(const unet_conv_desc* d, hipStream_t st) {
  const int nch = d->Cin / 32;
  const char* e = getenv("UNET_PW_XD");
  const int cap = e ? atoi(e) : 4;
  if constexpr (NB == 2) {
    if (cap >= 4 && nch % 4 == 0) {
      launch_pw_xd<T, NA, NB, 4>(d, st);
      return check_launch("pw_conv");
    }
  }
  if (cap >= 2 && nch % 2 == 0) launch_pw_xd<T, NA, NB, 2>(d, st);
  else launch_pw_xd<T, NA, NB, 1>(d, st);
  return check_launch("pw_conv");
}

template <typename T>
static int pw_conv_t(const unet_conv_desc* d, hipStream_t st) {
  int na, nb;
  pw_conv_geom(d, na, nb);
  if (na == 4) return launch_pw<T, 4, 2>(d, st);
  if (na == 2) return launch_pw<T, 2, 4>(d, st);
  return launch_pw<T, 1, 4>(d, st);
}

int pw_conv(const unet_conv_desc* d, hipStream_t st) {
  return d->dtype == UNET_F16 ? pw_conv_t<f16>(d, st) : pw_conv_t<bf16>(d, st);
}

int pw_conv_variant(const unet_conv_desc* d, char* buf, int len) {
  int na, nb;
  pw_conv_geom(d, na, nb);
  if (d->dtype == UNET_F16) snprintf(buf, len, "pw_conv_kernel<fp16,%d,%d>", na, nb);
  else snprintf(buf, len, "pw_conv_kernel<%d,%d>", na, nb);
  return 0;
}

struct PwWPlan {
  int ma, mb, splits, per_split;
  size_t ws_bytes;
};

bool pw_wgrad_ok(const unet_wgrad_desc* d) {
  const long long P = (long long)d->N * d->H * d->W;
  if ((d->dtype != UNET_BF16 && d->dtype != UNET_F16) || d->ksize != 1 || d->nsrc != 1 ||
      !pw_src_ok(d->src[0], d->Cin))
    return false;
  // smallest map served (pixels): wgrad2 won at 128^2 x bs4 when measured in round 4; UNET_PW_WGRAD_MINP re-tests it
  static const long long minp = [] {
    const char* e = getenv("UNET_PW_WGRAD_MINP");
    return e && atoll(e) > 0 ? atoll(e) : 131072LL;
  }();
  if (d->Cin % 64 || d->Cout % 16 || P < minp) return false;
  return (double)P * d->Cin * 2 < (double)PW_OOB && (double)P * d->Cout * 2 < (double)PW_OOB;
}

static PwWPlan pw_wplan(const unet_wgrad_desc* d) {
  PwWPlan p{};
  p.ma = d->Cout % 64 == 0 ? 4 : (d->Cout % 32 == 0 ? 2 : 1);
  p.mb = d->Cin % 128 == 0 ? 2 : 1;   // (MB = 4 needed 320-413 registers: one wave per SIMD or spills)
  const long long P = (long long)d->N * d->H * d->W;
  const long long ntiles = (P + PW_KP - 1) / PW_KP;
  const long long blocks_out = (long long)(d->Cout / (16 * p.ma)) * (d->Cin / (64 * p.mb));
  const size_t slab = (size_t)d->Cout * d->Cin * sizeof(float);
  // workgroup target: one or two per CU.  Each split writes (and the reduction reads back) a whole fp32 slab of
  // the weight gradient, so more splits cost slab traffic: with 4 tiles in flight per workgroup, 256 - 512
  // workgroups measured 10-26 % faster than the former 1024 (tools/pww_ab.py, profiles/r05_pww_blocks.txt)
  const char* e = getenv("UNET_PWW_BLOCKS");   // A/B of the workgroup target (read per call)
  const long long target = e && atoll(e) > 0 ? atoll(e) : (slab >= (16u << 10) ? 256 : 512);
  long long s = (target + blocks_out - 1) / blocks_out;
  const long long cap = (long long)(((size_t)64 << 20) / slab);  // slab traffic <= 64 MB
  if (s > cap) s = cap;
  if (s > ntiles) s = ntiles;
  if (s < 1) s = 1;
  p.per_split = cdiv(ntiles, s);
  p.splits = cdiv(ntiles, p.per_split);
  p.ws_bytes = slab * (p.splits + PW_RG);
  return p;
}

size_t pw_wgrad_ws(const unet_wgrad_desc* d) { return pw_wplan(d).ws_bytes; }

template <int MA, int MB>
static int launch_pww(const unet_wgrad_desc* d, const PwWPlan& p, hipStream_t st) {
  const long long P = (long long)d->N * d->H * d->W;
  dim3 grid(p.splits, d->Cin / (64 * MB), d->Cout / (16 * MA));
  const bool g = d->src[0].kind == UNET_SRC_ACT && d->src[0].gate_p;
  float* ws = (float*)d->workspace;
  if (d->dtype == UNET_F16) {
    if (g) hipLaunchKernelGGL((pw_wgrad_kernel<f16, MA, MB, true>), grid, dim3(256), 0, st, *d, P, p.per_split, ws);
    else hipLaunchKernelGGL((pw_wgrad_kernel<f16, MA, MB, false>), grid, dim3(256), 0, st, *d, P, p.per_split, ws);
  } else {
    if (g) hipLaunchKernelGGL((pw_wgrad_kernel<bf16, MA, MB, true>), grid, dim3(256), 0, st, *d, P, p.per_split, ws);
    else hipLaunchKernelGGL((pw_wgrad_kernel<bf16, MA, MB, false>), grid, dim3(256), 0, st, *d, P, p.per_split, ws);
  }
  return check_launch("pw_wgrad");
}

int pw_wgrad(const unet_wgrad_desc* d, hipStream_t st) {
  const PwWPlan p = pw_wplan(d);
  int e;
  if (p.ma == 4) e = p.mb == 2 ? launch_pww<4, 2>(d, p, st) : launch_pww<4, 1>(d, p, st);
  else if (p.ma == 2) e = p.mb == 2 ? launch_pww<2, 2>(d, p, st) : launch_pww<2, 1>(d, p, st);
  else e = p.mb == 2 ? launch_pww<1, 2>(d, p, st) : launch_pww<1, 1>(d, p, st);
  if (e) return e;
  // slabs -> PW_RG partial slabs (written after the split slabs in the workspace) -> dw
  const long long total = (long long)d->Cout * d->Cin;
  return slab_reduce_two_pass((const float*)d->workspace, p.splits, total,
                              (float*)d->workspace + (size_t)p.splits * total, d->dw, d->accum, st);
}

}  // namespace unet
