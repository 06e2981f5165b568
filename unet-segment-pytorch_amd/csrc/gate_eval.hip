// gate_eval.hip — the eval-mode AttentionGate forward in one pass.
//
// Reference: AttentionGate.forward (unet/models/layers.py:171-192) in eval mode, as scripts/predict.py
// runs it: with BatchNorm on its running statistics, W_g(g_up) + W_x(x) -> BN -> ReLU -> psi is a
// per-pixel function of the two inputs, so the gate's psi pre-activation
//   p = Σ_c wpsi[c] · relu(sg[c]·(W_g·g)[c] + bg[c] + sx[c]·(W_x·x)[c] + bx[c])
// is computed without storing the two Ci-channel projections: a wave runs both 1x1 GEMMs for 16·NB
// pixels on MFMA (packed weight fragment as the A operand from L2, one 16-byte NHWC load per lane as the
// B operand, the skip's BN+ReLU applied in registers), folds the two BN affines, the ReLU and the psi
// dot product into the accumulators, and writes one fp32 value per pixel.  The training path keeps the
// two-pass form (the BN batch statistics of the projections need the whole batch first).
#include "conv_common.h"

namespace unet {

struct GateEvalArgs {
  long long P;
  int Cg, Cx, Ci;
  const void* g;        // gating input at x's size (op dtype NHWC [P][Cg], stored)
  const void* x;        // skip activation y (op dtype NHWC [P][Cx]); the value is relu?(y*xs + xb)
  const float* xs;
  const float* xb;
  int xrelu;
  const void* wg;       // W_g / W_x packed by unet_pack_weight(transpose=0): rows Ci, reduction Cg / Cx
  const void* wx;
  const float* gab;     // [2][Ci] eval BN affine of W_g's output
  const float* xab;     // [2][Ci] eval BN affine of W_x's output
  const float* wpsi;    // [Ci]
  float* p;             // [P]
};

constexpr unsigned GE_OOB = 0x40000000u;  // >= every map admitted (host-checked), reads as 0
typedef __amdgpu_buffer_rsrc_t ge_rsrc_t;
__device__ __forceinline__ ge_rsrc_t ge_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 ge_ld(ge_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}

template <typename T, int NA, int NB>
__global__ __launch_bounds__(256) void gate_eval_kernel(const GateEvalArgs a) {
  using M = Mma<T>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g4 = lane >> 4;
  const long long p0 = ((long long)blockIdx.x * 4 + wave) * (16 * NB);
  const unsigned gpix = (unsigned)a.Cg * 2u, xpix = (unsigned)a.Cx * 2u;
  const ge_rsrc_t gr = ge_rsrc(a.g, (unsigned)(a.P * gpix));
  const ge_rsrc_t xr = ge_rsrc(a.x, (unsigned)(a.P * xpix));
  const int ncg = a.Cg / 32, ncx = a.Cx / 32;
  const unsigned ntiles = (unsigned)((a.Ci + 127) / 128 * 8);   // packed rows padded to 128 (conv.hip)
  const ge_rsrc_t wgr = ge_rsrc(a.wg, ntiles * (unsigned)ncg * 1024u);
  const ge_rsrc_t wxr = ge_rsrc(a.wx, ntiles * (unsigned)ncx * 1024u);
  const float lo = a.xrelu ? 0.f : -INFINITY;

  unsigned goff[NB], xoff[NB];
  bool ok[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const long long p = p0 + 16 * b + i16;
    ok[b] = p < a.P;
    goff[b] = ok[b] ? (unsigned)p * gpix + (unsigned)g4 * 16u : GE_OOB;
    xoff[b] = ok[b] ? (unsigned)p * xpix + (unsigned)g4 * 16u : GE_OOB;
  }
  float psum[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) psum[b] = 0.f;

  for (int grp = 0; grp < a.Ci; grp += 16 * NA) {
    f32x4 acc_g[NA][NB], acc_x[NA][NB];
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int b = 0; b < NB; ++b) { acc_g[i][b] = f32x4{0.f, 0.f, 0.f, 0.f}; acc_x[i][b] = acc_g[i][b]; }
    // W_g · g (stored map: the 16-byte vectors are the B fragments as loaded)
    for (int c = 0; c < ncg; ++c) {
      uint4 q[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) q[b] = ge_ld(gr, goff[b], (unsigned)c * 64u);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const typename M::frag w =
            __builtin_bit_cast(typename M::frag, ge_ld(wgr, (unsigned)lane * 16u, ((unsigned)(grp / 16 + i) * ncg + c) * 1024u));
#pragma unroll
        for (int b = 0; b < NB; ++b) acc_g[i][b] = M::mma(w, __builtin_bit_cast(typename M::frag, q[b]), acc_g[i][b]);
      }
    }
    // W_x · relu?(bn(y_x)) (the skip's affine + ReLU applied to the loaded vector; padding pixels stay 0)
    for (int c = 0; c < ncx; ++c) {
      uint4 q[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) q[b] = ge_ld(xr, xoff[b], (unsigned)c * 64u);
      const int ch = c * 32 + g4 * 8;
      const float4 s0 = *reinterpret_cast<const float4*>(a.xs + ch), s1 = *reinterpret_cast<const float4*>(a.xs + ch + 4);
      const float4 f0 = *reinterpret_cast<const float4*>(a.xb + ch), f1 = *reinterpret_cast<const float4*>(a.xb + ch + 4);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sf[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      uint4 v4[NB];
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        float v[8];
        unpack8_16<T>(q[b], v);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = ok[b] ? fmaxf(__builtin_fmaf(v[j], sc[j], sf[j]), lo) : 0.f;
        v4[b] = pack8_16<T>(v);
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const typename M::frag w =
            __builtin_bit_cast(typename M::frag, ge_ld(wxr, (unsigned)lane * 16u, ((unsigned)(grp / 16 + i) * ncx + c) * 1024u));
#pragma unroll
        for (int b = 0; b < NB; ++b) acc_x[i][b] = M::mma(w, __builtin_bit_cast(typename M::frag, v4[b]), acc_x[i][b]);
      }
    }
    // acc[i][b][r] = projection channel grp + 16 i + 4 g4 + r of pixel p0 + 16 b + i16
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int ch = grp + 16 * i + 4 * g4;   // Ci % (16 NA) == 0 (host-checked)
      const float4 gs = *reinterpret_cast<const float4*>(a.gab + ch), gb = *reinterpret_cast<const float4*>(a.gab + a.Ci + ch);
      const float4 xs = *reinterpret_cast<const float4*>(a.xab + ch), xb = *reinterpret_cast<const float4*>(a.xab + a.Ci + ch);
      const float4 wp = *reinterpret_cast<const float4*>(a.wpsi + ch);
      const float gs4[4] = {gs.x, gs.y, gs.z, gs.w}, gb4[4] = {gb.x, gb.y, gb.z, gb.w};
      const float xs4[4] = {xs.x, xs.y, xs.z, xs.w}, xb4[4] = {xb.x, xb.y, xb.z, xb.w};
      const float wp4[4] = {wp.x, wp.y, wp.z, wp.w};
#pragma unroll
      for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          psum[b] += wp4[r] * fmaxf(acc_g[i][b][r] * gs4[r] + gb4[r] + acc_x[i][b][r] * xs4[r] + xb4[r], 0.f);
    }
  }
  // the 4 lane groups hold disjoint channel quarters of the same 16 pixels
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    float v = psum[b];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (g4 == 0 && ok[b]) a.p[p0 + 16 * b + i16] = v;
  }
}

template <typename T>
static int launch_gate_eval(const GateEvalArgs& a, hipStream_t st) {
  constexpr int NB = 2;
  const long long blocks = (a.P + 64 * NB - 1) / (64 * NB);
  if (a.Ci % 64 == 0)
    hipLaunchKernelGGL((gate_eval_kernel<T, 4, NB>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((gate_eval_kernel<T, 2, NB>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return check_launch("gate_eval");
}

}  // namespace unet

using namespace unet;

extern "C" {

int unet_gate_psi_eval(int dtype, long long P, int Cg, int Cx, int Ci, const void* g, const void* x, const float* xs,
                       const float* xb, int xrelu, const void* wg_packed, const void* wx_packed, const float* gab,
                       const float* xab, const float* wpsi, float* p, void* stream) {
  if ((dtype != UNET_BF16 && dtype != UNET_F16) || P <= 0 || Cg <= 0 || Cx <= 0 || Ci <= 0 || Cg % 32 ||
      Cx % 32 || Ci % 32 || !g || !x || !xs || !xb || !wg_packed || !wx_packed || !gab || !xab || !wpsi || !p ||
      (double)P * Cg * 2 >= (double)GE_OOB || (double)P * Cx * 2 >= (double)GE_OOB) {
    set_error("unet_gate_psi_eval: needs 16-bit operands, channel counts divisible by 32, maps below 1 GiB");
    return UNET_ERR_ARG;
  }
  GateEvalArgs a{P, Cg, Cx, Ci, g, x, xs, xb, xrelu, wg_packed, wx_packed, gab, xab, wpsi, p};
  hipStream_t st = (hipStream_t)stream;
  return dtype == UNET_BF16 ? launch_gate_eval<bf16>(a, st) : launch_gate_eval<f16>(a, st);
}

}  // extern "C"
