// pack.hip — every conv weight of a step into the fragment-major MFMA operand layout, one launch
// (the implicit weight reads of nn.Conv2d, layers.py:32,35,120,152,158,164; layout: include/unet_hip.h
// unet_pack_weight).
//
// One workgroup per 16-row x 32-column x taps tile of one job: the tile's fp32 OIHW source is read into LDS
// with coalesced loads (16 contiguous row segments, or 32 for the transposed / 180-degree-flipped dgrad
// weights), then each lane gathers its 8 16-bit values of a fragment unit from LDS and writes 16 bytes.
// The per-unit global gather it replaces read each 4-byte weight from a different cache line (47 us per
// pack of the network's 17.6 M weights, ~1.5 TB/s effective).
#include "conv_common.h"

namespace unet {

constexpr int PT_MAX = UNET_PACK_MAX_JOBS;

struct PackTiles {
  unet_pack_job j[PT_MAX];
  int tile0[PT_MAX + 1];   // first tile (workgroup) of each job; tile0[count] = total
  int count;
};

// LDS tile layouts, padded so the gather below is bank-conflict free (ds_read_b32: two 32-lane groups, bank =
// dword mod 32; a lane reads row rr = lane & 15 of column block g = lane >> 4, 8 values e apart):
//  * forward:    [rr][g][e][tap], each 8-column block g of a row TAPS * 8 + 1 dwords (odd), rows PT_RS apart
//                (= 2 mod 32): rr spreads over the even banks, g = 1 adds an odd offset;
//  * transposed: [kk][rr][tap], kk rows PT_KS apart (= 2 mod 4): 9 rr mod 32 covers a set A of 16 banks and the
//                8 kk of the other column block land on A + 16, its complement (TAPS = 1: rr + 16 g).
// (the unpadded tile had rows 288 = 0 mod 32 dwords apart: 16-way conflicts on every gather read)
template <int TAPS> struct PackLds {
  static constexpr int G8 = 8 * TAPS + 1;
  static constexpr int RS = (4 * G8 + 29) / 32 * 32 + 2;     // smallest >= 4 * G8 that is 2 mod 32
  static constexpr int KS = 16 * TAPS + 2;                   // 2 mod 4
  static constexpr int SIZE = (16 * RS > 32 * KS) ? 16 * RS : 32 * KS;
};
constexpr int PT_LDS = PackLds<9>::SIZE;

// TAPS a compile-time constant (1 or 9): every index division below is by a constant
template <typename T, int TAPS>
__device__ __forceinline__ void pack_tile(const unet_pack_job& jb, int t, float* tile) {
  constexpr int KC = 32, R = 16, taps = TAPS;
  using Lay = PackLds<TAPS>;
  const int rows = jb.transpose ? jb.Cin : jb.Cout, cols = jb.transpose ? jb.Cout : jb.Cin;
  const int nchunks = (cols + KC - 1) / KC;
  const int chunk = t % nchunks, ntile = t / nchunks;
  const int r0 = ntile * R, c0 = chunk * KC;
  // the tile's fp32 source: 16 row segments of KC * taps contiguous floats (forward) or 32 of R * taps
  // (transposed); 16-byte loads when the whole tile is in range and the segments are 16-byte aligned
  constexpr int SEGF = KC * taps, SEGT = R * taps;
  const bool vec = r0 + R <= rows && c0 + KC <= cols && (jb.Cin * taps) % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(jb.w) & 15) == 0;
  if (!jb.transpose) {
    if (vec) {
      for (int f = threadIdx.x; f < R * SEGF / 4; f += 256) {
        const int rr = f / (SEGF / 4), rem = 4 * (f - rr * (SEGF / 4));
        const float4 v = *reinterpret_cast<const float4*>(jb.w + ((long long)(r0 + rr) * jb.Cin + c0) * taps + rem);
        float* d = tile + rr * Lay::RS + rem + rem / (8 * taps);   // 4 | 8 * taps: the 4 stay in one block
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    } else {
      for (int i = threadIdx.x; i < R * SEGF; i += 256) {
        const int rr = i / SEGF, rem = i - rr * SEGF;
        const int r = r0 + rr, cc = c0 + rem / taps;
        tile[rr * Lay::RS + rem + rem / (8 * taps)] =
            (r < rows && cc < cols) ? jb.w[((long long)r * jb.Cin + c0) * taps + rem] : 0.f;
      }
    }
  } else {
    if (vec) {
      for (int f = threadIdx.x; f < KC * SEGT / 4; f += 256) {
        const int kk = f / (SEGT / 4), rem = 4 * (f - kk * (SEGT / 4));
        const float4 v = *reinterpret_cast<const float4*>(jb.w + ((long long)(c0 + kk) * jb.Cin + r0) * taps + rem);
        float* d = tile + kk * Lay::KS + rem;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
      }
    } else {
      for (int i = threadIdx.x; i < KC * SEGT; i += 256) {
        const int kk = i / SEGT, rem = i - kk * SEGT;
        const int r = r0 + rem / taps, cc = c0 + kk;
        tile[kk * Lay::KS + rem] = (r < rows && cc < cols) ? jb.w[((long long)cc * jb.Cin + r0) * taps + rem] : 0.f;
      }
    }
  }
  __syncthreads();
  // the tile's units: packed order [ntile][chunk][tap][lane][8]; lane holds row rr = lane & 15, k = 8(lane>>4)+e
  const long long ubase = ((long long)ntile * nchunks + chunk) * taps * 64;
  T* out = (T*)jb.packed;
  for (int ul = threadIdx.x; ul < taps * 64; ul += 256) {
    const int tap = ul >> 6, lane = ul & 63, rr = lane & 15, g = lane >> 4;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = !jb.transpose ? tile[rr * Lay::RS + g * Lay::G8 + e * taps + tap]
                           : tile[(8 * g + e) * Lay::KS + rr * taps + (taps - 1 - tap)];
    }
    store_vec<T>(out + (ubase + ul) * 8, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pack_tile_kernel(const PackTiles pt) {
  __shared__ float tile[PT_LDS];
  const int b = blockIdx.x;
  int jx = 0;
  while (jx + 1 < pt.count && pt.tile0[jx + 1] <= b) ++jx;
  const unet_pack_job& jb = pt.j[jx];
  const int t = b - pt.tile0[jx];
  if (jb.ksize == 3) pack_tile<T, 9>(jb, t, tile);
  else pack_tile<T, 1>(jb, t, tile);
}

// 16-bit packs of unet_pack_weights (jobs validated by the caller)
int pack_tiles_launch(int dtype, int count, const unet_pack_job* jobs, hipStream_t st) {
  PackTiles pt;
  pt.count = count;
  int tot = 0;
  for (int i = 0; i < count; ++i) {
    pt.j[i] = jobs[i];
    pt.tile0[i] = tot;
    const int rows = jobs[i].transpose ? jobs[i].Cin : jobs[i].Cout, cols = jobs[i].transpose ? jobs[i].Cout : jobs[i].Cin;
    const int rows_pad = round_up(rows, PACK_NPAD);   // = packed_rows() of unet_packed_weight_elems
    tot += rows_pad / 16 * ((cols + 31) / 32);
  }
  pt.tile0[count] = tot;
  if (dtype == UNET_F16)
    hipLaunchKernelGGL(pack_tile_kernel<f16>, dim3(tot), dim3(256), 0, st, pt);
  else
    hipLaunchKernelGGL(pack_tile_kernel<bf16>, dim3(tot), dim3(256), 0, st, pt);
  return check_launch("pack_tiles");
}

}  // namespace unet
