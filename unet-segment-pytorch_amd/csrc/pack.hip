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

// TAPS a compile-time constant (1 or 9): every index division below is by a constant
template <typename T, int TAPS>
__device__ __forceinline__ void pack_tile(const unet_pack_job& jb, int t, float* tile) {
  constexpr int KC = 32, R = 16, taps = TAPS;
  const int rows = jb.transpose ? jb.Cin : jb.Cout, cols = jb.transpose ? jb.Cout : jb.Cin;
  const int nchunks = (cols + KC - 1) / KC;
  const int chunk = t % nchunks, ntile = t / nchunks;
  const int r0 = ntile * R, c0 = chunk * KC;
  const int n = R * KC * taps;
  for (int i = threadIdx.x; i < n; i += 256) {
    float v = 0.f;
    if (!jb.transpose) {   // tile[rr][kk][tap] <- w[r][c0 + kk][tap]: 16 contiguous KC*taps segments
      const int rr = i / (KC * taps), rem = i - rr * (KC * taps);
      const int r = r0 + rr, cc = c0 + rem / taps;
      if (r < rows && cc < cols) v = jb.w[((long long)r * jb.Cin + c0) * taps + rem];
    } else {               // tile[kk][rr][tap] <- w[c0 + kk][r0 + rr][tap]: 32 contiguous R*taps segments
      const int kk = i / (R * taps), rem = i - kk * (R * taps);
      const int r = r0 + rem / taps, cc = c0 + kk;
      if (r < rows && cc < cols) v = jb.w[((long long)cc * jb.Cin + r0) * taps + rem];
    }
    tile[i] = v;
  }
  __syncthreads();
  // the tile's units: packed order [ntile][chunk][tap][lane][8]; lane holds row rr = lane & 15, k = 8(lane>>4)+e
  const long long ubase = ((long long)ntile * nchunks + chunk) * taps * 64;
  T* out = (T*)jb.packed;
  for (int ul = threadIdx.x; ul < taps * 64; ul += 256) {
    const int tap = ul >> 6, lane = ul & 63, rr = lane & 15;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = 8 * (lane >> 4) + e;
      v[e] = !jb.transpose ? tile[(rr * KC + kk) * taps + tap] : tile[(kk * R + rr) * taps + (taps - 1 - tap)];
    }
    store_vec<T>(out + (ubase + ul) * 8, v);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void pack_tile_kernel(const PackTiles pt) {
  __shared__ float tile[16 * 32 * 9];
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
