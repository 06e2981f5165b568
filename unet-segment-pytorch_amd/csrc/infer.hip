// infer.hip — the device side of the reference's data path around the network:
//
//  * input pipeline (rows f3): what `LungTumorDataset.__getitem__` + `apply_basic_transforms` do per slice
//    on the CPU (unet/data/dataset.py:133-171, unet/data/augmentations.py:119-171), for a batch of
//    decoded 8-bit slices already on the device:
//      - the float round trip u8 -> /255 (fp32) -> *255 -> uint8 truncation of augmentations.py:150;
//      - PIL `Image.resize(BILINEAR)` (8-bit fixed-point separable resampling, horizontal then vertical;
//        the coefficient tables are computed on the host exactly as Pillow does) for images, and PIL
//        NEAREST for masks (augmentations.py:153-154);
//      - the per-image horizontal flip (augmentations.py:161-163), /255 and (x - mean) / std (:166), and
//        the mask binarisation (mask > 127, dataset.py:148-149) to int64;
//  * inference post-processing (row f1): `postprocess_mask` of scripts/predict.py:138-165 — softmax over
//    the classes, `p[cls] > threshold` -> 255 / 0, PIL NEAREST resize to the original size.
// All integer / byte work: bit-exact with Pillow and numpy (tests/test_gpu_pipeline.py).
#include "common.h"

namespace unet {

__device__ __forceinline__ int clip8(int v) {  // Pillow Resample.c clip8 after the >> PRECISION_BITS shift
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}
constexpr int PRECISION_BITS = 32 - 8 - 2;

// the dataset's float round trip: uint8(float32(float32(u) / 255) * 255) (truncation)
__device__ __forceinline__ unsigned char roundtrip_u8(unsigned char u) {
  const float v = __fdiv_rn((float)u, 255.0f);
  return (unsigned char)(int)__fmul_rn(v, 255.0f);
}

// horizontal pass: out[n][y][x] = clip8((1 << 21) + sum_k in[n][y][xmin + k] * kk[x][k] >> 22)
__global__ void resample_h_kernel(long long N, int H, int inW, int outW, const unsigned char* in, int roundtrip,
                                  const int* bounds, const int* kk, int ksize, unsigned char* out) {
  const long long total = N * H * outW;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % outW);
    const long long row = e / outW;
    const unsigned char* src = in + row * inW;
    const int xmin = bounds[2 * x], xn = bounds[2 * x + 1];
    const int* k = kk + (long long)x * ksize;
    int ss = 1 << (PRECISION_BITS - 1);
    for (int i = 0; i < xn; ++i) {
      const unsigned char u = src[xmin + i];
      ss += (int)(roundtrip ? roundtrip_u8(u) : u) * k[i];
    }
    out[e] = (unsigned char)clip8(ss >> PRECISION_BITS);
  }
}

// vertical pass: out[n][y][x] = clip8(... sum_k in[n][ymin + k][x] * kk[y][k] ...)
__global__ void resample_v_kernel(long long N, int inH, int W, int outH, const unsigned char* in, int roundtrip,
                                  const int* bounds, const int* kk, int ksize, unsigned char* out) {
  const long long total = N * outH * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % W);
    const long long t = e / W;
    const int y = (int)(t % outH);
    const long long n = t / outH;
    const int ymin = bounds[2 * y], yn = bounds[2 * y + 1];
    const int* k = kk + (long long)y * ksize;
    const unsigned char* src = in + (n * inH + ymin) * (long long)W + x;
    int ss = 1 << (PRECISION_BITS - 1);
    for (int i = 0; i < yn; ++i) {
      const unsigned char u = src[(long long)i * W];
      ss += (int)(roundtrip ? roundtrip_u8(u) : u) * k[i];
    }
    out[e] = (unsigned char)clip8(ss >> PRECISION_BITS);
  }
}

// PIL NEAREST source indices come from host tables (ytab[H], xtab[W]): Pillow walks the source coordinate
// by repeated double additions (ImagingScaleAffine), which floor((o + 0.5) * in / out) does not reproduce.
// mask: (m > 127) -> NEAREST resize -> optional horizontal flip -> int64
__global__ void mask_finish_kernel(long long N, int inH, int inW, const unsigned char* m, int H, int W,
                                   const int* ytab, const int* xtab, const unsigned char* flip, int64_t* out) {
  const long long total = N * H * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % W);
    const long long t = e / W;
    const int y = (int)(t % H);
    const long long n = t / H;
    const int xs = (flip && flip[n]) ? W - 1 - x : x;
    out[e] = m[(n * inH + ytab[y]) * (long long)inW + xtab[xs]] > 127 ? 1 : 0;
  }
}

// image: optional round trip (when no resize pass ran), optional flip, /255, (v - mean) / std -> fp32 NCHW
__global__ void image_finish_kernel(long long N, int H, int W, const unsigned char* r, int roundtrip,
                                    const unsigned char* flip, float mean, float stdv, float* out) {
  const long long total = N * H * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % W);
    const long long t = e / W;
    const long long n = t / H;
    const int xs = (flip && flip[n]) ? W - 1 - x : x;
    unsigned char u = r[t * W + xs];
    if (roundtrip) u = roundtrip_u8(u);
    const float v = __fdiv_rn((float)u, 255.0f);
    out[e] = __fdiv_rn(__fsub_rn(v, mean), stdv);
  }
}

// predict.py:138-165: softmax over K classes, p[cls] > threshold -> 255, NEAREST resize to (outH, outW)
__global__ void postprocess_mask_kernel(long long N, int K, int H, int W, const float* z, int cls, float thr, int outH,
                                        int outW, const int* ytab, const int* xtab, unsigned char* out) {
  const long long total = N * outH * outW;
  const long long HW = (long long)H * W;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const int x = (int)(e % outW);
    const long long t = e / outW;
    const int y = (int)(t % outH);
    const long long n = t / outH;
    const float* zp = z + n * K * HW + (long long)ytab[y] * W + xtab[x];
    float m = -INFINITY;
    for (int k = 0; k < K; ++k) m = fmaxf(m, zp[k * HW]);
    float se = 0.f, pc = 0.f;
    for (int k = 0; k < K; ++k) {
      const float ek = expf(zp[k * HW] - m);
      se += ek;
      if (k == cls) pc = ek;
    }
    out[e] = (pc / se) > thr ? 255 : 0;
  }
}

static int grid_for(long long total) {
  long long b = (total + 255) / 256;
  if (b > 16384) b = 16384;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace unet

using namespace unet;

extern "C" {

int unet_resample_u8(int axis, long long N, int inH, int inW, int out_len, const uint8_t* in, int roundtrip,
                     const int32_t* bounds, const int32_t* coeffs, int ksize, uint8_t* out, void* stream) {
  if (N <= 0 || inH <= 0 || inW <= 0 || out_len <= 0 || !in || !bounds || !coeffs || !out || ksize <= 0) {
    set_error("unet_resample_u8: bad arguments");
    return UNET_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  if (axis == 1) {
    const long long total = N * inH * (long long)out_len;
    hipLaunchKernelGGL(resample_h_kernel, dim3(grid_for(total)), dim3(256), 0, st, N, inH, inW, out_len, in, roundtrip,
                       bounds, coeffs, ksize, out);
  } else {
    const long long total = N * (long long)out_len * inW;
    hipLaunchKernelGGL(resample_v_kernel, dim3(grid_for(total)), dim3(256), 0, st, N, inH, inW, out_len, in, roundtrip,
                       bounds, coeffs, ksize, out);
  }
  return check_launch("resample_u8");
}

int unet_slice_finish(long long N, int H, int W, const uint8_t* img, int roundtrip, int mask_h, int mask_w,
                      const uint8_t* mask, const int32_t* ytab, const int32_t* xtab, const uint8_t* flip, float mean,
                      float stdv, float* out_img, int64_t* out_mask, void* stream) {
  if (N <= 0 || H <= 0 || W <= 0 || !img || !out_img ||
      (mask && (!out_mask || mask_h <= 0 || mask_w <= 0 || !ytab || !xtab))) {
    set_error("unet_slice_finish: bad arguments");
    return UNET_ERR_ARG;
  }
  hipStream_t st = (hipStream_t)stream;
  const long long total = N * (long long)H * W;
  hipLaunchKernelGGL(image_finish_kernel, dim3(grid_for(total)), dim3(256), 0, st, N, H, W, img, roundtrip, flip, mean,
                     stdv, out_img);
  if (int rc = check_launch("image_finish")) return rc;
  if (mask)
    hipLaunchKernelGGL(mask_finish_kernel, dim3(grid_for(total)), dim3(256), 0, st, N, mask_h, mask_w, mask, H, W, ytab,
                       xtab, flip, out_mask);
  return check_launch("mask_finish");
}

int unet_postprocess_mask(long long N, int K, int H, int W, const float* logits, int cls, float threshold, int outH,
                          int outW, const int32_t* ytab, const int32_t* xtab, uint8_t* out, void* stream) {
  if (N <= 0 || K < 1 || cls < 0 || cls >= K || H <= 0 || W <= 0 || outH <= 0 || outW <= 0 || !logits || !out ||
      !ytab || !xtab) {
    set_error("unet_postprocess_mask: bad arguments");
    return UNET_ERR_ARG;
  }
  const long long total = N * (long long)outH * outW;
  hipLaunchKernelGGL(postprocess_mask_kernel, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, N, K, H, W,
                     logits, cls, threshold, outH, outW, ytab, xtab, out);
  return check_launch("postprocess_mask");
}

}  // extern "C"
