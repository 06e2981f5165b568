// metrics.hip — on-device confusion matrix for segmentation metrics.
//
// Reference: SegmentationMetrics.update, unet/utils/metrics.py:55-84 — argmax over the class logits
// (dim 1, first maximum wins, NaN counts as the maximum like torch.argmax), then
// confusion[t, p] += 1 for every pixel with 0 <= t, p < K and t != ignore_index.  The reference runs a
// per-pixel Python loop on the host (0.24 s / 512^2 image); here one streaming pass over the logits
// (HBM-bound: 4·K bytes of logits + 8 bytes of target per pixel) with a per-workgroup LDS histogram
// and 64-bit integer atomics into the K x K matrix — integer arithmetic, so exact and order-independent.
#include "common.h"

namespace unet {

constexpr int CM_MAXK = 8;

// z: fp32 NCHW logits [N][K][HW] (labels == nullptr), or labels: int64 [N][HW] predicted classes
__global__ __launch_bounds__(256) void confusion_kernel(long long N, int K, long long HW, const float* z,
                                                        const int64_t* labels, const int64_t* t, long long ignore,
                                                        int has_ignore, unsigned long long* cm) {
  __shared__ unsigned int hist[CM_MAXK * CM_MAXK];
  for (int i = threadIdx.x; i < K * K; i += blockDim.x) hist[i] = 0u;
  __syncthreads();
  const long long P = N * HW;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < P; q += (long long)gridDim.x * blockDim.x) {
    const long long tv = t[q];
    if (has_ignore && tv == ignore) continue;
    long long pv;
    if (labels) {
      pv = labels[q];
    } else {
      const long long n = q / HW, hw = q - n * HW;
      const float* zp = z + n * K * HW + hw;
      float best = zp[0];
      int bi = 0;
      for (int k = 1; k < K; ++k) {
        const float v = zp[(long long)k * HW];
        if (!(best != best) && (v > best || v != v)) { best = v; bi = k; }  // first max; NaN is the max
      }
      pv = bi;
    }
    if (tv >= 0 && tv < K && pv >= 0 && pv < K) atomicAdd(&hist[tv * K + pv], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < K * K; i += blockDim.x)
    if (hist[i]) atomicAdd(&cm[i], (unsigned long long)hist[i]);
}

}  // namespace unet

using namespace unet;

extern "C" int unet_confusion_matrix(long long N, int K, long long HW, const float* logits, const int64_t* labels,
                                     const int64_t* targets, long long ignore_index, int has_ignore,
                                     int64_t* confusion, void* stream) {
  if (N <= 0 || HW <= 0 || K < 1 || K > CM_MAXK || (!logits && !labels) || !targets || !confusion) {
    set_error("unet_confusion_matrix: bad arguments (1 <= num_classes <= 8)");
    return UNET_ERR_ARG;
  }
  const long long P = N * HW;
  long long blocks = (P + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(confusion_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, N, K, HW, logits, labels,
                     targets, ignore_index, has_ignore, (unsigned long long*)confusion);
  return check_launch("confusion_matrix");
}
