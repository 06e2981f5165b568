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

// z: fp32 NCHW logits [N][C][HW] (labels == nullptr), or labels: int64 [N][HW] predicted classes.
// EXT = 0: confusion[t, p] for 0 <= t, p < K (SegmentationMetrics.update).  EXT = 1: a (K+1) x (K+1)
// matrix whose last row / column collects targets / predictions outside [0, K), so that every pixel is
// counted once — what compute_iou / compute_dice need (metrics.py:183-188, 217-221 count pred == cls
// whatever the target is, and accept C != num_classes logits).
template <int EXT>
__global__ __launch_bounds__(256) void confusion_kernel(long long N, int C, int K, long long HW, const float* z,
                                                        const int64_t* labels, const int64_t* t, long long ignore,
                                                        int has_ignore, unsigned long long* cm) {
  __shared__ unsigned int hist[(CM_MAXK + 1) * (CM_MAXK + 1)];
  const int KW = K + EXT;
  for (int i = threadIdx.x; i < KW * KW; i += blockDim.x) hist[i] = 0u;
  __syncthreads();
  const long long P = N * HW;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < P; q += (long long)gridDim.x * blockDim.x) {
    long long tv = t[q];
    if (has_ignore && tv == ignore) continue;
    long long pv;
    if (labels) {
      pv = labels[q];
    } else {
      const long long n = q / HW, hw = q - n * HW;
      const float* zp = z + n * C * HW + hw;
      float best = zp[0];
      int bi = 0;
      for (int k = 1; k < C; ++k) {
        const float v = zp[(long long)k * HW];
        if (!(best != best) && (v > best || v != v)) { best = v; bi = k; }  // first max; NaN is the max
      }
      pv = bi;
    }
    if (EXT) {
      if (tv < 0 || tv >= K) tv = K;
      if (pv < 0 || pv >= K) pv = K;
      atomicAdd(&hist[tv * KW + pv], 1u);
    } else if (tv >= 0 && tv < K && pv >= 0 && pv < K) {
      atomicAdd(&hist[tv * KW + pv], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < KW * KW; i += blockDim.x)
    if (hist[i]) atomicAdd(&cm[i], (unsigned long long)hist[i]);
}

}  // namespace unet

using namespace unet;

static int launch_confusion(int ext, long long N, int C, int K, long long HW, const float* logits,
                            const int64_t* labels, const int64_t* targets, long long ignore_index, int has_ignore,
                            int64_t* confusion, void* stream) {
  const long long P = N * HW;
  long long blocks = (P + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (ext)
    hipLaunchKernelGGL(confusion_kernel<1>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, N, C, K, HW, logits,
                       labels, targets, ignore_index, has_ignore, (unsigned long long*)confusion);
  else
    hipLaunchKernelGGL(confusion_kernel<0>, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, N, C, K, HW, logits,
                       labels, targets, ignore_index, has_ignore, (unsigned long long*)confusion);
  return check_launch("confusion_matrix");
}

extern "C" int unet_confusion_matrix(long long N, int C, int K, long long HW, const float* logits,
                                     const int64_t* labels, const int64_t* targets, long long ignore_index,
                                     int has_ignore, int64_t* confusion, void* stream) {
  if (N <= 0 || HW <= 0 || K < 1 || K > CM_MAXK || (logits && C < 1) || (!logits && !labels) || !targets ||
      !confusion) {
    set_error("unet_confusion_matrix: bad arguments (1 <= num_classes <= 8, C >= 1)");
    return UNET_ERR_ARG;
  }
  return launch_confusion(0, N, C, K, HW, logits, labels, targets, ignore_index, has_ignore, confusion, stream);
}

extern "C" int unet_confusion_matrix_ext(long long N, int C, int K, long long HW, const float* logits,
                                         const int64_t* labels, const int64_t* targets, int64_t* confusion,
                                         void* stream) {
  if (N <= 0 || HW <= 0 || K < 1 || K > CM_MAXK || (logits && C < 1) || (!logits && !labels) || !targets ||
      !confusion) {
    set_error("unet_confusion_matrix_ext: bad arguments (1 <= num_classes <= 8, C >= 1)");
    return UNET_ERR_ARG;
  }
  return launch_confusion(1, N, C, K, HW, logits, labels, targets, 0, 0, confusion, stream);
}
