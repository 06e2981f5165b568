// torch_ops.cpp — the tensor-shaped entry points of libunet_hip.so registered as PyTorch operators
// (TORCH_LIBRARY(unet_hip, ...)): the form north_star names ("HIP C++ kernels loaded as a torch cpp_extension"),
// for the ops whose arguments are plain tensors — the fused DiceBCE / Dice / BalancedCE loss (reference
// unet/utils/loss.py:18-191) and the segmentation confusion matrix (unet/utils/metrics.py:55-84).  Host code
// only: every op checks its tensors, allocates its outputs and calls the C ABI (include/unet_hip.h) on the
// current HIP stream; the kernels are the ones unet.utils.loss / unet.utils.metrics run through ctypes, so the
// results are bit-identical (tests/test_gpu_torch_ops.py).  The conv / BN / gate stages keep their descriptor
// ABI (a plan of ~150 launches per step is not a sequence of tensor ops).
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <torch/library.h>

#include "unet_hip.h"

namespace {

void* cur_stream() { return static_cast<void*>(c10::hip::getCurrentHIPStream().stream()); }

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, what, " failed: ", unet_last_error()); }

void check_gpu(const at::Tensor& x, const char* name) {
  TORCH_CHECK(x.device().is_cuda(), "unet_hip: ", name, " must be on the ROCm GPU (no CPU fallback)");
}

// predictions (N, K, H, W) fp32 + targets (N, H, W) int64, as DiceBCELoss.forward takes them (loss.py:178)
void check_loss_args(const at::Tensor& z, const at::Tensor& t) {
  check_gpu(z, "predictions");
  check_gpu(t, "targets");
  TORCH_CHECK(z.dim() == 4 && t.dim() == 3 && t.size(0) == z.size(0) && t.size(1) == z.size(2) &&
                  t.size(2) == z.size(3),
              "expected predictions (N, C, H, W) and targets (N, H, W); got ", z.sizes(), " and ", t.sizes());
}

// reduction: 0 mean, 1 sum, 2 none (loss (N, K - ignore_bg) per image and class)
std::tuple<at::Tensor, at::Tensor> loss_fwd(const at::Tensor& z, const at::Tensor& t, double ce_w, double dice_w,
                                            double class_w, double ce_smooth, double dice_smooth, bool ignore_bg,
                                            int64_t reduction) {
  check_loss_args(z, t);
  TORCH_CHECK(reduction >= 0 && reduction <= 2, "reduction must be 0 (mean), 1 (sum) or 2 (none)");
  const auto zc = z.to(at::kFloat).contiguous();
  const auto tc = t.to(at::kLong).contiguous();
  const long long N = zc.size(0), K = zc.size(1), HW = zc.size(2) * zc.size(3);
  const int rows = unet_loss_rows(HW);
  const auto f = zc.options();
  auto part = at::empty({N, rows, 4 + 3 * K}, f);
  void* st = cur_stream();
  check(unet_loss_reduce(N, (int)K, HW, zc.data_ptr<float>(), tc.data_ptr<int64_t>(), part.data_ptr<float>(), st),
        "unet_loss_reduce");
  auto coef = at::empty({N, 2 + 2 * K}, f);
  const long long nd = K - ((ignore_bg && K > 1) ? 1 : 0);
  auto loss = reduction == 2 ? at::empty({N, nd}, f) : at::empty({}, f);
  check(unet_loss_finalize(part.data_ptr<float>(), rows, N, (int)K, (float)ce_w, (float)dice_w, (float)class_w,
                           (float)ce_smooth, (float)dice_smooth, ignore_bg ? 1 : 0, (int)reduction,
                           loss.data_ptr<float>(), coef.data_ptr<float>(), st),
        "unet_loss_finalize");
  return {loss, coef};
}

// dz = gout * d loss / dz (gout: a scalar, or (N, K - ignore_bg) for reduction none)
at::Tensor loss_bwd(const at::Tensor& z, const at::Tensor& t, const at::Tensor& coef, const at::Tensor& gout,
                    int64_t reduction, bool ignore_bg) {
  check_loss_args(z, t);
  check_gpu(coef, "coef");
  check_gpu(gout, "gout");
  const auto zc = z.to(at::kFloat).contiguous();
  const auto tc = t.to(at::kLong).contiguous();
  const auto cc = coef.to(at::kFloat).contiguous();
  const auto go = gout.to(at::kFloat).contiguous();
  const long long N = zc.size(0), K = zc.size(1), HW = zc.size(2) * zc.size(3);
  TORCH_CHECK(cc.numel() == N * (2 + 2 * K), "coef must come from dice_bce_fwd on the same predictions");
  auto dz = at::empty_like(zc);
  check(unet_loss_grad(N, (int)K, HW, zc.data_ptr<float>(), tc.data_ptr<int64_t>(), cc.data_ptr<float>(),
                       go.data_ptr<float>(), reduction == 2 ? 1 : 0, ignore_bg ? 1 : 0, dz.data_ptr<float>(),
                       cur_stream()),
        "unet_loss_grad");
  return dz;
}

// confusion[t][p] (int64 [K][K]) of argmax(logits) against targets; pixels with t == ignore_index
// (ignore_index >= 0) or t / p outside [0, K) are skipped (metrics.py:68-84)
at::Tensor confusion_matrix(const at::Tensor& logits, const at::Tensor& target, int64_t num_classes,
                            int64_t ignore_index) {
  check_gpu(logits, "logits");
  check_gpu(target, "target");
  TORCH_CHECK(logits.dim() == 4 && target.dim() == 3 && target.size(0) == logits.size(0) &&
                  target.size(1) == logits.size(2) && target.size(2) == logits.size(3),
              "expected logits (N, C, H, W) and target (N, H, W); got ", logits.sizes(), " and ", target.sizes());
  TORCH_CHECK(num_classes > 0, "num_classes must be positive");
  const auto zc = logits.to(at::kFloat).contiguous();
  const auto tc = target.to(at::kLong).contiguous();
  auto cm = at::zeros({num_classes, num_classes}, zc.options().dtype(at::kLong));
  check(unet_confusion_matrix(zc.size(0), (int)zc.size(1), (int)num_classes, zc.size(2) * zc.size(3),
                              zc.data_ptr<float>(), nullptr, tc.data_ptr<int64_t>(), ignore_index,
                              ignore_index >= 0 ? 1 : 0, cm.data_ptr<int64_t>(), cur_stream()),
        "unet_confusion_matrix");
  return cm;
}

int64_t abi_version() { return unet_version(); }

}  // namespace

TORCH_LIBRARY(unet_hip, m) {
  m.def("abi_version() -> int", &abi_version);
  m.def("dice_bce_fwd(Tensor z, Tensor t, float ce_w, float dice_w, float class_w, float ce_smooth, "
        "float dice_smooth, bool ignore_bg, int reduction) -> (Tensor loss, Tensor coef)",
        &loss_fwd);
  m.def("dice_bce_bwd(Tensor z, Tensor t, Tensor coef, Tensor gout, int reduction, bool ignore_bg) -> Tensor",
        &loss_bwd);
  m.def("confusion_matrix(Tensor logits, Tensor target, int num_classes, int ignore_index=-1) -> Tensor",
        &confusion_matrix);
}
