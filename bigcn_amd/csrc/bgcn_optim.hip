// Fused multi-tensor Adam (one launch for every parameter of the model).
//
// Replaces the optimiser step of the reference's training loop:
//   torch.optim.Adam([{base}, {BU conv1, lr/5}, {BU conv2, lr/5}], lr, weight_decay)
//   (model/Twitter/BiGCN_Twitter.py:146-153, step at :189)
// with torch's Adam semantics (amsgrad = False, maximize = False, weight decay added to
// the gradient = L2):
//   g = grad * grad_scale + wd * p ; m = lerp(m, g, 1 - b1) ; v = b2 v + (1 - b2) g^2
//   p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// grad_scale folds the 1/world of the data-parallel mean into the step, so the reduced
// flat gradient bucket is consumed in place.
#include "bgcn_common.h"

namespace bgcn {
namespace {

constexpr int kChunkElems = 256 * 4 * 4;  // elements per block (256 threads x 4 float4)

__global__ __launch_bounds__(256) void k_adam(bgcn_adam_args a) {
  // locate this block's tensor (at most BGCN_ADAM_MAX_TENSORS, uniform scan)
  int k = 0;
  while (k + 1 < a.count && int64_t(blockIdx.x) >= a.block_start[k + 1]) ++k;
  const bgcn_adam_tensor& T = a.t[k];
  const int64_t base = (int64_t(blockIdx.x) - a.block_start[k]) * kChunkElems;
  const float b1 = a.beta1, b2 = a.beta2, wd = a.weight_decay, eps = a.eps;
  const float step = T.lr / a.bias_correction1;
  const float inv_bc2 = 1.0f / a.bias_correction2_sqrt;
  for (int u = 0; u < 4; ++u) {
    const int64_t e0 = base + (int64_t(u) * 256 + threadIdx.x) * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t e = e0 + j;
      if (e >= T.numel) break;
      float p = T.param[e];
      const float g = T.grad[e] * a.grad_scale + wd * p;
      float m = T.exp_avg[e];
      float v = T.exp_avg_sq[e];
      m = fmaf(1.0f - b1, g - m, m);          // exp_avg.lerp_(grad, 1 - beta1)
      v = fmaf(1.0f - b2, g * g, v * b2);     // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
      const float denom = sqrtf(v) * inv_bc2 + eps;
      p = p - step * (m / denom);
      T.param[e] = p;
      T.exp_avg[e] = m;
      T.exp_avg_sq[e] = v;
    }
  }
}

}  // namespace
}  // namespace bgcn

extern "C" int bgcn_adam_step(const bgcn_adam_args* args, bgcn_stream_t stream) {
  using namespace bgcn;
  if (!args || args->count < 1 || args->count > BGCN_ADAM_MAX_TENSORS)
    return fail(BGCN_EINVAL, "adam: 1..BGCN_ADAM_MAX_TENSORS tensors");
  bgcn_adam_args a = *args;
  int64_t blocks = 0;
  for (int k = 0; k < a.count; ++k) {
    const bgcn_adam_tensor& T = a.t[k];
    if (T.numel < 0 || (T.numel > 0 && (!T.param || !T.grad || !T.exp_avg || !T.exp_avg_sq)))
      return fail(BGCN_EINVAL, "adam: bad tensor");
    a.block_start[k] = blocks;
    blocks += (T.numel + kChunkElems - 1) / kChunkElems;
  }
  if (blocks == 0) return BGCN_OK;
  hipLaunchKernelGGL(k_adam, dim3(unsigned(blocks)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  BGCN_CHECK_LAUNCH();
  return BGCN_OK;
}
