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

constexpr int kChunkElems = 256 * 4;  // elements per block (256 threads x one float4)

struct AdamConst {
  float b1, b2, wd, eps, step, inv_bc2, gs;
};

__device__ __forceinline__ void adam_elem(float& p, float gr, float& m, float& v,
                                          const AdamConst& c) {
  const float g = gr * c.gs + c.wd * p;
  m = fmaf(1.0f - c.b1, g - m, m);            // exp_avg.lerp_(grad, 1 - beta1)
  v = fmaf(1.0f - c.b2, g * g, v * c.b2);     // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
  const float denom = sqrtf(v) * c.inv_bc2 + c.eps;
  p = p - c.step * (m / denom);
}

__global__ __launch_bounds__(256) void k_adam(bgcn_adam_args a) {
  if (a.skip_flag && *a.skip_flag != 0.0f) return;   // invalid step (any rank): no update
  // locate this block's tensor (at most BGCN_ADAM_MAX_TENSORS, uniform scan)
  int k = 0;
  while (k + 1 < a.count && int64_t(blockIdx.x) >= a.block_start[k + 1]) ++k;
  const bgcn_adam_tensor& T = a.t[k];
  const AdamConst c{a.beta1, a.beta2, a.weight_decay, a.eps, T.lr / a.bias_correction1,
                    1.0f / a.bias_correction2_sqrt, a.grad_scale};
  const int64_t e0 = (int64_t(blockIdx.x) - a.block_start[k]) * kChunkElems + threadIdx.x * 4;
  const bool vec = ((reinterpret_cast<uintptr_t>(T.param) | reinterpret_cast<uintptr_t>(T.grad) |
                     reinterpret_cast<uintptr_t>(T.exp_avg) |
                     reinterpret_cast<uintptr_t>(T.exp_avg_sq)) & 15u) == 0;
  if (vec && e0 + 4 <= T.numel) {
    float4 p = ld4(T.param + e0), g = ld4(T.grad + e0);
    float4 m = ld4(T.exp_avg + e0), v = ld4(T.exp_avg_sq + e0);
    adam_elem(p.x, g.x, m.x, v.x, c);
    adam_elem(p.y, g.y, m.y, v.y, c);
    adam_elem(p.z, g.z, m.z, v.z, c);
    adam_elem(p.w, g.w, m.w, v.w, c);
    st4(T.param + e0, p);
    st4(T.exp_avg + e0, m);
    st4(T.exp_avg_sq + e0, v);
    return;
  }
  for (int64_t e = e0; e < e0 + 4 && e < T.numel; ++e) {
    float p = T.param[e], m = T.exp_avg[e], v = T.exp_avg_sq[e];
    adam_elem(p, T.grad[e], m, v, c);
    T.param[e] = p;
    T.exp_avg[e] = m;
    T.exp_avg_sq[e] = v;
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
