// Optimizer step after backward (image_restoration_model.py:313-320; configs/colab/sid_newbp_rgb.yml:69-77):
//   torch.nn.utils.clip_grad_norm_(params, 0.01)  ->  torch.optim.AdamW(lr, betas, wd) step,
// fused over ONE flat fp32 parameter/gradient buffer.  The clip coefficient stays on the device (no host sync).
// grad_scale folds the data-parallel 1/world average into the same pass.
#include <math.h>

#include "nbp_common.h"

using namespace nbp;

namespace {

__global__ void sumsq_kernel(const float* __restrict__ g, long n, double* __restrict__ partial) {
  __shared__ double red[16];
  double s = 0.0;
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const float4 v = ld4(g + 4 * i);
    s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  for (long i = 4 * n4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += (double)g[i] * g[i];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// state[0] = total norm (of grad * grad_scale), state[1] = clip coefficient applied to the gradient
__global__ void clip_coef_kernel(const double* __restrict__ partial, int nb, float grad_scale, float max_norm,
                                 float* __restrict__ state) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += partial[i];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt(s) * grad_scale;
    float coef = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
    if (coef > 1.f) coef = 1.f;
    state[0] = norm;
    state[1] = coef * grad_scale;
  }
}

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long n, const float* __restrict__ state, float lr, float b1, float b2,
                             float eps, float wd, float step_size, float bc2_sqrt, const float* __restrict__ hyper) {
  if (hyper) {  // graph-replayable form: {lr, lr / bc1, sqrt(bc2)} of this step read from device memory
    lr = hyper[0];
    step_size = hyper[1];
    bc2_sqrt = hyper[2];
  }
  const float gs = state[1];
  const float decay = 1.f - lr * wd;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gi = g[i] * gs;
    float pi = p[i] * decay;
    float mi = m[i];
    mi = mi + (1.f - b1) * (gi - mi);
    float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    pi = pi - step_size * (mi / denom);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

inline int grid_for(long total) {
  long g = (total + 255) / 256;
  return (int)(g > 4096 ? 4096 : (g < 1 ? 1 : g));
}

}  // namespace

extern "C" {

size_t nbp_clip_workspace_doubles(long n) { return (size_t)grid_for(n / 4 + 1); }

// Computes state[0..1] = {||grad * grad_scale||, clip coefficient * grad_scale}; max_norm <= 0 disables clipping.
int nbp_grad_clip_coef(const float* grad, long n, float grad_scale, float max_norm, double* ws, float* state,
                       nbp_stream_t s) {
  NBP_REQUIRE(grad && ws && state && n > 0, "nbp_grad_clip_coef: bad args");
  const int g = grid_for(n / 4 + 1);
  sumsq_kernel<<<g, 256, 0, S(s)>>>(grad, n, ws);
  clip_coef_kernel<<<1, 256, 0, S(s)>>>(ws, g, grad_scale, max_norm, state);
  return check_launch("grad_clip_coef");
}

// One AdamW step (torch.optim.AdamW semantics, decoupled weight decay) using gradient * state[1].
int nbp_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n, const float* state,
                   float lr, float beta1, float beta2, float eps, float weight_decay, int step, nbp_stream_t s) {
  NBP_REQUIRE(param && grad && exp_avg && exp_avg_sq && state && n > 0 && step >= 1, "nbp_adamw_step: bad args");
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  adamw_kernel<<<grid_for(n), 256, 0, S(s)>>>(param, grad, exp_avg, exp_avg_sq, n, state, lr, beta1, beta2, eps,
                                              weight_decay, (float)(lr / bc1), (float)sqrt(bc2), nullptr);
  return check_launch("adamw_step");
}

// Same step with {lr, lr / (1 - beta1^t), sqrt(1 - beta2^t)} taken from device memory (hyper[3]), so that one
// captured HIP graph replays every step of a schedule.
int nbp_adamw_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n, const float* state,
                       const float* hyper, float beta1, float beta2, float eps, float weight_decay, nbp_stream_t s) {
  NBP_REQUIRE(param && grad && exp_avg && exp_avg_sq && state && hyper && n > 0, "nbp_adamw_step_dev: bad args");
  adamw_kernel<<<grid_for(n), 256, 0, S(s)>>>(param, grad, exp_avg, exp_avg_sq, n, state, 0.f, beta1, beta2, eps,
                                              weight_decay, 0.f, 1.f, hyper);
  return check_launch("adamw_step_dev");
}

}  // extern "C"
