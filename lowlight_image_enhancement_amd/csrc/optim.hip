// Optimizer step after backward (image_restoration_model.py:308-320; configs/colab/sid_newbp_rgb.yml:69-77):
//   [GradScaler: scale(loss).backward -> unscale_] -> torch.nn.utils.clip_grad_norm_(params, 0.01)
//   -> [scaler.step: skip on inf/nan] AdamW step -> [scaler.update]
// fused over ONE flat fp32 parameter/gradient buffer.  Everything the step decides (clip coefficient, the
// finiteness verdict, the AdamW step count and bias corrections, the dynamic loss scale) stays on the device, so the
// step has no host synchronisation and replays from one captured HIP graph.
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

// One workgroup.  The sum of squares is accumulated in double from fp32 values (|g|^2 <= 1.2e77), so it is finite
// exactly when every gradient element is: the same verdict as GradScaler's found_inf (unscale_ checks every
// element) without a separate pass.
//   state[0] total norm of the averaged, unscaled gradient   state[1] gradient multiplier for AdamW
//   state[2] 1 = skip this step (non-finite gradient)        state[3] lr / (1 - beta1^t)
//   state[4] sqrt(1 - beta2^t)                               state[5] lr        state[6] loss scale of this step
//   ctl[0] AdamW steps taken (t)   ctl[1] GradScaler growth tracker   ctl[2] skipped steps
//   scaler (nullable): {scale, growth_factor, backoff_factor, growth_interval}
__global__ void optim_prepare_kernel(const double* __restrict__ partial, int nb, float grad_scale, float max_norm,
                                     const float* __restrict__ lr_dev, float b1, float b2, float* __restrict__ state,
                                     int* __restrict__ ctl, float* __restrict__ scaler, float* __restrict__ up,
                                     const float* __restrict__ up_base, int n_up) {
  __shared__ double red[16];
  __shared__ float s_new;
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += partial[i];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) {
    const bool finite = isfinite(s);
    const float S = scaler ? scaler[0] : 1.f;
    const float inv_s = scaler ? (float)(1.0 / (double)S) : 1.f;  // GradScaler: scale.double().reciprocal().float()
    float norm = (float)sqrt(s) * grad_scale;
    if (scaler) norm *= inv_s;
    float coef = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
    if (coef > 1.f) coef = 1.f;
    state[0] = norm;
    state[1] = scaler ? coef * grad_scale * inv_s : coef * grad_scale;
    state[2] = finite ? 0.f : 1.f;
    const float lr = lr_dev[0];
    state[5] = lr;
    state[6] = S;
    if (finite) {
      const int t = ctl[0] + 1;
      ctl[0] = t;
      const double bc1 = 1.0 - pow((double)b1, (double)t);
      const double bc2 = 1.0 - pow((double)b2, (double)t);
      state[3] = (float)((double)lr / bc1);
      state[4] = (float)sqrt(bc2);
    } else {
      ctl[2] += 1;
    }
    float S_new = S;
    if (scaler) {  // torch.amp.GradScaler.update (_amp_update_scale_)
      if (!finite) {
        S_new = S * scaler[2];
        ctl[1] = 0;
      } else {
        const int g = ctl[1] + 1;
        if ((float)g >= scaler[3]) {
          S_new = S * scaler[1];
          ctl[1] = 0;
        } else {
          ctl[1] = g;
        }
      }
      scaler[0] = S_new;
    }
    s_new = S_new;
  }
  __syncthreads();
  if (up && up_base)
    for (int i = threadIdx.x; i < n_up; i += blockDim.x) up[i] = up_base[i] * s_new;
}

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long n, const float* __restrict__ state, float b1, float b2,
                             float eps, float wd) {
  if (state[2] != 0.f) return;  // non-finite gradient: parameters and moments untouched (scaler.step skip)
  const float gs = state[1];
  const float step_size = state[3], bc2_sqrt = state[4], lr = state[5];
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

int nbp_optim_prepare(const float* grad, long n, float grad_scale, float max_norm, double* ws, const float* lr,
                      float beta1, float beta2, float* state, int* ctl, float* scaler, float* up, const float* up_base,
                      int n_up, nbp_stream_t s) {
  NBP_REQUIRE(grad && ws && lr && state && ctl && n > 0, "nbp_optim_prepare: bad args");
  NBP_REQUIRE(n_up >= 0 && (n_up == 0 || (up && up_base)), "nbp_optim_prepare: up / up_base needed for n_up > 0");
  const int g = grid_for(n / 4 + 1);
  sumsq_kernel<<<g, 256, 0, S(s)>>>(grad, n, ws);
  optim_prepare_kernel<<<1, 256, 0, S(s)>>>(ws, g, grad_scale, max_norm, lr, beta1, beta2, state, ctl, scaler, up,
                                            up_base, n_up);
  return check_launch("optim_prepare");
}

int nbp_adamw_apply(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, long n, const float* state,
                    float beta1, float beta2, float eps, float weight_decay, nbp_stream_t s) {
  NBP_REQUIRE(param && grad && exp_avg && exp_avg_sq && state && n > 0, "nbp_adamw_apply: bad args");
  adamw_kernel<<<grid_for(n), 256, 0, S(s)>>>(param, grad, exp_avg, exp_avg_sq, n, state, beta1, beta2, eps,
                                              weight_decay);
  return check_launch("adamw_apply");
}

}  // extern "C"
