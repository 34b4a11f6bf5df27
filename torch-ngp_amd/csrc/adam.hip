// Fused Adam over a flat fp32 parameter vector.
//
// Same update as torch.optim.Adam(betas, eps, weight_decay) used by the
// reference trainer (main_nerf.py:194), one HBM pass: read p, g, m, v; write
// p, m, v (28 B per fp32-grad parameter, 26 B with fp16 grads). The gradient
// may be fp16 (the hash-grid backward's native precision, gridencoder
// grid.py:89) and is scaled by grad_scale (e.g. 1 / GradScaler scale), which
// folds the AMP unscale pass into the same sweep.
#include "ngp_common.h"

#include <cmath>

namespace {

template <typename G>
__global__ void __launch_bounds__(256)
k_adam(float* __restrict__ p, const G* __restrict__ g, float* __restrict__ m,
       float* __restrict__ v, size_t n, float lr_bc1, float beta1, float beta2, float eps,
       float wd, float inv_sqrt_bc2, float grad_scale) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * 4;
    for (size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i0 < n; i0 += stride) {
        if (i0 + 4 <= n) {
            float4 pv = *reinterpret_cast<float4*>(p + i0);
            float4 mv = *reinterpret_cast<float4*>(m + i0);
            float4 vv = *reinterpret_cast<float4*>(v + i0);
            float gv[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) gv[k] = (float)g[i0 + k] * grad_scale;
            float* pp = &pv.x; float* mm = &mv.x; float* vq = &vv.x;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float gk = gv[k];
                if (wd != 0.0f) gk = gk + wd * pp[k];
                mm[k] = mm[k] + (1.0f - beta1) * (gk - mm[k]);
                vq[k] = vq[k] * beta2 + (1.0f - beta2) * gk * gk;
                const float denom = sqrtf(vq[k]) * inv_sqrt_bc2 + eps;
                pp[k] = pp[k] - lr_bc1 * (mm[k] / denom);
            }
            *reinterpret_cast<float4*>(p + i0) = pv;
            *reinterpret_cast<float4*>(m + i0) = mv;
            *reinterpret_cast<float4*>(v + i0) = vv;
        } else {
            for (size_t i = i0; i < n; ++i) {
                float gk = (float)g[i] * grad_scale;
                if (wd != 0.0f) gk = gk + wd * p[i];
                m[i] = m[i] + (1.0f - beta1) * (gk - m[i]);
                v[i] = v[i] * beta2 + (1.0f - beta2) * gk * gk;
                const float denom = sqrtf(v[i]) * inv_sqrt_bc2 + eps;
                p[i] = p[i] - lr_bc1 * (m[i] / denom);
            }
        }
    }
}

}  // namespace

extern "C" int ngp_adam_step(float* params, const void* grads, int32_t grad_dtype, float* exp_avg,
                             float* exp_avg_sq, size_t n, float lr, float beta1, float beta2,
                             float eps, float weight_decay, int32_t step, float grad_scale,
                             void* stream) {
    NGP_REQUIRE(step >= 1, NGP_ERR_ARG, "adam: step must be >= 1");
    if (n == 0) return NGP_OK;
    NGP_REQUIRE(((reinterpret_cast<uintptr_t>(params) | reinterpret_cast<uintptr_t>(exp_avg) |
                  reinterpret_cast<uintptr_t>(exp_avg_sq)) & 15) == 0,
                NGP_ERR_ARG, "adam: state tensors must be 16-byte aligned");
    const double bc1 = 1.0 - std::pow((double)beta1, step);
    const double bc2 = 1.0 - std::pow((double)beta2, step);
    const float lr_bc1 = (float)(lr / bc1);
    const float inv_sqrt_bc2 = (float)(1.0 / std::sqrt(bc2));
    size_t blocks = (n / 4 + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipStream_t st = ngp_stream(stream);
    switch (grad_dtype) {
        case NGP_DTYPE_F32:
            k_adam<float><<<(uint32_t)blocks, 256, 0, st>>>(params, (const float*)grads, exp_avg, exp_avg_sq, n, lr_bc1, beta1, beta2, eps, weight_decay, inv_sqrt_bc2, grad_scale);
            break;
        case NGP_DTYPE_F16:
            k_adam<ngp_half><<<(uint32_t)blocks, 256, 0, st>>>(params, (const ngp_half*)grads, exp_avg, exp_avg_sq, n, lr_bc1, beta1, beta2, eps, weight_decay, inv_sqrt_bc2, grad_scale);
            break;
        default: return ngp_set_error(NGP_ERR_ARG, "adam: grads must be float32 or float16");
    }
    return ngp_check_launch("adam_step");
}
