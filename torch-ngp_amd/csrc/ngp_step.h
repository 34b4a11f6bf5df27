// Device step state of the fused train step and its GradScaler / LR / loss
// bookkeeping (shared by nerf_fused.hip and raymarching.hip, whose march
// emit launch can carry the bookkeeping of a deferred optimizer update).
#pragma once
#include "ngp_common.h"

namespace ngp_step {

// ---- device step state ------------------------------------------------------
struct StepState {
    float scale;           // GradScaler scale
    float loss_sum;        // sum over rays of the per-ray MSE (this step)
    float last_loss;       // mean loss of the last finished step
    float pad;
    int32_t growth_tracker;
    int32_t found_inf;     // bit 0 inf/nan in the grads, bit 1 gradient exchange overflow (update skipped)
    int32_t adam_step;     // optimizer steps taken (skipped steps excluded)
    int32_t epoch;         // LambdaLR epoch (every step)
    int32_t iter;          // finished steps (k_step_end)
    int32_t draw;          // batches drawn by the sampler (k_lego_rays)
    int32_t lego_done;     // k_lego_rays' finished-block count (last block bumps draw)
    int32_t local_inf;     // data parallel: this rank's own grads held an inf/nan (k_guard_*)
    int32_t end_pending;   // an optimizer update whose GradScaler/LR bookkeeping is deferred to k_step_head
    int32_t reserved[3];
};


// ---- Adam (torch.optim.Adam, weight_decay 0) on an unscaled fp16 grad -------
// Shared by the optimizer sweeps (ngp_head.h).
struct AdamConsts {
    float inv_scale;     // 1 / GradScaler scale (x grad_mult)
    float step_size;     // lr_t / bias_correction1
    float inv_bc2_sqrt;  // 1 / sqrt(bias_correction2)
    bool inv_bad;        // 1 / scale is not finite: GradScaler skips
};
// step = adam_step + 1, LambdaLR lr = base_lr * 0.1 ** min(epoch / iters, 1)
NGP_DEV AdamConsts adam_consts(const StepState* __restrict__ st, float base_lr, float beta1, float beta2,
                               int32_t iters, float grad_mult) {
    AdamConsts c;
    // GradScaler checks the UNSCALED grads: once the scale has backed off so far
    // that 1/scale is inf, every element (0 * inf = NaN) is non-finite and the
    // step is skipped, which the checks of the scaled fp16 grads cannot see
    c.inv_scale = (float)(1.0 / (double)st->scale) * grad_mult;
    c.inv_bad = !__builtin_isfinite(c.inv_scale);
    const int32_t step = st->adam_step + 1;
    const double lr = (double)base_lr * pow(0.1, fmin((double)st->epoch / (double)iters, 1.0));
    const double bc1 = 1.0 - pow((double)beta1, step);
    const double bc2 = 1.0 - pow((double)beta2, step);
    c.step_size = (float)(lr / bc1);
    c.inv_bc2_sqrt = 1.0f / (float)sqrt(bc2);
    return c;
}
NGP_DEV void adam_update(float& p, float& m, float& v, float gh, const AdamConsts& c, float beta1, float beta2,
                         float eps) {
    const float gk = gh * c.inv_scale;
    m = m + (1.0f - beta1) * (gk - m);
    v = v * beta2 + (1.0f - beta2) * gk * gk;
    const float denom = sqrtf(v) * c.inv_bc2_sqrt + eps;
    p = p - c.step_size * (m / denom);
}

struct ScalerArgs {
    float growth_factor, backoff_factor;
    int32_t growth_interval, enabled;
    float inv_n;
};

// GradScaler.update, LambdaLR epoch, Adam step count, loss bookkeeping (mean
// of the per-ray losses, fixed-order tree sum); also records this step's
// sample count into step_counter[iter % 16]
NGP_DEV void step_end_block(StepState* __restrict__ st, const ScalerArgs& sa, const int32_t* __restrict__ counter,
                            int32_t* __restrict__ step_counter, const float* __restrict__ loss_ray, uint32_t n_rays) {
    __shared__ float part[256];
    float acc = 0.0f;
    if (loss_ray && n_rays) {
        // 16 loads in flight per thread, then the adds in the original order
        // (one dependent round trip per load made the flush's standalone
        // k_step_end ~8 us)
        constexpr uint32_t U = 16;
        for (uint32_t base = threadIdx.x; base < n_rays; base += 256 * U) {
            float v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = loss_ray[min(base + u * 256, n_rays - 1)];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                if (base + u * 256 < n_rays) acc += v[u];
        }
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    if (loss_ray) st->loss_sum = part[0];
    // found_inf bit 0: an inf/nan (GradScaler backs off); bit 1: the replicated
    // step's gradient exchange overflowed its lists (the update is skipped on
    // every rank, the scale is left alone; csrc/exchange.hip)
    const bool skip = st->found_inf != 0;
    const bool inf = (st->found_inf & 1) != 0;
    if (sa.enabled) {
        if (inf) {
            st->scale *= sa.backoff_factor;
            st->growth_tracker = 0;
        } else if (!skip && ++st->growth_tracker == sa.growth_interval) {
            st->scale *= sa.growth_factor;
            st->growth_tracker = 0;
        }
    }
    if (!skip) st->adam_step += 1;
    st->epoch += 1;
    if (step_counter) {
        const int slot = st->iter % 16;
        step_counter[slot * 2] = counter[0];
        step_counter[slot * 2 + 1] = counter[1];
    }
    st->iter += 1;
    st->last_loss = st->loss_sum * sa.inv_n;
    st->loss_sum = 0.0f;
    st->found_inf = 0;
    st->end_pending = 0;
}


}  // namespace ngp_step
