// Fused NeRF train step (DESIGN.md "fused step"): the elementwise glue of the
// reference step (nerf/utils.py train_step :453-497, renderer.run_cuda
// :257-375, network_ff.forward :69-105, GradScaler + Adam) folded into a
// handful of kernels around the hot-path ops, so the whole step is ~22
// launches instead of ~150. Each kernel reproduces the reference's float
// operations (including torch's scalar-division-as-reciprocal-multiply and
// autocast casts) so the fused step and the autograd step agree to fp16/fp32
// rounding (tests/test_gpu_fused.py).
//
//   k_lego_rays       synthetic Lego batch: pose + pixels (counter-based RNG),
//                     rays (get_rays :52-136), analytic RGBA target, random
//                     background, march noise, near/far (raymarching.cu:91-145)
//   k_glue_fwd        sigma = ds * exp(h0); color_in = [half(SH4(d)) | h1..15 | 0]
//   k_composite_loss  per ray (one wave, shuffle scans): composite forward,
//                     background blend, MSE, d loss / d image (AMP-scaled),
//                     composite backward, cast/sigmoid/trunc_exp backward ->
//                     fp16 MLP-output grads
//   k_glue_bwd        geo-feature grads (color MLP grad_inputs 16..30) -> h1..15
//   k_nonfinite       GradScaler's inf/nan check over the fp16 grads
//   k_adam_multi      Adam over all parameter tensors, unscaled fp16 grads,
//                     skip on inf, device-side lr schedule; zeroes the grads
//   k_step_end        GradScaler.update, counters, loss
#include "ffmlp_pack.h"
#include "ngp_common.h"
#include "ngp_dpp.h"
#include "ngp_step.h"
#include "ngp_head.h"
#include "sh_basis.h"

#include <algorithm>
#include <cfloat>

namespace {

using ngp_step::ScalerArgs;
using ngp_step::StepState;
using ngp_step::step_end_block;
using namespace ngp_head;

NGP_DEV uint32_t clip_rows(uint32_t B, const int32_t* count) {
    if (!count) return B;
    const int32_t c = *count;
    return c <= 0 ? 0u : min(B, (uint32_t)c);
}

__global__ void __launch_bounds__(256)
k_lego_rays(const float* __restrict__ poses, LegoScene sc, uint32_t N, StepState* __restrict__ st, LegoOut out) {
    lego_rays_block(blockIdx.x, gridDim.x, poses, sc, N, st, out);
}

// ---- network glue -------------------------------------------------------------
// h: sigma-MLP output [B, 16] fp16 (col 0 = log density, 1..15 = geo features)
__global__ void __launch_bounds__(256)
k_glue_fwd(const ngp_half* __restrict__ h, const float* __restrict__ dirs, float density_scale,
           float* __restrict__ sigma, ngp_half* __restrict__ color_in, uint32_t B,
           const int32_t* __restrict__ count) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= clip_rows(B, count)) return;
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    const half8* hr = reinterpret_cast<const half8*>(h + (size_t)b * 16);
    const half8 h0 = hr[0], h1 = hr[1];
    // trunc_exp forward (activation.py: exp of the fp32-cast input), * density_scale
    sigma[b] = density_scale * expf((float)h0[0]);
    // SH degree 4 of the (unnormalised, size 1) direction, fp32 -> half
    float sh[16];
    ngp_sh::sh_basis<float>(dirs[b * 3], dirs[b * 3 + 1], dirs[b * 3 + 2], 4u,
                            [&](uint32_t k, float v) { sh[k] = v; });
    half8 o0, o1, o2, o3;
#pragma unroll
    for (int k = 0; k < 8; ++k) { o0[k] = ngp_f2h(sh[k]); o1[k] = ngp_f2h(sh[8 + k]); }
    // geo features h[1..15], then the zero pad column
#pragma unroll
    for (int k = 0; k < 7; ++k) o2[k] = h0[k + 1];
    o2[7] = h1[0];
#pragma unroll
    for (int k = 0; k < 7; ++k) o3[k] = h1[k + 1];
    o3[7] = (ngp_half)0.0f;
    half8* out = reinterpret_cast<half8*>(color_in + (size_t)b * 32);
    out[0] = o0; out[1] = o1; out[2] = o2; out[3] = o3;
}

// geo-feature grads: grad_h[b, 1..15] = grad_color_in[b, 16..30] (col 0 was
// written by k_composite_loss)
__global__ void __launch_bounds__(256)
k_glue_bwd(const ngp_half* __restrict__ grad_color_in, ngp_half* __restrict__ grad_h, uint32_t B,
           const int32_t* __restrict__ count) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= clip_rows(B, count)) return;
    const ngp_half* src = grad_color_in + (size_t)b * 32 + 16;
    ngp_half* dst = grad_h + (size_t)b * 16;
#pragma unroll
    for (int k = 1; k < 16; ++k) dst[k] = src[k - 1];
}

// ---- composite + loss + backward (one wave per ray) ---------------------------
// The transmittance recurrence T_{i+1} = T_i (1 - alpha_i) with
// 1 - alpha_i = exp(-sigma_i delta_i) is T_i = exp(-sum_{j<i} sigma_j delta_j),
// a prefix sum: each wave composites its ray 64 samples at a time with
// shuffle scans instead of a serial loop (whose length, up to several hundred
// samples on rays crossing the Lego body, set the kernel time). The result
// equals the sequential composite to float rounding (~1e-6 relative); the
// early stop is the first sample whose T falls below T_thresh, as in
// raymarching.cu:551/:665. The reference-API composite_rays_train keeps the
// bit-exact serial form.
constexpr uint32_t kLossWaves = 4;

// torch.sigmoid on a half tensor: fp32 math, half result
NGP_DEV float sigmoid_h(ngp_half x) { return (float)(ngp_half)(1.0f / (1.0f + expf(-(float)x))); }

// wave-wide prefix sums / sums on DPP lane moves (ngp_dpp.h); every lane of
// the wave is active wherever these are called
NGP_DEV float scan_incl(float v, uint32_t) { return ngp_dpp::scan_incl(v); }
NGP_DEV float lane63(float v) { return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63)); }
NGP_DEV float wave_sum(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ngp_dpp::scan_incl(v)), 63));
}

struct LossArgs {
    float T_thresh, density_scale, inv_n, inv_c;  // inv_n = 1/N, inv_c = 1/3 (torch mean backward)
    uint32_t gt_channels;                         // 4: RGBA with random background, 3: RGB on white
};

// One 64-sample chunk of a ray: per-lane sample data and the scanned quantities.
struct Chunk {
    bool ok, active;                 // lane holds a sample / sample is before the early stop
    float d0, c0, c1, c2, w, Tafter, t;
};

// The loaded rows of one chunk (what the scans and the backward read).
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
struct Raw {
    float sg, h0;
    float2 dd;
    half4 co;
};

NGP_DEV Raw load_raw(const float* __restrict__ sigma, const ngp_half* __restrict__ color_out,
                     const float* __restrict__ deltas, const ngp_half* __restrict__ h_sigma, uint32_t offset,
                     uint32_t base, uint32_t num_steps, uint32_t lane) {
    // unconditional loads (lanes past the ray read row 0 and drop the value):
    // a load under a divergent branch makes the compiler wait for it on the spot
    const uint32_t ic = base + lane < num_steps ? offset + base + lane : 0u;
    Raw r;
    r.sg = sigma[ic];
    r.dd = *reinterpret_cast<const float2*>(deltas + (size_t)ic * 2);
    r.co = *reinterpret_cast<const half4*>(color_out + (size_t)ic * 16);
    r.h0 = (float)h_sigma[(size_t)ic * 16];
    return r;
}

NGP_DEV Chunk scan_chunk(const Raw& rw, uint32_t base, uint32_t num_steps, uint32_t lane, float& S, float& tacc,
                         float T_thresh, bool& stop) {
    Chunk c;
    c.ok = base + lane < num_steps;
    const float sgl = rw.sg;
    const float2 ddl = rw.dd;
    const half4 co = rw.co;
    const float sg = c.ok ? sgl : 0.0f;
    c.d0 = c.ok ? ddl.x : 0.0f;
    const float d1 = c.ok ? ddl.y : 0.0f;
    c.c0 = c.ok ? sigmoid_h(co[0]) : 0.0f;
    c.c1 = c.ok ? sigmoid_h(co[1]) : 0.0f;
    c.c2 = c.ok ? sigmoid_h(co[2]) : 0.0f;
    const float sd = sg * c.d0;
    const float incl = scan_incl(sd, lane);
    // the exclusive prefix is the previous lane's inclusive one, NOT incl - sd:
    // once the density is large (sigma * delta >> the prefix, or inf) that
    // difference cancels to garbage (inf - inf = NaN), where the reference's
    // serial T *= 1 - alpha stays exact
    const float excl = __builtin_bit_cast(float, ngp_dpp::prev_lane(__builtin_bit_cast(uint32_t, incl)));  // lane 0: 0
    const float alpha = 1.0f - expf(-sd);
    const float Tbefore = expf(-(S + excl));
    c.Tafter = expf(-(S + incl));
    c.w = alpha * Tbefore;
    c.t = tacc + scan_incl(d1, lane);
    const uint64_t below = __ballot(c.ok && c.Tafter < T_thresh);
    const uint32_t last = below ? (uint32_t)__ffsll((unsigned long long)below) - 1 : 63u;
    c.active = c.ok && lane <= last;
    if (!c.active) c.w = 0.0f;
    stop = below != 0;
    S += lane63(incl);
    tacc = lane63(c.t);
    return c;
}

// Chunks of a ray whose rows are requested together, before the first scan
// (and kept for the backward): the serial per-chunk round trips of a long ray
// set the kernel's time (a ray of 256 samples took 4 dependent loads in the
// forward and 3 more in the backward).
constexpr uint32_t kLossPre = 4;

__global__ void __launch_bounds__(kLossWaves * 64)
k_composite_loss(const float* __restrict__ sigma, const ngp_half* __restrict__ color_out,
                 const ngp_half* __restrict__ h_sigma, const float* __restrict__ deltas,
                 const int32_t* __restrict__ rays, uint32_t M, uint32_t N,
                 const float* __restrict__ gt, const float* __restrict__ bg, LossArgs la,
                 StepState* __restrict__ st, ngp_half* __restrict__ grad_color_out,
                 ngp_half* __restrict__ grad_h, float* __restrict__ out_image,
                 float* __restrict__ out_ws, float* __restrict__ loss_ray, int32_t* __restrict__ ray_rows,
                 int32_t* __restrict__ live_cnt) {
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t n = blockIdx.x * kLossWaves + (threadIdx.x >> 6);
    if (n >= N) return;
    const uint32_t index = (uint32_t)rays[n * 3];
    const uint32_t offset = (uint32_t)rays[n * 3 + 1];
    const uint32_t num_steps = (uint32_t)rays[n * 3 + 2];
    const bool valid = num_steps != 0 && offset + num_steps <= M;
    // everything that only needs the ray's row is requested now, with the
    // first chunk: the background, the target and the first chunk's h0 (each
    // was a dependent round trip after the forward's scans)
    const float bg0 = bg[index * 3], bg1 = bg[index * 3 + 1], bg2 = bg[index * 3 + 2];
    // (RGB targets: alpha 1; loads without branches, see load_chunk)
    const uint32_t gch = la.gt_channels;
    float gt4[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float v = gt[(size_t)index * gch + min((uint32_t)k, gch - 1u)];
        gt4[k] = (uint32_t)k < gch ? v : 1.0f;
    }
    // the ray's first kLossPre chunks of rows (clamped: a short ray's spare
    // chunks read its row 0 again)
    const uint32_t nrows = valid ? num_steps : 0u;
    Raw raw[kLossPre];
#pragma unroll
    for (uint32_t k = 0; k < kLossPre; ++k)
        raw[k] = load_raw(sigma, color_out, deltas, h_sigma, offset, 64 * k, nrows, lane);

    // ---- forward (composite_rays_train_forward)
    // The first kLossPre 64-sample chunks (all of most rays) are kept for the
    // backward pass instead of being loaded and scanned again.
    float r = 0, g = 0, b = 0, ws = 0, d = 0;
    Chunk kept[kLossPre];
    float Sk[kLossPre], tk[kLossPre];
    bool stopk[kLossPre];
    uint32_t nkept = 0;  // kept chunks scanned (the forward stopped in the last of them, or ran on)
    if (valid) {
        float S = 0.0f, tacc = 0.0f;
        bool stop = false;
#pragma unroll
        for (uint32_t k = 0; k < kLossPre; ++k) {
            if (64 * k >= num_steps || stop) break;
            const Chunk c = scan_chunk(raw[k], 64 * k, num_steps, lane, S, tacc, la.T_thresh, stop);
            kept[k] = c;
            Sk[k] = S;
            tk[k] = tacc;
            stopk[k] = stop;
            nkept = k + 1;
            r += wave_sum(c.w * c.c0);
            g += wave_sum(c.w * c.c1);
            b += wave_sum(c.w * c.c2);
            ws += wave_sum(c.w);
            d += wave_sum(c.w * c.t);
        }
        for (uint32_t base = 64 * kLossPre; !stop && base < num_steps; base += 64) {
            const Chunk c = scan_chunk(load_raw(sigma, color_out, deltas, h_sigma, offset, base, num_steps, lane),
                                       base, num_steps, lane, S, tacc, la.T_thresh, stop);
            r += wave_sum(c.w * c.c0);
            g += wave_sum(c.w * c.c1);
            b += wave_sum(c.w * c.c2);
            ws += wave_sum(c.w);
            d += wave_sum(c.w * c.t);
        }
    }
    // ---- background blend + MSE (utils.py train_step) and its gradient
    const float one_m_ws = 1.0f - ws;
    const float p0 = r + one_m_ws * bg0, p1 = g + one_m_ws * bg1, p2 = b + one_m_ws * bg2;
    float q0, q1, q2;
    if (la.gt_channels == 4) {
        const float a = gt4[3], om = 1.0f - a;
        q0 = gt4[0] * a + bg0 * om;
        q1 = gt4[1] * a + bg1 * om;
        q2 = gt4[2] * a + bg2 * om;
    } else {
        q0 = gt4[0]; q1 = gt4[1]; q2 = gt4[2];
    }
    const float e0 = p0 - q0, e1 = p1 - q1, e2 = p2 - q2;
    if (lane == 0) {
        // per-ray loss; summed by k_step_end (one reduction, no contended atomics)
        loss_ray[n] = ((e0 * e0 + e1 * e1) + e2 * e2) * la.inv_c;
        if (out_image) {
            out_image[index * 3] = p0; out_image[index * 3 + 1] = p1; out_image[index * 3 + 2] = p2;
        }
        if (out_ws) out_ws[index] = ws;
    }
    // (loss * scale).backward(): mean -> mean(-1) -> pow(2) -> sub
    const float G = (st->scale * la.inv_n) * la.inv_c;
    const float gr = G * (2.0f * e0), gg = G * (2.0f * e1), gb = G * (2.0f * e2);
    const float gws = -((gr * bg0 + gg * bg1) + gb * bg2);  // d/dws of image + (1 - ws) * bg
    const float gd = 0.0f;                                  // depth is not in the loss

    // ---- backward (composite_rays_train_backward) + activation backward
    if (!valid) {
        if (live_cnt && lane == 0) live_cnt[n] = 0;
        // a ray dropped for overflowing M still owns rows [offset, M): zero their grads
        for (uint32_t k = offset + lane; k < min(offset + num_steps, M); k += 64) {
            const half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
            reinterpret_cast<half8*>(grad_color_out + (size_t)k * 16)[0] = z;
            reinterpret_cast<half8*>(grad_color_out + (size_t)k * 16)[1] = z;
            grad_h[(size_t)k * 16] = (ngp_half)0.0f;
        }
        return;
    }
    float S = 0.0f, tacc = 0.0f, rr = 0, rg = 0, rb = 0, rd = 0;
    bool stopped = false;
    uint32_t nlive = 0;  // rows of this ray with a nonzero gradient so far (listed in ray_rows)
    for (uint32_t base = 0; base < num_steps; base += 64) {
        if (stopped) {
            // past the early stop every row's gradient is exactly zero and
            // none is live (the chunk body gives +0 everywhere): the zeros
            // are written without the chunk's loads and scans (a ray hitting
            // the surface marches on behind it; those chunks were a load
            // round trip and a scan chain each)
            if (base + lane < num_steps) {
                const uint32_t i = offset + base + lane;
                const half8 z = {0, 0, 0, 0, 0, 0, 0, 0};
                half8* go = reinterpret_cast<half8*>(grad_color_out + (size_t)i * 16);
                go[0] = z;
                go[1] = z;
                grad_h[(size_t)i * 16] = (ngp_half)0.0f;
            }
            continue;
        }
        bool stop = false;
        Chunk c{};
        float h0 = 0.0f;
        const uint32_t kc = base / 64;
        if (kc < kLossPre) {
            // a kept chunk (every one up to the forward's stop), or a chunk past
            // the stop: inactive, only its rows' zero grads are written
#pragma unroll
            for (uint32_t k = 0; k < kLossPre; ++k)
                if (k == kc) {
                    if (k < nkept) {
                        c = kept[k];
                        S = Sk[k];
                        tacc = tk[k];
                        stop = stopk[k];
                    } else {
                        c.ok = base + lane < num_steps;
                    }
                    h0 = raw[k].h0;
                }
        } else {
            const Raw rw = load_raw(sigma, color_out, deltas, h_sigma, offset, base, num_steps, lane);
            c = scan_chunk(rw, base, num_steps, lane, S, tacc, la.T_thresh, stop);
            h0 = rw.h0;
        }
        if (stopped || (kc >= nkept && kc < kLossPre)) { c.active = false; c.w = 0.0f; }
        // running sums after this lane's sample (inclusive prefix)
        const float pr = rr + scan_incl(c.w * c.c0, lane);
        const float pg = rg + scan_incl(c.w * c.c1, lane);
        const float pb = rb + scan_incl(c.w * c.c2, lane);
        const float pd = rd + scan_incl(c.w * c.t, lane);
        rr = lane63(pr); rg = lane63(pg); rb = lane63(pb); rd = lane63(pd);
        bool lv = false;
        if (c.ok) {
            const uint32_t i = offset + base + lane;
            float gc0 = 0, gc1 = 0, gc2 = 0, gs = 0;
            if (c.active) {
                gc0 = gr * c.w; gc1 = gg * c.w; gc2 = gb * c.w;
                gs = c.d0 * (gr * (c.Tafter * c.c0 - (r - pr)) + gg * (c.Tafter * c.c1 - (g - pg)) +
                             gb * (c.Tafter * c.c2 - (b - pb)) + gd * (c.Tafter * c.t - (d - pd)) +
                             gws * (1 - ws));
            }
            // rgbs.float() <- half, then sigmoid_backward(grad, y) = grad * (1 - y) * y (fp32 math)
            half8 o0 = {0, 0, 0, 0, 0, 0, 0, 0}, o1 = {0, 0, 0, 0, 0, 0, 0, 0};
            o0[0] = ngp_f2h((float)ngp_f2h(gc0) * (1.0f - c.c0) * c.c0);
            o0[1] = ngp_f2h((float)ngp_f2h(gc1) * (1.0f - c.c1) * c.c1);
            o0[2] = ngp_f2h((float)ngp_f2h(gc2) * (1.0f - c.c2) * c.c2);
            half8* go = reinterpret_cast<half8*>(grad_color_out + (size_t)i * 16);
            go[0] = o0;
            go[1] = o1;
            // sigmas = ds * trunc_exp(h0): grad_h0 = (gs * ds) * exp(clamp(h0, -15, 15)), -> half
            const ngp_half gh0 = ngp_f2h((gs * la.density_scale) * expf(fminf(fmaxf(h0, -15.0f), 15.0f)));
            grad_h[(size_t)i * 16] = gh0;
            // a row whose gradient is zero in every component contributes
            // nothing to any weight or table gradient (the backward's products
            // with it are zeros): the others are listed below, in ray order
            lv = (float)o0[0] != 0.0f || (float)o0[1] != 0.0f || (float)o0[2] != 0.0f || (float)gh0 != 0.0f;
        }
        if (ray_rows) {  // every lane of the wave takes part
            const uint64_t m = __ballot(lv);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (lv) ray_rows[offset + nlive + below] = (int32_t)(offset + base + lane);
            nlive += (uint32_t)__popcll(m);
        }
        stopped = stopped || stop;
    }
    if (live_cnt && lane == 0) live_cnt[n] = (int32_t)nlive;
}

// The live rows of a step as one list in ray order: each workgroup sums the
// live counts of every ray before its block of 64 rays (16-byte loads, all of
// a thread's issued together: one round trip for up to 4,096 rays), scans its
// own rays' counts, then every thread copies list positions (a binary search
// over the block's offsets, the row loads independent of each other); the
// last block writes the total. A latency-bound launch: every step is one
// round trip, nothing waits on another workgroup.
constexpr uint32_t kLiveThreads = 256, kLiveRaysPerBlock = 64;
__global__ void __launch_bounds__(kLiveThreads)
k_live_compact(const int32_t* __restrict__ rays, const int32_t* __restrict__ live_cnt, const int32_t* __restrict__ ray_rows,
               uint32_t N, int32_t* __restrict__ live_rows, int32_t* __restrict__ live_total) {
    __shared__ uint32_t wsum[kLiveThreads / 64];
    __shared__ uint32_t s_off[kLiveRaysPerBlock + 1], s_src[kLiveRaysPerBlock];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const uint32_t r0 = blockIdx.x * kLiveRaysPerBlock, r1 = min(N, r0 + kLiveRaysPerBlock);
    // this block's rays (wave 0): their counts and first rows, requested with the sums below
    uint32_t c = 0, src = 0;
    if (wv == 0 && r0 + lane < r1) {
        c = (uint32_t)live_cnt[r0 + lane];
        src = (uint32_t)rays[(size_t)(r0 + lane) * 3 + 1];
    }
    // sum of the counts of rays [0, r0): r0 is a multiple of 64, so whole int4 groups
    const int4* cnt4 = reinterpret_cast<const int4*>(live_cnt);
    const uint32_t g4 = r0 / 4;
    uint32_t part = 0;
    for (uint32_t b = 0; b < g4; b += 4 * kLiveThreads) {
        int4 v[4];
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t g = b + q * kLiveThreads + t;
            v[q] = g < g4 ? cnt4[g] : int4{0, 0, 0, 0};
        }
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) part += (uint32_t)(v[q].x + v[q].y + v[q].z + v[q].w);
    }
#pragma unroll
    for (uint32_t o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
    if (lane == 0) wsum[wv] = part;
    // this block's rays: exclusive offsets (wave 0)
    if (wv == 0) {
        uint32_t incl = c;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        s_off[lane] = incl - c;
        s_src[lane] = src;
        if (lane == 63) s_off[64] = incl;
    }
    __syncthreads();
    const uint32_t before = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    const uint32_t btotal = s_off[64];
    if (t == 0 && r1 == N) *live_total = (int32_t)(before + btotal);
    // copy: list position before + j <- the row of ray i (largest i with s_off[i] <= j)
    for (uint32_t j = t; j < btotal; j += kLiveThreads) {
        uint32_t lo = 0, hi = kLiveRaysPerBlock;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_off[mid] <= j) lo = mid; else hi = mid;
        }
        live_rows[before + j] = ray_rows[s_src[lo] + (j - s_off[lo])];
    }
}

// GradScaler._unscale_grads_ inf/nan check over every grad (8 halves / lane)
__global__ void __launch_bounds__(256)
k_nonfinite(TensorList tl, StepState* __restrict__ st) {
    const uint64_t total = tl.start[tl.n];
    bool bad = false;
    for (uint64_t i0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i0 < total;
         i0 += (uint64_t)gridDim.x * blockDim.x * 8) {
        const int k = find_tensor(tl, i0);
        const uint64_t off = i0 - tl.start[k];
        const ngp_half* g = tl.g[k] + off;
        if (off + 8 <= tl.size[k] && ((reinterpret_cast<uintptr_t>(g) & 15) == 0)) {
            typedef _Float16 half8 __attribute__((ext_vector_type(8)));
            const half8 v = *reinterpret_cast<const half8*>(g);
#pragma unroll
            for (int j = 0; j < 8; ++j) bad |= !__builtin_isfinite((float)v[j]);
        } else {
            for (uint64_t j = 0; j < 8 && off + j < tl.size[k]; ++j) bad |= !__builtin_isfinite((float)g[j]);
        }
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&st->found_inf, 1);
}

__global__ void __launch_bounds__(kAdamThreads)
k_adam_multi(TensorList tl, StepState* __restrict__ st, AdamArgs aa) {
    adam_sweep(tl, st, aa, blockIdx.x, gridDim.x, threadIdx.x);
}

// ---- data-parallel GradScaler guard ----------------------------------------------
// With the sharded optimizer (nerf/fused.py, world > 1) each rank sees only
// its shard of the reduced gradient, but GradScaler must skip (and back off)
// on every rank together. Each rank checks its own pre-reduction fp16
// gradient; a rank that found an inf/nan writes a NaN into the first element
// of every rank's chunk. The reduction is an average (each input pre-scaled by
// 1/world), so finite inputs cannot overflow into an inf, and after the
// reduce-scatter every owner finds a non-finite value in its shard exactly
// when some rank had one: all ranks skip together.
__global__ void __launch_bounds__(256)
k_guard_scan(const ngp_half* __restrict__ g, uint64_t n8, StepState* __restrict__ st) {
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (uint64_t)gridDim.x * blockDim.x) {
        const half8 v = reinterpret_cast<const half8*>(g)[i];
#pragma unroll
        for (int j = 0; j < 8; ++j) bad |= !__builtin_isfinite((float)v[j]);
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&st->local_inf, 1);
}

__global__ void __launch_bounds__(64)
k_guard_poison(ngp_half* __restrict__ g, uint64_t chunk, int32_t world, StepState* __restrict__ st) {
    const bool bad = st->local_inf != 0;
    __syncthreads();
    if (bad)
        for (int r = threadIdx.x; r < world; r += 64) g[(uint64_t)r * chunk] = (ngp_half)__builtin_nanf("");
    if (threadIdx.x == 0) st->local_inf = 0;
}

__global__ void __launch_bounds__(256)
k_step_end(StepState* __restrict__ st, ScalerArgs sa, const int32_t* __restrict__ counter,
           int32_t* __restrict__ step_counter, const float* __restrict__ loss_ray, uint32_t n_rays) {
    step_end_block(st, sa, counter, step_counter, loss_ray, n_rays);
}

// The head of a fused step, one launch of three independent parts:
//   blocks [0, nlego)      the batch (k_lego_rays)
//   block nlego            the deferred end of the previous optimizer update
//                          (k_step_end: GradScaler.update, LR epoch, loss), if one is pending
//   blocks nlego + 1 ...   the MLP fragment images from the fp16 weights it wrote (ngp_ffmlp_pack)
// The parts touch disjoint state: the sampler only draw / lego_done /
// counter, the end only the scaler / optimizer fields; both read nothing the
// other writes. Each on its own was a latency-bound launch of ~5 us.
__global__ void __launch_bounds__(256)
k_step_head(const float* __restrict__ poses, LegoScene sc, uint32_t N, StepState* __restrict__ st, LegoOut out,
            uint32_t nlego, ScalerArgs sa, const float* __restrict__ loss_ray, ngp_pack::PackJobs jobs,
            uint4* __restrict__ clear, uint32_t clear16) {
    if (blockIdx.x < nlego) {
        lego_rays_block(blockIdx.x, nlego, poses, sc, N, st, out);
    } else if (blockIdx.x == nlego) {
        for (uint32_t i = threadIdx.x; i < clear16; i += blockDim.x) clear[i] = uint4{0u, 0u, 0u, 0u};
        if (st->end_pending) step_end_block(st, sa, nullptr, nullptr, loss_ray, N);
    } else {
        const ngp_pack::PackJob& j = jobs.job[blockIdx.x - nlego - 1];
        ngp_pack::build_frags(j.image, j.w, j.m, j.transposed != 0);
    }
}

// The fused step's first launch when an optimizer update is pending (world 1):
// Adam's sweep, the next batch and the grid backward's cursor clear as block
// ranges of one kernel. The three touch disjoint state (Adam: parameters,
// moments, grads and the scaler fields it reads; the sampler: draw / lego_done /
// counter). The bookkeeping and MLP packs, which need Adam finished, ride in
// the march emit launch (raymarching.hip EmitTail).
__global__ void __launch_bounds__(kAdamThreads)
k_adam_head(TensorList tl, StepState* __restrict__ st, AdamArgs aa, uint32_t nadam, const float* __restrict__ poses,
            LegoScene sc, uint32_t N, LegoOut out, uint32_t nlego, uint4* __restrict__ clear, uint32_t clear16) {
    // the batch and clear blocks come first: workgroups are dispatched in
    // index order, and behind Adam's thousands of blocks the sampler's
    // dependent chain (draw -> pose -> rays -> target) ran in the launch's tail
    if (blockIdx.x < nlego) {
        lego_rays_block(blockIdx.x, nlego, poses, sc, N, st, out);
    } else if (blockIdx.x == nlego) {
        for (uint32_t i = threadIdx.x; i < clear16; i += blockDim.x) clear[i] = uint4{0u, 0u, 0u, 0u};
    } else {
        adam_sweep(tl, st, aa, blockIdx.x - nlego - 1, nadam, threadIdx.x);
    }
}

struct HeadLaunch {  // the batch + clear parts of k_adam_head
    const float* poses;
    LegoScene sc;
    uint32_t N;
    LegoOut out;
    uint4* clear;
    uint32_t clear16;
};

uint32_t sweep_blocks(uint64_t total, uint32_t per_thread) {
    uint64_t b = (total / per_thread + 255) / 256;
    if (b > 8192) b = 8192;
    return b ? (uint32_t)b : 1u;
}

int optimizer_launch(int32_t n_tensors, float* const* params, void* const* grads, float* const* exp_avg,
                     float* const* exp_avg_sq, void* const* half_params, const uint64_t* sizes, float lr,
                     float beta1, float beta2, float eps, int32_t iters, int32_t zero_grads, float grad_mult,
                     float growth_factor, float backoff_factor, int32_t growth_interval, int32_t scaler_enabled,
                     uint32_t num_rays, const int32_t* counter, int32_t* step_counter, const float* loss_ray,
                     void* state, void* stream, bool defer_end, const HeadLaunch* head = nullptr) {
    NGP_REQUIRE(n_tensors >= 1 && n_tensors <= kMaxTensors, NGP_ERR_ARG,
                "fused_optimizer_step: 1..%d tensors", kMaxTensors);
    for (int k = 0; k < n_tensors; ++k)
        NGP_REQUIRE(((reinterpret_cast<uintptr_t>(params[k]) | reinterpret_cast<uintptr_t>(exp_avg[k]) |
                      reinterpret_cast<uintptr_t>(exp_avg_sq[k])) & 15) == 0 &&
                        (reinterpret_cast<uintptr_t>(grads[k]) & 7) == 0,
                    NGP_ERR_ARG, "fused_optimizer_step: tensor %d misaligned", k);
    hipStream_t s = ngp_stream(stream);
    StepState* st = static_cast<StepState*>(state);
    for (int k = 0; k < n_tensors; ++k)
        NGP_REQUIRE(!half_params || !half_params[k] || (reinterpret_cast<uintptr_t>(half_params[k]) & 7) == 0,
                    NGP_ERR_ARG, "fused_optimizer_step: half shadow %d misaligned", k);
    const TensorList tl = make_list(n_tensors, params, grads, exp_avg, exp_avg_sq, half_params, sizes);
    const uint64_t total = tl.start[n_tensors];
    if (scaler_enabled == NGP_SCALER_SCAN) k_nonfinite<<<sweep_blocks(total, 8), 256, 0, s>>>(tl, st);
    AdamArgs aa{lr, beta1, beta2, eps, iters, zero_grads, grad_mult, defer_end ? 1 : 0};
    const uint64_t nchunks = (total + kAdamChunk - 1) / kAdamChunk;
    const uint64_t adam_blocks = std::min<uint64_t>(nchunks, 16ull * ngp_num_cus());
    const uint32_t na = (uint32_t)(adam_blocks ? adam_blocks : 1);
    if (head) {
        const uint32_t nlego = ngp_div_up(head->N, 256);
        k_adam_head<<<na + nlego + 1, kAdamThreads, 0, s>>>(tl, st, aa, na, head->poses, head->sc, head->N,
                                                              head->out, nlego, head->clear, head->clear16);
    } else {
        k_adam_multi<<<na, kAdamThreads, 0, s>>>(tl, st, aa);
    }
    if (!defer_end) {
        ScalerArgs sa{growth_factor, backoff_factor, growth_interval, scaler_enabled,
                      num_rays ? 1.0f / (float)num_rays : 0.0f};
        k_step_end<<<1, 256, 0, s>>>(st, sa, counter, step_counter, loss_ray, num_rays);
    }
    return ngp_check_launch("fused_optimizer_step");
}

}  // namespace

extern "C" size_t ngp_fused_state_bytes(void) { return sizeof(StepState); }

extern "C" int ngp_fused_state_init(void* state, float init_scale, void* stream) {
    NGP_REQUIRE(state, NGP_ERR_ARG, "fused_state_init: null state");
    StepState s{};
    s.scale = init_scale;
    return hipMemcpyAsync(state, &s, sizeof(s), hipMemcpyHostToDevice, ngp_stream(stream)) == hipSuccess
               ? NGP_OK
               : ngp_set_error(NGP_ERR_HIP, "fused_state_init: copy failed");
}

extern "C" int ngp_lego_rays(const float* poses, uint32_t n_poses, const float* intrinsics4,
                             uint32_t H, uint32_t W, uint32_t N, const float* boxes, int32_t nboxes,
                             const float* aabb6, float min_near, uint32_t seed, void* state,
                             float* rays_o, float* rays_d, float* rgba, float* bg, float* nears,
                             float* fars, float* noises, int32_t* counter, int32_t* step_counter,
                             void* stream) {
    NGP_REQUIRE(nboxes >= 0 && nboxes <= kMaxBoxes, NGP_ERR_ARG, "lego_rays: at most %d boxes", kMaxBoxes);
    NGP_REQUIRE(n_poses > 0 && H > 0 && W > 0, NGP_ERR_ARG, "lego_rays: empty pose set or image");
    if (N == 0) return NGP_OK;
    const LegoScene sc = make_scene(n_poses, intrinsics4, H, W, boxes, nboxes, aabb6, min_near, seed);
    const LegoOut out{rays_o, rays_d, rgba, bg, nears, fars, noises, counter, step_counter};
    k_lego_rays<<<ngp_div_up(N, 256), 256, 0, ngp_stream(stream)>>>(poses, sc, N, static_cast<StepState*>(state),
                                                                     out);
    return ngp_check_launch("lego_rays");
}

extern "C" int ngp_nerf_glue_forward(const void* h_sigma, const float* dirs, float density_scale,
                                     float* sigma, void* color_in, uint32_t B, const int32_t* count,
                                     void* stream) {
    if (B == 0) return NGP_OK;
    k_glue_fwd<<<ngp_div_up(B, 256), 256, 0, ngp_stream(stream)>>>(
        (const ngp_half*)h_sigma, dirs, density_scale, sigma, (ngp_half*)color_in, B, count);
    return ngp_check_launch("nerf_glue_forward");
}

extern "C" int ngp_nerf_glue_backward(const void* grad_color_in, void* grad_h_sigma, uint32_t B,
                                      const int32_t* count, void* stream) {
    if (B == 0) return NGP_OK;
    k_glue_bwd<<<ngp_div_up(B, 256), 256, 0, ngp_stream(stream)>>>(
        (const ngp_half*)grad_color_in, (ngp_half*)grad_h_sigma, B, count);
    return ngp_check_launch("nerf_glue_backward");
}

extern "C" int ngp_nerf_composite_loss(const float* sigma, const void* color_out, const void* h_sigma,
                                       const float* deltas, const int32_t* rays, uint32_t M,
                                       uint32_t N, float T_thresh, float density_scale,
                                       const float* gt, uint32_t gt_channels, const float* bg,
                                       void* state, void* grad_color_out, void* grad_h_sigma,
                                       float* out_image, float* out_ws, float* loss_ray,
                                       void* stream) {
    NGP_REQUIRE(loss_ray, NGP_ERR_ARG, "composite_loss: loss_ray [N] buffer required");
    NGP_REQUIRE(gt_channels == 3 || gt_channels == 4, NGP_ERR_ARG, "composite_loss: gt must be RGB or RGBA");
    if (N == 0) return NGP_OK;
    LossArgs la;
    la.T_thresh = T_thresh;
    la.density_scale = density_scale;
    la.inv_n = 1.0f / (float)N;
    la.inv_c = 1.0f / 3.0f;
    la.gt_channels = gt_channels;
    k_composite_loss<<<ngp_div_up(N, kLossWaves), kLossWaves * 64, 0, ngp_stream(stream)>>>(
        sigma, (const ngp_half*)color_out, (const ngp_half*)h_sigma, deltas, rays, M, N, gt, bg, la,
        static_cast<StepState*>(state), (ngp_half*)grad_color_out, (ngp_half*)grad_h_sigma, out_image,
        out_ws, loss_ray, nullptr, nullptr);
    return ngp_check_launch("nerf_composite_loss");
}

extern "C" int ngp_nerf_composite_loss_live(const float* sigma, const void* color_out, const void* h_sigma,
                                            const float* deltas, const int32_t* rays, uint32_t M, uint32_t N,
                                            float T_thresh, float density_scale, const float* gt,
                                            uint32_t gt_channels, const float* bg, void* state,
                                            void* grad_color_out, void* grad_h_sigma, float* out_image,
                                            float* out_ws, float* loss_ray, int32_t* ray_rows, int32_t* live_cnt,
                                            int32_t* live_rows, int32_t* live_total, void* stream) {
    NGP_REQUIRE(loss_ray, NGP_ERR_ARG, "composite_loss_live: loss_ray [N] buffer required");
    NGP_REQUIRE(gt_channels == 3 || gt_channels == 4, NGP_ERR_ARG, "composite_loss_live: gt must be RGB or RGBA");
    NGP_REQUIRE(ray_rows && live_cnt && live_rows && live_total, NGP_ERR_ARG,
                "composite_loss_live: null ray_rows [M] / live_cnt [N] / live_rows [M] / live_total");
    NGP_REQUIRE((reinterpret_cast<uintptr_t>(live_cnt) & 15) == 0, NGP_ERR_ARG,
                "composite_loss_live: live_cnt must be 16-byte aligned");
    hipStream_t st = ngp_stream(stream);
    if (N == 0) {
        if (hipMemsetAsync(live_total, 0, sizeof(int32_t), st) != hipSuccess)
            return ngp_set_error(NGP_ERR_HIP, "composite_loss_live: memset failed");
        return NGP_OK;
    }
    LossArgs la;
    la.T_thresh = T_thresh;
    la.density_scale = density_scale;
    la.inv_n = 1.0f / (float)N;
    la.inv_c = 1.0f / 3.0f;
    la.gt_channels = gt_channels;
    k_composite_loss<<<ngp_div_up(N, kLossWaves), kLossWaves * 64, 0, st>>>(
        sigma, (const ngp_half*)color_out, (const ngp_half*)h_sigma, deltas, rays, M, N, gt, bg, la,
        static_cast<StepState*>(state), (ngp_half*)grad_color_out, (ngp_half*)grad_h_sigma, out_image,
        out_ws, loss_ray, ray_rows, live_cnt);
    k_live_compact<<<ngp_div_up(N, kLiveRaysPerBlock), kLiveThreads, 0, st>>>(rays, live_cnt, ray_rows, N, live_rows,
                                                                              live_total);
    return ngp_check_launch("nerf_composite_loss_live");
}

extern "C" int ngp_fused_optimizer_step(int32_t n_tensors, float* const* params, void* const* grads,
                                        float* const* exp_avg, float* const* exp_avg_sq,
                                        void* const* half_params, const uint64_t* sizes, float lr,
                                        float beta1, float beta2, float eps, int32_t iters,
                                        int32_t zero_grads, float grad_mult,
                                        float growth_factor, float backoff_factor,
                                        int32_t growth_interval, int32_t scaler_enabled,
                                        uint32_t num_rays, const int32_t* counter,
                                        int32_t* step_counter, const float* loss_ray, void* state,
                                        void* stream) {
    return optimizer_launch(n_tensors, params, grads, exp_avg, exp_avg_sq, half_params, sizes, lr, beta1, beta2,
                            eps, iters, zero_grads, grad_mult, growth_factor, backoff_factor, growth_interval,
                            scaler_enabled, num_rays, counter, step_counter, loss_ray, state, stream, false);
}

extern "C" int ngp_fused_optimizer_update(int32_t n_tensors, float* const* params, void* const* grads,
                                          float* const* exp_avg, float* const* exp_avg_sq,
                                          void* const* half_params, const uint64_t* sizes, float lr,
                                          float beta1, float beta2, float eps, int32_t iters,
                                          int32_t zero_grads, float grad_mult, int32_t scaler_enabled,
                                          void* state, void* stream) {
    return optimizer_launch(n_tensors, params, grads, exp_avg, exp_avg_sq, half_params, sizes, lr, beta1, beta2,
                            eps, iters, zero_grads, grad_mult, 0.0f, 0.0f, 0, scaler_enabled, 0, nullptr, nullptr,
                            nullptr, state, stream, true);
}

extern "C" int ngp_fused_step_head(const float* poses, uint32_t n_poses, const float* intrinsics4, uint32_t H,
                                   uint32_t W, uint32_t N, const float* boxes, int32_t nboxes, const float* aabb6,
                                   float min_near, uint32_t seed, void* state, float* rays_o, float* rays_d,
                                   float* rgba, float* bg, float* nears, float* fars, float* noises,
                                   int32_t* counter, int32_t* step_counter, float growth_factor,
                                   float backoff_factor, int32_t growth_interval, int32_t scaler_enabled,
                                   const float* loss_ray, int32_t n_nets, const void* const* mlp_weights,
                                   const uint32_t* in_dims, const uint32_t* hidden_dims,
                                   const uint32_t* num_layers, void* const* images, void* clear,
                                   uint32_t clear_bytes, void* stream) {
    NGP_REQUIRE(nboxes >= 0 && nboxes <= kMaxBoxes, NGP_ERR_ARG, "step_head: at most %d boxes", kMaxBoxes);
    NGP_REQUIRE(n_poses > 0 && H > 0 && W > 0 && N > 0, NGP_ERR_ARG, "step_head: empty pose set, image or batch");
    NGP_REQUIRE(state && loss_ray, NGP_ERR_ARG, "step_head: null state or loss_ray");
    NGP_REQUIRE(clear_bytes % 16 == 0 && (reinterpret_cast<uintptr_t>(clear) & 15) == 0, NGP_ERR_ARG,
                "step_head: clear must be 16-byte aligned, a multiple of 16 bytes");
    ngp_pack::PackJobs jobs{};
    if (n_nets > 0)
        if (int e = ngp_pack::build_jobs(n_nets, mlp_weights, in_dims, hidden_dims, num_layers, images, jobs))
            return e;
    const LegoScene sc = make_scene(n_poses, intrinsics4, H, W, boxes, nboxes, aabb6, min_near, seed);
    const LegoOut out{rays_o, rays_d, rgba, bg, nears, fars, noises, counter, step_counter};
    const ScalerArgs sa{growth_factor, backoff_factor, growth_interval, scaler_enabled, 1.0f / (float)N};
    const uint32_t nlego = ngp_div_up(N, 256);
    k_step_head<<<nlego + 1 + (uint32_t)jobs.n, 256, 0, ngp_stream(stream)>>>(
        poses, sc, N, static_cast<StepState*>(state), out, nlego, sa, loss_ray, jobs, static_cast<uint4*>(clear),
        clear ? clear_bytes / 16 : 0u);
    return ngp_check_launch("fused_step_head");
}

extern "C" int ngp_fused_optimizer_update_head(
    int32_t n_tensors, float* const* params, void* const* grads, float* const* exp_avg, float* const* exp_avg_sq,
    void* const* half_params, const uint64_t* sizes, float lr, float beta1, float beta2, float eps, int32_t iters,
    int32_t zero_grads, float grad_mult, int32_t scaler_enabled, void* state, const float* poses, uint32_t n_poses,
    const float* intrinsics4, uint32_t H, uint32_t W, uint32_t N, const float* boxes, int32_t nboxes,
    const float* aabb6, float min_near, uint32_t seed, float* rays_o, float* rays_d, float* rgba, float* bg,
    float* nears, float* fars, float* noises, int32_t* counter, int32_t* step_counter, void* clear,
    uint32_t clear_bytes, void* stream) {
    NGP_REQUIRE(state, NGP_ERR_ARG, "fused_optimizer_update_head: null state");
    NGP_REQUIRE(nboxes >= 0 && nboxes <= kMaxBoxes, NGP_ERR_ARG, "step_head: at most %d boxes", kMaxBoxes);
    NGP_REQUIRE(n_poses > 0 && H > 0 && W > 0 && N > 0, NGP_ERR_ARG, "step_head: empty pose set, image or batch");
    NGP_REQUIRE(clear_bytes % 16 == 0 && (reinterpret_cast<uintptr_t>(clear) & 15) == 0, NGP_ERR_ARG,
                "step_head: clear must be 16-byte aligned, a multiple of 16 bytes");
    HeadLaunch hl{};
    hl.poses = poses;
    hl.sc = make_scene(n_poses, intrinsics4, H, W, boxes, nboxes, aabb6, min_near, seed);
    hl.N = N;
    hl.out = LegoOut{rays_o, rays_d, rgba, bg, nears, fars, noises, counter, step_counter};
    hl.clear = static_cast<uint4*>(clear);
    hl.clear16 = clear ? clear_bytes / 16 : 0u;
    return optimizer_launch(n_tensors, params, grads, exp_avg, exp_avg_sq, half_params, sizes, lr, beta1, beta2,
                            eps, iters, zero_grads, grad_mult, 2.0f, 0.5f, 2000, scaler_enabled, 0, nullptr,
                            nullptr, nullptr, state, stream, true, &hl);
}

extern "C" int ngp_grad_guard(void* grad_half, uint64_t n, uint64_t chunk, int32_t world, void* state,
                              void* stream) {
    NGP_REQUIRE(grad_half && state, NGP_ERR_ARG, "grad_guard: null buffer");
    NGP_REQUIRE(n % 8 == 0 && (reinterpret_cast<uintptr_t>(grad_half) & 15) == 0, NGP_ERR_ARG,
                "grad_guard: gradient must be 16-byte aligned with a multiple of 8 elements");
    NGP_REQUIRE(world >= 1 && (n == 0 || (uint64_t)world * chunk <= n), NGP_ERR_ARG,
                "grad_guard: world * chunk exceeds the gradient");
    hipStream_t s = ngp_stream(stream);
    StepState* st = static_cast<StepState*>(state);
    if (n) k_guard_scan<<<sweep_blocks(n, 8), 256, 0, s>>>(static_cast<const ngp_half*>(grad_half), n / 8, st);
    k_guard_poison<<<1, 64, 0, s>>>(static_cast<ngp_half*>(grad_half), chunk, world, st);
    return ngp_check_launch("grad_guard");
}

extern "C" int32_t* ngp_fused_inf_flag(void* state, int32_t local) {
    StepState* st = static_cast<StepState*>(state);
    return st ? (local ? &st->local_inf : &st->found_inf) : nullptr;
}
