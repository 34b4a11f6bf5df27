// Device code of the fused step's head shared by nerf_fused.hip (its own
// head launches) and raymarching.hip (the march launch that carries the
// optimizer update, ngp_march_rays_train_prebuilt_adam): the synthetic Lego
// sampler and the Adam sweep. Header-only, internal linkage per translation unit.
#pragma once
#include "ngp_common.h"
#include "ngp_step.h"

#include <cfloat>


namespace ngp_head {

using ngp_step::StepState;

constexpr int kMaxBoxes = 8;
constexpr int kMaxTensors = 8;

// counter-based RNG (no state, graph-safe): 32-bit mix of (seed, a, b, c)
NGP_DEV uint32_t mix32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du;
    x ^= x >> 15; x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
NGP_DEV uint32_t rng_u32(uint32_t seed, uint32_t a, uint32_t b, uint32_t c) {
    return mix32(seed ^ mix32(a + 0x9e3779b9u * mix32(b ^ mix32(c + 0x85ebca6bu))));
}
NGP_DEV float rng_unit(uint32_t seed, uint32_t a, uint32_t b, uint32_t c) {
    return (float)(rng_u32(seed, a, b, c) >> 8) * (1.0f / 16777216.0f);
}

struct LegoScene {
    float lo[kMaxBoxes][3], hi[kMaxBoxes][3], rgb[kMaxBoxes][3];
    int nboxes;
    float fx, fy, cx, cy;
    uint32_t H, W, n_poses;
    float aabb[6];
    float min_near;
    uint32_t seed;
};

// near/far against the aabb, reference raymarching.cu:91-145 (same as
// k_near_far in raymarching.hip)
NGP_DEV void near_far(const float o[3], const float d[3], const float aabb[6], float min_near,
                      float& near, float& far) {
    const float rdx = 1 / d[0], rdy = 1 / d[1], rdz = 1 / d[2];
    near = (aabb[0] - o[0]) * rdx;
    far = (aabb[3] - o[0]) * rdx;
    if (near > far) { float c = near; near = far; far = c; }
    float ny = (aabb[1] - o[1]) * rdy, fy = (aabb[4] - o[1]) * rdy;
    if (ny > fy) { float c = ny; ny = fy; fy = c; }
    if (near > fy || ny > far) { near = far = FLT_MAX; return; }
    if (ny > near) near = ny;
    if (fy < far) far = fy;
    float nz = (aabb[2] - o[2]) * rdz, fz = (aabb[5] - o[2]) * rdz;
    if (nz > fz) { float c = nz; nz = fz; fz = c; }
    if (near > fz || nz > far) { near = far = FLT_MAX; return; }
    if (nz > near) near = nz;
    if (fz < far) far = fz;
    if (near < min_near) near = min_near;
}

struct LegoOut {
    float *rays_o, *rays_d, *rgba, *bg, *nears, *fars, *noises;
    int32_t *counter, *step_counter;
    // the draw runs while the previous batch's kernels may still read the
    // counter (the next batch drawn in the grid backward's bin launch): its
    // counts are recorded but the counter is left to the accumulate to reset
    int32_t keep_counter;
};

static inline LegoScene make_scene(uint32_t n_poses, const float* intrinsics4, uint32_t H, uint32_t W,
                                   const float* boxes, int32_t nboxes, const float* aabb6, float min_near,
                                   uint32_t seed) {
    LegoScene sc{};
    for (int b = 0; b < nboxes; ++b)
        for (int k = 0; k < 3; ++k) {
            sc.lo[b][k] = boxes[b * 9 + k];
            sc.hi[b][k] = boxes[b * 9 + 3 + k];
            sc.rgb[b][k] = boxes[b * 9 + 6 + k];
        }
    sc.nboxes = nboxes;
    sc.fx = intrinsics4[0]; sc.fy = intrinsics4[1]; sc.cx = intrinsics4[2]; sc.cy = intrinsics4[3];
    sc.H = H; sc.W = W; sc.n_poses = n_poses;
    for (int k = 0; k < 6; ++k) sc.aabb[k] = aabb6[k];
    sc.min_near = min_near;
    sc.seed = seed;
    return sc;
}

// Ray n of draw `it` (the fused sampler, reference get_rays utils.py:52-136 +
// the analytic target + background + march noise + near/far): writes the
// ray's outputs and returns its origin / direction / near / far / noise.
NGP_DEV void lego_ray(uint32_t n, uint32_t it, const float* __restrict__ poses, const LegoScene& sc,
                      const LegoOut& out, float (&o)[3], float (&d)[3], float& nr, float& fr, float& noise) {
    const uint32_t pose = rng_u32(sc.seed, it, 0xffffffffu, 0) % sc.n_poses;
    const float* P = poses + (size_t)pose * 16;
    const uint32_t pix = rng_u32(sc.seed, it, n, 1) % (sc.H * sc.W);
    // get_rays (utils.py:52-136): pixel centre, camera direction, normalise, rotate
    const float i = (float)(pix % sc.W) + 0.5f;
    const float j = (float)(pix / sc.W) + 0.5f;
    float xs = (i - sc.cx) / sc.fx, ys = (j - sc.cy) / sc.fy, zs = 1.0f;
    const float nrm = sqrtf(xs * xs + ys * ys + zs * zs);
    xs /= nrm; ys /= nrm; zs /= nrm;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        d[k] = fmaf(zs, P[k * 4 + 2], fmaf(ys, P[k * 4 + 1], xs * P[k * 4 + 0]));
        o[k] = P[k * 4 + 3];
        out.rays_o[n * 3 + k] = o[k];
        out.rays_d[n * 3 + k] = d[k];
    }
    // analytic RGBA: colour of the nearest box hit (SyntheticLego.target)
    float best = INFINITY;
    int arg = -1;
    for (int b = 0; b < sc.nboxes; ++b) {
        float tn = -INFINITY, tf = INFINITY;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float inv = 1.0f / d[k];
            const float t0 = (sc.lo[b][k] - o[k]) * inv, t1 = (sc.hi[b][k] - o[k]) * inv;
            tn = fmaxf(tn, fminf(t0, t1));
            tf = fminf(tf, fmaxf(t0, t1));
        }
        if (tf >= tn && tf > 0 && tn < best) { best = tn; arg = b; }
    }
    out.rgba[n * 4 + 0] = arg >= 0 ? sc.rgb[arg][0] : 0.0f;
    out.rgba[n * 4 + 1] = arg >= 0 ? sc.rgb[arg][1] : 0.0f;
    out.rgba[n * 4 + 2] = arg >= 0 ? sc.rgb[arg][2] : 0.0f;
    out.rgba[n * 4 + 3] = arg >= 0 ? 1.0f : 0.0f;
#pragma unroll
    for (int k = 0; k < 3; ++k) out.bg[n * 3 + k] = rng_unit(sc.seed, it, n, 2 + k);
    noise = rng_unit(sc.seed, it, n, 5);
    out.noises[n] = noise;
    near_far(o, d, sc.aabb, sc.min_near, nr, fr);
    out.nears[n] = nr;
    out.fars[n] = fr;
}

// Start of a draw, by ONE thread of the launch: the previous batch's counts
// go to step_counter (mean_count, update_extra_state) and the counter is reset.
NGP_DEV void lego_begin(uint32_t it, const LegoOut& out) {
    if (out.step_counter && it > 0) {
        const uint32_t slot = (it - 1) & 15u;
        out.step_counter[slot * 2] = out.counter[0];
        out.step_counter[slot * 2 + 1] = out.counter[1];
    }
    if (!out.keep_counter) {
        out.counter[0] = 0;
        out.counter[1] = 0;
    }
}

// End of a draw: after the whole workgroup has read `draw`, its first thread
// counts the workgroup done; the last of the `nblk` bumps the draw counter.
NGP_DEV void lego_end(uint32_t it, uint32_t nblk, StepState* __restrict__ st) {
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(&st->lego_done, 1) == (int32_t)nblk - 1) {
            st->draw = (int32_t)it + 1;
            st->lego_done = 0;
        }
    }
}

// Block `blk` of the `nblk` blocks (256 threads) drawing one batch.
NGP_DEV void lego_rays_block(uint32_t blk, uint32_t nblk, const float* __restrict__ poses, const LegoScene& sc,
                             uint32_t N, StepState* __restrict__ st, const LegoOut& out) {
    const uint32_t n = blk * blockDim.x + threadIdx.x;
    const uint32_t it = (uint32_t)st->draw;
    // Only this code touches draw / lego_done / counter / step_counter, so it
    // can run beside the previous step's optimizer (nerf/fused.py pipelining).
    if (n == 0) lego_begin(it, out);
    __syncthreads();  // every thread of the block has read draw before the last block bumps it
    lego_end(it, nblk, st);
    if (n >= N) return;
    float o[3], d[3], nr, fr, noise;
    lego_ray(n, it, poses, sc, out, o, d, nr, fr, noise);
}

// ---- optimizer ------------------------------------------------------------------
struct TensorList {
    int n;
    float* p[kMaxTensors];
    ngp_half* g[kMaxTensors];
    float* m[kMaxTensors];
    float* v[kMaxTensors];
    ngp_half* ph[kMaxTensors];        // optional fp16 shadow of p (the MLPs' forward weights)
    uint64_t size[kMaxTensors];
    uint64_t start[kMaxTensors + 1];  // flat index space; each tensor starts 8-aligned
};

static inline TensorList make_list(int n, float* const* p, void* const* g, float* const* m, float* const* v,
                                   void* const* ph, const uint64_t* sizes) {
    TensorList tl{};
    tl.n = n;
    tl.start[0] = 0;
    for (int k = 0; k < n; ++k) {
        tl.p[k] = p ? p[k] : nullptr;
        tl.g[k] = static_cast<ngp_half*>(g[k]);
        tl.m[k] = m ? m[k] : nullptr;
        tl.v[k] = v ? v[k] : nullptr;
        tl.ph[k] = ph ? static_cast<ngp_half*>(ph[k]) : nullptr;
        tl.size[k] = sizes[k];
        tl.start[k + 1] = tl.start[k] + (sizes[k] + 7) / 8 * 8;
    }
    return tl;
}

NGP_DEV int find_tensor(const TensorList& tl, uint64_t i) {
    int k = 0;
    while (k + 1 < tl.n && i >= tl.start[k + 1]) ++k;
    return k;
}

struct AdamArgs {
    float base_lr, beta1, beta2, eps;
    int32_t iters;   // LambdaLR: lr = base_lr * 0.1 ** min(epoch / iters, 1)
    int32_t zero_grads;
    float grad_mult; // e.g. 1 / world_size after a data-parallel all-reduce (sum)
    int32_t defer_end;  // the step's bookkeeping runs in the next k_step_head
};

// torch.optim.Adam (weight_decay 0) on p, with g = half_grad * (1 / scale);
// skipped (state untouched) when the check found an inf/nan, like
// GradScaler.step. Grads are zeroed afterwards either way. (Ending the step
// in Adam's last block instead of k_step_end was measured: 4096 blocks
// retiring through one counter cost ~180 us of contended atomics.)
//
// Layout: chunks of 1024 U elements of the flat (8-aligned per tensor)
// index space, chunk c to block c mod gridDim; every thread keeps U 16-byte
// groups of each stream in flight. A chunk inside one tensor (all but the few
// at the seams) takes its pointers from scalar loads.
// The grads are cleared where they are nonzero only (bits, so a -0 too): most
// of a step's gradient is zero already (the backward writes the entries its
// samples touch), and a 32-byte sector nobody stores to is never written
// back. NGP_ADAM_ZERO_ALL (A/B builds only) stores every group.
typedef _Float16 adam_half4 __attribute__((ext_vector_type(4)));
NGP_DEV bool grad_set(adam_half4 g) {
#ifdef NGP_ADAM_ZERO_ALL
    (void)g;
    return true;
#else
    const uint2 w = __builtin_bit_cast(uint2, g);
    return (w.x | w.y) != 0u;
#endif
}
// A group Adam leaves exactly as it is: m = v = +0 (never touched; they
// cannot become -0) and g = +-0 give m' = v' = +0 and p' = p - step * 0 = p,
// so its stores are dropped (on a hash grid most entries of the fine levels
// stay untouched). NGP_ADAM_STORE_ALL (A/B builds only) stores every group.
NGP_DEV bool adam_idle(const float4& m, const float4& v, adam_half4 g) {
#ifdef NGP_ADAM_STORE_ALL
    (void)m; (void)v; (void)g;
    return false;
#else
    const uint2 w = __builtin_bit_cast(uint2, g);
    return ((w.x | w.y) & 0x7fff7fffu) == 0u && m.x == 0.0f && m.y == 0.0f && m.z == 0.0f && m.w == 0.0f &&
           v.x == 0.0f && v.y == 0.0f && v.z == 0.0f && v.w == 0.0f;
#endif
}
constexpr uint32_t kAdamThreads = 256, kAdamChunk = kAdamThreads * 8;
// U: 16-byte groups of each stream per thread and chunk (chunk = 1024 U
// elements). The standalone sweep keeps 2 in flight; the sweep inside the
// march launch (a quarter of a CU's waves) keeps 4 to stream at HBM rate.
template <int U = 2>
NGP_DEV void adam_sweep(const TensorList& tl, StepState* __restrict__ st, const AdamArgs& aa, uint32_t blk,
                        uint32_t nblk, uint32_t tid) {
    constexpr uint32_t kChunk = kAdamThreads * 4 * U;
    const ngp_step::AdamConsts ac = ngp_step::adam_consts(st, aa.base_lr, aa.beta1, aa.beta2, aa.iters,
                                                          aa.grad_mult);
    const bool skip = st->found_inf != 0 || ac.inv_bad;
    if (blk == 0 && tid == 0) {
        if (ac.inv_bad) st->found_inf = 1;  // the scaler update backs off, as torch's would
        if (aa.defer_end) st->end_pending = 1;  // read by k_step_head only
    }
    typedef _Float16 half4 __attribute__((ext_vector_type(4)));
    // zero_grads bit 1 (NGP_ADAM_SHADOW_ALL): every fp16 shadow value is
    // written, updated or not (a shadow kept only now and then, the density
    // query's table copy); otherwise the groups left unchanged keep theirs
    const bool shadow_all = (aa.zero_grads & 2) != 0;
    auto adam1 = [&](float& p, float& m, float& v, float gh) {
        ngp_step::adam_update(p, m, v, gh, ac, aa.beta1, aa.beta2, aa.eps);
    };
    const uint64_t total = tl.start[tl.n];
    const uint64_t nchunks = (total + kChunk - 1) / kChunk;
    for (uint64_t c = blk; c < nchunks; c += nblk) {
        const uint64_t c0 = c * kChunk, c1 = min(c0 + kChunk, total);
        const int k = find_tensor(tl, c0);
        if (find_tensor(tl, c1 - 1) == k && c1 - tl.start[k] <= tl.size[k]) {
            // whole chunk inside tensor k: U float4 groups per thread, loads first
            const uint64_t base = c0 - tl.start[k] + tid * 4;
            float4 pv[U], mv[U], vv[U];
            half4 gh[U];
            bool in[U];
            // loads without branches: a group past the chunk's end reads the
            // chunk's first group and is dropped (a load under a divergent
            // branch made the compiler wait for each one before the next)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint64_t off = base + u * (kChunk / U);
                in[u] = c0 + (off - (c0 - tl.start[k])) < c1;
                const uint64_t lo = in[u] ? off : c0 - tl.start[k];
                pv[u] = *reinterpret_cast<const float4*>(tl.p[k] + lo);
                mv[u] = *reinterpret_cast<const float4*>(tl.m[k] + lo);
                vv[u] = *reinterpret_cast<const float4*>(tl.v[k] + lo);
                gh[u] = *reinterpret_cast<const half4*>(tl.g[k] + lo);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (!in[u]) continue;
                const uint64_t off = base + u * (kChunk / U);
                const bool upd = !skip && !adam_idle(mv[u], vv[u], gh[u]);
                if (upd) {
                    adam1(pv[u].x, mv[u].x, vv[u].x, (float)gh[u][0]);
                    adam1(pv[u].y, mv[u].y, vv[u].y, (float)gh[u][1]);
                    adam1(pv[u].z, mv[u].z, vv[u].z, (float)gh[u][2]);
                    adam1(pv[u].w, mv[u].w, vv[u].w, (float)gh[u][3]);
                    *reinterpret_cast<float4*>(tl.p[k] + off) = pv[u];
                    *reinterpret_cast<float4*>(tl.m[k] + off) = mv[u];
                    *reinterpret_cast<float4*>(tl.v[k] + off) = vv[u];
                }
                if (tl.ph[k] && (upd || shadow_all))
                    *reinterpret_cast<half4*>(tl.ph[k] + off) =
                        half4{(ngp_half)pv[u].x, (ngp_half)pv[u].y, (ngp_half)pv[u].z, (ngp_half)pv[u].w};
                if (aa.zero_grads && grad_set(gh[u])) *reinterpret_cast<half4*>(tl.g[k] + off) = half4{0, 0, 0, 0};
            }
            continue;
        }
        // a seam chunk: per element
        for (uint64_t i = c0 + tid; i < c1; i += kAdamThreads) {
            const int kk = find_tensor(tl, i);
            const uint64_t off = i - tl.start[kk];
            if (off >= tl.size[kk]) continue;  // alignment padding between tensors
            float p = tl.p[kk][off];
            if (!skip) {
                float m = tl.m[kk][off], v = tl.v[kk][off];
                adam1(p, m, v, (float)tl.g[kk][off]);
                tl.p[kk][off] = p;
                tl.m[kk][off] = m;
                tl.v[kk][off] = v;
            }
            if (tl.ph[kk] && (!skip || shadow_all)) tl.ph[kk][off] = (ngp_half)p;
            if (aa.zero_grads) tl.g[kk][off] = (ngp_half)0.0f;
        }
    }
}

// adam_sweep software-pipelined for few waves (the sweep inside the march
// launch: 12 of a CU's waves): the loads of this block's next chunk are
// issued before the current chunk is computed and stored, so every wave keeps
// a chunk's worth of loads in flight all the time (the plain sweep waits out a
// full memory round trip per chunk; ~4 chunks per block left it at 80 % of
// the standalone sweep's bandwidth). Same arithmetic, same stores.
template <int U>
NGP_DEV void adam_sweep_pipe(const TensorList& tl, StepState* __restrict__ st, const AdamArgs& aa, uint32_t blk,
                             uint32_t nblk, uint32_t tid) {
    constexpr uint32_t kChunk = kAdamThreads * 4 * U;
    typedef _Float16 half4 __attribute__((ext_vector_type(4)));
    const ngp_step::AdamConsts ac = ngp_step::adam_consts(st, aa.base_lr, aa.beta1, aa.beta2, aa.iters,
                                                          aa.grad_mult);
    const bool skip = st->found_inf != 0 || ac.inv_bad;
    if (blk == 0 && tid == 0) {
        if (ac.inv_bad) st->found_inf = 1;
        if (aa.defer_end) st->end_pending = 1;
    }
    // NGP_ADAM_SHADOW_ALL as in adam_sweep: every fp16 shadow value written,
    // updated or not (the flag meant the same in both sweeps only
    // while no caller passed it here)
    const bool shadow_all = (aa.zero_grads & 2) != 0;
    const uint64_t total = tl.start[tl.n];
    const uint64_t nchunks = (total + kChunk - 1) / kChunk;
    struct Buf {
        float4 p[U], m[U], v[U];
        half4 g[U];
    };
    // the chunk's tensor if the chunk lies inside one, else -1 (a seam)
    auto whole = [&](uint64_t c) {
        const uint64_t c0 = c * kChunk, c1 = min(c0 + kChunk, total);
        const int k = find_tensor(tl, c0);
        return find_tensor(tl, c1 - 1) == k && c1 - tl.start[k] <= tl.size[k] ? k : -1;
    };
    // (the default cache policy: streamed nontemporal, the sweep measured 25 %
    // slower, DESIGN.md "Measured and dropped")
    auto ld_f4 = [](const float* q) { return *reinterpret_cast<const float4*>(q); };
    auto st_f4 = [](float* q, float4 x) { *reinterpret_cast<float4*>(q) = x; };
    auto load = [&](uint64_t c, int k, Buf& b) {  // unconditional: past the end reads the chunk's first group
        const uint64_t c0 = c * kChunk, c1 = min(c0 + kChunk, total), first = c0 - tl.start[k];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t off = first + tid * 4 + u * (kChunk / U);
            const uint64_t lo = off + tl.start[k] < c1 ? off : first;
            b.p[u] = ld_f4(tl.p[k] + lo);
            b.m[u] = ld_f4(tl.m[k] + lo);
            b.v[u] = ld_f4(tl.v[k] + lo);
            b.g[u] = *reinterpret_cast<const half4*>(tl.g[k] + lo);
        }
    };
    auto apply = [&](uint64_t c, int k, Buf& b) {
        const uint64_t c0 = c * kChunk, c1 = min(c0 + kChunk, total), first = c0 - tl.start[k];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t off = first + tid * 4 + u * (kChunk / U);
            if (off + tl.start[k] >= c1) continue;
            const bool upd = !skip && !adam_idle(b.m[u], b.v[u], b.g[u]);
            if (upd) {
                ngp_step::adam_update(b.p[u].x, b.m[u].x, b.v[u].x, (float)b.g[u][0], ac, aa.beta1, aa.beta2, aa.eps);
                ngp_step::adam_update(b.p[u].y, b.m[u].y, b.v[u].y, (float)b.g[u][1], ac, aa.beta1, aa.beta2, aa.eps);
                ngp_step::adam_update(b.p[u].z, b.m[u].z, b.v[u].z, (float)b.g[u][2], ac, aa.beta1, aa.beta2, aa.eps);
                ngp_step::adam_update(b.p[u].w, b.m[u].w, b.v[u].w, (float)b.g[u][3], ac, aa.beta1, aa.beta2, aa.eps);
                st_f4(tl.p[k] + off, b.p[u]);
                st_f4(tl.m[k] + off, b.m[u]);
                st_f4(tl.v[k] + off, b.v[u]);
            }
            if (tl.ph[k] && (upd || shadow_all))
                *reinterpret_cast<half4*>(tl.ph[k] + off) =
                    half4{(ngp_half)b.p[u].x, (ngp_half)b.p[u].y, (ngp_half)b.p[u].z, (ngp_half)b.p[u].w};
            if (aa.zero_grads && grad_set(b.g[u])) *reinterpret_cast<half4*>(tl.g[k] + off) = half4{0, 0, 0, 0};
        }
    };
    auto seam = [&](uint64_t c) {  // per element (the few chunks across a tensor boundary)
        const uint64_t c0 = c * kChunk, c1 = min(c0 + kChunk, total);
        for (uint64_t i = c0 + tid; i < c1; i += kAdamThreads) {
            const int kk = find_tensor(tl, i);
            const uint64_t off = i - tl.start[kk];
            if (off >= tl.size[kk]) continue;
            float p = tl.p[kk][off];
            if (!skip) {
                float m = tl.m[kk][off], v = tl.v[kk][off];
                ngp_step::adam_update(p, m, v, (float)tl.g[kk][off], ac, aa.beta1, aa.beta2, aa.eps);
                tl.p[kk][off] = p;
                tl.m[kk][off] = m;
                tl.v[kk][off] = v;
            }
            if (tl.ph[kk] && (!skip || shadow_all)) tl.ph[kk][off] = (ngp_half)p;
            if (aa.zero_grads) tl.g[kk][off] = (ngp_half)0.0f;
        }
    };
    auto at = [](uint64_t i) { return i; };
    Buf a{}, b{};
    uint64_t c = blk;
    int ka = c < nchunks ? whole(at(c)) : -1;
    if (ka >= 0) load(at(c), ka, a);
    while (c < nchunks) {
        const uint64_t cn = c + nblk;
        const int kb = cn < nchunks ? whole(at(cn)) : -1;
        if (kb >= 0) load(at(cn), kb, b);  // in flight while this chunk computes
        if (ka >= 0) apply(at(c), ka, a);
        else seam(at(c));
        a = b;
        ka = kb;
        c = cn;
    }
}

}  // namespace ngp_head
