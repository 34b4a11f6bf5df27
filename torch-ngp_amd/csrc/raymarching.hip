// Ray marching over the cascaded density bitfield and volume compositing, gfx950.
//
// Reference semantics (raymarching/src/raymarching.cu):
//   helpers (clamp, signf, mip_from_pos/dt, morton)   :19-81
//   kernel_near_far_from_aabb                         :91-145
//   kernel_sph_from_ray                               :162-198
//   kernel_morton3D / _invert                         :214-254
//   kernel_packbits                                   :267-289
//   kernel_march_rays_train                           :311-480
//   kernel_composite_rays_train_forward / backward    :500-577 / :601-691
//   kernel_march_rays / kernel_composite_rays         :709-814 / :827-914
//
// MI355X design: the reference orders samples
// with two atomicAdd counters (:405-406), so its row order changes run to run.
// Here the per-ray sample counts are turned into offsets by a deterministic
// exclusive prefix sum in ray order: pass 1 counts (and reduces per
// workgroup), a one-workgroup scan turns the workgroup sums into bases, and
// pass 2 re-marches and writes at base + in-workgroup prefix (wave ballot +
// LDS scan). Output is a valid execution of the reference and is identical on
// every run, so parity can compare rows directly.
#include "ngp_common.h"

#include <cfloat>

namespace {

constexpr uint32_t kMarchBlock = 128;
constexpr float kSQRT3 = 1.7320508075688772f;
constexpr float kRPI = 0.3183098861837907f;

NGP_DEV float clampf(float x, float lo, float hi) { return fminf(hi, fmaxf(lo, x)); }
NGP_DEV float signf(float x) { return copysignf(1.0f, x); }

// frexpf exponent of a finite non-negative float, clamped to [0, C-1]
// (mip_from_pos / mip_from_dt, raymarching.cu:42-54).
NGP_DEV int frexp_level(float mx, int max_level) {
    int e = 0;
    if (mx != 0.0f) e = (int)((__float_as_uint(mx) >> 23) & 0xffu) - 126;
    return min(max_level, max(0, e));
}

NGP_DEV uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
NGP_DEV uint32_t morton3D(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
NGP_DEV uint32_t morton3D_invert(uint32_t x) {
    x = x & 0x49249249;
    x = (x | (x >> 2)) & 0xc30c30c3;
    x = (x | (x >> 4)) & 0x0f00f00f;
    x = (x | (x >> 8)) & 0xff0000ff;
    x = (x | (x >> 16)) & 0x0000ffff;
    return x;
}

struct MarchConst {
    float bound, dt_gamma, dt_min, dt_max, rH, H3;
    uint32_t max_steps, C, H;
};

static MarchConst make_march_const(float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
                                   uint32_t H) {
    MarchConst k;
    k.bound = bound;
    k.dt_gamma = dt_gamma;
    k.dt_min = 2 * kSQRT3 / (float)max_steps;
    k.dt_max = 2 * kSQRT3 * (float)(1u << (C - 1)) / (float)H;
    k.rH = 1 / (float)H;
    k.H3 = (float)(H * H * H);
    k.max_steps = max_steps;
    k.C = C;
    k.H = H;
    return k;
}

struct Ray {
    float ox, oy, oz, dx, dy, dz, rdx, rdy, rdz;
};

NGP_DEV Ray load_ray(const float* __restrict__ rays_o, const float* __restrict__ rays_d, size_t i) {
    Ray r;
    r.ox = rays_o[i * 3 + 0]; r.oy = rays_o[i * 3 + 1]; r.oz = rays_o[i * 3 + 2];
    r.dx = rays_d[i * 3 + 0]; r.dy = rays_d[i * 3 + 1]; r.dz = rays_d[i * 3 + 2];
    r.rdx = 1 / r.dx; r.rdy = 1 / r.dy; r.rdz = 1 / r.dz;
    return r;
}

// One marching step decision, shared by the count pass, the write pass and
// inference marching (raymarching.cu:359-400). Returns true if the sample at
// the current t is occupied; otherwise advances t past the empty cell.
struct Sample {
    float x, y, z, dt;
};

NGP_DEV bool march_step(const Ray& r, const MarchConst& k, const uint8_t* __restrict__ grid,
                        float& t, Sample& s) {
    s.x = clampf(fmaf(t, r.dx, r.ox), -k.bound, k.bound);
    s.y = clampf(fmaf(t, r.dy, r.oy), -k.bound, k.bound);
    s.z = clampf(fmaf(t, r.dz, r.oz), -k.bound, k.bound);
    s.dt = clampf(t * k.dt_gamma, k.dt_min, k.dt_max);

    const int maxl = (int)k.C - 1;
    const float mxp = fmaxf(fabsf(s.x), fmaxf(fabsf(s.y), fabsf(s.z)));
    const float mxd = s.dt * (float)k.H * 0.5f;
    const int level = max(frexp_level(mxp, maxl), frexp_level(mxd, maxl));

    const float mip_bound = fminf(scalbnf(1.0f, level), k.bound);
    const float mip_rbound = 1 / mip_bound;
    const float Hm1 = (float)(k.H - 1);
    const int nx = (int)clampf(0.5f * fmaf(s.x, mip_rbound, 1.0f) * (float)k.H, 0.0f, Hm1);
    const int ny = (int)clampf(0.5f * fmaf(s.y, mip_rbound, 1.0f) * (float)k.H, 0.0f, Hm1);
    const int nz = (int)clampf(0.5f * fmaf(s.z, mip_rbound, 1.0f) * (float)k.H, 0.0f, Hm1);

    const uint32_t index = (uint32_t)((float)level * k.H3 + (float)morton3D(nx, ny, nz));
    const bool occ = grid[index / 8] & (1u << (index % 8));
    if (occ) return true;

    const float tx = ((((float)nx + 0.5f + 0.5f * signf(r.dx)) * k.rH * 2 - 1) * mip_bound - s.x) * r.rdx;
    const float ty = ((((float)ny + 0.5f + 0.5f * signf(r.dy)) * k.rH * 2 - 1) * mip_bound - s.y) * r.rdy;
    const float tz = ((((float)nz + 0.5f + 0.5f * signf(r.dz)) * k.rH * 2 - 1) * mip_bound - s.z) * r.rdz;
    const float tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    do {
        t += clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
    } while (t < tt);
    return false;
}

NGP_DEV float ray_t0(float near, float noise, const MarchConst& k) {
    return fmaf(clampf(near * k.dt_gamma, k.dt_min, k.dt_max), noise, near);
}

// ---- kernels -----------------------------------------------------------------

__global__ void __launch_bounds__(128)
k_near_far(const float* __restrict__ rays_o, const float* __restrict__ rays_d,
           const float* __restrict__ aabb, uint32_t N, float min_near, float* nears,
           float* fars) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const Ray r = load_ray(rays_o, rays_d, n);
    float near = (aabb[0] - r.ox) * r.rdx;
    float far = (aabb[3] - r.ox) * r.rdx;
    if (near > far) { float c = near; near = far; far = c; }
    float near_y = (aabb[1] - r.oy) * r.rdy;
    float far_y = (aabb[4] - r.oy) * r.rdy;
    if (near_y > far_y) { float c = near_y; near_y = far_y; far_y = c; }
    if (near > far_y || near_y > far) { nears[n] = fars[n] = FLT_MAX; return; }
    if (near_y > near) near = near_y;
    if (far_y < far) far = far_y;
    float near_z = (aabb[2] - r.oz) * r.rdz;
    float far_z = (aabb[5] - r.oz) * r.rdz;
    if (near_z > far_z) { float c = near_z; near_z = far_z; far_z = c; }
    if (near > far_z || near_z > far) { nears[n] = fars[n] = FLT_MAX; return; }
    if (near_z > near) near = near_z;
    if (far_z < far) far = far_z;
    if (near < min_near) near = min_near;
    nears[n] = near;
    fars[n] = far;
}

__global__ void __launch_bounds__(128)
k_sph_from_ray(const float* __restrict__ rays_o, const float* __restrict__ rays_d, float radius,
               uint32_t N, float* coords) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const float ox = rays_o[n * 3], oy = rays_o[n * 3 + 1], oz = rays_o[n * 3 + 2];
    const float dx = rays_d[n * 3], dy = rays_d[n * 3 + 1], dz = rays_d[n * 3 + 2];
    const float A = dx * dx + dy * dy + dz * dz;
    const float Bh = ox * dx + oy * dy + oz * dz;
    const float Cc = ox * ox + oy * oy + oz * oz - radius * radius;
    const float t = (-Bh + sqrtf(Bh * Bh - A * Cc)) / A;
    const float x = ox + t * dx, y = oy + t * dy, z = oz + t * dz;
    const float theta = atan2f(sqrtf(x * x + z * z), y);
    const float phi = atan2f(z, x);
    coords[n * 2] = 2 * theta * kRPI - 1;
    coords[n * 2 + 1] = phi * kRPI;
}

__global__ void k_morton3D(const int32_t* __restrict__ coords, uint32_t N, int32_t* indices) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    indices[n] = (int32_t)morton3D(coords[n * 3], coords[n * 3 + 1], coords[n * 3 + 2]);
}

__global__ void k_morton3D_invert(const int32_t* __restrict__ indices, uint32_t N, int32_t* coords) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const uint32_t ind = (uint32_t)indices[n];
    coords[n * 3 + 0] = (int32_t)morton3D_invert(ind >> 0);
    coords[n * 3 + 1] = (int32_t)morton3D_invert(ind >> 1);
    coords[n * 3 + 2] = (int32_t)morton3D_invert(ind >> 2);
}

// 8 cells -> 1 byte; each lane reads 32 contiguous bytes (two dwordx4).
__global__ void k_packbits(const float* __restrict__ grid, uint32_t N, float thresh, uint8_t* bitfield) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const float4* g = reinterpret_cast<const float4*>(grid + (size_t)n * 8);
    const float4 a = g[0], b = g[1];
    uint32_t bits = 0;
    bits |= (a.x > thresh) ? 1u : 0u;
    bits |= (a.y > thresh) ? 2u : 0u;
    bits |= (a.z > thresh) ? 4u : 0u;
    bits |= (a.w > thresh) ? 8u : 0u;
    bits |= (b.x > thresh) ? 16u : 0u;
    bits |= (b.y > thresh) ? 32u : 0u;
    bits |= (b.z > thresh) ? 64u : 0u;
    bits |= (b.w > thresh) ? 128u : 0u;
    bitfield[n] = (uint8_t)bits;
}

// Workgroup-wide exclusive scan of one uint32 per thread (kMarchBlock threads):
// wave-level scan with DPP-free shuffles, then the two wave totals via LDS.
NGP_DEV uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds_waves, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    uint32_t incl = v;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if (lane >= o) incl += u;
    }
    if (lane == 63) lds_waves[wave] = incl;
    __syncthreads();
    uint32_t wave_base = 0;
    total = 0;
    for (uint32_t w = 0; w < kMarchBlock / 64; ++w) {
        const uint32_t s = lds_waves[w];
        if (w < wave) wave_base += s;
        total += s;
    }
    return wave_base + incl - v;
}

// Pass 1: count samples per ray; rays[n] = (n, -, count). The workgroup's sum is
// parked in the offset column of its first ray (rays[first*3+1]).
__global__ void __launch_bounds__(kMarchBlock)
k_march_count(const float* __restrict__ rays_o, const float* __restrict__ rays_d,
              const uint8_t* __restrict__ grid, MarchConst k, uint32_t N,
              const float* __restrict__ nears, const float* __restrict__ fars,
              const float* __restrict__ noises, int32_t* __restrict__ rays) {
    __shared__ uint32_t lds_waves[kMarchBlock / 64];
    const uint32_t n = blockIdx.x * kMarchBlock + threadIdx.x;
    uint32_t num_steps = 0;
    if (n < N) {
        const Ray r = load_ray(rays_o, rays_d, n);
        const float far = fars[n];
        float t = ray_t0(nears[n], noises[n], k);
        Sample s;
        while (t < far && num_steps < k.max_steps) {
            if (march_step(r, k, grid, t, s)) {
                num_steps++;
                t += s.dt;
            }
        }
        rays[n * 3 + 0] = (int32_t)n;
        rays[n * 3 + 2] = (int32_t)num_steps;
    }
    uint32_t total;
    block_exclusive_scan(num_steps, lds_waves, total);
    if (threadIdx.x == 0) rays[(size_t)blockIdx.x * kMarchBlock * 3 + 1] = (int32_t)total;
}

// One workgroup: exclusive scan over the per-workgroup sums (in place), then
// counter[0] += total, counter[1] += N.
__global__ void __launch_bounds__(1024)
k_march_scan(int32_t* __restrict__ rays, uint32_t num_blocks, uint32_t N, int32_t* counter) {
    __shared__ uint32_t lds[1024];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = (uint32_t)counter[0];
    __syncthreads();
    for (uint32_t base = 0; base < num_blocks; base += 1024) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < num_blocks ? (uint32_t)rays[(size_t)i * kMarchBlock * 3 + 1] : 0u;
        lds[threadIdx.x] = v;
        __syncthreads();
        // Hillis-Steele inclusive scan in LDS (num_blocks is small: N / 128).
        for (uint32_t o = 1; o < 1024; o <<= 1) {
            const uint32_t u = threadIdx.x >= o ? lds[threadIdx.x - o] : 0u;
            __syncthreads();
            lds[threadIdx.x] += u;
            __syncthreads();
        }
        const uint32_t excl = carry + lds[threadIdx.x] - v;
        if (i < num_blocks) rays[(size_t)i * kMarchBlock * 3 + 1] = (int32_t)excl;
        __syncthreads();
        if (threadIdx.x == 1023) carry += lds[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        counter[0] = (int32_t)carry;
        counter[1] += (int32_t)N;
    }
}

// Pass 2: offsets = workgroup base + in-workgroup prefix; re-march and write.
__global__ void __launch_bounds__(kMarchBlock)
k_march_write(const float* __restrict__ rays_o, const float* __restrict__ rays_d,
              const uint8_t* __restrict__ grid, MarchConst k, uint32_t N, uint32_t M,
              const float* __restrict__ nears, const float* __restrict__ fars,
              const float* __restrict__ noises, float* __restrict__ xyzs,
              float* __restrict__ dirs, float* __restrict__ deltas, int32_t* __restrict__ rays) {
    __shared__ uint32_t lds_waves[kMarchBlock / 64];
    const uint32_t n = blockIdx.x * kMarchBlock + threadIdx.x;
    const uint32_t block_base = (uint32_t)rays[(size_t)blockIdx.x * kMarchBlock * 3 + 1];
    const uint32_t num_steps = n < N ? (uint32_t)rays[n * 3 + 2] : 0u;
    __syncthreads();  // every lane has read the parked base before lane 0 overwrites it
    uint32_t total;
    const uint32_t point_index = block_base + block_exclusive_scan(num_steps, lds_waves, total);
    if (n >= N) return;
    rays[n * 3 + 1] = (int32_t)point_index;
    if (num_steps == 0) return;
    if (point_index + num_steps > M) return;

    const Ray r = load_ray(rays_o, rays_d, n);
    const float far = fars[n];
    float t = ray_t0(nears[n], noises[n], k);
    float last_t = t;
    float* xyz = xyzs + (size_t)point_index * 3;
    float* dir = dirs + (size_t)point_index * 3;
    float* dlt = deltas + (size_t)point_index * 2;
    uint32_t step = 0;
    Sample s;
    while (t < far && step < num_steps) {
        if (march_step(r, k, grid, t, s)) {
            xyz[0] = s.x; xyz[1] = s.y; xyz[2] = s.z;
            dir[0] = r.dx; dir[1] = r.dy; dir[2] = r.dz;
            t += s.dt;
            dlt[0] = s.dt;
            dlt[1] = t - last_t;
            last_t = t;
            xyz += 3; dir += 3; dlt += 2;
            step++;
        }
    }
}

__global__ void __launch_bounds__(128)
k_composite_train_fwd(const float* __restrict__ sigmas, const float* __restrict__ rgbs,
                      const float* __restrict__ deltas, const int32_t* __restrict__ rays,
                      uint32_t M, uint32_t N, float T_thresh, float* weights_sum, float* depth,
                      float* image) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const uint32_t index = (uint32_t)rays[n * 3];
    const uint32_t offset = (uint32_t)rays[n * 3 + 1];
    const uint32_t num_steps = (uint32_t)rays[n * 3 + 2];
    if (num_steps == 0 || offset + num_steps > M) {
        weights_sum[index] = 0;
        depth[index] = 0;
        image[index * 3] = 0;
        image[index * 3 + 1] = 0;
        image[index * 3 + 2] = 0;
        return;
    }
    const float* sg = sigmas + offset;
    const float* cl = rgbs + (size_t)offset * 3;
    const float* dl = deltas + (size_t)offset * 2;
    float T = 1.0f;
    float r = 0, g = 0, b = 0, ws = 0, t = 0, d = 0;
    for (uint32_t step = 0; step < num_steps; ++step) {
        const float alpha = 1.0f - expf(-sg[step] * dl[step * 2]);
        const float weight = alpha * T;
        r = fmaf(weight, cl[step * 3 + 0], r);
        g = fmaf(weight, cl[step * 3 + 1], g);
        b = fmaf(weight, cl[step * 3 + 2], b);
        t += dl[step * 2 + 1];
        d = fmaf(weight, t, d);
        ws += weight;
        T *= 1.0f - alpha;
        if (T < T_thresh) break;
    }
    weights_sum[index] = ws;
    depth[index] = d;
    image[index * 3] = r;
    image[index * 3 + 1] = g;
    image[index * 3 + 2] = b;
}

__global__ void __launch_bounds__(128)
k_composite_train_bwd(const float* __restrict__ grad_weights_sum, const float* __restrict__ grad_depth,
                      const float* __restrict__ grad_image, const float* __restrict__ sigmas,
                      const float* __restrict__ rgbs, const float* __restrict__ deltas,
                      const int32_t* __restrict__ rays, const float* __restrict__ weights_sum,
                      const float* __restrict__ depth, const float* __restrict__ image, uint32_t M,
                      uint32_t N, float T_thresh, float* grad_sigmas, float* grad_rgbs) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    const uint32_t index = (uint32_t)rays[n * 3];
    const uint32_t offset = (uint32_t)rays[n * 3 + 1];
    const uint32_t num_steps = (uint32_t)rays[n * 3 + 2];
    if (num_steps == 0 || offset + num_steps > M) return;

    const float gws = grad_weights_sum[index], gd = grad_depth[index];
    const float gr = grad_image[index * 3], gg = grad_image[index * 3 + 1], gb = grad_image[index * 3 + 2];
    const float r_final = image[index * 3], g_final = image[index * 3 + 1], b_final = image[index * 3 + 2];
    const float ws_final = weights_sum[index], d_final = depth[index];
    const float* sg = sigmas + offset;
    const float* cl = rgbs + (size_t)offset * 3;
    const float* dl = deltas + (size_t)offset * 2;
    float* gs = grad_sigmas + offset;
    float* gc = grad_rgbs + (size_t)offset * 3;

    float T = 1.0f;
    float r = 0, g = 0, b = 0, t = 0, d = 0;
    for (uint32_t step = 0; step < num_steps; ++step) {
        const float c0 = cl[step * 3 + 0], c1 = cl[step * 3 + 1], c2 = cl[step * 3 + 2];
        const float d0 = dl[step * 2];
        const float alpha = 1.0f - expf(-sg[step] * d0);
        const float weight = alpha * T;
        r = fmaf(weight, c0, r);
        g = fmaf(weight, c1, g);
        b = fmaf(weight, c2, b);
        t += dl[step * 2 + 1];
        d = fmaf(weight, t, d);
        T *= 1.0f - alpha;
        gc[step * 3 + 0] = gr * weight;
        gc[step * 3 + 1] = gg * weight;
        gc[step * 3 + 2] = gb * weight;
        gs[step] = d0 * (gr * (T * c0 - (r_final - r)) +
                         gg * (T * c1 - (g_final - g)) +
                         gb * (T * c2 - (b_final - b)) +
                         gd * (T * t - (d_final - d)) +
                         gws * (1 - ws_final));
        if (T < T_thresh) break;
    }
}

__global__ void __launch_bounds__(128)
k_march_rays(uint32_t n_alive, uint32_t n_step, const int32_t* __restrict__ rays_alive,
             const float* __restrict__ rays_t, const float* __restrict__ rays_o,
             const float* __restrict__ rays_d, MarchConst k, const uint8_t* __restrict__ grid,
             const float* __restrict__ nears, const float* __restrict__ fars, float* xyzs,
             float* dirs, float* deltas, const float* __restrict__ noises) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    const int index = rays_alive[n];
    const float noise = noises[n];
    const Ray r = load_ray(rays_o, rays_d, (size_t)index);
    float* xyz = xyzs + (size_t)n * n_step * 3;
    float* dir = dirs + (size_t)n * n_step * 3;
    float* dlt = deltas + (size_t)n * n_step * 2;
    float t = rays_t[index];
    const float far = fars[index];
    t = fmaf(clampf(t * k.dt_gamma, k.dt_min, k.dt_max), noise, t);
    float last_t = t;
    uint32_t step = 0;
    Sample s;
    while (t < far && step < n_step) {
        if (march_step(r, k, grid, t, s)) {
            xyz[0] = s.x; xyz[1] = s.y; xyz[2] = s.z;
            dir[0] = r.dx; dir[1] = r.dy; dir[2] = r.dz;
            t += s.dt;
            dlt[0] = s.dt;
            dlt[1] = t - last_t;
            last_t = t;
            xyz += 3; dir += 3; dlt += 2;
            step++;
        }
    }
}

__global__ void __launch_bounds__(128)
k_composite_rays(uint32_t n_alive, uint32_t n_step, float T_thresh, int32_t* rays_alive,
                 float* rays_t, const float* __restrict__ sigmas, const float* __restrict__ rgbs,
                 const float* __restrict__ deltas, float* weights_sum, float* depth, float* image) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_alive) return;
    const int index = rays_alive[n];
    const float* sg = sigmas + (size_t)n * n_step;
    const float* cl = rgbs + (size_t)n * n_step * 3;
    const float* dl = deltas + (size_t)n * n_step * 2;
    float t = rays_t[index];
    float weight_sum = weights_sum[index];
    float d = depth[index];
    float r = image[index * 3], g = image[index * 3 + 1], b = image[index * 3 + 2];
    uint32_t step = 0;
    while (step < n_step) {
        const float d0 = dl[step * 2];
        if (d0 == 0) break;
        const float alpha = 1.0f - expf(-sg[step] * d0);
        const float T = 1 - weight_sum;
        const float weight = alpha * T;
        weight_sum += weight;
        t += dl[step * 2 + 1];
        d = fmaf(weight, t, d);
        r = fmaf(weight, cl[step * 3 + 0], r);
        g = fmaf(weight, cl[step * 3 + 1], g);
        b = fmaf(weight, cl[step * 3 + 2], b);
        if (T < T_thresh) break;
        step++;
    }
    if (step < n_step) rays_alive[n] = -1;
    else rays_t[index] = t;
    weights_sum[index] = weight_sum;
    depth[index] = d;
    image[index * 3] = r;
    image[index * 3 + 1] = g;
    image[index * 3 + 2] = b;
}

int check_cascade(uint32_t C, uint32_t H, uint32_t max_steps) {
    NGP_REQUIRE(C >= 1 && C <= 8, NGP_ERR_ARG, "raymarching: cascade C must be in [1, 8], got %u", C);
    NGP_REQUIRE(H >= 1 && H <= 1024, NGP_ERR_ARG, "raymarching: grid size H must be in [1, 1024], got %u", H);
    NGP_REQUIRE(max_steps >= 1, NGP_ERR_ARG, "raymarching: max_steps must be >= 1");
    return NGP_OK;
}

}  // namespace

extern "C" int ngp_near_far_from_aabb(const float* rays_o, const float* rays_d, const float* aabb,
                                      uint32_t N, float min_near, float* nears, float* fars,
                                      void* stream) {
    if (N == 0) return NGP_OK;
    k_near_far<<<ngp_div_up(N, 128), 128, 0, ngp_stream(stream)>>>(rays_o, rays_d, aabb, N, min_near, nears, fars);
    return ngp_check_launch("near_far_from_aabb");
}

extern "C" int ngp_sph_from_ray(const float* rays_o, const float* rays_d, float radius, uint32_t N,
                                float* coords, void* stream) {
    if (N == 0) return NGP_OK;
    k_sph_from_ray<<<ngp_div_up(N, 128), 128, 0, ngp_stream(stream)>>>(rays_o, rays_d, radius, N, coords);
    return ngp_check_launch("sph_from_ray");
}

extern "C" int ngp_morton3D(const int32_t* coords, uint32_t N, int32_t* indices, void* stream) {
    if (N == 0) return NGP_OK;
    k_morton3D<<<ngp_div_up(N, 256), 256, 0, ngp_stream(stream)>>>(coords, N, indices);
    return ngp_check_launch("morton3D");
}

extern "C" int ngp_morton3D_invert(const int32_t* indices, uint32_t N, int32_t* coords, void* stream) {
    if (N == 0) return NGP_OK;
    k_morton3D_invert<<<ngp_div_up(N, 256), 256, 0, ngp_stream(stream)>>>(indices, N, coords);
    return ngp_check_launch("morton3D_invert");
}

extern "C" int ngp_packbits(const float* grid, uint32_t N, float density_thresh, uint8_t* bitfield,
                            void* stream) {
    if (N == 0) return NGP_OK;
    NGP_REQUIRE((reinterpret_cast<uintptr_t>(grid) & 15) == 0, NGP_ERR_ARG, "packbits: grid must be 16-byte aligned");
    k_packbits<<<ngp_div_up(N, 256), 256, 0, ngp_stream(stream)>>>(grid, N, density_thresh, bitfield);
    return ngp_check_launch("packbits");
}

extern "C" int ngp_march_rays_train(const float* rays_o, const float* rays_d, const uint8_t* grid,
                                    float bound, float dt_gamma, uint32_t max_steps, uint32_t N,
                                    uint32_t C, uint32_t H, uint32_t M, const float* nears,
                                    const float* fars, float* xyzs, float* dirs, float* deltas,
                                    int32_t* rays, int32_t* counter, const float* noises,
                                    void* stream) {
    if (int e = check_cascade(C, H, max_steps)) return e;
    NGP_REQUIRE(rays && counter, NGP_ERR_ARG, "march_rays_train: null rays/counter");
    if (N == 0) return NGP_OK;
    const MarchConst k = make_march_const(bound, dt_gamma, max_steps, C, H);
    hipStream_t st = ngp_stream(stream);
    const uint32_t nb = ngp_div_up(N, kMarchBlock);
    k_march_count<<<nb, kMarchBlock, 0, st>>>(rays_o, rays_d, grid, k, N, nears, fars, noises, rays);
    k_march_scan<<<1, 1024, 0, st>>>(rays, nb, N, counter);
    k_march_write<<<nb, kMarchBlock, 0, st>>>(rays_o, rays_d, grid, k, N, M, nears, fars, noises,
                                              xyzs, dirs, deltas, rays);
    return ngp_check_launch("march_rays_train");
}

extern "C" int ngp_composite_rays_train_forward(const float* sigmas, const float* rgbs,
                                                const float* deltas, const int32_t* rays,
                                                uint32_t M, uint32_t N, float T_thresh,
                                                float* weights_sum, float* depth, float* image,
                                                void* stream) {
    if (N == 0) return NGP_OK;
    k_composite_train_fwd<<<ngp_div_up(N, 128), 128, 0, ngp_stream(stream)>>>(
        sigmas, rgbs, deltas, rays, M, N, T_thresh, weights_sum, depth, image);
    return ngp_check_launch("composite_rays_train_forward");
}

extern "C" int ngp_composite_rays_train_backward(const float* grad_weights_sum,
                                                 const float* grad_depth, const float* grad_image,
                                                 const float* sigmas, const float* rgbs,
                                                 const float* deltas, const int32_t* rays,
                                                 const float* weights_sum, const float* depth,
                                                 const float* image, uint32_t M, uint32_t N,
                                                 float T_thresh, float* grad_sigmas,
                                                 float* grad_rgbs, void* stream) {
    if (N == 0) return NGP_OK;
    k_composite_train_bwd<<<ngp_div_up(N, 128), 128, 0, ngp_stream(stream)>>>(
        grad_weights_sum, grad_depth, grad_image, sigmas, rgbs, deltas, rays, weights_sum, depth,
        image, M, N, T_thresh, grad_sigmas, grad_rgbs);
    return ngp_check_launch("composite_rays_train_backward");
}

extern "C" int ngp_march_rays(uint32_t n_alive, uint32_t n_step, const int32_t* rays_alive,
                              const float* rays_t, const float* rays_o, const float* rays_d,
                              float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
                              uint32_t H, const uint8_t* grid, const float* nears,
                              const float* fars, float* xyzs, float* dirs, float* deltas,
                              const float* noises, void* stream) {
    if (int e = check_cascade(C, H, max_steps)) return e;
    if (n_alive == 0) return NGP_OK;
    const MarchConst k = make_march_const(bound, dt_gamma, max_steps, C, H);
    k_march_rays<<<ngp_div_up(n_alive, 128), 128, 0, ngp_stream(stream)>>>(
        n_alive, n_step, rays_alive, rays_t, rays_o, rays_d, k, grid, nears, fars, xyzs, dirs,
        deltas, noises);
    return ngp_check_launch("march_rays");
}

extern "C" int ngp_composite_rays(uint32_t n_alive, uint32_t n_step, float T_thresh,
                                  int32_t* rays_alive, float* rays_t, const float* sigmas,
                                  const float* rgbs, const float* deltas, float* weights_sum,
                                  float* depth, float* image, void* stream) {
    if (n_alive == 0) return NGP_OK;
    k_composite_rays<<<ngp_div_up(n_alive, 128), 128, 0, ngp_stream(stream)>>>(
        n_alive, n_step, T_thresh, rays_alive, rays_t, sigmas, rgbs, deltas, weights_sum, depth,
        image);
    return ngp_check_launch("composite_rays");
}
