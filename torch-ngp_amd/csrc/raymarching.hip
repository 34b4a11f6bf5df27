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
// MI355X design:
//   * the reference orders samples with two atomicAdd counters (:405-406), so
//     its row order changes run to run. Here offsets are a deterministic
//     exclusive prefix sum in ray order; the output is a valid execution of the
//     reference and identical on every run, so parity compares rows directly;
//   * each ray is marched ONCE (the reference marches twice): the t of every
//     occupied sample goes to a workspace row, and a flat per-sample pass
//     writes xyzs/dirs/deltas at the scanned offsets;
//   * occupancy lookups hit an LDS rank/select image of the bitfield (OccLds)
//     instead of L2: marching is a serial dependency chain per ray, so the
//     lookup latency is the step time.
#include "ffmlp_pack.h"
#include "ngp_common.h"
#include "ngp_dpp.h"
#include "ngp_head.h"
#include "ngp_step.h"

#include <algorithm>
#include <cfloat>

namespace {

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
    float bound, rbound, dt_gamma, dt_min, dt_max, rH, H3;
    uint32_t max_steps, C, H;
};

static MarchConst make_march_const(float bound, float dt_gamma, uint32_t max_steps, uint32_t C,
                                   uint32_t H) {
    MarchConst k;
    k.bound = bound;
    k.rbound = 1 / bound;  // IEEE division, as the device's 1 / mip_bound
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

// ---- occupancy lookups ----------------------------------------------------------
// Bit `index` of the cascaded bitfield, straight from HBM/L2.
struct OccGlobal {
    const uint8_t* __restrict__ grid;
    NGP_DEV bool operator()(uint32_t index) const { return (grid[index >> 3] >> (index & 7)) & 1u; }
};

// LDS-resident rank/select image of the bitfield (built per workgroup by
// k_occ_count/k_occ_compact, copied in by load_occ_index). Because Morton order interleaves the coordinate bits,
// bitfield byte b holds exactly the 2x2x2 cells of coarse cell b, so:
//   sum[w]   bit i  = (grid byte 32w+i != 0)          (coarse occupancy, 1 bit/byte)
//   pre[g]          = non-zero bytes before word 4g   (rank directory)
//   bytes[]         = the non-zero grid bytes, in order
// A lookup in empty space costs one ds_read_b128; an occupied coarse cell one
// more LDS read. The marching loop never waits on L2 (~10x the latency).
struct OccLds {
    const uint32_t* sum;
    const uint32_t* pre;
    const uint8_t* bytes;
    NGP_DEV bool operator()(uint32_t index) const {
        const uint32_t byte = index >> 3, w = byte >> 5, g = w >> 2, j = w & 3, bit = byte & 31;
        const uint4 q = reinterpret_cast<const uint4*>(sum)[g];
        const uint32_t m = j == 0 ? q.x : j == 1 ? q.y : j == 2 ? q.z : q.w;
        if (!((m >> bit) & 1u)) return false;
        uint32_t pos = pre[g] + __popc(m & ((1u << bit) - 1u));
        if (j > 0) pos += __popc(q.x);
        if (j > 1) pos += __popc(q.y);
        if (j > 2) pos += __popc(q.z);
        return (bytes[pos] >> (index & 7)) & 1u;
    }
};

// One marching step decision, shared by training and inference marching
// (raymarching.cu:359-400). Returns true if the sample at the current t is
// occupied; otherwise advances t past the empty cell.
struct Sample {
    float x, y, z, dt;
};

// ONE_LEVEL: C == 1, where both mip levels clamp to 0 (every Lego config).
// mip_rbound = 1 / min(2^level, bound) without a division: 2^-level is exact
// when 2^level <= bound, otherwise it is the host's IEEE 1 / bound.
// probe: the occupancy decision at t and the DDA skip target tt of its cell.
template <bool ONE_LEVEL, typename OCC>
NGP_DEV bool probe(const Ray& r, const MarchConst& k, const OCC& occupied, float t, Sample& s, float& tt) {
    s.x = clampf(fmaf(t, r.dx, r.ox), -k.bound, k.bound);
    s.y = clampf(fmaf(t, r.dy, r.oy), -k.bound, k.bound);
    s.z = clampf(fmaf(t, r.dz, r.oz), -k.bound, k.bound);
    s.dt = clampf(t * k.dt_gamma, k.dt_min, k.dt_max);

    int level = 0;
    if (!ONE_LEVEL) {
        const int maxl = (int)k.C - 1;
        const float mxp = fmaxf(fabsf(s.x), fmaxf(fabsf(s.y), fabsf(s.z)));
        const float mxd = s.dt * (float)k.H * 0.5f;
        level = max(frexp_level(mxp, maxl), frexp_level(mxd, maxl));
    }
    const float p2 = scalbnf(1.0f, level);
    const float mip_bound = fminf(p2, k.bound);
    const float mip_rbound = p2 <= k.bound ? scalbnf(1.0f, -level) : k.rbound;
    const float Hm1 = (float)(k.H - 1);
    const int nx = (int)clampf(0.5f * fmaf(s.x, mip_rbound, 1.0f) * (float)k.H, 0.0f, Hm1);
    const int ny = (int)clampf(0.5f * fmaf(s.y, mip_rbound, 1.0f) * (float)k.H, 0.0f, Hm1);
    const int nz = (int)clampf(0.5f * fmaf(s.z, mip_rbound, 1.0f) * (float)k.H, 0.0f, Hm1);

    const uint32_t index = (uint32_t)((float)level * k.H3 + (float)morton3D(nx, ny, nz));
    // the skip target does not depend on the lookup: computed in its shadow
    const float tx = ((((float)nx + 0.5f + 0.5f * signf(r.dx)) * k.rH * 2 - 1) * mip_bound - s.x) * r.rdx;
    const float ty = ((((float)ny + 0.5f + 0.5f * signf(r.dy)) * k.rH * 2 - 1) * mip_bound - s.y) * r.rdy;
    const float tz = ((((float)nz + 0.5f + 0.5f * signf(r.dz)) * k.rH * 2 - 1) * mip_bound - s.z) * r.rdz;
    tt = t + fmaxf(0.0f, fminf(tx, fminf(ty, tz)));
    return occupied(index);
}

template <bool ONE_LEVEL, typename OCC>
NGP_DEV bool march_step(const Ray& r, const MarchConst& k, const OCC& occupied, float& t, Sample& s) {
    float tt;
    if (probe<ONE_LEVEL>(r, k, occupied, t, s, tt)) return true;
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

// Workgroup-wide exclusive scan of one uint32 per thread (BLOCK threads):
// wave-level shuffle scan, then the wave totals via LDS. Ends with a barrier,
// so lds_waves can be reused right away.
template <uint32_t BLOCK>
NGP_DEV uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds_waves, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t incl = ngp_dpp::scan_incl_u32(v);  // DPP: no LDS-crossbar round trips
    if (lane == 63) lds_waves[wave] = incl;
    __syncthreads();
    uint32_t wave_base = 0;
    total = 0;
#pragma unroll
    for (uint32_t w = 0; w < BLOCK / 64; ++w) {
        const uint32_t s = lds_waves[w];
        if (w < wave) wave_base += s;
        total += s;
    }
    __syncthreads();
    return wave_base + incl - v;
}

// ---- march_rays_train ------------------------------------------------------------
// Three kernels, all deterministic:
//   k_march_train  one WAVE per ray (below): the t of every occupied sample goes
//                  to the workspace row ts[n][0..count), rays[n] = (n, -, count)
//   k_march_emit   per SAMPLE (flat, balanced): each workgroup forms its ray
//                  group's offsets itself (counts of all earlier rays + an
//                  in-group scan: an exclusive scan in ray order, no separate
//                  scan launch), writes rays[n].offset and counter, then
//                  xyzs/dirs/deltas recomputed from the recorded t with the
//                  reference's exact float ops
//
// Why one wave per ray. Marching is a serial recurrence on t: ~150-500 probes
// per Lego ray, ~130 dependent VALU each. One lane per ray gives 64 waves for
// 4096 rays — 1/16 of the SIMDs, each a pure latency chain. But the state of
// the recurrence is only t, and t only ever moves along ONE chain:
//     t_0 = near + noise * dt0,   t_{k+1} = t_k + clamp(t_k * dt_gamma, ...)
// (an occupied step and every iteration of the DDA skip loop apply the same
// update). A probe at chain index k goes to k+1 (occupied) or to the first j
// with t_j >= tt(t_k) (empty). So with dt_gamma == 0, where t_k has a closed
// form per binade (advance0), the chain splits into 64 index segments: lane s
// walks segment s speculatively from its first index, then the true walk is
// stitched across segments (a walk that reaches an index the speculative walk
// visited continues identically from there). With dt_gamma > 0 there is no
// closed form: the wave steps the bare chain first (three VALU operations per
// index against a probe's ~130 and its LDS/L2 lookups) and keeps every 16th t
// (ChainGamma). Exact for every ray; chains over 64 x 64 indices are marched
// serially by lane 0 (the reference loop).
constexpr uint32_t kMarchThreads = 256;   // rays per k_march_emit group
constexpr uint32_t kSegWaves = 16;        // rays (waves) per march workgroup
constexpr uint32_t kSegThreads = kSegWaves * 64;
constexpr uint32_t kMaxMarchBlocks = 256;
constexpr size_t kMarchLdsBytes = 156 * 1024;
// workgroups per ray group in k_march_emit: 8 left half the SIMDs idle on a
// 4096-ray batch (16 groups); 32 (same box, profiles/r04w_emit_split_ab.txt):
// the march + emit tick 33.6 -> 30.8 us
constexpr uint32_t kEmitSplit = 32;
constexpr uint32_t kInf = 0xffffffffu;

struct OccLayout {
    uint32_t nbytes, nwords, ngroups, cap;  // cap = LDS bytes left for the compacted bytes
};

// Global occupancy image (workspace), laid out exactly as OccLds in LDS:
//   [total (16 B)] [sum: 4 words / group] [pre: 1 word / group] [bytes]
NGP_DEV uint32_t* occ_sum(uint8_t* img) { return reinterpret_cast<uint32_t*>(img + 16); }

// 32 bitfield bytes starting at 32w as 8 dwords (vector loads when in range).
NGP_DEV void load_word32(const uint8_t* __restrict__ grid, uint32_t w, uint32_t nbytes, uint32_t (&d)[8]) {
    if (32 * w + 32 <= nbytes) {
        const uint4* g = reinterpret_cast<const uint4*>(grid + 32 * (size_t)w);
        const uint4 a = g[0], b = g[1];
        d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
        return;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = 0;
    for (uint32_t i = 0; i < 32 && 32 * w + i < nbytes; ++i) d[i >> 2] |= (uint32_t)grid[32 * w + i] << (8 * (i & 3));
}

NGP_DEV uint32_t nonzero_bytes(const uint32_t (&d)[8]) {
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) m |= ((d[i] >> (8 * j)) & 0xffu) ? (1u << (4 * i + j)) : 0u;
    return m;
}

// Two kernels build the image:
//   k_occ_count    summary words + per-group counts (count scratch after the
//                  image), 256 groups (32 KB of bitfield) per workgroup
//   k_occ_compact  one wave per group: base = counts of all earlier groups
//                  (each workgroup sums them itself: a few thousand L2 reads)
//                  -> rank directory, then the non-zero bytes written in order
constexpr uint32_t kBuildThreads = 256;
__global__ void __launch_bounds__(kBuildThreads)
k_occ_count(const uint8_t* __restrict__ grid, OccLayout L, uint8_t* __restrict__ img,
            uint32_t* __restrict__ cnt) {
    const uint32_t g = blockIdx.x * kBuildThreads + threadIdx.x;
    if (g >= L.ngroups) return;
    uint32_t d[4][8];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) load_word32(grid, 4 * g + i, L.nbytes, d[i]);
    uint32_t c = 0;
    uint4 m;
    m.x = nonzero_bytes(d[0]);
    m.y = nonzero_bytes(d[1]);
    m.z = nonzero_bytes(d[2]);
    m.w = nonzero_bytes(d[3]);
    reinterpret_cast<uint4*>(occ_sum(img))[g] = m;
    c = __popc(m.x) + __popc(m.y) + __popc(m.z) + __popc(m.w);
    cnt[g] = c;
}

// One wave per group (its 128 bitfield bytes, two per lane): the group's base
// is the sum of every earlier group's count (the workgroup's 256 threads sum
// them together, loads batched), each nonzero byte's rank inside the group
// comes from two ballots and mbcnt. (One thread per group walked its 128
// bytes serially: 8 workgroups for a 128^3 grid, ~14 us.)
constexpr uint32_t kCompactGroups = kBuildThreads / 64;
__global__ void __launch_bounds__(kBuildThreads)
k_occ_compact(const uint8_t* __restrict__ grid, OccLayout L, uint8_t* __restrict__ img,
              const uint32_t* __restrict__ cnt) {
    __shared__ uint32_t s_w[kBuildThreads / 64];
    __shared__ uint32_t s_cnt[kCompactGroups];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t g0 = blockIdx.x * kCompactGroups;
    uint32_t part = 0;
    constexpr uint32_t U = 8;  // loads in flight per thread (integer sum: any order)
    for (uint32_t q0 = threadIdx.x; q0 < g0; q0 += kBuildThreads * U) {
        uint32_t v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) v[u] = cnt[min(q0 + u * kBuildThreads, g0 - 1)];  // clamped: no branch
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) part += q0 + u * kBuildThreads < g0 ? v[u] : 0u;
    }
#pragma unroll
    for (uint32_t o = 32; o > 0; o >>= 1) part += __shfl_down(part, o, 64);
    if (lane == 0) s_w[wave] = part;
    if (threadIdx.x < kCompactGroups) {
        const uint32_t g = g0 + threadIdx.x;
        s_cnt[threadIdx.x] = g < L.ngroups ? cnt[g] : 0u;
    }
    __syncthreads();
    uint32_t base = 0, total = 0;
#pragma unroll
    for (uint32_t w = 0; w < kBuildThreads / 64; ++w) base += s_w[w];
#pragma unroll
    for (uint32_t w = 0; w < kCompactGroups; ++w) {
        base += w < wave ? s_cnt[w] : 0u;
        total += s_cnt[w];
    }
    const uint32_t g = g0 + wave;
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0)
        reinterpret_cast<uint32_t*>(img)[0] = base + total;  // wave 0: base = the earlier blocks' sum
    if (g >= L.ngroups) return;
    uint32_t* pre = occ_sum(img) + 4 * L.ngroups;
    uint8_t* bytes = reinterpret_cast<uint8_t*>(pre + L.ngroups);
    if (lane == 0) pre[g] = base;
    const uint32_t o = 128 * g + 2 * lane, last = L.nbytes - 1;
    const uint32_t v0 = grid[min(o, last)], v1 = grid[min(o + 1, last)];
    const uint32_t b0 = o < L.nbytes ? v0 : 0u, b1 = o + 1 < L.nbytes ? v1 : 0u;
    const uint64_t m0 = __ballot(b0 != 0u), m1 = __ballot(b1 != 0u);
    const uint32_t r = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u)) +
                       __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
    if (b0) bytes[r] = (uint8_t)b0;
    if (b1) bytes[r + (b0 ? 1u : 0u)] = (uint8_t)b1;
}

// Copies the global image into this workgroup's LDS when its bytes fit.
// Returns false (workgroup-uniform) otherwise: lookups then go to HBM/L2.
NGP_DEV bool load_occ_index(const uint8_t* __restrict__ img, const OccLayout& L, uint4* lds) {
    const uint32_t total = reinterpret_cast<const uint32_t*>(img)[0];
    if (total > L.cap) return false;
    const uint32_t n16 = (20 * L.ngroups + total + 15) / 16;
    const uint4* src = reinterpret_cast<const uint4*>(img + 16);
#pragma unroll 8
    for (uint32_t i = threadIdx.x; i < n16; i += blockDim.x) lds[i] = src[i];
    __syncthreads();
    return true;
}

template <bool ONE_LEVEL, typename OCC>
NGP_DEV uint32_t march_ray_train(const Ray& r, const MarchConst& k, const OCC& occ, float t, float far,
                                 float* __restrict__ ts) {
    uint32_t num_steps = 0;
    Sample s;
    while (t < far && num_steps < k.max_steps) {
        if (march_step<ONE_LEVEL>(r, k, occ, t, s)) {
            ts[num_steps++] = t;
            t += s.dt;
        }
    }
    return num_steps;
}

// Exact f^m(t) for f(t) = t + delta in float (round to nearest even): inside a
// binade [2^e, 2^(e+1)) every step adds the same multiple of the ulp unless
// delta / ulp ends in exactly .5 (a tie), so whole runs of steps are one
// exact multiply-add; ties and binade crossings are stepped one by one.
NGP_DEV float advance0(float t, uint32_t m, float delta) {
    const uint32_t db = __float_as_uint(delta);
    const int ed = (int)((db >> 23) & 0xffu);
    const uint32_t md = (db & 0x7fffffu) | 0x800000u;
    while (m > 0) {
        const float t1 = t + delta;
        const int e = (int)((__float_as_uint(t) >> 23) & 0xffu);
        const int sh = e - ed;
        const bool tie = sh >= 1 && sh <= 24 && (md & ((1u << sh) - 1u)) == (1u << (sh - 1));
        if (e == 0 || e >= 254 || tie || !(t1 > t)) {
            t = t1;
            --m;
            continue;
        }
        const float step = t1 - t;  // exact: t, t1 are multiples of ulp(t) in [t, 2t]
        const float top = __uint_as_float((uint32_t)(e + 1) << 23);
        const double room = ((double)top - (double)delta - (double)t) / (double)step;
        uint32_t j = room > 2.0 ? (uint32_t)fmin(room - 2.0, 4.0e9) : 0u;
        if (j > m) j = m;
        if (j == 0) {
            t = t1;
            --m;
            continue;
        }
        t = t + (float)j * step;  // exact: j * step < 2^e and a multiple of ulp(t)
        m -= j;
    }
    return t;
}

// The chain t_{k+1} = f(t_k) the walk moves along, two forms:
//   ChainConst (dt_gamma == 0): f(t) = t + delta, t_i in closed form (advance0);
//   ChainGamma (dt_gamma > 0):  f(t) = t + clamp(t * dt_gamma, dt_min, dt_max),
//     no closed form, so the wave steps the chain once up front (wave-uniform,
//     three dependent VALU operations per index, no memory) and keeps every
//     16th value in registers: record r = t_{16 r} sits in lane r % 64 of
//     rec[r / 64], 256 records cover 4096 indices. t_i is then record i / 16
//     plus i % 16 steps.
// seek_u(i): t_i for a wave-uniform i (every lane gets it); start(a): t_a for
// a lane's own a (a multiple of 16 for ChainGamma, all lanes active).
NGP_DEV float chain_step_g(float t, const MarchConst& k) { return t + clampf(t * k.dt_gamma, k.dt_min, k.dt_max); }

struct ChainConst {
    float t0, delta;
    NGP_DEV float step(float t) const { return t + delta; }
    NGP_DEV float start(uint32_t a) const { return advance0(t0, a, delta); }
    NGP_DEV float seek_u(uint32_t i) const { return advance0(t0, i, delta); }
};

constexpr uint32_t kRecStride = 16, kRecRegs = 4;
constexpr uint32_t kGammaMaxChain = kRecStride * 64 * kRecRegs;  // 4096 = 64 segments x 64
static_assert(kGammaMaxChain == 64 * 64, "the records cover exactly the indices 64 segments of <= 64 hold");

struct ChainGamma {
    float rec[kRecRegs];
    MarchConst k;
    uint32_t nrec;  // records written: ceil(K / 16)
    NGP_DEV float step(float t) const { return chain_step_g(t, k); }
    NGP_DEV float start(uint32_t a) const {
        const uint32_t r = a / kRecStride;
        // a segment past the chain's end (a >= K) starts at +inf: its walk ends at once
        float v = __builtin_inff();
#pragma unroll
        for (uint32_t j = 0; j < kRecRegs; ++j) {
            const float x = __shfl(rec[j], (int)(r & 63u), 64);
            if ((r >> 6) == j && r < nrec) v = x;
        }
        return v;  // a % kRecStride == 0 by construction (segment lengths)
    }
    NGP_DEV float seek_u(uint32_t i) const {
        const uint32_t r = i / kRecStride, j = r >> 6;
        const float base = j == 0 ? rec[0] : j == 1 ? rec[1] : j == 2 ? rec[2] : rec[3];
        float t = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(base), (int)(r & 63u)));
        for (uint32_t m = i % kRecStride; m > 0; --m) t = step(t);
        return t;
    }
};

// Steps the chain from t0 (wave-uniform) and fills the records. Returns the
// chain length K = the first index with t_K >= far (the walk only visits
// indices below it), or kInf if K > kGammaMaxChain.
NGP_DEV uint32_t chain_records(float t0, float far, const MarchConst& k, float (&rec)[kRecRegs]) {
    const uint32_t lane = threadIdx.x & 63;
    float t = t0;
#pragma unroll
    for (uint32_t j = 0; j < kRecRegs; ++j) {
        rec[j] = 0.0f;
        for (uint32_t rr = 0; rr < 64; ++rr) {
            if (!(t < far)) return (j * 64 + rr) * kRecStride;  // t_{16 r} >= far: K <= 16 r
            if (lane == rr) rec[j] = t;
            float u = t;
#pragma unroll
            for (uint32_t m = 0; m < kRecStride; ++m) u = chain_step_g(u, k);
            if (!(u < far)) {  // K in (16 r, 16 r + 16]: find it
                uint32_t kk = (j * 64 + rr) * kRecStride;
                while (t < far) {
                    t = chain_step_g(t, k);
                    ++kk;
                }
                return kk;
            }
            t = u;
        }
    }
    return kInf;
}

// One ray, one wave: the chain splits into 64 index segments of L indices
// (L <= 64; a multiple of 16 for ChainGamma). Returns the sample count (all lanes).
template <bool ONE_LEVEL, typename OCC, typename CHAIN>
NGP_DEV uint32_t march_ray_segmented(const Ray& r, const MarchConst& k, const OCC& occ, const CHAIN& ch,
                                     float far, uint32_t L, float* __restrict__ ts) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t a = lane * L, b = a + L;
    const float ta = ch.start(a);
    // speculative walk of segment [a, b) from a
    uint64_t vis = 0, occm = 0;
    uint32_t kk = a;
    float t = ta;
    Sample s;
    auto walk = [&](uint32_t from, float tf) {
        vis = 0;
        occm = 0;
        kk = from;
        t = tf;
        while (t < far && kk < b) {
            const uint64_t bit = 1ull << (kk - a);
            vis |= bit;
            float tt;
            if (probe<ONE_LEVEL>(r, k, occ, t, s, tt)) {
                occm |= bit;
                t = ch.step(t);  // == t + s.dt, the reference's occupied step
                ++kk;
            } else {
                do {
                    t = ch.step(t);
                    ++kk;
                } while (t < tt);
            }
        }
    };
    walk(a, ta);
    // exit index of the segment's walk; kInf once t >= far (the ray ends there)
    uint32_t X = t < far ? kk : kInf;
    uint32_t kend = kk;
    bool ended = !(t < far);

    uint32_t in = kInf;
    for (;;) {
        // stitch: in_s = first index >= a_s the true walk visits
        uint32_t cur = 0;
        // segment exits by v_readlane (uniform lane index): a __shfl here was
        // an LDS-crossbar round trip per segment, 64 in a row
        for (uint32_t sg = 0; sg < 64; ++sg) {
            if (lane == sg) in = cur;
            const uint32_t Xs = (uint32_t)__builtin_amdgcn_readlane((int)X, (int)sg);
            if (cur < (sg + 1) * L) cur = Xs;
        }
        const bool inside = in < b && !(ended && in >= kend);
        const bool merged = !inside || ((vis >> (in - a)) & 1ull);
        const uint64_t bad = __ballot(!merged);
        if (!bad) break;
        // re-walk the first unmerged segment from its true entry (t of the
        // entry found wave-uniformly: ChainGamma reads another lane's record)
        const uint32_t fb = (uint32_t)__ffsll((unsigned long long)bad) - 1;
        const float tin = ch.seek_u((uint32_t)__builtin_amdgcn_readlane((int)in, (int)fb));
        if (lane == fb) {
            walk(in, tin);
            X = t < far ? kk : kInf;
            kend = kk;
            ended = !(t < far);
        }
    }
    const bool inside = in < b && !(ended && in >= kend);
    const uint64_t mine = inside ? occm & ~((1ull << (in - a)) - 1ull) : 0ull;
    const uint32_t cnt = __popcll(mine);
    const uint32_t incl = ngp_dpp::scan_incl_u32(cnt);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    uint32_t off = incl - cnt;
    if (mine && off < k.max_steps) {
        float tj = ta;
        uint64_t m = mine;
        for (uint32_t j = 0; m && off < k.max_steps; ++j, tj = ch.step(tj)) {
            if ((m >> j) & 1ull) {
                ts[off++] = tj;
                m &= m - 1;
            }
        }
    }
    return total < k.max_steps ? total : k.max_steps;
}

template <bool ONE_LEVEL, typename OCC>
NGP_DEV uint32_t march_ray_wave(const Ray& r, const MarchConst& k, const OCC& occ, float t0, float far,
                                float* __restrict__ ts) {
    if (!(t0 < far)) return 0;
    if (k.dt_gamma == 0.0f) {
        const float delta = clampf(0.0f, k.dt_min, k.dt_max);  // the update when dt_gamma == 0
        // every chain step is >= delta - ulp(far); chain length to far bounds
        const float ulp_far = __uint_as_float(((__float_as_uint(far) >> 23) & 0xffu) << 23) * 1.1920929e-7f;
        const double smin = (double)delta - (double)ulp_far;
        if (smin > 0.0) {
            const double kest = ceil(((double)far - (double)t0) / smin) + 2.0;
            const uint32_t L = (uint32_t)ceil(kest / 64.0);
            if (L <= 64) return march_ray_segmented<ONE_LEVEL>(r, k, occ, ChainConst{t0, delta}, far, L, ts);
        }
    } else if (k.dt_gamma > 0.0f) {
        ChainGamma ch;
        ch.k = k;
        const uint32_t K = chain_records(t0, far, k, ch.rec);
        if (K != kInf) {
            ch.nrec = ngp_div_up(K, kRecStride);
            const uint32_t L = kRecStride * ngp_div_up(ngp_div_up(K, 64u), kRecStride);
            return march_ray_segmented<ONE_LEVEL>(r, k, occ, ch, far, L > 0 ? L : kRecStride, ts);
        }
    }
    uint32_t n = 0;
    if ((threadIdx.x & 63) == 0) n = march_ray_train<ONE_LEVEL>(r, k, occ, t0, far, ts);
    return (uint32_t)__builtin_amdgcn_readlane((int)n, 0);
}

// Sample kk of ray rn at output row p: xyz / dir / delta recomputed from the
// recorded t with the reference's float ops (raymarching.cu:418-444).
NGP_DEV void emit_sample(const float* __restrict__ rays_o, const float* __restrict__ rays_d, const MarchConst& k,
                         const float* __restrict__ nears, const float* __restrict__ noises,
                         const float* __restrict__ ts, uint32_t rn, uint32_t kk, size_t p, float* __restrict__ xyzs,
                         float* __restrict__ dirs, float* __restrict__ deltas) {
    const float* row = ts + (size_t)rn * k.max_steps;
    const float t = row[kk];
    // all loads unconditional (a load under the kk == 0 branch made the
    // compiler wait for each one on the spot)
    const float tp = row[kk ? kk - 1 : 0u];
    const float nr = nears[rn], nz = noises[rn];
    const float prev = kk == 0 ? ray_t0(nr, nz, k) : tp + clampf(tp * k.dt_gamma, k.dt_min, k.dt_max);
    const float ox = rays_o[rn * 3], oy = rays_o[rn * 3 + 1], oz = rays_o[rn * 3 + 2];
    const float dx = rays_d[rn * 3], dy = rays_d[rn * 3 + 1], dz = rays_d[rn * 3 + 2];
    const float dt = clampf(t * k.dt_gamma, k.dt_min, k.dt_max);
    xyzs[p * 3 + 0] = clampf(fmaf(t, dx, ox), -k.bound, k.bound);
    xyzs[p * 3 + 1] = clampf(fmaf(t, dy, oy), -k.bound, k.bound);
    xyzs[p * 3 + 2] = clampf(fmaf(t, dz, oz), -k.bound, k.bound);
    dirs[p * 3 + 0] = dx;
    dirs[p * 3 + 1] = dy;
    dirs[p * 3 + 2] = dz;
    deltas[p * 2 + 0] = dt;
    deltas[p * 2 + 1] = (t + dt) - prev;
}

// The optimizer update a march launch may carry (ngp_march_rays_train_prebuilt_adam):
// the march's workgroups keep their 16 waves and their LDS image, waves
// [0, kMarchAdamWaves) march rays and the rest sweep Adam as virtual
// 256-thread blocks (adam_sweep has no barriers). The occupancy lookups are an
// LDS latency chain and Adam an HBM stream: one CU runs both at once.
struct MarchAdam {
    ngp_head::TensorList tl;
    ngp_head::AdamArgs aa;
    ngp_step::StepState* st;  // null: no Adam in this launch
    uint4* clear;             // also zeroed (the grid backward's bin cursors), or null
    uint32_t clear16;
    bool emit_launch;         // the samples emitted by a launch of their own (NGP_ADAM_JOB_EMIT_LAUNCH)
};
constexpr uint32_t kMarchAdamWaves = 4;

// The emit inside the march + Adam launch (world 1; ngp_march_rays_train_prebuilt_adam):
// the march waves finish long before the Adam waves, so they also emit the
// samples. Each workgroup takes a ticket at its start and marches the ray
// block [rank * RB, rank * RB + RB), rank = ticket % G; once its block is
// marched it publishes the block's sample total as one 8-byte agent-scope
// atomic word ((epoch + 1) << 32 | total, epoch = ticket / G: the words need
// no reset between launches), and reads the words of every lower rank for
// its block's first output row. A lower rank's workgroup took its ticket
// earlier, so it is running or done: no workgroup waits for one that may not
// be resident. The rows are the emit launch's (ray order), bit for bit.
constexpr uint32_t kEmitMaxBlockRays = 64;
struct MarchEmit {
    uint32_t* ticket;            // null: the emit launch does it; else the workspace's ticket counter
    uint32_t* error;             // bit 0: a lower rank's total never arrived, bit 1: the block's offsets never did
    unsigned long long* words;   // [G] published block totals
    int32_t* counter;            // counter[0] = end, counter[1] += N (the last rank)
    float *xyzs, *dirs, *deltas;
    uint32_t M, rb;              // output capacity; rays per block (<= kEmitMaxBlockRays)
};

NGP_DEV unsigned long long agent_load_u64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <uint32_t MW>  // march waves per workgroup (kSegWaves: the whole workgroup)
__global__ void __launch_bounds__(kSegThreads)
k_march_train(const float* __restrict__ rays_o, const float* __restrict__ rays_d,
              const uint8_t* __restrict__ grid, const uint8_t* __restrict__ img, OccLayout L,
              MarchConst k, uint32_t N, const float* __restrict__ nears, const float* __restrict__ fars,
              const float* __restrict__ noises, int32_t* __restrict__ rays, float* __restrict__ ts,
              const int32_t* __restrict__ counter, uint32_t* __restrict__ scan, MarchAdam ma, MarchEmit me) {
    extern __shared__ uint4 dyn[];
    __shared__ uint32_t s_ticket, s_base0, s_arrive, s_ready, s_first;
    __shared__ uint32_t s_off[kEmitMaxBlockRays + 1];
    const bool emit = me.ticket != nullptr;  // launch-uniform
    // scan[0] = the offset of the first sample (the reference's counter[0] on entry,
    // raymarching.cu:405); scan[4 + n] = ray n's count (read by k_march_emit)
    if (blockIdx.x == 0 && threadIdx.x == 0) scan[0] = (uint32_t)counter[0];
    if (emit && threadIdx.x == 0) {
        s_ticket = atomicAdd(me.ticket, 1u);
        s_base0 = (uint32_t)counter[0];  // read before this block publishes (the last rank rewrites it)
        s_arrive = 0;
        s_ready = 0;
    }
    uint32_t* sum = reinterpret_cast<uint32_t*>(dyn);
    uint32_t* pre = sum + 4 * L.ngroups;
    const bool lds = L.ngroups > 0 && load_occ_index(img, L, dyn);  // every wave copies (one barrier)
    if (emit) __syncthreads();  // the ticket (load_occ_index returns before its barrier when the image is too big)
    const uint32_t wave = threadIdx.x >> 6;
    if (MW < kSegWaves && wave >= MW) {  // the Adam waves (workgroup-uniform split, no barrier follows)
        constexpr uint32_t kVirt = (kSegWaves - MW) / 4;  // 256-thread virtual blocks per workgroup
        if (blockIdx.x == 0 && wave == MW)
            for (uint32_t i = threadIdx.x & 63u; i < ma.clear16; i += 64) ma.clear[i] = uint4{0u, 0u, 0u, 0u};
        ngp_head::adam_sweep_pipe<2>(ma.tl, ma.st, ma.aa, blockIdx.x * kVirt + (wave - MW) / 4,
                                                    gridDim.x * kVirt, threadIdx.x & 255u);
        return;
    }
    const OccLds occ_lds{sum, pre, reinterpret_cast<const uint8_t*>(pre + L.ngroups)};
    const OccGlobal occ_glb{grid};
    const uint32_t G = gridDim.x;
    const uint32_t rank = emit ? s_ticket % G : blockIdx.x, epoch1 = emit ? s_ticket / G + 1u : 0u;
    const uint32_t n0 = emit ? rank * me.rb : 0u, n1 = emit ? min(N, n0 + me.rb) : N;
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t n = emit ? n0 + wave : blockIdx.x * MW + wave; n < n1; n += emit ? MW : G * MW) {
        const Ray r = load_ray(rays_o, rays_d, n);
        const float t0 = ray_t0(nears[n], noises[n], k);
        const float far = fars[n];
        float* row = ts + (size_t)n * k.max_steps;
        uint32_t cnt;
        if (lds) {
            cnt = k.C == 1 ? march_ray_wave<true>(r, k, occ_lds, t0, far, row)
                           : march_ray_wave<false>(r, k, occ_lds, t0, far, row);
        } else {
            cnt = k.C == 1 ? march_ray_wave<true>(r, k, occ_glb, t0, far, row)
                           : march_ray_wave<false>(r, k, occ_glb, t0, far, row);
        }
        if (lane == 0) {
            rays[n * 3 + 0] = (int32_t)n;
            rays[n * 3 + 2] = (int32_t)cnt;
            scan[4 + n] = cnt;
            if (emit) s_off[n - n0] = cnt;
        }
    }
    if (!emit) return;
    // ---- the in-launch emit (march waves only: no workgroup barrier, the Adam
    // waves are elsewhere; the march waves meet through LDS counters)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // this wave's ts rows and counts are out
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    uint32_t last = 0;
    if (lane == 0) last = atomicAdd(&s_arrive, 1u) == MW - 1 ? 1u : 0u;
    last = (uint32_t)__builtin_amdgcn_readfirstlane((int)last);
    const uint32_t nb = n1 > n0 ? n1 - n0 : 0u;
    if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        // the block's counts -> exclusive offsets (one wave: nb <= 64)
        const uint32_t c = lane < nb ? s_off[lane] : 0u;
        uint32_t incl = c;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        // publish this block's total, then sum the lower ranks' totals
        if (lane == 0)
            __hip_atomic_store(me.words + rank, ((unsigned long long)epoch1 << 32) | total, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        // (bounded: a word that never arrives -- a broken launch, not a slow
        // one: the march itself takes ~20 us -- ends the wait after ~0.1 s
        // with wrong offsets rather than a hung GPU, and records it in the
        // workspace's error word, which the host reads: ngp_march_rays_train_error)
        uint32_t part = 0;
        bool lost = false;
        for (uint32_t p = lane; p < rank; p += 64) {
            unsigned long long v = agent_load_u64(me.words + p);
            for (uint32_t spin = 0; (uint32_t)(v >> 32) != epoch1 && spin < (1u << 20); ++spin) {
                __builtin_amdgcn_s_sleep(2);
                v = agent_load_u64(me.words + p);
            }
            lost |= (uint32_t)(v >> 32) != epoch1;
            part += (uint32_t)v;
        }
        if (__ballot(lost) && lane == 0) atomicOr(me.error, 1u);
#pragma unroll
        for (uint32_t o = 32; o > 0; o >>= 1) part += __shfl_xor(part, o, 64);
        if (lane < nb) s_off[lane] = incl - c;
        if (lane == 0) {
            s_off[nb] = total;
            s_first = s_base0 + part;
            if (rank == G - 1) {  // every lower rank's total is in: the batch's end (reference :405-406)
                me.counter[0] = (int32_t)(s_base0 + part + total);
                me.counter[1] += (int32_t)N;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(&s_ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
        for (uint32_t spin = 0; __hip_atomic_load(&s_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u &&
                                spin < (1u << 22); ++spin)
            __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(&s_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0u && lane == 0)
            atomicOr(me.error, 2u);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    const uint32_t base = s_first, btotal = s_off[nb];
    const uint32_t t = threadIdx.x;  // 0 .. 64 MW - 1
    for (uint32_t i = t; i < nb; i += 64 * MW) rays[(size_t)(n0 + i) * 3 + 1] = (int32_t)(base + s_off[i]);
    for (uint32_t j = t; j < btotal; j += 64 * MW) {
        uint32_t lo = 0, hi = nb;  // largest ray i with s_off[i] <= j
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (s_off[mid] <= j) lo = mid; else hi = mid;
        }
        if (base + s_off[lo + 1] > me.M) continue;  // whole ray dropped, like the reference
        emit_sample(rays_o, rays_d, k, nears, noises, ts, n0 + lo, j - s_off[lo], (size_t)base + j, me.xyzs,
                    me.dirs, me.deltas);
    }
}
static_assert((kSegWaves - kMarchAdamWaves) % 4 == 0, "Adam waves form 256-thread virtual blocks");

// Grid (ray groups of 256, kEmitSplit): each workgroup sums the counts of all
// rays before its group (a few thousand coalesced L2 reads), scans the
// group's counts, and writes its 1/kEmitSplit slice of the group's samples;
// the y == 0 workgroup of each group also writes the group's offsets, and the
// last group's the counter (counter[0] = end, counter[1] += N, the
// reference's two atomics :405-406). Outputs of rays with offset + count > M
// are skipped (reference :416).
// Optional tail of the emit launch (the fused step, nerf/fused.py): one extra
// row of blocks that runs the deferred GradScaler / LR / loss bookkeeping of the
// optimizer update before this step (block 0) and packs the MLP fragment
// images from the fp16 weights it wrote (blocks 1..), beside the emit blocks
// instead of in a latency-bound launch of their own.
struct EmitTail {
    ngp_step::StepState* st;  // null: no tail row
    bool end;                 // run the bookkeeping
    ngp_step::ScalerArgs sa;
    const float* loss_ray;
    uint32_t n_rays, groups;  // groups: emit ray groups (gridDim.x may be wider)
    ngp_pack::PackJobs jobs;
};

__global__ void __launch_bounds__(kMarchThreads)
k_march_emit(const float* __restrict__ rays_o, const float* __restrict__ rays_d, MarchConst k,
             uint32_t N, uint32_t M, const float* __restrict__ nears, const float* __restrict__ noises,
             const float* __restrict__ ts, float* __restrict__ xyzs, float* __restrict__ dirs,
             float* __restrict__ deltas, int32_t* __restrict__ rays, const uint32_t* __restrict__ scan,
             int32_t* __restrict__ counter, EmitTail tail) {
    // the tail row is row 0 (dispatched first: behind the emit rows its
    // dependent chains, the bookkeeping and the fragment packs, ran in the
    // launch's tail); the emit rows follow
    const bool has_tail = tail.st != nullptr;
    if (has_tail && blockIdx.y == 0) {  // the tail row (block-uniform)
        if (blockIdx.x == 0) {
            if (tail.end && tail.st->end_pending)
                ngp_step::step_end_block(tail.st, tail.sa, nullptr, nullptr, tail.loss_ray, tail.n_rays);
        } else if (blockIdx.x - 1 < (uint32_t)tail.jobs.n) {
            const ngp_pack::PackJob& j = tail.jobs.job[blockIdx.x - 1];
            ngp_pack::build_frags(j.image, j.w, j.m, j.transposed != 0);
        }
        return;
    }
    if (blockIdx.x >= tail.groups) return;
    __shared__ uint32_t off[kMarchThreads + 1];
    __shared__ uint32_t lds_waves[kMarchThreads / 64];
    const uint32_t* __restrict__ counts = scan + 4;
    const uint32_t n0 = blockIdx.x * kMarchThreads;
    // the counts of all earlier rays, 8 loads in flight per thread (one load
    // per iteration waited out an L2 round trip each: 15 of them for the last
    // group of a 4096-ray batch); indices past n0 read count 0's slot and drop it
    uint32_t part = 0;
    for (uint32_t i0 = threadIdx.x; i0 < n0; i0 += 8 * kMarchThreads) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const uint32_t i = i0 + u * kMarchThreads;
            v[u] = counts[i < n0 ? i : 0u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) part += i0 + u * kMarchThreads < n0 ? v[u] : 0u;
    }
    uint32_t before;
    block_exclusive_scan<kMarchThreads>(part, lds_waves, before);
    const uint32_t base = scan[0] + before;
    const uint32_t n = n0 + threadIdx.x;
    const uint32_t c = n < N ? counts[n] : 0u;
    uint32_t total;
    const uint32_t excl = block_exclusive_scan<kMarchThreads>(c, lds_waves, total);
    off[threadIdx.x] = excl;
    if (threadIdx.x == 0) off[kMarchThreads] = total;
    const uint32_t ey = blockIdx.y - (has_tail ? 1u : 0u);  // emit row
    if (ey == 0) {
        if (n < N) rays[(size_t)n * 3 + 1] = (int32_t)(base + excl);
        if (blockIdx.x == tail.groups - 1 && threadIdx.x == 0) {
            counter[0] = (int32_t)(base + total);
            counter[1] += (int32_t)N;
        }
    }
    __syncthreads();

    const uint32_t chunk = ngp_div_up(total, kEmitSplit);
    const uint32_t j0 = ey * chunk, j1 = min(total, j0 + chunk);
    for (uint32_t j = j0 + threadIdx.x; j < j1; j += kMarchThreads) {
        uint32_t lo = 0, hi = kMarchThreads;  // largest ray r with off[r] <= j
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (off[mid] <= j) lo = mid; else hi = mid;
        }
        const uint32_t rn = n0 + lo, kk = j - off[lo];
        if (base + off[lo + 1] > M) continue;  // whole ray dropped, like the reference
        emit_sample(rays_o, rays_d, k, nears, noises, ts, rn, kk, (size_t)base + j, xyzs, dirs, deltas);
    }
}

OccLayout occ_layout(const uint8_t* grid, uint32_t C, uint32_t H) {
    OccLayout L{};
    const size_t nbytes = (size_t)C * H * H * H / 8;
    L.nbytes = (uint32_t)nbytes;
    L.nwords = (uint32_t)((nbytes + 31) / 32);
    L.ngroups = (L.nwords + 3) / 4;
    const size_t dir_bytes = (size_t)L.ngroups * 20;
    // LDS image only when the directory leaves room for bytes and the bitfield
    // can be read with 16-byte loads; otherwise every lookup goes to HBM/L2.
    if ((reinterpret_cast<uintptr_t>(grid) & 15) != 0 || dir_bytes + 4096 > kMarchLdsBytes) {
        L.ngroups = 0;
        return L;
    }
    L.cap = (uint32_t)(kMarchLdsBytes - dir_bytes);
    return L;
}

// bytes of the global occupancy image (0 when the LDS path is off)
size_t occ_image_bytes(const OccLayout& L) {
    return L.ngroups ? ((16 + (size_t)L.ngroups * 20 + L.nbytes + 15) / 16) * 16 : 0;
}
// per-group count scratch of the build, after the image
size_t occ_scratch_bytes(const OccLayout& L) { return (size_t)L.ngroups * 4; }

// ---- composite_rays_train (one WAVE per ray) ------------------------------------
// The compositing recurrence (T, rgb, depth, weight sum) is sequential per ray
// and must stay in sample order to match the reference bit for bit. One lane
// per ray left 64 waves for 4096 rays, each stalling on every sample's loads.
// Here a wave owns a ray: lanes load 64 samples at once (coalesced) and
// compute their alphas in parallel; the recurrence then runs wave-uniform over
// readlane'd operands, and (backward) each lane keeps the running state of
// "its" sample so the per-sample gradients are computed and stored in parallel.
constexpr uint32_t kCompWaves = 4;

NGP_DEV float lanef(float v, uint32_t j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)j));
}

__global__ void __launch_bounds__(kCompWaves * 64)
k_composite_train_fwd(const float* __restrict__ sigmas, const float* __restrict__ rgbs,
                      const float* __restrict__ deltas, const int32_t* __restrict__ rays,
                      uint32_t M, uint32_t N, float T_thresh, float* weights_sum, float* depth,
                      float* image) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t n = blockIdx.x * kCompWaves + (threadIdx.x >> 6);
    if (n >= N) return;
    const uint32_t index = (uint32_t)rays[n * 3];
    const uint32_t offset = (uint32_t)rays[n * 3 + 1];
    const uint32_t num_steps = (uint32_t)rays[n * 3 + 2];
    float T = 1.0f;
    float r = 0, g = 0, b = 0, ws = 0, t = 0, d = 0;
    if (num_steps != 0 && offset + num_steps <= M) {
        for (uint32_t base = 0; base < num_steps; base += 64) {
            const uint32_t i = offset + base + lane;
            const bool valid = base + lane < num_steps;
            const float sg = valid ? sigmas[i] : 0.0f;
            const float d0 = valid ? deltas[(size_t)i * 2] : 0.0f;
            const float d1 = valid ? deltas[(size_t)i * 2 + 1] : 0.0f;
            const float c0 = valid ? rgbs[(size_t)i * 3 + 0] : 0.0f;
            const float c1 = valid ? rgbs[(size_t)i * 3 + 1] : 0.0f;
            const float c2 = valid ? rgbs[(size_t)i * 3 + 2] : 0.0f;
            const float alpha = 1.0f - expf(-sg * d0);
            const uint32_t cnt = min(64u, num_steps - base);
            bool stop = false;
            for (uint32_t j = 0; j < cnt; ++j) {
                const float a = lanef(alpha, j);
                const float weight = a * T;
                r = fmaf(weight, lanef(c0, j), r);
                g = fmaf(weight, lanef(c1, j), g);
                b = fmaf(weight, lanef(c2, j), b);
                t += lanef(d1, j);
                d = fmaf(weight, t, d);
                ws += weight;
                T *= 1.0f - a;
                if (T < T_thresh) {
                    stop = true;
                    break;
                }
            }
            if (stop) break;
        }
    }
    if (lane == 0) {
        weights_sum[index] = ws;
        depth[index] = d;
        image[index * 3] = r;
        image[index * 3 + 1] = g;
        image[index * 3 + 2] = b;
    }
}

__global__ void __launch_bounds__(kCompWaves * 64)
k_composite_train_bwd(const float* __restrict__ grad_weights_sum, const float* __restrict__ grad_depth,
                      const float* __restrict__ grad_image, const float* __restrict__ sigmas,
                      const float* __restrict__ rgbs, const float* __restrict__ deltas,
                      const int32_t* __restrict__ rays, const float* __restrict__ weights_sum,
                      const float* __restrict__ depth, const float* __restrict__ image, uint32_t M,
                      uint32_t N, float T_thresh, float* grad_sigmas, float* grad_rgbs) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t n = blockIdx.x * kCompWaves + (threadIdx.x >> 6);
    if (n >= N) return;
    const uint32_t index = (uint32_t)rays[n * 3];
    const uint32_t offset = (uint32_t)rays[n * 3 + 1];
    const uint32_t num_steps = (uint32_t)rays[n * 3 + 2];
    if (num_steps == 0 || offset + num_steps > M) return;

    const float gws = grad_weights_sum[index], gd = grad_depth[index];
    const float gr = grad_image[index * 3], gg = grad_image[index * 3 + 1], gb = grad_image[index * 3 + 2];
    const float r_final = image[index * 3], g_final = image[index * 3 + 1], b_final = image[index * 3 + 2];
    const float ws_final = weights_sum[index], d_final = depth[index];

    float T = 1.0f;
    float r = 0, g = 0, b = 0, t = 0, d = 0;
    for (uint32_t base = 0; base < num_steps; base += 64) {
        const uint32_t i = offset + base + lane;
        const bool valid = base + lane < num_steps;
        const float sg = valid ? sigmas[i] : 0.0f;
        const float d0 = valid ? deltas[(size_t)i * 2] : 0.0f;
        const float d1 = valid ? deltas[(size_t)i * 2 + 1] : 0.0f;
        const float c0 = valid ? rgbs[(size_t)i * 3 + 0] : 0.0f;
        const float c1 = valid ? rgbs[(size_t)i * 3 + 1] : 0.0f;
        const float c2 = valid ? rgbs[(size_t)i * 3 + 2] : 0.0f;
        const float alpha = 1.0f - expf(-sg * d0);
        const uint32_t cnt = min(64u, num_steps - base);
        // running state after this lane's sample
        float mw = 0, mT = 0, mr = 0, mg = 0, mb = 0, mt = 0, md = 0;
        uint32_t done = cnt;
        for (uint32_t j = 0; j < cnt; ++j) {
            const float a = lanef(alpha, j);
            const float weight = a * T;
            r = fmaf(weight, lanef(c0, j), r);
            g = fmaf(weight, lanef(c1, j), g);
            b = fmaf(weight, lanef(c2, j), b);
            t += lanef(d1, j);
            d = fmaf(weight, t, d);
            T *= 1.0f - a;
            if (lane == j) {
                mw = weight; mT = T; mr = r; mg = g; mb = b; mt = t; md = d;
            }
            if (T < T_thresh) {
                done = j + 1;
                break;
            }
        }
        if (lane < done) {
            grad_rgbs[(size_t)i * 3 + 0] = gr * mw;
            grad_rgbs[(size_t)i * 3 + 1] = gg * mw;
            grad_rgbs[(size_t)i * 3 + 2] = gb * mw;
            grad_sigmas[i] = d0 * (gr * (mT * c0 - (r_final - mr)) +
                                   gg * (mT * c1 - (g_final - mg)) +
                                   gb * (mT * c2 - (b_final - mb)) +
                                   gd * (mT * mt - (d_final - md)) +
                                   gws * (1 - ws_final));
        }
        if (done < cnt || T < T_thresh) break;
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
    const OccGlobal occ{grid};
    while (t < far && step < n_step) {
        if (march_step<false>(r, k, occ, t, s)) {
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

// ---- device-driven inference loop (renderer.py:376-426) ------------------------
// The reference's test render loops on the host: count the alive rays, pick
// n_step = max(min(N // n_alive, 8), 1), march / network / composite, compact
// rays_alive[rays_alive >= 0], step += n_step, until step >= max_steps or no
// ray is alive -- a host round trip per iteration. Here the loop state lives
// in a two-slot device record (iteration i reads slot i & 1 and prepares slot
// (i + 1) & 1), every kernel derives n_step from it, and the composite kernel
// appends its surviving rays to the other alive list (one atomic per wave),
// so a hipGraph holds any number of iterations and the host checks the state
// once per replay. Per ray everything is the reference's arithmetic: the
// list's order only moves a ray's samples to other rows, and the grid / MLP
// kernels compute every row from that row alone.
struct RenderSlot {
    int32_t count;    // samples this iteration: n_alive * n_step (0 once done); the grid / MLP count
    int32_t n_alive;  // rays in this iteration's alive list
    int32_t step;     // the reference's `step` before this iteration
    int32_t pad;
};

NGP_DEV bool render_live(const RenderSlot& s, uint32_t max_steps) {
    return s.n_alive > 0 && (uint32_t)s.step < max_steps;
}
NGP_DEV uint32_t render_n_step(uint32_t N, uint32_t n_alive) {
    return max(min(N / n_alive, 8u), 1u);
}

__global__ void __launch_bounds__(256)
k_render_init(uint32_t N, const float* __restrict__ nears, int32_t* rays_alive, float* rays_t, float* weights_sum,
              float* depth, float* image, RenderSlot* state) {
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n == 0) {
        state[0] = RenderSlot{0, (int32_t)N, 0, 0};
        state[1] = RenderSlot{0, 0, 0, 0};
    }
    if (n >= N) return;
    rays_alive[n] = (int32_t)n;
    rays_t[n] = nears[n];
    weights_sum[n] = 0.0f;
    depth[n] = 0.0f;
    image[n * 3] = 0.0f; image[n * 3 + 1] = 0.0f; image[n * 3 + 2] = 0.0f;
}

// kernel_march_rays (raymarching.cu:709-814) with n_alive / n_step from the
// state; slots past a ray's last sample are zeroed (the reference allocates
// xyzs / dirs / deltas with torch.zeros every iteration); noise only in the
// first iteration (`perturb if step == 0 else False`, renderer.py:407).
__global__ void __launch_bounds__(128)
k_render_march(uint32_t N, RenderSlot* __restrict__ state, uint32_t cur, const int32_t* __restrict__ rays_alive,
               const float* __restrict__ rays_t, const float* __restrict__ rays_o,
               const float* __restrict__ rays_d, MarchConst k, const uint8_t* __restrict__ grid,
               const float* __restrict__ fars, float* xyzs, float* dirs, float* deltas,
               const float* __restrict__ noises) {
    const RenderSlot S = state[cur];
    const bool live = render_live(S, k.max_steps);
    const uint32_t n_alive = live ? (uint32_t)S.n_alive : 0u;
    const uint32_t n_step = live ? render_n_step(N, n_alive) : 0u;
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n == 0) {
        state[cur].count = (int32_t)(n_alive * n_step);
        state[cur ^ 1u] = RenderSlot{0, 0, S.step + (int32_t)n_step, 0};
    }
    if (n >= n_alive) return;
    const int index = rays_alive[n];
    const float noise = (S.step == 0 && noises) ? noises[n] : 0.0f;
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
    const OccGlobal occ{grid};
    while (t < far && step < n_step) {
        if (march_step<false>(r, k, occ, t, s)) {
            xyz[step * 3] = s.x; xyz[step * 3 + 1] = s.y; xyz[step * 3 + 2] = s.z;
            dir[step * 3] = r.dx; dir[step * 3 + 1] = r.dy; dir[step * 3 + 2] = r.dz;
            t += s.dt;
            dlt[step * 2] = s.dt;
            dlt[step * 2 + 1] = t - last_t;
            last_t = t;
            step++;
        }
    }
    for (; step < n_step; ++step) {
        xyz[step * 3] = 0.0f; xyz[step * 3 + 1] = 0.0f; xyz[step * 3 + 2] = 0.0f;
        dir[step * 3] = 0.0f; dir[step * 3 + 1] = 0.0f; dir[step * 3 + 2] = 0.0f;
        dlt[step * 2] = 0.0f; dlt[step * 2 + 1] = 0.0f;
    }
}

// torch.sigmoid on the colour network's half output: fp32 math, half result
// (autocast), then composite_rays' float32 cast.
NGP_DEV float render_sigmoid_h(ngp_half x) { return (float)(ngp_half)(1.0f / (1.0f + expf(-(float)x))); }

// kernel_composite_rays (raymarching.cu:827-914) on sigma = density_scale *
// trunc_exp(h0) (the MLP epilogue) and rgb = sigmoid of the colour logits;
// a ray that stays alive joins the next iteration's list.
__global__ void __launch_bounds__(256)
k_render_composite(uint32_t N, uint32_t max_steps, RenderSlot* __restrict__ state, uint32_t cur, float T_thresh,
                   const int32_t* __restrict__ rays_alive, int32_t* __restrict__ rays_alive_next, float* rays_t,
                   const float* __restrict__ sigmas, const ngp_half* __restrict__ color_out,
                   const float* __restrict__ deltas, float* weights_sum, float* depth, float* image) {
    const RenderSlot S = state[cur];
    const bool live = render_live(S, max_steps);
    if (!live) return;  // the whole grid: no wave reaches the ballot
    const uint32_t n_alive = (uint32_t)S.n_alive;
    const uint32_t n_step = render_n_step(N, n_alive);
    const uint32_t n = blockIdx.x * blockDim.x + threadIdx.x;
    if (blockIdx.x * blockDim.x >= n_alive) return;  // whole workgroup past the list
    bool survives = false;
    int index = 0;
    if (n < n_alive) {
        index = rays_alive[n];
        const float* sg = sigmas + (size_t)n * n_step;
        const ngp_half* cl = color_out + (size_t)n * n_step * 16;
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
            r = fmaf(weight, render_sigmoid_h(cl[step * 16 + 0]), r);
            g = fmaf(weight, render_sigmoid_h(cl[step * 16 + 1]), g);
            b = fmaf(weight, render_sigmoid_h(cl[step * 16 + 2]), b);
            if (T < T_thresh) break;
            step++;
        }
        survives = step >= n_step;
        if (survives) rays_t[index] = t;
        weights_sum[index] = weight_sum;
        depth[index] = d;
        image[index * 3] = r;
        image[index * 3 + 1] = g;
        image[index * 3 + 2] = b;
    }
    // rays_alive[rays_alive >= 0]: the survivors of this wave take consecutive
    // places after one atomic on the next slot's count
    const uint64_t mask = __ballot(survives);
    if (mask == 0) return;
    const uint32_t lane = threadIdx.x & 63u;
    int32_t base = 0;
    if (lane == (uint32_t)__ffsll((long long)mask) - 1u)
        base = atomicAdd(&state[cur ^ 1u].n_alive, (int32_t)__popcll(mask));
    base = __shfl(base, __ffsll((long long)mask) - 1, 64);
    if (survives) rays_alive_next[base + __popcll(mask & ((1ull << lane) - 1ull))] = index;
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

// workspace = [t scratch: N * max_steps floats][scan: base + N counts][occupancy image][its build scratch]
static size_t march_ts_bytes(uint32_t N, uint32_t max_steps) {
    return ((size_t)N * max_steps * sizeof(float) + 255) / 256 * 256;
}
static size_t march_scan_bytes(uint32_t N) { return ((size_t)(N + 4) * sizeof(uint32_t) + 255) / 256 * 256; }

// the in-launch emit's ticket counter (16 B) and published block totals (8 B per workgroup)
static size_t march_sync_bytes() { return 256 + 8 * (size_t)kMaxMarchBlocks; }

extern "C" size_t ngp_march_rays_train_workspace_bytes(uint32_t N, uint32_t max_steps, uint32_t C,
                                                        uint32_t H) {
    // the image size does not depend on the grid pointer's alignment
    OccLayout L = occ_layout(nullptr, C, H);
    return march_ts_bytes(N, max_steps) + march_scan_bytes(N) + (occ_image_bytes(L) + occ_scratch_bytes(L) + 255) /
           256 * 256 + march_sync_bytes();
}

// The in-launch emit's error word (MarchEmit::error; 0 = none), from the
// workspace's sync header: sticky until the caller clears it.
extern "C" size_t ngp_march_rays_train_error_offset(uint32_t N, uint32_t max_steps, uint32_t C, uint32_t H) {
    const OccLayout L = occ_layout(nullptr, C, H);
    return march_ts_bytes(N, max_steps) + march_scan_bytes(N) +
           (occ_image_bytes(L) + occ_scratch_bytes(L) + 255) / 256 * 256 + 4;
}

// The march + Adam launch emits the samples itself (MarchEmit) unless the job
// asks for the emit launch (NGP_ADAM_JOB_EMIT_LAUNCH) or a ray block would
// exceed kEmitMaxBlockRays.

static int march_train_impl(const float* rays_o, const float* rays_d, const uint8_t* grid,
                             float bound, float dt_gamma, uint32_t max_steps, uint32_t N, uint32_t C,
                             uint32_t H, uint32_t M, const float* nears, const float* fars,
                             float* xyzs, float* dirs, float* deltas, int32_t* rays, int32_t* counter,
                             const float* noises, void* workspace, size_t workspace_bytes,
                             bool build_image, void* stream, const EmitTail* tail = nullptr,
                             const MarchAdam* ma = nullptr) {
    if (int e = check_cascade(C, H, max_steps)) return e;
    NGP_REQUIRE(rays && counter, NGP_ERR_ARG, "march_rays_train: null rays/counter");
    if (N == 0) return NGP_OK;
    const size_t need = ngp_march_rays_train_workspace_bytes(N, max_steps, C, H);
    NGP_REQUIRE(workspace && workspace_bytes >= need, NGP_ERR_ARG,
                "march_rays_train: workspace of %zu bytes required, got %zu", need, workspace_bytes);
    NGP_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, NGP_ERR_ARG,
                "march_rays_train: workspace must be 16-byte aligned");
    const MarchConst k = make_march_const(bound, dt_gamma, max_steps, C, H);
    const OccLayout L = occ_layout(grid, C, H);
    hipStream_t st = ngp_stream(stream);
    const uint32_t groups = ngp_div_up(N, kMarchThreads);
    const uint32_t wgs = ngp_div_up(N, kSegWaves);
    const uint32_t blocks = wgs < kMaxMarchBlocks ? wgs : kMaxMarchBlocks;
    float* ts = static_cast<float*>(workspace);
    uint32_t* scan = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(workspace) + march_ts_bytes(N, max_steps));
    uint8_t* img = reinterpret_cast<uint8_t*>(scan) + march_scan_bytes(N);
    if (L.ngroups && build_image) {
        uint32_t* cnt = reinterpret_cast<uint32_t*>(img + occ_image_bytes(L));
        const uint32_t wg = ngp_div_up(L.ngroups, kBuildThreads);
        k_occ_count<<<wg, kBuildThreads, 0, st>>>(grid, L, img, cnt);
        k_occ_compact<<<ngp_div_up(L.ngroups, kCompactGroups), kBuildThreads, 0, st>>>(grid, L, img, cnt);
    }
    MarchEmit me{};
    if (ma && ma->st) {  // every CU gets a workgroup: the Adam waves sweep 1/gridDim of the parameters each
        const uint32_t rb = ngp_div_up(N, kMaxMarchBlocks);
        if (rb <= kEmitMaxBlockRays && !ma->emit_launch) {
            uint8_t* sync = img + (occ_image_bytes(L) + occ_scratch_bytes(L) + 255) / 256 * 256;
            me = MarchEmit{reinterpret_cast<uint32_t*>(sync), reinterpret_cast<uint32_t*>(sync) + 1,
                           reinterpret_cast<unsigned long long*>(sync + 256), counter, xyzs, dirs, deltas, M, rb};
        }
        k_march_train<kMarchAdamWaves><<<kMaxMarchBlocks, kSegThreads, L.ngroups ? kMarchLdsBytes : 0, st>>>(
            rays_o, rays_d, grid, img, L, k, N, nears, fars, noises, rays, ts, counter, scan, *ma, me);
    } else {
        k_march_train<kSegWaves><<<blocks, kSegThreads, L.ngroups ? kMarchLdsBytes : 0, st>>>(
            rays_o, rays_d, grid, img, L, k, N, nears, fars, noises, rays, ts, counter, scan, MarchAdam{},
            MarchEmit{});
    }
    if (me.ticket && !tail) return ngp_check_launch("march_rays_train");  // emitted, no tail: one launch
    EmitTail et{};
    if (tail) et = *tail;
    et.groups = me.ticket ? 0u : groups;  // emitted in the march launch: the tail row alone
    const uint32_t gx = tail ? std::max<uint32_t>(et.groups, 1u + (uint32_t)tail->jobs.n) : groups;
    const uint32_t gy = me.ticket ? 1u : kEmitSplit + (tail ? 1u : 0u);
    k_march_emit<<<dim3(gx, gy), kMarchThreads, 0, st>>>(rays_o, rays_d, k, N, M, nears, noises, ts, xyzs, dirs,
                                                         deltas, rays, scan, counter, et);
    return ngp_check_launch("march_rays_train");
}

extern "C" int ngp_march_rays_train(const float* rays_o, const float* rays_d, const uint8_t* grid,
                                    float bound, float dt_gamma, uint32_t max_steps, uint32_t N,
                                    uint32_t C, uint32_t H, uint32_t M, const float* nears,
                                    const float* fars, float* xyzs, float* dirs, float* deltas,
                                    int32_t* rays, int32_t* counter, const float* noises,
                                    void* workspace, size_t workspace_bytes, void* stream) {
    return march_train_impl(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, M, nears, fars,
                            xyzs, dirs, deltas, rays, counter, noises, workspace, workspace_bytes, true,
                            stream);
}

extern "C" int ngp_march_occupancy_build(const uint8_t* grid, uint32_t C, uint32_t H, uint32_t N,
                                         uint32_t max_steps, void* workspace, size_t workspace_bytes,
                                         void* stream) {
    if (int e = check_cascade(C, H, max_steps)) return e;
    const size_t need = ngp_march_rays_train_workspace_bytes(N, max_steps, C, H);
    NGP_REQUIRE(workspace && workspace_bytes >= need, NGP_ERR_ARG,
                "march_occupancy_build: workspace of %zu bytes required, got %zu", need, workspace_bytes);
    const OccLayout L = occ_layout(grid, C, H);
    if (!L.ngroups) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    uint8_t* img = static_cast<uint8_t*>(workspace) + march_ts_bytes(N, max_steps) + march_scan_bytes(N);
    uint32_t* cnt = reinterpret_cast<uint32_t*>(img + occ_image_bytes(L));
    const uint32_t wg = ngp_div_up(L.ngroups, kBuildThreads);
    k_occ_count<<<wg, kBuildThreads, 0, st>>>(grid, L, img, cnt);
    k_occ_compact<<<ngp_div_up(L.ngroups, kCompactGroups), kBuildThreads, 0, st>>>(grid, L, img, cnt);
    return ngp_check_launch("march_occupancy_build");
}

extern "C" int ngp_march_rays_train_prebuilt(const float* rays_o, const float* rays_d,
                                             const uint8_t* grid, float bound, float dt_gamma,
                                             uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H,
                                             uint32_t M, const float* nears, const float* fars,
                                             float* xyzs, float* dirs, float* deltas, int32_t* rays,
                                             int32_t* counter, const float* noises, void* workspace,
                                             size_t workspace_bytes, void* stream) {
    return march_train_impl(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, M, nears, fars,
                            xyzs, dirs, deltas, rays, counter, noises, workspace, workspace_bytes, false,
                            stream);
}

extern "C" int ngp_march_rays_train_prebuilt_tail(const float* rays_o, const float* rays_d,
                                                  const uint8_t* grid, float bound, float dt_gamma,
                                                  uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H,
                                                  uint32_t M, const float* nears, const float* fars,
                                                  float* xyzs, float* dirs, float* deltas, int32_t* rays,
                                                  int32_t* counter, const float* noises, void* workspace,
                                                  size_t workspace_bytes, void* state, float growth_factor,
                                                  float backoff_factor, int32_t growth_interval,
                                                  int32_t scaler_enabled, const float* loss_ray, int32_t n_nets,
                                                  const void* const* mlp_weights, const uint32_t* in_dims,
                                                  const uint32_t* hidden_dims, const uint32_t* num_layers,
                                                  void* const* images, void* stream) {
    NGP_REQUIRE(state && loss_ray, NGP_ERR_ARG, "march_rays_train_prebuilt_tail: null state or loss_ray");
    EmitTail tail{};
    tail.st = static_cast<ngp_step::StepState*>(state);
    tail.end = true;
    tail.sa = ngp_step::ScalerArgs{growth_factor, backoff_factor, growth_interval, scaler_enabled,
                                   N ? 1.0f / (float)N : 0.0f};
    tail.loss_ray = loss_ray;
    tail.n_rays = N;
    if (n_nets > 0)
        if (int e = ngp_pack::build_jobs(n_nets, mlp_weights, in_dims, hidden_dims, num_layers, images, tail.jobs))
            return e;
    return march_train_impl(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, M, nears, fars,
                            xyzs, dirs, deltas, rays, counter, noises, workspace, workspace_bytes, false,
                            stream, &tail);
}

extern "C" int ngp_march_rays_train_prebuilt_adam(const float* rays_o, const float* rays_d,
                                                  const uint8_t* grid, float bound, float dt_gamma,
                                                  uint32_t max_steps, uint32_t N, uint32_t C, uint32_t H,
                                                  uint32_t M, const float* nears, const float* fars,
                                                  float* xyzs, float* dirs, float* deltas, int32_t* rays,
                                                  int32_t* counter, const float* noises, void* workspace,
                                                  size_t workspace_bytes, void* state, float growth_factor,
                                                  float backoff_factor, int32_t growth_interval,
                                                  int32_t scaler_enabled, const float* loss_ray, int32_t n_nets,
                                                  const void* const* mlp_weights, const uint32_t* in_dims,
                                                  const uint32_t* hidden_dims, const uint32_t* num_layers,
                                                  void* const* images, const ngp_adam_job* job, void* stream) {
    NGP_REQUIRE(state && loss_ray && job, NGP_ERR_ARG, "march_rays_train_prebuilt_adam: null state, loss_ray or job");
    NGP_REQUIRE(job->n_tensors >= 1 && job->n_tensors <= ngp_head::kMaxTensors, NGP_ERR_ARG,
                "march_rays_train_prebuilt_adam: 1..%d tensors", ngp_head::kMaxTensors);
    for (int q = 0; q < job->n_tensors; ++q) {
        NGP_REQUIRE(((reinterpret_cast<uintptr_t>(job->params[q]) | reinterpret_cast<uintptr_t>(job->exp_avg[q]) |
                      reinterpret_cast<uintptr_t>(job->exp_avg_sq[q])) & 15) == 0 &&
                        (reinterpret_cast<uintptr_t>(job->grads[q]) & 7) == 0 &&
                        (reinterpret_cast<uintptr_t>(job->half_params[q]) & 7) == 0,
                    NGP_ERR_ARG, "march_rays_train_prebuilt_adam: tensor %d misaligned", q);
    }
    EmitTail tail{};
    tail.st = static_cast<ngp_step::StepState*>(state);
    tail.end = true;
    tail.sa = ngp_step::ScalerArgs{growth_factor, backoff_factor, growth_interval, scaler_enabled,
                                   N ? 1.0f / (float)N : 0.0f};
    tail.loss_ray = loss_ray;
    tail.n_rays = N;
    if (n_nets > 0)
        if (int e = ngp_pack::build_jobs(n_nets, mlp_weights, in_dims, hidden_dims, num_layers, images, tail.jobs))
            return e;
    MarchAdam ma{};
    ma.tl = ngp_head::make_list(job->n_tensors, job->params, job->grads, job->exp_avg, job->exp_avg_sq,
                                job->half_params, job->sizes);
    // the bookkeeping is deferred to the emit tail (defer_end)
    ma.aa = ngp_head::AdamArgs{job->lr, job->beta1, job->beta2, job->eps, job->iters, job->zero_grads,
                               job->grad_mult, 1};
    ma.st = tail.st;
    NGP_REQUIRE(job->clear_bytes % 16 == 0 && (reinterpret_cast<uintptr_t>(job->clear) & 15) == 0, NGP_ERR_ARG,
                "march_rays_train_prebuilt_adam: clear must be 16-byte aligned, a multiple of 16 bytes");
    ma.clear = static_cast<uint4*>(job->clear);
    ma.clear16 = job->clear ? job->clear_bytes / 16 : 0u;
    ma.emit_launch = (job->flags & NGP_ADAM_JOB_EMIT_LAUNCH) != 0;
    // NGP_ADAM_JOB_TAIL_LATER: the bookkeeping and the packs ride in the next
    // launch (ngp_grid_encode_forward_fused_tail)
    const bool later = (job->flags & NGP_ADAM_JOB_TAIL_LATER) != 0;
    return march_train_impl(rays_o, rays_d, grid, bound, dt_gamma, max_steps, N, C, H, M, nears, fars,
                            xyzs, dirs, deltas, rays, counter, noises, workspace, workspace_bytes, false,
                            stream, later ? nullptr : &tail, &ma);
}

extern "C" int ngp_composite_rays_train_forward(const float* sigmas, const float* rgbs,
                                                const float* deltas, const int32_t* rays,
                                                uint32_t M, uint32_t N, float T_thresh,
                                                float* weights_sum, float* depth, float* image,
                                                void* stream) {
    if (N == 0) return NGP_OK;
    k_composite_train_fwd<<<ngp_div_up(N, kCompWaves), kCompWaves * 64, 0, ngp_stream(stream)>>>(
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
    k_composite_train_bwd<<<ngp_div_up(N, kCompWaves), kCompWaves * 64, 0, ngp_stream(stream)>>>(
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

/* ---- device-driven inference render loop --------------------------------- */

extern "C" size_t ngp_render_state_bytes(void) { return 2 * sizeof(RenderSlot); }

extern "C" int32_t* ngp_render_count(void* state, uint32_t iter) {
    return state ? &static_cast<RenderSlot*>(state)[iter & 1u].count : nullptr;
}

extern "C" int ngp_render_init(uint32_t N, const float* nears, int32_t* rays_alive, float* rays_t,
                               float* weights_sum, float* depth, float* image, void* state, void* stream) {
    NGP_REQUIRE(N >= 1 && N <= 0x7fffffffu / 8u, NGP_ERR_ARG, "render: N must be in [1, 2^28), got %u", N);
    NGP_REQUIRE(state && nears && rays_alive && rays_t && weights_sum && depth && image, NGP_ERR_ARG,
                "render_init: null buffer");
    k_render_init<<<ngp_div_up(N, 256), 256, 0, ngp_stream(stream)>>>(N, nears, rays_alive, rays_t, weights_sum,
                                                                      depth, image, static_cast<RenderSlot*>(state));
    return ngp_check_launch("render_init");
}

extern "C" int ngp_render_march(uint32_t N, uint32_t iter, void* state, const int32_t* rays_alive,
                                const float* rays_t, const float* rays_o, const float* rays_d, float bound,
                                float dt_gamma, uint32_t max_steps, uint32_t C, uint32_t H, const uint8_t* grid,
                                const float* fars, float* xyzs, float* dirs, float* deltas, const float* noises,
                                void* stream) {
    if (int e = check_cascade(C, H, max_steps)) return e;
    NGP_REQUIRE(N >= 1 && N <= 0x7fffffffu / 8u, NGP_ERR_ARG, "render: N must be in [1, 2^28), got %u", N);
    const MarchConst k = make_march_const(bound, dt_gamma, max_steps, C, H);
    k_render_march<<<ngp_div_up(N, 128), 128, 0, ngp_stream(stream)>>>(
        N, static_cast<RenderSlot*>(state), iter & 1u, rays_alive, rays_t, rays_o, rays_d, k, grid, fars, xyzs, dirs,
        deltas, noises);
    return ngp_check_launch("render_march");
}

extern "C" int ngp_render_composite(uint32_t N, uint32_t iter, uint32_t max_steps, void* state, float T_thresh,
                                    const int32_t* rays_alive, int32_t* rays_alive_next, float* rays_t,
                                    const float* sigmas, const void* color_out, const float* deltas,
                                    float* weights_sum, float* depth, float* image, void* stream) {
    NGP_REQUIRE(N >= 1 && N <= 0x7fffffffu / 8u, NGP_ERR_ARG, "render: N must be in [1, 2^28), got %u", N);
    NGP_REQUIRE(rays_alive != rays_alive_next, NGP_ERR_ARG, "render_composite: the alive lists must differ");
    k_render_composite<<<ngp_div_up(N, 256), 256, 0, ngp_stream(stream)>>>(
        N, max_steps, static_cast<RenderSlot*>(state), iter & 1u, T_thresh, rays_alive, rays_alive_next, rays_t,
        sigmas, static_cast<const ngp_half*>(color_out), deltas, weights_sum, depth, image);
    return ngp_check_launch("render_composite");
}
