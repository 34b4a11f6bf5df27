// Density-grid update of the NeRF renderer (reference nerf/renderer.py
// update_extra_state :498-598) on the device: the query points of an update,
// the EMA of the grid, its mean and the occupancy bitfield, with no host
// round trip between them. The densities themselves come from the fused grid
// forward + the sigma FFMLP's density epilogue (ngp_nerf_density_forward).
//
//   k_density_points  cascade-ordered points -> world xyz (the reference's
//                     float ops, :524-533 / :563-569) + flat cell index
//                     cascade * H^3 + morton3D (raymarching.cu:56-71)
//   k_density_ema     valid = grid >= 0 && tmp >= 0: grid = max(grid * decay,
//                     tmp) (:582-583); tmp reset to -1 for the next update;
//                     sum of clamp(grid, 0) for mean_density (:584)
//   k_density_pack    packbits (raymarching.cu:274-300) at min(mean_density,
//                     density_thresh) (:589-590), read on the device
//   k_density_occ_*   the partial update's "random occupied cells" draw
//                     (:555-558) without a host nonzero(): occupied cells of a
//                     cascade compacted in cell order, then sampled
//   k_density_draw    counter-based draws (the fused trainer's update): cell
//                     coordinates and noise
#include "ngp_common.h"

#include <algorithm>
#include <cfloat>

namespace {

constexpr uint32_t kMaxCascades = 16;

NGP_DEV uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
NGP_DEV uint32_t morton3(uint32_t x, uint32_t y, uint32_t z) {
    return expand_bits(x) | (expand_bits(y) << 1) | (expand_bits(z) << 2);
}
NGP_DEV uint32_t compact_bits(uint32_t x) {
    x &= 0x09249249u;
    x = (x ^ (x >> 2)) & 0x030C30C3u;
    x = (x ^ (x >> 4)) & 0x0300F00Fu;
    x = (x ^ (x >> 8)) & 0xFF0000FFu;
    x = (x ^ (x >> 16)) & 0x000003FFu;
    return x;
}

struct CascadeScales {
    float s[kMaxCascades];    // float(bound_c - hgs): the world extent of the cascade's cell centres
    float hgs[kMaxCascades];  // float(bound_c / H): half a cell
};

// Host side of :528-529: bound_c = min(2^c, bound), hgs = bound_c / H in double
// (Python floats), each rounded to float where torch multiplies by it.
static CascadeScales cascade_scales(uint32_t C, uint32_t H, float bound) {
    CascadeScales cs{};
    for (uint32_t c = 0; c < C && c < kMaxCascades; ++c) {
        const double bc = std::min((double)(1u << c), (double)bound);
        const double hgs = bc / (double)H;
        cs.s[c] = (float)(bc - hgs);
        cs.hgs[c] = (float)hgs;
    }
    return cs;
}

// counter-based RNG (as the fused sampler's, nerf_fused.hip)
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

// Point p of cascade p / ppc. coords: [P, 3] cell coordinates, or null for
// every cell of each cascade (ppc = H^3), whose noise rows are in the
// reference's meshgrid(x, y, z, 'ij') order. noise: [P, 3] uniform [0, 1).
__global__ void __launch_bounds__(256)
k_density_points(const int32_t* __restrict__ coords, const float* __restrict__ noise, uint32_t P, uint32_t ppc,
                 uint32_t H, CascadeScales cs, float* __restrict__ xyzs, int32_t* __restrict__ indices) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    const uint32_t cas = p / ppc;
    uint32_t c[3];
    size_t q = p;  // the draw's row of this point (noise)
    if (coords) {
        c[0] = (uint32_t)coords[(size_t)p * 3];
        c[1] = (uint32_t)coords[(size_t)p * 3 + 1];
        c[2] = (uint32_t)coords[(size_t)p * 3 + 2];
    } else {
        // every cell of the cascade: point i is the cell of Morton code i, so
        // a wave's 64 points form a 4x4x4 brick and their coarse levels'
        // corners share cache lines in the query's grid forward (row order
        // of the points: meshgrid, as the reference's draws, :521-533, read
        // from the cell's meshgrid row)
        // (H a power of two, where the Morton codes below H^3 are exactly the
        // cube's cells; otherwise meshgrid order)
        const uint32_t i = p - cas * ppc;
        if ((H & (H - 1)) == 0) {
            c[0] = compact_bits(i);
            c[1] = compact_bits(i >> 1);
            c[2] = compact_bits(i >> 2);
            q = (size_t)cas * ppc + ((size_t)c[0] * H + c[1]) * H + c[2];
        } else {
            c[0] = i / (H * H);
            c[1] = (i / H) % H;
            c[2] = i % H;
        }
    }
    // xyzs = 2 * coords.float() / (H - 1) - 1 (tensor / scalar: times the fp32 reciprocal)
    const float inv = 1.0f / (float)(H - 1);
    const float s = cs.s[cas], h = cs.hgs[cas];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float x = 2.0f * (float)c[k];
        x = x * inv;
        x = x - 1.0f;
        x = x * s;                                  // cas_xyzs = xyzs * (bound - hgs)
        const float n = noise[q * 3 + k];
        float j = n * 2.0f;                         // (rand * 2 - 1) * hgs
        j = j - 1.0f;
        j = j * h;
        xyzs[(size_t)p * 3 + k] = x + j;
    }
    indices[p] = (int32_t)(cas * H * H * H + morton3(c[0], c[1], c[2]));
}

NGP_DEV float torch_maximum(float a, float b) {  // torch.maximum: NaN propagates
    if (__builtin_isnan(a) || __builtin_isnan(b)) return __builtin_nanf("");
    return a > b ? a : b;
}

constexpr uint32_t kEmaThreads = 256;

// per-block partial sums (fixed order, no atomics) that k_density_pack adds up
constexpr uint32_t kEmaMaxBlocks = 1024;

__global__ void __launch_bounds__(kEmaThreads)
k_density_ema(float* __restrict__ grid, float* __restrict__ tmp, uint32_t n, float decay,
              double* __restrict__ partial) {
    __shared__ double wsum[kEmaThreads / 64];
    double acc = 0.0;
    // U cells' loads in flight per thread, then the cells in the original
    // order (the fp64 sum's order is unchanged)
    constexpr uint32_t U = 4;
    const uint32_t stride = gridDim.x * kEmaThreads;
    for (uint32_t i0 = blockIdx.x * kEmaThreads + threadIdx.x; i0 < n; i0 += U * stride) {
        float gv[U], tv[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t i = min(i0 + u * stride, n - 1);
            gv[u] = grid[i];
            tv[u] = tmp[i];
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t i = i0 + u * stride;
            if (i >= n) break;
            float g = gv[u];
            const float t = tv[u];
            if (g >= 0 && t >= 0) {
                g = torch_maximum(g * decay, t);
                grid[i] = g;
            }
            tmp[i] = -1.0f;
            acc += g < 0 ? 0.0 : (double)g;  // clamp(min=0)
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double b = 0.0;
#pragma unroll
        for (uint32_t w = 0; w < kEmaThreads / 64; ++w) b += wsum[w];
        partial[blockIdx.x] = b;
    }
}

// packbits at thresh = min(mean_density, density_thresh): mean_density is
// torch.mean(...).item() of the fp32 grid (a float32 value), compared with
// the Python float density_thresh in double; the winner is cast to float.
__global__ void __launch_bounds__(256)
k_density_pack(const float* __restrict__ grid, uint32_t nbytes, uint32_t n, const double* __restrict__ partial,
               uint32_t nparts, double density_thresh, uint8_t* __restrict__ bitfield, double* __restrict__ stats) {
    // every block adds the EMA's partial sums up in the same order
    __shared__ double s_sum[256];
    double acc = 0.0;
    {  // the loads in flight together, then the adds in the original order
        constexpr uint32_t U = 4;
        for (uint32_t i0 = threadIdx.x; i0 < nparts; i0 += 256 * U) {
            double v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = partial[min(i0 + 256 * u, nparts - 1)];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u)
                if (i0 + 256 * u < nparts) acc += v[u];
        }
    }
    s_sum[threadIdx.x] = acc;
    __syncthreads();
    for (uint32_t o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) s_sum[threadIdx.x] += s_sum[threadIdx.x + o];
        __syncthreads();
    }
    const double sum = s_sum[0];
    if (blockIdx.x == 0 && threadIdx.x == 0) stats[0] = sum;
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nbytes) return;
    const double mean = (double)(float)(sum / (double)n);
    const float thresh = (float)(mean < density_thresh ? mean : density_thresh);
    const float4* g = reinterpret_cast<const float4*>(grid + (size_t)b * 8);
    const float4 a = g[0], c = g[1];
    uint32_t bits = 0;
    bits |= (a.x > thresh) ? 1u : 0u;
    bits |= (a.y > thresh) ? 2u : 0u;
    bits |= (a.z > thresh) ? 4u : 0u;
    bits |= (a.w > thresh) ? 8u : 0u;
    bits |= (c.x > thresh) ? 16u : 0u;
    bits |= (c.y > thresh) ? 32u : 0u;
    bits |= (c.z > thresh) ? 64u : 0u;
    bits |= (c.w > thresh) ? 128u : 0u;
    bitfield[b] = (uint8_t)bits;
}

// ---- occupied-cell draw (partial update) ---------------------------------------
// Cells of a cascade are counted per 1024-cell block, the block counts scanned,
// and the occupied cells (grid > 0) written in cell order, so occ[k] is the
// k-th occupied cell of the cascade, as torch.nonzero lists them.
constexpr uint32_t kOccBlock = 1024;

__global__ void __launch_bounds__(kOccBlock)
k_density_occ_count(const float* __restrict__ grid, uint32_t H3, uint32_t* __restrict__ bcount) {
    __shared__ uint32_t wc[kOccBlock / 64];
    const uint32_t cas = blockIdx.y;
    const uint32_t i = blockIdx.x * kOccBlock + threadIdx.x;
    const bool occ = i < H3 && grid[(size_t)cas * H3 + i] > 0.0f;
    const uint64_t m = __ballot(occ);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
#pragma unroll
        for (uint32_t w = 0; w < kOccBlock / 64; ++w) s += wc[w];
        bcount[cas * gridDim.x + blockIdx.x] = s;
    }
}

// One workgroup per cascade: exclusive scan of its block counts in place;
// total[cas] = the cascade's occupied cells.
__global__ void __launch_bounds__(1024)
k_density_occ_scan(uint32_t* __restrict__ bcount, uint32_t nblk, uint32_t* __restrict__ total) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const uint32_t cas = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint32_t* bc = bcount + (size_t)cas * nblk;
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nblk; base += 1024) {
        const uint32_t v = base + t < nblk ? bc[base + t] : 0u;
        uint32_t incl = v;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = carry, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < 16; ++w) {
            before += w < wv ? wsum[w] : 0u;
            all += wsum[w];
        }
        if (base + t < nblk) bc[base + t] = before + incl - v;
        __syncthreads();
        if (t == 0) carry += all;
        __syncthreads();
    }
    if (t == 0) total[cas] = carry;
}

__global__ void __launch_bounds__(kOccBlock)
k_density_occ_write(const float* __restrict__ grid, uint32_t H3, const uint32_t* __restrict__ bcount,
                    uint32_t* __restrict__ occ) {
    __shared__ uint32_t wc[kOccBlock / 64];
    const uint32_t cas = blockIdx.y;
    const uint32_t i = blockIdx.x * kOccBlock + threadIdx.x;
    const bool o = i < H3 && grid[(size_t)cas * H3 + i] > 0.0f;
    const uint64_t m = __ballot(o);
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) wc[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = bcount[cas * gridDim.x + blockIdx.x];
    for (uint32_t w = 0; w < wv; ++w) before += wc[w];
    const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (o) occ[(size_t)cas * H3 + before + below] = i;
}

// The density draws' own RNG domain: the seed is XORed with this tag, so an
// update's draws are not functions of the same 32-bit values as the training
// sampler's (ngp_head.h lego_ray: rng_u32(seed, draw, ray, 0..5) with the same
// seed on rank 0).
constexpr uint32_t kDensityRngDomain = 0xd3a5b1c7u;

// Draws of the fused trainer's update (counter RNG over (seed ^ domain, update,
// point, stream)): full mode (occ null) draws only the noise of every cell;
// partial mode per cascade N = ppc / 2 uniform cells, then N cells drawn from
// the occupied list (uniform cells again where the cascade has none, as the
// reference's occ[randint(0, 0)] cannot), each with its noise.
struct PartialDraw {
    uint32_t ppc, H, seed, update;  // seed: already XORed with kDensityRngDomain
    const uint32_t* occ;            // occupied cells of each cascade, cell order
    const uint32_t* total;          // their counts
};

// The cell of partial-update point p (a pure function of the counter RNG and
// the occupied list, so the sorted query regenerates it instead of storing it)
NGP_DEV void partial_cell(const PartialDraw& d, uint32_t p, uint32_t c[3]) {
    const uint32_t cas = p / d.ppc, k = p - cas * d.ppc, half = d.ppc / 2;
    const uint32_t n_occ = d.total[cas];
    if (k >= half && n_occ > 0) {
        const uint32_t cell = d.occ[(size_t)cas * d.H * d.H * d.H + rng_u32(d.seed, d.update, p, 7) % n_occ];
        c[0] = compact_bits(cell);
        c[1] = compact_bits(cell >> 1);
        c[2] = compact_bits(cell >> 2);
    } else {
#pragma unroll
        for (int j = 0; j < 3; ++j) c[j] = rng_u32(d.seed, d.update, p, 8 + j) % d.H;
    }
}

__global__ void __launch_bounds__(256)
k_density_draw(uint32_t P, PartialDraw d, bool partial, int32_t* __restrict__ coords, float* __restrict__ noise) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    if (partial) {
        uint32_t c[3];
        partial_cell(d, p, c);
#pragma unroll
        for (int j = 0; j < 3; ++j) coords[(size_t)p * 3 + j] = (int32_t)c[j];
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) noise[(size_t)p * 3 + j] = rng_unit(d.seed, d.update, p, 1 + j);
}

// ---- partial-update points in brick order ----------------------------------------
// The partial update's cells are random draws, so consecutive points of a wave
// gather unrelated corners in the query's grid forward. tmp_grid is a max over
// the points, whatever their order, so the points of [lo, hi) are bucketed by
// their cell's Morton code >> shift (bricks of 2^shift cells, cascade-major):
// count (a block-private LDS histogram, flushed with one global atomic per
// nonzero bucket), scan, scatter (LDS ranks + one reservation per nonzero
// bucket and block). The order inside a bucket is unspecified; each rank sorts
// only its own slice of the draws, so the union over ranks is the draws.
constexpr uint32_t kSortThreads = 1024, kSortPerThread = 16,
                   kSortTile = kSortThreads * kSortPerThread;
constexpr uint32_t kSortMaxBuckets = 8192;

struct SortPlan {
    uint32_t lo, n, ppc, H, shift, nb;  // nb: buckets per cascade
};

NGP_DEV uint32_t sort_bucket(const int32_t* __restrict__ coords, uint32_t p, const SortPlan& sp) {
    const uint32_t cas = p / sp.ppc;
    const uint32_t m = morton3((uint32_t)coords[(size_t)p * 3], (uint32_t)coords[(size_t)p * 3 + 1],
                               (uint32_t)coords[(size_t)p * 3 + 2]);
    return cas * sp.nb + (m >> sp.shift);
}

__global__ void __launch_bounds__(kSortThreads)
k_density_sort_count(const int32_t* __restrict__ coords, SortPlan sp, uint32_t* __restrict__ counts) {
    __shared__ uint32_t hist[kSortMaxBuckets];
    const uint32_t nbt = sp.nb * ((sp.lo + sp.n - 1) / sp.ppc + 1);  // buckets up to the last point's cascade
    for (uint32_t b = threadIdx.x; b < nbt; b += kSortThreads) hist[b] = 0;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * kSortTile;
#pragma unroll 4
    for (uint32_t k = 0; k < kSortPerThread; ++k) {
        const uint32_t i = t0 + k * kSortThreads + threadIdx.x;
        if (i < sp.n) atomicAdd(&hist[sort_bucket(coords, sp.lo + i, sp)], 1u);
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbt; b += kSortThreads)
        if (hist[b]) atomicAdd(&counts[b], hist[b]);
}

// One workgroup: counts -> exclusive offsets in place.
__global__ void __launch_bounds__(1024)
k_density_sort_scan(uint32_t* __restrict__ counts, uint32_t nbt) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    if (t == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < nbt; base += 1024) {
        const uint32_t v = base + t < nbt ? counts[base + t] : 0u;
        uint32_t incl = v;
#pragma unroll
        for (uint32_t o = 1; o < 64; o <<= 1) {
            const uint32_t u = __shfl_up(incl, o, 64);
            if (lane >= o) incl += u;
        }
        if (lane == 63) wsum[wv] = incl;
        __syncthreads();
        uint32_t before = carry, all = 0;
#pragma unroll
        for (uint32_t w = 0; w < 16; ++w) {
            before += w < wv ? wsum[w] : 0u;
            all += wsum[w];
        }
        if (base + t < nbt) counts[base + t] = before + incl - v;
        __syncthreads();
        if (t == 0) carry += all;
        __syncthreads();
    }
}

// Same tiles as the count: each point's rank inside its bucket and block from
// an LDS atomic, one global reservation per nonzero bucket, then the point
// (k_density_points' arithmetic) at its slot.
__global__ void __launch_bounds__(kSortThreads)
k_density_sort_scatter(const int32_t* __restrict__ coords, const float* __restrict__ noise, SortPlan sp,
                       CascadeScales cs, uint32_t* __restrict__ cursor, float* __restrict__ xyzs,
                       int32_t* __restrict__ indices) {
    __shared__ uint32_t hist[kSortMaxBuckets];
    const uint32_t nbt = sp.nb * ((sp.lo + sp.n - 1) / sp.ppc + 1);
    for (uint32_t b = threadIdx.x; b < nbt; b += kSortThreads) hist[b] = 0;
    __syncthreads();
    const uint32_t t0 = blockIdx.x * kSortTile;
    uint32_t bk[kSortPerThread], rk[kSortPerThread];
#pragma unroll
    for (uint32_t k = 0; k < kSortPerThread; ++k) {
        const uint32_t i = t0 + k * kSortThreads + threadIdx.x;
        bk[k] = i < sp.n ? sort_bucket(coords, sp.lo + i, sp) : 0u;
        rk[k] = i < sp.n ? atomicAdd(&hist[bk[k]], 1u) : 0u;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbt; b += kSortThreads)
        if (hist[b]) hist[b] = atomicAdd(&cursor[b], hist[b]);
    __syncthreads();
    const float inv = 1.0f / (float)(sp.H - 1);
#pragma unroll
    for (uint32_t k = 0; k < kSortPerThread; ++k) {
        const uint32_t i = t0 + k * kSortThreads + threadIdx.x;
        if (i >= sp.n) continue;
        const uint32_t p = sp.lo + i, cas = p / sp.ppc;
        const uint32_t slot = hist[bk[k]] + rk[k];
        const float s = cs.s[cas], h = cs.hgs[cas];
        uint32_t c[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) c[j] = (uint32_t)coords[(size_t)p * 3 + j];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            float x = 2.0f * (float)c[j];
            x = x * inv;
            x = x - 1.0f;
            x = x * s;
            float jt = noise[(size_t)p * 3 + j] * 2.0f;
            jt = jt - 1.0f;
            jt = jt * h;
            xyzs[(size_t)slot * 3 + j] = x + jt;
        }
        indices[slot] = (int32_t)(cas * sp.H * sp.H * sp.H + morton3(c[0], c[1], c[2]));
    }
}

// shift and buckets per cascade: bricks of >= 2^9 cells, at most
// kSortMaxBuckets buckets over the cascades
static SortPlan sort_plan(uint32_t C, uint32_t H, uint32_t ppc, uint32_t lo, uint32_t n, uint32_t min_shift = 9) {
    uint32_t bits = 0;
    while ((1u << bits) < H) ++bits;
    const uint32_t mbits = 3 * bits;  // Morton codes of the cube are < 2^mbits
    uint32_t shift = std::min<uint32_t>(min_shift, mbits);
    while (shift < mbits && (size_t)C << (mbits - shift) > kSortMaxBuckets) ++shift;
    return SortPlan{lo, n, ppc, H, shift, 1u << (mbits - shift)};
}

// ---- partial-update draws generated in Morton order (the fused trainer) ---------
// A partial update draws, per cascade, N = H^3/4 uniform cells and N cells
// out of the occupied list, i.i.d. with replacement (renderer.py:548-558).
// tmp_grid is a max over the points, so only the multiset of draws matters,
// and the same multiset comes out sorted when each half's draws are made as
// uniform order statistics: U_(k) = S_k / S_N with S_k the prefix sums of N+1
// i.i.d. exponentials (Renyi). The uniform half's cell is then the Morton code
// floor(U_(k) H^3) and the occupied half's the occupied cell floor(U_(k) n_occ)
// (the list is in Morton order), so both halves come out in Morton order: the
// query's waves read neighbouring cells, as the full update's do, with no sort.
// Reproducible bit for bit (tests restate it in numpy): the exponentials come
// from the counter RNG through a fixed double-precision log (no libm) and are
// summed in 2^-32 fixed point (exact, any order); t and the cells in double.
constexpr uint32_t kOstatThreads = 256, kOstatPer = 4, kOstatChunk = kOstatThreads * kOstatPer;
constexpr uint32_t kOstatStream = 16;  // RNG streams 16 + 2 cascade + half (the draws' own: 1..10)

// -ln(u), u = (r >> 8 + 1) / 2^24, as 2^-32 fixed point: ln(v) of the integer
// v = 2^e m (m in [1, 2)) by the atanh series of s = (m - 1) / (m + 1), Horner
// in s^2, every operation a plain IEEE double one (-ffp-contract=off)
NGP_DEV uint64_t exp_fixed(uint32_t r) {
    const uint32_t v = (r >> 8) + 1u;                 // [1, 2^24]
    const int e = 31 - __clz(v);
    const double m = (double)v / (double)(1u << e);  // exact
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
    double q = 1.0 / 15.0;
    q = q * s2 + 1.0 / 13.0;
    q = q * s2 + 1.0 / 11.0;
    q = q * s2 + 1.0 / 9.0;
    q = q * s2 + 1.0 / 7.0;
    q = q * s2 + 1.0 / 5.0;
    q = q * s2 + 1.0 / 3.0;
    q = q * s2 + 1.0;
    const double lnm = 2.0 * s * q;
    const double E = (double)(24 - e) * 0.6931471805599453 - lnm;  // -ln(v / 2^24) >= 0
    return E > 0.0 ? (uint64_t)(E * 4294967296.0) : 0ull;
}

struct Ostat {
    uint32_t C, H, N, seed, update;  // N = draws per half; seed already XORed with the domain
    const uint32_t* occ;
    const uint32_t* total;
};

// exponential j of segment g = 2 cascade + half (j in [0, N])
NGP_DEV uint64_t ostat_exp(const Ostat& o, uint32_t g, uint32_t j) {
    return exp_fixed(rng_u32(o.seed, o.update, j, kOstatStream + g));
}

// Each block sums one chunk of a segment's N + 1 exponentials.
__global__ void __launch_bounds__(kOstatThreads)
k_ostat_sums(Ostat o, uint32_t chunks, unsigned long long* __restrict__ sums) {
    const uint32_t g = blockIdx.x / chunks, ch = blockIdx.x - g * chunks;
    unsigned long long acc = 0;
    for (uint32_t i = 0; i < kOstatPer; ++i) {
        const uint32_t j = ch * kOstatChunk + i * kOstatThreads + threadIdx.x;
        if (j <= o.N) acc += ostat_exp(o, g, j);
    }
#pragma unroll
    for (uint32_t off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    __shared__ unsigned long long w[kOstatThreads / 64];
    if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = w[0] + w[1] + w[2] + w[3];
}

// Each block: its chunk's prefix sums (the earlier chunks' sums + a block scan,
// exact integers), then its points k < N of the segment that fall in
// [lo, hi): cell, k_density_points' xyz arithmetic, index; in point order.
__global__ void __launch_bounds__(kOstatThreads)
k_ostat_points(Ostat o, uint32_t chunks, const unsigned long long* __restrict__ sums, uint32_t lo, uint32_t hi,
               CascadeScales cs, float* __restrict__ xyzs, int32_t* __restrict__ indices) {
    const uint32_t g = blockIdx.x / chunks, ch = blockIdx.x - g * chunks;
    const uint32_t cas = g >> 1, half = g & 1, ppc = 2 * o.N;
    const uint32_t p0 = cas * ppc + half * o.N;  // the segment's first point
    const uint32_t k0 = ch * kOstatChunk;
    if (p0 + k0 >= hi || p0 + min(k0 + kOstatChunk, o.N) <= lo) return;  // no point of the slice
    __shared__ unsigned long long s_w[kOstatThreads / 64];
    __shared__ unsigned long long s_base, s_tot;
    if (threadIdx.x < 64) {  // the earlier chunks' sums and the segment's total, wave 0
        unsigned long long b = 0, t = 0;
        constexpr uint32_t U = 8;  // loads in flight per lane (exact integer sums: any order)
        for (uint32_t c0 = threadIdx.x; c0 < chunks; c0 += 64 * U) {
            unsigned long long v[U];
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = sums[g * chunks + min(c0 + 64 * u, chunks - 1)];  // clamped
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) v[u] = c0 + 64 * u < chunks ? v[u] : 0ull;
#pragma unroll
            for (uint32_t u = 0; u < U; ++u) {
                const uint32_t c = c0 + 64 * u;
                b += c < ch ? v[u] : 0ull;
                t += v[u];
            }
        }
#pragma unroll
        for (uint32_t off = 32; off > 0; off >>= 1) {
            b += __shfl_down(b, off, 64);
            t += __shfl_down(t, off, 64);
        }
        if (threadIdx.x == 0) s_base = b, s_tot = t;
    }
    // thread t takes kOstatPer consecutive exponentials: j = k0 + t * kOstatPer + i
    uint64_t e[kOstatPer];
    unsigned long long mine = 0;
#pragma unroll
    for (uint32_t i = 0; i < kOstatPer; ++i) {
        const uint32_t j = k0 + threadIdx.x * kOstatPer + i;
        e[i] = j <= o.N ? ostat_exp(o, g, j) : 0ull;
        mine += e[i];
    }
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long incl = mine;
#pragma unroll
    for (uint32_t off = 1; off < 64; off <<= 1) {
        const unsigned long long u = __shfl_up(incl, off, 64);
        if (lane >= off) incl += u;
    }
    if (lane == 63) s_w[wv] = incl;
    __syncthreads();
    unsigned long long run = s_base + incl - mine;
    for (uint32_t w = 0; w < wv; ++w) run += s_w[w];
    const double tot = (double)s_tot;
    const uint32_t H3 = o.H * o.H * o.H, n_occ = half ? o.total[cas] : 0u;
    const float inv = 1.0f / (float)(o.H - 1);
    const float sc = cs.s[cas], hg = cs.hgs[cas];
#pragma unroll
    for (uint32_t i = 0; i < kOstatPer; ++i) {
        run += e[i];  // S_k, k = j: the (k+1)-th smallest of N uniforms is S_k / S_N
        const uint32_t k = k0 + threadIdx.x * kOstatPer + i, p = p0 + k;
        if (k >= o.N || p < lo || p >= hi) continue;
        const double t = (double)run / tot;
        uint32_t cell;
        if (half && n_occ > 0) {
            const uint32_t q = (uint32_t)fmin(floor(t * (double)n_occ), (double)(n_occ - 1));
            cell = o.occ[(size_t)cas * H3 + q];
        } else {
            cell = (uint32_t)fmin(floor(t * (double)H3), (double)(H3 - 1));
        }
        const uint32_t c[3] = {compact_bits(cell), compact_bits(cell >> 1), compact_bits(cell >> 2)};
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {  // k_density_points' arithmetic
            float x = 2.0f * (float)c[jj];
            x = x * inv;
            x = x - 1.0f;
            x = x * sc;
            float jt = rng_unit(o.seed, o.update, p, 1 + jj) * 2.0f;
            jt = jt - 1.0f;
            jt = jt * hg;
            xyzs[(size_t)(p - lo) * 3 + jj] = x + jt;
        }
        indices[p - lo] = (int32_t)(cas * H3 + cell);
    }
}

// The densities of the Morton-ordered points [lo, hi) -> tmp_grid: the draws
// of one cell are adjacent within a half, so the first point of each run takes
// the run's max and folds it in with one integer atomic max (a cell's runs in
// the uniform and the occupied half meet there; the two halves as two launches
// with a plain store and a read-modify-write were one launch more).
__global__ void __launch_bounds__(256)
k_density_run_max(const float* __restrict__ sigma, const int32_t* __restrict__ indices, uint32_t lo, uint32_t hi,
                  uint32_t N, float* __restrict__ tmp) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x, p = lo + i;
    if (p >= hi) return;
    const uint32_t seg_end = min(hi, (p / N + 1) * N);
    const int32_t c = indices[i];
    if (p > lo && p % N != 0 && indices[i - 1] == c) return;  // not the run's first point
    float m = sigma[i];
    for (uint32_t q = p + 1; q < seg_end && indices[q - lo] == c; ++q) m = fmaxf(m, sigma[q - lo]);
    // a cell can have a run in each half: the max as an integer max of the
    // float bits (sigma >= 0 and tmp's -1 order as their bits do as signed
    // integers), exact in any order, in one launch for both halves
    atomicMax(reinterpret_cast<int*>(tmp) + c, __float_as_int(m));
}

// The reference's bookkeeping after an update (renderer.py:593-595):
// mean_count = int(mean of the sample counts of the last `total` batches), from
// the fused trainer's step-counter ring (slot = batch % 16, written when the
// next batch is drawn) and the newest batch's counter. One thread.
__global__ void k_density_mean_count(const int32_t* __restrict__ step_counter, const int32_t* __restrict__ draw,
                                     const int32_t* __restrict__ counter, uint32_t total, uint32_t ahead,
                                     int64_t* __restrict__ out) {
    if (threadIdx.x != 0) return;
    const int32_t d = *draw;
    int64_t sum = 0;
    if (ahead) {  // the next batch is drawn: the newest count is in the ring too
        for (uint32_t k = 0; k < total; ++k) sum += step_counter[((d - 2 - (int32_t)k) & 15) * 2];
    } else {
        for (uint32_t k = 1; k < total; ++k) sum += step_counter[((d - 1 - (int32_t)k) & 15) * 2];
        sum += counter[0];
    }
    *out = sum / (int64_t)total;  // counts are >= 0: floor division
}

}  // namespace

extern "C" int ngp_density_mean_count(const int32_t* step_counter, const int32_t* draw, const int32_t* counter,
                                      uint32_t total, uint32_t ahead, int64_t* out, void* stream) {
    NGP_REQUIRE(step_counter && draw && counter && out, NGP_ERR_ARG, "density_mean_count: null pointer");
    NGP_REQUIRE(total >= 1 && total <= 16, NGP_ERR_ARG, "density_mean_count: total %u not in [1, 16]", total);
    k_density_mean_count<<<1, 64, 0, ngp_stream(stream)>>>(step_counter, draw, counter, total, ahead, out);
    return ngp_check_launch("density_mean_count");
}

extern "C" size_t ngp_density_grid_sort_workspace_bytes(uint32_t C, uint32_t H) {
    const SortPlan sp = sort_plan(C, H, 1, 0, 1);
    return (size_t)C * sp.nb * sizeof(uint32_t);
}

extern "C" int ngp_density_grid_points_sorted(const int32_t* coords, const float* noise, uint32_t P, uint32_t ppc,
                                              uint32_t C, uint32_t H, float bound, uint32_t lo, uint32_t hi,
                                              void* ws, size_t ws_bytes, float* xyzs, int32_t* indices,
                                              void* stream) {
    NGP_REQUIRE(coords && noise && xyzs && indices && ws, NGP_ERR_ARG,
                "density_grid_points_sorted: null coords / noise / xyzs / indices / workspace");
    NGP_REQUIRE(C >= 1 && C <= kMaxCascades && H >= 2 && H <= 1024, NGP_ERR_ARG,
                "density_grid_points_sorted: cascade %u / grid size %u out of range", C, H);
    NGP_REQUIRE(ppc > 0 && P == ppc * C && lo <= hi && hi <= P, NGP_ERR_ARG,
                "density_grid_points_sorted: P = %u is not %u points x %u cascades, or [%u, %u) outside it", P, ppc,
                C, lo, hi);
    NGP_REQUIRE(ws_bytes >= ngp_density_grid_sort_workspace_bytes(C, H), NGP_ERR_ARG,
                "density_grid_points_sorted: workspace of %zu bytes required, got %zu",
                ngp_density_grid_sort_workspace_bytes(C, H), ws_bytes);
    if (hi == lo) return NGP_OK;
    const SortPlan sp = sort_plan(C, H, ppc, lo, hi - lo);
    hipStream_t st = ngp_stream(stream);
    const size_t nbt = (size_t)C * sp.nb;
    if (hipMemsetAsync(ws, 0, nbt * sizeof(uint32_t), st) != hipSuccess)
        return ngp_set_error(NGP_ERR_HIP, "density_grid_points_sorted: counter clear failed");
    uint32_t* counts = static_cast<uint32_t*>(ws);
    const uint32_t blocks = ngp_div_up(sp.n, kSortTile);
    k_density_sort_count<<<blocks, kSortThreads, 0, st>>>(coords, sp, counts);
    k_density_sort_scan<<<1, 1024, 0, st>>>(counts, (uint32_t)nbt);
    k_density_sort_scatter<<<blocks, kSortThreads, 0, st>>>(coords, noise, sp, cascade_scales(C, H, bound), counts,
                                                            xyzs, indices);
    return ngp_check_launch("density_grid_points_sorted");
}

extern "C" int ngp_density_grid_points(const int32_t* coords, const float* noise, uint32_t P, uint32_t ppc,
                                       uint32_t C, uint32_t H, float bound, float* xyzs, int32_t* indices,
                                       void* stream) {
    NGP_REQUIRE(noise && xyzs && indices, NGP_ERR_ARG, "density_grid_points: null noise / xyzs / indices");
    NGP_REQUIRE(C >= 1 && C <= kMaxCascades && H >= 2 && H <= 1024, NGP_ERR_ARG,
                "density_grid_points: cascade %u / grid size %u out of range", C, H);
    NGP_REQUIRE(ppc > 0 && P == ppc * C, NGP_ERR_ARG, "density_grid_points: P = %u is not %u points x %u cascades",
                P, ppc, C);
    NGP_REQUIRE(coords || ppc == H * H * H, NGP_ERR_ARG, "density_grid_points: all-cell mode needs ppc = H^3");
    if (P == 0) return NGP_OK;
    k_density_points<<<ngp_div_up(P, 256), 256, 0, ngp_stream(stream)>>>(coords, noise, P, ppc, H,
                                                                         cascade_scales(C, H, bound), xyzs, indices);
    return ngp_check_launch("density_grid_points");
}

extern "C" int ngp_density_grid_ema_pack(float* grid, float* tmp_grid, uint32_t C, uint32_t H, float decay,
                                         double density_thresh, double* stats, uint8_t* bitfield, void* stream) {
    NGP_REQUIRE(grid && tmp_grid && stats && bitfield, NGP_ERR_ARG, "density_grid_ema_pack: null pointer");
    NGP_REQUIRE(H % 2 == 0 && C >= 1, NGP_ERR_ARG, "density_grid_ema_pack: grid size %u must be even", H);
    const uint32_t n = C * H * H * H;
    hipStream_t st = ngp_stream(stream);
    // stats: [0] the sum, [1..] the EMA blocks' partial sums
    const uint32_t blocks = std::min<uint32_t>(ngp_div_up(n, kEmaThreads), kEmaMaxBlocks);
    k_density_ema<<<blocks, kEmaThreads, 0, st>>>(grid, tmp_grid, n, decay, stats + 1);
    k_density_pack<<<ngp_div_up(n / 8, 256), 256, 0, st>>>(grid, n / 8, n, stats + 1, blocks, density_thresh,
                                                           bitfield, stats);
    return ngp_check_launch("density_grid_ema_pack");
}

extern "C" size_t ngp_density_grid_ostat_workspace_bytes(uint32_t C, uint32_t H) {
    const uint32_t N = H * H * H / 4, chunks = (N + 1 + kOstatChunk - 1) / kOstatChunk;
    return (size_t)2 * C * chunks * sizeof(unsigned long long);
}

extern "C" int ngp_density_grid_draw_sorted(const float* grid, uint32_t C, uint32_t H, uint32_t seed, uint32_t update,
                                            float bound, uint32_t lo, uint32_t hi, void* draw_ws, size_t draw_ws_bytes,
                                            void* ostat_ws, size_t ostat_ws_bytes, float* xyzs, int32_t* indices,
                                            void* stream) {
    NGP_REQUIRE(grid && draw_ws && ostat_ws && xyzs && indices, NGP_ERR_ARG, "density_grid_draw_sorted: null pointer");
    NGP_REQUIRE(C >= 1 && C <= kMaxCascades && H >= 2 && H <= 1024 && (H & (H - 1)) == 0 && H % 2 == 0, NGP_ERR_ARG,
                "density_grid_draw_sorted: cascade %u / grid size %u (a power of two) out of range", C, H);
    const uint32_t H3 = H * H * H, N = H3 / 4, P = C * 2 * N;
    NGP_REQUIRE(lo <= hi && hi <= P, NGP_ERR_ARG, "density_grid_draw_sorted: [%u, %u) outside the %u draws", lo, hi,
                P);
    NGP_REQUIRE(draw_ws_bytes >= ngp_density_grid_draw_workspace_bytes(C, H) &&
                    ostat_ws_bytes >= ngp_density_grid_ostat_workspace_bytes(C, H),
                NGP_ERR_ARG, "density_grid_draw_sorted: workspace too small");
    hipStream_t st = ngp_stream(stream);
    const uint32_t nblk = ngp_div_up(H3, kOccBlock);
    uint32_t* bcount = static_cast<uint32_t*>(draw_ws);
    uint32_t* total = bcount + (size_t)C * nblk;
    uint32_t* occ = reinterpret_cast<uint32_t*>(static_cast<char*>(draw_ws) +
                                                ((C * nblk + C) * sizeof(uint32_t) + 255) / 256 * 256);
    k_density_occ_count<<<dim3(nblk, C), kOccBlock, 0, st>>>(grid, H3, bcount);
    k_density_occ_scan<<<C, 1024, 0, st>>>(bcount, nblk, total);
    k_density_occ_write<<<dim3(nblk, C), kOccBlock, 0, st>>>(grid, H3, bcount, occ);
    if (hi == lo) return ngp_check_launch("density_grid_draw_sorted");
    const Ostat o{C, H, N, seed ^ kDensityRngDomain, update, occ, total};
    const uint32_t chunks = ngp_div_up(N + 1, kOstatChunk);
    unsigned long long* sums = static_cast<unsigned long long*>(ostat_ws);
    k_ostat_sums<<<2 * C * chunks, kOstatThreads, 0, st>>>(o, chunks, sums);
    k_ostat_points<<<2 * C * chunks, kOstatThreads, 0, st>>>(o, chunks, sums, lo, hi, cascade_scales(C, H, bound),
                                                             xyzs, indices);
    return ngp_check_launch("density_grid_draw_sorted");
}

extern "C" int ngp_density_grid_run_max(const float* sigma, const int32_t* indices, uint32_t C, uint32_t H,
                                        uint32_t lo, uint32_t hi, float* tmp_grid, void* stream) {
    NGP_REQUIRE(sigma && indices && tmp_grid, NGP_ERR_ARG, "density_grid_run_max: null pointer");
    const uint32_t N = H * H * H / 4;
    NGP_REQUIRE(N > 0 && lo <= hi && hi <= C * 2 * N, NGP_ERR_ARG, "density_grid_run_max: bad range");
    if (hi == lo) return NGP_OK;
    hipStream_t st = ngp_stream(stream);
    k_density_run_max<<<ngp_div_up(hi - lo, 256), 256, 0, st>>>(sigma, indices, lo, hi, N, tmp_grid);
    return ngp_check_launch("density_grid_run_max");
}

extern "C" size_t ngp_density_grid_draw_workspace_bytes(uint32_t C, uint32_t H) {
    const size_t H3 = (size_t)H * H * H, nblk = (H3 + kOccBlock - 1) / kOccBlock;
    return ((C * nblk + C) * sizeof(uint32_t) + 255) / 256 * 256 + C * H3 * sizeof(uint32_t);
}

extern "C" int ngp_density_grid_draw(const float* grid, uint32_t C, uint32_t H, uint32_t partial, uint32_t seed,
                                     uint32_t update, int32_t* coords, float* noise, void* ws, size_t ws_bytes,
                                     void* stream) {
    NGP_REQUIRE(noise && (!partial || (coords && grid && ws)), NGP_ERR_ARG, "density_grid_draw: null pointer");
    NGP_REQUIRE(!partial || ws_bytes >= ngp_density_grid_draw_workspace_bytes(C, H), NGP_ERR_ARG,
                "density_grid_draw: workspace too small");
    const uint32_t H3 = H * H * H;
    const uint32_t ppc = partial ? 2 * (H3 / 4) : H3, P = C * ppc;
    hipStream_t st = ngp_stream(stream);
    uint32_t *bcount = nullptr, *total = nullptr, *occ = nullptr;
    if (partial) {
        const uint32_t nblk = ngp_div_up(H3, kOccBlock);
        bcount = static_cast<uint32_t*>(ws);
        total = bcount + (size_t)C * nblk;
        occ = reinterpret_cast<uint32_t*>(static_cast<char*>(ws) + ((C * nblk + C) * sizeof(uint32_t) + 255) / 256 * 256);
        k_density_occ_count<<<dim3(nblk, C), kOccBlock, 0, st>>>(grid, H3, bcount);
        k_density_occ_scan<<<C, 1024, 0, st>>>(bcount, nblk, total);
        k_density_occ_write<<<dim3(nblk, C), kOccBlock, 0, st>>>(grid, H3, bcount, occ);
    }
    const PartialDraw d{ppc, H, seed ^ kDensityRngDomain, update, occ, total};
    k_density_draw<<<ngp_div_up(P, 256), 256, 0, st>>>(P, d, partial != 0, coords, noise);
    return ngp_check_launch("density_grid_draw");
}
