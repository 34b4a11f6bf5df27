// Touched-entry gradient exchange of the replicated data-parallel step
// (nerf/exchange.py, DESIGN.md §7 option B).
//
// The reference trains data parallel through DDP (nerf/utils.py:325-327): an
// all-reduce of every gradient, then the full Adam on every rank. The fused
// step's live-row backward leaves the hash-table gradient a few percent dense,
// so instead each rank lists its nonzero (channel pair, half2) words, the
// lists are all-gathered, and every rank sums all ranks' lists into the same
// flat gradient and runs the same full Adam (world 1's march + Adam launch).
//
// Layout. The flat fp16 gradient is cut into bins of kBinPairs channel pairs
// (16 KB). A rank's list is one int64 buffer, [header (2 words) | bin table
// (n_bins words) | items (cap words)], so the step all-gathers one buffer of a
// fixed size (no host round trip: the exchange is captured with the step):
//   header  int32 count, int32 flags (bit 0: a non-finite value or the rank's
//           own GradScaler flag), 0, 0; zero before the list kernel runs (a
//           new buffer is; the reduce launch clears its rank's header)
//   table   per bin: (count << 32) | start of its items in the item area
//   items   (half2 bits << 32) | pair index, a bin's items contiguous
// A rank with more nonzero pairs than cap lists only cap of them; every rank
// sees that in the gathered headers, and every rank skips the update (the
// GradScaler flag's bit 1: no scale back-off) instead of applying a partial
// sum; the host sees that in the exchange's statistics and grows cap at its
// next check (SparseExchange.check, run from FusedTrainer.flush).
//
// Reduction. One workgroup per bin sums every rank's items of the bin into
// an LDS image of int64 values in 2^-24 fixed point (fp16 values are
// multiples of 2^-24 and at most 65504: exact, so the order the LDS atomics
// land in does not matter), then writes the whole bin of the gradient densely
// as fp16(sum / world): the integer sum (< 2^49) and 2^24 * world are exact
// doubles, so the double quotient is the correctly rounded mean; it is exact
// whenever the mean is an fp16 tie, and otherwise lies too far from any fp16
// tie for the double rounding to cross one (world < 2^10), so fp16() of it
// rounds the exact mean once. Every rank computes the same bits, and the ranks'
// parameters stay bit-identical with no parameter collective.
#include "ngp_common.h"

namespace {

constexpr uint32_t kThreads = 256;
constexpr uint32_t kBinPairs = 4096;                // 16 KB of the fp16 gradient
constexpr uint32_t kPerThread = kBinPairs / kThreads;  // 16 pairs = 4 x 16-B loads
constexpr uint32_t kHeader = 2;                     // int64 words before the bin table
constexpr double kFixed = 16777216.0;               // 2^24

NGP_DEV bool pair_nonfinite(uint32_t w) { return (w & 0x7c00u) == 0x7c00u || (w & 0x7c000000u) == 0x7c000000u; }

// Block-wide exclusive scan of one value per thread (256 threads).
NGP_DEV uint32_t block_scan(uint32_t v, uint32_t& total) {
    __shared__ uint32_t s_w[kThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
#pragma unroll
    for (uint32_t w = 0; w < kThreads / 64; ++w) {
        if (w < wave) base += s_w[w];
        total += s_w[w];
    }
    return base + x - v;
}

// One workgroup per bin: its nonzero pairs -> the item area, in index order.
__global__ void __launch_bounds__(kThreads)
k_xchg_list(const uint32_t* __restrict__ words, uint64_t n_pairs, const int32_t* __restrict__ inf_flag,
            int64_t* __restrict__ send, uint32_t n_bins, uint32_t cap) {
    const uint32_t bin = blockIdx.x;
    int32_t* hdr = reinterpret_cast<int32_t*>(send);
    const uint64_t p0 = (uint64_t)bin * kBinPairs;
    // thread t holds pairs p0 + 4 (t + 256 j) + k, j < 4, k < 4 (coalesced 16-B loads)
    uint32_t w[kPerThread];
#pragma unroll
    for (uint32_t j = 0; j < kPerThread / 4; ++j) {
        const uint64_t q = p0 / 4 + threadIdx.x + kThreads * j;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (q * 4 < n_pairs) v = reinterpret_cast<const uint4*>(words)[q];  // n_pairs % 4 == 0
        w[4 * j] = v.x, w[4 * j + 1] = v.y, w[4 * j + 2] = v.z, w[4 * j + 3] = v.w;
    }
    uint32_t mine = 0;
    bool bad = false;
#pragma unroll
    for (uint32_t i = 0; i < kPerThread; ++i) {
        const bool nf = pair_nonfinite(w[i]);
        bad |= nf;
        mine += ((w[i] & 0x7fff7fffu) != 0u && !nf) ? 1u : 0u;
    }
    if (__ballot(bad) != 0 && (threadIdx.x & 63) == 0) atomicOr(hdr + 1, 1);
    if (bin == 0 && threadIdx.x == 0 && inf_flag && *inf_flag) atomicOr(hdr + 1, 1);
    uint32_t total;
    uint32_t pos = block_scan(mine, total);
    __shared__ uint32_t s_start;
    if (threadIdx.x == 0) {
        s_start = total ? atomicAdd(reinterpret_cast<uint32_t*>(hdr), total) : 0u;
        send[kHeader + bin] = (int64_t)(((uint64_t)total << 32) | s_start);
    }
    __syncthreads();
    if (mine == 0) return;
    int64_t* items = send + kHeader + n_bins;
    pos += s_start;
#pragma unroll
    for (uint32_t i = 0; i < kPerThread; ++i) {
        if ((w[i] & 0x7fff7fffu) == 0u || pair_nonfinite(w[i])) continue;
        if (pos < cap) {
            const uint64_t p = p0 + 4 * (threadIdx.x + kThreads * (i / 4)) + (i & 3);
            items[pos] = (int64_t)(((uint64_t)w[i] << 32) | p);
        }
        ++pos;
    }
}

NGP_DEV long long half_fixed(uint32_t bits16) {
    union { uint16_t u; ngp_half h; } c;
    c.u = (uint16_t)bits16;
    return (long long)((double)c.h * kFixed);
}

// One workgroup per bin: every rank's items of the bin -> LDS int64 sums ->
// the bin of the gradient, dense.
__global__ void __launch_bounds__(kThreads)
k_xchg_reduce(const int64_t* __restrict__ recv, uint32_t world, uint64_t stride, uint32_t n_bins, uint32_t cap,
              uint64_t n_values, ngp_half* __restrict__ grad, int32_t* __restrict__ inf_flag,
              int32_t* __restrict__ stats, int64_t* __restrict__ send) {
    __shared__ unsigned long long acc[2 * kBinPairs];  // 64 KB
    const uint32_t bin = blockIdx.x;
    bool inf = false, over = false;
    uint32_t peak = 0;
    for (uint32_t r = 0; r < world; ++r) {
        const int32_t* h = reinterpret_cast<const int32_t*>(recv + r * stride);
        inf |= (h[1] & 1) != 0;
        over |= (uint32_t)h[0] > cap;
        peak = max(peak, (uint32_t)h[0]);
    }
    if (bin == 0 && threadIdx.x == 0) {
        // this rank's header starts the next step's list from zero (the
        // collective has read it: this launch is ordered after it)
        if (send) send[0] = 0;
        if (inf || over) atomicOr(inf_flag, (inf ? 1 : 0) | (over ? 2 : 0));
        if (over) atomicAdd(stats, 1);      // overflowed exchanges
        atomicMax(stats + 1, (int32_t)peak);  // the largest list seen
    }
    for (uint32_t i = threadIdx.x; i < 2 * kBinPairs; i += kThreads) acc[i] = 0ull;
    __syncthreads();
    if (!over) {
        const uint64_t p0 = (uint64_t)bin * kBinPairs;
        for (uint32_t r = 0; r < world; ++r) {
            const int64_t* base = recv + r * stride;
            const uint64_t t = (uint64_t)base[kHeader + bin];
            const uint32_t start = (uint32_t)t, cnt = (uint32_t)(t >> 32);
            const int64_t* items = base + kHeader + n_bins + start;
            for (uint32_t i = threadIdx.x; i < cnt; i += kThreads) {
                const uint64_t it = (uint64_t)items[i];
                const uint32_t p = (uint32_t)it - (uint32_t)p0, wv = (uint32_t)(it >> 32);
                if (p >= kBinPairs) continue;  // not this bin's: a corrupt list is not followed
                const long long a = half_fixed(wv & 0xffffu), b = half_fixed(wv >> 16);
                if (a) atomicAdd(&acc[2 * p], (unsigned long long)a);
                if (b) atomicAdd(&acc[2 * p + 1], (unsigned long long)b);
            }
        }
    }
    __syncthreads();
    // the bin's values, 8 per thread per round (16-B stores); an overflowed
    // exchange leaves zeros (the update is skipped on every rank)
    const double den = kFixed * (double)world;  // exact; divided, not multiplied by an inexact reciprocal
    const uint64_t v0 = (uint64_t)bin * 2 * kBinPairs;
    typedef _Float16 half8 __attribute__((ext_vector_type(8)));
    for (uint32_t c = threadIdx.x; c < 2 * kBinPairs / 8; c += kThreads) {
        if (v0 + 8 * c >= n_values) break;  // n_values % 8 == 0
        half8 o;
#pragma unroll
        for (uint32_t k = 0; k < 8; ++k) o[k] = (ngp_half)((double)(long long)acc[8 * c + k] / den);
        *reinterpret_cast<half8*>(grad + v0 + 8 * c) = o;
    }
}

}  // namespace

extern "C" uint32_t ngp_grad_exchange_bins(uint64_t n_values) {
    return (uint32_t)((n_values / 2 + kBinPairs - 1) / kBinPairs);
}

extern "C" uint64_t ngp_grad_exchange_words(uint64_t n_values, uint32_t cap) {
    return kHeader + ngp_grad_exchange_bins(n_values) + (uint64_t)cap;
}

extern "C" int ngp_grad_exchange_list(const void* grad_half, uint64_t n_values, const int32_t* inf_flag, void* send,
                                      uint32_t cap, void* stream) {
    NGP_REQUIRE(grad_half && send, NGP_ERR_ARG, "grad_exchange_list: null pointer");
    NGP_REQUIRE(n_values % 8 == 0 && n_values / 2 < 0xffffffffull, NGP_ERR_ARG,
                "grad_exchange_list: n_values % 8 == 0 and n_values / 2 < 2^32");
    NGP_REQUIRE((reinterpret_cast<uintptr_t>(grad_half) & 15) == 0 && (reinterpret_cast<uintptr_t>(send) & 7) == 0,
                NGP_ERR_ARG, "grad_exchange_list: grad 16-byte and send 8-byte aligned");
    hipStream_t st = ngp_stream(stream);
    const uint32_t n_bins = ngp_grad_exchange_bins(n_values);
    if (n_bins == 0) return NGP_OK;
    k_xchg_list<<<n_bins, kThreads, 0, st>>>(static_cast<const uint32_t*>(grad_half), n_values / 2, inf_flag,
                                             static_cast<int64_t*>(send), n_bins, cap);
    return ngp_check_launch("grad_exchange_list");
}

extern "C" int ngp_grad_exchange_reduce(const void* recv, int32_t world, uint32_t cap, void* grad_half,
                                        uint64_t n_values, int32_t* inf_flag, int32_t* stats, void* send,
                                        void* stream) {
    NGP_REQUIRE(recv && grad_half && inf_flag && stats, NGP_ERR_ARG, "grad_exchange_reduce: null pointer");
    NGP_REQUIRE(world >= 1 && world < 1024, NGP_ERR_ARG, "grad_exchange_reduce: 1 <= world < 1024 (the mean's single rounding)");
    NGP_REQUIRE(n_values % 8 == 0 && n_values / 2 < 0xffffffffull, NGP_ERR_ARG,
                "grad_exchange_reduce: n_values % 8 == 0 and n_values / 2 < 2^32");
    NGP_REQUIRE((reinterpret_cast<uintptr_t>(grad_half) & 15) == 0, NGP_ERR_ARG,
                "grad_exchange_reduce: grad 16-byte aligned");
    const uint32_t n_bins = ngp_grad_exchange_bins(n_values);
    if (n_bins == 0) return NGP_OK;
    k_xchg_reduce<<<n_bins, kThreads, 0, ngp_stream(stream)>>>(
        static_cast<const int64_t*>(recv), (uint32_t)world, ngp_grad_exchange_words(n_values, cap), n_bins, cap,
        n_values, static_cast<ngp_half*>(grad_half), inf_flag, stats, static_cast<int64_t*>(send));
    return ngp_check_launch("grad_exchange_reduce");
}
