// Wave-64 scans on DPP lane moves (row_shr within 16-lane rows, then
// row_bcast:15 / row_bcast:31 across rows): each step is one VALU
// instruction with a DPP source instead of a ds_bpermute round trip through
// the LDS crossbar (__shfl_up), so a 6-step scan is a short dependent chain
// of ALU ops. Lanes whose source is outside the move (or masked off) take
// the identity. gfx9-family only (row_bcast does not exist on gfx10+).
#pragma once
#include "ngp_common.h"

namespace ngp_dpp {

// DPP controls (GFX9 encoding)
constexpr int kRowShr1 = 0x111, kRowShr2 = 0x112, kRowShr4 = 0x114, kRowShr8 = 0x118;
constexpr int kRowBcast15 = 0x142, kRowBcast31 = 0x143;
constexpr int kWaveShr1 = 0x138;
constexpr int kQuadXor1 = 0xB1;  // quad_perm [1, 0, 3, 2]: the lane pair partner

template <int CTRL, int ROW_MASK>
NGP_DEV uint32_t mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xf, false);
}
template <int CTRL, int ROW_MASK>
NGP_DEV float movf(float v) {
    return __builtin_bit_cast(float, mov<CTRL, ROW_MASK>(__builtin_bit_cast(uint32_t, v)));
}

// one step of the segmented scan: (a, f) <- src (+) mine
template <int CTRL, int ROW_MASK>
NGP_DEV void seg_step2(float& a, float& b, uint32_t& f) {
    const float ta = movf<CTRL, ROW_MASK>(a), tb = movf<CTRL, ROW_MASK>(b);
    const uint32_t tf = mov<CTRL, ROW_MASK>(f);
    if (!f) {
        a += ta;
        b += tb;
    }
    f |= tf;
}

// Inclusive segmented sum of (a, b) over the wave: a lane with head set
// starts a new segment. Returns, per lane, the sum from its segment's head
// up to itself.
NGP_DEV void seg_scan2(float& a, float& b, bool head) {
    uint32_t f = head ? 1u : 0u;
    seg_step2<kRowShr1, 0xf>(a, b, f);
    seg_step2<kRowShr2, 0xf>(a, b, f);
    seg_step2<kRowShr4, 0xf>(a, b, f);
    seg_step2<kRowShr8, 0xf>(a, b, f);
    seg_step2<kRowBcast15, 0xa>(a, b, f);
    seg_step2<kRowBcast31, 0xc>(a, b, f);
}

// seg_scan2 for N value pairs sharing one segment structure (one flag move
// per step instead of one per pair).
template <int CTRL, int ROW_MASK, int N>
NGP_DEV void seg_stepn(float (&a)[N][2], uint32_t& f) {
    float t[N][2];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        t[i][0] = movf<CTRL, ROW_MASK>(a[i][0]);
        t[i][1] = movf<CTRL, ROW_MASK>(a[i][1]);
    }
    const uint32_t tf = mov<CTRL, ROW_MASK>(f);
    if (!f) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            a[i][0] += t[i][0];
            a[i][1] += t[i][1];
        }
    }
    f |= tf;
}

template <int N>
NGP_DEV void seg_scan_pairs(float (&a)[N][2], bool head) {
    uint32_t f = head ? 1u : 0u;
    seg_stepn<kRowShr1, 0xf, N>(a, f);
    seg_stepn<kRowShr2, 0xf, N>(a, f);
    seg_stepn<kRowShr4, 0xf, N>(a, f);
    seg_stepn<kRowShr8, 0xf, N>(a, f);
    seg_stepn<kRowBcast15, 0xa, N>(a, f);
    seg_stepn<kRowBcast31, 0xc, N>(a, f);
}

// Inclusive prefix sum over the wave.
NGP_DEV float scan_incl(float v) {
    v += movf<kRowShr1, 0xf>(v);
    v += movf<kRowShr2, 0xf>(v);
    v += movf<kRowShr4, 0xf>(v);
    v += movf<kRowShr8, 0xf>(v);
    v += movf<kRowBcast15, 0xa>(v);
    v += movf<kRowBcast31, 0xc>(v);
    return v;
}

// Inclusive prefix sum over the wave (integers).
NGP_DEV uint32_t scan_incl_u32(uint32_t v) {
    v += mov<kRowShr1, 0xf>(v);
    v += mov<kRowShr2, 0xf>(v);
    v += mov<kRowShr4, 0xf>(v);
    v += mov<kRowShr8, 0xf>(v);
    v += mov<kRowBcast15, 0xa>(v);
    v += mov<kRowBcast31, 0xc>(v);
    return v;
}

// The value of the lane pair partner (lane ^ 1): __shfl_xor(v, 1) without
// the LDS crossbar.
NGP_DEV float pair_swap(float v) { return movf<kQuadXor1, 0xf>(v); }

// The previous lane's value (lane 0 gets 0): __shfl_up(v, 1) without the
// LDS crossbar.
NGP_DEV uint32_t prev_lane(uint32_t v) { return mov<kWaveShr1, 0xf>(v); }

}  // namespace ngp_dpp
