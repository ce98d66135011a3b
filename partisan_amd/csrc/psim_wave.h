// psim_wave.h -- wave-level list primitives shared by the node-round kernels
// (psim_consume.hip: HyParView + Plumtree; psim_strategy.hip: pluggable
// manager strategies).  A node's list lives one entry per lane (lanes >= n
// hold 0); membership, --, insert/delete in order become ballots and DPP
// lane shifts.
#pragma once
#include "psim_device.h"

namespace psim {

#define DEV __device__ __forceinline__

// ------------------------------------------------------------ wave ops --
DEV uint32_t lane_id() { return __lane_id(); }
DEV uint64_t ballot(bool p) { return __ballot(p); }
DEV uint32_t popc(uint64_t m) { return (uint32_t)__popcll(m); }
DEV int ffs64(uint64_t m) { return m ? __ffsll((long long)m) - 1 : -1; }
DEV uint64_t lt_mask() { return (1ull << lane_id()) - 1ull; }
DEV uint32_t shfl(uint32_t v, int src) { return (uint32_t)__shfl((int)v, src); }
DEV uint64_t shfl64(uint64_t v, int src) {
    uint32_t lo = shfl((uint32_t)v, src), hi = shfl((uint32_t)(v >> 32), src);
    return ((uint64_t)hi << 32) | lo;
}
DEV uint32_t rl(uint32_t v, int i) { return __builtin_amdgcn_readlane(v, i); }
DEV uint64_t rl64(uint64_t v, int i) {
    return ((uint64_t)rl((uint32_t)(v >> 32), i) << 32) | rl((uint32_t)v, i);
}
DEV uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// lane-distributed list V of n entries (lanes >= n hold 0)
DEV bool has(uint32_t V, uint32_t n, uint32_t e) { return ballot(lane_id() < n && V == e) != 0; }
DEV int idx_of(uint32_t V, uint32_t n, uint32_t e) { return ffs64(ballot(lane_id() < n && V == e)); }

// whole-wave DPP shifts (gfx9 wave_shl:1 / wave_shr:1): lane l reads lane
// l+1 / l-1 in one VALU op instead of an LDS permute
DEV uint32_t from_next(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}
DEV uint32_t from_prev(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}

// delete entry k (order preserving)
DEV void vdel(uint32_t& V, uint32_t& n, uint32_t k) {
    uint32_t l = lane_id();
    uint32_t nx = from_next(V);
    V = l < k ? V : (l + 1 < n ? nx : 0u);
    n--;
}
DEV void vdel64(uint64_t& V, uint32_t& n, uint32_t k) {
    uint32_t l = lane_id();
    uint64_t nx = ((uint64_t)from_next((uint32_t)(V >> 32)) << 32) | from_next((uint32_t)V);
    V = l < k ? V : (l + 1 < n ? nx : 0ull);
    n--;
}
// insert e at position pos
DEV void vins(uint32_t& V, uint32_t& n, uint32_t pos, uint32_t e) {
    uint32_t l = lane_id();
    uint32_t pv = from_prev(V);
    V = l < pos ? V : (l == pos ? e : (l <= n ? pv : 0u));
    n++;
}
DEV void vins64(uint64_t& V, uint32_t& n, uint32_t pos, uint64_t e) {
    uint32_t l = lane_id();
    uint64_t pv = ((uint64_t)from_prev((uint32_t)(V >> 32)) << 32) | from_prev((uint32_t)V);
    V = l < pos ? V : (l == pos ? e : (l <= n ? pv : 0ull));
    n++;
}
DEV bool vdel_val(uint32_t& V, uint32_t& n, uint32_t e) {
    int k = idx_of(V, n, e);
    if (k < 0) return false;
    vdel(V, n, (uint32_t)k);
    return true;
}
// sets:add_element/2 in sets:to_list/1 order: after every element whose
// bucket is <= the new element's bucket (new = youngest of its bucket)
DEV void view_add(uint32_t& V, uint32_t& n, uint32_t e) {
    uint32_t b = bucket16(e);
    uint32_t pos = popc(ballot(lane_id() < n && bucket16(V) <= b));
    vins(V, n, pos, e);
}

// v mod n for n < 2^16 with 32-bit arithmetic: v = hi*2^32 + lo
DEV uint32_t mod58(uint64_t v, uint32_t n) {
    uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    uint32_t p32 = (uint32_t)(0x100000000ull % n);
    return ((hi % n) * p32 + lo % n) % n;
}

// v mod n for n in [1, 64]: Horner over 15-bit digits; each digit step
// x = r * 2^15 + d < 2^21 divides by a v_rcp_f32 reciprocal, whose error
// moves the truncated quotient by at most one, fixed by one correction.
DEV uint32_t mod_small(uint64_t v, uint32_t n) {
    const float rn = __builtin_amdgcn_rcpf((float)n);
    uint32_t r = 0;
#pragma unroll
    for (int sh = 45; sh >= 0; sh -= 15) {
        uint32_t x = (r << 15) | (uint32_t)((v >> sh) & 0x7FFFu);
        uint32_t q = (uint32_t)((float)x * rn);
        int32_t rr = (int32_t)(x - q * n);
        rr = rr < 0 ? rr + (int32_t)n : rr;
        rr = rr >= (int32_t)n ? rr - (int32_t)n : rr;
        r = (uint32_t)rr;
    }
    return r;
}

}  // namespace psim
