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

// minimum over the wave's 64 lanes (DPP: row shifts, then the row
// broadcasts; lanes without a source keep their own value), in an SGPR
template <int CTRL, int ROW_MASK, int BANK_MASK>
DEV uint32_t dpp_min(uint32_t x) {
    const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, CTRL, ROW_MASK, BANK_MASK, false);
    return x < y ? x : y;
}
DEV uint32_t wave_min(uint32_t x) {
    x = dpp_min<0x111, 0xF, 0xF>(x);     // row_shr:1
    x = dpp_min<0x112, 0xF, 0xF>(x);     // row_shr:2
    x = dpp_min<0x113, 0xF, 0xF>(x);     // row_shr:3
    x = dpp_min<0x114, 0xF, 0xE>(x);     // row_shr:4, banks 1-3
    x = dpp_min<0x118, 0xF, 0xC>(x);     // row_shr:8, banks 2-3
    x = dpp_min<0x142, 0xA, 0xF>(x);     // row_bcast:15, rows 1 and 3
    x = dpp_min<0x143, 0xC, 0xF>(x);     // row_bcast:31, rows 2 and 3
    return __builtin_amdgcn_readlane(x, 63);
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
// bucket is <= the new element's bucket (new = youngest of its bucket);
// `bt` = the handle's bucket table (RoundArgs::btab, nullptr = default)
DEV void view_add(const uint8_t* bt, uint32_t& V, uint32_t& n, uint32_t e) {
    uint32_t b = bucket16(bt, e);
    uint32_t pos = popc(ballot(lane_id() < n && bucket16(bt, V) <= b));
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
// ceil(2^32 / n) for 2 <= n <= 64: for x < 2^26, x / n = mul_hi(x, M) exactly
// (the error x * (M - 2^32/n) / 2^32 < 1/64 never crosses an integer)
__constant__ const uint32_t kMagic[65] = {
    0x00000000u, 0x00000000u, 0x80000000u, 0x55555556u, 0x40000000u, 0x33333334u, 0x2AAAAAABu, 0x24924925u,
    0x20000000u, 0x1C71C71Du, 0x1999999Au, 0x1745D175u, 0x15555556u, 0x13B13B14u, 0x12492493u, 0x11111112u,
    0x10000000u, 0x0F0F0F10u, 0x0E38E38Fu, 0x0D79435Fu, 0x0CCCCCCDu, 0x0C30C30Du, 0x0BA2E8BBu, 0x0B21642Du,
    0x0AAAAAABu, 0x0A3D70A4u, 0x09D89D8Au, 0x097B425Fu, 0x0924924Au, 0x08D3DCB1u, 0x08888889u, 0x08421085u,
    0x08000000u, 0x07C1F07Du, 0x07878788u, 0x07507508u, 0x071C71C8u, 0x06EB3E46u, 0x06BCA1B0u, 0x06906907u,
    0x06666667u, 0x063E7064u, 0x06186187u, 0x05F417D1u, 0x05D1745Eu, 0x05B05B06u, 0x0590B217u, 0x0572620Bu,
    0x05555556u, 0x0539782Au, 0x051EB852u, 0x05050506u, 0x04EC4EC5u, 0x04D4873Fu, 0x04BDA130u, 0x04A7904Bu,
    0x04924925u, 0x047DC120u, 0x0469EE59u, 0x0456C798u, 0x04444445u, 0x04325C54u, 0x04210843u, 0x04104105u,
    0x04000000u,
};

// v mod n for a 58-bit v and 1 <= n <= 64: Horner over an 18-bit and two
// 20-bit digits, each step x = r * 2^20 + d < 2^26 divided by one mul_hi;
// all operands are wave-uniform, so this runs on the SALU
DEV uint32_t mod_small_m(uint64_t v, uint32_t n, uint32_t M) {
    if (n == 1) return 0;
    uint32_t x = (uint32_t)(v >> 40);
    uint32_t r = x - __umulhi(x, M) * n;
    x = (r << 20) | (uint32_t)((v >> 20) & 0xFFFFFu);
    r = x - __umulhi(x, M) * n;
    x = (r << 20) | (uint32_t)(v & 0xFFFFFu);
    return x - __umulhi(x, M) * n;
}
DEV uint32_t mod_small(uint64_t v, uint32_t n) { return mod_small_m(v, n, kMagic[n]); }
// the table in a register: lane l holds kMagic[l] (lane 0: kMagic[64]), so
// a lookup is one v_readlane instead of a scalar load and its wait
DEV uint32_t magic_lanes() {
    const uint32_t l = lane_id();
    return kMagic[l == 0 ? 64 : l];
}

}  // namespace psim
