// orbfe_kernels.hip — gfx950 (CDNA4) kernels of the ORB front-end hot path.
//
//   k_resize     cv::resize INTER_LINEAR 8U cascade (ComputePyramid, ORBextractor.cpp:1106-1132)
//   k_detect     per-cell FAST-9/16 + 3x3 NMS + iniTh/minTh fallback + ordered compaction
//                (ComputeKeyPointsOctTree cell loop, ORBextractor.cpp:768-828)
//   k_octree     DistributeOctTree (ORBextractor.cpp:539-762), one workgroup per (level, image)
//   k_orb        IC_Angle + GaussianBlur 7x7 (per keypoint neighbourhood) + steered BRIEF, one wavefront
//                per keypoint (ORBextractor.cpp:77-147, 1074-1103)
//   k_stereo     Frame.compute_stereo_matches (Frame.py:161-279), one wavefront per left keypoint
//   k_hamming_*  ORBMatcher.descriptor_distance batched (ORBMatcher.py:12-14)
//
// Integer / bitwise work: no MFMA.  Built with -ffp-contract=off; the only fused multiply-adds are the
// explicit fmaf() of the two descriptor sample coordinates (the reference build contracts exactly
// those, see oracle/orb_oracle.cpp) and glibc's sinf/cosf polynomials (fma in double).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "orbfe_common.h"
#include <type_traits>

#include "orbfe_kernels.h"

namespace orbfe {

// (x0, y0, x1, y1) of the 256 point pairs as floats: lane j reads bits j + 64 i as 4 x 16-byte loads
__constant__ __attribute__((aligned(16))) float c_pattern[1024] = {
#include "brief_pattern.inc"
};

// ------------------------------------------------------------------------------- small helpers
typedef float df2 __attribute__((ext_vector_type(2)));  // packed f32 (v_pk_mul/fma/add_f32)

// Buffer resource for a wave-uniform base pointer: loads take a 32-bit lane offset (no 64-bit address
// arithmetic per lane).  Dword 3 = 0x00020000, the gfx9 raw-buffer format word.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), 0, 0x7FFFFFFF, 0x00020000);
}

// Buffer resource over the wave-uniform p, bounded to nbytes bytes.  The halves go through uint32_t: the
// builtin returns int, and a sign-extended low half OR-ed into the 64-bit address corrupts its high bits
// whenever bit 31 of the address is set.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bounded_rsrc(const void* p, uint32_t nbytes) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | lo), 0,
                                             __builtin_amdgcn_readfirstlane(nbytes), 0x00020000);
}

// Buffer resource over the dword-aligned address at or below the wave-uniform p, bounded to
// bias + nbytes bytes; *bias = p's misalignment, so byte i of p sits at resource offset bias + i and a
// dword-aligned load covering it starts at (bias + i) & ~3 (never below the resource base).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t aligned_rsrc(const void* p, uint32_t nbytes, uint32_t* bias) {
    const uint64_t a = (uint64_t)(uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    *bias = lo & 3u;
    const uint32_t nb = __builtin_amdgcn_readfirstlane(nbytes);  // wave-uniform: an SGPR resource, never waterfalled
    return __builtin_amdgcn_make_buffer_rsrc((void*)(uintptr_t)(((uint64_t)hi << 32) | (lo & ~3u)), 0, nb + (lo & 3u),
                                             0x00020000);
}

// Wave-wide sum (wave-uniform result): DPP quad_perm / row_ror sums inside each 16-lane row, then the
// four row sums through v_readlane (no LDS-crossbar round trips).
// Two wave-wide sums at once: the DPP steps of the two interleave, so neither waits out the other's
// VALU-write -> DPP-read hazard (the s_nop the compiler puts between dependent DPP adds).
__device__ __forceinline__ void wave_sum2(int& a, int& b) {
    a += __builtin_amdgcn_update_dpp(0, a, 0xB1, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0xB1, 0xF, 0xF, false);
    a += __builtin_amdgcn_update_dpp(0, a, 0x4E, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0x4E, 0xF, 0xF, false);
    a += __builtin_amdgcn_update_dpp(0, a, 0x124, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0x124, 0xF, 0xF, false);
    a += __builtin_amdgcn_update_dpp(0, a, 0x128, 0xF, 0xF, false);
    b += __builtin_amdgcn_update_dpp(0, b, 0x128, 0xF, 0xF, false);
    a = __builtin_amdgcn_readlane(a, 0) + __builtin_amdgcn_readlane(a, 16) + __builtin_amdgcn_readlane(a, 32) +
        __builtin_amdgcn_readlane(a, 48);
    b = __builtin_amdgcn_readlane(b, 0) + __builtin_amdgcn_readlane(b, 16) + __builtin_amdgcn_readlane(b, 32) +
        __builtin_amdgcn_readlane(b, 48);
}

__device__ __forceinline__ int wave_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
           __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ int reflect101(int p, int n) {
    // one reflection suffices: every caller overshoots by less than n
    p = p < 0 ? -p : p;
    return p >= n ? 2 * n - 2 - p : p;
}

// cv::borderInterpolate(BORDER_REFLECT_101) for any overshoot: the reflection iterates (period 2 n - 2), a
// 1-pixel side maps everything to 0 — the 19-pixel padding of levels up to 19 px (copyMakeBorder,
// ORBextractor.cpp:1122-1128)
__device__ __forceinline__ int reflect101_iter(int p, int n) {
    if (n == 1) return 0;
    const int per = 2 * n - 2;
    p = (p < 0 ? -p : p) % per;
    return p >= n ? per - p : p;
}

// the scalar tail of the vertical pass: FixedPtCast<int, uchar, 22> (round half up) of INTER_LINEAR, or for
// the INTER_AREA fast path saturate_cast<uchar>(sum * 0.25f), i.e. sum / 4 rounded half to even (t = sum << 20)
__device__ __forceinline__ uint32_t resize_tail(uint32_t t, int area) {
    if (!area) return (t + (1u << 21)) >> 22;
    const uint32_t q = t >> 22, r = t & 0x3FFFFFu;
    return q + (r > 0x200000u || (r == 0x200000u && (q & 1u)));
}

__device__ __forceinline__ const uint8_t* level_ptr(const Geo& g, int l, const uint8_t* in, int64_t in_pitch,
                                                    const uint8_t* ws, int img, int* stride) {
    if (l == 0) {
        *stride = g.W;
        return in + (int64_t)img * in_pitch;
    }
    *stride = g.lv[l].pitch;
    return ws + (int64_t)img * g.ws_bytes + g.lv[l].ws_off;
}

// A FAST cell's geometry as dword scalar loads (s_load) and SALU unpacking: reading the int16 fields
// directly compiles to a per-lane global_load_ushort whose vmcnt wait also drains the next cell's ROI
// prefetch — a full memory round trip per cell on the critical path.
__device__ __forceinline__ CellGeo load_cell(const CellGeo* __restrict__ cells, int c) {
    static_assert(sizeof(CellGeo) == 20, "CellGeo layout: 5 dwords");
    const uint32_t* p = (const uint32_t*)(cells + c);
    const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
    CellGeo cg;
    cg.level = (int16_t)(w0 & 0xFFFFu);
    cg.kw = (int16_t)(w0 >> 16);
    cg.x0 = (int16_t)(w1 & 0xFFFFu);
    cg.y0 = (int16_t)(w1 >> 16);
    cg.x1 = (int16_t)(w2 & 0xFFFFu);
    cg.y1 = (int16_t)(w2 >> 16);
    cg.slot_off = (int)w3;
    cg.slot_cap = (int)w4;
    return cg;
}

// A packed level key's coordinates ((x + y * w) | score << 24, kKeyXYBits): y = mul_hi(xy, mag) >> sh is
// floor(xy / w) for every xy < 2^24 (mag = ceil(2^(31 + s) / w), sh = s - 1, s = ceil(log2 w): the error term
// xy * (mag * w - 2^(31 + s)) < 2^24 * w < 2^(31 + s)), then x = xy - y * w (both < 2^24: v_mad_u32_u24).
struct KeyDiv {
    uint32_t w, mag, sh;
};
__device__ __forceinline__ KeyDiv key_div(const LevelGeo& L) {
    return KeyDiv{(uint32_t)__builtin_amdgcn_readfirstlane(L.w), (uint32_t)__builtin_amdgcn_readfirstlane((int)L.kmag),
                  (uint32_t)__builtin_amdgcn_readfirstlane(L.ksh)};
}
__device__ __forceinline__ void key_xy(uint32_t k, KeyDiv kd, int& x, int& y) {
    const uint32_t xy = k & 0xFFFFFFu;
    const uint32_t q = __umulhi(xy, kd.mag) >> kd.sh;
    y = (int)q;
    x = (int)(xy - __umul24(q, kd.w));
}

// XCD-aware remap of a (gridDim.x, gridDim.y) grid.  Hardware block i (flattened, x fastest) runs on
// XCD i % 8; the remap hands each XCD a contiguous run of logical blocks, so neighbouring tiles / cells /
// bands — which share halo rows and partly used cache lines — meet in the same L2 instead of being
// fetched from HBM by several XCDs.  Wave-uniform results (SGPRs).
__device__ __forceinline__ void xcd_block(int& bx, int& by) {
    const int nb = gridDim.x * gridDim.y, hw = blockIdx.y * gridDim.x + blockIdx.x, per = nb >> 3;
    const int lb = hw < 8 * per ? (hw & 7) * per + (hw >> 3) : hw;
    by = __builtin_amdgcn_readfirstlane(lb / (int)gridDim.x);
    bx = __builtin_amdgcn_readfirstlane(lb - by * (int)gridDim.x);
}

// Block-wide exclusive scan of a[0..n) in LDS, in place; returns the total.  The first 256 threads own
// contiguous chunks, so prefixes follow array order; further threads (blocks of up to 1024) only take
// part in the barriers.  tmp: 257 ints of LDS.
__device__ int block_excl_scan(int* a, int n, int* tmp) {
    const int t = threadIdx.x;
    const int per = (n + 255) >> 8;
    const int b = t < 256 ? min(t * per, n) : n, e = min(b + per, n);
    int s = 0;
    for (int i = b; i < e; ++i) s += a[i];
    if (t < 256) tmp[t] = s;
    __syncthreads();
    if (t < 64) {
        const int v0 = tmp[4 * t], v1 = tmp[4 * t + 1], v2 = tmp[4 * t + 2], v3 = tmp[4 * t + 3];
        const int tot = v0 + v1 + v2 + v3;
        int inc = tot;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(inc, o, 64);
            if (t >= o) inc += y;
        }
        const int ex = inc - tot;
        tmp[4 * t] = ex;
        tmp[4 * t + 1] = ex + v0;
        tmp[4 * t + 2] = ex + v0 + v1;
        tmp[4 * t + 3] = ex + v0 + v1 + v2;
        if (t == 63) tmp[256] = inc;
    }
    __syncthreads();
    int run = t < 256 ? tmp[t] : 0;
    for (int i = b; i < e; ++i) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    const int total = tmp[256];
    __syncthreads();
    return total;
}

__device__ int block_sum(int v, int* red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    int s = 0;
    for (int i = 0; i < nw; ++i) s += red[i];
    __syncthreads();
    return s;
}

// ------------------------------------------------------------------------------- k_resize
// One 256-thread workgroup per band of kRsRows output rows of level l (l >= 1), full width.
//  * staging: the source rows the band reads (sy0(first) .. sy1(last) of level l-1) are one contiguous
//    byte range in memory for every level (stride W for the input, the 16-byte pitch for derived levels),
//    so they are copied to LDS as a flat run of aligned dwords, every load issued before the first wait;
//    LDS byte sh0 + r * stride + c holds source row ys_lo + r, column c (sh0 = the range's misalignment).
//  * the level's x coefficients become, per 4-pixel group, v_perm selectors into an 8-byte tap window
//    starting at the group's first sx plus the packed (a0, a1) weights, stored once per block as SoA.
//  * compute: per group and row, 2 x (3 LDS dwords, 2 v_alignbyte, 4 v_perm + 4 v_dot2_u32_u16) for the
//    horizontal taps, then OpenCV's vertical rounding; one aligned dword store per 4 output pixels.
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

// Horizontal taps of a group's 4th pixel from a window of its own (LevelGeo::wide): A3 = LDS byte address of
// its source pixel sx3, aa = its (a0, a1) weights.
__device__ __forceinline__ uint32_t resize_tap3(uint32_t A3, uint32_t aa) {
    typedef __attribute__((address_space(3))) const uint32_t lds_c32;
    const uint32_t o = A3 & 3u;
    lds_c32* w = (lds_c32*)(uintptr_t)(A3 - o);
    const uint32_t x = __builtin_amdgcn_alignbyte(w[1], w[0], o);
    return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(x, x, 0x0c010c00u)),
                                  __builtin_bit_cast(us2, aa), 0u, false);
}
constexpr int kRsSlots = 16;  // staged dwords per thread per pass

#ifdef ORBFE_DEV_VARIANTS  // the round-2 item-mapped kernel, for tools/microbench.py (tools/dbg/build_variant.sh)
template <int V>  // V: 0 full kernel; ablations for tools/microbench.py: 1 staging only, 2 compute only
__global__ __launch_bounds__(256) void k_resize(Geo g, int l, const uint8_t* __restrict__ in, int64_t in_pitch,
                                                uint8_t* __restrict__ ws, const ResizeX* __restrict__ xt,
                                                const ResizeY* __restrict__ yt) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rs_lds[];
    const LevelGeo& L = g.lv[l];
    uint4* s_xa = (uint4*)rs_lds;                        // per group: v_perm selectors, then (a0, a1) weights
    int* s_sx0 = (int*)(s_xa + 2 * L.rs_ngrp);
    // per output row of the band: LDS byte offsets of its two source rows' starts and b0 << 12, b1 << 12
    uint4* s_ry = (uint4*)(s_sx0 + L.rs_ngrp);
    uint32_t* s_src = (uint32_t*)(s_ry + kRsRows);       // staged source rows
    const LevelGeo& P = g.lv[l - 1];
    int bx, img;
    xcd_block(bx, img);  // neighbouring bands share source rows: keep them in one L2
    const int t = threadIdx.x;
    const int dy0 = bx * kRsRows, nrow = min(kRsRows, L.h - dy0);
    const int ngrp = (L.w + 3) >> 2;
    int sstride;
    const uint8_t* src = level_ptr(g, l - 1, in, in_pitch, ws, img, &sstride);
    const int ys_lo = yt[L.ytab_off + dy0].sy0, ys_hi = yt[L.ytab_off + dy0 + nrow - 1].sy1;
    const uintptr_t a0 = (uintptr_t)(src + (int64_t)ys_lo * sstride);
    const int sh0 = (int)(a0 & 3);
    const uint32_t* gsrc = (const uint32_t*)(a0 - sh0);
    const int ndw = ((ys_hi - ys_lo) * sstride + P.w + sh0 + 3) >> 2;
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    const uint32_t src_lds = (uint32_t)(uintptr_t)(lds_u32*)s_src;  // LDS address of the staged rows
    for (int base = 0; base < (V == 2 ? 0 : ndw); base += 256 * kRsSlots) {
        uint32_t v[kRsSlots];
#pragma unroll
        for (int k = 0; k < kRsSlots; ++k) {
            const int i = base + t + 256 * k;
            v[k] = i < ndw ? gsrc[i] : 0u;
        }
        if (base == 0) {
            const uint4* xg = (const uint4*)(xt + L.xtab_off);  // xtab_off is a multiple of 4
            for (int gi = t; gi < ngrp; gi += 256) {
                const uint4 q0 = xg[2 * gi], q1 = xg[2 * gi + 1];
                const uint32_t sx0 = q0.x;
                // byte r and r + 1 of the window as a u16 pair (selector 0x0c = zero byte)
                auto sel = [&](uint32_t sx) { const uint32_t r = sx - sx0; return r | ((r + 1) << 16) | 0x0c000c00u; };
                s_xa[2 * gi] = uint4{sel(q0.x), sel(q0.z), sel(q1.x), sel(q1.z)};
                s_xa[2 * gi + 1] = uint4{q0.y, q0.w, q1.y, q1.w};
                s_sx0[gi] = (int)sx0;
            }
            if (t < nrow) {
                const ResizeY y = yt[L.ytab_off + dy0 + t];
                s_ry[t] = uint4{src_lds + (uint32_t)(sh0 + (y.sy0 - ys_lo) * sstride),
                                src_lds + (uint32_t)(sh0 + (y.sy1 - ys_lo) * sstride), (uint32_t)y.b0 << 12,
                                (uint32_t)y.b1 << 12};
            }
        }
#pragma unroll
        for (int k = 0; k < kRsSlots; ++k) {
            const int i = base + t + 256 * k;
            if (i < ndw) s_src[i] = v[k];
        }
    }
    if (V == 2 && t < nrow) {
        const ResizeY y = yt[L.ytab_off + dy0 + t];
        s_ry[t] = uint4{src_lds + (uint32_t)(sh0 + (y.sy0 - ys_lo) * sstride),
                        src_lds + (uint32_t)(sh0 + (y.sy1 - ys_lo) * sstride), (uint32_t)y.b0 << 12, (uint32_t)y.b1 << 12};
    }
    __syncthreads();
    uint8_t* dst = ws + (int64_t)img * g.ws_bytes + L.ws_off + (int64_t)dy0 * L.pitch;
    if (V == 1) {
        if (t == 0) dst[0] = ((const uint8_t*)s_src)[sh0];
        return;
    }
    const int step_r = 256 / ngrp, step_g = 256 - step_r * ngrp;
    int rr = t / ngrp, grp = t - rr * ngrp;
    while (rr < nrow) {
        const uint4 ry = s_ry[rr];  // (LDS address of source row 0, of row 1, b0 << 12, b1 << 12)
        const uint4 e = s_xa[2 * grp], aa = s_xa[2 * grp + 1];
        const int sx0 = s_sx0[grp];
        auto taps = [&](uint32_t roff, uint32_t (&h)[4]) {
            const int A = (int)roff + sx0, o = A & 3;
            lds_u32* w = (lds_u32*)(uintptr_t)(uint32_t)(A - o);
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
            const uint32_t d0 = __builtin_amdgcn_alignbyte(w1, w0, o), d1 = __builtin_amdgcn_alignbyte(w2, w1, o);
            // S[sx] * a0 + S[sx + 1] * a1 (a1 = 0 past xmax: OpenCV's S[sx] * 2048)
            h[0] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.x)),
                                          __builtin_bit_cast(us2, aa.x), 0u, false);
            h[1] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.y)),
                                          __builtin_bit_cast(us2, aa.y), 0u, false);
            h[2] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.z)),
                                          __builtin_bit_cast(us2, aa.z), 0u, false);
            h[3] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.w)),
                                          __builtin_bit_cast(us2, aa.w), 0u, false);
        };
        uint32_t h0[4], h1[4];
        taps(ry.x, h0);
        taps(ry.y, h1);
        // OpenCV VResizeLinearVec_32s8u: v_mul_hi(S >> 4, beta) on int16 lanes, (x + 2) >> 2; h >> 4 <= 32640 so
        // the int16 pack never saturates and (x * b) >> 16 == mul_hi(x, b << 16) == mul_hi(x << 4, b << 12) ==
        // mul_hi(h & ~15, b << 12): a (fast) v_and instead of a (4-cycle) shift; the result is <= 255
        const uint32_t B0 = ry.z, B1 = ry.w;
        const int dx = 4 * grp;
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (__umulhi(h0[k] & ~15u, B0) + __umulhi(h1[k] & ~15u, B1) + 2) >> 2;
        if (dx + 3 >= L.xvec) {  // FixedPtCast<int, uchar, 22> past the last SIMD block
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (dx + k >= L.xvec) v[k] = resize_tail(h0[k] * (B0 >> 12) + h1[k] * (B1 >> 12), L.area);
        }
        // pixels past L.w land in the row's pitch padding
        *(uint32_t*)(dst + rr * L.pitch + dx) = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
        rr += step_r;
        grp += step_g;
        if (grp >= ngrp) {
            grp -= ngrp;
            ++rr;
        }
    }
}
#endif

// k_resize_rows: the same band, with the compute mapped so that a wave's row is uniform.  The block holds
// R_s row sets of W_g waves (64 W_g >= the level's groups): lane (w % W_g) * 64 + lane of a set owns one
// 4-pixel group for the whole band, its x selectors / weights in registers; set w / W_g takes rows
// set, set + R_s, ...  A row's source-row LDS addresses and vertical weights come from scalar loads of the
// y table, the store is a buffer store with the row offset in soffset: per 4 pixels only the taps, the
// vertical rounding and the pack are VALU work (k_resize's per-item row / table LDS reads, index wrap
// and 64-bit store address are gone).  Blocks of 256 <= 64 W_g R_s <= 512 threads (the host picks R_s).
template <bool MULTI>
__global__ __launch_bounds__(512) void k_resize_rows(Geo g, int l, const uint8_t* __restrict__ in, int64_t in_pitch,
                                                     uint8_t* __restrict__ ws, const ResizeX* __restrict__ xt,
                                                     const ResizeY* __restrict__ yt, int wg, int remw, int wgl,
                                                     int* __restrict__ zero_word) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rs_lds[];
    // staged source rows; the staging's pointers carry their address spaces (generic ones compile to flat
    // loads, which the compiler must wait for with vmcnt and lgkmcnt together)
    typedef __attribute__((address_space(3))) uint32_t lds_w32;
    typedef __attribute__((address_space(1))) const uint32_t glb_u32;
    lds_w32* s_src = (lds_w32*)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)rs_lds;
    const LevelGeo& L = g.lv[l];
    const LevelGeo& P = g.lv[l - 1];
    int bx, img;
    xcd_block(bx, img);
    const int t = threadIdx.x, nthr = blockDim.x;
    if (zero_word && blockIdx.x == 0 && blockIdx.y == 0 && t == 0) *zero_word = 0;
    const int rows = L.rs_rows;  // kRsRows, fewer for very wide levels (LevelGeo::rs_rows)
    const int dy0 = bx * rows, nrow = min(rows, L.h - dy0);
    const int ngrp = (L.w + 3) >> 2;
    int sstride;
    const uint8_t* src = level_ptr(g, l - 1, in, in_pitch, ws, img, &sstride);
    const ResizeY* yb = yt + L.ytab_off + dy0;
    const int ys_lo = yb[0].sy0, ys_hi = yb[nrow - 1].sy1;
    const uintptr_t a0 = (uintptr_t)(src + (int64_t)ys_lo * sstride);
    const int sh0 = (int)(a0 & 3);
    glb_u32* gsrc = (glb_u32*)(a0 - sh0);
    const int ndw = ((ys_hi - ys_lo) * sstride + P.w + sh0 + 3) >> 2;
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    const uint32_t src_lds = (uint32_t)(uintptr_t)s_src;
    // this thread's group: x selectors / weights straight from the table (issued with the staging loads)
    // remw = 1: the last wave takes the groups past the wg full 64-group chunks (rem < 64 of them) for all
    // rows of the band: lane j owns group wg * 64 + j % rem and rows j / rem, + 64 / rem, ... (a per-lane
    // row), instead of a mostly idle row-uniform wave per row.  A set has wgl <= 8 waves: when a level has
    // more chunks than that (rows wider than 2 048 px), a set's wave walks chunks c, c + wgl, ...
    const int wv = t >> 6, fullw = (nthr >> 6) - remw, nset = fullw / wgl;
    const bool remwave = wv >= fullw;
    const int set = __builtin_amdgcn_readfirstlane(remwave ? 0 : wv / wgl);
    const int rem = ngrp - wg * 64, lane = t & 63;
    const int rstep = remwave ? 64 / rem : nset;  // rows between a lane's rows in the remainder wave
    const int row0 = remwave ? lane / rem : set;
    int ch = remwave ? wg : wv - set * wgl;       // this wave's first 64-group chunk
    const int ch_step = remwave ? 1 : wgl, ch_end = remwave ? wg + 1 : wg;
    int grp = 0;
    bool own = false;
    uint4 e{}, aa{};
    int sx0 = 0;
    uint32_t d3 = 0;  // LevelGeo::wide: the 4th pixel's source column past the group's first
    auto chunk = [&](int c) {
        grp = remwave ? wg * 64 + lane % rem : c * 64 + lane;
        own = remwave ? lane < rstep * rem : grp < ngrp;
        if (own) {
            const uint4* xg = (const uint4*)(xt + L.xtab_off);
            const uint4 q0 = xg[2 * grp], q1 = xg[2 * grp + 1];
            sx0 = (int)q0.x;
            d3 = q1.z - q0.x;
            auto sel = [&](uint32_t sx) { const uint32_t r = sx - q0.x; return r | ((r + 1) << 16) | 0x0c000c00u; };
            e = uint4{sel(q0.x), sel(q0.z), sel(q1.x), sel(q1.z)};
            aa = uint4{q0.y, q0.w, q1.y, q1.w};
        }
    };
    chunk(ch);
    // staging by the first 256 threads (blocks have >= 256): compile-time strides, immediate LDS offsets.  The
    // loads go through a wave-uniform buffer resource: one VGPR offset for all slots, the slot and pass in the
    // SGPR offset, no 64-bit address arithmetic; the range test is one compare of the thread index against a
    // wave-uniform limit per slot, shared by the load and the LDS store (≈ 8 VALU per staged dword before, a
    // quarter of the stage's VALU).  The test must guard the load itself: the resource's bounds check does not
    // include the SGPR offset, so an unguarded slot past the run reads past the buffer.
    if (t < 256) {
        const __amdgpu_buffer_rsrc_t rsrc = bounded_rsrc((const void*)(uintptr_t)gsrc, (uint32_t)(4 * ndw));
        for (int base = 0; base < ndw; base += 256 * kRsSlots) {
            const int left = ndw - base;
            uint32_t v[kRsSlots];
#pragma unroll
            for (int k = 0; k < kRsSlots; ++k) {
                v[k] = 0u;
                if (t < left - 256 * k)
                    v[k] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, (uint32_t)(4 * t), (uint32_t)(4 * (base + 256 * k)), 0);
            }
            // one LDS address per pass (immediate offsets per slot)
            lds_w32* sp = s_src + base + t;
#pragma unroll
            for (int k = 0; k < kRsSlots; ++k)
                if (t < left - 256 * k) sp[256 * k] = v[k];
        }
    }
    __syncthreads();
    uint8_t* dst = ws + (int64_t)img * g.ws_bytes + L.ws_off + (int64_t)dy0 * L.pitch;
    const __amdgpu_buffer_rsrc_t rd = uniform_rsrc(dst);
    for (;;) {
        if (!own) return;  // only a level's last chunk is partial
        const int dx = 4 * grp;
        const bool tail = dx + 3 >= L.xvec;  // FixedPtCast<int, uchar, 22> past the last SIMD block
        const uint32_t lsrc = src_lds + (uint32_t)sh0 + (uint32_t)sx0;
        // psy: the previous row's second source row.  Full waves walk consecutive rows, and a row's first
        // source row is mostly the previous row's second: its taps are reused, not recomputed.  The two tap
        // sets alternate between ha and hb over a 2-row unrolled loop, so the reuse needs no register copies
        // (4-5 v_mov per row and 4-pixel group before)
        int psy = -1;
        auto row = [&](int rr, uint32_t (&h0)[4], uint32_t (&h1)[4], bool reuse) {
            const ResizeY y = yb[rr];  // full waves: uniform, scalar loads
            const uint32_t r0 = (uint32_t)((y.sy0 - ys_lo) * sstride), r1 = (uint32_t)((y.sy1 - ys_lo) * sstride);
            const uint32_t B0 = (uint32_t)y.b0 << 12, B1 = (uint32_t)y.b1 << 12;
            auto taps = [&](uint32_t roff, uint32_t (&h)[4]) {
                const uint32_t A = lsrc + roff, o = A & 3u;
                lds_u32* w = (lds_u32*)(uintptr_t)(A - o);
                const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
                const uint32_t d0 = __builtin_amdgcn_alignbyte(w1, w0, o), d1 = __builtin_amdgcn_alignbyte(w2, w1, o);
                h[0] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.x)),
                                              __builtin_bit_cast(us2, aa.x), 0u, false);
                h[1] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.y)),
                                              __builtin_bit_cast(us2, aa.y), 0u, false);
                h[2] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.z)),
                                              __builtin_bit_cast(us2, aa.z), 0u, false);
                h[3] = L.wide ? resize_tap3(A + d3, aa.w)
                              : __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.w)),
                                                       __builtin_bit_cast(us2, aa.w), 0u, false);
            };
            // h0 holds the taps of source row psy (the previous row's h1) when reuse applies
            if (!(reuse && y.sy0 == psy)) taps(r0, h0);
            taps(r1, h1);
            if (reuse) psy = y.sy1;
            uint32_t v[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = (__umulhi(h0[k] & ~15u, B0) + __umulhi(h1[k] & ~15u, B1) + 2) >> 2;
            if (tail) {
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    if (dx + k >= L.xvec) v[k] = resize_tail(h0[k] * (B0 >> 12) + h1[k] * (B1 >> 12), L.area);
            }
            // pixels past L.w land in the row's pitch padding
            __builtin_amdgcn_raw_buffer_store_b32(v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24), rd, (uint32_t)dx,
                                                  (uint32_t)(rr * L.pitch), 0);
        };
        uint32_t ha[4] = {0u, 0u, 0u, 0u}, hb[4] = {0u, 0u, 0u, 0u};
        if (!remwave) {  // set s: rows [s * per, (s + 1) * per), consecutive
            const int per = (nrow + nset - 1) / nset, rend = min(set * per + per, nrow);
            psy = -1;
            int rr = set * per;
            for (; rr + 1 < rend; rr += 2) {
                row(rr, ha, hb, true);
                row(rr + 1, hb, ha, true);
            }
            if (rr < rend) row(rr, ha, hb, true);
        } else {
            for (int rr = row0; rr < nrow; rr += rstep) row(rr, ha, hb, false);
        }
        if (!MULTI) return;  // one chunk per wave (every level up to 2 048 px): round 3's code exactly
        ch += ch_step;
        if (ch >= ch_end) return;
        chunk(ch);
    }
}

// k_resize_cascade: the whole pyramid (levels 1 .. L-1) in ONE launch for small batches, where the seven
// per-level launches are seven latency chains of a few microseconds each (8 pairs: 58 us of 233 per step).
// One 512-thread workgroup per (horizontal strip, image).  Strip s computes at every level the rows the
// next level's rows of the strip need (its own rows, plus a halo its neighbours also compute) and stores
// the rows it owns; ownership partitions every level (host: resize_strips), so each output row is written
// exactly once, with the arithmetic of k_resize_rows (same taps, same vertical rounding).  Level 0's source
// rows are staged from the input like k_resize_rows; every later level reads the previous level's strip
// from LDS, ping-ponging between two buffers (A: level 0 staging and even levels, B: odd levels).
// tab: per (strip, level) int16 {computed lo, hi, owned lo, hi}; offB / offX: byte offsets of buffer B and
// of the per-level x selector table in the dynamic LDS.
#ifndef ORBFE_CASCADE_NT
#define ORBFE_CASCADE_NT 1024
#endif
constexpr int kCasNT = ORBFE_CASCADE_NT;  // threads per strip workgroup
__global__ __launch_bounds__(kCasNT) void k_resize_cascade(Geo g, const uint8_t* __restrict__ in, int64_t in_pitch,
                                                        uint8_t* __restrict__ ws, const ResizeX* __restrict__ xt,
                                                        const ResizeY* __restrict__ yt, const int16_t* __restrict__ tab,
                                                        int offB, int offX, int* __restrict__ zero_word,
                                                        long long* __restrict__ prof) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rs_lds[];
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    typedef __attribute__((address_space(3))) uint32_t lds_w32;
    const int strip = blockIdx.x, img = blockIdx.y, t = threadIdx.x, lane = t & 63;
    const int wv = __builtin_amdgcn_readfirstlane(t >> 6), nwv = blockDim.x >> 6;
    if (zero_word && strip == 0 && img == 0 && t == 0) *zero_word = 0;
    // orbfe_debug_cascade_profile: wall-clock marks of the first thread, 32 per (image, strip): 0 start,
    // 1 staging issued + stored, 2 + l level l's rows may start (after its first barrier), 12 + l level l done
    long long* pm = prof ? prof + ((int64_t)img * gridDim.x + strip) * 32 : nullptr;
    auto mark = [&](int id) {
        if (pm && t == 0) pm[id] = (long long)wall_clock64();
    };
    mark(0);
    const int L = g.nlevels;
    const int16_t* st = tab + (int64_t)strip * L * 4;
    const uint32_t baseA = (uint32_t)(uintptr_t)(lds_u32*)rs_lds;
    const uint32_t baseB = baseA + (uint32_t)offB;
    // per group: v_perm selectors, then (a0, a1) weights; its first source column — double-buffered by level
    // parity: level l + 1's entries are loaded into registers while level l computes.  Every LDS and global
    // access goes through an address-space-qualified pointer: a generic one (an array of LDS pointers indexed
    // by the level's parity) compiles to flat loads, which count in vmcnt too — the item loop then waited for
    // the previous item's global stores before each table read.
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4u lds_u4;
    typedef __attribute__((address_space(3))) int lds_i32;
    typedef __attribute__((address_space(1))) const v4u glb_u4;
    auto u4 = [](v4u v) { return uint4{v.x, v.y, v.z, v.w}; };
    typedef __attribute__((address_space(1))) const uint32_t glb_u32;
    auto s_xa_of = [&](int par) { return (lds_u4*)(uintptr_t)(baseA + (uint32_t)offX + (uint32_t)(par * 32 * g.rs_ngrp)); };
    auto s_sx_of = [&](int par) {
        return (lds_i32*)(uintptr_t)(baseA + (uint32_t)offX + (uint32_t)(64 * g.rs_ngrp + par * 4 * g.rs_ngrp));
    };
    constexpr int kPre = 1024 / kCasNT;  // groups per thread held in registers (levels up to 4 096 px)
    uint4 pq0[kPre], pq1[kPre];
    auto prefetch = [&](int l) {
        if (l >= g.nlevels) return;
        glb_u4* xg = (glb_u4*)(xt + g.lv[l].xtab_off);
        const int ng = (g.lv[l].w + 3) >> 2;
#pragma unroll
        for (int k = 0; k < kPre; ++k) {
            const int gi = t + kCasNT * k;
            if (gi < ng) {
                pq0[k] = u4(xg[2 * gi]);
                pq1[k] = u4(xg[2 * gi + 1]);
            }
        }
    };
    auto commit = [&](int l) {
        lds_u4* sxa = s_xa_of(l & 1);
        lds_i32* ssx = s_sx_of(l & 1);
        const int ng = (g.lv[l].w + 3) >> 2;
#pragma unroll
        for (int k = 0; k < kPre; ++k) {
            const int gi = t + kCasNT * k;
            if (gi < ng) {
                const uint4 q0 = pq0[k], q1 = pq1[k];
                auto sel = [&](uint32_t sx) { const uint32_t r = sx - q0.x; return r | ((r + 1) << 16) | 0x0c000c00u; };
                sxa[2 * gi] = v4u{sel(q0.x), sel(q0.z), sel(q1.x), sel(q1.z)};
                sxa[2 * gi + 1] = v4u{q0.y, q0.w, q1.y, q1.w};
                ssx[gi] = (int)(q0.x | ((q1.z - q0.x) << 24));  // sx0, and the 4th pixel's offset (wide levels)
            }
        }
    };
    prefetch(1);
    // ---- level 0 rows the strip's level 1 needs, staged as a flat dword run (k_resize_rows' staging)
    uint32_t src_base = baseA, src_sh;
    int src_row0, src_stride;
    {
        const LevelGeo& L1 = g.lv[1];
        const ResizeY* yb = yt + L1.ytab_off;
        const int c0 = st[4], c1 = st[5];
        const int ys_lo = yb[c0].sy0, ys_hi = yb[c1 - 1].sy1;
        const uintptr_t a0 = (uintptr_t)(in + (int64_t)img * in_pitch + (int64_t)ys_lo * g.W);
        src_sh = (uint32_t)(a0 & 3);
        glb_u32* gsrc = (glb_u32*)(a0 - src_sh);
        const int ndw = ((ys_hi - ys_lo) * g.W + g.W + (int)src_sh + 3) >> 2;
        lds_w32* s_src = (lds_w32*)(uintptr_t)baseA;
        for (int base = 0; base < ndw; base += kCasNT * kRsSlots / 2) {
            uint32_t v[kRsSlots / 2];
#pragma unroll
            for (int k = 0; k < kRsSlots / 2; ++k) {
                const int i = base + t + kCasNT * k;
                v[k] = i < ndw ? gsrc[i] : 0u;
            }
#pragma unroll
            for (int k = 0; k < kRsSlots / 2; ++k) {
                const int i = base + t + kCasNT * k;
                if (i < ndw) s_src[i] = v[k];
            }
        }
        src_row0 = ys_lo;
        src_stride = g.W;
    }
    mark(1);
    for (int l = 1; l < L; ++l) {
        const LevelGeo& Lv = g.lv[l];
        const int c0 = st[4 * l], c1 = st[4 * l + 1], o0 = st[4 * l + 2], o1 = st[4 * l + 3];
        const int ngrp = (Lv.w + 3) >> 2, nch = (ngrp + 63) >> 6;
        // x selectors / weights of the level (k_resize's per-group form), loaded during the previous level
        commit(l);
        prefetch(l + 1);
        const lds_u4* s_xa = s_xa_of(l & 1);
        const lds_i32* s_sx0 = s_sx_of(l & 1);
        const ResizeY* yb = yt + Lv.ytab_off;
        const uint32_t dst_base = (l & 1) ? baseB : baseA;
        __syncthreads();  // selectors staged; the source rows complete (previous level / staging)
        mark(2 + l);
        uint8_t* gdst = ws + (int64_t)img * g.ws_bytes + Lv.ws_off;
        const int pitch = Lv.pitch;
        // the level's fields in registers (read from the kernel arguments once, not per item)
        const int lv_wide = __builtin_amdgcn_readfirstlane(Lv.wide), lv_xvec = __builtin_amdgcn_readfirstlane(Lv.xvec),
                  lv_area = __builtin_amdgcn_readfirstlane(Lv.area);
        // items (row, chunk), row-major; wave wv takes items wv, wv + nwv, ...: row / chunk advanced
        // incrementally (uniform), no division per item.  (Measured slower here: k_resize_rows' row sets — a
        // wave walks consecutive rows of one chunk, reusing the previous row's taps — 39 -> 43 us at 8 pairs,
        // and two items per step with both items' reads issued before either waits, 39 -> 49 us.)
        // items = rows: wave wv takes rows c0 + wv, + nwv, ...; per row its y entry and offsets once (scalar),
        // then every 64-group chunk of the row (a uniform loop).  Measured (tools/cascade_profile.py, traces
        // at 8 pairs): (row, chunk) items 39.7 us, rows 36.4; also tried and slower: row sets with the previous
        // row's taps reused (43), two items per step with all reads issued first (49), the y entries staged in
        // LDS instead of scalar loads (42).
        for (int r = c0 + wv; r < c1; r += nwv) {
            const ResizeY y = yb[r];
            const uint32_t r0 = (uint32_t)((y.sy0 - src_row0) * src_stride), r1 = (uint32_t)((y.sy1 - src_row0) * src_stride);
            const uint32_t B0 = (uint32_t)y.b0 << 12, B1 = (uint32_t)y.b1 << 12;
            const bool own = r >= o0 && r < o1;
            const uint32_t lrow = dst_base + (uint32_t)((r - c0) * pitch);
            uint8_t* grow = gdst + (int64_t)r * pitch;
            for (int ch = 0; ch < nch; ++ch) {
                const int grp = ch * 64 + lane;
                if (grp < ngrp) {
                    const uint4 e = u4(s_xa[2 * grp]), aa = u4(s_xa[2 * grp + 1]);
                    const int sxp = s_sx0[grp];
                    const uint32_t d3 = (uint32_t)sxp >> 24;
                    const uint32_t lsrc = src_base + src_sh + (uint32_t)(sxp & 0xFFFFFF);
                    auto taps = [&](uint32_t roff, uint32_t (&h)[4]) {
                        const uint32_t A = lsrc + roff, o = A & 3u;
                        lds_u32* w = (lds_u32*)(uintptr_t)(A - o);
                        const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
                        const uint32_t d0 = __builtin_amdgcn_alignbyte(w1, w0, o), d1 = __builtin_amdgcn_alignbyte(w2, w1, o);
                        h[0] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.x)),
                                                      __builtin_bit_cast(us2, aa.x), 0u, false);
                        h[1] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.y)),
                                                      __builtin_bit_cast(us2, aa.y), 0u, false);
                        h[2] = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.z)),
                                                      __builtin_bit_cast(us2, aa.z), 0u, false);
                        h[3] = lv_wide ? resize_tap3(A + d3, aa.w)
                                       : __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_perm(d1, d0, e.w)),
                                                                __builtin_bit_cast(us2, aa.w), 0u, false);
                    };
                    uint32_t h0[4], h1[4];
                    taps(r0, h0);
                    taps(r1, h1);
                    const int dx = 4 * grp;
                    uint32_t v[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) v[k] = (__umulhi(h0[k] & ~15u, B0) + __umulhi(h1[k] & ~15u, B1) + 2) >> 2;
                    if (dx + 3 >= lv_xvec) {  // FixedPtCast<int, uchar, 22> past the last SIMD block
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            if (dx + k >= lv_xvec) v[k] = resize_tail(h0[k] * (B0 >> 12) + h1[k] * (B1 >> 12), lv_area);
                    }
                    const uint32_t px = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
                    *(lds_w32*)(uintptr_t)(lrow + (uint32_t)dx) = px;
                    if (own) *(uint32_t*)(grow + dx) = px;  // pitch padding past w
                }
            }
        }
        src_base = dst_base;
        src_sh = 0;
        src_row0 = c0;
        src_stride = pitch;
        __syncthreads();  // this level's rows complete before the next level reads them / the selectors change
        mark(12 + l);
    }
}

// ------------------------------------------------------------------------------- k_detect
// One wavefront per (cell, image).  FAST "M" of a pixel:
//   M = max(v - min_arc max9, max_arc min9 - v) over the 16 arcs of 9 contiguous circle pixels;
//   the pixel is a segment-test corner at threshold t iff M > t, and OpenCV's cornerScore is M - 1.
// Work is done on horizontal pixel pairs (x, x + 1), x even, in packed f16: pixel values live in LDS as
// u16 0x3C00 | p, normal f16 numbers in [1, 2) ordered exactly like p, so v_pk_maximum3/minimum3_f16
// are exact and differences of the raw u16 bits are differences of p.
//  1. ROI -> LDS (u16, pitch RP, ROI column c at index c + 1 so even window columns are dword
//     aligned): 16 lanes per row each read one dword from the 4-byte aligned start of column -1, take
//     the next dword from the neighbour lane (DPP), re-align with v_alignbyte and widen with v_perm; the
//     next cell's loads are in flight during this cell's compute.
//  2. Pre-test, every pair: P = max(v - min_k max(c_k, c_k+1), max_k min(c_k, c_k+1) - v) over the
//     circularly adjacent cardinal pairs (circle points 0, 4, 8, 12) bounds M from above, because every
//     arc of 9 contains such a pair (computed as max(v - max(min(c0, c2), min(c1, c3)), ...): every
//     cycle edge joins an even and an odd cardinal).  Pairs with P <= tq = min(iniTh, minTh) in both pixels have M <= tq:
//     neither corners nor relevant NMS neighbours at either threshold; they keep M = 0.  The others are
//     queued in row-major order (ballot + mbcnt).  (Queueing single pixels halves the M work per pixel
//     but not per cell: a cell's queue is a few 64-entry steps either way, measured slower.)
//  3. Exact M of the queued pairs -> a u8 M map with a zero border (half the LDS of a u16 map: detect is
//     occupancy-bound, one 64-thread workgroup per wave); pairs with a pixel above max(tq, 1) are
//     compacted in place into the same queue (row-major) for NMS.
//  4. NMS over that queue, two pixels per lane.  For t >= 1, "score > every 8-neighbour's score at t" (neighbours outside the
//     window or not corners at t score 0) is equivalent to M > t and M > max(8-neighbour M): a neighbour
//     with M <= t is below M anyway.  So the local-max test is threshold independent: one pass decides
//     iniTh and minTh together, and the iniTh -> minTh fallback (ORBextractor.cpp:811-815) only picks
//     which survivor list is kept.  Kept pixels are written in the queue's row-major order, i.e.
//     cv::FAST's output order.
typedef _Float16 fd_h2 __attribute__((ext_vector_type(2)));
typedef short fd_s2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ fd_h2 fd_h(uint32_t v) { return __builtin_bit_cast(fd_h2, v); }
__device__ __forceinline__ fd_s2 fd_s(fd_h2 v) { return __builtin_bit_cast(fd_s2, v); }
__device__ __forceinline__ fd_h2 fd_max(fd_h2 a, fd_h2 b) { return __builtin_elementwise_maximum(a, b); }
__device__ __forceinline__ fd_h2 fd_min(fd_h2 a, fd_h2 b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ fd_h2 fd_max3(fd_h2 a, fd_h2 b, fd_h2 c) { return fd_max(fd_max(a, b), c); }
__device__ __forceinline__ fd_h2 fd_min3(fd_h2 a, fd_h2 b, fd_h2 c) { return fd_min(fd_min(a, b), c); }
template <int DX>
__device__ __forceinline__ fd_h2 fd_pair(const uint32_t* q) {  // u16 pair at column offset DX
    if constexpr ((DX & 1) == 0) return fd_h(q[DX / 2]);
    else return fd_h(__builtin_amdgcn_alignbyte(q[(DX + 1) / 2], q[(DX - 1) / 2], 2));
}

// Upper bounds of the two adjacent pixel pairs at dwords R and R + 1 (pixels x .. x + 3), sharing the
// cardinal rows: 6 dwords of the centre row, 2 above, 2 below.
template <int S>
__device__ __forceinline__ void fast_bound_quad(const uint32_t* R, fd_s2& bA, fd_s2& bB) {
    const uint32_t m2 = R[-2], m1 = R[-1], z0 = R[0], p1 = R[1], p2 = R[2], p3 = R[3];
    const uint32_t u0 = R[-3 * S], u1 = R[-3 * S + 1], d0 = R[3 * S], d1 = R[3 * S + 1];
    auto bound = [](uint32_t v, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
        const fd_h2 h0 = fd_h(c0), h1 = fd_h(c1), h2 = fd_h(c2), h3 = fd_h(c3);
        // min over the 4 cycle edges (i, i + 1) of max(h_i, h_i+1): every edge joins an even and an odd
        // cardinal, so it is max(min(h0, h2), min(h1, h3)) (3 ops instead of 6); dually for b
        const fd_h2 a = fd_max(fd_min(h0, h2), fd_min(h1, h3));
        const fd_h2 b = fd_min(fd_max(h0, h2), fd_max(h1, h3));
        const fd_s2 vs = __builtin_bit_cast(fd_s2, v);
        return __builtin_elementwise_max(vs - fd_s(a), fd_s(b) - vs);
    };
    // cardinals in circle order: 0 = (0, +3), 4 = (+3, 0), 8 = (0, -3), 12 = (-3, 0)
    bA = bound(z0, d0, __builtin_amdgcn_alignbyte(p2, p1, 2), u0, __builtin_amdgcn_alignbyte(m1, m2, 2));
    bB = bound(p1, d1, __builtin_amdgcn_alignbyte(p3, p2, 2), u1, __builtin_amdgcn_alignbyte(z0, m1, 2));
}

// Exact M of the pixel pair at dword R (row stride S dwords), as biased u16 x2.
template <int S>
__device__ __forceinline__ uint32_t fast_m_pair(const uint32_t* R) {
    const fd_h2 p[16] = {fd_pair<0>(R + 3 * S),  fd_pair<1>(R + 3 * S),  fd_pair<2>(R + 2 * S),  fd_pair<3>(R + S),
                         fd_pair<3>(R),          fd_pair<3>(R - S),      fd_pair<2>(R - 2 * S),  fd_pair<1>(R - 3 * S),
                         fd_pair<0>(R - 3 * S),  fd_pair<-1>(R - 3 * S), fd_pair<-2>(R - 2 * S), fd_pair<-3>(R - S),
                         fd_pair<-3>(R),         fd_pair<-3>(R + S),     fd_pair<-2>(R + 2 * S), fd_pair<-1>(R + 3 * S)};
    fd_h2 mx3[16], mn3[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mx3[k] = fd_max3(p[k], p[(k + 1) & 15], p[(k + 2) & 15]);
        mn3[k] = fd_min3(p[k], p[(k + 1) & 15], p[(k + 2) & 15]);
    }
    fd_h2 lo = fd_max3(mx3[0], mx3[3], mx3[6]), hi = fd_min3(mn3[0], mn3[3], mn3[6]);
#pragma unroll
    for (int k = 1; k < 15; k += 2) {
        lo = fd_min3(lo, fd_max3(mx3[k], mx3[(k + 3) & 15], mx3[(k + 6) & 15]),
                     fd_max3(mx3[k + 1], mx3[(k + 4) & 15], mx3[(k + 7) & 15]));
        hi = fd_max3(hi, fd_min3(mn3[k], mn3[(k + 3) & 15], mn3[(k + 6) & 15]),
                     fd_min3(mn3[k + 1], mn3[(k + 4) & 15], mn3[(k + 7) & 15]));
    }
    lo = fd_min(lo, fd_max3(mx3[15], mx3[2], mx3[5]));
    hi = fd_max(hi, fd_min3(mn3[15], mn3[2], mn3[5]));
    const fd_s2 v = __builtin_bit_cast(fd_s2, R[0]);
    const fd_s2 m = __builtin_elementwise_max(__builtin_elementwise_max(v - fd_s(lo), fd_s(hi) - v), fd_s2{0, 0});
    return __builtin_bit_cast(uint32_t, m) | 0x3C003C00u;
}

__device__ __forceinline__ int imax3(int a, int b, int c) { return max(max(a, b), c); }

// o +/- (this lane's bit of the lane mask m): one v_addc / v_subb with the mask as the carry (the compiler's
// form of o + (int)inverse_ballot(m) is a v_cndmask and an add)
__device__ __forceinline__ int fd_plus_bit(int o, uint64_t m) {
    int r;
    uint64_t co;
    asm("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(o), "s"(m));
    return r;
}
__device__ __forceinline__ int fd_minus_bit(int o, uint64_t m) {
    int r;
    uint64_t co;
    asm("v_subb_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(co) : "v"(o), "s"(m));
    return r;
}

// cells per k_detect wavefront: 4 (the next cell's ROI loads overlap this one), or 1 for batches too small to
// give the chip >= 8 waves per CU that way (a frame pair: 610 waves of 4 cells, 2 440 of one)
constexpr int kFdCells = 4;
#ifndef ORBFE_FD_SMALL_CELLS
#define ORBFE_FD_SMALL_CELLS 1
#endif
constexpr int kFdSmallCells = ORBFE_FD_SMALL_CELLS;  // cells per wave for small batches (1 or 2)

__device__ __forceinline__ int lanes_below(uint64_t b) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0));
}

// u16 elements of k_detect's ROI area: the ROI itself, and after the M stage the minTh survivors of a cell
// (u32 records, at most slot_cap = Geo::fd_alt); a multiple of 8 so the M map after it is 16-byte aligned
__host__ __device__ inline int detect_roi_elems(const Geo& g, int rp) {
    const int n = rp * g.max_rh > 2 * g.fd_alt ? rp * g.max_rh : 2 * g.fd_alt;
    return (n + 7) & ~7;
}

// V: 0 full kernel; ablations for tools/microbench.py: 1 ROI staging only, 2 + pre-test, 3 + M.
// RP: ROI pitch in u16 (48, 64 or 96; >= widest ROI + 3).  NS: staged row slots (4 rows each, >= max_rh / 4).
// 5 waves per SIMD (<= 96 VGPRs; 4 for the wider / taller ROI variants, which need the registers) and
// <= 8 KiB of LDS for KITTI / EuRoC cells: detect is bound by how many
// cells are in flight per CU (16 -> 10 resident waves costs +32 %, tools/microbench.py variant 8).
template <int V, int RP, int NS, int CPW, bool ST = false>
__global__ __launch_bounds__(64, (RP == 48 && NS <= 12) ? 5 : 4) void k_detect(Geo g, const CellGeo* __restrict__ cells, const uint8_t* __restrict__ in,
                                               int64_t in_pitch, const uint8_t* __restrict__ ws,
                                               int* __restrict__ cell_count, uint32_t* __restrict__ slots,
                                               int* __restrict__ stats) {
    constexpr int S = RP / 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // ROI (max_rh rows x RP u16); after the M stage the same bytes stage the minTh survivors (u32 records)
    uint16_t* roi = (uint16_t*)lds;
    // u8 M map, (max_wh + 2) rows of MP = RP bytes: px (x, y) at (y + 1) * MP + x + 2, i.e. at the pair's queue
    // entry + MP
    constexpr int MP = RP;
    uint8_t* mm = (uint8_t*)(roi + detect_roi_elems(g, RP));
    // pair queue: entry = y * RP + x + 2 (x even; fd_pq entries), the ROI u16 index of the dword that holds
    // the top-left corner of the pair's circles (ROI row y = window row y - 3, pair at ROI index
    // entry + 3 RP + 2), so the M stage's ROI reads are the entry plus non-negative immediate offsets and its map
    // address the entry plus MP; the M stage compacts the queue in place into the NMS queue
    uint16_t* pq = (uint16_t*)(mm + MP * (g.max_wh + 2));
    int bx, img;
    xcd_block(bx, img);  // neighbouring cells' ROIs overlap by 6 rows / columns: keep them in one L2
    const int lane = threadIdx.x;
    const int c_first = bx * CPW, c_last = min(c_first + CPW, g.ncells);
    // ROI staging, 8 lanes per row (dwords 2d, 2d + 1), 8 rows per step (NS / 2 steps): lane d loads two
    // dwords of the row from the 4-byte aligned start of column -1 and takes dword 2d + 2 from its
    // neighbour lane (DPP row_shl:1) to re-align 8 bytes with v_alignbyte (rows are <= 59 px, so 16
    // dwords cover every row; what lane 7 receives from the next row's lane only lands in columns >= 60).
    // The loads of the next cell are issued before this cell's compute (prefetch into NS registers).
    constexpr int NS2 = NS / 2;
    const int d = lane & 7, r0 = lane >> 3;
    uint2 raw[NS2];
    // Every slot loads unconditionally, through a resource bounded to the level (a row past it reads 0): rows
    // past the ROI and dwords past its width land only in LDS the commit below never writes or in columns
    // past the ROI, and the per-slot range tests, zero fills and branches are gone (one v_add per slot)
    auto issue = [&](int c) {
        const CellGeo cg = load_cell(cells, c);
        int stride;
        const uint8_t* lvl = level_ptr(g, cg.level, in, in_pitch, ws, img, &stride);
        const __amdgpu_buffer_rsrc_t rs = bounded_rsrc(lvl, (uint32_t)(stride * g.lv[cg.level].h));
        const uint32_t lvl_lo = (uint32_t)(uintptr_t)lvl;
        const uint32_t off0 = (uint32_t)((cg.y0 + r0) * stride + cg.x0 - 1);
        // rows r0 + 8 k share the alignment of row r0 (8 k * stride is a multiple of 4)
        const uint32_t al0 = off0 - ((lvl_lo + off0) & 3u) + 8u * d;
#pragma unroll
        for (int k = 0; k < NS2; ++k)
            raw[k] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, al0 + (uint32_t)(8 * k * stride), 0, 0));
    };
    if (c_first < c_last) issue(c_first);
    for (int c = c_first; c < c_last; ++c) {
        const CellGeo cg = load_cell(cells, c);
        const int rw = cg.x1 - cg.x0, rh = cg.y1 - cg.y0;
        const int ww = rw - 6, wh = rh - 6;  // detection window = ROI rows/cols 3 .. n-4
        {
            int stride;
            const uint8_t* lvl = level_ptr(g, cg.level, in, in_pitch, ws, img, &stride);
            const uint32_t lvl_lo = (uint32_t)(uintptr_t)lvl;
            const uint32_t off0 = (uint32_t)((cg.y0 + r0) * stride + cg.x0 - 1);
            const int n8 = (rw + 8) >> 3;  // 8-column groups of columns -1 .. rw-1 (8 * n8 <= RP)
#pragma unroll
            for (int k = 0; k < NS2; ++k) {
                // every lane takes part in the DPP (uniform control flow); lanes 15 of a DPP row get 0 (bound_ctrl:
                // the same 0 as an `old` operand, without the v_mov that would materialise it)
                const uint32_t nb = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)raw[k].x, 0x101, 0xF, 0xF, true);
                const int r = r0 + 8 * k;
                if (r < rh && d < n8) {
                    const int sh = (int)((lvl_lo + off0 + (uint32_t)(8 * k * stride)) & 3u);
                    const uint32_t w0 = __builtin_amdgcn_alignbyte(raw[k].y, raw[k].x, sh);
                    const uint32_t w1 = __builtin_amdgcn_alignbyte(nb, raw[k].y, sh);
                    uint4 u;
                    u.x = __builtin_amdgcn_perm(0x3C3C3C3Cu, w0, 0x04010400u);
                    u.y = __builtin_amdgcn_perm(0x3C3C3C3Cu, w0, 0x04030402u);
                    u.z = __builtin_amdgcn_perm(0x3C3C3C3Cu, w1, 0x04010400u);
                    u.w = __builtin_amdgcn_perm(0x3C3C3C3Cu, w1, 0x04030402u);
                    *(uint4*)(roi + r * RP + 8 * d) = u;
                }
            }
            // the M map with its zero border
            uint4* m128 = (uint4*)mm;
            for (int i = lane; i < (MP / 16) * (wh + 2); i += 64) m128[i] = uint4{0u, 0u, 0u, 0u};
        }
        if (c + 1 < c_last) issue(c + 1);  // in flight during this cell's compute
        __syncthreads();
        auto process = [&]() {
            if (V == 1) {  // ablation: ROI staging only
                if (lane == 0) cell_count[(int64_t)img * g.ncells + c] = roi[rw * rh / 2] & 0;
                return;
            }
            if (ww <= 0 || wh <= 0) {
                if (lane == 0) cell_count[(int64_t)img * g.ncells + c] = 0;
                return;
            }
        const int tq = min(g.ini_th, g.min_th);
        // ---- 2. pre-test, two adjacent pairs (pixels x .. x + 3) per lane and step, quads in row-major
        //         order (lane -> quad i0 + lane); the pair queue stays row-major (two ballots per step)
        const int qrow = (ww + 3) >> 2, nquad = qrow * wh;
        // n / qrow for n <= 64 without an integer division: (n + 0.5) / qrow is >= 0.5 / qrow >= 1/28 away
        // from an integer, far more than the reciprocal's error
        const float rq = __builtin_amdgcn_rcpf((float)qrow);
        auto div_q = [&](int n) { return (int)__builtin_fmaf((float)n, rq, 0.5f * rq); };
        const int step_y = div_q(64), step_x = 64 - step_y * qrow;
        // Two queues when minTh < iniTh (ORBextractor.cpp:795-815: FAST at iniTh, then minTh only for a
        // cell where iniTh found nothing): B = pairs whose bound exceeds minTh (from the front of pq), and
        // its subset A = bound above iniTh (from the back, growing down).  Exact M, NMS and output run on A
        // first; B is processed only for a cell that A leaves empty.  A pixel outside every A pair has
        // M <= bound <= iniTh, so it can neither be an iniTh corner nor beat one in the NMS: the iniTh pass
        // needs M of the A pairs only.  Should the two queues meet (a cell where more than half of the pairs
        // pass at minTh), the cell takes the one-pass path below instead (both thresholds over B).
        const bool two = g.min_th < g.ini_th;
        const int tA = g.ini_th;
        const int cap = g.fd_pq;
        int npq = 0, npa = 0;
        {
            // two 64-quad steps per iteration: both steps' ROI reads are issued before either waits
            // (one LDS round trip per 128 quads); lanes past the window read a clamped row and vote 0
            int qy = div_q(lane), qx = lane - qy * qrow;
            auto advance = [&](int& y, int& x) {
                y += step_y;
                x += step_x;
                if (x >= qrow) {
                    x -= qrow;
                    ++y;
                }
            };
            // the pass conditions as lane masks (v_cmp straight into SGPR pairs, combined on the SALU): a
            // bool per lane would cost a v_cndmask + v_cmp round trip per ballot.  Only the last quad of a
            // row can hold pixels past the window (x4 == xl); rem = ww - xl of its 4 are inside.
            const int xl = 4 * (qrow - 1), rem = ww - xl;
            auto gt = [](int a, int b) { return (uint64_t)__builtin_amdgcn_sicmp(a, b, 38); };  // ICMP_SGT
            auto bound_at = [&](const uint32_t* R, uint64_t in, uint64_t last, uint64_t& ca, uint64_t& cb, uint64_t& aa,
                                uint64_t& ab) {
                fd_s2 ba, bb;
                fast_bound_quad<S>(R, ba, bb);
                const uint64_t va = rem > 1 ? ~0ull : ~last, vb2 = rem > 2 ? ~0ull : ~last,
                               vb3 = rem > 3 ? ~0ull : ~last;
                ca = in & (gt(ba.x, tq) | (gt(ba.y, tq) & va));
                cb = in & vb2 & (gt(bb.x, tq) | (gt(bb.y, tq) & vb3));
                aa = ca & (gt(ba.x, tA) | (gt(ba.y, tA) & va));
                ab = cb & (gt(bb.x, tA) | (gt(bb.y, tA) & vb3));
            };
            auto bound = [&](int i, int y, int x4, uint64_t& ca, uint64_t& cb, uint64_t& aa, uint64_t& ab) {
                bound_at((const uint32_t*)(roi + (min(y, wh - 1) + 3) * RP + x4 + 4),
                         __builtin_amdgcn_sicmp(i, nquad, 40), __builtin_amdgcn_sicmp(x4, xl, 32), ca, cb, aa, ab);
            };
            // entries in lane order, a lane's first before its second: the lane's first goes after every entry
            // of the lanes below it (one mbcnt chain over both masks, seeded with the queue length), its second
            // one further when it has a first
            auto below2 = [](uint64_t m0, uint64_t m1, int base) {
                return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1,
                       __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, base))));
            };
            auto emit = [&](int n, uint64_t b0, uint64_t b1, uint64_t a0, uint64_t a1) {
                const bool ca = __builtin_amdgcn_inverse_ballot_w64(b0), cb = __builtin_amdgcn_inverse_ballot_w64(b1);
                const uint16_t e = (uint16_t)n;
                const int o = below2(b0, b1, npq);
                if (ca) pq[o] = e;
                if (cb) pq[fd_plus_bit(o, b0)] = (uint16_t)(e + 2);
                npq += __popcll(b0) + __popcll(b1);
                if (two) {
                    const bool aa = __builtin_amdgcn_inverse_ballot_w64(a0), ab = __builtin_amdgcn_inverse_ballot_w64(a1);
                    const int na = __popcll(a0) + __popcll(a1);
                    // both counts only grow: once the queues would meet they stay met (collide below), and A
                    // stops writing so that B stays intact for the one-pass path
                    if (npq + npa + na <= cap) {
                        const int oa = cap - 1 - below2(a0, a1, npa);
                        if (aa) pq[oa] = e;
                        if (ab) pq[fd_minus_bit(oa, a0)] = (uint16_t)(e + 2);
                    }
                    npa += na;
                }
            };
            if (qrow <= 8) {
                // rows of 8 lanes (every KITTI / EuRoC cell but EuRoC level 7's): lane 8 r + qx takes quad qx
                // of row y0 + r (lanes qx >= qrow idle), so the lane order is the row-major queue order and
                // the ROI address and the entry are per-lane constants plus a uniform row offset.  Lanes of
                // rows past the window read (and vote 0 on) rows below it: still inside the LDS allocation
                // (ROI rows, then the M map).
                const int r = lane >> 3, qx = lane & 7;
                const uint64_t colok = __builtin_amdgcn_sicmp(qx, qrow, 40), last = __builtin_amdgcn_sicmp(4 * qx, xl, 32);
                const uint32_t* R0 = (const uint32_t*)(roi + (r + 3) * RP + 4 * qx + 4);
                for (int y0 = 0; y0 < wh; y0 += 16) {
                    uint64_t ca0, cb0, ca1, cb1, aa0, ab0, aa1, ab1;
                    bound_at(R0 + y0 * S, colok & __builtin_amdgcn_sicmp(r, wh - y0, 40), last, ca0, cb0, aa0, ab0);
                    bound_at(R0 + (y0 + 8) * S, colok & __builtin_amdgcn_sicmp(r, wh - y0 - 8, 40), last, ca1, cb1, aa1,
                             ab1);
                    emit((y0 + r) * RP + 4 * qx + 2, ca0, cb0, aa0, ab0);
                    emit((y0 + r + 8) * RP + 4 * qx + 2, ca1, cb1, aa1, ab1);
                }
            } else {
                for (int i0 = 0; i0 < nquad; i0 += 128) {
                    int qy2 = qy, qx2 = qx;
                    advance(qy2, qx2);
                    uint64_t ca0, cb0, ca1, cb1, aa0, ab0, aa1, ab1;
                    bound(i0 + lane, qy, 4 * qx, ca0, cb0, aa0, ab0);
                    bound(i0 + 64 + lane, qy2, 4 * qx2, ca1, cb1, aa1, ab1);
                    emit(qy * RP + 4 * qx + 2, ca0, cb0, aa0, ab0);
                    emit(qy2 * RP + 4 * qx2 + 2, ca1, cb1, aa1, ab1);
                    qy = qy2;
                    qx = qx2;
                    advance(qy, qx);
                }
            }
        }
        __syncthreads();
        if (V == 2) {  // ablation: + pre-test / pair queue
            if (lane == 0) cell_count[(int64_t)img * g.ncells + c] = npq & 0;
            return;
        }
        // ---- 3. exact M of a queue's pairs -> M map; the pairs with a pixel above tl are compacted in place
        //         (entry i at qb[dir * i]: dir -1 for A at the back of pq) into the NMS queue; returns its length
        auto m_stage = [&](uint16_t* qb, int dir, int n, int tl) {
            int nn = 0;
            // the queue entry of the next step is read one step ahead (its LDS round trip overlaps this step)
            uint32_t e_next = lane < n ? qb[dir * lane] : 2u;  // idle lanes: pixel (0, 0)
            for (int k0 = 0; k0 < n; k0 += 64) {
                // every lane computes (a lane past n repeats an earlier entry of its own, harmlessly); the map
                // store and the compaction take the lanes of this step's entries (lane masks, as the pre-test)
                const uint32_t e = e_next;
                if (k0 + 64 + lane < n) e_next = qb[dir * (k0 + 64 + lane)];
                const uint64_t inr = __builtin_amdgcn_sicmp(k0 + lane, n, 40);  // ICMP_SLT
                const uint32_t m = fast_m_pair<S>((const uint32_t*)(roi + e) + 3 * S + 1);
                // the u8 map keeps M itself (low byte of each biased half); odd width: the last pair's second
                // pixel lies outside the window, its map entry is cleared after this stage
                if (__builtin_amdgcn_inverse_ballot_w64(inr))
                    *(uint16_t*)(mm + e + MP) = (uint16_t)__builtin_amdgcn_perm(0u, m, 0x0c0c0200u);
                // slots below k0 + 64 are written; every read of the queue (this step's entries, the next
                // step's prefetch) was issued before
                const uint64_t bh = inr & ((uint64_t)__builtin_amdgcn_sicmp((int)(m & 0x3FFu), tl, 38) |
                                           (uint64_t)__builtin_amdgcn_sicmp((int)((m >> 16) & 0x3FFu), tl, 38));
                if (__builtin_amdgcn_inverse_ballot_w64(bh)) qb[dir * (nn + lanes_below(bh))] = (uint16_t)e;
                nn += __popcll(bh);
            }
            // odd width: column ww (right of the window) got the outside pixel's M from the last pairs; NMS
            // reads it as a neighbour (and as that pixel's own score) and needs 0 there
            if ((ww & 1) && lane < wh) mm[(lane + 1) * MP + ww + 2] = 0;
            __syncthreads();
            return nn;
        };
        // ---- 4. NMS (local max) over an NMS queue + ordered compaction.  For t >= 1, "score > every
        //         8-neighbour's score at t" is M > t and M > max(neighbour M) (a neighbour with M <= t is
        //         below anyway).  Kept pixels: pairs row-major, pixel x before x + 1 = cv::FAST's order.
        //         thb1 >= 1: also test the second threshold and stage its survivors in `alt` (one-pass path).
        uint32_t* out = slots + (int64_t)img * g.slot_total + cg.slot_off;
        uint32_t* alt = (uint32_t*)roi;  // >= 2 * slot_cap u16 (detect_roi_elems)
        auto nms_stage = [&](const uint16_t* qb, int dir, int nn, int thb0, int thb1, int& t0, int& t1) {
            t0 = t1 = 0;
            for (int k0 = 0; k0 < nn; k0 += 64) {
                // every lane computes on an entry in range; lane masks select the kept pixels
                const uint64_t inr = __builtin_amdgcn_sicmp(k0 + lane, nn, 40);  // ICMP_SLT
                const int e = qb[dir * min(k0 + lane, nn - 1)];
                const uint8_t* q = mm + e + MP;  // pixel A = (x, y); B = (x + 1, y)
                const int t_0 = q[-MP - 1], t_1 = q[-MP], t_2 = q[-MP + 1], t_3 = q[-MP + 2];
                const int m_0 = q[-1], owna = q[0], ownb = q[1], m_3 = q[2];
                const int b_0 = q[MP - 1], b_1 = q[MP], b_2 = q[MP + 1], b_3 = q[MP + 2];
                const int c1 = max(t_1, b_1), c2 = max(t_2, b_2);  // the pair's columns without its own row
                const int na = max(imax3(t_0, m_0, b_0), imax3(c1, c2, ownb));
                const int nb = max(imax3(t_3, m_3, b_3), imax3(c1, c2, owna));
                // (x + 3, y + 3) = (e % RP + 1, e / RP + 3)
                const uint32_t xy = (uint32_t)(cg.x0 + (int)((uint32_t)e % RP) + 1) +
                                    __umul24((uint32_t)(cg.y0 + (int)((uint32_t)e / RP) + 3), (uint32_t)cg.kw);
                const uint32_t reca = xy | ((uint32_t)(owna - 1) << 24);
                const uint32_t recb = (xy + 1u) | ((uint32_t)(ownb - 1) << 24);
                auto keep = [&](int th, uint64_t& ba, uint64_t& bb, int& t, uint32_t* dst) {
                    ba = inr & (uint64_t)__builtin_amdgcn_sicmp(owna, max(na, th), 38);
                    bb = inr & (uint64_t)__builtin_amdgcn_sicmp(ownb, max(nb, th), 38);
                    const bool ka = __builtin_amdgcn_inverse_ballot_w64(ba), kb = __builtin_amdgcn_inverse_ballot_w64(bb);
                    const int o = t + lanes_below(ba) + lanes_below(bb);
                    // slot_cap holds by the strict NMS (no two kept pixels are 8-neighbours); never write past it
                    if (ka && o < cg.slot_cap) dst[o] = reca;
                    if (kb) {
                        const int ob = fd_plus_bit(o, ba);
                        if (ob < cg.slot_cap) dst[ob] = recb;
                    }
                    t += __popcll(ba) + __popcll(bb);
                };
                uint64_t ba, bb;
                keep(thb0, ba, bb, t0, out);
                if (thb1 > 0) keep(thb1, ba, bb, t1, alt);
            }
        };
        const bool collide = npq + npa > cap;
        // orbfe_debug_detect_stats: cells that took the one-pass path despite two thresholds (the queues met)
        if (ST && lane == 0 && two && collide) atomicAdd(&stats[1], 1);
        int total = 0;
        if (two && !collide) {
            int t0, t1;
            const int nna = m_stage(pq + cap - 1, -1, npa, max(tA, 1));
            if (V == 3) {  // ablation: + exact M
                if (lane == 0) cell_count[(int64_t)img * g.ncells + c] = nna & 0;
                return;
            }
            nms_stage(pq + cap - 1, -1, nna, max(g.ini_th, 1), 0, t0, t1);
            total = t0;
            if (t0 == 0) {  // minTh fallback: every pair of B (the A pairs' M is recomputed, identically)
                if (ST && lane == 0) atomicAdd(&stats[2], 1);
                const int nnb = m_stage(pq, 1, npq, max(g.min_th, 1));
                nms_stage(pq, 1, nnb, max(g.min_th, 1), 0, t0, t1);
                total = t0;
            }
        } else {
            // one pass over B at tq = min(iniTh, minTh), both thresholds in the NMS: iniTh survivors go
            // straight out, minTh survivors are staged in the (dead) ROI area and copied out only if iniTh
            // kept nothing
            const int nnq = m_stage(pq, 1, npq, max(tq, 1));
            if (V == 3) {  // ablation: + exact M
                if (lane == 0) cell_count[(int64_t)img * g.ncells + c] = nnq & 0;
                return;
            }
            const bool fb = g.min_th != g.ini_th;
            int t0, t1;
            nms_stage(pq, 1, nnq, max(g.ini_th, 1), fb ? max(g.min_th, 1) : 0, t0, t1);
            total = t0;
            if (t0 == 0 && t1 > 0) {
                __syncthreads();
                for (int i = lane; i < min(t1, cg.slot_cap); i += 64) out[i] = alt[i];
                total = t1;
            }
        }
        if (lane == 0) cell_count[(int64_t)img * g.ncells + c] = min(total, cg.slot_cap);
        if (ST && lane == 0) atomicAdd(&stats[0], 1);
        };
        process();
        __syncthreads();  // the next cell overwrites the ROI and the M map
    }
}

// ------------------------------------------------------------------------------- k_octree
// DistributeOctTree as a sequence of data-parallel passes.  The std::list of the reference is held as
// an array ordered by list position; push_front / erase become "children of this pass at the front in
// reverse creation order, surviving nodes after them in their old order".  Every candidate key keeps
// the list position of its node (kn[]), re-mapped after each pass.  Equal-size ties in the careful
// phase resolve by node creation order (see oracle/orb_oracle.cpp).
//
// LDS layout (dynamic, NC = Geo::max_ncap node slots):
//   box[2][NC] u64 (x0,y0,x1,y1 int16) | cnt[2][NC] i32 | cnt4[4NC] i32 | cpos[4NC] u16 |
//   sa[NC] sb[NC] sd[NC] proc[NC] i32 | srt[pow2(NC)] u64 | coff[maxcell+1] i32 |
//   kd[g.oct_keys] u32 | kn[g.oct_keys] u16   (the candidates, when the level has at most g.oct_keys; else they
//   stay in the global kd/kn arrays)
constexpr int kOctThreads = 512;   // 8 waves: the per-pass candidate loops are latency chains
constexpr int kOctGather = 16;     // candidate slot loads in flight per thread in the gather
struct OctLds {
    uint64_t *box0, *box1;
    int *cnt0, *cnt1;
    int* cnt4;
    uint16_t* cpos;
    int *sa, *sb, *sd, *proc;
    uint64_t* srt;
    int* coff;
    uint32_t* kd;
    uint16_t* kn;
};

__device__ __forceinline__ int quad_of(uint32_t key, uint64_t box, KeyDiv kv) {
    int x, y;
    key_xy(key, kv, x, y);
    x -= kBorder;
    y -= kBorder;
    const int x0 = (int16_t)(box & 0xFFFF), y0 = (int16_t)((box >> 16) & 0xFFFF);
    const int x1 = (int16_t)((box >> 32) & 0xFFFF), y1 = (int16_t)((box >> 48) & 0xFFFF);
    const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);  // ceil((float)d/2), d >= 0
    return (x < mx ? 0 : 1) + (y < my ? 0 : 2);
}

// Child-quadrant counts of one octree pass: bins 4 p + quadrant of every candidate k whose node p is
// divided (div(p)).  Thread t takes the contiguous candidates [t * per, (t + 1) * per), two per step with
// their LDS loads in flight together, and adds a run length to the LDS counter whenever the bin changes.
template <typename Div>
__device__ __forceinline__ void octree_count_runs(int K, int t, const uint16_t* kn, const uint32_t* kd, Div div,
                                                  const uint64_t* box, int* bins, KeyDiv kv) {
    const int per = (K + kOctThreads - 1) / kOctThreads;
    const int kb = min(t * per, K), ke = min(kb + per, K);
    int cur = -1, run = 0;
    auto add = [&](int p, uint32_t key) {
        if (!div(p)) return;
        const int b = 4 * p + quad_of(key, box[p], kv);
        if (b != cur) {
            if (run) atomicAdd(&bins[cur], run);
            cur = b;
            run = 0;
        }
        ++run;
    };
    int k = kb;
    for (; k + 1 < ke; k += 2) {
        const int p0 = kn[k], p1 = kn[k + 1];
        const uint32_t k0 = kd[k], k1 = kd[k + 1];
        add(p0, k0);
        add(p1, k1);
    }
    if (k < ke) add(kn[k], kd[k]);
    if (run) atomicAdd(&bins[cur], run);
}

__device__ __forceinline__ uint64_t pack_box(int x0, int y0, int x1, int y1) {
    return (uint64_t)(uint16_t)x0 | ((uint64_t)(uint16_t)y0 << 16) | ((uint64_t)(uint16_t)x1 << 32) |
           ((uint64_t)(uint16_t)y1 << 48);
}

// ExtractorNode::DivideNode child boxes (ORBextractor.cpp:483-509), q = 0..3 -> n1..n4
__device__ __forceinline__ uint64_t child_box(uint64_t box, int q) {
    const int x0 = (int16_t)(box & 0xFFFF), y0 = (int16_t)((box >> 16) & 0xFFFF);
    const int x1 = (int16_t)((box >> 32) & 0xFFFF), y1 = (int16_t)((box >> 48) & 0xFFFF);
    const int mx = x0 + ((x1 - x0 + 1) >> 1), my = y0 + ((y1 - y0 + 1) >> 1);
    switch (q) {
        case 0: return pack_box(x0, y0, mx, my);
        case 1: return pack_box(mx, y0, x1, my);
        case 2: return pack_box(x0, my, mx, y1);
        default: return pack_box(mx, my, x1, y1);
    }
}

__global__ __launch_bounds__(kOctThreads) void k_octree(Geo g, const CellGeo* __restrict__ cells,
                                                const int* __restrict__ cell_count, const uint32_t* __restrict__ slots,
                                                uint32_t* __restrict__ kd_all, uint16_t* __restrict__ kn_all,
                                                uint32_t* __restrict__ lvl_kp, int* __restrict__ lvl_count,
                                                int* __restrict__ overflow, int maxcell, int stop,
                                                long long* __restrict__ prof) {
    // stop (tools/microbench.py ablations): 1 after the candidate gather, 2 after the initial columns,
    // 3 after the full-division phase, 16 + l only level l, 64 + 8 l + n only level l and stop before
    // pass n; 0 = the whole algorithm
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ int scan_tmp[257];
    __shared__ int s_S, s_C, s_phase, s_cur, s_nexp, s_P, s_done;
    // grid (image, level): level-major dispatch, the long level-0 workgroups start first
    const int img = blockIdx.x, l = blockIdx.y, t = threadIdx.x;
    if (stop >= 16 && stop < 64 && l != stop - 16) return;
    if (stop >= 64 && l != (stop - 64) / 8) return;
    // prof (orbfe_debug_octree_profile): 64 wall-clock marks (100 MHz) per (image, level)
    long long* pm = prof ? prof + ((int64_t)img * g.nlevels + l) * 64 : nullptr;
    auto mark = [&](int id) {
        if (pm && t == 0 && id < 64) pm[id] = (long long)wall_clock64();
    };
    mark(0);
    const LevelGeo& L = g.lv[l];
    const KeyDiv kv = key_div(L);
    const int NC = g.max_ncap;
    int pow2 = 1;
    while (pow2 < NC) pow2 <<= 1;
    OctLds d;
    {
        unsigned char* p = lds;
        d.box0 = (uint64_t*)p; p += 8 * NC;
        d.box1 = (uint64_t*)p; p += 8 * NC;
        d.srt = (uint64_t*)p; p += 8 * pow2;
        d.cnt0 = (int*)p; p += 4 * NC;
        d.cnt1 = (int*)p; p += 4 * NC;
        d.cnt4 = (int*)p; p += 16 * NC;
        d.cpos = (uint16_t*)p; p += 8 * NC;
        d.sa = (int*)p; p += 4 * NC;
        d.sb = (int*)p; p += 4 * NC;
        d.sd = (int*)p; p += 4 * NC;
        d.proc = (int*)p; p += 4 * NC;
        d.coff = (int*)p; p += 4 * ((maxcell + 4) & ~3);
        d.kd = (uint32_t*)p; p += 4 * g.oct_keys;
        d.kn = (uint16_t*)p;
    }
    const int N = L.n_feat;
    const int ncell = L.ncell;
    uint32_t* kd_g = kd_all + (int64_t)img * g.key_total + L.key_off;
    uint16_t* kn_g = kn_all + (int64_t)img * g.key_total + L.key_off;
    uint32_t* out = lvl_kp + (int64_t)img * g.lvl_kp_cap + L.kp_off;

    // 1. gather the level's candidates in cell order (= vToDistributeKeys order).  Each cell's slot
    //    offset goes to LDS (cnt4 is free until pass 2) next to its count, so a key finds its slot with
    //    LDS reads only and one global load
    const bool soff_lds = ncell <= 4 * NC;
    for (int i = t; i < ncell; i += kOctThreads) {  // both loads in flight before either store
        const int n = cell_count[(int64_t)img * g.ncells + L.cell0 + i];
        const int so = soff_lds ? cells[L.cell0 + i].slot_off : 0;
        d.coff[i] = n;
        if (soff_lds) d.cnt4[i] = so;
    }
    __syncthreads();
    const int K = block_excl_scan(d.coff, ncell, scan_tmp);
    if (t == 0) d.coff[ncell] = K;
    __syncthreads();
    // the pass loops below read every candidate several times per pass: keep them in LDS when they fit
    auto run = [&](auto in_lds) {
        uint32_t* kd;
        uint16_t* kn;
        if constexpr (decltype(in_lds)::value) {
            kd = d.kd;
            kn = d.kn;
        } else {
            kd = kd_g;
            kn = kn_g;
        }
        const uint32_t* islots = slots + (int64_t)img * g.slot_total;
        if (soff_lds) {
            // key -> cell map in kn (rewritten by pass 2), one thread per cell
            for (int i = t; i < ncell; i += kOctThreads)
                for (int k = d.coff[i]; k < d.coff[i + 1]; ++k) kn[k] = (uint16_t)i;
            __syncthreads();
            // kOctGather keys per thread and step (coalesced across threads): a level's slot loads are one
            // round trip, not one per 4 keys
            for (int k0 = t; k0 < K; k0 += kOctGather * kOctThreads) {
                uint32_t v[kOctGather];
#pragma unroll
                for (int u = 0; u < kOctGather; ++u) {
                    const int k = k0 + u * kOctThreads;
                    v[u] = 0;
                    if (k < K) {
                        const int c = kn[k];
                        v[u] = islots[d.cnt4[c] + (k - d.coff[c])];
                    }
                }
#pragma unroll
                for (int u = 0; u < kOctGather; ++u)
                    if (k0 + u * kOctThreads < K) kd[k0 + u * kOctThreads] = v[u];
            }
            __syncthreads();  // pass 2 clears cnt4 (the slot offsets) and rewrites kn
        } else {
            for (int k0 = t; k0 < K; k0 += 4 * kOctThreads) {
                uint32_t v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int k = k0 + u * kOctThreads;
                    v[u] = 0;
                    if (k < K) {
                        int lo = 0, hi = ncell - 1;  // last cell with coff <= k
                        while (lo < hi) {
                            const int mid = (lo + hi + 1) >> 1;
                            if (d.coff[mid] <= k) lo = mid; else hi = mid - 1;
                        }
                        v[u] = islots[cells[L.cell0 + lo].slot_off + (k - d.coff[lo])];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (k0 + u * kOctThreads < K) kd[k0 + u * kOctThreads] = v[u];
            }
        }
        mark(1);
        if (stop == 1) return;
        // 2. initial columns (:543-584); a key goes to column (size_t)(x / hX)
        const int nIni = L.n_ini;
        for (int i = t; i < 4 * NC; i += kOctThreads) d.cnt4[i] = 0;
        __syncthreads();
        {  // contiguous candidate runs per thread, one LDS atomic per change of column (octree_count_runs)
            const int per = (K + kOctThreads - 1) / kOctThreads;
            const int kb = min(t * per, K), ke = min(kb + per, K);
            int cur = -1, run = 0;
            for (int k = kb; k < ke; ++k) {
                int x, y;
                key_xy(kd[k], kv, x, y);
                x -= kBorder;
                const int col = min((int)((float)x / L.hx), nIni - 1);
                kn[k] = (uint16_t)col;
                if (col != cur) {
                    if (run) atomicAdd(&d.cnt4[cur], run);
                    cur = col;
                    run = 0;
                }
                ++run;
            }
            if (run) atomicAdd(&d.cnt4[cur], run);
        }
        __syncthreads();
        if (t == 0) {
            int S = 0;
            for (int i = 0; i < nIni; ++i) {
                const int n = d.cnt4[i];
                d.cpos[i] = S;
                if (n > 0) {
                    d.box0[S] = pack_box((int)(L.hx * (float)i), 0, (int)(L.hx * (float)(i + 1)), L.span_y);
                    d.cnt0[S] = n;
                    ++S;
                }
            }
            s_S = S;
            s_C = 0;
            s_cur = 0;
            s_phase = 0;
            s_done = (S == 0);
            s_nexp = 0;
            if (S > NC) { s_done = 1; atomicOr(overflow, 1); }
        }
        __syncthreads();
        for (int k = t; k < K; k += kOctThreads) kn[k] = (uint16_t)d.cpos[kn[k]];
        __syncthreads();
        mark(2);
        if (stop == 2) return;

        for (int iter = 0; !s_done; ++iter) {
            const int S = s_S, C = s_C, cur = s_cur, nxt = cur ^ 1;
            const uint64_t* box = cur ? d.box1 : d.box0;
            const int* cnt = cur ? d.cnt1 : d.cnt0;
            uint64_t* nbox = cur ? d.box0 : d.box1;
            int* ncnt = cur ? d.cnt0 : d.cnt1;
            if (iter > 4 * NC + 64) {  // cannot happen (each step grows the list or finishes); never hang
                if (t == 0) { atomicOr(overflow, 2); s_done = 1; }
                __syncthreads();
                break;
            }
            if (stop == 3 && s_phase != 0) return;
            if (stop >= 64 && iter == (stop - 64) % 8) return;
            mark(8 + 4 * iter);
            if (s_phase == 0) {
                // ---------------- full pass (:605-664): divide every node holding more than one key
                for (int i = t; i < 4 * S; i += kOctThreads) d.cnt4[i] = 0;
                if (t == 0) s_nexp = 0;
                __syncthreads();
                // each thread counts a contiguous run of candidates: consecutive candidates (cell order)
                // mostly fall into the same child, so a thread adds one run length per change of bin instead
                // of one LDS atomic per candidate on a handful of hot counters
                octree_count_runs(K, t, kn, kd, [&](int p) { return cnt[p] > 1; }, box, d.cnt4, kv);
                __syncthreads();
                mark(9 + 4 * iter);
                for (int p = t; p < S; p += kOctThreads) {
                    int nc = 0;
                    if (cnt[p] > 1)
                        for (int q = 0; q < 4; ++q) nc += d.cnt4[4 * p + q] > 0;
                    d.sa[p] = nc;
                    d.sb[p] = cnt[p] == 1;
                }
                __syncthreads();
                const int Cn = block_excl_scan(d.sa, S, scan_tmp);
                const int Kk = block_excl_scan(d.sb, S, scan_tmp);
                mark(10 + 4 * iter);
                int nexp = 0;
                bool ovf = false;
                for (int p = t; p < S; p += kOctThreads) {
                    if (cnt[p] > 1) {
                        int c = d.sa[p];
                        for (int q = 0; q < 4; ++q) {
                            const int n = d.cnt4[4 * p + q];
                            if (n == 0) continue;
                            const int np = Cn - 1 - c++;
                            if (np < NC) {
                                nbox[np] = child_box(box[p], q);
                                ncnt[np] = n;
                            } else {
                                ovf = true;
                            }
                            d.cpos[4 * p + q] = np;
                            nexp += n > 1;
                        }
                    } else {
                        const int np = Cn + d.sb[p];
                        if (np < NC) {
                            nbox[np] = box[p];
                            ncnt[np] = cnt[p];
                        } else {
                            ovf = true;
                        }
                        d.cpos[4 * p] = np;
                    }
                }
                if (nexp) atomicAdd(&s_nexp, nexp);
                if (ovf) atomicOr(overflow, 4);
                __syncthreads();
                for (int k0 = t; k0 < K; k0 += 4 * kOctThreads) {
                    int np[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int k = k0 + u * kOctThreads;
                        if (k < K) {
                            const int p = kn[k];
                            np[u] = cnt[p] > 1 ? d.cpos[4 * p + quad_of(kd[k], box[p], kv)] : d.cpos[4 * p];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (k0 + u * kOctThreads < K) kn[k0 + u * kOctThreads] = (uint16_t)np[u];
                }
                __syncthreads();
                if (t == 0) {
                    const int Sn = Cn + Kk;
                    s_S = Sn;
                    s_C = Cn;
                    s_cur = nxt;
                    if (Sn > NC) s_done = 1;
                    else if (Sn >= N || Sn == S) s_done = 1;            // :668-671
                    else if (Sn + 3 * s_nexp > N) s_phase = 1;          // :672
                }
                __syncthreads();
            } else {
                // ---------------- careful phase (:675-736): divide the largest nodes of the last step first
                for (int i = t; i < 4 * C; i += kOctThreads) d.cnt4[i] = 0;
                for (int p = t; p < S; p += kOctThreads) d.proc[p] = 0;
                if (t == 0) s_P = 0x7fffffff;
                __syncthreads();
                octree_count_runs(K, t, kn, kd, [&](int p) { return p < C && cnt[p] > 1; }, box, d.cnt4, kv);
                for (int p = t; p < C; p += kOctThreads) d.sa[p] = cnt[p] > 1;
                __syncthreads();
                const int M = block_excl_scan(d.sa, C, scan_tmp);
                for (int p = t; p < C; p += kOctThreads)
                    if (cnt[p] > 1)  // size desc, then creation desc (= list position asc)
                        d.srt[d.sa[p]] = ((uint64_t)(uint32_t)cnt[p] << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)p);
                __syncthreads();
                // rank sort, descending (size, then creation desc = position asc); the keys are unique, so
                // rank = number of greater keys; ranks go through d.sd, then srt is rewritten as rank -> p
                for (int i = t; i < M; i += kOctThreads) {
                    const uint64_t v = d.srt[i];
                    int r = 0;
#pragma unroll 8
                    for (int j = 0; j < M; ++j) r += d.srt[j] > v;
                    d.sd[i] = r;
                }
                __syncthreads();
                int* sp = (int*)d.srt;  // aliases srt[0 .. M/2): every srt read is behind the barriers
                for (int i = t; i < M; i += kOctThreads) d.sb[i] = (int)(0xFFFFFFFFu - (uint32_t)(d.srt[i] & 0xFFFFFFFFu));
                __syncthreads();
                for (int i = t; i < M; i += kOctThreads) sp[d.sd[i]] = d.sb[i];
                __syncthreads();
                // sorted candidate j -> position p, children count, running list size
                for (int j = t; j < M; j += kOctThreads) {
                    const int p = sp[j];
                    int nc = 0;
                    for (int q = 0; q < 4; ++q) nc += d.cnt4[4 * p + q] > 0;
                    d.sb[j] = nc - 1;
                    d.sd[j] = nc;
                }
                __syncthreads();
                block_excl_scan(d.sb, M, scan_tmp);
                for (int j = t; j < M; j += kOctThreads)
                    if (S + d.sb[j] + d.sd[j] - 1 >= N) atomicMin(&s_P, j);  // :729-730 break
                __syncthreads();
                mark(9 + 4 * iter);
                const int P = s_P == 0x7fffffff ? M : s_P + 1;
                for (int j = t; j < M; j += kOctThreads) {
                    if (j >= P) d.sd[j] = 0;
                    else {
                        const int p = sp[j];
                        d.proc[p] = 1;
                    }
                }
                __syncthreads();
                const int Cn = block_excl_scan(d.sd, M, scan_tmp);
                for (int p = t; p < S; p += kOctThreads) d.sa[p] = d.proc[p] == 0;
                __syncthreads();
                const int Kk = block_excl_scan(d.sa, S, scan_tmp);
                mark(10 + 4 * iter);
                bool ovf = false;
                for (int j = t; j < P; j += kOctThreads) {
                    const int p = sp[j];
                    int c = d.sd[j];
                    for (int q = 0; q < 4; ++q) {
                        const int n = d.cnt4[4 * p + q];
                        if (n == 0) continue;
                        const int np = Cn - 1 - c++;
                        if (np < NC) {
                            nbox[np] = child_box(box[p], q);
                            ncnt[np] = n;
                        } else {
                            ovf = true;
                        }
                        d.cpos[4 * p + q] = np;
                    }
                }
                for (int p = t; p < S; p += kOctThreads) {
                    if (d.proc[p]) continue;
                    const int np = Cn + d.sa[p];
                    if (np < NC) {
                        nbox[np] = box[p];
                        ncnt[np] = cnt[p];
                    } else {
                        ovf = true;
                    }
                    d.cpos[4 * p] = np;
                }
                if (ovf) atomicOr(overflow, 8);
                __syncthreads();
                for (int k0 = t; k0 < K; k0 += 4 * kOctThreads) {
                    int np[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int k = k0 + u * kOctThreads;
                        if (k < K) {
                            const int p = kn[k];
                            np[u] = d.proc[p] ? d.cpos[4 * p + quad_of(kd[k], box[p], kv)] : d.cpos[4 * p];
                        }
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u)
                        if (k0 + u * kOctThreads < K) kn[k0 + u * kOctThreads] = (uint16_t)np[u];
                }
                __syncthreads();
                if (t == 0) {
                    const int Sn = Cn + Kk;
                    s_S = Sn;
                    s_C = Cn;
                    s_cur = nxt;
                    if (Sn > NC || Sn >= N || Sn == S) s_done = 1;  // :733-734
                }
                __syncthreads();
            }
        }
        // 3. keep the first maximum-response key of every node (:740-759), list order
        const int S = min(s_S, NC);
        uint32_t* best = (uint32_t*)d.cnt4;
        for (int p = t; p < S; p += kOctThreads) best[p] = 0;
        __syncthreads();
        {  // contiguous candidate runs per thread: one LDS atomicMax per change of node
            const int per = (K + kOctThreads - 1) / kOctThreads;
            const int kb = min(t * per, K), ke = min(kb + per, K);
            int cur = -1;
            uint32_t m = 0;
            for (int k = kb; k < ke; ++k) {
                const int p = kn[k];
                const uint32_t v = (kd[k] & 0xFF000000u) | (0xFFFFFFu - (uint32_t)k);
                if (p != cur) {
                    if (cur >= 0 && cur < S) atomicMax(&best[cur], m);
                    cur = p;
                    m = 0;
                }
                m = max(m, v);
            }
            if (cur >= 0 && cur < S) atomicMax(&best[cur], m);
        }
        __syncthreads();
        for (int p = t; p < S; p += kOctThreads) {
            const uint32_t k = 0xFFFFFFu - (best[p] & 0xFFFFFFu);
            if (best[p] != 0u && (int)k < K) {
                out[p] = kd[k];
            } else {  // a node without keys cannot occur; flag instead of reading out of range
                out[p] = 0u;
                atomicOr(overflow, 16);
            }
        }
        if (t == 0) lvl_count[img * g.nlevels + l] = S;
        mark(63);
    };
    if (K <= g.oct_keys) run(std::true_type{});
    else run(std::false_type{});
}

// ------------------------------------------------------------------------------- k_octree_bins
// DistributeOctTree (ORBextractor.cpp:539-762) with the candidates counted once instead of once per pass.
// A key's quadrant at every depth is fixed by its own x / y and the level geometry (orbfe_host.hip
// octree_tables), so its whole path is a Morton code read from two tables, and a node of depth d is "the
// keys whose code starts with its d digits".  One 256-thread workgroup per (image, level):
//   1. all four waves sweep the level's candidates once (cell order = vToDistributeKeys order, each thread
//      a contiguous run): codes from the tables (staged in LDS), a histogram over the depth-D0 nodes
//      ("bins", column-major) and the code / response of every key into the per-image scratch;
//   2. wave 0 scans the histogram (the key count of ANY node of depth <= D0, and of each of its four
//      children, is then a difference of two LDS words) and runs the passes of the reference (full
//      division, then the careful largest-first phase) on the node list only, kept in list order exactly
//      as in k_octree (children of a pass in front in reverse creation order, surviving nodes after them
//      in their old order);
//   3. all waves give every key its final node (bin -> node map) and keep the first maximum response per
//      node (response << 24 | 0xFFFFFF - key index, atomicMax); the list goes out in list order.
// A division below depth D0 (the host picks D0 with ~2 N bins, at most 2 048: the synthetic batch images
// end at depth <= 4, but the clustered corners of the C3 sequence's nearby planes reach depth 8 - 10 at
// levels 0 / 1) counts that node's children with an extra sweep over the keys, which wave 0 hands to every
// wave of the workgroup; the sweeps read the keys from a key-order copy the first sweep leaves in global
// scratch.  Equal-size ties of the careful phase resolve by creation order, as in k_octree.
constexpr int kObThreads = 256;
#ifndef ORBFE_OB_BATCH
#define ORBFE_OB_BATCH 4
#endif
constexpr int kObBatch = ORBFE_OB_BATCH;    // slot loads in flight per thread in the first sweep
constexpr uint32_t kObDeep = 0x80000000u;   // bin flag: holds nodes deeper than D0 (deep sweep / final map)
// The node passes keep the list in wave 0's registers (kObNpl consecutive nodes per lane) when the level's
// node capacity fits, i.e. max_ncap <= 64 kObNpl (every KITTI / EuRoC configuration up to ~3 900 features);
// larger ones take the LDS-list passes (REG = false).
constexpr int kObNpl = 8;
__host__ __device__ inline bool octree_reg_passes(int max_ncap) { return max_ncap <= 64 * kObNpl; }

// LDS ordering inside wave 0's node passes (the other waves wait at a workgroup barrier meanwhile)
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int wave_incl_sum(int v) {
    const int l = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (l >= o) v += y;
    }
    return v;
}

// Exclusive scan of a[0..n) in LDS by one wavefront (lane l owns a contiguous chunk); returns the total.
__device__ int wave_scan_lds(int* a, int n) {
    const int t = threadIdx.x & 63;
    const int per = (n + 63) >> 6;
    const int b = min(t * per, n), e = min(b + per, n);
    int s = 0;
    for (int i = b; i < e; ++i) s += a[i];
    const int inc = wave_incl_sum(s);
    int run = inc - s;
    for (int i = b; i < e; ++i) {
        const int v = a[i];
        a[i] = run;
        run += v;
    }
    const int tot = __shfl(inc, 63, 64);
    wsync();
    return tot;
}

// DPP row_shr:S (within 16-lane rows); lanes without a source lane get `old`
template <int S>
__device__ __forceinline__ uint32_t dpp_shr(uint32_t old, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x110 + S, 0xF, 0xF, false);
}

// Wave-wide inclusive scan (sum) with DPP row shifts and row broadcasts (no LDS, no bpermute); every lane
// active.  Lane 63 holds the total.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 into rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 into rows 2, 3
    return v;
}
__device__ __forceinline__ int wave_total_dpp(int v) { return __builtin_amdgcn_readlane(wave_incl_scan_dpp(v), 63); }
// wave maximum of non-negative values, in every lane
__device__ __forceinline__ int wave_max_dpp(int v) {
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false));
    v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false));
    return __builtin_amdgcn_readlane(v, 63);
}
// Exclusive scan, in place, of a list held lane-major in registers (lane l holds elements l N .. l N + N - 1);
// returns the total.
template <int N>
__device__ __forceinline__ int chunk_excl_scan(int (&v)[N]) {
    int s = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int x = v[k];
        v[k] = s;
        s += x;
    }
    const int inc = wave_incl_scan_dpp(s);
    const int ex = inc - s;
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] += ex;
    return __builtin_amdgcn_readlane(inc, 63);
}

// NB rounds of one key per lane (the atomics of all rounds after their scans), its bin b (0xFFFFFFFF: no key)
// and value v = response << 24 | 0xFFFFFF - index.  Lanes of a wave mostly hold consecutive keys of one
// cell, i.e. a few bins each held by a run of lanes, so the histogram / maximum go through the run heads /
// tails instead of 64 same-address LDS atomics: counts: the head of each run of equal bins (across the
// wave) adds the run length; maxima: a segmented max inside each 16-lane row (idempotent, so reaching
// further than the run is harmless) and the last lane of each run within a row applies it.
template <int NB>
__device__ __forceinline__ void bin_add_runs(uint32_t* hist, uint32_t* bmax, const uint32_t (&bb)[NB],
                                             const uint32_t (&vv)[NB]) {
    const int lane = threadIdx.x & 63;
    const uint32_t nob = 0xFFFFFFFEu;
    int cnt[NB];
    uint32_t mx[NB];
    bool tl[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const uint32_t b = bb[u];
        const uint32_t prev = (uint32_t)__shfl_up((int)b, 1, 64);
        const bool valid = b != 0xFFFFFFFFu;
        const bool head = valid && (lane == 0 || prev != b);
        const uint64_t heads = __ballot(head) | ~__ballot(valid);  // an invalid lane also ends a run
        const uint64_t after = lane == 63 ? 0ull : heads & (~0ull << (lane + 1));
        cnt[u] = head ? (after ? __builtin_ctzll(after) : 64) - lane : 0;
        uint32_t m = vv[u];
        uint32_t pb = dpp_shr<1>(nob, b), pv = dpp_shr<1>(0u, m);
        if (pb == b) m = max(m, pv);
        pb = dpp_shr<2>(nob, b); pv = dpp_shr<2>(0u, m);
        if (pb == b) m = max(m, pv);
        pb = dpp_shr<4>(nob, b); pv = dpp_shr<4>(0u, m);
        if (pb == b) m = max(m, pv);
        pb = dpp_shr<8>(nob, b); pv = dpp_shr<8>(0u, m);
        if (pb == b) m = max(m, pv);
        mx[u] = m;
        // run tails from the ballot, like the heads: the next lane starts a run, holds no key or has left the
        // caller's key loop (a shuffle from an inactive lane would read 0, i.e. bin 0: ADVICE r3)
        tl[u] = valid && ((lane & 15) == 15 || lane == 63 || ((heads >> (lane + 1)) & 1ull));
    }
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        if (cnt[u]) atomicAdd(&hist[bb[u]], (uint32_t)cnt[u]);
        if (tl[u]) atomicMax(&bmax[bb[u]], mx[u]);
    }
}

struct ObLds {
    uint32_t* bins;        // B + 1: histogram -> cumulative counts (bit 31: kObDeep) -> final node map
    int *coff, *soff;      // per cell: first key index (ncell + 1), slot offset
    uint32_t *code0, *code1;  // node list (double-buffered): left-aligned path code, key count, depth
    int *cnt0, *cnt1;
    uint8_t *dep0, *dep1;
    int *sa, *sb, *sd, *sp;
    uint64_t* srt;
    uint32_t* c4;          // deep nodes' child counts, two u16 per word
    int* dl;               // nodes deeper than D0 being divided / in the final list
    uint8_t* proc;
    uint32_t* tab;         // the level's X then Y table
    uint32_t* bmax;        // per bin: max of (response << 24 | 0xFFFFFF - key index)
    uint16_t* bcell;       // per key block (kObKblkSh): the cell of its first key (the first oct_kblk_max blocks)
    uint64_t* lst2;        // FLAT: the second node list (packed code | (count << 8 | depth) << 32)
};

__host__ __device__ inline size_t ob_align(size_t v) { return (v + 15) & ~(size_t)15; }

// NC node slots, B bins, CM cells, TW table words
template <typename F>
__host__ __device__ inline size_t ob_carve(int NC, int B, int CM, int TW, int KB, F&& at) {
    size_t o = 0;
    auto take = [&](int id, size_t bytes) { at(id, o); o += ob_align(bytes); };
    take(0, 4 * (size_t)(B + 1));
    take(1, 4 * (size_t)(CM + 1));
    take(2, 4 * (size_t)CM);
    take(3, 4 * (size_t)NC);
    take(4, 4 * (size_t)NC);
    take(5, 4 * (size_t)NC);
    take(6, 4 * (size_t)NC);
    take(7, (size_t)NC);
    take(8, (size_t)NC);
    take(9, 4 * (size_t)NC);
    take(10, 4 * (size_t)NC);
    take(11, 4 * (size_t)NC);
    take(12, 4 * (size_t)NC);
    take(13, 8 * (size_t)(NC > 64 * kObNpl ? NC : 64 * kObNpl));  // + the register passes' full-chunk reads
    take(14, 8 * (size_t)NC);
    take(15, 4 * (size_t)NC);
    take(16, (size_t)NC);
    take(17, 4 * (size_t)TW);
    take(18, 4 * (size_t)B);
    take(19, 2 * (size_t)KB);
    take(20, 8 * (size_t)(NC <= 64 * kObNpl ? 64 * kObNpl : 0));  // the flat passes' second list buffer
    return o;
}

// NT threads: 256 (large batches: the workgroups of many images share the CUs) or kObSmallNT (512) for small batches,
// where a few images' workgroups are the critical path.
template <int NT, bool FLAT>
__global__ __launch_bounds__(NT) void k_octree_bins(Geo g, const CellGeo* __restrict__ cells,
                                                            const int* __restrict__ cell_count,
                                                            const uint32_t* __restrict__ slots,
                                                            const uint32_t* __restrict__ octab,
                                                            uint32_t* __restrict__ lvl_kp, int* __restrict__ lvl_count,
                                                            int* __restrict__ overflow, int maxcell,
                                                            uint32_t* __restrict__ kcache_all,
                                                            long long* __restrict__ prof) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    __shared__ int s_K, s_S, s_cur, s_nd, s_cmd;
    const int img = blockIdx.x, l = blockIdx.y, t = threadIdx.x;
    long long* pm = prof ? prof + ((int64_t)img * g.nlevels + l) * 64 : nullptr;
    auto mark = [&](int id) {
        if (pm && t == 0 && id < 64) pm[id] = (long long)wall_clock64();
    };
    mark(0);
    const LevelGeo& L = g.lv[l];
    const KeyDiv kv = key_div(L);
    const int NC = g.max_ncap;
    ObLds d;
    ob_carve(NC, g.oct_bins_max, maxcell, g.oct_tab_max, g.oct_kblk_max, [&](int id, size_t off) {
        unsigned char* p = lds + off;
        switch (id) {
            case 0: d.bins = (uint32_t*)p; break;
            case 1: d.coff = (int*)p; break;
            case 2: d.soff = (int*)p; break;
            case 3: d.code0 = (uint32_t*)p; break;
            case 4: d.code1 = (uint32_t*)p; break;
            case 5: d.cnt0 = (int*)p; break;
            case 6: d.cnt1 = (int*)p; break;
            case 7: d.dep0 = p; break;
            case 8: d.dep1 = p; break;
            case 9: d.sa = (int*)p; break;
            case 10: d.sb = (int*)p; break;
            case 11: d.sd = (int*)p; break;
            case 12: d.sp = (int*)p; break;
            case 13: d.srt = (uint64_t*)p; break;
            case 14: d.c4 = (uint32_t*)p; break;
            case 15: d.dl = (int*)p; break;
            case 16: d.proc = p; break;
            case 17: d.tab = (uint32_t*)p; break;
            case 18: d.bmax = (uint32_t*)p; break;
            case 19: d.bcell = (uint16_t*)p; break;
            default: d.lst2 = (uint64_t*)p; break;
        }
    });
    const int N = L.n_feat, ncell = L.ncell;
    uint32_t* out = lvl_kp + (int64_t)img * g.lvl_kp_cap + L.kp_off;
    int* count_out = lvl_count + img * g.nlevels + l;
    if (ncell == 0) {
        if (t == 0) *count_out = 0;
        return;
    }
    const int D = L.oct_d, D0 = L.oct_d0, B = L.oct_bins, bsh = 2 * (D - D0);
    const int nx = L.oct_nx, ny = L.oct_ny;
    // ---- 1. per-cell key offsets (cell order = vToDistributeKeys order), the level's tables, empty bins
    for (int i = t; i < ncell; i += NT) {
        d.coff[i] = cell_count[(int64_t)img * g.ncells + L.cell0 + i];
        d.soff[i] = cells[L.cell0 + i].slot_off;
    }
    for (int i = t; i < nx + ny; i += NT) d.tab[i] = octab[L.oct_xt + i];  // X then Y (adjacent)
    for (int i = t; i <= B; i += NT) d.bins[i] = 0;
    for (int i = t; i < B; i += NT) d.bmax[i] = 0;
    __syncthreads();
    mark(3);
    if (t < 64) {
        const int K = wave_scan_lds(d.coff, ncell);
        if (t == 0) {
            d.coff[ncell] = K;
            s_K = K;
        }
    }
    __syncthreads();
    mark(4);
    const int K = s_K;
    if (K == 0) {
        if (t == 0) *count_out = 0;
        return;
    }
    // every key's cell: a u16 per key in the node-list region (code0 .. proc, untouched until the passes)
    // when the level's keys fit there (K <= kcap: every KITTI / EuRoC level); otherwise the first cell of
    // every key block (the cells whose key range holds a multiple of 16; keys past the table's
    // Geo::oct_kblk_max blocks start from its last entry), walked forward by the sweep
    uint16_t* const kcell = (uint16_t*)d.code0;
    const int kcap = (int)(((unsigned char*)d.tab - (unsigned char*)d.code0) >> 1);
    const bool kdirect = K <= kcap;
    const int nblk = g.oct_kblk_max;
    for (int c = t; c < ncell; c += NT) {
        const int a = d.coff[c], e = d.coff[c + 1];
        if (kdirect) {
            for (int k = a; k < e; ++k) kcell[k] = (uint16_t)c;
        } else {
            for (int b = (a + (1 << kObKblkSh) - 1) >> kObKblkSh; (b << kObKblkSh) < e && b < nblk; ++b)
                d.bcell[b] = (uint16_t)c;
        }
    }
    __syncthreads();
    const uint32_t* islots = slots + (int64_t)img * g.slot_total;
    const uint32_t* X = d.tab;
    const uint32_t* Y = d.tab + nx;
    auto key_code = [&](uint32_t v) {
        int x, y;
        key_xy(v, kv, x, y);
        x = min(max(x - kBorder, 0), nx - 1);
        y = min(max(y - kBorder, 0), ny - 1);
        return X[x] | Y[y];
    };
    // The first sweep, every key once: keys k = t, t + NT, ... (consecutive keys in consecutive lanes:
    // coalesced slot reads), OB of them per thread per round; a key's cell from kcell (or its block's first
    // cell walked forward); the OB keys' codes and run heads / tails first, then their LDS atomics (one
    // key's atomics would otherwise order the next key's table reads behind them).  OB: 4 at 256 threads, 2 at
    // 512 (small batches: 8 pairs 30.3 -> 29.2 us; 4 / 8 at 256 threads: 0.358 / 0.371 ms standalone)
    constexpr int OB = NT >= 512 ? kObBatch / 2 : kObBatch;
    // the first sweep also leaves every key's slot value in key order in global scratch (kc, the level's
    // 16-byte aligned range of the handle's candidate scratch), so the later sweeps (children of nodes
    // deeper than D0, the final map) read keys with dwordx4 loads instead of walking cells: for_cached,
    // keys 4 (tid + nthr j) .. + 3, kObBatch / 2 loads in flight; fn(k, value, code) also for k >= K (the
    // padding of the last 4 keys), which fn ignores.  Written and read inside this workgroup (same CU, the
    // barrier between orders them).
    uint32_t* kc = kcache_all + (int64_t)img * g.key_total + L.key_off;
    auto for_cached = [&](int tid, int nthr, auto nbc, auto&& fn) {
        constexpr int NB = decltype(nbc)::value;
        for (int k0 = 4 * tid; k0 < K; k0 += 4 * nthr * NB) {
            uint4 v[NB];
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int k = k0 + 4 * nthr * u;
                v[u] = k < K ? *(const uint4*)(kc + k) : uint4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int k = k0 + 4 * nthr * u;
                fn(k, v[u].x, key_code(v[u].x));
                fn(k + 1, v[u].y, key_code(v[u].y));
                fn(k + 2, v[u].z, key_code(v[u].z));
                fn(k + 3, v[u].w, key_code(v[u].w));
            }
        }
    };
    mark(5);
    for (int k0 = t; k0 < K; k0 += NT * OB) {
        int lo[OB];
        if (kdirect) {
#pragma unroll
            for (int u = 0; u < OB; ++u) lo[u] = kcell[min(k0 + NT * u, K - 1)];
        } else {
#pragma unroll
            for (int u = 0; u < OB; ++u) lo[u] = d.bcell[min(min(k0 + NT * u, K - 1) >> kObKblkSh, nblk - 1)];
            bool more = true;
            while (__ballot(more)) {
                more = false;
#pragma unroll
                for (int u = 0; u < OB; ++u) {
                    const bool f = d.coff[lo[u] + 1] <= k0 + NT * u && k0 + NT * u < K;
                    lo[u] += f;
                    more |= f;
                }
            }
        }
        uint32_t v[OB], bn[OB], bv[OB];
#pragma unroll
        for (int u = 0; u < OB; ++u) {
            const int k = k0 + NT * u;
            v[u] = k < K ? islots[d.soff[lo[u]] + (k - d.coff[lo[u]])] : 0u;
        }
#pragma unroll
        for (int u = 0; u < OB; ++u) {
            const int k = k0 + NT * u;
            bn[u] = k < K ? key_code(v[u]) >> bsh : 0xFFFFFFFFu;
            bv[u] = (v[u] & 0xFF000000u) | (0xFFFFFFu - (uint32_t)k);
            if (k < K) kc[k] = v[u];
        }
        bin_add_runs<OB>(d.bins, d.bmax, bn, bv);
    }
    mark(6);
    __syncthreads();
    mark(1);

    // The nn nodes deeper than D0 listed in d.dl (list `code`) sorted by code into d.sp (codes) / d.sd (list
    // positions), by every thread (rank = number of smaller codes; the nodes are disjoint, so their
    // left-aligned codes differ).  A key's node is then the last one whose code is <= the key's, if the
    // key lies inside it: a binary search instead of a scan over all deep nodes per key.
    auto deep_sort = [&](int nn, const uint32_t* code) {
        for (int i = t; i < nn; i += NT) {
            const int p = d.dl[i];
            const uint32_t ci = code[p];
            int r = 0;
            for (int j = 0; j < nn; ++j) r += code[d.dl[j]] < ci;
            d.sp[r] = (int)ci;
            d.sd[r] = p;
        }
    };
    // list position of the sorted deep node holding key code cd (-1: none)
    auto deep_find = [&](int nn, const uint32_t* code, const uint8_t* dep, uint32_t cd) {
        int lo = 0, hi = nn - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((uint32_t)d.sp[mid] <= cd) lo = mid; else hi = mid - 1;
        }
        const int p = d.sd[lo];
        return (uint32_t)d.sp[lo] <= cd && ((cd ^ code[p]) >> (2 * (D - dep[p]))) == 0u ? p : -1;
    };
    // sweep over the keys for the children counts of the deep nodes (list `lst`): every wave takes part
    // (wave 0 hands it out from inside its passes, see deep_counts)
    auto deep_sweep = [&](int nn, int lst) {
        const uint32_t* code = lst ? d.code1 : d.code0;
        const uint8_t* dep = lst ? d.dep1 : d.dep0;
        deep_sort(nn, code);
        __syncthreads();
        for_cached(t, NT, std::integral_constant<int, 1>{}, [&](int kk, uint32_t, uint32_t cd) {
            if (kk >= K || !(d.bins[cd >> bsh] & kObDeep)) return;
            const int p = deep_find(nn, code, dep, cd);
            if (p >= 0) {
                const int q = (int)((cd >> (2 * (D - dep[p] - 1))) & 3u);
                atomicAdd(&d.c4[2 * p + (q >> 1)], (q & 1) ? 0x10000u : 1u);
            }
        });
    };
    // FLAT: node lists by position in LDS, packed (code | (count << 8 | depth) << 32); the deep sweeps read
    // the current one in place
    uint64_t* lst = d.srt;
    auto node_code = [](const uint64_t* l, int p) { return (uint32_t)l[p]; };
    auto node_cnt = [](const uint64_t* l, int p) { return (int)(l[p] >> 40); };
    auto node_dep = [](const uint64_t* l, int p) { return (int)((l[p] >> 32) & 0xFFu); };
    auto deep_sort_l = [&](int nn, const uint64_t* l) {
        for (int i = t; i < nn; i += NT) {
            const int p = d.dl[i];
            const uint32_t ci = node_code(l, p);
            int r = 0;
            for (int j = 0; j < nn; ++j) r += node_code(l, d.dl[j]) < ci;
            d.sp[r] = (int)ci;
            d.sd[r] = p;
        }
    };
    auto deep_find_l = [&](int nn, uint32_t cd, const uint64_t* l) {
        int lo = 0, hi = nn - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((uint32_t)d.sp[mid] <= cd) lo = mid; else hi = mid - 1;
        }
        const int p = d.sd[lo];
        return (uint32_t)d.sp[lo] <= cd && ((cd ^ node_code(l, p)) >> (2 * (D - node_dep(l, p)))) == 0u ? p : -1;
    };
    // ---- 2. wave 0: cumulative counts, initial columns (:543-584), the passes (:585-737); the other waves
    //      wait for deep sweeps (s_cmd: 1 | list << 1 with s_nd nodes; 0 when the passes are over)
    if constexpr (FLAT) {
        // ---------------- all threads (FLAT).  The full passes (:593-671) in closed form from the bin
        // histogram: after pass j the list is the depth-j nodes created in pass j (every nonempty child of a
        // node holding >= 2 keys) in reverse creation order, then the single-key nodes created in passes
        // j-1, ..., 0, each group in its own reverse creation order (push_front keeps them in place).
        // Creation order alternates direction from depth to depth, so every group's list order is the
        // numeric order of the node's Morton index with every other 2-bit digit (and, at odd depths, the
        // column) mirrored: the list is one flat enumeration + one block scan.  The careful phase
        // (:675-737) divides candidates in (size desc, creation desc) order: a stable radix sort of the
        // candidates by size, a scan of the list growth in that order for the break, scans for the
        // positions.  Nodes deeper than D0 take the deep sweeps (every thread).
        constexpr int CAPL = 64 * kObNpl;
        constexpr int LP = (CAPL + NT - 1) / NT;      // list positions per thread (p = t LP + k)
        constexpr int EB = (2048 + 1 + NT - 1) / NT;  // bins (+ the total) per thread
        constexpr int EP = (2816 + NT - 1) / NT;      // closed-form enumeration: sum over depths <= D0 of nodes
        constexpr int NW = NT / 64;
        __shared__ int s_red[2][NW];
        int red_par = 0;
        __shared__ int s_dc[3][16];                    // per depth: listed nodes, of which single-key, >= 2 keys
        __shared__ int s_cw[2][NW][16];                // radix: per-wave digit counts (by pass parity)
        __shared__ int s_m[4];
        const int lane = t & 63, wv = t >> 6;
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        // exclusive block scan of v (thread-contiguous order t * E + k), in place; returns the total
        auto bscan = [&](auto& v) -> int {
            constexpr int E = sizeof(v) / sizeof(v[0]);
            int s0 = 0;
#pragma unroll
            for (int k = 0; k < E; ++k) {
                const int x = v[k];
                v[k] = s0;
                s0 += x;
            }
            const int inc = wave_incl_scan_dpp(s0);
            // the wave totals alternate between two buffers: the next scan writes the other one, and the one
            // after it comes after the next scan's barrier, i.e. after every wave has read this one
            int* red = s_red[red_par];
            red_par ^= 1;
            if (lane == 63) red[wv] = inc;
            __syncthreads();
            int off = 0, tot = 0;
#pragma unroll
            for (int i = 0; i < NW; ++i) {
                const int r = red[i];
                off += i < wv ? r : 0;
                tot += r;
            }
            const int ex = off + inc - s0;
#pragma unroll
            for (int k = 0; k < E; ++k) v[k] += ex;
            return tot;
        };
        // workgroup OR of a predicate, one barrier (the scans' alternating wave-total buffers)
        auto bor = [&](bool q) -> bool {
            int* red = s_red[red_par];
            red_par ^= 1;
            const bool wq = __ballot(q) != 0ull;
            if (lane == 0) red[wv] = wq;
            __syncthreads();
            int any = 0;
#pragma unroll
            for (int i = 0; i < NW; ++i) any |= red[i];
            return any != 0;
        };
        auto pack = [](uint32_t code, int n, int dp) {
            return (uint64_t)code | ((uint64_t)(((uint32_t)n << 8) | (uint32_t)dp) << 32);
        };
        for (int i = t; i < NC; i += NT) d.proc[i] = 0;  // (ordered before use by bscan's barriers)
        for (int i = t; i < 2 * 16 * NW; i += NT) (&s_cw[0][0][0])[i] = 0;
        // cumulative bin counts, bins[B] = K
        {
            int v[EB];
#pragma unroll
            for (int k = 0; k < EB; ++k) {
                const int i = t * EB + k;
                v[k] = i < B ? (int)d.bins[i] : 0;
            }
            bscan(v);
#pragma unroll
            for (int k = 0; k < EB; ++k)
                if (t * EB + k <= B) d.bins[t * EB + k] = (uint32_t)v[k];
            if (t < 48) (&s_dc[0][0])[t] = 0;
            __syncthreads();
        }
        mark(40);
        auto cum = [&](int b) { return (int)(d.bins[b] & ~kObDeep); };
        auto ncnt = [&](int dd, int i) {
            const int sh = 2 * (D0 - dd);
            return cum((i + 1) << sh) - cum(i << sh);
        };
        // per depth d <= D0: nodes a pass creates (nonempty, parent holds >= 2 keys; every nonempty column at
        // depth 0), how many of them hold one key, how many >= 2
        for (int dd = 0; dd <= D0; ++dd) {
            const int P = L.n_ini << (2 * dd);
            for (int i0 = 0; i0 < P; i0 += NT) {
                const int i = i0 + t;
                int c = 0, pc = 2;
                if (i < P) {
                    c = ncnt(dd, i);
                    if (dd) pc = ncnt(dd - 1, i >> 2);
                }
                const bool q = i < P && c >= 1 && pc >= 2;
                const uint64_t ba = __ballot(q), b1 = __ballot(q && c == 1), bx = __ballot(q && c >= 2);
                if (lane == 0 && ba) {
                    atomicAdd(&s_dc[0][dd], __popcll(ba));
                    atomicAdd(&s_dc[1][dd], __popcll(b1));
                    atomicAdd(&s_dc[2][dd], __popcll(bx));
                }
            }
        }
        __syncthreads();
        mark(41);
        // the passes the reference makes (:668-672), replayed on the counts: J passes, then finish (1),
        // the careful phase (2), or more full passes below D0 (3)
        int J = 0, mode = 0, S = s_dc[0][0];
        {
            int sprev = S, n1 = 0;
            for (int j = 1;; ++j) {
                if (j > D0) {
                    J = D0;
                    mode = 3;
                    S = sprev;
                    break;
                }
                n1 += s_dc[1][j - 1];
                const int Sj = s_dc[0][j] + n1;
                if (Sj >= N || Sj == sprev) {
                    J = j;
                    mode = 1;
                    S = Sj;
                    break;
                }
                if (Sj + 3 * s_dc[2][j] > N) {
                    J = j;
                    mode = 2;
                    S = Sj;
                    break;
                }
                sprev = Sj;
            }
        }
        uint64_t* cur = lst;
        uint64_t* nxt = d.lst2;
        // the list after pass J: depth J (every created node), then depths J-1 .. 0 (single-key nodes)
        {
            // every entry's depth from one scalar walk over the depths (not one per entry), then all entries'
            // bin reads issued together (clamped, unconditional) and waited once: per-entry branches had
            // serialised the entries' LDS round trips
            const int nini = __builtin_amdgcn_readfirstlane(L.n_ini);
            int v[EP], dk[EP], ik[EP], rr[EP];
#pragma unroll
            for (int k = 0; k < EP; ++k) {
                dk[k] = -1;
                rr[k] = 0;
            }
            {
                int o = 0;
                for (int e = J; e >= 0; --e) {
                    const int P = nini << (2 * e);
#pragma unroll
                    for (int k = 0; k < EP; ++k) {
                        const int f = t * EP + k;
                        if (dk[k] < 0 && f < o + P) {
                            dk[k] = e;
                            rr[k] = f - o;
                        }
                    }
                    o += P;
                }
            }
            int a0[EP], a1[EP], b0[EP], b1[EP];
#pragma unroll
            for (int k = 0; k < EP; ++k) {
                const int dd = max(dk[k], 0), sh = 2 * dd, r = rr[k];
                const int colp = r >> sh;
                const int col = (dd & 1) ? nini - 1 - colp : colp;
                const int i = (col << sh) | ((r & ((1 << sh) - 1)) ^ (0x33333333 & ((1 << sh) - 1)));
                ik[k] = i;
                const int bs = 2 * (D0 - dd);  // ncnt(dd, i) and, below, ncnt(dd - 1, i >> 2)
                a0[k] = (int)d.bins[i << bs];
                a1[k] = (int)d.bins[(i + 1) << bs];
                const int pi = dd ? i >> 2 : 0, ps = dd ? bs + 2 : bs;
                b0[k] = (int)d.bins[pi << ps];
                b1[k] = (int)d.bins[(pi + 1) << ps];
            }
            int cc[EP];
#pragma unroll
            for (int k = 0; k < EP; ++k) {
                const int dd = dk[k];
                const int c = (a1[k] & ~(int)kObDeep) - (a0[k] & ~(int)kObDeep);
                const int pc = dd > 0 ? (b1[k] & ~(int)kObDeep) - (b0[k] & ~(int)kObDeep) : 2;
                cc[k] = c;
                v[k] = dd >= 0 && c >= 1 && pc >= 2 && (dd == J || c == 1);
            }
            int fl[EP];
#pragma unroll
            for (int k = 0; k < EP; ++k) fl[k] = v[k];
            bscan(v);
#pragma unroll
            for (int k = 0; k < EP; ++k)
                if (fl[k] && v[k] < CAPL) cur[v[k]] = pack((uint32_t)ik[k] << (2 * (D - dk[k])), cc[k], dk[k]);
        }
        if (S > CAPL) {  // cannot happen (S <= N or <= 4 nIni, both within kp_cap <= CAPL)
            if (t == 0) atomicOr(overflow, 4);
            S = CAPL;
            mode = 1;
        }
        int C = s_dc[0][J];
        __syncthreads();
        mark(2);
        mark(42);
        // children counts of node p of list l (registers: code, depth)
        auto child_counts = [&](uint32_t code, int dp, int p) {
            int4 cc;
            if (dp < D0) {
                const int lo = (int)(code >> bsh), w = 1 << (2 * (D0 - dp - 1));
                const int c0 = cum(lo), c1 = cum(lo + w), c2 = cum(lo + 2 * w), c3 = cum(lo + 3 * w), c4 = cum(lo + 4 * w);
                cc = int4{c1 - c0, c2 - c1, c3 - c2, c4 - c3};
            } else {
                const uint32_t a = d.c4[2 * p], b = d.c4[2 * p + 1];
                cc = int4{(int)(a & 0xFFFFu), (int)(a >> 16), (int)(b & 0xFFFFu), (int)(b >> 16)};
            }
            return cc;
        };
        auto nonempty = [](const int4& cc) { return (cc.x > 0) + (cc.y > 0) + (cc.z > 0) + (cc.w > 0); };
        // children counts of the nodes deeper than D0 among the division candidates sel(p): one sweep of every
        // thread over the cached keys
        auto deep_counts = [&](auto&& sel) {
            // (a pass without deep candidates costs one barrier: the OR)
            bool any = false;
#pragma unroll
            for (int k = 0; k < LP; ++k) any |= sel(t * LP + k) && node_dep(cur, t * LP + k) >= D0;
            if (t == 0) s_m[0] = 0;
            if (!bor(any)) return;
#pragma unroll
            for (int k = 0; k < LP; ++k) {
                const int p = t * LP + k;
                if (sel(p) && node_dep(cur, p) >= D0) {
                    d.dl[atomicAdd(&s_m[0], 1)] = p;
                    d.c4[2 * p] = 0u;
                    d.c4[2 * p + 1] = 0u;
                    atomicOr(&d.bins[node_code(cur, p) >> bsh], kObDeep);
                }
            }
            __syncthreads();
            const int nd = s_m[0];
            deep_sort_l(nd, cur);
            __syncthreads();
            for_cached(t, NT, std::integral_constant<int, 1>{}, [&](int kk, uint32_t, uint32_t cd) {
                if (kk >= K || !(d.bins[cd >> bsh] & kObDeep)) return;
                const int p = deep_find_l(nd, cd, cur);
                if (p >= 0) {
                    const int q = (int)((cd >> (2 * (D - node_dep(cur, p) - 1))) & 3u);
                    atomicAdd(&d.c4[2 * p + (q >> 1)], (q & 1) ? 0x10000u : 1u);
                }
            });
            __syncthreads();
            for (int i = t; i < nd; i += NT) atomicAnd(&d.bins[node_code(cur, d.dl[i]) >> bsh], ~kObDeep);
            __syncthreads();
        };
        // writes node p's children (counts cc, already known non-empty count) to nxt from position top
        // downwards: push_front of n1 .. n4 (:620-659, :690-725)
        auto put_children = [&](uint32_t code, int dp, const int4& cc, int top) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int n = q == 0 ? cc.x : q == 1 ? cc.y : q == 2 ? cc.z : cc.w;
                if (n > 0) nxt[top--] = pack(code | ((uint32_t)q << (2 * (D - dp - 1))), n, dp + 1);
            }
        };
        bool ovf = false;
        int rpass = 0;  // radix passes so far (the digit-count buffer's parity)
        for (int iter = 0; mode >= 2; ++iter) {
            if (iter > 4 * CAPL + 64) {  // cannot happen (each pass grows the list or finishes); never hang
                if (t == 0) atomicOr(overflow, 2);
                break;
            }
            mark(8 + 4 * iter);
            int Sn, Cn;
            if (mode == 3) {
                // ---------------- a full pass below D0 (:605-664): divide every node holding > 1 key
                deep_counts([&](int p) { return p < S && node_cnt(cur, p) > 1; });
                int cb[LP], kp[LP], ne = 0;
#pragma unroll
                for (int k = 0; k < LP; ++k) {
                    const int p = t * LP + k;
                    const int n = p < S ? node_cnt(cur, p) : 0;
                    const int4 cc = n > 1 ? child_counts(node_code(cur, p), node_dep(cur, p), p) : int4{0, 0, 0, 0};
                    cb[k] = nonempty(cc);
                    ne += (cc.x > 1) + (cc.y > 1) + (cc.z > 1) + (cc.w > 1);
                    kp[k] = n == 1;
                }
                int nev[1] = {ne};
                const int nexp = bscan(nev);
                Cn = bscan(cb);
                const int Kk = bscan(kp);
                Sn = Cn + Kk;
                if (Sn <= CAPL) {
#pragma unroll
                    for (int k = 0; k < LP; ++k) {
                        const int p = t * LP + k;
                        const int n = p < S ? node_cnt(cur, p) : 0;
                        if (n > 1)
                            put_children(node_code(cur, p), node_dep(cur, p),
                                         child_counts(node_code(cur, p), node_dep(cur, p), p), Cn - 1 - cb[k]);
                        else if (n == 1)
                            nxt[Cn + kp[k]] = cur[p];
                    }
                }
                if (Sn > CAPL) { ovf = true; mode = 0; }
                else if (Sn >= N || Sn == S) mode = 0;              // :668-671
                else if (Sn + 3 * nexp > N) mode = 2;               // :672
            } else {
                // ---------------- careful phase (:675-736): the expandable nodes of the last step (its
                // children, positions < C) by size descending, equal sizes in creation order descending (=
                // position ascending), divided until the list reaches N
                auto cand = [&](int p) { return p < C && node_cnt(cur, p) > 1; };
                if (t == 0) s_m[3] = 0;  // (read last iteration after its proc barrier; the atomics come after 3+ barriers)
                deep_counts(cand);
                if (iter == 0) mark(43);
                // candidates in position order -> (size, position | children << 16) at their compacted index
                int mi[LP], ncl[LP];
                int mx = 0;
#pragma unroll
                for (int k = 0; k < LP; ++k) {
                    const int p = t * LP + k;
                    const bool c = cand(p);
                    ncl[k] = c ? nonempty(child_counts(node_code(cur, p), node_dep(cur, p), p)) : 0;
                    mi[k] = c;
                    if (c) mx = max(mx, node_cnt(cur, p));
                }
                int cf[LP];
#pragma unroll
                for (int k = 0; k < LP; ++k) cf[k] = mi[k];
                if (t == 0) s_m[1] = 0;
                const int M = bscan(mi);  // (its barriers order s_m[1]'s reset before the maxima)
                if (mx) atomicMax(&s_m[1], mx);
                int* ka = d.sa;  // sizes (ping-pong: ka / kb) and payloads (pa / pb)
                int* kb = d.sb;
                int* pa = d.sd;
                int* pb = d.sp;
#pragma unroll
                for (int k = 0; k < LP; ++k)
                    if (cf[k]) {
                        const int p = t * LP + k;
                        ka[mi[k]] = node_cnt(cur, p);
                        pa[mi[k]] = p | (ncl[k] << 16);
                    }
                __syncthreads();
                if (iter == 0) mark(44);
                // stable LSD radix sort by size, descending, 4-bit digits while the largest size has any
                for (int sh = 0; sh < 32 && (s_m[1] >> sh) != 0; sh += 4) {
                    int dg[LP], rk[LP];
#pragma unroll
                    for (int k = 0; k < LP; ++k) {
                        const int e = t * LP + k;
                        dg[k] = e < M ? 15 - ((ka[e] >> sh) & 15) : -1;
                    }
                    // stable ranks inside the wave: elements (lane, k) in that order; the lanes whose element j
                    // holds digit x are valid_j & (x's bits of the four digit-bit ballots) — no loop over digits
                    uint64_t bb[LP][4], vb[LP];
#pragma unroll
                    for (int k = 0; k < LP; ++k) {
                        vb[k] = __ballot(dg[k] >= 0);
#pragma unroll
                        for (int bit = 0; bit < 4; ++bit) bb[k][bit] = __ballot(dg[k] >= 0 && ((dg[k] >> bit) & 1));
                    }
#pragma unroll
                    for (int k = 0; k < LP; ++k) {
                        rk[k] = 0;
                        if (dg[k] < 0) continue;
#pragma unroll
                        for (int j = 0; j < LP; ++j) {
                            uint64_t m = vb[j];
#pragma unroll
                            for (int bit = 0; bit < 4; ++bit) m &= ((dg[k] >> bit) & 1) ? bb[j][bit] : ~bb[j][bit];
                            rk[k] += __popcll(m & lt) + (j < k && dg[j] == dg[k]);
                        }
                        atomicAdd(&s_cw[rpass & 1][wv][dg[k]], 1);
                    }
                    // the other buffer, for the next pass: its readers (the previous pass) are past that pass's
                    // last barrier; the next pass's counts come after this pass's two
                    for (int i = t; i < 16 * NW; i += NT) (&s_cw[(rpass + 1) & 1][0][0])[i] = 0;
                    __syncthreads();
                    // every wave its own offsets, lane b = digit b: every smaller digit, then earlier waves' b
                    int below = 0, tot = 0;
                    if (lane < 16) {
#pragma unroll
                        for (int w = 0; w < NW; ++w) {
                            const int c = s_cw[rpass & 1][w][lane];
                            below += w < wv ? c : 0;
                            tot += c;
                        }
                    }
                    const int myoff = wave_incl_scan_dpp(tot) - tot + below;  // (lanes >= 16 add nothing)
                    ++rpass;
#pragma unroll
                    for (int k = 0; k < LP; ++k) {
                        const int o = __shfl(myoff, dg[k] < 0 ? 0 : dg[k]) + rk[k];
                        if (dg[k] >= 0) {
                            const int e = t * LP + k;
                            kb[o] = ka[e];
                            pb[o] = pa[e];
                        }
                    }
                    __syncthreads();
                    int* tk = ka; ka = kb; kb = tk;
                    int* tp = pa; pa = pb; pb = tp;
                }
                if (iter == 0) mark(45);
                // growth (children - 1) and children in processing order: a candidate is divided iff the list
                // before it is below N (:729-730); the divided ones are a prefix
                int gv[LP];
#pragma unroll
                for (int k = 0; k < LP; ++k) {
                    const int e = t * LP + k;
                    const int nc = e < M ? pa[e] >> 16 : 0;
                    gv[k] = e < M ? (nc - 1) | (nc << 16) : 0;
                }
                bscan(gv);
#pragma unroll
                for (int k = 0; k < LP; ++k) {
                    const int e = t * LP + k;
                    if (e < M && S + (gv[k] & 0xFFFF) < N) {
                        atomicMax(&s_m[3], (gv[k] >> 16) + (pa[e] >> 16));  // children up to and including it
                        d.proc[pa[e] & 0xFFFF] = 1;
                    }
                }
                __syncthreads();
                if (iter == 0) mark(46);
                Cn = s_m[3];
                int kp[LP];
#pragma unroll
                for (int k = 0; k < LP; ++k) {
                    const int p = t * LP + k;
                    kp[k] = p < S && !d.proc[p];
                }
                const int Kk = bscan(kp);
                Sn = Cn + Kk;
                if (Sn <= CAPL) {
#pragma unroll
                    for (int k = 0; k < LP; ++k) {
                        const int e = t * LP + k;
                        if (e < M && S + (gv[k] & 0xFFFF) < N) {
                            const int p = pa[e] & 0xFFFF;
                            put_children(node_code(cur, p), node_dep(cur, p),
                                         child_counts(node_code(cur, p), node_dep(cur, p), p), Cn - 1 - (gv[k] >> 16));
                        }
                        const int p = t * LP + k;
                        if (p < S && !d.proc[p]) nxt[Cn + kp[k]] = cur[p];
                    }
                }
                // proc[p] is read only by p's own thread (above and in kp): it clears it; the loop's last barrier
                // orders that before the next iteration's marks
#pragma unroll
                for (int k = 0; k < LP; ++k)
                    if (t * LP + k < S) d.proc[t * LP + k] = 0;
                if (Sn > CAPL) { ovf = true; mode = 0; }
                else if (Sn >= N || Sn == S) mode = 0;             // :733-734
            }
            __syncthreads();
            mark(9 + 4 * iter);
            if (Sn <= CAPL) {
                uint64_t* tl = cur; cur = nxt; nxt = tl;
                S = Sn;
                C = Cn;
            }
        }
        if (ovf && t == 0) atomicOr(overflow, 4);
        // nodes deeper than D0 of the final list, for the final map
        if (t == 0) s_m[0] = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < LP; ++k) {
            const int p = t * LP + k;
            if (p < S && node_dep(cur, p) > D0) d.dl[atomicAdd(&s_m[0], 1)] = p;
        }
        __syncthreads();
        if (t == 0) {
            s_S = S;
            s_cur = cur == lst ? 0 : 1;
            s_nd = s_m[0];
        }
    } else if (t >= 64) {
        for (;;) {
            __syncthreads();  // a command (deep_counts) or the end of the passes
            const int cmd = s_cmd;
            if (cmd == 0) break;
            deep_sweep(s_nd, cmd >> 1);
            __syncthreads();  // sweep complete
        }
    } else {
        wave_scan_lds((int*)d.bins, B);
        if (t == 0) d.bins[B] = (uint32_t)K;
        wsync();
        auto cum = [&](int b) { return (int)(d.bins[b] & ~kObDeep); };
        int S = 0;
        bool ovf = false;
        for (int i0 = 0; i0 < L.n_ini; i0 += 64) {  // empty columns removed, column order
            const int i = i0 + t;
            int n = 0;
            if (i < L.n_ini) n = cum((i + 1) << (2 * D0)) - cum(i << (2 * D0));
            const uint64_t bm = __ballot(n > 0);
            if (n > 0) {
                const int p = S + lanes_below(bm);
                if (p < NC) {
                    d.code0[p] = (uint32_t)i << (2 * D);
                    d.cnt0[p] = n;
                    d.dep0[p] = 0;
                }
            }
            S += __popcll(bm);
        }
        if (S > NC) {  // cannot happen: kp_cap >= 4 nIni + 2
            if (t == 0) atomicOr(overflow, 1);
            S = NC;
        }
        wsync();
        mark(2);
        int C = 0, cur = 0, phase = 0;
        bool done = false;
        // the current list's arrays (wave-uniform selects: no dynamically indexed pointer arrays)
        auto L_code = [&]() { return cur ? d.code1 : d.code0; };
        auto L_cnt = [&]() { return cur ? d.cnt1 : d.cnt0; };
        auto L_dep = [&]() { return cur ? d.dep1 : d.dep0; };
        // the four children's key counts of node p of the current list
        auto child_counts = [&](int p) {
            const int dp = L_dep()[p];
            int4 cc;
            if (dp < D0) {
                const int lo = (int)(L_code()[p] >> bsh), w = 1 << (2 * (D0 - dp - 1));
                const int c0 = cum(lo), c1 = cum(lo + w), c2 = cum(lo + 2 * w), c3 = cum(lo + 3 * w), c4 = cum(lo + 4 * w);
                cc = int4{c1 - c0, c2 - c1, c3 - c2, c4 - c3};
            } else {
                const uint32_t a = d.c4[2 * p], b = d.c4[2 * p + 1];
                cc = int4{(int)(a & 0xFFFFu), (int)(a >> 16), (int)(b & 0xFFFFu), (int)(b >> 16)};
            }
            return cc;
        };
        auto cc_at = [](const int4& cc, int q) { return q == 0 ? cc.x : q == 1 ? cc.y : q == 2 ? cc.z : cc.w; };
        // children counts of the nodes deeper than D0 among those that may divide (sel(p), p < nsel): one
        // sweep of wave 0 over the keys (scratch codes written by every thread: read at device scope)
        auto deep_counts = [&](int nsel, auto&& sel) {
            int nd = 0;
            for (int p0 = 0; p0 < nsel; p0 += 64) {
                const int p = p0 + t;
                const bool deep = p < nsel && sel(p) && L_dep()[p] >= D0;
                const uint64_t bm = __ballot(deep);
                if (deep) {
                    d.dl[nd + lanes_below(bm)] = p;
                    d.c4[2 * p] = 0u;
                    d.c4[2 * p + 1] = 0u;
                    atomicOr(&d.bins[L_code()[p] >> bsh], kObDeep);
                }
                nd += __popcll(bm);
            }
            if (nd == 0) return;
            if (t == 0) {
                s_cmd = 1 | (cur << 1);
                s_nd = nd;
            }
            __syncthreads();  // the other waves start the sweep
            deep_sweep(nd, cur);
            __syncthreads();  // every wave's counts are in
            for (int i = t; i < nd; i += 64) atomicAnd(&d.bins[L_code()[d.dl[i]] >> bsh], ~kObDeep);
            wsync();
        };
        auto put = [&](int np, uint32_t code, int n, int dp) {
            if (np < NC) {
                (cur ? d.code0 : d.code1)[np] = code;
                (cur ? d.cnt0 : d.cnt1)[np] = n;
                (cur ? d.dep0 : d.dep1)[np] = (uint8_t)dp;
            } else {
                ovf = true;
            }
        };

        for (int iter = 0; !done; ++iter) {
            if (iter > 4 * NC + 64) {  // cannot happen (each pass grows the list or finishes); never hang
                if (t == 0) atomicOr(overflow, 2);
                break;
            }
            mark(8 + 4 * iter);
            const uint32_t* code = L_code();
            const int* cnt = L_cnt();
            const uint8_t* dep = L_dep();
            if (phase == 0) {
                // ---------------- full pass (:605-664): divide every node holding more than one key
                deep_counts(S, [&](int p) { return cnt[p] > 1; });
                int nexp = 0;
                for (int p = t; p < S; p += 64) {
                    int nc = 0;
                    if (cnt[p] > 1) {
                        const int4 cc = child_counts(p);
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            nc += cc_at(cc, q) > 0;
                            nexp += cc_at(cc, q) > 1;
                        }
                    }
                    d.sa[p] = nc;
                    d.sb[p] = cnt[p] == 1;
                }
                wsync();
                const int Cn = wave_scan_lds(d.sa, S);
                const int Kk = wave_scan_lds(d.sb, S);
                nexp = __shfl(wave_incl_sum(nexp), 63, 64);
                for (int p = t; p < S; p += 64) {
                    if (cnt[p] > 1) {
                        const int4 cc = child_counts(p);
                        int c = d.sa[p];
                        const int dp = dep[p];
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (cc_at(cc, q) > 0)
                                put(Cn - 1 - c++, code[p] | ((uint32_t)q << (2 * (D - dp - 1))), cc_at(cc, q), dp + 1);
                    } else {
                        put(Cn + d.sb[p], code[p], cnt[p], dep[p]);
                    }
                }
                wsync();
                const int Sn = Cn + Kk;
                if (Sn > NC) {
                    ovf = true;
                    done = true;
                } else if (Sn >= N || Sn == S) {
                    done = true;                                     // :668-671
                } else if (Sn + 3 * nexp > N) {
                    phase = 1;                                       // :672
                }
                S = min(Sn, NC);
                C = min(Cn, NC);
                cur ^= 1;
            } else {
                // ---------------- careful phase (:675-736): divide the largest nodes of the last step first
                deep_counts(C, [&](int p) { return cnt[p] > 1; });
                // candidates (position order) -> ranked by size desc, then position asc (creation desc)
                // keys: size desc, then position asc (creation desc); unique.  32-bit (size << 16 |
                // 0xFFFF - position) when every size and position fits 16 bits, else 64-bit
                int bigl = 0;
                for (int p = t; p < C; p += 64) bigl |= cnt[p] > 0xFFFF;
                const bool k32path = !__ballot(bigl) && NC <= 0x10000;
                uint32_t* k32 = (uint32_t*)d.srt;
                int M = 0;
                for (int p0 = 0; p0 < C; p0 += 64) {
                    const int p = p0 + t;
                    const bool cand = p < C && cnt[p] > 1;
                    const uint64_t bm = __ballot(cand);
                    if (cand) {
                        const int m = M + lanes_below(bm);
                        if (k32path) k32[m] = ((uint32_t)cnt[p] << 16) | (0xFFFFu - (uint32_t)p);
                        else d.srt[m] = ((uint64_t)(uint32_t)cnt[p] << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)p);
                    }
                    M += __popcll(bm);
                }
                for (int p = t; p < S; p += 64) d.proc[p] = 0;
                wsync();
                mark(9 + 4 * iter);
                if (k32path) {
                    // rank = #{larger key}: 4 candidates per lane against every candidate (LDS broadcast reads,
                    // 8 in flight; a bitonic sort in LDS measured slower: 36 dependent stages for M ~ 200)
                    for (int i0 = 0; i0 < M; i0 += 256) {
                        uint32_t v[4];
                        int r[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int i = i0 + 64 * u + t;
                            v[u] = i < M ? k32[i] : 0u;
                            r[u] = 0;
                        }
                        int j = 0;
                        for (; j + 8 <= M; j += 8) {
                            uint32_t w[8];
#pragma unroll
                            for (int e = 0; e < 8; ++e) w[e] = k32[j + e];
#pragma unroll
                            for (int e = 0; e < 8; ++e)
#pragma unroll
                                for (int u = 0; u < 4; ++u) r[u] += w[e] > v[u];
                        }
                        for (; j < M; ++j) {
                            const uint32_t w = k32[j];
#pragma unroll
                            for (int u = 0; u < 4; ++u) r[u] += w > v[u];
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (i0 + 64 * u + t < M) d.sp[r[u]] = (int)(0xFFFFu - (v[u] & 0xFFFFu));
                    }
                } else {
                    // rank = #{larger key}: 4 candidates per lane against every candidate (broadcast reads)
                    for (int i0 = 0; i0 < M; i0 += 256) {
                        uint64_t v[4];
                        int r[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int i = i0 + 64 * u + t;
                            v[u] = i < M ? d.srt[i] : 0;
                            r[u] = 0;
                        }
                        for (int j = 0; j < M; ++j) {
                            const uint64_t w = d.srt[j];
#pragma unroll
                            for (int u = 0; u < 4; ++u) r[u] += w > v[u];
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (i0 + 64 * u + t < M) d.sp[r[u]] = (int)(0xFFFFFFFFu - (uint32_t)v[u]);
                    }
                }
                wsync();
                mark(10 + 4 * iter);
                for (int j = t; j < M; j += 64) {
                    const int4 cc = child_counts(d.sp[j]);
                    const int nc = (cc.x > 0) + (cc.y > 0) + (cc.z > 0) + (cc.w > 0);
                    d.sb[j] = nc - 1;
                    d.sd[j] = nc;
                }
                wsync();
                wave_scan_lds(d.sb, M);
                int pmin = 0x7fffffff;
                for (int j = t; j < M; j += 64)
                    if (S + d.sb[j] + d.sd[j] - 1 >= N) pmin = min(pmin, j);  // :729-730 break
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) pmin = min(pmin, __shfl_xor(pmin, o, 64));
                const int P = pmin == 0x7fffffff ? M : pmin + 1;
                for (int j = t; j < M; j += 64) {
                    if (j >= P) d.sd[j] = 0;
                    else d.proc[d.sp[j]] = 1;
                }
                wsync();
                const int Cn = wave_scan_lds(d.sd, M);
                for (int p = t; p < S; p += 64) d.sa[p] = d.proc[p] == 0;
                wsync();
                const int Kk = wave_scan_lds(d.sa, S);
                for (int j = t; j < P; j += 64) {
                    const int p = d.sp[j];
                    const int4 cc = child_counts(p);
                    int c = d.sd[j];
                    const int dp = dep[p];
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (cc_at(cc, q) > 0)
                            put(Cn - 1 - c++, code[p] | ((uint32_t)q << (2 * (D - dp - 1))), cc_at(cc, q), dp + 1);
                }
                for (int p = t; p < S; p += 64)
                    if (!d.proc[p]) put(Cn + d.sa[p], code[p], cnt[p], dep[p]);
                wsync();
                const int Sn = Cn + Kk;
                if (Sn > NC) ovf = true;
                if (Sn > NC || Sn >= N || Sn == S) done = true;  // :733-734
                S = min(Sn, NC);
                C = min(Cn, NC);
                cur ^= 1;
            }
        }
        if (__ballot(ovf) && t == 0) atomicOr(overflow, 4);
        // nodes deeper than D0 of the final list, for the final map
        const uint8_t* dep = L_dep();
        int nd = 0;
        for (int p0 = 0; p0 < S; p0 += 64) {
            const int p = p0 + t;
            const bool deep = p < S && dep[p] > D0;
            const uint64_t bm = __ballot(deep);
            if (deep) d.dl[nd + lanes_below(bm)] = p;
            nd += __popcll(bm);
        }
        if (t == 0) {
            s_S = S;
            s_cur = cur;
            s_cmd = 0;
        }
        __syncthreads();  // the other waves leave their command loop
        if (t == 0) s_nd = nd;  // (they have read s_nd for their last sweep before that barrier)
    }
    __syncthreads();
    mark(60);

    // ---- 3. the first maximum-response key of every node (:740-759), list order
    const int S = s_S, nd = s_nd;
    const uint32_t* code = s_cur ? d.code1 : d.code0;
    const uint8_t* dep = s_cur ? d.dep1 : d.dep0;
    const uint64_t* flst = s_cur ? d.lst2 : lst;
    auto fcode = [&](int p) { return FLAT ? node_code(flst, p) : code[p]; };
    auto fdep = [&](int p) { return FLAT ? node_dep(flst, p) : (int)dep[p]; };
    uint32_t* best = (uint32_t*)d.sa;
    // a node of depth <= D0 covers whole bins: its best key is the maximum of their maxima
    for (int p = t; p < S; p += NT) {
        const int dp = fdep(p);
        const int lo = (int)(fcode(p) >> bsh);
        uint32_t m = 0u;
        if (dp <= D0) {
            const int w = 1 << (2 * (D0 - dp));
            if (w == 1) {
                m = d.bmax[lo];
            } else {  // w a power of 4 and lo a multiple of w: 16-byte aligned runs of 4 bins
                for (int b = lo; b < lo + w; b += 4) {
                    const uint4 q = *(const uint4*)(d.bmax + b);
                    m = max(m, max(max(q.x, q.y), max(q.z, q.w)));
                }
            }
        }
        best[p] = m;
    }
    __syncthreads();
    // nodes deeper than D0: a sweep over the keys of their bins (bin flag, then the sorted deep nodes)
    if (nd > 0) {
        for (int i = t; i < nd; i += NT) d.bins[fcode(d.dl[i]) >> bsh] = kObDeep;
        __syncthreads();
    }
    if (nd > 0) {
        if constexpr (FLAT) deep_sort_l(nd, flst);
        else deep_sort(nd, code);
        __syncthreads();
        for_cached(t, NT, std::integral_constant<int, 2>{}, [&](int kk, uint32_t v, uint32_t cd) {
            if (kk >= K || d.bins[cd >> bsh] != kObDeep) return;
            const int q = FLAT ? deep_find_l(nd, cd, flst) : deep_find(nd, code, dep, cd);
            if (q >= 0) atomicMax(&best[q], (v & 0xFF000000u) | (0xFFFFFFu - (uint32_t)kk));
        });
    }
    __syncthreads();
    for (int p = t; p < S; p += NT) {
        const uint32_t bv = best[p];
        const int k = 0xFFFFFF - (int)(bv & 0xFFFFFFu);
        if (bv != 0u && k < K) {
            out[p] = kc[k];  // the first sweep's copy of the key's slot value (no binary search over the cells)
        } else {  // a node without keys cannot occur; flag instead of reading out of range
            out[p] = 0u;
            atomicOr(overflow, 16);
        }
    }
    if (t == 0) *count_out = S;
    mark(63);
}

// ------------------------------------------------------------------------------- descriptor math
// glibc 2.35 x86-64 sinf / cosf (FMA ifunc variant; ARM optimized-routines algorithm), |x| < 120.
// glibc's two coefficient tables differ only in the sign of the cosine coefficients, so the second
// table's cosine polynomial is the negated first one (fma(a, -b, -c) == -fma(a, b, c), exactly), and the
// quadrant sign {1, -1, -1, 1}[n & 3] is a negation when bit 0 ^ bit 1 of n is set.  Everything is an
// immediate: a lane-indexed __constant__ table compiles to two dependent vector memory round trips.
namespace sc {
constexpr double hpi_inv = 0x1.45f306dc9c883p+23, hpi = 0x1.921fb54442d18p+0;
constexpr double c0 = 0x1p+0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
                 c4 = 0x1.99343027bf8c3p-16;
constexpr double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
}  // namespace sc

__device__ __forceinline__ float sc_sin_poly(double x, double x2) {
    const double x3 = x * x2, s1 = __fma_rn(x2, sc::s3, sc::s2), x5 = x2 * x3, s = __fma_rn(x3, sc::s1, x);
    return (float)__fma_rn(x5, s1, s);
}
__device__ __forceinline__ float sc_cos_poly(double x2) {
    const double x4 = x2 * x2, c1 = __fma_rn(x2, sc::c1, sc::c0), c2 = __fma_rn(x2, sc::c4, sc::c3), x6 = x2 * x4;
    const double c = __fma_rn(x4, sc::c2, c1);
    return (float)__fma_rn(x6, c2, c);
}
// n / d correctly rounded for 0 <= n <= d with d in [1, 2^24], or n = 0: the compiler's IEEE __fdiv_rn sequence
// (reciprocal, one Newton step on it, the quotient, two residual corrections) without its range scaling
// (v_div_scale, v_div_fixup), which leaves such operands unchanged
__device__ __forceinline__ float div_rn_unit(float n, float d) {
    const float r0 = __builtin_amdgcn_rcpf(d);
    const float r = __fmaf_rn(__fmaf_rn(-d, r0, 1.0f), r0, r0);
    float q = __fmul_rn(n, r);
    q = __fmaf_rn(__fmaf_rn(-d, q, n), r, q);
    return __fmaf_rn(__fmaf_rn(-d, q, n), r, q);
}

// cv::fastAtan2 of integer moments y, x (|y|, |x| < 2^24: the float conversions are exact), per lane (k_orb
// evaluates a keypoint pair at once: lanes 0..31 one keypoint, 32..63 the other).  The same IEEE float
// operations in the same order as cv::fastAtan2 on the converted floats (plain IEEE float ops, no
// contraction): (ax >= ay) == (|x| >= |y|), (x < 0) == (x_int < 0); its three branches are selects.
__device__ __forceinline__ float fast_atan2_lanes(int yi, int xi) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const int axi = xi < 0 ? -xi : xi, ayi = yi < 0 ? -yi : yi;
    const float num = (float)min(axi, ayi), den = (float)max(axi, ayi);  // xge: (ay, ax), else (ax, ay)
    const float c = div_rn_unit(num, __fadd_rn(den, (float)2.220446049250313e-16)), c2 = __fmul_rn(c, c);
    float a = __fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(__fadd_rn(__fmul_rn(p7, c2), p5), c2), p3), c2), p1), c);
    a = axi >= ayi ? a : __fsub_rn(90.f, a);
    a = xi < 0 ? __fsub_rn(180.f, a) : a;
    return yi < 0 ? __fsub_rn(360.f, a) : a;
}
// glibc sincosf for y in [0, 2 pi), per lane.  glibc evaluates the polynomials on y unreduced for y < 0.75
// (top <= 0x3f3; below top 0x397 it returns (y, 1)); there the reduction gives n = 0 and x = y, and its
// reduced branch returns the same two floats for every float in [0, 0.75) (checked exhaustively in double with
// FMA: tools/dbg/sincos_paths.c), so only the reduced branch is issued and lanes never diverge.
__device__ __forceinline__ void sincosf_glibc_lanes(float y, float* sn, float* cs) {
    double x = y;
    const double r = x * sc::hpi_inv;
    const int n = (((int)r) + 0x800000) >> 24;
    x = __fma_rn(-(double)n, sc::hpi, x);
    const double x2 = x * x;
    const double xs = ((n ^ (n >> 1)) & 1) ? -x : x;
    const float cp = ((n >> 1) & 1) ? -sc_cos_poly(x2) : sc_cos_poly(x2);
    const float sp = sc_sin_poly(xs, x2);
    *sn = (n & 1) ? cp : sp;
    *cs = (n & 1) ? sp : cp;
}

__device__ __forceinline__ int reflect101c(int p, int n) {  // reflect-101, clamped for far-out rows
    p = p < 0 ? -p : (p >= n ? 2 * n - 2 - p : p);
    return min(max(p, 0), n - 1);
}

// ------------------------------------------------------------------------------- k_orb
// IC_Angle + GaussianBlur 7x7 + steered BRIEF fused (ORBextractor.cpp:77-147, 1084-1089) for every kept
// keypoint: the blurred level is never materialised.  A BRIEF sample lies within 18.385 px of the keypoint
// (the pattern's largest radius) plus 0.71 px of rounding, so each keypoint needs the blur only on that
// disc, i.e. the 7x7 taps of 43 x 43 unblurred pixels around it; the arithmetic is OpenCV's 8U fixed point
// (SURVEY.md Appendix A.3): out = (sum_j k_j sum_i k_i I + 2^15) >> 16, k = [18,34,48,56,48,34,18].
// One wavefront per keypoint at a time, kOrbKpw consecutive keypoints of one level per wave, taken in pairs
// that share one angle evaluation (lanes 0..31 / 32..63); the next window's loads are in flight while the
// current one is computed:
//  * staging: rows cy-21 .. cy+21, columns cx-25 .. cx+22 as 12 dwords per row in LDS (byte j = column
//    cx - 25 + j, the same layout for every keypoint), lane r re-aligning row r with v_alignbyte from three
//    buffer dwordx4 + one dword loads; keypoints whose window reaches past the level (reflect-101 at the
//    w x h clone's border, as the reference blurs a clone of the level) load byte by byte;
//  * centroid on the staged unblurred bytes: the 213 dwords of the umax disc (rows 6 .. 36) from a table
//    of (signed byte weights u, v, dword), 2 signed v_dot4 each on the bytes I - 128;
//  * horizontal taps: the 189 (row pair, 4-column group) items the disc needs (a per-lane table), 10 v_dot4
//    with shifted byte weights per row, stored row-pair interleaved as u16 pairs (dword = (H[2m][c], H[2m+1][c]));
//  * BRIEF: lane j evaluates bits j + 64 i (i = 0..3); each of its 8 samples takes its vertical taps from
//    4 interleaved dwords (2 ds_read2) with 4 v_dot2 whose weights depend on the sample row's parity; one
//    ballot per 64 bits.
constexpr int kSrcRows = 43, kSrcDw = 12;
constexpr int kHPairs = 22, kHGrp = 10, kHDw = 4 * kHGrp;  // H: 22 row pairs x 40 columns (dwords)
constexpr int kOrbHItems = 3;          // horizontal items per lane (189 of 192 used)
constexpr int kOrbCSlots = 4;          // centroid slots per lane (213 of 256 used)

// v_writelane_b32 (no clang builtin in this toolchain): lane `lane` (wave-uniform) of `old` becomes the
// uniform `v`.  gfx9's constant-bus rule puts the lane select in M0, which the asm sets itself.  M0 is a
// reserved register the compiler does not preserve across inline asm; no other instruction of the kernels
// that use this reads M0 (no LDS DMA, s_sendmsg, GWS or movrel), which tests/test_build.py checks in the
// built code object.
__device__ __forceinline__ uint32_t writelane_m0(uint32_t old, uint32_t v, int lane) {
    asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(old) : "s"(v), "s"(lane) : "m0");
    return old;
}

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int NT>
__device__ void stereo_bucket_pair(const Geo& g, const StereoArgs& A, int pr, int* cnt, int* tmp);

// tab: [0, 192) horizontal items (src dword | hbuf uint4 index << 16, ~0 = none), then 256 centroid slots
// as uint4 (u byte weights, v byte weights, src dword, 0) — built by the host
// (orbfe_host.hip: orb_tables).
template <int WAVES, int kOrbKpw>
__global__ __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(5))) void k_orb(Geo g, const uint8_t* __restrict__ in, int64_t in_pitch,
                                                    const uint8_t* __restrict__ ws, const uint32_t* __restrict__ lvl_kp,
                                                    const int* __restrict__ lvl_count, orbfe_keypoint* __restrict__ out_kp,
                                                    uint8_t* __restrict__ out_desc, int* __restrict__ out_count,
                                                    const uint32_t* __restrict__ tab, int gx, StereoArgs sa, int n_bucket) {
    __shared__ float4 s_pat[256];
    __shared__ uint2 s_cw[64 * kOrbCSlots];                // centroid slot: signed byte weights (u, v)
    __shared__ uint32_t s_src[WAVES][kSrcRows * kSrcDw];  // staged unblurred window
    __shared__ uint32_t s_h[WAVES][kHPairs * kHDw];       // horizontal taps, row-pair interleaved u16
    // the first n_bucket workgroups build the stereo row buckets of pairs 0 .. n_bucket - 1 (they need the
    // octree's level keypoints only, stereo_bucket_pair): dispatched first, they run under the descriptor
    // workgroups instead of as a launch of their own after them (the host fuses only when H + 1 counters fit
    // s_h and the block is 256 threads)
    // n_lead: the bucket workgroups rounded up to a multiple of 8 (the extra ones return at once), so that the
    // descriptor workgroups' hw & 7 below is still their XCD
    const int n_lead = (n_bucket + 7) & ~7;
    if ((int)blockIdx.x < n_lead) {
        if constexpr (WAVES == 4)
            if ((int)blockIdx.x < n_bucket) stereo_bucket_pair<256>(g, sa, blockIdx.x, (int*)&s_h[0][0], (int*)&s_src[0][0]);
        return;
    }
    const int nb = (int)gridDim.x - n_lead, hw = (int)blockIdx.x - n_lead;  // 1-D grid: n_lead + gx images
    const int per = nb >> 3;
    const int lb = hw < 8 * per ? (hw & 7) * per + (hw >> 3) : hw;  // XCD-aware: runs of waves per L2
    const int img = __builtin_amdgcn_readfirstlane(lb / gx);
    const int blk = __builtin_amdgcn_readfirstlane(lb - img * gx);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int wv = __builtin_amdgcn_readfirstlane(blk * WAVES + wid);
    // the lane's centroid slots: window dword (two 16-bit halves per register), the same for
    // every keypoint
    const float4 pat_r = threadIdx.x < 256 ? ((const float4*)c_pattern)[threadIdx.x] : float4{};
    uint32_t cslot[kOrbCSlots / 2];
#pragma unroll
    for (int k = 0; k < kOrbCSlots / 2; ++k) {
        const uint4 a = ((const uint4*)(tab + 192))[lane + 64 * (2 * k)], b = ((const uint4*)(tab + 192))[lane + 64 * (2 * k + 1)];
        cslot[k] = a.z | (b.z << 16);  // window dwords; LDS byte addresses once the wave's window is known
    }
    uint2 cw_r[(64 * kOrbCSlots + 64 * WAVES - 1) / (64 * WAVES)];
#pragma unroll
    for (int k = 0; k < (64 * kOrbCSlots + 64 * WAVES - 1) / (64 * WAVES); ++k) {
        const int i = threadIdx.x + 64 * WAVES * k;
        const uint4 c = i < 64 * kOrbCSlots ? ((const uint4*)(tab + 192))[i] : uint4{};
        cw_r[k] = uint2{c.x, c.y};
    }
    uint32_t hit[kOrbHItems];  // per item: LDS byte address of its source dwords | of its H slot << 16
#pragma unroll
    for (int k = 0; k < kOrbHItems; ++k) hit[k] = tab[lane + 64 * k];
    // wave -> (level, first keypoint) from the level capacities (host constants)
    int l = 0, w0 = 0;
    {
        bool go = true;
#pragma unroll
        for (int i = 0; i + 1 < kMaxLevels; ++i) {
            const int wc = (g.lv[i].kp_cap + kOrbKpw - 1) / kOrbKpw;
            if (go && i + 1 < g.nlevels && wv >= w0 + wc) {
                w0 += wc;
                l = i + 1;
            } else {
                go = false;
            }
        }
    }
    const LevelGeo& L = g.lv[l];
    const int* cnt = lvl_count + img * g.nlevels;
    int pre[kMaxLevels + 1];
    pre[0] = 0;
#pragma unroll
    for (int i = 0; i < kMaxLevels; ++i) pre[i + 1] = pre[i] + (i < g.nlevels ? cnt[i] : 0);
    if (blk == 0 && threadIdx.x == 0) out_count[img] = pre[kMaxLevels];
    const int n_l = pre[l + 1] - pre[l];
    const int k0 = kOrbKpw * (wv - w0);
    const int nk = __builtin_amdgcn_readfirstlane(max(0, min(kOrbKpw, n_l - k0)));
    const uint32_t mykey = lane < nk ? lvl_kp[(int64_t)img * g.lvl_kp_cap + L.kp_off + k0 + lane] : 0u;
    int stride;
    const uint8_t* lvl = level_ptr(g, l, in, in_pitch, ws, img, &stride);
    uint32_t bias;
    // the level's size in SGPRs for the whole wave (a per-keypoint s_load of the kernel argument would come
    // with an s_waitcnt lgkmcnt(0) that also drains the wave's LDS traffic)
    const int Lw = __builtin_amdgcn_readfirstlane(L.w), Lh = __builtin_amdgcn_readfirstlane(L.h);
    const KeyDiv kv = key_div(L);
    const __amdgpu_buffer_rsrc_t rs = aligned_rsrc(lvl, (uint32_t)(stride * Lh), &bias);
    uint32_t* src = s_src[wid];
    uint32_t* hb = s_h[wid];
    {
        typedef __attribute__((address_space(3))) uint32_t lds_w32;
        const uint32_t src_a = (uint32_t)(uintptr_t)(lds_w32*)src, hb_a = (uint32_t)(uintptr_t)(lds_w32*)hb;
#pragma unroll
        for (int k = 0; k < kOrbHItems; ++k)
            hit[k] = (src_a + 4u * (hit[k] & 0xFFFFu)) | ((hb_a + 16u * (hit[k] >> 16)) << 16);
#pragma unroll
        for (int k = 0; k < kOrbCSlots / 2; ++k)
            cslot[k] = (src_a + 4u * (cslot[k] & 0xFFFFu)) | ((src_a + 4u * (cslot[k] >> 16)) << 16);
    }
    if (threadIdx.x < 256) s_pat[threadIdx.x] = pat_r;
#pragma unroll
    for (int k = 0; k < (64 * kOrbCSlots + 64 * WAVES - 1) / (64 * WAVES); ++k) {
        const int i = threadIdx.x + 64 * WAVES * k;
        if (i < 64 * kOrbCSlots) s_cw[i] = cw_r[k];
    }
    __syncthreads();  // tables
    uint4 rw[3];
    uint32_t rx, rsh = 0;
    auto key_of = [&](int j) { return (uint32_t)__builtin_amdgcn_readlane((int)mykey, j); };
    // columns cx - 25 .. cx + 22 inside the level: dword staging (rows past the top / bottom are reflected
    // per lane); otherwise byte loads with reflect-101 in both directions
    auto inside = [&](int cx) { return cx >= 25 && cx + 22 < Lw; };
    // lane r stages window row r (43 rows; lanes past them repeat the last row's loads and store nothing):
    // three dwordx4 + one dword from the dword at or below the row's first byte
    const int it_r = min(lane, kSrcRows - 1);
    const uint32_t it_off = (uint32_t)(it_r * stride);
    auto row_off = [&](int cy, bool rows_in) {  // byte offset from column cx - 25 of level row cy - 21
        if (rows_in) return it_off;
        const int y = reflect101c(cy - 21 + it_r, Lh);
        return (uint32_t)((y - (cy - 21)) * stride);
    };
    auto issue = [&](int cx, int cy) {
        const bool rows_in = cy >= 21 && cy + 21 < Lh;
        const uint32_t a = (uint32_t)((cy - 21) * stride + cx - 25) + bias + row_off(cy, rows_in), al = a & ~3u;
        rsh = a & 3u;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            rw[k] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, al + 16u * k, 0, 0));
        rx = __builtin_amdgcn_raw_buffer_load_b32(rs, al + 48u, 0, 0);
    };
    auto commit = [&]() {  // re-align the row by its start's misalignment: window dwords 12 r .. 12 r + 11
        if (lane < kSrcRows) {
            const uint32_t w[13] = {rw[0].x, rw[0].y, rw[0].z, rw[0].w, rw[1].x, rw[1].y, rw[1].z,
                                    rw[1].w, rw[2].x, rw[2].y, rw[2].z, rw[2].w, rx};
#pragma unroll
            for (int k = 0; k < 3; ++k)
                *(uint4*)(src + 12 * lane + 4 * k) =
                    uint4{__builtin_amdgcn_alignbyte(w[4 * k + 1], w[4 * k], rsh), __builtin_amdgcn_alignbyte(w[4 * k + 2], w[4 * k + 1], rsh),
                          __builtin_amdgcn_alignbyte(w[4 * k + 3], w[4 * k + 2], rsh), __builtin_amdgcn_alignbyte(w[4 * k + 4], w[4 * k + 3], rsh)};
        }
    };
    // reflect-101 at the level border: lane r stages window row r (its reflected level row, one offset per
    // lane) from byte loads whose reflected column is wave-uniform (SGPR soffset), 16 bytes in flight at a time
    auto stage_border = [&](int cx, int cy) {
        const uint32_t ro = (uint32_t)(reflect101c(cy - 21 + it_r, Lh) * stride) + bias;
#pragma unroll 1
        for (int q0 = 0; q0 < kSrcDw; q0 += 4) {
            uint32_t v[16];
#pragma unroll
            for (int t = 0; t < 16; ++t)
                v[t] = __builtin_amdgcn_raw_buffer_load_b8(rs, ro, (uint32_t)reflect101c(cx - 25 + 4 * q0 + t, Lw), 0);
            uint4 u;
            uint32_t* uw = (uint32_t*)&u;
#pragma unroll
            for (int q = 0; q < 4; ++q)
                uw[q] = __builtin_amdgcn_perm(v[4 * q + 1], v[4 * q], 0x0c0c0400u) |
                        __builtin_amdgcn_perm(v[4 * q + 3], v[4 * q + 2], 0x04000c0cu);
            if (lane < kSrcRows) *(uint4*)(src + kSrcDw * lane + q0) = u;
        }
    };
    int cx = 0, cy = 0;
    if (nk > 0) {
        const uint32_t k = key_of(0);
        key_xy(k, kv, cx, cy);
        if (inside(cx)) issue(cx, cy);
    }
    auto w4 = [](uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return a | (b << 8) | (c << 16) | (d << 24); };
    auto w2 = [](uint32_t a, uint32_t b) { return __builtin_bit_cast(us2, a | (b << 16)); };
    // results stay in registers until the wave's last keypoint: lane 4 j + i holds bits 64 i .. 64 i + 63 of
    // keypoint j's descriptor, lane j its keypoint record.  A store inside the loop would sit in front of
    // the next window's loads in the in-order vmcnt, and the wait for those loads then waits for the store.
    uint32_t mine_lo = 0, mine_hi = 0, kp_x = 0, kp_y = 0, kp_angle = 0, kp_resp = 0;
    // ---- stage the window whose loads are in flight (cx, cy): the wave's earlier reads of src / hb are
    //      complete (each was waited before the ballot or the LDS store that consumed it)
    auto stage = [&]() {
        wave_sync_lds();
        if (inside(cx)) commit();
#ifndef ORBFE_X_ORB_NOBORDER  // ablation (wrong bits): border keypoints keep the previous window
        else stage_border(cx, cy);
#endif
        wave_sync_lds();
    };
    auto prefetch = [&](int jn) {  // the loads of keypoint jn's window in flight from here
        const uint32_t k = key_of(jn);
        key_xy(k, kv, cx, cy);
        if (inside(cx)) issue(cx, cy);
    };
    // ---- horizontal taps of the disc's (row pair, group) items: src -> hb
    auto hpass = [&]() {
#pragma unroll
        for (int k = 0; k < kOrbHItems; ++k) {
            {  // lanes without an item run the dummy one (orb_tables)
                typedef __attribute__((address_space(3))) uint32_t lds_w32;
                const lds_w32* q = (const lds_w32*)(uintptr_t)(hit[k] & 0xFFFFu);
                uint32_t h[2][4];
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) {
                    const uint32_t d0 = q[rr * kSrcDw], d1 = q[rr * kSrcDw + 1], d2 = q[rr * kSrcDw + 2];
                    h[rr][0] = __builtin_amdgcn_udot4(d1, w4(56, 48, 34, 18),
                                                      __builtin_amdgcn_udot4(d0, w4(0, 18, 34, 48), 0u, false), false);
                    h[rr][1] = __builtin_amdgcn_udot4(
                        d2, w4(18, 0, 0, 0),
                        __builtin_amdgcn_udot4(d1, w4(48, 56, 48, 34), __builtin_amdgcn_udot4(d0, w4(0, 0, 18, 34), 0u, false),
                                               false),
                        false);
                    h[rr][2] = __builtin_amdgcn_udot4(
                        d2, w4(34, 18, 0, 0),
                        __builtin_amdgcn_udot4(d1, w4(34, 48, 56, 48), __builtin_amdgcn_udot4(d0, w4(0, 0, 0, 18), 0u, false),
                                               false),
                        false);
                    h[rr][3] = __builtin_amdgcn_udot4(d2, w4(48, 34, 18, 0),
                                                      __builtin_amdgcn_udot4(d1, w4(18, 34, 48, 56), 0u, false), false);
                }
                // (row 2p, row 2p + 1) as u16 pairs: one v_perm each (the sums are < 2^16)
                auto pk = [](uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x05040100u); };
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                *(__attribute__((address_space(3))) u32x4*)(uintptr_t)(hit[k] >> 16) =
                    u32x4{pk(h[0][0], h[1][0]), pk(h[0][1], h[1][1]), pk(h[0][2], h[1][2]), pk(h[0][3], h[1][3])};
            }
        }
    };
    // ---- intensity centroid on the unblurred disc (rows 6 .. 36 = cy - 15 .. cy + 15) of the window in src,
    //      on the bytes I - 128 (signed) with signed weights u, v (0 off the disc): the disc is symmetric,
    //      so sum(u) = sum(v) = 0 over it and sum u (I - 128) = sum u I = m_10 (and m_01) exactly; per-lane
    //      partial sums
    auto centroid = [&](int& m10, int& m01) {
        m10 = 0;
        m01 = 0;
#pragma unroll
        for (int k = 0; k < kOrbCSlots; ++k) {
            typedef __attribute__((address_space(3))) const uint32_t lds_c32;
            const uint2 cw = s_cw[lane + 64 * k];  // unused slots: weights 0
            const uint32_t ad = (k & 1) ? cslot[k >> 1] >> 16 : cslot[k >> 1] & 0xFFFFu;
            const int d = (int)(*(lds_c32*)(uintptr_t)ad ^ 0x80808080u);
            m10 = __builtin_amdgcn_sdot4(d, (int)cw.x, m10, false);
            m01 = __builtin_amdgcn_sdot4(d, (int)cw.y, m01, false);
        }
    };
    // ---- steered BRIEF of keypoint jj from hb with the vertical taps per sample: sample (row, col) is
    //      blurred row o = row + 18 (H rows o .. o + 6), column c = col + 21.  rint by the 1.5 * 2^23 trick:
    //      the f32 bits are xb = 0x4B400000 + R with R = rint(row) in [-18, 18], so the row pair m = o >> 1 =
    //      floor(R / 2) + 9 is (xb >> 1) - 0x25A00000, and the byte address of H pair (m, c) is one
    //      v_mad_u32_u24 (which reads the low 24 bits of xb >> 1, 0xA00000 + floor(R / 2)) over one
    //      v_lshl_add of the column bits; the constants fold into kc.  The 4 dwords P[m .. m + 3] hold
    //      rows 2m .. 2m + 7: for even o the taps are their low / high halves in order, for odd o every
    //      tap sits one u16 higher, so the data is shifted by 16 * (R & 1) bits (v_alignbit takes bits
    //      4:0 of xb << 4) and the weights stay fixed.  The last dword's high half has weight 0.
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    const uint32_t kc = (uint32_t)(uintptr_t)(lds_u32*)hb + (uint32_t)(4 * (9 * kHDw + 21)) -
                        (uint32_t)(4 * kHDw) * 0xA00000u - (__float_as_uint(12582912.0f) << 2);
    auto brief = [&](float a, float b, int jj) {
#pragma unroll 1
        for (int i = 0; i < 4; ++i) {
            const float4 pt = s_pat[lane + 64 * i];
            uint32_t v2[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const float px = e ? pt.z : pt.x, py = e ? pt.w : pt.y;
                const df2 mm = (df2){py, py} * (df2){a, -b};
                const df2 rc = __builtin_elementwise_fma((df2){px, px}, (df2){b, a}, mm) + (df2){12582912.0f, 12582912.0f};
                const uint32_t xb = __float_as_uint(rc.x), yb = __float_as_uint(rc.y);
                // v_mad_u32_u24 over a v_lshl_add (the compiler's v_mul_u32_u24 + v_lshlrev + v_add3 is one more)
                static_assert(4 * kHDw == 0xA0, "H row-pair stride of the v_mad_u32_u24 operand");
                uint32_t addr;
                asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(addr) : "v"(xb >> 1), "s"(0xA0u), "v"((yb << 2) + kc));
                lds_u32* p = (lds_u32*)(uintptr_t)addr;
#ifdef ORBFE_X_ORB_PREBLURRED
                // ablation (wrong bits; VERDICT r5 item 6's bound): a sample read as ONE byte of a window that
                // would already be blurred (a blurred pyramid level) instead of the 7 vertical taps
                v2[e] = *(const __attribute__((address_space(3))) uint8_t*)(uintptr_t)addr;
                continue;
#endif
                const uint32_t p0 = p[0], p1 = p[kHDw], p2 = p[2 * kHDw], p3 = p[3 * kHDw];
                const uint32_t sh = xb << 4;
                uint32_t s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_alignbit(p1, p0, sh)), w2(18, 34), 32768u, false);
                s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_alignbit(p2, p1, sh)), w2(48, 56), s, false);
                s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, __builtin_amdgcn_alignbit(p3, p2, sh)), w2(48, 34), s, false);
                s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, p3 >> (sh & 31u)), w2(18, 0), s, false);
                v2[e] = s >> 16;
            }
            const uint64_t bb = __ballot(v2[0] < v2[1]);  // one SDWA compare of the high halves
            // lane 4 jj + i keeps this ballot: two v_writelane (a select chain or a store per iteration measured
            // 3-5 % slower in round 2)
            mine_lo = writelane_m0(mine_lo, (uint32_t)bb, 4 * jj + i);
            mine_hi = writelane_m0(mine_hi, (uint32_t)(bb >> 32), 4 * jj + i);
        }
    };
    auto record = [&](int jj, int kx, int ky, float angle, uint32_t key) {
        if (lane == jj) {
            kp_x = __float_as_uint(l ? __fmul_rn((float)kx, L.scale) : (float)kx);
            kp_y = __float_as_uint(l ? __fmul_rn((float)ky, L.scale) : (float)ky);
            kp_angle = __float_as_uint(angle);
            kp_resp = __float_as_uint((float)(int)(key >> 24));
        }
    };
    // Keypoints in pairs (A = j, B = j + 1), so that one angle chain (fastAtan2 + sincosf, ~55 instructions
    // that every lane would otherwise issue for one keypoint) serves two: lanes 0..31 evaluate A's, lanes
    // 32..63 B's.  With one src and one hb buffer per wave the order is: stage A, H(A) -> hb, centroid A;
    // stage B into src (A's src reads are done), centroid B; angles; BRIEF A; H(B) -> hb; BRIEF B.  The next
    // window's loads are in flight from the previous stage on.
    for (int j = 0; j < nk; j += 2) {
        const bool has_b = j + 1 < nk;
        const uint32_t keyA = key_of(j);
        stage();
        const int ax = cx, ay = cy;
        if (has_b) prefetch(j + 1);
#ifndef ORBFE_X_ORB_PREBLURRED  // (the ablation: no horizontal pass either)
        hpass();
#endif
        int m10a, m01a, m10b = 0, m01b = 0;
        centroid(m10a, m01a);
        int bx = 0, by = 0;
        uint32_t keyB = 0;
        if (has_b) {
            keyB = key_of(j + 1);
            stage();
            bx = cx;
            by = cy;
            if (j + 2 < nk) prefetch(j + 2);
            centroid(m10b, m01b);
        }
        wave_sum2(m10a, m01a);
        if (has_b) wave_sum2(m10b, m01b);
        const bool lo = lane < 32;
        const float ang = fast_atan2_lanes(lo ? m01a : m01b, lo ? m10a : m10b);
        float sv, cv;
        sincosf_glibc_lanes(__fmul_rn(ang, (float)(M_PI / 180.f)), &sv, &cv);
        const float angA = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ang), 0));
        const float aA = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv), 0));
        const float bA = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv), 0));
        const float angB = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ang), 32));
        const float aB = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cv), 32));
        const float bB = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sv), 32));
        wave_sync_lds();  // hb complete
        brief(aA, bA, j);
        record(j, ax, ay, angA, keyA);
        if (has_b) {
            wave_sync_lds();  // BRIEF A's hb reads are complete (waited before its ballots)
#ifndef ORBFE_X_ORB_PREBLURRED
            hpass();
#endif
            wave_sync_lds();  // hb complete
            brief(aB, bB, j + 1);
            record(j + 1, bx, by, angB, keyB);
        }
    }
    const int64_t o0 = (int64_t)img * g.kp_cap + pre[l] + k0;  // the wave's first output slot
    if (lane < 4 * nk) *(uint2*)(out_desc + o0 * 32 + 8 * lane) = uint2{mine_lo, mine_hi};
    if (lane < nk) {
        orbfe_keypoint kp;
        kp.x = __uint_as_float(kp_x);
        kp.y = __uint_as_float(kp_y);
        kp.size = L.size;
        kp.angle = __uint_as_float(kp_angle);
        kp.response = __uint_as_float(kp_resp);
        kp.octave = l;
        out_kp[o0 + lane] = kp;
    }
}

// ------------------------------------------------------------------------------- k_undistort
// cv::undistortPoints(pts, K, D, R = noArray(), P = K) (OpenCV 4.x cvUndistortPointsInternal), the call of
// Frame.undistort_keypoints (Frame.py:306) and Tracking.compute_image_bounds (Tracking.py:132): in double,
// x0 = (u - cx) / fx, y0 = (v - cy) / fy, then 5 fixed-point iterations (TermCriteria(COUNT, 5, 0.01))
//   r2 = x^2 + y^2, icdist = 1 / (1 + ((k3 r2 + k2) r2 + k1) r2)   (k4..k6 = 0: 4- or 5-coefficient models)
//   dx = 2 p1 x y + p2 (r2 + 2 x^2), dy = p1 (r2 + 2 y^2) + 2 p2 x y, x = (x0 - dx) icdist, y = (y0 - dy) icdist
// (a negative icdist stops at the normalised input, as OpenCV >= 4.2 does), then P = K back to pixels, stored
// as float.  One thread per point; no FMA contraction (built with -ffp-contract=off).
__global__ __launch_bounds__(256) void k_undistort(const float* __restrict__ xy_in, int n, int stride_in,
                                                   float* __restrict__ xy_out, UndistortArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double u = xy_in[(int64_t)i * stride_in], v = xy_in[(int64_t)i * stride_in + 1];
    const double ifx = 1. / a.fx, ify = 1. / a.fy;
    const double x0 = (u - a.cx) * ifx, y0 = (v - a.cy) * ify;
    double x = x0, y = y0;
    for (int it = 0; it < 5; ++it) {
        const double r2 = x * x + y * y;
        const double icdist = 1. / (1. + ((a.k3 * r2 + a.k2) * r2 + a.k1) * r2);
        if (icdist < 0) {
            x = x0;
            y = y0;
            break;
        }
        const double dx = 2 * a.p1 * x * y + a.p2 * (r2 + 2 * x * x);
        const double dy = a.p1 * (r2 + 2 * y * y) + 2 * a.p2 * x * y;
        x = (x0 - dx) * icdist;
        y = (y0 - dy) * icdist;
    }
    xy_out[2 * (int64_t)i] = (float)(x * a.fx + a.cx);
    xy_out[2 * (int64_t)i + 1] = (float)(y * a.fy + a.cy);
}

hipError_t launch_undistort(const float* xy_in, int n, int stride_in, float* xy_out, const UndistortArgs& a,
                            hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, s, xy_in, n, stride_in, xy_out, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------- k_shear
// GetImagePyramid as the reference returns it (orb_extractor.cpp:30): the Mat -> ndarray caster ignores
// Mat::step (opencv_type_casters.h:232-239), so row r of level l's (h, w) array is bytes
// [19 (w + 38) + 19 + r w, + w) of the 19-px reflect-101 padded level buffer (ORBextractor.cpp:1112-1128).
// One thread per 4 output bytes of all levels of an image (dword stores; a level's tail bytes singly;
// every level's region starts 4-byte aligned).
__global__ __launch_bounds__(256) void k_shear(Geo g, const uint8_t* __restrict__ in, int64_t in_pitch,
                                               const uint8_t* __restrict__ ws, uint8_t* __restrict__ out) {
    const int img = blockIdx.y;
    const int64_t i0 = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x);
    if (i0 >= g.shear_bytes) return;
    int l = 0;
    while (l + 1 < g.nlevels && i0 >= g.lv[l + 1].shear_off) ++l;
    const LevelGeo& L = g.lv[l];
    int stride;
    const uint8_t* lvl = level_ptr(g, l, in, in_pitch, ws, img, &stride);
    const int pw = L.w + 2 * kEdge;
    const int64_t i = i0 - L.shear_off, n = (int64_t)L.w * L.h;
    uint8_t* o = out + (int64_t)img * g.shear_bytes + i0;
    uint32_t v = 0;
    for (int b = 0; b < 4 && i + b < n; ++b) {
        const int64_t f = (int64_t)kEdge * pw + kEdge + i + b;
        const int pr = (int)(f / pw), pc = (int)(f - (int64_t)pr * pw);
        const uint8_t px = lvl[(int64_t)reflect101_iter(pr - kEdge, L.h) * stride + reflect101_iter(pc - kEdge, L.w)];
        v |= (uint32_t)px << (8 * b);
        if (i + 4 > n) o[b] = px;  // the level's last bytes (its region is padded to 4 bytes)
    }
    if (i + 4 <= n) *(uint32_t*)o = v;  // levels start at 4-byte aligned offsets (host: shear_off)
}

// ------------------------------------------------------------------------------- k_stereo
__device__ __forceinline__ double py_round(double v) { return rint(v); }  // Python round(): half to even

// Row buckets of the right keypoints (Frame.py:170-179): right keypoint iR is listed in every row of
// [floor(y - 2s), ceil(y + 2s)] (double arithmetic, s = scale of its octave).  One workgroup per pair:
// LDS histogram -> block scan -> fill.  The order inside a bucket is irrelevant: k_stereo reduces
// (distance, iR) lexicographically, which is the reference's first minimum in ascending iR.
// Also writes the compact (x, octave) record of every right keypoint.  The right keypoints are read from the
// octree's level keypoints (lvl_kp, lvl_count: x | y << 12 | score << 24 in level pixels), with the
// coordinates k_orb will write (ORBextractor.cpp:1094-1100: x = f32(level x) * scale[l] for l > 0) and the
// index iR = the level-major position — so the buckets need the octree only, and the frame and batch paths
// build them inside k_orb's launch (extra workgroups, stereo_bucket_pair) instead of after it.
// cnt: H + 1 ints of LDS, tmp: 257 + 5 kMaxLevels + 1 ints.
template <int NT>
__device__ void stereo_bucket_pair(const Geo& g, const StereoArgs& A, int pr, int* cnt, int* tmp) {
    const int t = threadIdx.x;
    const int H = g.H;
    const uint32_t* lk = A.lkpR + pr * A.lkp_stride;
    const int* lc = A.lcntR + pr * A.lcnt_stride;
    int* off = A.bucket_off + (int64_t)pr * (H + 1);
    uint16_t* idx = A.bucket_idx + (int64_t)pr * A.bucket_cap;
    float2* rinfo = A.rinfo + pr * A.out_stride;
    int* scan_tmp = tmp;
    float* s_scale = (float*)(tmp + 257);     // per-octave scales (a lane-indexed kernel-argument read would be
    int* s_pre = tmp + 257 + kMaxLevels;     // a vector memory load); first right keypoint of every level
    uint32_t* s_kd = (uint32_t*)(tmp + 257 + 2 * kMaxLevels + 1);  // every level's key divisor (w, mag, sh)
    if (t < kMaxLevels) {
        s_scale[t] = g.scale[t];
        s_kd[3 * t] = (uint32_t)g.lv[t].w;
        s_kd[3 * t + 1] = g.lv[t].kmag;
        s_kd[3 * t + 2] = (uint32_t)g.lv[t].ksh;
    }
    if (t == 0) {
        int p0 = 0;
        for (int l = 0; l < kMaxLevels; ++l) {
            s_pre[l] = p0;
            p0 += l < g.nlevels ? lc[l] : 0;
        }
        s_pre[kMaxLevels] = p0;
    }
    for (int i = t; i <= H; i += NT) cnt[i] = 0;
    __syncthreads();
    const int nR = s_pre[kMaxLevels];
    // right keypoint i: its octave, y (as k_orb computes it) and x
    auto right_kp = [&](int i, int& l, float& x, float& y) {
        l = 0;
#pragma unroll
        for (int j = 1; j < kMaxLevels; ++j) l += j < g.nlevels && s_pre[j] <= i;
        const uint32_t key = lk[g.lv[l].kp_off + (i - s_pre[l])];
        int xi, yi;
        key_xy(key, KeyDiv{s_kd[3 * l], s_kd[3 * l + 1], s_kd[3 * l + 2]}, xi, yi);
        const float xl = (float)xi, yl = (float)yi;
        x = l ? __fmul_rn(xl, s_scale[l]) : xl;
        y = l ? __fmul_rn(yl, s_scale[l]) : yl;
    };
    for (int i = t; i < nR; i += NT) {
        int l;
        float x, y;
        right_kp(i, l, x, y);
        rinfo[i] = make_float2(x, __int_as_float(l));
        const double r = 2.0 * (double)s_scale[l];
        const int lo = max((int)floor((double)y - r), 0), hi = min((int)ceil((double)y + r), H - 1);
        for (int yy = lo; yy <= hi; ++yy) atomicAdd(&cnt[yy], 1);
    }
    __syncthreads();
    const int total = block_excl_scan(cnt, H, scan_tmp);
    if (t == 0) cnt[H] = total;
    __syncthreads();
    for (int i = t; i <= H; i += NT) off[i] = cnt[i];
    __syncthreads();
    for (int i = t; i < nR; i += NT) {
        int l;
        float x, y;
        right_kp(i, l, x, y);
        const double r = 2.0 * (double)s_scale[l];
        const int lo = max((int)floor((double)y - r), 0), hi = min((int)ceil((double)y + r), H - 1);
        for (int yy = lo; yy <= hi; ++yy) {
            const int pos = atomicAdd(&cnt[yy], 1);
            if (pos < A.bucket_cap) idx[pos] = (uint16_t)i;
        }
    }
}

// The buckets as a kernel of their own (the separate extract / stereo calls, orbfe_stereo_match).  NT = 1 024
// threads for small batches: one latency chain per pair (load, count, scan, fill); 256 for large ones.
template <int NT>
__global__ __launch_bounds__(NT) void k_stereo_bucket(Geo g, StereoArgs A) {
    extern __shared__ __attribute__((aligned(16))) int cnt[];  // H + 1 counters
    __shared__ int tmp[257 + 5 * kMaxLevels + 1];
    stereo_bucket_pair<NT>(g, A, blockIdx.x, cnt, tmp);
}

// Four left keypoints per wavefront, 16 lanes each (Frame.py:186-278); row q = lane >> 4 of the wave.
//  search: the row bucket of int(vL); gates |octR - octL| <= 1 and uL - maxD <= uR <= uL; Hamming
//          distance by 8 popcounts; (distance, iR) lexicographic minimum as one u32 (distance << 16 | iR)
//          reduced by DPP over the 16-lane row; accept if < 75 (TH_HIGH start 100,
//          thOrbDist = (TH_HIGH + TH_LOW) / 2).
//  refine: the 11 x 11 left patch and the 11 x 21 right strip of the *sheared* pyramid views are staged
//          in LDS one row per lane (one index division per row: consecutive sheared pixels advance
//          linearly and wrap at most once), 11 shifts x 11 rows of SAD sums, first minimum, parabola and
//          depth in IEEE float32 like the NumPy-2 chain of the reference.
__device__ __forceinline__ uint32_t row16_min(uint32_t v) {
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
    v = min(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
    return v;
}

// Padded (row, column) of pixel (r, c0) of a level's sheared view: the view's row r starts r * w bytes after
// its first pixel in the (w + 2 kEdge)-wide reflect-101 padded level (one index division per row; consecutive
// pixels advance linearly and wrap at most once inside a window row).
__device__ __forceinline__ void sheared_pos(int w, int r, int c0, int& pr, int& pc) {
    const int pw = w + 2 * kEdge;
    const int f = kEdge * pw + kEdge + r * w + c0;
    pr = f / pw;
    pc = f - pr * pw;
}

// n consecutive pixels (row r, columns c0 ..) of the sheared view as NDW dwords (byte j of the run = byte j % 4 of
// w[j / 4]; n + 3 <= 4 NDW: the left patch's 11 bytes in 4 dwords, the right strip's 21 in 6), when the run
// lies inside the level (returns false otherwise: a border row, whose bytes k_stereo gathers lane-parallel).
// The loads are one dwordx4 (+ one dwordx2): 2 memory instructions per row instead of 6 dword loads (VERDICT r5
// item 4; partially out-of-range dwords read 0 per dword, the loads are not merged past it).
// rs: a wave-uniform resource over the buffer holding the level (the pair's input image or its workspace),
// bias its base misalignment, lvl_off the level's byte offset in it (per lane): the loads need no
// per-lane resource (a per-lane one makes the compiler waterfall every load over the wave's distinct
// resources).  Bytes of the 24 past the run are whatever follows it in the buffer (0 past its end);
// k_stereo masks them.
template <int NDW>
__device__ __forceinline__ bool sheared_words(__amdgpu_buffer_rsrc_t rs, uint32_t bias, uint32_t lvl_off, int stride,
                                              int w, int h, int r, int c0, int n, uint32_t (&wd)[NDW]) {
    static_assert(NDW == 4 || NDW == 6, "4 or 6 dwords");
    int pr, pc;
    sheared_pos(w, r, c0, pr, pc);
    if (!(pr >= kEdge && pr < kEdge + h && pc >= kEdge && pc + n <= kEdge + w)) return false;
    const uint32_t off = bias + lvl_off + (uint32_t)((pr - kEdge) * stride + (pc - kEdge));
    const uint32_t sh = off & 3u, al = off - sh;
    uint32_t d[NDW + 1];
    const uint4 q = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, al, 0, 0));
    d[0] = q.x;
    d[1] = q.y;
    d[2] = q.z;
    d[3] = q.w;
    if constexpr (NDW == 6) {
        const uint2 t = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(rs, al + 16u, 0, 0));
        d[4] = t.x;
        d[5] = t.y;
    }
    d[NDW] = 0;
#pragma unroll
    for (int k = 0; k < NDW; ++k) wd[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
    return true;
}

__global__ __launch_bounds__(256) void k_stereo(Geo g, StereoArgs A) {
    __shared__ int sad[16][11];
    // the 11 x 11 left and 11 x 21 right windows as u16 pixel + 512: left columns (2k, 2k + 1) per dword,
    // right columns (2k, 2k + 1) and (2k + 1, 2k + 2) per dword (both alignments of a shift's window)
    __shared__ uint32_t sP[16][11][6];
    __shared__ uint32_t sE[16][11][11];
    __shared__ uint32_t sO[16][11][10];
    // per-octave geometry (scale, inverse scale, w, h, pitch, ws_off) in LDS: indexed by a keypoint's octave
    // the kernel argument would be read with vector memory loads, two dependent round trips in the refine
    __shared__ float s_sc[kMaxLevels], s_isc[kMaxLevels];
    __shared__ int s_w[kMaxLevels], s_h[kMaxLevels], s_pitch[kMaxLevels];
    __shared__ int64_t s_wsoff[kMaxLevels];
    if (threadIdx.x < kMaxLevels) {
        const int i = threadIdx.x;
        s_sc[i] = g.scale[i];
        s_isc[i] = g.inv_scale[i];
        s_w[i] = g.lv[i].w;
        s_h[i] = g.lv[i].h;
        s_pitch[i] = g.lv[i].pitch;
        s_wsoff[i] = g.lv[i].ws_off;
    }
    __syncthreads();
    int bx, pr;
    xcd_block(bx, pr);  // a pair's blocks read the same pyramids, descriptors and buckets: one L2
    const int lane = threadIdx.x & 63, sl = lane & 15;
    const int kq = threadIdx.x >> 4;  // keypoint of this 16-lane group inside the block
    const int iL = bx * 16 + kq;
    const int nL = A.countL[pr * A.cnt_stride];
    const bool active = iL < nL;
    const orbfe_keypoint* KL = A.kpsL + pr * A.kp_stride;
    const uint8_t* DL = A.descL + pr * A.kp_stride * 32;
    const uint8_t* DR = A.descR + pr * A.kp_stride * 32;
    const float2* rinfo = A.rinfo + pr * A.out_stride;
    // the pair's two input images and two workspaces (levels >= 1) as wave-uniform buffer resources
    const uint8_t* lvl0L = A.lvl0L + pr * A.lvl0_stride;
    const uint8_t* lvl0R = A.lvl0R + pr * A.lvl0_stride;
    const uint8_t* wsL = A.wsL + pr * A.ws_stride;
    const uint8_t* wsR = A.wsR + pr * A.ws_stride;
    uint32_t bL0, bR0, bLW, bRW;
    const uint32_t img_bytes = (uint32_t)g.W * (uint32_t)g.H;
    const __amdgpu_buffer_rsrc_t rsL0 = aligned_rsrc(lvl0L, img_bytes, &bL0), rsR0 = aligned_rsrc(lvl0R, img_bytes, &bR0);
    const __amdgpu_buffer_rsrc_t rsLW = aligned_rsrc(wsL, (uint32_t)g.ws_bytes, &bLW),
                                 rsRW = aligned_rsrc(wsR, (uint32_t)g.ws_bytes, &bRW);
    if (sl < 11) sad[kq][sl] = 0;
    uint32_t key = 0xFFFFFFFFu;  // (distance << 16) | iR
    float kx = 0.f;              // x of this lane's best right keypoint (rinfo: the x k_orb writes to KR)
    // the left record is read before the count is known (iL < kp_cap: inside the array), so the two
    // loads overlap
    orbfe_keypoint kl = KL[iL];
    if (!active) kl = orbfe_keypoint{};
    if (active) {
        const int row = min((int)(double)kl.y, g.H - 1);
        const int* off = A.bucket_off + (int64_t)pr * (g.H + 1);
        const uint16_t* bidxs = A.bucket_idx + (int64_t)pr * A.bucket_cap;
        const int b = off[row], e = min(off[row + 1], A.bucket_cap);
        const float minU = __fsub_rn(kl.x, A.maxD);
        const uint4* dl4 = (const uint4*)(DL + (int64_t)iL * 32);
        const uint4 a0 = dl4[0], a1 = dl4[1];
        // kStU candidates per lane and step: all bucket reads, then all (x, octave) records and
        // descriptors (read whether or not the gates pass) are in flight together — two dependent round
        // trips per step instead of two per candidate
        constexpr int kStU = 2;
        // the next step's bucket slots are read with this step's records (one dependent round trip less per
        // further step of a long bucket)
        int nx[kStU];
#pragma unroll
        for (int j = 0; j < kStU; ++j) nx[j] = b + sl + 16 * j < e ? (int)bidxs[b + sl + 16 * j] : -1;
#ifdef ORBFE_X_ST_NOSEARCH  // ablation (wrong results): no candidate loop, every keypoint matches right keypoint 0
        key = 0u;
        for (int k0 = e; k0 < e; k0 += 16 * kStU) {
#else
        for (int k0 = b + sl; k0 < e; k0 += 16 * kStU) {
#endif
            int iR[kStU];
#pragma unroll
            for (int j = 0; j < kStU; ++j) iR[j] = nx[j];
#pragma unroll
            for (int j = 0; j < kStU; ++j) {
                const int kn = k0 + 16 * (kStU + j);
                nx[j] = kn < e ? (int)bidxs[kn] : -1;
            }
            float2 ri[kStU];
            uint4 b0[kStU], b1[kStU];
#pragma unroll
            for (int j = 0; j < kStU; ++j) {
                const int r = max(iR[j], 0);
                ri[j] = rinfo[r];
                const uint4* dr4 = (const uint4*)(DR + (int64_t)r * 32);
                b0[j] = dr4[0];
                b1[j] = dr4[1];
            }
#pragma unroll
            for (int j = 0; j < kStU; ++j) {
                const int oct = __float_as_int(ri[j].y);
                const bool ok = iR[j] >= 0 && oct >= kl.octave - 1 && oct <= kl.octave + 1 && minU <= ri[j].x &&
                                (double)ri[j].x <= (double)kl.x;
                const uint32_t dist = __popc(a0.x ^ b0[j].x) + __popc(a0.y ^ b0[j].y) + __popc(a0.z ^ b0[j].z) +
                                      __popc(a0.w ^ b0[j].w) + __popc(a1.x ^ b1[j].x) + __popc(a1.y ^ b1[j].y) +
                                      __popc(a1.z ^ b1[j].z) + __popc(a1.w ^ b1[j].w);
                if (ok) {
                    const uint32_t c = (dist << 16) | (uint32_t)iR[j];
                    if (c < key) {
                        key = c;
                        kx = ri[j].x;
                    }
                }
            }
        }
    }
    const uint32_t mine = key;
    key = row16_min(key);
    // the winner's x from the lane that holds it (keys are unique: a right keypoint is listed once per row
    // bucket) instead of a KR[bidx] load after the search: one dependent global round trip less per wave
    const uint64_t holds = __ballot(mine == key);
    const uint64_t grp_holds = (holds >> (lane & 48)) & 0xFFFFull;
    const float uR0w = __shfl(kx, grp_holds ? (lane & 48) + __builtin_ctzll(grp_holds) : lane, 64);
    const int best = (int)(key >> 16), bidx = (int)(key & 0xFFFFu);
    int status = 0;
    float uR = -1.f, depth = -1.f;
    const bool refine = active && best < 75;  // TH_HIGH start, thOrbDist = 75 (:166, :203, :222)
    int scaleduR0 = 0;
    bool do_sad = false;
    // a window row that reaches the level's reflected border (or wraps into the next padded row): its padded
    // (row, column) start, for the lane-parallel gather below
    bool bdl = false, bdr = false;
    int wrow = 0, c0l = 0, c0r = 0;  // this lane's window row and the two windows' first columns
    if (refine) {
        const int oct = kl.octave;
        const double isf = (double)s_isc[oct];
        const float uR0 = uR0w;  // == KR[bidx].x
        const int scaleduL = (int)py_round((double)kl.x * isf);
        const int scaledvL = (int)py_round((double)kl.y * isf);
        scaleduR0 = (int)py_round((double)uR0 * isf);
        const int lw = s_w[oct], lh = s_h[oct];
        const int lstride = oct == 0 ? g.W : s_pitch[oct];
        // iniu < 0 or endu >= cols (:240-243); the slices stay inside the level otherwise
        do_sad = !(scaleduR0 < 0 || scaleduR0 + 11 >= lw) && scaledvL - 5 >= 0 && scaledvL + 6 <= lh &&
                 scaleduL - 5 >= 0 && scaleduL + 6 <= lw && scaleduR0 - 10 >= 0;
#ifdef ORBFE_X_ST_NOSAD  // ablation (wrong results): no window staging, SAD or parabola
        do_sad = false;
#endif
        if (do_sad && sl < 11) {  // lane sl stages window row sl
            uint32_t wl[4], wr[6];
            wrow = scaledvL - 5 + sl;
            c0l = scaleduL - 5;
            c0r = scaleduR0 - 10;
            // one pass per distinct octave among the active lanes (nearly always one), each with wave-uniform
            // resources: a resource selected per lane makes the compiler waterfall every window load
            for (;;) {
                const int ou = __builtin_amdgcn_readfirstlane(oct);
                if (oct == ou) {
                    const bool z = ou == 0;
                    const uint32_t lo = z ? 0u : (uint32_t)s_wsoff[oct];
                    uint32_t bl, br;
                    const __amdgpu_buffer_rsrc_t rl = aligned_rsrc(z ? lvl0L : wsL, z ? img_bytes : (uint32_t)g.ws_bytes, &bl);
                    const __amdgpu_buffer_rsrc_t rr = aligned_rsrc(z ? lvl0R : wsR, z ? img_bytes : (uint32_t)g.ws_bytes, &br);
                    bdl = !sheared_words(rl, bl, lo, lstride, lw, lh, wrow, c0l, 11, wl);
                    bdr = !sheared_words(rr, br, lo, lstride, lw, lh, wrow, c0r, 21, wr);
                    break;
                }
            }
            constexpr uint32_t k512 = 0x02000200u;
            // bytes (b, b + 1) of a dword pair as two u16 (0x0c selects a zero byte)
            auto lo2 = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c010c00u); };
            auto hi2 = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c030c02u); };
            auto mid2 = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c020c01u); };
            auto cross2 = [](uint32_t x, uint32_t nx) { return __builtin_amdgcn_perm(nx, x, 0x0c040c03u); };
            auto add = [](uint32_t a, uint32_t b) {
                return __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, a) + __builtin_bit_cast(us2, b));
            };
            if (!bdl) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    sP[kq][sl][2 * k] = add(lo2(wl[k]), k512);
                    sP[kq][sl][2 * k + 1] = add(hi2(wl[k]), k512);
                }
            }
            if (!bdr) {
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    if (2 * k < 11) sE[kq][sl][2 * k] = add(lo2(wr[k]), k512);
                    if (2 * k + 1 < 11) sE[kq][sl][2 * k + 1] = add(hi2(wr[k]), k512);
                    if (2 * k < 10) sO[kq][sl][2 * k] = add(mid2(wr[k]), k512);
                    if (2 * k + 1 < 10) sO[kq][sl][2 * k + 1] = add(cross2(wr[k], k + 1 < 6 ? wr[k + 1] : 0u), k512);
                }
            }
        }
    }
    // Border rows (reflect-101 bytes of the padded level, or a run wrapping into the next padded row): 4-14 % of
    // the window rows on KITTI levels, but in most refining waves.  Up to three rows per pass, one per 21-lane
    // slot of the wave (lane 21 k + j takes byte j of the pass's row k: its padded start, level and image from
    // the owning lane through ds_bpermute, the byte through a global load at its own address), each byte stored
    // as its u16 (pixel + 512) entry of the staged window; bytes past n stay unwritten (the SAD masks them).
    // A per-lane byte loop over its own row made every wave with one border row run 34 dependent-address byte
    // loads per lane (stereo 541 -> 534 us with one row per pass, this form below).
    {
        uint64_t mL = __ballot(bdl), mR = __ballot(bdr);
        const int slot = lane / 21, jb = lane - 21 * slot;  // slot 3 (lane 63) idles
        while (mL | mR) {
            int own = 0;
            bool rt = false, ok = false;
#pragma unroll
            for (int k = 0; k < 3; ++k) {  // the pass's rows, right windows first (wave-uniform)
                const bool okk = (mL | mR) != 0, rtk = mR != 0;
                const int ownk = okk ? __builtin_ctzll(rtk ? mR : mL) : 0;
                if (rtk) mR &= mR - 1;
                else mL &= mL - 1;
                if (slot == k) {
                    own = ownk;
                    rt = rtk;
                    ok = okk;
                }
            }
            const int orow = __shfl(wrow, own, 64), ocl = __shfl(c0l, own, 64), ocr = __shfl(c0r, own, 64);
            const int oct = __shfl(kl.octave, own, 64);
            if (ok && jb < (rt ? 21 : 11)) {
                const int w = s_w[oct], h = s_h[oct], pw = w + 2 * kEdge;
                const int stride = oct == 0 ? g.W : s_pitch[oct];
                int r, c;
                sheared_pos(w, orow, rt ? ocr : ocl, r, c);
                c += jb;
                if (c >= pw) {
                    c -= pw;
                    ++r;
                }
                const uint8_t* base = oct == 0 ? (rt ? lvl0R : lvl0L) : (rt ? wsR : wsL) + s_wsoff[oct];
                const uint16_t e = (uint16_t)(base[(int64_t)reflect101(r - kEdge, h) * stride + reflect101(c - kEdge, w)] + 512u);
                // the owner's group in the block
                const int gq = (int)(threadIdx.x >> 6) * 4 + (own >> 4), gs = own & 15;
                if (rt) {
                    ((uint16_t*)&sE[gq][gs][0])[jb] = e;
                    if (jb >= 1) ((uint16_t*)&sO[gq][gs][0])[jb - 1] = e;
                } else {
                    ((uint16_t*)&sP[gq][gs][0])[jb] = e;
                }
            }
        }
    }
    // sL / sR / sad are per 16-lane group, i.e. per wavefront: a wavefront barrier orders them (the
    // wavefronts of the block need not wait for each other's searches)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (do_sad && sl < 11) {
        // lane s: SAD of shift s, sum over the 11 rows of |(IL - IL[5,5]) - (IR - IR[5,5 + s])| =
        // |(IL + 512 + d) - (IR + 512)| with d = IR[5,5 + s] - IL[5,5] (the left term stays in [257, 1022]:
        // exact in u16), two columns per v_sad_u16; the 12th column of the last pair is masked to zero
        const int s = sl;
        const int lc = (int)((sP[kq][5][2] >> 16) & 0xFFFFu);  // IL[5][5] + 512
        const uint32_t rw = sE[kq][5][(s + 5) >> 1];  // columns (s + 4, s + 5) or (s + 5, s + 6)
        const int rc = (int)((s & 1) ? (rw & 0xFFFFu) : (rw >> 16));  // IR[5][5 + s] + 512
        const uint32_t d = (uint32_t)(rc - lc) & 0xFFFFu;
        const uint32_t dd = d | (d << 16);
        const int b0 = s >> 1;
        uint32_t acc = 0;
#pragma unroll
        for (int r = 0; r < 11; ++r) {
            const uint32_t* bp = (s & 1) ? &sO[kq][r][b0] : &sE[kq][r][b0];
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const uint32_t a = __builtin_bit_cast(uint32_t, __builtin_bit_cast(us2, sP[kq][r][k]) +
                                                                    __builtin_bit_cast(us2, dd));
                const uint32_t b = bp[k];
                acc = k < 5 ? __builtin_amdgcn_sad_u16(a, b, acc) : __builtin_amdgcn_sad_u16(a & 0xFFFFu, b & 0xFFFFu, acc);
            }
        }
        sad[kq][s] = (int)acc;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (do_sad && sl == 0) {
        int bi = 0, bd = sad[kq][0];
        for (int s = 1; s < 11; ++s)
            if (sad[kq][s] < bd) {
                bd = sad[kq][s];
                bi = s;
            }
        if (bi != 0 && bi != 10) {
            const int d1 = sad[kq][bi - 1], d2 = sad[kq][bi], d3 = sad[kq][bi + 1];
            const float deltaR = __fdiv_rn((float)(d1 - d3), (float)(2 * (d1 + d3 - 2 * d2)));
            if (!(deltaR < -1.f || deltaR > 1.f)) {
                const float bestuR = __fmul_rn(s_sc[kl.octave], __fadd_rn((float)(scaleduR0 + bi - 5), deltaR));
                const float disparity = __fsub_rn(kl.x, bestuR);
                if (0.f <= disparity && disparity < A.maxD) {
                    if (disparity <= 0.f) {  // Python-double substitution, recomputed on the host
                        status = 2;
                        uR = (float)((double)kl.x - 0.01);
                        depth = (float)(A.bf / 0.01);
                    } else {
                        status = 1;
                        uR = bestuR;
                        depth = __fdiv_rn(A.bf32, disparity);
                    }
                }
            }
        }
    }
    if (active && sl == 0) {
        const int64_t o = pr * A.out_stride + iL;
        A.u_right[o] = status ? uR : -1.f;
        A.depth[o] = status ? depth : -1.f;
        A.status[o] = (int8_t)status;
        A.match_r[o] = status ? bidx : -1;
    }
}

// ------------------------------------------------------------------------------- Hamming
// All-pairs distances: one thread per (a, b) pair, descriptors as 2 x uint4.
__global__ __launch_bounds__(256) void k_hamming_matrix(const uint8_t* __restrict__ a, int na, const uint8_t* __restrict__ b,
                                                        int nb, int* __restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x, i = blockIdx.y;
    if (j >= nb) return;
    const uint4* A4 = (const uint4*)(a + (int64_t)i * 32);
    const uint4* B4 = (const uint4*)(b + (int64_t)j * 32);
    const uint4 a0 = A4[0], a1 = A4[1], b0 = B4[0], b1 = B4[1];
    out[(int64_t)i * nb + j] = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                               __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// Candidate-list search: one wavefront per query; keeps the two smallest (dist, position) pairs in
// lexicographic order, which is what the sequential `dist < best ... elif dist < best2` scan of
// search_by_projection_f_p (ORBMatcher.py:258-274) leaves in best / best2.  Also writes every
// candidate distance (CSR order) for host-side control logic that depends on earlier matches.
__global__ __launch_bounds__(256) void k_hamming_search(const uint8_t* __restrict__ q, int nq, const uint8_t* __restrict__ tr,
                                                        const int* __restrict__ off, const int* __restrict__ idx,
                                                        int* __restrict__ best_d, int* __restrict__ best_i,
                                                        int* __restrict__ sec_d, int* __restrict__ sec_i,
                                                        int* __restrict__ all_d) {
    const int qi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (qi >= nq) return;
    const uint4* Q4 = (const uint4*)(q + (int64_t)qi * 32);
    const uint4 a0 = Q4[0], a1 = Q4[1];
    const int b = off[qi], e = off[qi + 1];
    int d1 = 256, p1 = 0x7fffffff, d2 = 256, p2 = 0x7fffffff;
    for (int pos = b + lane; pos < e; pos += 64) {
        const uint4* T4 = (const uint4*)(tr + (int64_t)idx[pos] * 32);
        const uint4 b0 = T4[0], b1 = T4[1];
        const int d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
                      __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
        if (all_d) all_d[pos] = d;
        if (d < d1) {
            d2 = d1; p2 = p1; d1 = d; p1 = pos;
        } else if (d < d2) {
            d2 = d; p2 = pos;
        }
    }
    // merge top-2 lists across the wave (lexicographic (dist, pos))
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const int od1 = __shfl_xor(d1, o, 64), op1 = __shfl_xor(p1, o, 64);
        const int od2 = __shfl_xor(d2, o, 64), op2 = __shfl_xor(p2, o, 64);
        int cd[4] = {d1, d2, od1, od2}, cp[4] = {p1, p2, op1, op2};
        int bd1 = 257, bp1 = 0x7fffffff, bd2 = 257, bp2 = 0x7fffffff;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const bool lt1 = cd[k] < bd1 || (cd[k] == bd1 && cp[k] < bp1);
            const bool lt2 = cd[k] < bd2 || (cd[k] == bd2 && cp[k] < bp2);
            if (lt1) { bd2 = bd1; bp2 = bp1; bd1 = cd[k]; bp1 = cp[k]; }
            else if (lt2) { bd2 = cd[k]; bp2 = cp[k]; }
        }
        d1 = bd1; p1 = bp1; d2 = bd2; p2 = bp2;
    }
    if (lane == 0) {
        best_d[qi] = p1 == 0x7fffffff ? 256 : d1;
        best_i[qi] = p1 == 0x7fffffff ? -1 : idx[p1];
        sec_d[qi] = p2 == 0x7fffffff ? 256 : d2;
        sec_i[qi] = p2 == 0x7fffffff ? -1 : idx[p2];
    }
}

// ------------------------------------------------------------------------------- launchers
hipError_t launch_resize(const Geo& g, int l, const uint8_t* in, int64_t in_pitch, uint8_t* ws, const ResizeX* xt,
                         const ResizeY* yt, int n_images, hipStream_t s, int variant, int* zero_word) {
    const LevelGeo& L = g.lv[l];  // LDS sized for this level (tables + its bands' source rows)
    dim3 grid((L.h + L.rs_rows - 1) / L.rs_rows, n_images);
    // production: k_resize_rows (profiles/r03/resize_rows_ab_r3f.log: 414 -> 394 us per 256 pairs
    // standalone, +0.8 % on the 4-handle step); variants (tools/microbench.py): 4 = the item-mapped
    // k_resize, 1 / 2 = its staging-only / compute-only ablations
    if (variant == 0 || variant == 3 || variant == 5) {
        // a level whose groups leave a last chunk of fewer than 40 (of 64) takes it in one remainder wave
        // (variant 5: never, every chunk row-uniform); at most 8 waves per row set, each walking several
        // chunks on rows wider than 2 048 px, so the block stays within __launch_bounds__(512)
        const int ngrp = (L.w + 3) / 4, rem = ngrp % 64;
        const int wg0 = (ngrp + 63) / 64;
        const int remw = (variant != 5 && ngrp >= 64 && wg0 <= 8 && rem > 0 && rem < 40) ? 1 : 0;
        const int wg = remw ? ngrp / 64 : wg0;
        const int wgl = std::min(wg, 8 - remw);
        const int sets = std::max(1, (4 - remw + wgl - 1) / wgl);  // >= 256 threads per block (the staging threads)
        const int threads = 64 * (wgl * sets + remw);
        if (threads < 256 || threads > 512) return hipErrorInvalidConfiguration;
        // MULTI: a wave walks several 64-group chunks (levels wider than 2 048 px); the one-chunk form is
        // instantiated apart (the loop around it cost 3 % on KITTI, tools/dbg/mb_ab.sh, round 4)
        auto k = wg > wgl ? k_resize_rows<true> : k_resize_rows<false>;
        hipLaunchKernelGGL(k, grid, dim3(threads), (size_t)L.rs_nsrc * L.rs_sp + 16, s, g, l, in, in_pitch, ws, xt, yt, wg,
                           remw, wgl, zero_word);
        return hipGetLastError();
    }
#ifdef ORBFE_DEV_VARIANTS
    if (L.wide) return hipErrorInvalidValue;  // the round-2 kernel gathers every pixel from the group's 8 bytes
    const size_t lds = (size_t)L.rs_ngrp * 36 + 16 * kRsRows + (size_t)L.rs_nsrc * L.rs_sp + 16;
    if (L.rs_rows != kRsRows || lds > 150 * 1024) return hipErrorInvalidValue;  // kRsRows-row bands only
    auto k = variant == 1 ? k_resize<1> : variant == 2 ? k_resize<2> : k_resize<0>;  // variant 4: k_resize<0>
    hipLaunchKernelGGL(k, grid, dim3(256), lds, s, g, l, in, in_pitch, ws, xt, yt);
    return hipGetLastError();
#else
    return hipErrorInvalidValue;  // the microbench variants exist only in ORBFE_DEV_VARIANTS builds
#endif
}

int detect_rp(const Geo& g) { return g.max_rw + 3 <= 48 ? 48 : g.max_rw + 3 <= 64 ? 64 : 96; }

size_t detect_lds_bytes(const Geo& g) {
    // ROI, the M map (pitch RP bytes), the pair queue
    return 2 * (size_t)detect_roi_elems(g, detect_rp(g)) + (size_t)detect_rp(g) * (g.max_wh + 2) + 2 * (size_t)g.fd_pq;
}

// cells per wave for a batch: 4 unless that leaves fewer than 8 waves per CU (variant 4 / 1 force 4 / 1)
int detect_cpw(const Geo& g, int n_images, int variant) {
    if (variant == 4) return 4;
    if (variant == 5) return 1;
    // 8 pairs: 39 us with one cell per wave against 47 with four (tools/microbench.py, round 4)
    return n_images < kSmallBatchImages || (int64_t)n_images * ((g.ncells + kFdCells - 1) / kFdCells) < 8 * 256
               ? kFdSmallCells
               : kFdCells;
}

template <int RP, int NS>
static void launch_detect_rp(const Geo& g, const CellGeo* cells, const uint8_t* in, int64_t in_pitch, const uint8_t* ws,
                             int* cell_count, uint32_t* slots, int n_images, hipStream_t s, int variant, int* stats) {
    const int cpw = detect_cpw(g, n_images, variant);
    const dim3 grid((g.ncells + cpw - 1) / cpw, n_images), blk(64);
#ifdef ORBFE_DEV_VARIANTS
    // variants 8 / 9: the full kernel with 6 / 12 KiB of extra (unused) LDS, to measure how detect
    // time depends on occupancy; 1 / 2 / 3: the ablations (tools/microbench.py)
    const size_t lds = detect_lds_bytes(g) + (variant == 8 ? 6144 : variant == 9 ? 12288 : 0);
    auto k = variant == 1 ? k_detect<1, RP, NS, kFdCells> : variant == 2 ? k_detect<2, RP, NS, kFdCells>
           : variant == 3 ? k_detect<3, RP, NS, kFdCells> : cpw == 1 ? k_detect<0, RP, NS, 1>
           : cpw == kFdSmallCells ? k_detect<0, RP, NS, kFdSmallCells> : k_detect<0, RP, NS, kFdCells>;
#else
    const size_t lds = detect_lds_bytes(g);
    auto k = stats ? (cpw == kFdSmallCells ? k_detect<0, RP, NS, kFdSmallCells, true> : k_detect<0, RP, NS, kFdCells, true>)  // debug counters
                   : (cpw == kFdSmallCells ? k_detect<0, RP, NS, kFdSmallCells> : k_detect<0, RP, NS, kFdCells>);
#endif
    hipLaunchKernelGGL(k, grid, blk, lds, s, g, cells, in, in_pitch, ws, cell_count, slots, stats);
}

hipError_t launch_detect(const Geo& g, const CellGeo* cells, const uint8_t* in, int64_t in_pitch, const uint8_t* ws,
                         int* cell_count, uint32_t* slots, int n_images, hipStream_t s, int variant, int* stats) {
    // ROIs of at most 48 rows (KITTI, EuRoC) stage from 12 registers, taller ones (<= 64) from 16
    const bool tall = g.max_rh > 48;
    switch (detect_rp(g)) {
        case 48:
            if (tall) launch_detect_rp<48, 16>(g, cells, in, in_pitch, ws, cell_count, slots, n_images, s, variant, stats);
            else launch_detect_rp<48, 12>(g, cells, in, in_pitch, ws, cell_count, slots, n_images, s, variant, stats);
            break;
        case 64:
            if (tall) launch_detect_rp<64, 16>(g, cells, in, in_pitch, ws, cell_count, slots, n_images, s, variant, stats);
            else launch_detect_rp<64, 12>(g, cells, in, in_pitch, ws, cell_count, slots, n_images, s, variant, stats);
            break;
        default: launch_detect_rp<96, 16>(g, cells, in, in_pitch, ws, cell_count, slots, n_images, s, variant, stats);
    }
    return hipGetLastError();
}

size_t octree_lds_bytes(const Geo& g, int maxcell) {
    const int NC = g.max_ncap;
    int pow2 = 1;
    while (pow2 < NC) pow2 <<= 1;
    return (size_t)8 * NC * 2 + 8 * pow2 + 4 * NC * 2 + 16 * NC + 8 * NC + 4 * NC * 4 + 4 * ((maxcell + 4) & ~3) +
           6 * (size_t)g.oct_keys;
}

size_t octree_bins_lds_bytes(const Geo& g, int maxcell) {
    return ob_carve(g.max_ncap, g.oct_bins_max, maxcell, g.oct_tab_max, g.oct_kblk_max, [](int, size_t) {});
}

// gfx950: up to 160 KiB of LDS per workgroup, above 64 KiB on request.  Raised (never lowered) once per
// process and kernel, when a geometry is built (orbfe_host.hip prepare_kernels): launches, which may be
// inside a graph capture, only check.
// hipFuncSetAttribute acts on the current device, so the raised limits are remembered per device
// (a process with handles on two GPUs must raise them on each).
constexpr int kMaxDevices = 64;
struct LdsAttr {
    std::vector<std::pair<const void*, int>> raised;  // kernel -> dynamic LDS limit raised on this device
    int get(const void* fn) const {
        for (const auto& e : raised)
            if (e.first == fn) return e.second;
        return 64 * 1024;
    }
    void set(const void* fn, int v) {
        for (auto& e : raised)
            if (e.first == fn) { e.second = v; return; }
        raised.emplace_back(fn, v);
    }
};
static LdsAttr g_lds[kMaxDevices];
static std::mutex g_lds_mu;

static LdsAttr* lds_attr() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return nullptr;
    return &g_lds[dev];
}

static hipError_t raise_lds(const void* fn, int bytes) {
    std::lock_guard<std::mutex> lk(g_lds_mu);
    LdsAttr* a = lds_attr();
    if (!a) return hipErrorInvalidDevice;
    if (bytes <= a->get(fn)) return hipSuccess;
    if (bytes > 160 * 1024) return hipErrorInvalidValue;
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) a->set(fn, bytes);
    return e;
}

// the limit raised on the current device for kernel fn
static int lds_limit(const void* fn) {
    std::lock_guard<std::mutex> lk(g_lds_mu);
    const LdsAttr* a = lds_attr();
    return a ? a->get(fn) : 0;
}

hipError_t prepare_resize_cascade(int lds_bytes) { return raise_lds((const void*)k_resize_cascade, lds_bytes); }

#ifndef ORBFE_OB_SMALL_NT
#define ORBFE_OB_SMALL_NT 512
#endif
// k_octree_bins threads for small batches: 512 (8 pairs: 35.5 -> 33.1 us against 1 024 — the passes run on
// <= 512 list positions, so waves 8-15 only added issue contention; level 0's key sweep is slower, but the
// kernel's critical path is a small level's careful iterations; tools/octree_profile.py, round 5)
constexpr int kObSmallNT = ORBFE_OB_SMALL_NT;
static const void* octree_bins_fn(const Geo& g, bool wide) {
    const bool reg = octree_reg_passes(g.max_ncap);
    return wide ? (reg ? (const void*)k_octree_bins<kObSmallNT, true> : (const void*)k_octree_bins<kObSmallNT, false>)
                : (reg ? (const void*)k_octree_bins<kObThreads, true> : (const void*)k_octree_bins<kObThreads, false>);
}

hipError_t prepare_octree(const Geo& g, int maxcell) {
    const size_t nb = octree_bins_lds_bytes(g, maxcell), no = octree_lds_bytes(g, maxcell);
    hipError_t e = hipSuccess;
    if (nb <= 160 * 1024) {
        if ((e = raise_lds(octree_bins_fn(g, false), (int)nb)) != hipSuccess) return e;
        if ((e = raise_lds(octree_bins_fn(g, true), (int)nb)) != hipSuccess) return e;
    }
    if (no <= 160 * 1024) e = raise_lds((const void*)k_octree, (int)no);
    return e;
}

hipError_t launch_resize_cascade(const Geo& g, const uint8_t* in, int64_t in_pitch, uint8_t* ws, const ResizeX* xt,
                                 const ResizeY* yt, const int16_t* strips, int n_strips, int off_b, int off_x,
                                 int lds_bytes, int n_images, hipStream_t s, int* zero_word, long long* prof) {
    if (g.nlevels < 2 || n_images <= 0) return hipSuccess;
    if (lds_bytes > lds_limit((const void*)k_resize_cascade)) return hipErrorInvalidConfiguration;  // prepare_resize_cascade was not run
    hipLaunchKernelGGL(k_resize_cascade, dim3(n_strips, n_images), dim3(kCasNT), (size_t)lds_bytes, s, g, in, in_pitch, ws,
                       xt, yt, strips, off_b, off_x, zero_word, prof);
    return hipGetLastError();
}

hipError_t launch_octree(const Geo& g, const CellGeo* cells, const int* cell_count, const uint32_t* slots,
                         const uint32_t* octab, uint32_t* kd, uint16_t* kn, uint32_t* lvl_kp, int* lvl_count, int* overflow,
                         int maxcell, int n_images, hipStream_t s, int variant, long long* prof) {
    if (g.oct_v == 0) {
        const size_t lds = octree_bins_lds_bytes(g, maxcell);
        // kObSmallNT threads for small batches (variant 1 / 2 force 256 / kObSmallNT, tools/microbench.py)
        const bool wide = variant == 2 || (variant != 1 && n_images < kSmallBatchImages);
        const void* fn = octree_bins_fn(g, wide);
        if ((int)lds > lds_limit(fn)) return hipErrorInvalidConfiguration;  // prepare_octree
        const bool reg = octree_reg_passes(g.max_ncap);
        auto k = wide ? (reg ? k_octree_bins<kObSmallNT, true> : k_octree_bins<kObSmallNT, false>)
                      : (reg ? k_octree_bins<kObThreads, true> : k_octree_bins<kObThreads, false>);
        hipLaunchKernelGGL(k, dim3(n_images, g.nlevels), dim3(wide ? kObSmallNT : kObThreads), lds, s, g, cells, cell_count,
                           slots, octab, lvl_kp, lvl_count, overflow, maxcell, kd, prof);
        return hipGetLastError();
    }
    const size_t lds = octree_lds_bytes(g, maxcell);
    if ((int)lds > lds_limit((const void*)k_octree)) return hipErrorInvalidConfiguration;
    hipLaunchKernelGGL(k_octree, dim3(n_images, g.nlevels), dim3(kOctThreads), lds, s, g, cells, cell_count, slots, kd, kn,
                       lvl_kp, lvl_count, overflow, maxcell, variant, prof);
    return hipGetLastError();
}

static int orb_waves(const Geo& g, int kpw) {
    int waves = 0;
    for (int l = 0; l < g.nlevels; ++l) waves += (g.lv[l].kp_cap + kpw - 1) / kpw;
    return waves;
}

template <int NW, int KPW>
static void launch_orb_nw(const Geo& g, const uint8_t* in, int64_t in_pitch, const uint8_t* ws, const uint32_t* lvl_kp,
                          const int* lvl_count, orbfe_keypoint* out_kp, uint8_t* out_desc, int* out_count, int n_images,
                          const uint32_t* tab, hipStream_t s, const StereoArgs* bucket, int n_bucket) {
    const int waves = orb_waves(g, KPW);  // most waves an image can need: KPW keypoints per wave, per level
    const int gx = (waves + NW - 1) / NW;
    const int nbk = bucket && NW == 4 ? n_bucket : 0;
    hipLaunchKernelGGL((k_orb<NW, KPW>), dim3(((nbk + 7) & ~7) + gx * n_images), dim3(64 * NW), 0, s, g, in, in_pitch, ws, lvl_kp,
                       lvl_count, out_kp, out_desc, out_count, tab, gx, bucket ? *bucket : StereoArgs{}, nbk);
}

// k_orb can carry the stereo buckets when the (H + 1) counters fit its s_h buffer (256-thread workgroups)
bool orb_fuses_bucket(const Geo& g) { return g.H + 1 <= 4 * kHPairs * kHDw; }

#ifndef ORBFE_ORB_SMALL_KPW
#define ORBFE_ORB_SMALL_KPW 2
#endif
constexpr int kOrbSmallKpw = ORBFE_ORB_SMALL_KPW;  // keypoints per wave below the 4-keypoint threshold (2 or 4)
// keypoints per wave for a batch: 8 (4 waves per workgroup: 953 -> 914 us per 256 pairs against 4, same-box
// A/B, round 1) while the batch gives >= 16 waves per CU that way, else 4, else 2 (a frame pair: 508 waves of
// 8 keypoints, 2 028 of 2).  Variants (microbench): 1 / 9 / 2 force 8 / 4 / 2.
int orb_kpw(const Geo& g, int n_images, int variant) {
    if (variant == 1) return 8;
    if (variant == 9) return 4;
    if (variant == 2 || variant == 12) return 2;
    for (int k : {8, 4})
        if ((int64_t)orb_waves(g, k) * n_images >= 16 * 256) return k;
    return kOrbSmallKpw;
}

hipError_t launch_orb(const Geo& g, const uint8_t* in, int64_t in_pitch, const uint8_t* ws, const uint32_t* lvl_kp,
                      const int* lvl_count, orbfe_keypoint* out_kp, uint8_t* out_desc, int* out_count, int n_images,
                      const uint32_t* tab, hipStream_t s, int variant, const StereoArgs* bucket, int n_bucket) {
    if (bucket && !orb_fuses_bucket(g)) return hipErrorInvalidValue;
#ifdef ORBFE_DEV_VARIANTS
    if (variant == 8) {
        launch_orb_nw<8, 4>(g, in, in_pitch, ws, lvl_kp, lvl_count, out_kp, out_desc, out_count, n_images, tab, s, nullptr, 0);
        return hipGetLastError();
    }
    if (variant == 10) {
        launch_orb_nw<4, 16>(g, in, in_pitch, ws, lvl_kp, lvl_count, out_kp, out_desc, out_count, n_images, tab, s, bucket,
                             n_bucket);
        return hipGetLastError();
    }
#endif
    switch (orb_kpw(g, n_images, variant)) {
        case 2: launch_orb_nw<4, 2>(g, in, in_pitch, ws, lvl_kp, lvl_count, out_kp, out_desc, out_count, n_images, tab, s,
                                    bucket, n_bucket); break;
        case 4: launch_orb_nw<4, 4>(g, in, in_pitch, ws, lvl_kp, lvl_count, out_kp, out_desc, out_count, n_images, tab, s,
                                    bucket, n_bucket); break;
        default: launch_orb_nw<4, 8>(g, in, in_pitch, ws, lvl_kp, lvl_count, out_kp, out_desc, out_count, n_images, tab, s,
                                     bucket, n_bucket);
    }
    return hipGetLastError();
}

hipError_t launch_stereo(const Geo& g, const StereoArgs& a, int n_pairs, hipStream_t s, bool buckets_built) {
    if (buckets_built) {
    } else if (2 * n_pairs < kSmallBatchImages)
        hipLaunchKernelGGL(k_stereo_bucket<1024>, dim3(n_pairs), dim3(1024), (size_t)4 * (g.H + 1), s, g, a);
    else
        hipLaunchKernelGGL(k_stereo_bucket<256>, dim3(n_pairs), dim3(256), (size_t)4 * (g.H + 1), s, g, a);
    hipLaunchKernelGGL(k_stereo, dim3((g.kp_cap + 15) / 16, n_pairs), dim3(256), 0, s, g, a);
    return hipGetLastError();
}

hipError_t launch_shear(const Geo& g, const uint8_t* in, int64_t in_pitch, const uint8_t* ws, uint8_t* out, int n_images,
                        hipStream_t s) {
    if (n_images <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_shear, dim3((unsigned)((g.shear_bytes + 1023) / 1024), n_images), dim3(256), 0, s, g, in, in_pitch,
                       ws, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------- k_pack
// One fixed-capacity record per stereo pair for the rank-0 gather of the batched-frames mode
// (pyorbslam_amd/dist.py record layout): counts L, R (2 x i32) | keypoints L, R (cap x 24 B each) |
// descriptors L, R (cap x 32 B each) | u_right, depth (cap x f32) | status (cap x i8).  Every region but
// the last is a whole number of dwords at a dword offset: dword copies, the status bytes singly.
__global__ __launch_bounds__(256) void k_pack(PackArgs a, uint8_t* __restrict__ out, int pair0) {
    const int p = blockIdx.y, gp = pair0 + p;
    uint8_t* rec = out + (int64_t)p * a.rec_bytes;
    const int64_t cap = a.kp_cap;
    const uint32_t* src[7] = {
        (const uint32_t*)(a.count + 2 * (int64_t)gp),
        (const uint32_t*)(a.kps + (2 * (int64_t)gp) * cap), (const uint32_t*)(a.kps + (2 * (int64_t)gp + 1) * cap),
        (const uint32_t*)(a.desc + (2 * (int64_t)gp) * cap * 32), (const uint32_t*)(a.desc + (2 * (int64_t)gp + 1) * cap * 32),
        (const uint32_t*)(a.u_right + gp * cap), (const uint32_t*)(a.depth + gp * cap)};
    const int64_t words[7] = {2, cap * 6, cap * 6, cap * 8, cap * 8, cap, cap};
    const int64_t nw = 2 + cap * 30;  // dwords of regions 0..6
    for (int64_t w = (int64_t)blockIdx.x * 256 + threadIdx.x; w < nw + cap; w += (int64_t)gridDim.x * 256) {
        if (w >= nw) {  // status bytes
            const int64_t i = w - nw;
            rec[4 * nw + i] = (uint8_t)a.status[gp * cap + i];
            continue;
        }
        int r = 0;
        int64_t o = w;
        while (o >= words[r]) o -= words[r++];
        ((uint32_t*)rec)[w] = src[r][o];
    }
}

// Compact records (orbfe_batch_pack_compact_device, pyorbslam_amd/dist.py unpack_compact): counts L, R (2 x i32)
// | keypoints L, R (cap x {u32 x | y << 14 | octave << 28 in level pixels, f32 angle}) | descriptors L, R
// (cap x 32 B) | u_right, depth (cap x f32) | scores L, R (cap x u8) | status (cap x i8): 8 + 91 cap bytes
// against 8 + 121 cap.  A keypoint's x, y, size and response follow from (x, y, octave, score) on the host
// exactly as k_orb computed them (x = f32(level x) * scale[octave]; the level coordinate is recovered here
// as rint(x * inv_scale), exact for coordinates < 2^22).  The record keeps 14 bits per level coordinate
// (kCompactXYBits) and 8 bits of response: exact while every level is at most 16 383 px per side
// (orbfe_batch_pack_compact_device refuses larger geometries) and the FAST score M - 1 <= 254 (u8 pixels).
__global__ __launch_bounds__(256) void k_pack_compact(PackArgs a, CompactScales sc, uint8_t* __restrict__ out, int pair0) {
    const int p = blockIdx.y, gp = pair0 + p, t = blockIdx.x * 256 + threadIdx.x, nt = gridDim.x * 256;
    uint8_t* rec = out + (int64_t)p * a.rec_bytes;
    const int64_t cap = a.kp_cap;
    uint32_t* w = (uint32_t*)rec;
    if (t < 2) w[t] = (uint32_t)a.count[2 * (int64_t)gp + t];
    for (int s = 0; s < 2; ++s) {  // keypoints and scores of image 2 gp + s
        const orbfe_keypoint* kp = a.kps + (2 * (int64_t)gp + s) * cap;
        uint32_t* kw = w + 2 + s * 2 * cap;
        uint8_t* sb = rec + 8 + cap * 88 + s * cap;
        for (int64_t i = t; i < cap; i += nt) {
            const orbfe_keypoint k = kp[i];
            const int o = k.octave & 15;
            const uint32_t m = (1u << kCompactXYBits) - 1u;
            const uint32_t x = (uint32_t)__float2int_rn(k.x * sc.inv_scale[o]) & m;
            const uint32_t y = (uint32_t)__float2int_rn(k.y * sc.inv_scale[o]) & m;
            kw[2 * i] = x | (y << kCompactXYBits) | ((uint32_t)o << (2 * kCompactXYBits));
            kw[2 * i + 1] = __float_as_uint(k.angle);
            sb[i] = (uint8_t)(int)k.response;
        }
    }
    const uint32_t* d = (const uint32_t*)(a.desc + (2 * (int64_t)gp) * cap * 32);  // L then R: adjacent
    uint32_t* dw = w + 2 + 4 * cap;
    for (int64_t i = t; i < 16 * cap; i += nt) dw[i] = d[i];
    uint32_t* uw = dw + 16 * cap;
    for (int64_t i = t; i < cap; i += nt) {
        uw[i] = __float_as_uint(a.u_right[gp * cap + i]);
        uw[cap + i] = __float_as_uint(a.depth[gp * cap + i]);
    }
    uint8_t* st = rec + 8 + cap * 90;
    for (int64_t i = t; i < cap; i += nt) st[i] = (uint8_t)a.status[gp * cap + i];
}

hipError_t launch_pack_compact(const PackArgs& a, const CompactScales& sc, uint8_t* out, int pair0, int n_pairs,
                               hipStream_t s) {
    if (n_pairs <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_compact, dim3(16, n_pairs), dim3(256), 0, s, a, sc, out, pair0);
    return hipGetLastError();
}

hipError_t launch_pack(const PackArgs& a, uint8_t* out, int pair0, int n_pairs, hipStream_t s) {
    if (n_pairs <= 0) return hipSuccess;
    const int64_t items = 2 + (int64_t)a.kp_cap * 31;
    const unsigned bx = (unsigned)std::min<int64_t>((items + 255) / 256, 64);
    hipLaunchKernelGGL(k_pack, dim3(bx, n_pairs), dim3(256), 0, s, a, out, pair0);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------- k_copy_segments
// Several dword-aligned device -> (device-visible page-locked host) copies in one launch: the per-frame path's
// results go to the host as one kernel's stores over PCIe instead of eight copy-engine transfers of a few
// microseconds of fixed cost each.  blockIdx.y = segment.
// 16-byte stores (the segments start 16-byte aligned: device allocations and 256-byte aligned offsets into the
// page-locked buffer), the last dwords of a segment by block 0
__global__ __launch_bounds__(256) void k_copy_segments(CopySegs a) {
    const CopySegs::Seg sg = a.seg[blockIdx.y];
    const uint32_t n4 = sg.dwords >> 2;
    const uint4* src4 = (const uint4*)sg.src;
    uint4* dst4 = (uint4*)sg.dst;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n4; i += gridDim.x * 256u) dst4[i] = src4[i];
    if (blockIdx.x == 0 && threadIdx.x < (sg.dwords & 3u)) sg.dst[4 * n4 + threadIdx.x] = sg.src[4 * n4 + threadIdx.x];
}

hipError_t launch_copy_segments(const CopySegs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    uint32_t most = 0;
    for (int k = 0; k < a.n; ++k) {
        if (((uintptr_t)a.seg[k].src | (uintptr_t)a.seg[k].dst) & 15u) return hipErrorInvalidValue;
        most = std::max(most, a.seg[k].dwords);
    }
    // enough waves for the PCIe stores of the largest segment (the frame's sheared views, ~0.7 M dwords)
    const unsigned bx = std::max(1u, std::min((most / 4u + 1023u) / 1024u, 128u));
    hipLaunchKernelGGL(k_copy_segments, dim3(bx, a.n), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_hamming_matrix(const uint8_t* a, int na, const uint8_t* b, int nb, int* out, hipStream_t s) {
    if (na == 0 || nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hamming_matrix, dim3((nb + 255) / 256, na), dim3(256), 0, s, a, na, b, nb, out);
    return hipGetLastError();
}

hipError_t launch_hamming_search(const uint8_t* q, int nq, const uint8_t* tr, const int* off, const int* idx, int* bd,
                                 int* bi, int* sd, int* si, int* all_d, hipStream_t s) {
    if (nq == 0) return hipSuccess;
    hipLaunchKernelGGL(k_hamming_search, dim3((nq + 3) / 4), dim3(256), 0, s, q, nq, tr, off, idx, bd, bi, sd, si, all_d);
    return hipGetLastError();
}

}  // namespace orbfe
