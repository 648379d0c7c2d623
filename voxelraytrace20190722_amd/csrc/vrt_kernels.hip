// vrt_kernels.hip -- gfx950 (CDNA4, wave64) kernels of the primary-ray hot
// path: fused camera ray generation (T1), octree ray march (T2-T6), primary
// shading (T7) and Film accumulation (T8) -- SURVEY §8(a).
//
// One ray per lane.  A 256-thread workgroup owns one 8x8-pixel screen tile;
// each wave covers a 4x4-pixel quadrant x the 4 gen_rays4 samples (lane =
// pixel*4 + sample), so the four samples of a pixel sit in adjacent lanes
// and are summed in the reference's order with cross-lane reads.
//
// Traversal keeps the reference's result exactly (first DFS leaf with any
// hit; nearest of that leaf's triangles), but restructures the work:
//  * a node's 8 child boxes are never loaded: split() makes them from the
//    parent box with exact float ops (VRT/voxel_octree.cc:27-39), so one
//    32-B node record gives all 8 slab tests from 9 plane distances;
//  * every child is slab-tested when its parent is expanded (the reference
//    tests it when popped -- same outcome), and only the hit children are
//    kept, ordered by the (dist, child index) key that libstdc++'s stable
//    insertion sort produces (VRT/voxel_octree.cc:77-97), packed 3 bits
//    each into one 24-bit word;
//  * the DFS stack lives in LDS, [level][lane], 8 B per entry.
//
// VRT/x = /root/reference/VoxelRayTrace20190722/x
#include "vrt.h"
#include "vrt_internal.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <mutex>
#include <vector>

namespace vrt {

constexpr int kBlock = 256;
// DFS stack entries per lane.  ray_march pushes only when it descends into
// an internal child with siblings left, while walking the children of a
// node at depth d <= max_depth - 2 (internal nodes end at depth
// max_depth - 1), so at most max_depth - 2 entries are live.
constexpr int kStack = 10;
static_assert(kStack >= VRT_MAX_DEPTH - 1, "DFS stack too small for VRT_MAX_DEPTH");

struct RayK {
        f3 o, d, dinv;
        float tmin, tmax;
};

__device__ __forceinline__ void load_node(const NodeRec *__restrict__ nodes,
                                          uint32_t i, float bmin[3],
                                          float bmax[3], uint32_t &a,
                                          uint32_t &b)
{
        const float4 *q = reinterpret_cast<const float4 *>(nodes + i);
        const float4 q0 = q[0];
        const float4 q1 = q[1];
        bmin[0] = q0.x; bmin[1] = q0.y; bmin[2] = q0.z;
        bmax[0] = q0.w; bmax[1] = q1.x; bmax[2] = q1.y;
        a = __float_as_uint(q1.z);
        b = __float_as_uint(q1.w);
}

// DevScene::xnodes record i: the node record and the triangle box below it
__device__ __forceinline__ void load_xnode(const XNodeRec *__restrict__ x, uint32_t i, float bmin[3],
                                           float bmax[3], uint32_t &a, uint32_t &b, float tmn[3], float tmx[3])
{
        const float4 *q = reinterpret_cast<const float4 *>(x + i);
        const float4 q0 = q[0];
        const float4 q1 = q[1];
        const float4 q2 = q[2];
        const float2 q3 = *reinterpret_cast<const float2 *>(q + 3);
        bmin[0] = q0.x; bmin[1] = q0.y; bmin[2] = q0.z;
        bmax[0] = q0.w; bmax[1] = q1.x; bmax[2] = q1.y;
        a = __float_as_uint(q1.z);
        b = __float_as_uint(q1.w);
        tmn[0] = q2.x; tmn[1] = q2.y; tmn[2] = q2.z;
        tmx[0] = q2.w; tmx[1] = q3.x; tmx[2] = q3.y;
}

// ---------------------------------------------------------------------------
// Diagnostic build only (VRT_PHASE_STAMPS=1, never the product): per-wave
// phase cycles (s_memtime) and lane activity of the fast march, summed over
// all waves into g_phase (read by vrt_diag_phases).
#ifndef VRT_PHASE_STAMPS
#define VRT_PHASE_STAMPS 0
#endif
// bit ci of m -> bit ci ^ s (children renumbered so that ascending order is
// the ray's direction-sign order)
__device__ __forceinline__ uint32_t xor_permute8(uint32_t m, uint32_t s)
{
        m = (s & 4u) ? (((m & 0x0Fu) << 4) | ((m >> 4) & 0x0Fu)) : m;
        m = (s & 2u) ? (((m & 0x33u) << 2) | ((m >> 2) & 0x33u)) : m;
        m = (s & 1u) ? (((m & 0x55u) << 1) | ((m >> 1) & 0x55u)) : m;
        return m;
}

// children in ascending (ci ^ s): the near half of each axis first
__device__ __forceinline__ uint32_t dir_signs(const RayK &r)
{
        return (r.d.x < 0.f ? 4u : 0u) | (r.d.y < 0.f ? 2u : 0u) | (r.d.z < 0.f ? 1u : 0u);
}

// wave reductions (every lane of the wave active)
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
        for (int o = 32; o > 0; o >>= 1)
                v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
        return v;
}
__device__ __forceinline__ uint32_t lane_id()
{
        int lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        return (uint32_t)lane;
}
// LDS written by some lanes of a wave, then read by others of the same wave
__device__ __forceinline__ void wave_lds_sync()
{
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// Diagnostic build only (VRT_LIGHT_DIAG=1): per light-pass wave, its walk's
// cycles and per-lane node visits / leaf phases / triangle tests (maximum and
// sum over the lanes), dumped by the host after each light pass.
#ifndef VRT_LIGHT_DIAG
#define VRT_LIGHT_DIAG 0
#endif
#if VRT_LIGHT_DIAG
constexpr int kLightDiagWaves = 1 << 20;
__device__ uint32_t g_light_diag[kLightDiagWaves * 8];
#endif
#if VRT_PHASE_STAMPS || VRT_LIGHT_DIAG
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
        for (int o = 32; o > 0; o >>= 1)
                v += (uint32_t)__shfl_xor((int)v, o, 64);
        return v;
}
#endif
// Diagnostic build only (VRT_UNIT_DIAG=1): per unit of the persistent
// render: its start / end time (low 32 bits of s_memrealtime, 100 MHz: the
// one clock all XCDs share), the wave that ran it and its slice, dumped by
// the host after each launch (tools/unit_tail.py reads them).
#ifndef VRT_UNIT_DIAG
#define VRT_UNIT_DIAG 0
#endif
#if VRT_UNIT_DIAG
constexpr int kUnitDiagMax = 1 << 20;
__device__ uint32_t g_unit_diag[kUnitDiagMax * 4];
__device__ uint32_t g_unit_walk[kUnitDiagMax * 4];  // with VRT_LIGHT_DIAG: wave max / sum of node visits, triangle tests
#endif
#if VRT_PHASE_STAMPS
// [0..11] per-wave phase totals (ray_march); [12..19] wave iterations of the
// node-visit loop in which some lane: [12] iterates at all, [13] pops a stack
// entry, [14] is skipped by the triangle-box line test, [15] expands an
// internal node, [16] orders >= 2 hit children, [17] > 4 (rank_order8),
// [18] 3-4 (net4_order) with none > 4, [19] stops at a leaf; cycles of the
// persistent render per unit (wave lead): [20] the dequeue (take_unit),
// [21] render_unit's entry to the march call (tile, ray, fast-path vote),
// [22] the march call (ray_march: root + walk), [23] the march's return to
// render_unit's end (shading, film sum and store)
constexpr int kPhaseWords = 24;
__device__ unsigned long long g_phase[kPhaseWords];
// counted by the first active lane of the wave only: summed over the
// lanes, each wave iteration counts once
__device__ __forceinline__ uint32_t wave_lead()
{
        const uint64_t act = __ballot(1);
        int lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        return (uint32_t)lane == (uint32_t)(__ffsll((long long)act) - 1) ? 1u : 0u;
}
#endif

// ---------------------------------------------------------------------------
// travorder's child order (VRT/voxel_octree.cc:77-97): std::sort of the 8
// Items {ci, dist} with `lhs.dist < rhs.dist`.  For 8 elements libstdc++'s
// std::sort is one __insertion_sort (the introsort loop stops at 16
// elements): move-to-front when val < first, else __unguarded_linear_insert
// (shift while val < prev).  With no NaN among the distances that is the
// stable order on (dist, ci); a NaN dist breaks the total order, and only the
// insertion sort itself reproduces the result.  The kernel keeps only the
// children whose slab test passed (hm), in that order, 3 bits each (first
// child in bits 0-2).  These helpers are the kernel's own sort code, called
// by expand_* below and by k_selftest_order, which pins them against the
// real libstdc++ std::sort (tests/golden/travorder_std.cpp).
// ---------------------------------------------------------------------------

// The insertion sort itself on a packed permutation word (3-bit field p =
// child at position p), as adjacent swaps of val from position j to j-1:
// all of them when val < a[0], else until the first failing comparison.
// dist_of(ci) returns child ci's distance (recomputed per use: few live
// registers on this rare path).
template <class DistOf>
__device__ __forceinline__ uint32_t insertion_perm8(DistOf dist_of)
{
        uint32_t perm = 0xFAC688u;  // position p holds child p
#pragma unroll
        for (int i = 1; i < 8; ++i) {
                const uint32_t vi = (perm >> (3 * i)) & 7u;
                const float v = dist_of(vi);
                const bool front = v < dist_of(perm & 7u);
                bool go = true;
#pragma unroll
                for (int j = i; j >= 1; --j) {
                        const uint32_t pk = (perm >> (3 * (j - 1))) & 7u;
                        go = go && (front || v < dist_of(pk));
                        const uint32_t sw = (perm & ~(63u << (3 * (j - 1)))) | (pk << (3 * j)) |
                                            (vi << (3 * (j - 1)));
                        perm = go ? sw : perm;
                }
        }
        return perm;
}

// The hit children of a full order `perm`, in order; n = their number;
// full_pos (kFullPos) = the position of each child ci in the full order,
// bits 3ci (the reference's test counts).
template <bool kFullPos>
__device__ __forceinline__ uint32_t perm_filter(uint32_t perm, uint32_t hm, int &n, uint32_t &full_pos)
{
        uint32_t order = 0;
        int k = 0;
        full_pos = 0;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
                const uint32_t ci = (perm >> (3 * p)) & 7u;
                const bool hc = (hm >> ci) & 1u;
                order |= hc ? (ci << (3 * k)) : 0u;
                k += hc ? 1 : 0;
                if (kFullPos)
                        full_pos |= (uint32_t)p << (3 * ci);
        }
        n = k;
        return order;
}

// No NaN: the rank of each hit child among the hit children under the
// stable (dist, index) order (j < i precedes i <=> !(dist_i < dist_j));
// full_pos (kFullPos) = rank among all 8.
template <bool kFullPos>
__device__ __forceinline__ uint32_t rank_order8(const float dist[8], uint32_t hm, uint32_t &full_pos)
{
        uint32_t rk[8], fp[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
                rk[i] = 0;
                fp[i] = 0;
        }
#pragma unroll
        for (int i = 1; i < 8; ++i) {
#pragma unroll
                for (int j = 0; j < i; ++j) {
                        const bool c = dist[i] < dist[j];  // i strictly first
                        rk[j] += (uint32_t)(c & ((hm >> i) & 1u));
                        rk[i] += (uint32_t)(!c & ((hm >> j) & 1u));
                        if (kFullPos) {
                                fp[j] += (uint32_t)c;
                                fp[i] += (uint32_t)!c;
                        }
                }
        }
        uint32_t order = 0;
        full_pos = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
                order |= ((hm >> i) & 1u) ? ((uint32_t)i << (3 * rk[i])) : 0u;
                if (kFullPos)
                        full_pos |= fp[i] << (3 * i);
        }
        return order;
}

// No NaN, at most 2 hit children: one comparator (ties keep index order,
// i0 < i1).
template <class DistOf>
__device__ __forceinline__ uint32_t two_slot_order(DistOf dist_of, uint32_t hm)
{
        const uint32_t i0 = (uint32_t)__builtin_ctz(hm | 0x100u);
        const uint32_t m1 = hm & (hm - 1u);
        const uint32_t i1 = (uint32_t)__builtin_ctz(m1 | 0x100u);
        const float d0 = dist_of(i0);
        const float d1 = i1 < 8u ? dist_of(i1) : __int_as_float(0x7f800000);
        const bool sw = d1 < d0;
        return sw ? ((i1 & 7u) | ((i0 & 7u) << 3)) : ((i0 & 7u) | ((i1 & 7u) << 3));
}

__device__ __forceinline__ void ce4(float &da, uint32_t &ia, float &db, uint32_t &ib)
{
        const bool sw = (db < da) | ((db == da) & (ib < ia));
        const float td = da;
        const uint32_t ti = ia;
        da = sw ? db : da;
        ia = sw ? ib : ia;
        db = sw ? td : db;
        ib = sw ? ti : ib;
}

__device__ __forceinline__ void ce4_lt(float &da, uint32_t &ia, float &db, uint32_t &ib)
{
        const bool sw = db < da;
        const float td = da;
        const uint32_t ti = ia;
        da = sw ? db : da;
        ia = sw ? ib : ia;
        db = sw ? td : db;
        ib = sw ? ti : ib;
}

// No NaN, at most 4 hit children (a line through the 8 octants of a box
// crosses at most 4, barring degenerate boxes): the children go into 4
// slots in index order (empty slots sort last) and a 5-comparator network
// orders them on the total order (dist, index).  The slots start in index
// order, so in the first two layers the element in the lower slot always
// has the lower index ((0,1),(2,3) trivially; (0,2),(1,3) compare a
// slot-{0,1} child with a slot-{2,3} one): ties keep the order and the
// comparison reduces to dist.  Only the last comparator (1,2) needs the
// index.
template <class DistOf>
__device__ __forceinline__ uint32_t net4_order(DistOf dist_of, uint32_t hm)
{
        float d[4];
        uint32_t id[4];
        uint32_t m = hm;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
                const uint32_t i = m ? (uint32_t)__builtin_ctz(m) : 8u;
                m &= m - 1u;
                const float dv = dist_of(i);
                d[k] = i < 8u ? dv : __int_as_float(0x7f800000);
                id[k] = i;
        }
        ce4_lt(d[0], id[0], d[1], id[1]);
        ce4_lt(d[2], id[2], d[3], id[3]);
        ce4_lt(d[0], id[0], d[2], id[2]);
        ce4_lt(d[1], id[1], d[3], id[3]);
        ce4(d[1], id[1], d[2], id[2]);
        return (id[0] & 7u) | ((id[1] & 7u) << 3) | ((id[2] & 7u) << 6) | ((id[3] & 7u) << 9);
}

// Expand an internal node with box [bmin,bmax]: slab-test its 8 children
// (boxes from split()'s exact arithmetic) and return the hit children in
// travorder order, 3 bits each (first child in bits 0-2); cnt = number.
// full_pos (instrumented only): 3-bit position of each child ci (bits 3ci)
// in the full 8-child travorder order, for the reference's test counts.
//
// kFast (chosen per wave when every lane's ray and the scene are finite and
// no direction component is a non-zero denormal): no slab distance can be
// NaN, so IEEE min/max (v_min/v_max/v_min3/v_max3) give the same values as
// std::min/max and max_element/min_element up to the sign of a zero, which
// no later comparison can observe.  The exact path keeps the reference's
// select semantics for everything else.
template <bool kFullPos, bool kFast>
__device__ __forceinline__ uint32_t expand_v1(const float bmin[3],
                                              const float bmax[3],
                                              const RayK &r, int &cnt,
                                              uint32_t &full_pos,
                                              uint32_t content)
{
        const float oo[3] = { r.o.x, r.o.y, r.o.z };
        const float dd[3] = { r.d.x, r.d.y, r.d.z };
        const float di[3] = { r.dinv.x, r.dinv.y, r.dinv.z };
        float nr[3][2], fr[3][2], q[3][2];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
                // split(): mask-0 child [min + 0*h, min + 0*h + h], mask-1
                // child [min + h, min + h + h].  With a finite h (fast
                // path: finite scene), min + 0*h and (min+0*h)+h equal min
                // and min+h up to the sign of a zero, which no slab
                // comparison or distance order can observe, so the planes
                // are min, b = min+h, c = b+h.
                const float h = (bmax[k] - bmin[k]) / 2.0f;
                const float a0 = kFast ? bmin[k] : bmin[k] + 0.0f * h;
                const float b = bmin[k] + h;
                const float a1 = kFast ? b : a0 + h;
                const float c = b + h;
                const float ta = (a0 - oo[k]) * di[k];
                const float tb0 = (a1 - oo[k]) * di[k];
                const float tb1 = kFast ? tb0 : (b - oo[k]) * di[k];
                const float tc = (c - oo[k]) * di[k];
                if (kFast) {
                        nr[k][0] = fminf(ta, tb0);
                        fr[k][0] = fmaxf(ta, tb0);
                        nr[k][1] = fminf(tb1, tc);
                        fr[k][1] = fmaxf(tb1, tc);
                } else {
                        nr[k][0] = std_min(ta, tb0);
                        fr[k][0] = std_max(ta, tb0);
                        nr[k][1] = std_min(tb1, tc);
                        fr[k][1] = std_max(tb1, tc);
                }
                q[k][0] = dd[k] * ((a0 + a1) * .5f - oo[k]);
                q[k][1] = dd[k] * ((b + c) * .5f - oo[k]);
        }
        const float qx0 = 0.0f + q[0][0], qx1 = 0.0f + q[0][1];
        uint32_t hm = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
                const int mx = (i >> 2) & 1, my = (i >> 1) & 1, mz = i & 1;
                float t0, t1;
                if (kFast) {
                        t0 = fmaxf(fmaxf(nr[0][mx], nr[1][my]), nr[2][mz]);
                        t1 = fminf(fminf(fr[0][mx], fr[1][my]), fr[2][mz]);
                } else {
                        t0 = nr[0][mx];
                        t1 = fr[0][mx];
                        if (t0 < nr[1][my]) t0 = nr[1][my];
                        if (t0 < nr[2][mz]) t0 = nr[2][mz];
                        if (fr[1][my] < t1) t1 = fr[1][my];
                        if (fr[2][mz] < t1) t1 = fr[2][mz];
                }
                // !(t0 > t1) && (t0 in [tmin,tmax] || t1 in [tmin,tmax]),
                // evaluated without branches
                const bool h = ((content >> i) & 1u) & !(t0 > t1) & (((t0 >= r.tmin) & (t0 <= r.tmax)) |
                                                                     ((t1 >= r.tmin) & (t1 <= r.tmax)));
                hm |= (uint32_t)h << i;
        }
        // travorder: dot(d, center - o), center = (min + max) * .5f, summed
        // x + y + z from 0
        auto dist_of = [&](uint32_t ci) {
                return (((ci & 4u) ? qx1 : qx0) + ((ci & 2u) ? q[1][1] : q[1][0])) +
                       ((ci & 1u) ? q[2][1] : q[2][0]);
        };
        if (!kFast)
                return perm_filter<kFullPos>(insertion_perm8(dist_of), hm, cnt, full_pos);
        float dist[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
                dist[i] = dist_of((uint32_t)i);
        cnt = __popc(hm);
        return rank_order8<kFullPos>(dist, hm, full_pos);
}

// v2 (fast path, uninstrumented): the same slab tests as v1, the hit
// children ordered by two_slot_order / net4_order when no lane of the wave
// has more than 2 / 4 of them (rank_order8 otherwise); the travorder
// distances are finished only when some lane orders >= 2 children.
// kStd == 2: tmax == FLT_MAX, tmin is not NaN and
// every |dinv| <= 2^64 (no zero or tiny direction component), so with
// |plane - o| < 2^61 (fast_ok) every slab distance is finite and the
// reference's test !(t0 > t1) && (t0 in [tmin, FLT_MAX] || t1 in [tmin,
// FLT_MAX]) is exactly t0 <= t1 && t1 >= tmin (the second clause follows
// from t1 >= tmin when t0 <= t1, and neither endpoint can be +inf), i.e.
// max(t0, tmin) <= t1: tmin is folded into one axis's near distances once
// per expansion, leaving max3, min3 and one compare per child.
template <int kStd>  // 0 or 2
__device__ __forceinline__ uint32_t expand_v2(const float bmin[3], const float bmax[3], const RayK &r, int &cnt,
                                              uint32_t content)
{
        const float oo[3] = { r.o.x, r.o.y, r.o.z };
        const float dd[3] = { r.d.x, r.d.y, r.d.z };
        const float di[3] = { r.dinv.x, r.dinv.y, r.dinv.z };
        float nr[3][2], fr[3][2], cm[3][2];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
                const float h = (bmax[k] - bmin[k]) / 2.0f;
                const float a0 = bmin[k];
                const float b = bmin[k] + h;
                const float c = b + h;
                cm[k][0] = (a0 + b) * .5f;  // child centres (AABB::center)
                cm[k][1] = (b + c) * .5f;
                if (!kStd) {  // eager: cheaper in registers for the secondary-ray kernels
                        cm[k][0] = dd[k] * (cm[k][0] - oo[k]);
                        cm[k][1] = dd[k] * (cm[k][1] - oo[k]);
                }
                const float ta = (a0 - oo[k]) * di[k];
                const float tb = (b - oo[k]) * di[k];
                const float tc = (c - oo[k]) * di[k];
                nr[k][0] = fminf(ta, tb);
                fr[k][0] = fmaxf(ta, tb);
                nr[k][1] = fminf(tb, tc);
                fr[k][1] = fmaxf(tb, tc);
        }
        if (kStd == 2) {
                nr[2][0] = fmaxf(nr[2][0], r.tmin);
                nr[2][1] = fmaxf(nr[2][1], r.tmin);
        }
        uint32_t hm = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
                const int mx = (i >> 2) & 1, my = (i >> 1) & 1, mz = i & 1;
                // one v_max3 / v_min3 per child: the compiler otherwise
                // shares the pairwise max of two axes (24 ops instead of 16)
                float t0, t1;
                asm("v_max3_f32 %0, %1, %2, %3" : "=v"(t0) : "v"(nr[0][mx]), "v"(nr[1][my]), "v"(nr[2][mz]));
                asm("v_min3_f32 %0, %1, %2, %3" : "=v"(t1) : "v"(fr[0][mx]), "v"(fr[1][my]), "v"(fr[2][mz]));
                bool h;
                if (kStd == 2) {
                        h = t0 <= t1;  // t0 = max(near distances, 0)
                } else {  // kStd == 0: the reference's range test
                        const bool in0 = (t0 >= r.tmin) & (t0 <= r.tmax);
                        const bool in1 = (t1 >= r.tmin) & (t1 <= r.tmax);
                        h = !(t0 > t1) & (in0 | in1);
                }
                hm |= (uint32_t)h << i;
        }
        hm &= content;
        const int n = __popc(hm);
        cnt = n;
        if (__all(n <= 1))
                return (uint32_t)__builtin_ctz(hm | 0x100u) & 7u;  // one or no hit child: nothing to order
        // travorder distances dot(d, centre - o), finished only when some
        // lane orders >= 2 children (camera rays, kStd)
        float q[3][2];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
                q[k][0] = kStd ? dd[k] * (cm[k][0] - oo[k]) : cm[k][0];
                q[k][1] = kStd ? dd[k] * (cm[k][1] - oo[k]) : cm[k][1];
        }
        const float qx0 = 0.0f + q[0][0], qx1 = 0.0f + q[0][1];
        auto dist_of = [&](uint32_t ci) {
                return (((ci & 4u) ? qx1 : qx0) + ((ci & 2u) ? q[1][1] : q[1][0])) +
                       ((ci & 1u) ? q[2][1] : q[2][0]);
        };
        if (__any(n > 4)) {
                // rare: the full rank order over the same mask
                float dist[8];
#pragma unroll
                for (int i = 0; i < 8; ++i)
                        dist[i] = dist_of((uint32_t)i);
                uint32_t fp_unused;
                return rank_order8<false>(dist, hm, fp_unused);
        }
        if (__all(n <= 2))
                return two_slot_order(dist_of, hm);  // common case
        return net4_order(dist_of, hm);
}

template <bool kFullPos, bool kFast, int kStd = 0>
__device__ __forceinline__ uint32_t expand(const float bmin[3],
                                           const float bmax[3],
                                           const RayK &r, int &cnt,
                                           uint32_t &full_pos, uint32_t content)
{
        if (kFast && !kFullPos)
                return expand_v2<kStd>(bmin, bmax, r, cnt, content);
        return expand_v1<kFullPos, kFast>(bmin, bmax, r, cnt, full_pos, content);
}

struct MarchResult {
        bool hit;
        uint32_t node;  // hit leaf
        uint32_t tri;
        float u, v;     // clamped barycentrics of the best triangle
        f3 hp;          // ISect::hit
        uint32_t A, L, T;  // reference-equivalent counters (instrumented)
        bool deferred;  // the walk stopped at its record budget (ray_march kBudget)
};

// ray_march_isect's std::min_element over the records (VRT/voxel_octree.cc:
// 122-125, `lhs.depth < rhs.depth`): a record replaces the best one only when
// none is kept yet or its depth is strictly smaller, so the FIRST minimum in
// leaf order wins (pinned against the real std::min_element by
// k_selftest_order / tests/golden/travorder_std.cpp).
__device__ __forceinline__ bool first_min_takes(bool any, float best, float depth)
{
        return !any || depth < best;
}

// ray_march_isect (VRT/voxel_octree.cc:99-129) over one leaf's records, with
// intersect_triangle3 (VRT/raytri.cc:197-249) inlined in a register-frugal
// order.  Every value is the same IEEE double operation on the same
// operands as mt_isect(); only the evaluation order of independent terms
// differs, and inv_det = 1.0/det -- side-effect free -- is evaluated only
// for a triangle that passes every test, so the results are identical.
// The best hit keeps (float)t; ISect::hit = o + (float)t*d is rebuilt once.
// One record of ray_march_isect's loop: intersect_triangle3 on the record
// (q0..q2 = the 48-B RefRec48, or q0 + qd1..qd3 = the RefRec64) and the
// first-minimum update of the best hit (any, best, best_t, m.tri/u/v).
template <bool kR64>
__device__ __forceinline__ bool mt_record(const float4 q0, const float4 q1, const float4 q2, const double2 qd1,
                                          const double2 qd2, const double2 qd3, const RayK &r, bool &any,
                                          float &best, float &best_t, MarchResult &m)
{
        const double v0x = q0.x, v0y = q0.y, v0z = q0.z;
        const double dx = r.d.x, dy = r.d.y, dz = r.d.z;
        // edge1 = vert1 - vert0, edge2 = vert2 - vert0 (VRT/raytri.cc:
        // 209-210): stored in double (RefRec64) or made here in the
        // register-frugal order edge2, pvec, edge1 (RefRec48)
        double e2x, e2y, e2z;
        if (kR64) {
                e2x = qd2.y, e2y = qd3.x, e2z = qd3.y;
        } else {
                e2x = (double)q1.z - v0x, e2y = (double)q1.w - v0y, e2z = (double)q2.x - v0z;
        }
        // pvec = dir x edge2
        const double px = dy * e2z - dz * e2y;
        const double py = dz * e2x - dx * e2z;
        const double pz = dx * e2y - dy * e2x;
        const double e1x = kR64 ? qd1.x : (double)q0.w - v0x;
        const double e1y = kR64 ? qd1.y : (double)q1.x - v0y;
        const double e1z = kR64 ? qd2.x : (double)q1.y - v0z;
        // det
        const double det = e1x * px + e1y * py + e1z * pz;
        if (!(det > 0.000001) && !(det < -0.000001))
                return false;  // parallel
        // small-leaf scenes: the origin is widened per record instead of
        // holding 6 VGPRs of doubles across the march (part of what lets the
        // persistent render run 6 waves per SIMD without spilling in its
        // advance loop; +3 % per frame); large-leaf scenes keep it hoisted
        // (their leaf loop dominates)
        float rox = r.o.x, roy = r.o.y, roz = r.o.z;
        if (!kR64)
                asm volatile("" : "+v"(rox), "+v"(roy), "+v"(roz));
        const double tx = (double)rox - v0x, ty = (double)roy - v0y, tz = (double)roz - v0z;
        const double uu = tx * px + ty * py + tz * pz;
        const bool pos = det > 0.000001;
        // det < 0 branch folded onto the det > 0 one by negation (exact;
        // round-to-nearest is symmetric, so -(uu + vv) == (-uu) + (-vv)):
        // the same accept/reject decisions, without divergent sign branches
        const double sdet = pos ? det : -det, suu = pos ? uu : -uu;
        if (suu < 0.0 || suu > sdet)
                return false;
        const double qx = ty * e1z - tz * e1y;
        const double qy = tz * e1x - tx * e1z;
        const double qz = tx * e1y - ty * e1x;
        const double vv = dx * qx + dy * qy + dz * qz;
        const double svv = pos ? vv : -vv;
        if (svv < 0.0 || suu + svv > sdet)
                return false;
        const double inv_det = 1.0 / det;
        const double t = (e2x * qx + e2y * qy + e2z * qz) * inv_det;
        // Triangle::isect (VRT/voxel_octree.cc:449-454)
        const float fu = clampf((float)(uu * inv_det), 0, 1);
        const float fv = clampf((float)(vv * inv_det), 0, 1);
        const float tf = (float)t;
        const f3 hp = r.o + r.d * tf;
        const float depth = length(hp - r.o);
        if (first_min_takes(any, best, depth)) {
                any = true;
                best = depth;
                best_t = tf;
                m.tri = __float_as_uint(kR64 ? q0.w : q2.y);
                m.u = fu;
                m.v = fv;
                return true;
        }
        return false;
}

// ray_march_isect (VRT/voxel_octree.cc:99-129) over one leaf's records, with
// intersect_triangle3 (VRT/raytri.cc:197-249) inlined in a register-frugal
// order.  Every value is the same IEEE double operation on the same
// operands as mt_isect(); only the evaluation order of independent terms
// differs, and inv_det = 1.0/det -- side-effect free -- is evaluated only
// for a triangle that passes every test, so the results are identical.
// The best hit keeps (float)t; ISect::hit = o + (float)t*d is rebuilt once.
template <bool kCount, bool kR64>
__device__ __forceinline__ bool leaf_isect_v2(const void *__restrict__ refs,
                                              uint32_t first, uint32_t n,
                                              const RayK &r, MarchResult &m)
{
        bool any = false;
        float best = 0.f, best_t = 0.f;
#pragma unroll 1
        for (uint32_t k = 0; k < n; ++k) {
                const float4 *q = kR64 ? reinterpret_cast<const float4 *>(static_cast<const RefRec64 *>(refs) + first + k)
                                       : reinterpret_cast<const float4 *>(static_cast<const RefRec48 *>(refs) + first + k);
                const double2 *qd = reinterpret_cast<const double2 *>(q);
                const float4 q0 = q[0];
                float4 q1 = q0, q2 = q0;
                double2 qd1 = {}, qd2 = {}, qd3 = {};
                if (kR64) {
                        qd1 = qd[1];
                        qd2 = qd[2];
                        qd3 = qd[3];
                } else {
                        q1 = q[1];
                        q2 = q[2];
                }
                mt_record<kR64>(q0, q1, q2, qd1, qd2, qd3, r, any, best, best_t, m);
        }
        if (any)
                m.hp = r.o + r.d * best_t;
        if (kCount)
                m.T += n;
        return any;
}

// The wave-uniform large-leaf loop (leaf_isect's scalar-cache path): the
// records are consumed in order as leaf_isect_v2 does, but fetched kG at a
// time (all kG records' loads issued before the first MT), so a long leaf is
// not one load latency per record.  A/B at depth 6 (1080p primary): kG = 2
// +3.7 %, 4 +3.4 %, 8 -17 % (SGPR spills); the light pass and the trace
// render are unchanged (their longest waves are not bound by this chain).
constexpr int kUniGroup = 2;
template <bool kCount>
__device__ __forceinline__ bool leaf_isect_uni(const RefRec64 *__restrict__ recs, uint32_t n, const RayK &r,
                                               MarchResult &m)
{
        constexpr int kG = kUniGroup;
        bool any = false;
        float best = 0.f, best_t = 0.f;
        uint32_t k = 0;
        for (; k + kG <= n; k += kG) {
                float4 q0[kG];
                double2 qd1[kG], qd2[kG], qd3[kG];
#pragma unroll
                for (int g = 0; g < kG; ++g) {
                        const float4 *q = reinterpret_cast<const float4 *>(recs + k + g);
                        const double2 *qd = reinterpret_cast<const double2 *>(q);
                        q0[g] = q[0];
                        qd1[g] = qd[1];
                        qd2[g] = qd[2];
                        qd3[g] = qd[3];
                }
#pragma unroll
                for (int g = 0; g < kG; ++g)
                        mt_record<true>(q0[g], q0[g], q0[g], qd1[g], qd2[g], qd3[g], r, any, best, best_t, m);
        }
        for (; k < n; ++k) {
                const float4 *q = reinterpret_cast<const float4 *>(recs + k);
                const double2 *qd = reinterpret_cast<const double2 *>(q);
                mt_record<true>(q[0], q[0], q[0], qd[1], qd[2], qd[3], r, any, best, best_t, m);
        }
        if (any)
                m.hp = r.o + r.d * best_t;
        if (kCount)
                m.T += n;
        return any;
}

// minimum / OR over each aligned group of kG lanes (every lane of the group
// active)
template <int kG>
__device__ __forceinline__ uint64_t group_min_u64(uint64_t v)
{
#pragma unroll
        for (int o = kG / 2; o > 0; o >>= 1) {
                const uint64_t w = (uint64_t)__shfl_xor((long long)v, o, 64);
                v = w < v ? w : v;
        }
        return v;
}
template <int kG>
__device__ __forceinline__ uint32_t group_or_u32(uint32_t v)
{
#pragma unroll
        for (int o = kG / 2; o > 0; o >>= 1)
                v |= (uint32_t)__shfl_xor((int)v, o, 64);
        return v;
}

// One ray per aligned group of kG lanes (every lane of a group holds the
// same ray and walks the same leaf): the leaf's records are split over the
// group (lane l tests records l % kG, + kG, ...) and the winner is
// ray_march_isect's first minimum over the whole leaf.  A lane's own first
// minimum is exact for its records unless its first hit had a NaN depth
// (which std::min_element would then keep); a NaN kept by any lane of the
// group sends the leaf through the serial loop (the group's lanes alike).
// Otherwise the leaf's winner is the least (depth, record) pair -- depth >=
// +0, so its float bits order as integers -- and every lane of the group
// re-tests that one record to take its (tri, u, v, hit) exactly as the
// serial loop would.
template <int kG, bool kR64>
__device__ __forceinline__ bool leaf_isect_grp(const void *__restrict__ refs, uint32_t first, uint32_t n,
                                               const RayK &r, MarchResult &m)
{
        bool any = false;
        float best = 0.f, best_t = 0.f;
        uint32_t kb = 0;
        for (uint32_t k = lane_id() & (kG - 1); k < n; k += kG) {
                const float4 *q = kR64 ? reinterpret_cast<const float4 *>(static_cast<const RefRec64 *>(refs) + first + k)
                                       : reinterpret_cast<const float4 *>(static_cast<const RefRec48 *>(refs) + first + k);
                const double2 *qd = reinterpret_cast<const double2 *>(q);
                const float4 q0 = q[0];
                float4 q1 = q0, q2 = q0;
                double2 qd1 = {}, qd2 = {}, qd3 = {};
                if (kR64) {
                        qd1 = qd[1];
                        qd2 = qd[2];
                        qd3 = qd[3];
                } else {
                        q1 = q[1];
                        q2 = q[2];
                }
                if (mt_record<kR64>(q0, q1, q2, qd1, qd2, qd3, r, any, best, best_t, m))
                        kb = k;
        }
        if (group_or_u32<kG>(any && isnan(best) ? 1u : 0u))
                return leaf_isect_v2<false, kR64>(refs, first, n, r, m);
        const uint64_t key = any ? ((uint64_t)__float_as_uint(best) << 32 | kb) : ~0ull;
        const uint64_t win = group_min_u64<kG>(key);
        if (win == ~0ull)
                return false;
        return leaf_isect_v2<false, kR64>(refs, first + (uint32_t)win, 1, r, m);
}

// kUni: 0 each lane its own leaf, 1 the same leaf may be shared (scalar
// loads when every lane tests it), >= 2 (a power of two) one ray per group
// of kUni lanes (leaf_isect_grp)
template <bool kCount, int kUni, bool kR64>
__device__ __forceinline__ bool leaf_isect(const DevScene &sc, uint32_t first, uint32_t n,
                                           const RayK &r, MarchResult &m)
{
        if (kUni >= 2)
                return leaf_isect_grp<(kUni >= 2 ? kUni : 2), kR64>(sc.refs, first, n, r, m);
        if (kR64 && kUni && !kCount) {
                // every active lane tests the same leaf (coherent rays,
                // large leaves): the records' address and count are
                // wave-uniform, so they come through the scalar cache.
                // Only for scenes with large leaves (RefRec64 scenes): with
                // a few records per leaf the check costs more than it saves
                const uint32_t f0 = __builtin_amdgcn_readfirstlane(first);
                const uint32_t n0 = __builtin_amdgcn_readfirstlane(n);
                if (__all(first == f0 && n == n0))
                        return leaf_isect_uni<kCount>(static_cast<const RefRec64 *>(sc.refs) + f0, n0, r, m);
        }
        return leaf_isect_v2<kCount, kR64>(sc.refs, first, n, r, m);
}

// Does the ray's whole line (every t, as intersect_triangle3 accepts hits
// behind the origin) meet the box?  The fast path's slab distances (finite:
// fin_ok); used on DevScene::xnodes' enlarged triangle boxes.
__device__ __forceinline__ bool line_meets_box(const float bmin[3], const float bmax[3], const RayK &r)
{
        const float ax = (bmin[0] - r.o.x) * r.dinv.x, bx = (bmax[0] - r.o.x) * r.dinv.x;
        const float ay = (bmin[1] - r.o.y) * r.dinv.y, by = (bmax[1] - r.o.y) * r.dinv.y;
        const float az = (bmin[2] - r.o.z) * r.dinv.z, bz = (bmax[2] - r.o.z) * r.dinv.z;
        float t0, t1;
        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(t0) : "v"(fminf(ax, bx)), "v"(fminf(ay, by)), "v"(fminf(az, bz)));
        asm("v_min3_f32 %0, %1, %2, %3" : "=v"(t1) : "v"(fmaxf(ax, bx)), "v"(fmaxf(ay, by)), "v"(fmaxf(az, bz)));
        return t0 <= t1;
}
// the ray may skip nodes by their triangle boxes (DevScene::xnodes)
__device__ __forceinline__ bool leaf_box_ok(const DevScene &sc, const RayK &r)
{
        return fabsf(r.o.x - sc.lb_center[0]) <= sc.lb_reach && fabsf(r.o.y - sc.lb_center[1]) <= sc.lb_reach &&
               fabsf(r.o.z - sc.lb_center[2]) <= sc.lb_reach;
}

// gi::ray_march (VRT/voxel_octree.cc:131-188).  stk_* are this lane's LDS
// stack columns (stride kBlock).  The finite-slab fast walk (kStd == 2)
// reads DevScene::xnodes and skips a node whose triangles' box the ray's
// line misses (no triangle below it can pass; the reference visits it and
// finds no record).
// kBudget > 0: the walk gives up (m.deferred) before a leaf that would take
// its triangle tests past kBudget; a caller re-walks such a ray elsewhere.
template <bool kCount, bool kFast, int kS, int kStd, int kUni, bool kR64, int kBudget = 0>
__device__ __forceinline__ void ray_march(const DevScene &sc, const RayK &r,
                                          uint2 *stk,
                                          uint32_t *stk_aux,
                                          uint32_t *path_rem,
                                          MarchResult &m)
{
        m.hit = false;
        m.deferred = false;
        m.A = 1;
        m.L = 0;
        m.T = 0;
        uint32_t used = 0;  // triangle tests so far (kBudget)
        float bmin[3], bmax[3];
        uint32_t a, b;
        constexpr bool kLB = kFast && kStd == 2 && !kCount;
        constexpr bool kNB = kLB;  // every visited node by its triangle box
        const NodeRec *__restrict__ nodes = sc.nodes;  // kNB: xnodes instead
        const bool lbok = kLB && __all(leaf_box_ok(sc, r));  // wave-uniform: held in SGPRs
        load_node(sc.nodes, 0, bmin, bmax, a, b);
        if (!aabb_isect(bmin, bmax, r.o, r.dinv, r.tmin, r.tmax))
                return;
        if (a & kLeafBit) {
                if (kCount)
                        m.L++;
                if (leaf_isect<kCount, kUni, kR64>(sc, b, a & ~kLeafBit, r, m)) {
                        m.hit = true;
                        m.node = 0;
                }
                return;
        }
        int cnt;
        uint32_t fpos;
        uint32_t order = expand<kCount, kFast, kStd>(bmin, bmax, r, cnt, fpos, kCount ? 0xFFu : b);
        uint32_t base = a;
        uint32_t depth = 1;  // depth of the node whose children we walk
        uint32_t nexp = 1;
        int sp = 0;
        // while-while: every lane first advances (pop / expand) to its next
        // non-empty leaf in DFS order, then the lanes test their leaves
        // together -- expand and leaf code no longer interleave per lane.
#if VRT_PHASE_STAMPS
        uint32_t d_it = 0, d_lp = 0, d_tri = 0, d_lpmax = 0, d_lpsum = 0, d_phmax = 0;
        unsigned long long d_tin = 0, d_tleaf = 0;
        uint32_t d_ev[8] = {};  // g_phase[12..19], counted by the wave's first active lane
#endif
        // VRT_LIGHT_DIAG builds: node visits, leaf phases and triangle tests
        // of this lane's walk, into m.A / m.L / m.T
        uint32_t dg_it = 0, dg_lp = 0, dg_tri = 0;
        for (;;) {
                bool leaf = false;
                uint32_t node = 0, nref = 0;
#if VRT_PHASE_STAMPS
                const unsigned long long d_t0 = __builtin_amdgcn_s_memtime();
#endif
                for (;;) {
#if VRT_PHASE_STAMPS
                        ++d_it;
                        {
                                const uint32_t ld = wave_lead();
                                d_ev[0] += ld;
                                d_ev[1] += ld & (__ballot(cnt == 0 && sp > 0) != 0ull);
                        }
#endif
                        if (VRT_LIGHT_DIAG)
                                ++dg_it;
                        if (cnt == 0) {
                                if (sp == 0)
                                        break;
                                --sp;
                                const uint2 e = stk[sp * kS];
                                base = e.x;
                                const uint32_t w = e.y;
                                order = w & 0xFFFFFFu;
                                cnt = (int)(w >> 24);
                                if (kCount) {
                                        const uint32_t x = stk_aux[sp * kS];
                                        fpos = x & 0xFFFFFFu;
                                        depth = x >> 24;
                                }
                                // a pushed entry always has cnt > 0, so the
                                // popped level's next child is visited in this
                                // same iteration
                        }
                        const uint32_t ci = order & 7u;
                        order >>= 3;
                        --cnt;
                        node = base + ci;
                        if (kCount)
                                path_rem[depth * kS] = 7u - ((fpos >> (3 * ci)) & 7u);
                        if (kNB) {
                                float tmn[3], tmx[3];
                                load_xnode(sc.xnodes, node, bmin, bmax, a, b, tmn, tmx);
                                const bool skip = lbok && !line_meets_box(tmn, tmx, r);
#if VRT_PHASE_STAMPS
                                d_ev[2] += wave_lead() & (__ballot(skip) != 0ull);
#endif
                                if (skip)
                                        continue;  // no triangle below this node can pass
                        } else {
                                load_node(nodes, node, bmin, bmax, a, b);
                        }
#if VRT_PHASE_STAMPS
                        d_ev[7] += wave_lead() & (__ballot((a & kLeafBit) != 0u) != 0ull);
#endif
                        if (!(a & kLeafBit)) {
                                if (cnt) {
                                        stk[sp * kS] = make_uint2(base, order | ((uint32_t)cnt << 24));
                                        if (kCount)
                                                stk_aux[sp * kS] = fpos | (depth << 24);
                                        ++sp;
                                }
                                order = expand<kCount, kFast, kStd>(bmin, bmax, r, cnt, fpos, kCount ? 0xFFu : b);
#if VRT_PHASE_STAMPS
                                {
                                        const uint32_t ld = wave_lead();
                                        d_ev[3] += ld;
                                        d_ev[4] += ld & (__ballot(cnt >= 2) != 0ull);
                                        const bool big = __ballot(cnt > 4) != 0ull;
                                        d_ev[5] += ld & big;
                                        d_ev[6] += ld & !big & (__ballot(cnt >= 3) != 0ull);
                                }
#endif
                                base = a;
                                ++depth;
                                ++nexp;
                                continue;
                        }
                        if (kCount)
                                m.L++;
                        nref = a & ~kLeafBit;
                        if (nref == 0)
                                continue;  // empty leaf (instrumented walk only)
                        leaf = true;
                        break;
                }
#if VRT_PHASE_STAMPS
                const unsigned long long d_t1 = __builtin_amdgcn_s_memtime();
                d_tin += d_t1 - d_t0;
                {
                        // over the lanes with a leaf (inactive lanes take no part)
                        d_lpmax = 0;
                        uint64_t lm = __ballot(leaf);
                        while (lm) {
                                const int l = __ffsll((long long)lm) - 1;
                                const uint32_t v = __builtin_amdgcn_readlane(nref, l);
                                d_lpmax = d_lpmax > v ? d_lpmax : v;  // this phase's longest leaf
                                d_lpsum += v;
                                lm &= lm - 1;
                        }
                        d_phmax += d_lpmax;
                }
#endif
                if (!leaf)
                        break;
                if (kBudget) {
                        used += nref;
                        if (used > (uint32_t)kBudget) {
                                m.deferred = true;
                                break;
                        }
                }
#if VRT_PHASE_STAMPS
                ++d_lp;
                d_tri += nref;
#endif
                if (VRT_LIGHT_DIAG) {
                        ++dg_lp;
                        dg_tri += nref;
                }
                const bool lh = leaf_isect<kCount, kUni, kR64>(sc, b, nref, r, m);
#if VRT_PHASE_STAMPS
                d_tleaf += __builtin_amdgcn_s_memtime() - d_t1;
#endif
                if (lh) {
                        m.hit = true;
                        m.node = node;
                        break;
                }
        }
#if VRT_PHASE_STAMPS
        {
                // every lane has left the loop: wave-level totals
                const uint32_t itmax = wave_max_u32(d_it), itsum = wave_sum_u32(d_it);
                const uint32_t lpmax = wave_max_u32(d_lp), lpsum = wave_sum_u32(d_lp);
                const uint32_t trimax = wave_max_u32(d_tri), trisum = wave_sum_u32(d_tri);
                // the stamps are per lane but the loop ran as one wave: the
                // lane with the longest walk saw all of it
                unsigned long long tin = d_tin, tleaf = d_tleaf;
                for (int o = 32; o > 0; o >>= 1) {
                        tin = max(tin, (unsigned long long)__shfl_xor((long long)tin, o, 64));
                        tleaf = max(tleaf, (unsigned long long)__shfl_xor((long long)tleaf, o, 64));
                }
                // wave-uniform sums kept by every lane while it walked: the
                // lane that walked longest holds the full totals
                const uint32_t lpm = wave_max_u32(d_phmax);
                const uint32_t lps = wave_max_u32(d_lpsum);
                if ((threadIdx.x & 63) == 0) {
                        atomicAdd(&g_phase[0], (unsigned long long)itmax);
                        atomicAdd(&g_phase[1], (unsigned long long)itsum);
                        atomicAdd(&g_phase[2], (unsigned long long)lpmax);
                        atomicAdd(&g_phase[3], (unsigned long long)lpsum);
                        atomicAdd(&g_phase[4], (unsigned long long)trimax);
                        atomicAdd(&g_phase[5], (unsigned long long)trisum);
                        atomicAdd(&g_phase[6], (unsigned long long)lpm);
                        atomicAdd(&g_phase[7], (unsigned long long)lps);
                        atomicAdd(&g_phase[8], tin);
                        atomicAdd(&g_phase[9], tleaf);
                        atomicAdd(&g_phase[11], 1ull);
                }
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                        const uint32_t t = wave_sum_u32(d_ev[e]);
                        if ((threadIdx.x & 63) == 0)
                                atomicAdd(&g_phase[12 + e], (unsigned long long)t);
                }
        }
#endif
        if (VRT_LIGHT_DIAG) {
                m.A = dg_it;
                m.L = dg_lp;
                m.T = dg_tri;
        }
        if (kCount) {
                // 1 root test + 8 per expanded node, minus the children the
                // reference never popped on the path it stopped on.
                uint32_t A = 1 + 8 * nexp;
                if (m.hit)
                        for (uint32_t lv = 1; lv <= depth; ++lv)
                                A -= path_rem[lv * kS];
                m.A = A;
        }
}

__device__ __forceinline__ RayK make_rayk(f3 o, f3 dn, float tmin, float tmax)
{
        RayK r;
        r.o = o;
        r.d = dn;
        r.dinv = mk3(dinv_of(dn.x), dinv_of(dn.y), dinv_of(dn.z));
        r.tmin = tmin;
        r.tmax = tmax;
        return r;
}

// Rays for which expand's fast path is exact (see expand_v1): finite
// origin and direction, no non-zero denormal direction component, |o| <
// 2^60 and |d| < 2^64 per component (the scene's own flag bounds the boxes
// by 2^60), so every travorder distance d.(centre - o) is finite (< 2^127):
// never NaN, a total order.
__device__ __forceinline__ bool fast_ok(const RayK &r)
{
        const float lim = 0x1p60f;
        bool ok = fabsf(r.o.x) < lim && fabsf(r.o.y) < lim && fabsf(r.o.z) < lim;
        const float d[3] = { r.d.x, r.d.y, r.d.z };
#pragma unroll
        for (int k = 0; k < 3; ++k)
                ok = ok && (d[k] == 0.f || (fabsf(d[k]) >= kFltMin && fabsf(d[k]) < 0x1p64f));
        return ok;
}

// expand_v2<2> / child_hit_mask<.., true> preconditions beyond fast_ok():
// tmax = FLT_MAX, tmin not NaN, every |dinv| <= 2^64 (finite slab distances)
__device__ __forceinline__ bool fin_ok(const RayK &r)
{
        return r.tmax == kFltMax && !isnan(r.tmin) && fabsf(r.dinv.x) <= 0x1p64f && fabsf(r.dinv.y) <= 0x1p64f &&
               fabsf(r.dinv.z) <= 0x1p64f;
}

template <bool kCount, int kS, int kUni, bool kR64, int kBudget = 0>
__device__ __forceinline__ void ray_march_dispatch(const DevScene &sc, const RayK &r,
                                                   uint2 *sb, uint32_t *sa, uint32_t *pr,
                                                   MarchResult &m)
{
        if (__all(sc.fast_ok && fast_ok(r))) {
                if (!kCount && __all(fin_ok(r)))
                        ray_march<kCount, true, kS, 2, kUni, kR64, kBudget>(sc, r, sb, sa, pr, m);
                else
                        ray_march<kCount, true, kS, 0, kUni, kR64, kBudget>(sc, r, sb, sa, pr, m);
        } else
                ray_march<kCount, false, kS, 0, kUni, kR64, kBudget>(sc, r, sb, sa, pr, m);
}

// True when ray_march's fast instantiation for camera rays is exact for
// every lane of the wave: standard range (tmin = +0, tmax = FLT_MAX) and
// finite slab distances (fin_ok).
constexpr int kFastStd = 2;
__device__ __forceinline__ bool wave_fast_std(const DevScene &sc, const RayK &r)
{
        return __all(sc.fast_ok && fast_ok(r) && __float_as_uint(r.tmin) == 0u && r.tmax == kFltMax && fin_ok(r));
}

// ---------------------------------------------------------------------------
// Occlusion query: the boolean gi::ray_march returns, without the leaf or
// triangle it found.  ray_march (VRT/voxel_octree.cc:131-188) returns true
// iff some leaf whose box and every ancestor's box pass AABB3D::isect holds a
// triangle for which intersect_triangle3 returns 1 (Triangle::isect returns
// exactly that, VRT/voxel_octree.cc:446-448; ray_march_isect returns true iff
// any record exists, :110-120).  travorder only decides WHICH such leaf is
// found first, so the boolean is the same in every child order: this walk
// visits the hit children in direction-sign order (no travorder distances,
// no sorting) and stops at the first triangle that passes the MT tests (no
// t, no inv_det, no nearest-record search).  The slab tests and MT tests are
// the same IEEE operations as ray_march's.
// ---------------------------------------------------------------------------

// The 8 children's slab tests (kFast: expand_v2's planes and v_max3/v_min3;
// otherwise expand_v1's exact select semantics) -> hit mask, bit ci.
// kFin (with kFast; the wave's rays have tmax == FLT_MAX, a tmin that is not
// NaN and every |dinv| <= 2^64, so every slab distance is finite): the
// reference's range test !(t0 > t1) && (t0 in [tmin, tmax] || t1 in [tmin,
// tmax]) is exactly max(t0, tmin) <= t1 (as expand_v2<2> with tmin = +0).
template <bool kFast, bool kFin = false>
__device__ __forceinline__ uint32_t child_hit_mask(const float bmin[3], const float bmax[3], const RayK &r)
{
        const float oo[3] = { r.o.x, r.o.y, r.o.z };
        const float di[3] = { r.dinv.x, r.dinv.y, r.dinv.z };
        float nr[3][2], fr[3][2];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
                const float h = (bmax[k] - bmin[k]) / 2.0f;
                const float a0 = kFast ? bmin[k] : bmin[k] + 0.0f * h;
                const float b = bmin[k] + h;
                const float a1 = kFast ? b : a0 + h;
                const float c = b + h;
                const float ta = (a0 - oo[k]) * di[k];
                const float tb0 = (a1 - oo[k]) * di[k];
                const float tb1 = kFast ? tb0 : (b - oo[k]) * di[k];
                const float tc = (c - oo[k]) * di[k];
                if (kFast) {
                        nr[k][0] = fminf(ta, tb0);
                        fr[k][0] = fmaxf(ta, tb0);
                        nr[k][1] = fminf(tb1, tc);
                        fr[k][1] = fmaxf(tb1, tc);
                } else {
                        nr[k][0] = std_min(ta, tb0);
                        fr[k][0] = std_max(ta, tb0);
                        nr[k][1] = std_min(tb1, tc);
                        fr[k][1] = std_max(tb1, tc);
                }
        }
        if (kFin) {
                nr[2][0] = fmaxf(nr[2][0], r.tmin);
                nr[2][1] = fmaxf(nr[2][1], r.tmin);
        }
        uint32_t hm = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
                const int mx = (i >> 2) & 1, my = (i >> 1) & 1, mz = i & 1;
                float t0, t1;
                if (kFast) {
                        asm("v_max3_f32 %0, %1, %2, %3" : "=v"(t0) : "v"(nr[0][mx]), "v"(nr[1][my]), "v"(nr[2][mz]));
                        asm("v_min3_f32 %0, %1, %2, %3" : "=v"(t1) : "v"(fr[0][mx]), "v"(fr[1][my]), "v"(fr[2][mz]));
                        if (kFin) {
                                hm |= (uint32_t)(t0 <= t1) << i;  // t0 = max(near distances, tmin)
                                continue;
                        }
                } else {
                        t0 = nr[0][mx];
                        t1 = fr[0][mx];
                        if (t0 < nr[1][my]) t0 = nr[1][my];
                        if (t0 < nr[2][mz]) t0 = nr[2][mz];
                        if (fr[1][my] < t1) t1 = fr[1][my];
                        if (fr[2][mz] < t1) t1 = fr[2][mz];
                }
                const bool h = !(t0 > t1) & (((t0 >= r.tmin) & (t0 <= r.tmax)) | ((t1 >= r.tmin) & (t1 <= r.tmax)));
                hm |= (uint32_t)h << i;
        }
        return hm;
}

// true iff some record of the leaf passes intersect_triangle3's tests
// (VRT/raytri.cc:197-249, the same operations as leaf_isect_v2)
template <bool kR64>
__device__ __forceinline__ bool leaf_any(const void *__restrict__ refs, uint32_t first, uint32_t n, const RayK &r)
{
        const double dx = r.d.x, dy = r.d.y, dz = r.d.z;
        for (uint32_t k = 0; k < n; ++k) {
                const float4 *q = kR64 ? reinterpret_cast<const float4 *>(static_cast<const RefRec64 *>(refs) + first + k)
                                       : reinterpret_cast<const float4 *>(static_cast<const RefRec48 *>(refs) + first + k);
                const float4 q0 = q[0];
                const double v0x = q0.x, v0y = q0.y, v0z = q0.z;
                const double2 *qd = reinterpret_cast<const double2 *>(q);
                float4 q1, q2;
                double2 qd1, qd2, qd3;
                double e2x, e2y, e2z;
                if (kR64) {
                        qd1 = qd[1];
                        qd2 = qd[2];
                        qd3 = qd[3];
                        e2x = qd2.y, e2y = qd3.x, e2z = qd3.y;
                } else {
                        q1 = q[1];
                        q2 = q[2];
                        e2x = (double)q1.z - v0x, e2y = (double)q1.w - v0y, e2z = (double)q2.x - v0z;
                }
                const double px = dy * e2z - dz * e2y;
                const double py = dz * e2x - dx * e2z;
                const double pz = dx * e2y - dy * e2x;
                const double e1x = kR64 ? qd1.x : (double)q0.w - v0x;
                const double e1y = kR64 ? qd1.y : (double)q1.x - v0y;
                const double e1z = kR64 ? qd2.x : (double)q1.y - v0z;
                const double det = e1x * px + e1y * py + e1z * pz;
                if (!(det > 0.000001) && !(det < -0.000001))
                        continue;
                const double tx = (double)r.o.x - v0x, ty = (double)r.o.y - v0y, tz = (double)r.o.z - v0z;
                const double uu = tx * px + ty * py + tz * pz;
                const bool pos = det > 0.000001;
                const double sdet = pos ? det : -det, suu = pos ? uu : -uu;
                if (suu < 0.0 || suu > sdet)
                        continue;
                const double qx = ty * e1z - tz * e1y;
                const double qy = tz * e1x - tx * e1z;
                const double qz = tx * e1y - ty * e1x;
                const double vv = dx * qx + dy * qy + dz * qz;
                const double svv = pos ? vv : -vv;
                if (svv < 0.0 || suu + svv > sdet)
                        continue;
                return true;
        }
        return false;
}

// The occlusion walk's state between two node visits: the child block being
// walked (base), its children still to visit (mask, bit = ci ^ s) and the
// DFS stack depth (the entries are in the lane's LDS stack column).
struct OcclState {
        uint32_t base, mask;
        int sp;
};
enum { kOcclMiss = 0, kOcclHit = 1, kOcclSpill = 2, kOcclWalk = 3 };

// The root: kOcclMiss / kOcclHit when it decides the ray (its box missed, or
// a leaf root), else kOcclWalk with w = the root's hit children.
template <bool kFast, bool kR64, bool kFin = false>
__device__ __forceinline__ int occl_start(const DevScene &sc, const RayK &r, OcclState &w)
{
        float bmin[3], bmax[3];
        uint32_t a, b;
        load_node(sc.nodes, 0, bmin, bmax, a, b);
        if (!aabb_isect(bmin, bmax, r.o, r.dinv, r.tmin, r.tmax))
                return kOcclMiss;
        if (a & kLeafBit)
                return leaf_any<kR64>(sc.refs, b, a & ~kLeafBit, r) ? kOcclHit : kOcclMiss;
        w.mask = xor_permute8(child_hit_mask<kFast, kFin>(bmin, bmax, r) & b, dir_signs(r));
        w.base = a;
        w.sp = 0;
        return kOcclWalk;
}

// The walk from state w.  kSpill: at each leaf boundary, when fewer than
// spill_t lanes of the wave are still walking (a wave-uniform decision), the
// walk stops and returns kOcclSpill with w = where it stopped.
template <bool kFast, int kS, bool kR64, bool kFin = false, bool kSpill = false>
__device__ __forceinline__ int occl_walk(const DevScene &sc, const RayK &r, uint2 *stk, OcclState &w,
                                         uint32_t spill_t = 0)
{
        float bmin[3], bmax[3];
        uint32_t a, b;
        // finite-slab walk: leaves skipped by their triangle boxes (as ray_march)
        constexpr bool kLB = kFast && kFin;
        constexpr bool kNB = kLB;  // every visited node by its triangle box
        const NodeRec *__restrict__ nodes = sc.nodes;  // kNB: xnodes instead
        const bool lbok = kLB && __all(leaf_box_ok(sc, r));  // wave-uniform: held in SGPRs
        const uint32_t s = dir_signs(r);
        uint32_t mask = w.mask;
        uint32_t base = w.base;
        int sp = w.sp;
        for (;;) {
                if (kSpill && (uint32_t)__popcll(__ballot(1)) < spill_t) {
                        w.base = base;
                        w.mask = mask;
                        w.sp = sp;
                        return kOcclSpill;
                }
                // advance to the next non-empty leaf (while-while, as ray_march)
                bool leaf = false;
                uint32_t nref = 0;
                for (;;) {
                        if (mask == 0) {
                                if (sp == 0)
                                        break;
                                --sp;
                                const uint2 e = stk[sp * kS];
                                base = e.x;
                                mask = e.y;  // pushed masks are non-zero: visit now
                        }
                        const uint32_t ci = (uint32_t)__builtin_ctz(mask) ^ s;
                        mask &= mask - 1u;
                        if (kNB) {
                                float tmn[3], tmx[3];
                                load_xnode(sc.xnodes, base + ci, bmin, bmax, a, b, tmn, tmx);
                                if (lbok && !line_meets_box(tmn, tmx, r))
                                        continue;  // no triangle below this node can pass
                        } else {
                                load_node(nodes, base + ci, bmin, bmax, a, b);
                        }
                        if (!(a & kLeafBit)) {
                                if (mask) {
                                        stk[sp * kS] = make_uint2(base, mask);
                                        ++sp;
                                }
                                mask = xor_permute8(child_hit_mask<kFast, kFin>(bmin, bmax, r) & b, s);
                                base = a;
                                continue;
                        }
                        nref = a & ~kLeafBit;  // > 0: the content mask skips empty leaves
                        leaf = true;
                        break;
                }
                if (!leaf)
                        return kOcclMiss;
                if (kR64) {
                        // large leaves: when every active lane tests the same
                        // leaf (rays of one origin), the records come through
                        // the scalar cache (as leaf_isect)
                        const uint32_t f0 = __builtin_amdgcn_readfirstlane(b);
                        const uint32_t n0 = __builtin_amdgcn_readfirstlane(nref);
                        if (__all(b == f0 && nref == n0)) {
                                if (leaf_any<true>(static_cast<const RefRec64 *>(sc.refs) + f0, 0, n0, r))
                                        return kOcclHit;
                                continue;
                        }
                }
                if (leaf_any<kR64>(sc.refs, b, nref, r))
                        return kOcclHit;
        }
}

template <bool kFast, int kS, bool kR64, bool kFin = false>
__device__ __forceinline__ bool ray_occluded(const DevScene &sc, const RayK &r, uint2 *stk)
{
        OcclState w;
        const int st = occl_start<kFast, kR64, kFin>(sc, r, w);
        if (st != kOcclWalk)
                return st == kOcclHit;
        return occl_walk<kFast, kS, kR64, kFin>(sc, r, stk, w) == kOcclHit;
}

template <int kS, bool kR64>
__device__ __forceinline__ bool ray_occluded_dispatch(const DevScene &sc, const RayK &r, uint2 *stk)
{
        // the fast walk is the finite-distance one (child_hit_mask's kFin); a
        // wave with a ray outside it (a tiny or zero direction component,
        // tmax != FLT_MAX, a NaN tmin) takes the exact walk
        if (__all(sc.fast_ok && fast_ok(r) && fin_ok(r)))
                return ray_occluded<true, kS, kR64, true>(sc, r, stk);
        return ray_occluded<false, kS, kR64>(sc, r, stk);
}

// The same walk with compaction (SpillQueues): from the root, or (resume)
// from the saved state w; returns kOcclMiss / kOcclHit, or kOcclSpill with
// w = where the walk stopped (fewer than spill_t lanes still walking).  The
// fast / exact choice is made per wave as in ray_occluded_dispatch; both
// walks keep the same state (node indices, child masks of the same hit
// children), so a state saved by one continues in the other.
template <int kS, bool kR64, bool kFastOnly = false>
__device__ __forceinline__ int occl_dispatch_spill(const DevScene &sc, const RayK &r, uint2 *stk, OcclState &w,
                                                   bool resume, uint32_t spill_t)
{
        // kFastOnly: the caller has checked that every ray of the wave takes the
        // fast walk (secondary_pixel defers the other pixels): the exact walk is
        // not compiled in
        if (kFastOnly || __all(sc.fast_ok && fast_ok(r) && fin_ok(r))) {
                if (!resume) {
                        const int st = occl_start<true, kR64, true>(sc, r, w);
                        if (st != kOcclWalk)
                                return st;
                }
                return occl_walk<true, kS, kR64, true, true>(sc, r, stk, w, spill_t);
        }
        if (!resume) {
                const int st = occl_start<false, kR64>(sc, r, w);
                if (st != kOcclWalk)
                        return st;
        }
        return occl_walk<false, kS, kR64, false, true>(sc, r, stk, w, spill_t);
}

// ---------------------------------------------------------------------------
// Pooled occlusion walk (config 5).  Only each ray's boolean is needed, and a
// ray's walk state is a set of independent subtrees -- the children left in
// the block it is walking and every DFS stack entry (a block and its
// children still to visit) -- whose answer is the OR of theirs (ray_march
// returns true iff some leaf below a box-passing path holds a triangle that
// passes, whatever the order, occl_walk).  So a wave's lanes can be one pool
// over up to 64 rays (slots): lane l starts on slot l's walk state, and
// whenever some lanes are idle, each busy lane with work to spare hands one
// piece to one idle lane -- its bottom stack entry (the shallowest pending
// block, the largest subtree set), or else the upper half of the children
// left in its current block -- through an LDS mailbox, with the slot; the
// receiver rebuilds that slot's ray (direction from LDS; origin the wave's,
// or the slot pixel's primary hit point with kSlotOrigin) and walks the
// piece on an empty stack of its own.  A leaf that passes sets its slot's bit
// of an LDS hit word; every lane walking a piece of a hit slot drops it.  The
// pool is done when no lane has work.  Returns the hit slots' mask.  The
// slab, box and MT tests are occl_walk's, so every ray's boolean is
// unchanged; only work after a ray's first passing leaf differs (pieces of
// it walked in parallel until the bit is seen at their next leaf).
// Used for the resume round of the compaction (64 saved rays of unrelated
// pixels).
// dirs: [64][3] slot directions (LDS); opix: slot -> pixel (LDS, kSlotOrigin;
// origin = prim[8 pix + 1..3]); mbox: 64 uint2 (LDS); hword: one 64-bit LDS
// word; stk: this lane's LDS stack column (stride kS) holding its initial
// state's sp entries.
// ---------------------------------------------------------------------------
template <bool kSlotOrigin>
__device__ __forceinline__ RayK pool_ray(f3 o, const float *prim, const uint32_t *opix, const float (*dirs)[3],
                                         uint32_t slot, float tmin)
{
        if (kSlotOrigin) {
                const float *pr = prim + 8 * (size_t)opix[slot];
                o = mk3(pr[1], pr[2], pr[3]);
        }
        return make_rayk(o, mk3(dirs[slot][0], dirs[slot][1], dirs[slot][2]), tmin, kFltMax);
}

template <bool kFast, int kS, bool kR64, bool kFin, bool kSlotOrigin>
__device__ __forceinline__ uint64_t occl_pool(const DevScene &sc, f3 o, const float *prim, const uint32_t *opix,
                                              float tmin, const float (*dirs)[3], uint2 *mbox,
                                              unsigned long long *hword, uint2 *stk, bool busy, uint32_t base,
                                              uint32_t mask, int sp, uint64_t hitm)
{
        constexpr bool kLB = kFast && kFin;
        constexpr bool kNB = kLB;
        const NodeRec *__restrict__ nodes = sc.nodes;  // kNB: xnodes instead
        const uint32_t lane = lane_id();
        uint32_t slot = lane;
        RayK r = pool_ray<kSlotOrigin>(o, prim, opix, dirs, slot, tmin);
        // one origin per wave (kSlotOrigin: the slots' origins all qualify)
        const bool lbok = kLB && __all(!busy || leaf_box_ok(sc, r));
        uint32_t s = dir_signs(r);
        int bot = 0;
        if (lane == 0)
                *hword = hitm;
        for (;;) {
                // hand work to idle lanes (wave-uniform decisions)
                const uint64_t idle = __ballot(!busy);
                if (idle == ~0ull)
                        break;
                const bool spare = busy && (sp > bot || __popc(mask) >= 2);
                const uint64_t don = __ballot(spare);
                if (idle != 0ull && don != 0ull) {
                        const uint32_t n = min((uint32_t)__popcll(idle), (uint32_t)__popcll(don));
                        if (spare) {
                                const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(don >> 32),
                                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)don, 0u));
                                if (k < n) {
                                        uint2 e;
                                        if (sp > bot) {
                                                e = stk[bot * kS];
                                                ++bot;
                                        } else {
                                                // keep the lower half of the children left, give the rest
                                                uint32_t give = mask;
                                                for (int c = (__popc(mask) + 1) >> 1; c > 0; --c)
                                                        give &= give - 1u;
                                                mask ^= give;
                                                e = make_uint2(base, give);
                                        }
                                        mbox[k] = make_uint2(e.x, e.y | (slot << 8));
                                }
                        }
                        wave_lds_sync();
                        if (!busy) {
                                const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                                if (k < n) {
                                        const uint2 e = mbox[k];
                                        slot = e.y >> 8;
                                        base = e.x;
                                        mask = e.y & 0xFFu;
                                        sp = bot = 0;
                                        busy = true;
                                        r = pool_ray<kSlotOrigin>(o, prim, opix, dirs, slot, tmin);
                                        s = dir_signs(r);
                                }
                        }
                        wave_lds_sync();  // the mailbox is rewritten next time
                }
                // advance to the next non-empty leaf of this lane's piece (as occl_walk)
                bool leaf = false;
                uint32_t nref = 0, b = 0;
                if (busy) {
                        float bmin[3], bmax[3];
                        uint32_t a;
                        for (;;) {
                                if (mask == 0) {
                                        if (sp == bot)
                                                break;
                                        --sp;
                                        const uint2 e = stk[sp * kS];
                                        base = e.x;
                                        mask = e.y;
                                }
                                const uint32_t ci = (uint32_t)__builtin_ctz(mask) ^ s;
                                mask &= mask - 1u;
                                if (kNB) {
                                        float tmn[3], tmx[3];
                                        load_xnode(sc.xnodes, base + ci, bmin, bmax, a, b, tmn, tmx);
                                        if (lbok && !line_meets_box(tmn, tmx, r))
                                                continue;
                                } else {
                                        load_node(nodes, base + ci, bmin, bmax, a, b);
                                }
                                if (!(a & kLeafBit)) {
                                        if (mask) {
                                                stk[sp * kS] = make_uint2(base, mask);
                                                ++sp;
                                        }
                                        mask = xor_permute8(child_hit_mask<kFast, kFin>(bmin, bmax, r) & b, s);
                                        base = a;
                                        continue;
                                }
                                nref = a & ~kLeafBit;
                                leaf = true;
                                break;
                        }
                        if (!leaf) {
                                busy = false;
                                sp = bot = 0;
                        }
                }
                bool hit = false;
                if (leaf) {
                        bool done = false;
                        if (kR64) {
                                const uint32_t f0 = __builtin_amdgcn_readfirstlane(b);
                                const uint32_t n0 = __builtin_amdgcn_readfirstlane(nref);
                                if (__all(b == f0 && nref == n0)) {
                                        hit = leaf_any<true>(sc.refs, f0, n0, r);
                                        done = true;
                                }
                        }
                        if (!done)
                                hit = leaf_any<kR64>(sc.refs, b, nref, r);
                }
                if (__ballot(hit) != 0ull) {
                        if (hit)
                                atomicOr(hword, 1ull << slot);
                        wave_lds_sync();
                        hitm = *hword;
                        if (busy && ((hitm >> slot) & 1ull)) {  // this slot is decided
                                busy = false;
                                mask = 0;
                                sp = bot = 0;
                        }
                }
        }
        return hitm;
}

// One stopped ray's record (SpillRec, 64 B): its pixel and sample, walk
// state and direction, the stack entries copied out of the lane's LDS column
// (block << 8 | children left: blocks < 2^24, spill_setup).
template <int kS>
__device__ __forceinline__ void spill_write(SpillRec *o, uint32_t pix, uint32_t sample, f3 d, const OcclState &w,
                                            const uint2 *stk)
{
        uint4 *q = reinterpret_cast<uint4 *>(o);
        q[0] = make_uint4(pix | sample << 26, w.base, w.mask | (uint32_t)w.sp << 8, __float_as_uint(d.x));
        q[1].x = __float_as_uint(d.y);
        q[1].y = __float_as_uint(d.z);
        for (int k = 0; k < w.sp; ++k) {
                const uint2 e = stk[k * kS];
                o->stk[k] = e.x << 8 | e.y;
        }
}

// A record's walk state back: (pix | sample << 26, base, mask | sp << 8, d)
// into h / d, its stack entries into the lane's LDS column (stride kS).
template <int kS>
__device__ __forceinline__ void spill_read(const SpillRec *q, uint4 &h, f3 &d, uint2 *stk)
{
        h = reinterpret_cast<const uint4 *>(q)[0];
        const uint2 t = reinterpret_cast<const uint2 *>(q)[2];
        d = mk3(__uint_as_float(h.w), __uint_as_float(t.x), __uint_as_float(t.y));
        const int sp = (int)(h.z >> 8);
        for (int k = 0; k < sp; ++k) {
                const uint32_t e = q->stk[k];
                stk[k * kS] = make_uint2(e >> 8, e & 0xFFu);
        }
}

// (float)spp at the point of use: the compiler otherwise hoists the
// conversion out of the persistent loops into a VGPR it spills
__device__ __forceinline__ float spp_f(int32_t spp)
{
        asm volatile("" : "+s"(spp));
        return (float)spp;
}

// lane 0 adds n to *ctr, the wave reads lane 0's result (as take_unit)
__device__ __forceinline__ uint32_t take_n(uint32_t *ctr, uint32_t n)
{
        int lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        const uint32_t old = atomicAdd(ctr, lane == 0 ? n : 0u);
        return __builtin_amdgcn_readlane(old, 0);
}

// A wave's place in a compaction queue (SpillQueues): the chunk it fills and
// the records in it so far (wave-uniform).
constexpr uint32_t kSpillNone = 0xFFFFFFFFu;  // no chunk yet
constexpr uint32_t kSpillFull = 0xFFFFFFFEu;  // the queue has no chunk left
struct SpillCursor {
        uint32_t chunk, fill;
};

// The chunk's fill count, for the round that reads the queue, and the
// queue's record total (ctr[2], vrt_secondary_spill_counts).  Every lane
// active: the total is one folded whole-wave add (as take_unit).
__device__ __forceinline__ void spill_close(uint32_t *fills, uint32_t *ctr, const SpillCursor &c)
{
        if (c.chunk >= kSpillFull)
                return;
        int lane;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        if (lane == 0)
                fills[c.chunk] = c.fill;
        atomicAdd(ctr + 2, lane == 0 ? c.fill : 0u);
}

// The stop threshold a group of rays may use: t, or 0 (no compaction, or
// the queue was found full).
__device__ __forceinline__ uint32_t spill_threshold(const SpillQueues &q, const SpillCursor &c, uint32_t t)
{
        return (q.nchunks == 0 || t == 0 || c.chunk == kSpillFull) ? 0u : t;
}

// After a group's walks, n > 0 of its rays stopped (every lane active,
// wave-uniform): room for n more records in the cursor's chunk, taking the
// queue's next chunk when they do not fit -- so chunks fill up whatever the
// group sizes.  false: the queue is full (the caller finishes those rays in
// place); their count goes to ctr[5] (the host sizes the next frame's queue
// from ctr[2] + ctr[5]).
__device__ __forceinline__ bool spill_room(const SpillQueues &q, uint32_t *ctr, uint32_t *fills, SpillCursor &c,
                                           uint32_t n)
{
        if (c.chunk != kSpillFull && c.chunk != kSpillNone && c.fill + n <= kSpillChunk)
                return true;
        if (c.chunk != kSpillFull) {
                spill_close(fills, ctr, c);
                const uint32_t k = take_n(ctr, 1u);
                c.chunk = k < q.nchunks ? k : kSpillFull;
                c.fill = 0;
        }
        if (c.chunk != kSpillFull)
                return true;
        take_n(ctr + 5, n);
        return false;
}

// The stopped rays of a group (`spilled`, after the walks): each writes its
// record at the cursor's next free slots in lane order.
template <int kS>
__device__ __forceinline__ void spill_group(SpillRec *rec, SpillCursor &c, bool spilled, uint32_t pix,
                                            uint32_t sample, f3 d, const OcclState &w, const uint2 *stk)
{
        const uint64_t sm = __ballot(spilled);
        if (sm == 0)
                return;
        if (spilled) {
                const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u));
                spill_write<kS>(rec + (size_t)c.chunk * kSpillChunk + c.fill + below, pix, sample, d, w, stk);
        }
        c.fill += (uint32_t)__popcll(sm);
}


// Triangle::get_albedo (VRT/voxel_octree.cc:472-484) with Triangle::isect's
// normal (VRT/voxel_octree.cc:451-453).
__device__ __forceinline__ f3 hit_albedo(const DevScene &sc, const MarchResult &m, f3 &normal)
{
        const TriAttr *ta = sc.tri_attr + m.tri;
        const float4 *q = reinterpret_cast<const float4 *>(ta);
        const float4 a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3];
        // the vertices (textured materials only) are loaded beside the
        // attributes, not after the material that says they are needed
        const float4 *pp = reinterpret_cast<const float4 *>(sc.tri_pos + m.tri);
        const float4 p0 = pp[0], p1 = pp[1], p2 = pp[2];
        const f3 n0 = mk3(a0.x, a0.y, a0.z), n1 = mk3(a0.w, a1.x, a1.y),
                 n2 = mk3(a1.z, a1.w, a2.x);
        const float t0u = a2.y, t0v = a2.z, t1u = a2.w, t1v = a3.x,
                    t2u = a3.y, t2v = a3.z;
        const int mat = __float_as_int(a3.w);
        const float w = clampf(1.0f - m.u - m.v, 0, 1);
        normal = normalize((n0 * w + n1 * m.u) + n2 * m.v);
        const MatRec mr = sc.mats[mat];
        f3 albedo;
        if (mr.tex < 0) {
                albedo = mk3(mr.kd[0], mr.kd[1], mr.kd[2]);
        } else {
                f3 bc = barycentric(m.hp, mk3(p0.x, p0.y, p0.z),
                                    mk3(p0.w, p1.x, p1.y),
                                    mk3(p1.z, p1.w, p2.x));
                bc.x = clampf(bc.x, 0.f, 1.f);
                bc.y = clampf(bc.y, 0.f, 1.f);
                bc.z = clampf(bc.z, 0.f, 1.f);
                const float tu = (bc.x * t0u + bc.y * t1u) + bc.z * t2u;
                const float tv = (bc.x * t0v + bc.y * t1v) + bc.z * t2v;
                const TexRec tx = mr.tx;  // texs[mr.tex], inline
                const int x = clampi((int)(unit_cycle(tu) * (float)tx.w), 0, tx.w - 1);
                int y = clampi((int)(unit_cycle(tv) * (float)tx.h), 0, tx.h - 1);
                y = tx.h - 1 - y;
                const uint8_t *p = sc.tex_data + tx.off +
                                   ((int64_t)y * tx.w + x) * tx.c;
                const float c0 = (float)p[0];
                const float c1 = tx.c > 1 ? (float)p[1] : 0.f;
                const float c2 = tx.c > 2 ? (float)p[2] : 0.f;
                albedo = mk3(c0 / 255.f, c1 / 255.f, c2 / 255.f);
        }
        return albedo;
}

// Triangle::get_diffuse(isect, ray, (1,1,1)) (VRT/voxel_octree.cc:462-470)
__device__ __forceinline__ f3 shade_hit(const DevScene &sc, const RayK &r,
                                        const MarchResult &m, f3 &normal)
{
        const f3 albedo = hit_albedo(sc, m, normal);
        float tmp = dot(normal, -r.d);
        tmp = clampf(tmp, 0.f, 1.f);
        const f3 c = albedo * tmp;
        return mk3(c.x * 1.0f, c.y * 1.0f, c.z * 1.0f);  // * color (1,1,1)
}

// ---------------------------------------------------------------------------
// Primary render: an 8x8 tile = 4 waves of 4x4 pixels x 4 samples, one wave
// per workgroup (a finished wave frees its slot and LDS at once).
// ---------------------------------------------------------------------------
// This rank's k-th tile (wave-uniform k): one rank with a magic divisor ->
// one multiply (RenderParams::ntx_magic: the raster order deal_tile gives one
// rank); several ranks with a tabled deal -> one scalar load (tile_xy);
// otherwise deal_tile itself.
__device__ __forceinline__ void rank_tile(int ntx, int nty, int nr, int rk, uint64_t magic, const uint32_t *tab,
                                          int k, int &tx, int &ty)
{
        if (nr == 1 && magic) {
                const uint32_t q = (uint32_t)(((uint64_t)(uint32_t)k * magic) >> 40);
                ty = (int)q;
                tx = k - (int)q * ntx;
        } else if (tab) {
                // constant address space, wave-uniform index: a scalar load
                typedef const __attribute__((address_space(4))) uint32_t ConstU;
                const uint32_t v = ((ConstU *)tab)[k];
                tx = (int)(v & 0xFFFFu);
                ty = (int)(v >> 16);
        } else {
                deal_tile(tile_deal(ntx, nty, nr), rk, k, tx, ty);
        }
}

constexpr int kRenderBlock = 64;
// One work unit of the primary render: the 4x4-pixel quadrant `wave` of
// this rank's k-th 8x8 tile, 4 gen_rays4 samples per pixel, one ray per
// lane (lane = 4*pixel + sample).  stk_* are this lane's LDS stack columns.
// kSamples: the per-sample outputs p.so may be set (k_render); the
// persistent kernels never write them.  kFastOnly: only ray_march's fast,
// standard-range instantiation is compiled in (fewer live registers); a wave
// whose rays need another path returns false before writing anything and the
// caller defers the unit to k_render_defer.
template <bool kCount, bool kR64, int kS, bool kSamples = true, bool kFastOnly = false>
__device__ __forceinline__ bool render_unit(const RenderParams &p, int k, int wave, int lane, uint2 *stk,
                                            uint32_t *stk_aux, uint32_t *path_rem)
{
        // the lane id is re-read per unit (volatile asm: not hoisted out of
        // a persistent loop), so its derived per-lane constants are
        // recomputed instead of being held -- and spilled -- across units
        auto lane_now = [&]() {
                int l = lane;
                if (!kSamples)
                        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
                return l;
        };
#if VRT_PHASE_STAMPS
        const unsigned long long d_r0 = __builtin_amdgcn_s_memtime();
#endif
        const CamParams &c = p.cam;
        int tx, ty;
        {
                // the deal's sizes pass through an opaque copy per unit, so
                // the divisions they feed are redone per unit (a few scalar
                // instructions) rather than hoisted as loop invariants that
                // hold SGPRs -- and spill -- across every march
                int ntx = p.ntx, nty = p.nty, nr = p.nranks, rk = p.rank;
                if (!kSamples)
                        asm volatile("" : "+s"(ntx), "+s"(nty), "+s"(nr), "+s"(rk));
                rank_tile(ntx, nty, nr, rk, p.ntx_magic, p.tile_xy, k, tx, ty);
                // the tile is wave-uniform: keep it in SGPRs (the deal's
                // divisions may run on the VALU), not in VGPRs held -- and
                // spilled -- across the march
                tx = __builtin_amdgcn_readfirstlane(tx);
                ty = __builtin_amdgcn_readfirstlane(ty);
        }
        ty += p.ty0;
        // pixel, sample and Camera::gen_rays4 direction (VRT/camera.cc:95-112)
        // of lane l
        auto sample_of = [&](int l, int &px, int &py, int &s, int &lx, int &ly) {
                s = l & 3;
                const int pix = l >> 2;
                // unit = a 4x4 quadrant of the tile
                lx = (wave & 1) * 4 + (pix & 3);
                ly = (wave >> 1) * 4 + (pix >> 2);
                px = tx * 8 + lx;
                py = ty * 8 + ly;
                // opaque per unit, as the deal's sizes above: the film size and
                // the camera terms that are the same for every ray (nf * z, e *
                // 0) are recomputed per unit, not held in VGPRs across marches
                int nx = c.nx, ny = c.ny;
                float nf[3] = { c.nf[0], c.nf[1], c.nf[2] }, e[3] = { c.e[0], c.e[1], c.e[2] }, z = c.z;
                if (!kSamples)
                        asm volatile("" : "+s"(nx), "+s"(ny), "+s"(nf[0]), "+s"(nf[1]), "+s"(nf[2]), "+s"(e[0]),
                                     "+s"(e[1]), "+s"(e[2]), "+s"(z));
                return camera_dir(c.s, c.u, nf, e, z, nx, ny, px, py, sample_x(s), sample_y(s));
        };
        int px, py, s, lx, ly;
        f3 dn = sample_of(lane_now(), px, py, s, lx, ly);
        const RayK r = make_rayk(mk3(c.origin[0], c.origin[1], c.origin[2]), dn, c.tmin, c.tmax);

        MarchResult m;
#if VRT_PHASE_STAMPS
        unsigned long long d_m1 = 0;
#endif
        if (kFastOnly) {
                if (!wave_fast_std(p.sc, r) || (p.test_flags & VRT_TEST_FORCE_DEFER))
                        return false;
#if VRT_PHASE_STAMPS
                const unsigned long long d_m0 = __builtin_amdgcn_s_memtime();
                if (lane_now() == 0)
                        atomicAdd(&g_phase[21], d_m0 - d_r0);
#endif
                ray_march<false, true, kS, kFastStd, true, kR64>(p.sc, r, stk, nullptr, nullptr, m);
#if VRT_PHASE_STAMPS
                d_m1 = __builtin_amdgcn_s_memtime();
                if (lane_now() == 0)
                        atomicAdd(&g_phase[22], d_m1 - d_m0);
#endif
        } else {
                ray_march_dispatch<kCount, kS, true, kR64>(p.sc, r, stk, stk_aux, path_rem, m);
        }
#if VRT_UNIT_DIAG && VRT_LIGHT_DIAG
        if (kFastOnly) {
                const uint32_t v[4] = { wave_max_u32(m.A), wave_sum_u32(m.A), wave_max_u32(m.T), wave_sum_u32(m.T) };
                const int ku = k * 4 + wave;
                if (lane < 4 && ku < kUnitDiagMax)
                        g_unit_walk[(size_t)ku * 4 + lane] = lane == 0 ? v[0] : lane == 1 ? v[1] : lane == 2 ? v[2] : v[3];
        }
#endif
        // persistent kernels: the pixel is made again -- the same
        // operations, so the same bits -- rather than held live across the
        // march
        if (!kSamples)
                (void)sample_of(lane_now(), px, py, s, lx, ly);

        f3 col;
        if (m.hit) {
                f3 nrm;
                RayK rs;  // shade_hit reads the direction only
                rs.d = dn;
                col = shade_hit(p.sc, rs, m, nrm);
        } else {
                col = sky(dn.y);
        }
        lane = lane_now();

        const size_t si = ((size_t)py * c.nx + px) * 4 + s;
        if (kSamples) {
                if (p.so.hit) p.so.hit[si] = m.hit ? 1 : 0;
                if (p.so.tri) p.so.tri[si] = m.hit ? (int32_t)m.tri : -1;
                if (p.so.vox) p.so.vox[si] = m.hit ? p.sc.node_vox[m.node] : 0xFFFFFFFFu;
                if (p.so.rgb) {
                        p.so.rgb[3 * si + 0] = col.x;
                        p.so.rgb[3 * si + 1] = col.y;
                        p.so.rgb[3 * si + 2] = col.z;
                }
        }
        if (kCount && p.so.cnt) {
                p.so.cnt[4 * si + 0] = m.A;
                p.so.cnt[4 * si + 1] = m.L;
                p.so.cnt[4 * si + 2] = m.T;
                p.so.cnt[4 * si + 3] = m.hit ? 1u : 0u;
        }

        // Film::add(px, py, c * .25f) for samples 0..3 in order, starting
        // from the zero-initialised film (VRT/camera.cc:17-20, main.cc:121).
        const f3 cq = col * .25f;
        const int l0 = lane & ~3;
        float acc[3] = { 0.0f, 0.0f, 0.0f };
        const float cv[3] = { cq.x, cq.y, cq.z };
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int q = 0; q < 3; ++q)  // lane l0 + j's value (a wave64 permute by our own lane id)
                        acc[q] += __int_as_float(__builtin_amdgcn_ds_bpermute((l0 + j) << 2, __float_as_int(cv[q])));
        }
        if (s == 0) {
                float *o;
                if (p.image_layout)
                        o = p.out + ((size_t)py * c.nx + px) * 3;
                else
                        o = p.out + ((size_t)k * 64 + ly * 8 + lx) * 3;
                o[0] = acc[0];
                o[1] = acc[1];
                o[2] = acc[2];
        }
#if VRT_PHASE_STAMPS
        if (kFastOnly && lane_now() == 0)
                atomicAdd(&g_phase[23], __builtin_amdgcn_s_memtime() - d_m1);
#endif
        return true;
}

template <bool kCount, bool kR64>
#ifndef VRT_WAVES_PER_EU
// 6 waves per SIMD (80 VGPRs, a 32-B/lane spill) measured 8% faster than
// the unconstrained 4 waves/SIMD (99 VGPRs): the march is latency-bound.
#define VRT_WAVES_PER_EU 6
#endif
__global__ __launch_bounds__(kRenderBlock, kCount ? 1 : VRT_WAVES_PER_EU) void k_render(RenderParams p)
{
        constexpr int kB = kRenderBlock;
        __shared__ uint2 stk[kStack * kB];
        __shared__ uint32_t stk_aux[kCount ? kStack * kB : 1];
        __shared__ uint32_t path_rem[kCount ? (kStack + 1) * kB : 1];

        const int tid = threadIdx.x;
        // XCD-aware order: blocks b, b+8, ... run on one XCD; give them
        // consecutive work units (a unit = kUnitsPerTile-th of an 8x8 tile)
        // so each XCD's L2 serves one screen region.
        constexpr int kQ = 4;  // units per tile
        const int nb = gridDim.x;
        const int b = blockIdx.x;
        const int per = (nb + 7) >> 3;
        const int xcd = b & 7, slot = b >> 3;
        int u = xcd * per + slot;
        if ((nb & 7) != 0) {
                // uneven grid: fall back to the identity map
                u = b;
        }
        if (u >= p.tiles_this_rank * kQ)
                return;
        const int k = u / kQ;
        const int wave = (u % kQ) + (tid >> 6), lane = tid & 63;
        render_unit<kCount, kR64, kB>(p, k, wave, lane, stk + tid, stk_aux + (kCount ? tid : 0),
                                      path_rem + (kCount ? tid : 0));
}

// One dequeue from a WorkQueue counter for the whole wave: every lane takes
// part in the add (lane 0 adds 1, the others 0; the compiler folds that into
// one atomic) and the wave reads lane 0's result.  No lane-0-only branch
// around the atomic: inside k_secondary_p's persistent loop that divergent
// region was structurized into a loop that re-ran one pixel forever.
__device__ __forceinline__ uint32_t take_unit(uint32_t *ctr)
{
        int lane;  // read here, not held across the persistent loop
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        const uint32_t old = atomicAdd(ctr, lane == 0 ? 1u : 0u);
        return __builtin_amdgcn_readlane(old, 0);
}

// Persistent variant (uninstrumented, no per-sample outputs): 4-wave
// workgroups sized to fill the chip once; every wave pulls quadrant units
// from a per-XCD counter (blocks b, b+8, ... share an XCD and its L2; an
// XCD's counter covers slice x of the units, 512-unit chunks dealt round
// robin to the 8 slices, slice_unit) and, once its own slice is exhausted,
// from the next XCD's counter (kPersistHelp).
// At VRT_PERSIST_WAVES_PER_EU = 6 (80 VGPRs, no scratch) the 256-thread
// workgroups keep 6 waves per SIMD = 24 per CU resident; the waves of a
// workgroup share nothing but its LDS stack array, so none waits for a
// sibling.  The counters belong to this launch alone (WorkQueue,
// vrt_internal.h): nothing is reset at the end.
// kFastOnly (camera rays of a finite scene, decided on the host): only the
// fast standard-range march is compiled in; a wave with a ray that needs the
// exact path (a non-zero denormal direction component) appends its unit to
// the launch's deferred list, which k_render_defer renders afterwards.
constexpr int kPersistBlock = 256;
// Block slots (256 threads, 4 waves each) a persistent launch for one rank of
// a multi-GPU frame leaves free, so the RCCL kernel moving the previous frame
// finds CU room beside the persistent grid instead of waiting for it to
// drain: 32 of ~1280 resident slots, a multiple of 8 (the XCD map needs a
// grid of whole XCD rounds).
constexpr int kCollectiveReserve = 32;
// Slices a wave takes units from: its XCD's own, then the next one's.  The
// chunked slices drain together, so one helper XCD per slice is enough:
// 2 beats 8 by 3.6 % on a full frame and 3.8 % on an 8-rank share, 1 loses
// 1 % on a full frame.
constexpr int kPersistHelp = 2;
#ifndef VRT_PERSIST_WAVES_PER_EU
#define VRT_PERSIST_WAVES_PER_EU 6
#endif
template <bool kFastOnly>
__global__ __launch_bounds__(kPersistBlock, VRT_PERSIST_WAVES_PER_EU) void k_render_p(RenderParams p)
{
        __shared__ uint2 stk[kStack * kPersistBlock];
        const int tid = threadIdx.x, lane = tid & 63;
        const int xcd = blockIdx.x & 7;
        for (int j = 0; j < kPersistHelp; ++j) {
                const int x = (xcd + j) & 7;
                const int units = p.tiles_this_rank * 4, n = slice_size(units, x, VRT_SLICE_CHUNK);
                if (n <= 0)
                        continue;
                for (;;) {
#if VRT_PHASE_STAMPS
                        const unsigned long long d_q0 = __builtin_amdgcn_s_memtime();
#endif
                        const uint32_t u = take_unit(p.q.ctr + x * kQueueStride) - p.q.base[x];
#if VRT_PHASE_STAMPS
                        if (lane == 0)
                                atomicAdd(&g_phase[20], __builtin_amdgcn_s_memtime() - d_q0);
#endif
                        if (u >= (uint32_t)n)
                                break;
                        const int kq = slice_unit(units, x, (int)u, VRT_SLICE_CHUNK);
#if VRT_PHASE_STAMPS
                        const unsigned long long d_u0 = __builtin_amdgcn_s_memtime();
#endif
#if VRT_UNIT_DIAG
                        const uint32_t dg_u0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
                        const bool done = render_unit<false, false, kPersistBlock, false, kFastOnly>(
                                p, kq >> 2, kq & 3, lane, stk + tid, nullptr, nullptr);
#if VRT_UNIT_DIAG
                        {
                                const uint32_t dg_u1 = (uint32_t)__builtin_amdgcn_s_memrealtime();
                                const uint32_t v[4] = { dg_u0, dg_u1, (uint32_t)(blockIdx.x * 4 + (tid >> 6)),
                                                        (uint32_t)x };
                                if (lane < 4 && kq < kUnitDiagMax)
                                        g_unit_diag[(size_t)kq * 4 + lane] =
                                                lane == 0 ? v[0] : lane == 1 ? v[1] : lane == 2 ? v[2] : v[3];
                        }
#endif
#if VRT_PHASE_STAMPS
                        if (lane == 0)
                                atomicAdd(&g_phase[10], __builtin_amdgcn_s_memtime() - d_u0);
#endif
                        // `done` is wave-uniform (wave_fast_std is a whole-wave
                        // vote): the append is one whole-wave take_unit, never
                        // a lane-0-only atomic inside this loop, and every lane
                        // stores the same word
                        if (!done) {
                                // past the cap the slice is re-rendered whole: no more appends
                                uint32_t *cnt = p.q.defer + x * kQueueStride + kDeferCount;
                                const uint32_t c = __builtin_amdgcn_readfirstlane(
                                        __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                                if (c <= (uint32_t)kDeferSliceCap) {
                                        const uint32_t d = take_unit(cnt);
                                        if (d < (uint32_t)kDeferSliceCap)
                                                p.q.defer[kDeferList + x * kDeferSliceCap + d] = (uint32_t)kq;
                                }
                        }
                }
        }
}

// The units k_render_p<true> deferred (normally none), rendered with the
// general march (ray_march_dispatch) by half as many workgroups as the
// persistent launch (so even a frame whose every unit was deferred runs on
// half the resident slots; a latency-bound march loses far less than half
// its rate).  No deferred unit: every wave returns after 8 scalar loads.
// Otherwise each wave walks the XCD slices like k_render_p (its own first),
// taking a slice's list entries -- or, past kDeferSliceCap, every unit of
// the slice (the render is deterministic, so units already written are
// rewritten with the same values) -- from the slice's take counter with
// whole-wave atomics; the last wave to finish zeroes the counts and
// counters for the queue slot's next launch (every other wave has finished
// reading them: its done-add follows its last, returned, take).
__global__ __launch_bounds__(kPersistBlock, VRT_PERSIST_WAVES_PER_EU) void k_render_defer(RenderParams p)
{
        __shared__ uint2 stk[kStack * kPersistBlock];
        const int tid = threadIdx.x, lane = tid & 63;
        uint32_t any = 0;
#pragma unroll
        for (int x = 0; x < 8; ++x)
                any |= __builtin_amdgcn_readfirstlane(p.q.defer[x * kQueueStride + kDeferCount]);
        if (any == 0u)
                return;
        const int xcd = blockIdx.x & 7;
        for (int j = 0; j < 8; ++j) {
                const int x = (xcd + j) & 7;
                const uint32_t n = __builtin_amdgcn_readfirstlane(p.q.defer[x * kQueueStride + kDeferCount]);
                if (n == 0u)
                        continue;
                const int units = p.tiles_this_rank * 4;
                const bool all = n > (uint32_t)kDeferSliceCap;
                const uint32_t m = all ? (uint32_t)slice_size(units, x, VRT_SLICE_CHUNK) : n;
                for (;;) {
                        const uint32_t i = take_unit(p.q.defer + x * kQueueStride + kDeferTake);
                        if (i >= m)
                                break;
                        const uint32_t unit = all ? (uint32_t)slice_unit(units, x, (int)i, VRT_SLICE_CHUNK)
                                                  : __builtin_amdgcn_readfirstlane(
                                                            p.q.defer[kDeferList + x * kDeferSliceCap + i]);
                        render_unit<false, false, kPersistBlock, false, false>(
                                p, (int)(unit >> 2), (int)(unit & 3), lane, stk + tid, nullptr, nullptr);
                }
        }
        const uint32_t fin = take_unit(p.q.defer + kDeferDoneWord);
        if (fin == gridDim.x * (uint32_t)(kPersistBlock / 64) - 1u) {
#pragma unroll
                for (int x = 0; x < 8; ++x) {
                        p.q.defer[x * kQueueStride + kDeferCount] = 0u;
                        p.q.defer[x * kQueueStride + kDeferTake] = 0u;
                }
                p.q.defer[kDeferDoneWord] = 0u;
        }
}

// ---------------------------------------------------------------------------
// Batched gi::ray_march over arbitrary rays: one ray per lane.
// Output record = vrt_hit {hit, tri, voxel, hit_p[3], normal[3]} (36 B).
// ---------------------------------------------------------------------------
template <bool kR64>
__global__ __launch_bounds__(kBlock) void k_ray_march(DevScene sc,
                                                      const float *__restrict__ rays,
                                                      int64_t n,
                                                      uint32_t *__restrict__ out)
{
        __shared__ uint2 stk[kStack * kBlock];
        const int tid = threadIdx.x;
        const int64_t i = (int64_t)blockIdx.x * kBlock + tid;
        if (i >= n)
                return;
        const float *rr = rays + 8 * i;
        const RayK r = make_rayk(mk3(rr[0], rr[1], rr[2]), mk3(rr[3], rr[4], rr[5]),
                                 rr[6], rr[7]);
        MarchResult m;
        ray_march_dispatch<false, kBlock, true, kR64>(sc, r, stk + tid, nullptr, nullptr, m);
        uint32_t *o = out + 9 * i;
        if (m.hit) {
                f3 nrm;
                const TriAttr *ta = sc.tri_attr + m.tri;
                const f3 n0 = mk3(ta->n[0], ta->n[1], ta->n[2]);
                const f3 n1 = mk3(ta->n[3], ta->n[4], ta->n[5]);
                const f3 n2 = mk3(ta->n[6], ta->n[7], ta->n[8]);
                const float w = clampf(1.0f - m.u - m.v, 0, 1);
                nrm = normalize((n0 * w + n1 * m.u) + n2 * m.v);
                o[0] = 1;
                o[1] = m.tri;
                o[2] = sc.node_vox[m.node];
                o[3] = __float_as_uint(m.hp.x);
                o[4] = __float_as_uint(m.hp.y);
                o[5] = __float_as_uint(m.hp.z);
                o[6] = __float_as_uint(nrm.x);
                o[7] = __float_as_uint(nrm.y);
                o[8] = __float_as_uint(nrm.z);
        } else {
                o[0] = 0;
                o[1] = 0xFFFFFFFFu;
                o[2] = 0xFFFFFFFFu;
                for (int q = 3; q < 9; ++q)
                        o[q] = 0;
        }
}

// ---------------------------------------------------------------------------
// Config 5: one primary hit per pixel, then `spp` stochastic
// secondary rays Ray{hit, normal + random_point_in_unit_sphere(pcg), res}.
// ---------------------------------------------------------------------------
constexpr uint64_t kPcgMul = 6364136223846793005ULL;
constexpr uint64_t kPcgInc = 1442695040888963407ULL;

// jql::PCG::operator() (VRT/graphics_math.h:836-849)
__device__ __forceinline__ uint32_t pcg_next(uint64_t &s)
{
        s = s * kPcgMul + kPcgInc;
        const uint32_t xorshift = (uint32_t)((s ^ (s >> 18u)) >> 27u);
        const uint32_t shift = (uint32_t)(s >> 59u);
        return (xorshift >> shift) | (xorshift << ((0u - shift) & 31u));
}

// libstdc++ 11 uniform_real_distribution<float>{-1,1}: generate_canonical
// <float,24> = float(g) / 2^32 (clamped below 1), then u * 2 + -1.
__device__ __forceinline__ float uniform_m11(uint64_t &s)
{
        float sum = 0.0f;
        sum += (float)pcg_next(s) * 1.0f;
        float ret = sum / 4294967296.0f;
        if (ret >= 1.0f)
                ret = 0.99999994f;  // nextafter(1.f, 0.f)
        return (ret * (1.0f - -1.0f)) + -1.0f;
}

// State after n more LCG steps (O(log n) jump-ahead, mod 2^64).
__device__ __forceinline__ uint64_t pcg_advance(uint64_t s, uint64_t n)
{
        uint64_t am = 1, ap = 0, cm = kPcgMul, cp = kPcgInc;
        while (n) {
                if (n & 1) {
                        am *= cm;
                        ap = ap * cm + cp;
                }
                cp = (cm + 1) * cp;
                cm *= cm;
                n >>= 1;
        }
        return am * s + ap;
}

// pcg_advance(s, 3 * lane) for the 64 lanes as (multiplier, increment)
// pairs, made at compile time by the same loop: a pixel's lane-staggered
// start state is one 16-B load and a 64-bit multiply-add instead of a
// divergent 8-step jump with four 64-bit products per step.
struct PcgJump3 {
        uint64_t ac[64][2];
        constexpr PcgJump3() : ac()
        {
                for (int l = 0; l < 64; ++l) {
                        uint64_t n = 3u * (uint64_t)l, am = 1, ap = 0, cm = kPcgMul, cp = kPcgInc;
                        while (n) {
                                if (n & 1) {
                                        am *= cm;
                                        ap = ap * cm + cp;
                                }
                                cp = (cm + 1) * cp;
                                cm *= cm;
                                n >>= 1;
                        }
                        ac[l][0] = am;
                        ac[l][1] = ap;
                }
        }
};
__constant__ PcgJump3 c_pcg_jump3 = PcgJump3();

// Pass 1: pixel-centre primary ray (Camera::gen_rays1, VRT/camera.cc:77-93)
// over the 8*(n/8) render area, one pixel per lane -> {hit, hit xyz, normal}.
template <bool kR64>
__global__ __launch_bounds__(kBlock) void k_primary1(RenderParams p, float *__restrict__ prim)
{
        __shared__ uint2 stk[kStack * kBlock];
        const int tid = threadIdx.x;
        const int W8 = 8 * p.ntx;
        // a wave per 8x8 tile (lane = 8 * row + column; tiles in raster
        // order): 64 neighbouring rays walk much the same nodes, where a
        // 64-pixel row strip spreads them 8x wider
        const int64_t t = (int64_t)blockIdx.x * (kBlock / 64) + (tid >> 6);
        if (t >= (int64_t)p.ntx * p.nty)
                return;
        const int px = (int)(t % p.ntx) * 8 + (tid & 7), py = (int)(t / p.ntx) * 8 + ((tid >> 3) & 7);
        const int64_t i = (int64_t)py * W8 + px;
        const CamParams &c = p.cam;
        const f3 dn = camera_dir(c.s, c.u, c.nf, c.e, c.z, c.nx, c.ny, px, py, 0.5f, 0.5f);
        const RayK r = make_rayk(mk3(c.origin[0], c.origin[1], c.origin[2]), dn, c.tmin, c.tmax);
        MarchResult m;
        ray_march_dispatch<false, kBlock, true, kR64>(p.sc, r, stk + tid, nullptr, nullptr, m);
        float *o = prim + 8 * i;
        if (!m.hit) {
                o[0] = 0.f;
                return;
        }
        const TriAttr *ta = p.sc.tri_attr + m.tri;
        const f3 n0 = mk3(ta->n[0], ta->n[1], ta->n[2]);
        const f3 n1 = mk3(ta->n[3], ta->n[4], ta->n[5]);
        const f3 n2 = mk3(ta->n[6], ta->n[7], ta->n[8]);
        const float w = clampf(1.0f - m.u - m.v, 0, 1);
        const f3 nrm = normalize((n0 * w + n1 * m.u) + n2 * m.v);
        o[0] = 1.f;
        o[1] = m.hp.x;
        o[2] = m.hp.y;
        o[3] = m.hp.z;
        o[4] = nrm.x;
        o[5] = nrm.y;
        o[6] = nrm.z;
}

// Pass 2: one wave per pixel, lane s = secondary ray s.  The reference
// draws points sequentially (rejection sampling, 3 draws per attempt); here
// lane l evaluates attempt l (+64 per round) from a jump-ahead PCG state and
// the accepted attempts are ranked in attempt order with a ballot, so ray s
// gets exactly the reference's s-th accepted point.
struct SecondaryParams {
        DevScene sc;
        const uint32_t *tile_xy;  // nranks > 1: the rank's tiles (RenderParams::tile_xy) or nullptr
        int32_t nx, W8, H8, spp;
        int32_t rank, nranks;  // this rank's 8x8 tiles: tile_deal
        float res;
        float *prim;           // 8 floats per pixel: k_primary1's record, [7] the compaction counts
        float *vis;            // nx*ny, this rank's pixels written
        int32_t *s_hit, *s_tri;
        uint32_t *s_vox;
        int32_t units;         // this rank's pixels (persistent launch)
        int32_t test_flags;    // VRT_TEST_SEC_DEFER
        WorkQueue q;           // persistent launch only
        SpillQueues sq;        // ray compaction (kAny, persistent launch); sq.nchunks == 0: off
};

// the persistent config-5 kernels (k_secondary_p, k_sec_resume): 4-wave workgroups
constexpr int kSecPBlock = 256;
// pixels a k_secondary_p wave takes per dequeue (one device-scope atomic)
#ifndef VRT_SEC_TAKE
#define VRT_SEC_TAKE 2
#endif
constexpr uint32_t kSecTake = VRT_SEC_TAKE;
static_assert(kSecTake >= 1, "VRT_SEC_TAKE");
#ifndef VRT_SECP_WAVES_PER_EU
#define VRT_SECP_WAVES_PER_EU 6
#endif

// One pixel of config 5: this rank's k-th pixel (pixel k % 64 of its tile
// k / 64), the wave's 64 lanes = its secondary rays.
// pts = this wave's 64 sphere points in LDS.
// kAny (no per-ray ids requested): the visibility image needs only each
// ray's hit boolean -> the occlusion walk (ray_occluded), same booleans.
template <bool kR64, bool kAny, int kS, bool kFastOnly = false>
__device__ __forceinline__ void secondary_pixel(const SecondaryParams &p, int64_t k, int lane, uint2 *stk,
                                                float (*pts)[3], SpillCursor &cur)
{
        // lane id re-read per pixel (not held across k_secondary_p's loop)
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
        // this rank's tile k / 64 (the 8x8-pixel tiles dealt as the primary
        // render's, tile_deal), pixel k % 64 of it, row-major
        // the deal's sizes pass through an opaque copy per pixel (see
        // render_unit): its divisions are redone, not held in SGPRs
        int ntx = p.W8 >> 3, nty = p.H8 >> 3, nr = p.nranks, rk = p.rank;
        asm volatile("" : "+s"(ntx), "+s"(nty), "+s"(nr), "+s"(rk));
        int tx, ty;
        if (nr == 1) {
                // one rank: raster order (deal_tile's own one-rank form),
                // without tile_deal / deal_count's divisions (the magic
                // divisor of rank_tile costs this kernel 20 B/lane of scratch)
                if ((k >> 6) >= (int64_t)ntx * nty)
                        return;
                const int T = (int)(k >> 6);
                tx = T % ntx;
                ty = T / ntx;
        } else if (p.tile_xy) {
                // the rank's deal, tabled (p.units = its tiles x 64)
                if (k >= (int64_t)p.units)
                        return;
                rank_tile(ntx, nty, nr, rk, 0, p.tile_xy, (int)(k >> 6), tx, ty);
        } else {
                const TileDeal dl = tile_deal(ntx, nty, nr);
                if ((k >> 6) >= (int64_t)deal_count(dl, rk))
                        return;
                deal_tile(dl, rk, (int)(k >> 6), tx, ty);
        }
        const int px = tx * 8 + (int)(k & 7), py = ty * 8 + (int)((k >> 3) & 7);
        const int64_t pix = (int64_t)py * p.W8 + px;
        const float *pr = p.prim + 8 * pix;
        const size_t vi = (size_t)py * p.nx + px;
        // the pixel is wave-uniform: read its hit flag as a scalar so that
        // the early exit is a uniform branch (a divergent exit inside the
        // persistent loop of k_secondary_p is miscompiled into a loop that
        // never takes another unit)
        if (__builtin_amdgcn_readfirstlane(__float_as_uint(pr[0])) == 0u) {  // primary miss (+0.f)
                if (lane == 0)
                        p.vis[vi] = 1.0f;
                return;
        }
        const f3 hp = mk3(pr[1], pr[2], pr[3]);
        const f3 nrm = mk3(pr[4], pr[5], pr[6]);
        const uint64_t seed = 0xc01dbeefULL ^ (uint64_t)((uint64_t)py * (uint64_t)p.nx + (uint64_t)px);
        const ulonglong2 jl = reinterpret_cast<const ulonglong2 *>(c_pcg_jump3.ac)[lane];
        uint64_t st = jl.x * seed + jl.y;  // pcg_advance(seed, 3 * lane)
        int have = 0;
        while (have < p.spp) {  // wave-uniform
                uint64_t s2 = st;
                const float x = uniform_m11(s2);
                const float y = uniform_m11(s2);
                const float z = uniform_m11(s2);
                const bool acc = length(mk3(x, y, z)) < 1.f;
                const uint64_t mask = __ballot(acc);
                const int rk = have + (int)__popcll(mask & ((1ull << lane) - 1ull));
                if (acc && rk < p.spp) {
                        pts[rk][0] = x;
                        pts[rk][1] = y;
                        pts[rk][2] = z;
                }
                have += (int)__popcll(mask);
                st = pcg_advance(st, 192);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // with compaction: the rays still walking when fewer than t_first
        // lanes are go to queue 0 (SpillQueues)
        const uint32_t t = kAny ? spill_threshold(p.sq, cur, p.sq.t_first) : 0u;
        bool hit = false, spilled = false;
        OcclState w;
        f3 dn;
        RayK r;
        if (lane < p.spp) {
                const f3 pt = mk3(pts[lane][0], pts[lane][1], pts[lane][2]);
                dn = normalize(nrm + pt);  // Ray{hit, n + p, res} normalises d
                r = make_rayk(hp, dn, p.res, kFltMax);
        }
        if (kFastOnly && (!__all(lane >= p.spp || (fast_ok(r) && fin_ok(r))) ||
                          ((p.test_flags & VRT_TEST_SEC_DEFER) && (k & 1)))) {
                // a ray off the fast walk (a zero or tiny direction component):
                // the pixel goes to the deferred list, which k_secondary_defer
                // renders with the exact walk after this launch (every lane in
                // the add, as take_unit; the branch is wave-uniform)
                const uint32_t j = take_n(p.sq.ctr + 6, 1u);
                if (lane == 0)
                        p.sq.dpix[j] = (uint32_t)k;
                return;
        }
        if (kAny) {
                // one call site for the walk: a group whose stopped rays find
                // the queue full walks them on in place from where they stopped
                // (state and LDS stack intact) in a second turn of the loop
                bool resume = false;
                uint32_t tt = t;
                for (;;) {
                        if (lane < p.spp && (!resume || spilled)) {
                                const int res = occl_dispatch_spill<kS, kR64, kFastOnly>(p.sc, r, stk, w, resume, tt);
                                hit = res == kOcclHit;
                                spilled = res == kOcclSpill;
                        }
                        if (!tt)
                                break;
                        const uint64_t sm0 = __ballot(spilled);
                        if (sm0 == 0ull)
                                break;
                        if (spill_room(p.sq, p.sq.ctr, p.sq.fill[0], cur, (uint32_t)__popcll(sm0))) {
                                spill_group<kS>(p.sq.rec[0], cur, spilled, (uint32_t)pix, (uint32_t)lane, dn, w,
                                                stk);
                                break;
                        }
                        resume = true;
                        tt = 0;
                }
                if (p.s_hit && lane < p.spp && !spilled)
                        p.s_hit[vi * (size_t)p.spp + lane] = hit ? 1 : 0;
        } else if (lane < p.spp) {
                const size_t si = vi * (size_t)p.spp + lane;
                MarchResult m;
                ray_march_dispatch<false, kS, false, kR64>(p.sc, r, stk, nullptr, nullptr, m);
                hit = m.hit;
                if (p.s_hit) p.s_hit[si] = m.hit ? 1 : 0;
                if (p.s_tri) p.s_tri[si] = m.hit ? (int32_t)m.tri : -1;
                if (p.s_vox) p.s_vox[si] = m.hit ? p.sc.node_vox[m.node] : 0xFFFFFFFFu;
        }
        const uint64_t hm = __ballot(hit);
        const uint64_t sm = kAny ? __ballot(spilled) : 0ull;
        if (lane == 0) {
                if (sm == 0)
                        p.vis[vi] = (float)(p.spp - (int)__popcll(hm)) / spp_f(p.spp);
                else  // hits so far << 8 | rays still out: the resume rounds finish the pixel
                        reinterpret_cast<uint32_t *>(p.prim + 8 * pix)[7] =
                                ((uint32_t)__popcll(hm) << 8) | (uint32_t)__popcll(sm);
        }
}

// The resume round of the compaction (SpillQueues): queue 0's rays walk on
// from their saved states to their ends; a ray that ends adds to its pixel's
// counts (prim[8*pix+7]: hits << 8 | rays out) and the one that brings the
// rays out to zero writes the pixel.
struct ResumeParams {
        DevScene sc;
        float *prim;
        float *vis;
        int32_t *s_hit;
        int32_t spp;
        float res;
        int32_t nx, W8;  // pixel index <-> primary record index
        int32_t test_flags;
        SpillQueues sq;
};

// One chunk of queue 0 (or a 64-ray piece of it): its rays 64 at a time as one
// pool (occl_pool with each slot's origin its pixel's primary hit point), each
// batch walked to the end; then lane j reports slot j's ray to its pixel.
template <bool kR64>
__device__ __forceinline__ void resume_pool_chunk(const ResumeParams &p, const SpillRec *rec, uint32_t fill,
                                                  uint2 *stk, float (*dirs)[3], uint32_t *opix, uint2 *mbox,
                                                  unsigned long long *hword)
{
        for (uint32_t g = 0; g < fill; g += 64) {
                const uint32_t lane = lane_id();
                const uint32_t i = g + lane;
                bool busy = false, ok = true;
                uint32_t base = 0, mask = 0;
                int sp = 0;
                uint4 h0 = reinterpret_cast<const uint4 *>(rec + g)[0];  // lanes past the fill: a valid pixel
                f3 dn = mk3(0.f, 0.f, 1.f);
                if (i < fill) {
                        spill_read<kSecPBlock>(rec + i, h0, dn, stk);
                        sp = (int)(h0.z >> 8);
                        base = h0.y;
                        mask = h0.z & 0xFFu;
                        const float *pr = p.prim + 8 * (size_t)(h0.x & 0x3FFFFFFu);
                        const RayK r = make_rayk(mk3(pr[1], pr[2], pr[3]), dn, p.res, kFltMax);
                        ok = p.sc.fast_ok && fast_ok(r) && fin_ok(r);
                        busy = true;
                }
                dirs[lane][0] = dn.x;
                dirs[lane][1] = dn.y;
                dirs[lane][2] = dn.z;
                const uint32_t pix = h0.x & 0x3FFFFFFu, smp = h0.x >> 26;
                opix[lane] = pix;
                wave_lds_sync();
                const uint64_t hm =
                        __all(ok) ? occl_pool<true, kSecPBlock, kR64, true, true>(
                                            p.sc, mk3(0.f, 0.f, 0.f), p.prim, opix, p.res, dirs, mbox, hword, stk,
                                            busy, base, mask, sp, 0ull)
                                  : occl_pool<false, kSecPBlock, kR64, false, true>(
                                            p.sc, mk3(0.f, 0.f, 0.f), p.prim, opix, p.res, dirs, mbox, hword, stk,
                                            busy, base, mask, sp, 0ull);
                if (i < fill) {
                        const uint32_t hit = (uint32_t)((hm >> lane) & 1ull);
                        const uint32_t vi = (pix / (uint32_t)p.W8) * (uint32_t)p.nx + pix % (uint32_t)p.W8;
                        if (p.s_hit)
                                p.s_hit[(size_t)vi * (size_t)p.spp + smp] = (int32_t)hit;
                        float *pr = p.prim + 8 * (size_t)pix;
                        const uint32_t old = atomicAdd(reinterpret_cast<uint32_t *>(pr) + 7, hit ? 255u : 0xFFFFFFFFu);
                        if ((old & 0xFFu) == 1u)  // the pixel's last ray
                                p.vis[vi] = (float)(p.spp - (int)((old >> 8) + hit)) / spp_f(p.spp);
                }
                wave_lds_sync();  // dirs / opix / mbox / hword are rewritten by the next batch
        }
}


// ---------------------------------------------------------------------------
// The resume round as one stream per wave.  The wave's lanes
// are a pool over 64 slots (as occl_pool), but a slot whose ray has ended is
// refilled at once with the next saved ray of the queue (chunks taken with
// take_n), so lanes idle only when no piece can be handed over AND the
// queue is empty -- the batch pool instead waits for its 64 rays' longest
// walk before taking the next 64.  Per iteration: idle lanes first take
// pieces handed over by busy lanes (bottom stack entry, or the upper half of
// the children left); idle lanes left over take new rays into free slots;
// every busy lane advances to its next leaf and tests it; a passing leaf
// sets its slot's bit of the LDS hit word (pieces of hit slots drop); then a
// slot that no lane still walks (a wave OR of the busy lanes' slot bits) has
// ended, and lane j reports slot j's ray to its pixel (hits << 8 | rays out,
// as the batch path) and frees the slot.  A chunk not wholly on the fast
// walk (a degenerate direction, an origin far from the scene) is appended
// to a list (queue 1's fill array, count at ctr[3]) that a batch-pool launch
// after this one works through (k_sec_resume, leftover mode).
// LDS per wave: dirs [64][3], sinfo [64] = primary record index | sample <<
// 26 (the host uses this path only for films under 2^26 pixels), mbox [64]
// (also the free-slot map), the hit word.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_or_u64(uint64_t v)
{
#pragma unroll
        for (int o = 32; o > 0; o >>= 1)
                v |= (uint64_t)__shfl_xor((long long)v, o, 64);
        return v;
}

template <bool kR64>
__device__ __forceinline__ bool stream_chunk_fast(const ResumeParams &p, const SpillRec *rec, uint32_t fill,
                                                  uint32_t c)
{
        const uint32_t lane = lane_id();
        bool ok = !((p.test_flags & VRT_TEST_STREAM_LEFTOVER) && (c & 1u));  // test hook: odd chunks left over
        for (uint32_t i = lane; i < fill; i += 64) {
                const uint4 h0 = reinterpret_cast<const uint4 *>(rec + i)[0];
                const uint2 t = reinterpret_cast<const uint2 *>(rec + i)[2];
                const float *pr = p.prim + 8 * (size_t)(h0.x & 0x3FFFFFFu);
                const RayK r = make_rayk(mk3(pr[1], pr[2], pr[3]),
                                         mk3(__uint_as_float(h0.w), __uint_as_float(t.x), __uint_as_float(t.y)),
                                         p.res, kFltMax);
                ok = ok && p.sc.fast_ok && fast_ok(r) && fin_ok(r) && leaf_box_ok(p.sc, r);
        }
        return __all(ok);
}

// resume_stream tests its lanes' leaves once at least this many hold one
// (or no idle lane can get more work); 0: every turn
#ifndef VRT_STREAM_LEAF_T
#define VRT_STREAM_LEAF_T 32
#endif
constexpr uint32_t kStreamLeafT = VRT_STREAM_LEAF_T;

template <bool kR64>
__device__ __forceinline__ void resume_stream(const ResumeParams &p, uint32_t *cin, uint32_t nch,
                                              const uint32_t *fins, const SpillRec *in, uint2 *stk,
                                              float (*dirs)[3], uint32_t *sinfo, uint2 *mbox,
                                              unsigned long long *hword)
{
        constexpr bool kFin = true;
        constexpr bool kNB = kFin;
        const DevScene &sc = p.sc;
        const NodeRec *__restrict__ nodes = sc.nodes;  // kNB: xnodes instead
        const uint32_t lane = lane_id();
        const uint64_t lt = (1ull << lane) - 1ull;
        uint64_t assigned = 0;  // wave-uniform: slots holding a ray
        uint32_t chunk = 0, cur = 0, fill = 0;
        bool more = true;  // wave-uniform: chunks may remain in the queue
        bool busy = false;
        uint32_t slot = lane, base = 0, mask = 0, s = 0;
        int sp = 0, bot = 0;
        bool leaf = false;  // this lane holds a leaf (b, nref) not yet tested
        uint32_t nref = 0, b = 0;
        RayK r;
        r.o = r.d = r.dinv = mk3(0.f, 0.f, 0.f);
        r.tmin = p.res;
        r.tmax = kFltMax;
        if (lane == 0)
                *hword = 0ull;
        wave_lds_sync();
        for (;;) {
                // 0. slots no lane walks any more have ended (their pieces all
                // walked, or a hit): report and free them
                const uint64_t live = wave_or_u64(busy ? 1ull << slot : 0ull);
                const uint64_t done = assigned & ~live;
                if (done != 0ull) {
                        const uint64_t hm = *hword;
                        if ((done >> lane) & 1ull) {
                                const uint32_t inf = sinfo[lane];
                                const uint32_t pix = inf & 0x3FFFFFFu, smp = inf >> 26;
                                const uint32_t vi = (pix / (uint32_t)p.W8) * (uint32_t)p.nx + pix % (uint32_t)p.W8;
                                const uint32_t h = (uint32_t)((hm >> lane) & 1ull);
                                if (p.s_hit)
                                        p.s_hit[(size_t)vi * (size_t)p.spp + smp] = (int32_t)h;
                                float *pr = p.prim + 8 * (size_t)pix;
                                const uint32_t old = atomicAdd(reinterpret_cast<uint32_t *>(pr) + 7, h ? 255u : 0xFFFFFFFFu);
                                if ((old & 0xFFu) == 1u)  // the pixel's last ray
                                        p.vis[vi] = (float)(p.spp - (int)((old >> 8) + h)) / spp_f(p.spp);
                        }
                        assigned &= ~done;
                }
                // 1. hand pieces to idle lanes
                uint64_t idle = __ballot(!busy);
                const bool spare = busy && (sp > bot || __popc(mask) >= 2);
                const uint64_t don = __ballot(spare);
                uint32_t given = 0;
                if (idle != 0ull && don != 0ull) {
                        given = min((uint32_t)__popcll(idle), (uint32_t)__popcll(don));
                        if (spare) {
                                const uint32_t k = (uint32_t)__popcll(don & lt);
                                if (k < given) {
                                        uint2 e;
                                        if (sp > bot) {
                                                e = stk[bot * kSecPBlock];
                                                ++bot;
                                        } else {
                                                uint32_t give = mask;
                                                for (int c = (__popc(mask) + 1) >> 1; c > 0; --c)
                                                        give &= give - 1u;
                                                mask ^= give;
                                                e = make_uint2(base, give);
                                        }
                                        mbox[k] = make_uint2(e.x, e.y | (slot << 8));
                                }
                        }
                        wave_lds_sync();
                        if (!busy) {
                                const uint32_t k = (uint32_t)__popcll(idle & lt);
                                if (k < given) {
                                        const uint2 e = mbox[k];
                                        slot = e.y >> 8;
                                        base = e.x;
                                        mask = e.y & 0xFFu;
                                        sp = bot = 0;
                                        busy = true;
                                        const float *pr = p.prim + 8 * (size_t)(sinfo[slot] & 0x3FFFFFFu);
                                        r = make_rayk(mk3(pr[1], pr[2], pr[3]),
                                                      mk3(dirs[slot][0], dirs[slot][1], dirs[slot][2]), p.res,
                                                      kFltMax);
                                        s = dir_signs(r);
                                }
                        }
                        wave_lds_sync();
                }
                // 2. idle lanes left over take new rays into free slots
                uint32_t left = (uint32_t)__popcll(idle) - given;
                if (left > 0 && more) {
                        if (cur >= fill) {
                                const uint32_t c = take_n(cin + 1, 1u);
                                if (c >= nch) {
                                        more = false;
                                } else {
                                        const uint32_t f = __builtin_amdgcn_readfirstlane(fins[c]);
                                        if (stream_chunk_fast<kR64>(p, in + (size_t)c * kSpillChunk, f, c)) {
                                                chunk = c;
                                                cur = 0;
                                                fill = f;
                                        } else {
                                                // left to the batch pool's launch after this one
                                                const uint32_t j = take_n(p.sq.ctr + 3, 1u);
                                                if (lane == 0)
                                                        p.sq.fill[1][j] = c;
                                        }
                                }
                        }
                        if (more && cur < fill) {
                                const uint64_t freem = ~assigned;
                                const uint32_t ntake = min(min(left, (uint32_t)__popcll(freem)), fill - cur);
                                const bool fr = (freem >> lane) & 1ull;
                                const uint32_t rank = (uint32_t)__popcll(freem & lt);
                                const uint64_t taken = __ballot(fr && rank < ntake);
                                uint32_t *map = reinterpret_cast<uint32_t *>(mbox);
                                if (fr && rank < ntake)
                                        map[rank] = lane;
                                wave_lds_sync();
                                const uint64_t still = __ballot(!busy);
                                if (!busy) {
                                        const uint32_t k = (uint32_t)__popcll(still & lt);
                                        if (k < ntake) {
                                                slot = map[k];
                                                uint4 h0;
                                                f3 d;
                                                spill_read<kSecPBlock>(in + (size_t)chunk * kSpillChunk + cur + k, h0,
                                                                       d, stk);
                                                sp = (int)(h0.z >> 8);
                                                bot = 0;
                                                base = h0.y;
                                                mask = h0.z & 0xFFu;
                                                dirs[slot][0] = d.x;
                                                dirs[slot][1] = d.y;
                                                dirs[slot][2] = d.z;
                                                sinfo[slot] = h0.x;  // pix | sample << 26
                                                const float *pr = p.prim + 8 * (size_t)(h0.x & 0x3FFFFFFu);
                                                r = make_rayk(mk3(pr[1], pr[2], pr[3]), d, p.res, kFltMax);
                                                s = dir_signs(r);
                                                busy = true;
                                        }
                                }
                                assigned |= taken;
                                cur += ntake;
                                if (lane == 0)
                                        *hword &= ~taken;
                                wave_lds_sync();
                        }
                }
                if (__ballot(busy) == 0ull) {
                        if (!more)
                                break;
                        if (cur >= fill)
                                continue;  // take the next chunk
                }
                // 3. every busy lane without a leaf in hand: advance to its next
                // leaf (occl_walk); a lane holding one from an earlier turn keeps it
                if (busy && !leaf) {
                        float bmin[3], bmax[3];
                        uint32_t a;
                        for (;;) {
                                if (mask == 0) {
                                        if (sp == bot)
                                                break;
                                        --sp;
                                        const uint2 e = stk[sp * kSecPBlock];
                                        base = e.x;
                                        mask = e.y;
                                }
                                const uint32_t ci = (uint32_t)__builtin_ctz(mask) ^ s;
                                mask &= mask - 1u;
                                if (kNB) {
                                        float tmn[3], tmx[3];
                                        load_xnode(sc.xnodes, base + ci, bmin, bmax, a, b, tmn, tmx);
                                        if (!line_meets_box(tmn, tmx, r))
                                                continue;
                                } else {
                                        load_node(nodes, base + ci, bmin, bmax, a, b);
                                }
                                if (!(a & kLeafBit)) {
                                        if (mask) {
                                                stk[sp * kSecPBlock] = make_uint2(base, mask);
                                                ++sp;
                                        }
                                        mask = xor_permute8(child_hit_mask<true, kFin>(bmin, bmax, r) & b, s);
                                        base = a;
                                        continue;
                                }
                                nref = a & ~kLeafBit;
                                leaf = true;
                                break;
                        }
                        if (!leaf) {
                                busy = false;
                                sp = bot = 0;
                        }
                }
                // 4. the leaf tests, together: while fewer than kStreamLeafT
                // lanes hold a leaf and idle lanes can still get work (a
                // donor with a piece to spare, or more saved rays), the
                // holders wait and the others take work and advance first, so
                // the MT loop runs on more lanes at a time (which leaves are
                // tested when does not change a slot's OR of hits)
                const uint64_t lm = __ballot(leaf);
                if (lm != 0ull && (uint32_t)__popcll(lm) < kStreamLeafT && lm != ~0ull &&
                    (more || __ballot(leaf && (sp > bot || __popc(mask) >= 2)) != 0ull))
                        continue;
                bool hit = false;
                if (leaf) {
                        bool done = false;
                        if (kR64) {
                                const uint32_t f0 = __builtin_amdgcn_readfirstlane(b);
                                const uint32_t n0 = __builtin_amdgcn_readfirstlane(nref);
                                if (__all(b == f0 && nref == n0)) {
                                        hit = leaf_any<true>(sc.refs, f0, n0, r);
                                        done = true;
                                }
                        }
                        if (!done)
                                hit = leaf_any<kR64>(sc.refs, b, nref, r);
                        leaf = false;
                }
                if (__ballot(hit) != 0ull) {
                        if (hit)
                                atomicOr(hword, 1ull << slot);
                        wave_lds_sync();
                        const uint64_t hm = *hword;
                        if (busy && ((hm >> slot) & 1ull)) {
                                busy = false;
                                mask = 0;
                                sp = bot = 0;
                        }
                }
        }
}

// The streaming resume round (films under 2^26 pixels): one
// resident generation, each wave one stream (resume_stream) over queue 0.
#ifndef VRT_STREAM_WAVES_PER_EU
#define VRT_STREAM_WAVES_PER_EU VRT_SECP_WAVES_PER_EU
#endif
template <bool kR64>
__global__ __launch_bounds__(kSecPBlock, VRT_STREAM_WAVES_PER_EU) void k_sec_stream(ResumeParams p)
{
        __shared__ uint2 stk[kStack * kSecPBlock];
        __shared__ float dirs[kSecPBlock / 64][64][3];
        __shared__ uint32_t sinfo[kSecPBlock / 64][64];
        __shared__ uint2 mbox[kSecPBlock / 64][64];
        __shared__ unsigned long long hword[kSecPBlock / 64];
        const int tid = threadIdx.x, w = tid >> 6;
        uint32_t *cin = p.sq.ctr;
        const uint32_t n = min(cin[0], p.sq.nchunks);
        resume_stream<kR64>(p, cin, n, p.sq.fill[0], p.sq.rec[0], stk + tid, dirs[w], sinfo[w], mbox[w], hword + w);
}

template <bool kR64>
__global__ __launch_bounds__(kSecPBlock, VRT_SECP_WAVES_PER_EU) void k_sec_resume(ResumeParams p)
{
        __shared__ uint2 stk[kStack * kSecPBlock];
        __shared__ float dirs[kSecPBlock / 64][64][3];
        __shared__ uint32_t opix[kSecPBlock / 64][64];
        __shared__ uint2 mbox[kSecPBlock / 64][64];
        __shared__ unsigned long long hword[kSecPBlock / 64];
        const int tid = threadIdx.x;
        const uint32_t *fin = p.sq.fill[0];
        const SpillRec *in = p.sq.rec[0];
        // the chunks k_sec_stream listed (normally none), from ctr[4], each as
        // kSpillChunk / 64 pieces of 64 rays on different waves (the few
        // leftover chunks of a frame would otherwise leave one wave walking a
        // whole chunk's batches one after the other)
        constexpr uint32_t kParts = kSpillChunk / 64;
        const uint32_t nl = p.sq.ctr[3] * kParts;
        for (;;) {
                const uint32_t j = take_n(p.sq.ctr + 4, 1u);
                if (j >= nl)
                        break;
                const uint32_t c = __builtin_amdgcn_readfirstlane(p.sq.fill[1][j / kParts]), part = j % kParts;
                const int w = tid >> 6;
                const uint32_t f = fin[c], lo = part * 64u;
                if (lo >= f)
                        continue;
                const uint32_t cnt = min(64u, f - lo);
                resume_pool_chunk<kR64>(p, in + (size_t)c * kSpillChunk + lo, cnt, stk + tid, dirs[w], opix[w],
                                        mbox[w], hword + w);
        }
}

// Persistent config 5: one resident generation of 4-wave workgroups; each
// wave pulls one pixel at a time from the per-XCD counters of the launch's
// WorkQueue (XCD x owns a contiguous slice of this rank's pixels, then
// helps the others), so no wave waits for a slow pixel of a sibling and the
// resident-wave count is not capped by the per-CU workgroup limit.
template <bool kR64, bool kAny, bool kFastOnly>
__global__ __launch_bounds__(kSecPBlock, VRT_SECP_WAVES_PER_EU) void k_secondary_p(SecondaryParams p)
{
        __shared__ uint2 stk[kStack * kSecPBlock];
        __shared__ float pts[kSecPBlock / 64][64][3];
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        const int xcd = blockIdx.x & 7;
        SpillCursor cur;
        cur.chunk = kSpillNone;
        cur.fill = 0;
        for (int j = 0; j < 8; ++j) {
                const int x = (xcd + j) & 7;
                const int n = slice_size(p.units, x, VRT_SEC_SLICE_CHUNK);
                if (n <= 0)
                        continue;
                for (;;) {
                        // kSecTake consecutive pixels per dequeue (every add is
                        // kSecTake: launch_secondary's base accounting)
                        const uint32_t u = take_n(p.q.ctr + x * kQueueStride, kSecTake) - p.q.base[x];
                        if (u >= (uint32_t)n)
                                break;
                        const uint32_t e = min(u + kSecTake, (uint32_t)n);
                        for (uint32_t v = u; v < e; ++v)
                                secondary_pixel<kR64, kAny, kSecPBlock, kFastOnly>(
                                        p, (int64_t)slice_unit(p.units, x, (int)v, VRT_SEC_SLICE_CHUNK), lane,
                                        stk + tid, pts[wave], cur);
                }
        }
        if (kAny)
                spill_close(p.sq.fill[0], p.sq.ctr, cur);
}

// The pixels k_secondary_p<.., kFastOnly> deferred (a ray off the fast walk;
// normally a few per frame, none in most): each on the general walk, without
// compaction (the pixel writes its visibility directly).  No deferred pixel:
// every wave returns after one scalar load.  Launched after the fast kernel
// (and the resume rounds) on the same stream, so the list is complete.
template <bool kR64>
__global__ __launch_bounds__(kSecPBlock, VRT_SECP_WAVES_PER_EU) void k_secondary_defer(SecondaryParams p)
{
        __shared__ uint2 stk[kStack * kSecPBlock];
        __shared__ float pts[kSecPBlock / 64][64][3];
        const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
        const uint32_t n = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(p.sq.ctr + 6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (n == 0)
                return;
        SpillCursor cur;
        cur.chunk = kSpillFull;  // no compaction here
        cur.fill = 0;
        for (;;) {
                const uint32_t j = take_n(p.sq.ctr + 7, 1u);
                if (j >= n)
                        break;
                const uint32_t k = __builtin_amdgcn_readfirstlane(p.sq.dpix[j]);
                secondary_pixel<kR64, true, kSecPBlock, false>(p, (int64_t)k, lane, stk + tid, pts[wave], cur);
        }
}

#ifndef VRT_SEC_SPILL_T
// phase A stops below this many walking lanes (0: no compaction).  Round 5
// (64-B packed records): 8 / 12 / 14 / 16 / 18 / 20 / 24 = 18.11 / 17.21 /
// 16.96 / 16.81 / 16.75 / 16.81 / 16.93 ms per frame (round 4, 128-B records:
// 12 was best, 17.21 vs 17.28 at 16)
#define VRT_SEC_SPILL_T 18
#endif
static_assert(kSpillStack >= kStack, "SpillRec stack");

// The rank's tiles in deal order (RenderParams::tile_xy): one thread per
// tile, deal_tile itself.
__global__ __launch_bounds__(256) void k_deal_map(int ntx, int nty, int nranks, int rank, int n,
                                                  uint32_t *__restrict__ out)
{
        const int k = (int)(blockIdx.x * 256 + threadIdx.x);
        if (k >= n)
                return;
        int tx, ty;
        deal_tile(tile_deal(ntx, nty, nranks), rank, k, tx, ty);
        out[k] = (uint32_t)tx | (uint32_t)ty << 16;
}

hipError_t launch_deal_map(int ntx, int nty, int nranks, int rank, uint32_t *out, hipStream_t st)
{
        const int n = deal_count(tile_deal(ntx, nty, nranks), rank);
        if (n <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(k_deal_map, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ntx, nty, nranks, rank, n,
                           out);
        return hipGetLastError();
}

SpillQueues spill_defaults()
{
        SpillQueues q;
        std::memset(&q, 0, sizeof q);
        q.t_first = VRT_SEC_SPILL_T;
        q.stream = 0;  // set per launch (launch_secondary: films under 2^26 pixels)
        return q;
}

hipError_t launch_secondary(const RenderParams &rp, int spp, int rank, int nranks, float res,
                            float *prim, float *vis, int32_t *s_hit, int32_t *s_tri,
                            uint32_t *s_vox, const WorkQueue *q, hipStream_t st, int *q_waves, int slice_units[8],
                            const SpillQueues *sq, const SideLaunch *side)
{
        *q_waves = 0;
        for (int x = 0; x < 8; ++x)
                slice_units[x] = 0;
        const int64_t npix = (int64_t)rp.ntx * 8 * rp.nty * 8;
        if (npix <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(rp.sc.wide_leaves ? k_primary1<true> : k_primary1<false>, dim3((unsigned)((npix + kBlock - 1) / kBlock)), dim3(kBlock), 0, st,
                           rp, prim);
        if (hipError_t e = hipGetLastError())
                return e;
        SecondaryParams sp;
        std::memset(&sp, 0, sizeof sp);
        sp.sc = rp.sc;
        sp.nx = rp.cam.nx;
        sp.W8 = rp.ntx * 8;
        sp.H8 = rp.nty * 8;
        sp.spp = spp;
        sp.rank = rank;
        sp.nranks = nranks;
        sp.res = res;
        sp.prim = prim;
        sp.vis = vis;
        sp.s_hit = s_hit;
        sp.s_tri = s_tri;
        sp.s_vox = s_vox;
        sp.test_flags = rp.test_flags;
        sp.tile_xy = nranks > 1 ? rp.tile_xy : nullptr;
        // pixels of this rank: its 8x8 tiles (tile_deal)
        const int64_t mine = deal_count(tile_deal(rp.ntx, rp.nty, nranks), rank);
        const int64_t waves = mine * 64;
        if (waves == 0)
                return hipGetLastError();
        // no per-ray ids requested: the occlusion walk (+ compaction)
        const bool any = !s_tri && !s_vox;
        const bool w = sp.sc.wide_leaves != 0;
        if (!q || !secondary_uses_queue(rp.sc) || waves > INT_MAX)
                return hipErrorInvalidValue;
        {
                sp.units = (int32_t)waves;
                sp.q = *q;
                const int cap = nranks > 1 ? std::max(8, rp.sc.sec_blocks - kCollectiveReserve) : rp.sc.sec_blocks;
                const int g = (int)std::min<int64_t>(cap, ((waves + 3) / 4 + 7) & ~7LL);
                const bool spill = any && sq && sq->t_first > 0 && sq->nchunks > 0;
                // with compaction (and its deferred-pixel list) in a scene the
                // fast walk covers, the fast-only kernel: the exact walk's waves
                // go to k_secondary_defer
                const bool fo = spill && sq->dpix && sp.sc.fast_ok;
                void (*kern)(SecondaryParams) =
                        fo ? (w ? k_secondary_p<true, true, true> : k_secondary_p<false, true, true>)
                           : w ? (any ? k_secondary_p<true, true, false> : k_secondary_p<true, false, false>)
                               : (any ? k_secondary_p<false, true, false> : k_secondary_p<false, false, false>);
                if (spill) {
                        sp.sq = *sq;
                        if (rp.test_flags & VRT_TEST_SPILL_ALL)  // test hook: stop at the first ray's end
                                sp.sq.t_first = 64;
                }
                hipLaunchKernelGGL(kern, dim3(g), dim3(kSecPBlock), 0, st, sp);
                // every add is kSecTake: the successful takes cover a slice's
                // pixels rounded up to whole takes, and each wave's one failing
                // take per slice adds kSecTake too (queue_release)
                *q_waves = g * (kSecPBlock / 64) * (int)kSecTake;
                for (int x = 0; x < 8; ++x) {
                        const int n = slice_size((int)waves, x, VRT_SEC_SLICE_CHUNK);
                        slice_units[x] = (n + (int)kSecTake - 1) / (int)kSecTake * (int)kSecTake;
                }
                if (hipError_t e = hipGetLastError())
                        return e;
                // the deferred pixels (normally a few, each one long exact
                // walk): a quarter of the resident grid, each wave gone after
                // one load if none.  With a side stream they run beside the
                // resume round (they write other pixels than its rays do: a
                // deferred pixel stopped none), joined before the launch ends.
                SecondaryParams dp = sp;
                dp.sq.t_first = 0;
                const dim3 dgrid((unsigned)std::max(8, (g / 4) & ~7));
                auto defer_kern = w ? k_secondary_defer<true> : k_secondary_defer<false>;
                const bool fork = fo && side && side->st;
                if (fork) {
                        if (hipError_t e = hipEventRecord(side->fork, st))
                                return e;
                        if (hipError_t e = hipStreamWaitEvent(side->st, side->fork, 0))
                                return e;
                        hipLaunchKernelGGL(defer_kern, dgrid, dim3(kSecPBlock), 0, side->st, dp);
                        if (hipError_t e = hipGetLastError())
                                return e;
                        if (hipError_t e = hipEventRecord(side->join, side->st)) {
                                // no join for the caller's stream to wait on: the
                                // deferred walk finishes before the set can be
                                // reused or freed (its event covers st only)
                                (void)hipStreamSynchronize(side->st);
                                return e;
                        }
                }
                if (spill) {
                        // the resume round: one resident generation walking
                        // queue 0's records to their ends (an empty queue ends
                        // the launch at once)
                        ResumeParams rp2;
                        std::memset(&rp2, 0, sizeof rp2);
                        rp2.sc = rp.sc;
                        rp2.prim = prim;
                        rp2.vis = vis;
                        rp2.s_hit = s_hit;
                        rp2.spp = spp;
                        rp2.res = res;
                        rp2.nx = rp.cam.nx;
                        rp2.test_flags = rp.test_flags;
                        rp2.W8 = rp.ntx * 8;
                        rp2.sq = sp.sq;
                        // the streaming round (the host compacts only films under 2^26
                        // pixels: resume_stream packs the pixel index in 26 bits)
                        rp2.sq.stream = 1;
                        hipLaunchKernelGGL(w ? k_sec_stream<true> : k_sec_stream<false>, dim3(g), dim3(kSecPBlock),
                                           0, st, rp2);
                        // the chunks the stream left (normally none): a small batch-pool launch
                        hipLaunchKernelGGL(w ? k_sec_resume<true> : k_sec_resume<false>, dim3(8), dim3(kSecPBlock), 0,
                                           st, rp2);
                }
                if (fork) {
                        if (hipError_t e = hipStreamWaitEvent(st, side->join, 0))
                                return e;
                } else if (fo) {
                        hipLaunchKernelGGL(defer_kern, dgrid, dim3(kSecPBlock), 0, st, dp);
                }
                return hipGetLastError();
        }
}

// Rank-0 re-assembly of gathered per-rank tile buffers into the image.
__global__ void k_unpack(int nx, int ny, int ntx, int nty, int nranks,
                         int tpr, const float *__restrict__ src,
                         float *__restrict__ dst)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= (int64_t)nx * ny)
                return;
        const int px = (int)(i % nx), py = (int)(i / nx);
        const int tx = px >> 3, ty = py >> 3;
        float v0 = 0.f, v1 = 0.f, v2 = 0.f;
        if (tx < ntx && ty < nty) {
                int r, k;
                deal_slot(tile_deal(ntx, nty, nranks), tx, ty, r, k);
                const float *q = src + (((int64_t)r * tpr + k) * 64 + (py & 7) * 8 + (px & 7)) * 3;
                v0 = q[0];
                v1 = q[1];
                v2 = q[2];
        }
        dst[3 * i + 0] = v0;
        dst[3 * i + 1] = v1;
        dst[3 * i + 2] = v2;
}

// The same for films whose sides are multiples of 8 (every pixel in a
// tile): one thread per 16-B chunk of the image, so both sides move in
// dwordx4 -- a tile row is 8 pixels x 12 B = 6 chunks, 16-B aligned in the
// image (nx % 4 == 0) and in the packed buffer (768-B tiles, 96-B rows).
__global__ void k_unpack4(int nx, int ny, int ntx, int nty, int nranks, int tpr,
                          const float4 *__restrict__ src, float4 *__restrict__ dst)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        const int rq = nx * 3 / 4;  // chunks per image row
        if (i >= (int64_t)rq * ny)
                return;
        const int py = (int)(i / rq), q = (int)(i % rq);
        const int tx = q / 6, c = q % 6, ty = py >> 3;
        int r, k;
        deal_slot(tile_deal(ntx, nty, nranks), tx, ty, r, k);
        dst[i] = src[((int64_t)r * tpr + k) * 48 + (py & 7) * 6 + c];
}

// Any component count (config 5's visibility: 1 float per pixel): rank
// rank's tiles of a (ny, nx, comps) image -> its packed buffer (tile k at
// k * 64 * comps, pixels row-major inside the tile), and the gathered
// buffers of every rank -> the image (zero outside the tile grid).  One
// thread per float of the packed buffer / the image.
__global__ void k_pack_c(int nx, int ntx, int nty, int rank, int nranks, int comps, int64_t n,
                         const float *__restrict__ img, float *__restrict__ dst)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n)
                return;
        const int64_t e = i / comps;
        const int c = (int)(i % comps);
        const int k = (int)(e >> 6), pp = (int)(e & 63);
        int tx, ty;
        deal_tile(tile_deal(ntx, nty, nranks), rank, k, tx, ty);
        const int px = tx * 8 + (pp & 7), py = ty * 8 + (pp >> 3);
        dst[i] = img[((int64_t)py * nx + px) * comps + c];
}

__global__ void k_unpack_c(int nx, int ny, int ntx, int nty, int nranks, int tpr, int comps,
                           const float *__restrict__ src, float *__restrict__ dst)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= (int64_t)nx * ny * comps)
                return;
        const int64_t e = i / comps;
        const int c = (int)(i % comps);
        const int px = (int)(e % nx), py = (int)(e / nx);
        const int tx = px >> 3, ty = py >> 3;
        float v = 0.f;
        if (tx < ntx && ty < nty) {
                int r, k;
                deal_slot(tile_deal(ntx, nty, nranks), tx, ty, r, k);
                v = src[(((int64_t)r * tpr + k) * 64 + (py & 7) * 8 + (px & 7)) * comps + c];
        }
        dst[i] = v;
}

hipError_t launch_pack_c(int nx, int ny, int rank, int nranks, int comps, const float *img, float *dst,
                         hipStream_t st)
{
        const int ntx = nx / 8, nty = ny / 8;
        const int64_t n = (int64_t)deal_count(tile_deal(ntx, nty, nranks), rank) * 64 * comps;
        if (n <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(k_pack_c, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nx, ntx, nty, rank,
                           nranks, comps, n, img, dst);
        return hipGetLastError();
}

hipError_t launch_unpack_c(int nx, int ny, int nranks, int tpr, int comps, const float *src, float *dst,
                           hipStream_t st)
{
        const int64_t n = (int64_t)nx * ny * comps;
        if (n <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(k_unpack_c, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nx, ny, nx / 8, ny / 8,
                           nranks, tpr, comps, src, dst);
        return hipGetLastError();
}

// Device copies of the MT / SAT leaves for bit-exact KATs.
__global__ void k_selftest(const double *mt_in, double *mt_out,
                           const float *sat_in, int32_t *sat_out, int64_t n)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n)
                return;
        if (mt_in) {
                const double *q = mt_in + 15 * i;
                double t = 0, u = 0, v = 0;
                const int ret = mt_isect(q, q + 3, q + 6, q + 9, q + 12, &t, &u, &v);
                mt_out[4 * i + 0] = ret;
                mt_out[4 * i + 1] = ret ? t : 0.0;
                mt_out[4 * i + 2] = ret ? u : 0.0;
                mt_out[4 * i + 3] = ret ? v : 0.0;
        }
        if (sat_in) {
                const float *q = sat_in + 15 * i;
                sat_out[i] = tri_box_overlap(q, q + 3, q + 6);
        }
}

// The kernel's own travorder / min_element code on arbitrary inputs (the
// std::sort / std::min_element pin, tests/golden/travorder_std.cpp).  Per
// case i: dist[8i..8i+7], hit mask hm[i] ->
//   out[6i+0] insertion_perm8 (the full order, 3-bit fields)
//   out[6i+1] perm_filter of it | count << 24 (the exact path's result)
//   out[6i+2] rank_order8 | popc(hm) << 24     (fast paths: no NaN)
//   out[6i+3] two_slot_order                    (no NaN, <= 2 hit children)
//   out[6i+4] net4_order                        (no NaN, <= 4 hit children)
//   out[6i+5] rank_order8's full position word  (instrumented counters)
// and per record list j: depth[j*stride .. + len[j]) -> argmin[j] (first
// minimum by first_min_takes, -1 if empty).
__global__ void k_selftest_order(const float *__restrict__ dist, const uint32_t *__restrict__ hm, int64_t n,
                                 uint32_t *__restrict__ out, const float *__restrict__ depth,
                                 const int32_t *__restrict__ len, int64_t m, int32_t stride,
                                 int32_t *__restrict__ argmin)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i < n) {
                float d[8];
#pragma unroll
                for (int k = 0; k < 8; ++k)
                        d[k] = dist[8 * i + k];
                const uint32_t mask = hm[i] & 0xFFu;
                auto dist_of = [&](uint32_t ci) { return d[ci & 7u]; };
                const uint32_t perm = insertion_perm8(dist_of);
                int cnt = 0;
                uint32_t fp = 0;
                const uint32_t ex = perm_filter<false>(perm, mask, cnt, fp);
                const uint32_t rk = rank_order8<true>(d, mask, fp);
                out[6 * i + 0] = perm;
                out[6 * i + 1] = ex | ((uint32_t)cnt << 24);
                out[6 * i + 2] = rk | ((uint32_t)__popc(mask) << 24);
                out[6 * i + 3] = two_slot_order(dist_of, mask);
                out[6 * i + 4] = net4_order(dist_of, mask);
                out[6 * i + 5] = fp;
        }
        if (i < m) {
                bool any = false;
                float best = 0.f;
                int32_t bi = -1;
                for (int32_t k = 0; k < len[i]; ++k) {
                        const float v = depth[i * stride + k];
                        if (first_min_takes(any, best, v)) {
                                any = true;
                                best = v;
                                bi = k;
                        }
                }
                argmin[i] = bi;
        }
}

hipError_t launch_selftest_order(const float *dist, const uint32_t *hm, int64_t n, uint32_t *out,
                                 const float *depth, const int32_t *len, int64_t m, int32_t stride,
                                 int32_t *argmin, hipStream_t st)
{
        const int64_t nt = std::max(n, m);
        if (nt <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(k_selftest_order, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, dist, hm, n,
                           out, depth, len, m, stride, argmin);
        return hipGetLastError();
}

// persistent waves for RefRec48 scenes without per-sample outputs;
// large-leaf (RefRec64) scenes keep one-wave workgroups (-11 % persistent at
// depth 6).  The fast-only kernel when the camera makes standard-range
// rays (tmin = +0, tmax = FLT_MAX) from a finite origin in a finite scene;
// the kernel itself re-checks every wave and defers what is not exact.
RenderKind render_kind(const RenderParams &p, bool instrumented)
{
        const SampleOut &so = p.so;
        if (instrumented || so.hit || so.tri || so.vox || so.rgb || so.cnt || p.sc.wide_leaves ||
            p.sc.persist_blocks <= 0)
                return kRenderGrid;
        const CamParams &c = p.cam;
        bool fast = p.sc.fast_ok && __builtin_bit_cast(uint32_t, c.tmin) == 0u &&
                    c.tmax == kFltMax;
        for (int k = 0; k < 3; ++k)
                fast = fast && std::fabs(c.origin[k]) < 0x1p60f;
        return fast ? kRenderPersistFast : kRenderPersist;
}

// Host bound on the camera rays of a frame that make k_render_p<true> defer
// their unit (so the deferred pass is launched only for frames that have
// some, on a grid sized to them).  Every ray has tmin = +0, tmax = FLT_MAX
// and a finite origin (render_kind); it defers iff a direction component
// fails fin_ok / fast_ok, i.e. |d_q| < 2^-64 (an exact zero included).
// d = normalize(acc) with acc_q = fl(fl(a + b) + c), a = fl(s_q x_) over the
// film's columns, b = fl(u_q y_) over its rows, c = fl(nf_q z) (+ e_q * 0,
// which adds a zero: camera_dir).  The two float additions are off from the
// real a + b + c by at most 2.01 * 2^-24 * M_q (M_q >= |a| + |b| + |c|,
// + 2^-140 for subnormals).  For every row b the distinct a values within
// that bound + T (T = 2^-58 * M, M = sum of the M_q >= len) of -(b + c) are
// found by binary search and their float sum is evaluated exactly as the
// kernel does; a sum of at most 2^-62 * M counts the columns holding that a
// value.  Every other ray has |acc_q| > 2^-62 * M, so |d_q| = |acc_q| / len
// > 2^-62 / 1.01 > 2^-64.  The count is an upper bound (a ray may count for
// two components); a non-finite term returns INT64_MAX.  On the 16-pose
// 1080p sweep about half the poses have a ray or two with an exactly zero
// component.  Cost: O(ny log nx) per sample and component; the last 32
// cameras' answers are kept (a camera sweep repeats its poses).
static int64_t camera_defer_count(const CamParams &c);
int64_t camera_defer_bound(const CamParams &c)
{
        struct Entry {
                CamParams c;
                int64_t n;
        };
        static std::mutex mu;
        static Entry cache[32];
        static int n = 0, next = 0;
        {
                std::lock_guard<std::mutex> lk(mu);
                for (int i = 0; i < n; ++i)
                        if (std::memcmp(&cache[i].c, &c, sizeof c) == 0)
                                return cache[i].n;
        }
        const int64_t r = camera_defer_count(c);
        std::lock_guard<std::mutex> lk(mu);
        cache[next] = Entry{ c, r };
        next = (next + 1) % 32;
        n = std::min(n + 1, 32);
        return r;
}

static int64_t camera_defer_count(const CamParams &c)
{
        const int nx = c.nx, ny = c.ny;
        if (nx < 1 || ny < 1)
                return 0;
        std::vector<float> xs((size_t)nx), ys((size_t)ny), a, b((size_t)ny);
        std::vector<int> mult;
        a.reserve((size_t)nx);
        int64_t count = 0;
        for (int s = 0; s < 4; ++s) {
                const float sx = sample_x(s), sy = sample_y(s);
                // the same float ops as camera_dir
                for (int px = 0; px < nx; ++px)
                        xs[px] = ((float)(px - nx / 2) + sx) / (float)nx;
                for (int py = 0; py < ny; ++py)
                        ys[py] = ((float)((ny - 1 - py) - ny / 2) + sy) / (float)ny;
                double m[3], mtot = 0.0;
                for (int q = 0; q < 3; ++q) {
                        const double ax = std::max(std::fabs((double)(c.s[q] * xs[0])),
                                                   std::fabs((double)(c.s[q] * xs[nx - 1])));
                        const double by = std::max(std::fabs((double)(c.u[q] * ys[0])),
                                                   std::fabs((double)(c.u[q] * ys[ny - 1])));
                        m[q] = ax + by + std::fabs((double)(c.nf[q] * c.z));
                        if (!std::isfinite(m[q]) || !std::isfinite((double)c.e[q]) || m[q] > 0x1p100)
                                return INT64_MAX;
                        mtot += m[q];
                }
                const double T = 0x1p-58 * mtot;                  // beyond the window: |acc_q| > T
                const float exact_min = (float)(0x1p-62 * mtot);  // inside it: the float sum itself
                for (int q = 0; q < 3; ++q) {
                        const float sq = c.s[q], uq = c.u[q], cq = c.nf[q] * c.z;
                        // the distinct a values, ascending, with their column counts
                        a.clear();
                        for (int px = 0; px < nx; ++px)
                                a.push_back(sq * xs[px]);
                        std::sort(a.begin(), a.end());
                        mult.clear();
                        size_t w = 0;
                        for (size_t i = 0; i < a.size(); ++i) {
                                if (w > 0 && a[i] == a[w - 1]) {
                                        ++mult[w - 1];
                                } else {
                                        a[w++] = a[i];
                                        mult.push_back(1);
                                }
                        }
                        a.resize(w);
                        for (int py = 0; py < ny; ++py)
                                b[py] = uq * ys[py];
                        const double err = 2.01 * 0x1p-24 * m[q] + 0x1p-140 + T;
                        for (int py = 0; py < ny; ++py) {
                                const double t = -((double)b[py] + (double)cq);
                                size_t i = std::lower_bound(a.begin(), a.end(), (float)(t - err * 1.001)) - a.begin();
                                for (; i < a.size() && (double)a[i] <= t + err * 1.001; ++i) {
                                        // a near-cancellation: camera_dir's own float sum
                                        float acc = a[i];
                                        acc += b[py];
                                        acc += cq;
                                        if (!(std::fabs(acc) > exact_min))
                                                count += mult[i];
                                }
                        }
                }
        }
        return count;
}

bool secondary_uses_queue(const DevScene &sc)
{
        return sc.sec_blocks > 0;
}

static int resident_blocks(const void *kern, int block, const hipDeviceProp_t &prop, hipError_t *e)
{
        int per_cu = 0;
        *e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, block, 0);
        return std::max(8, (per_cu * prop.multiProcessorCount) & ~7);
}

hipError_t persistent_blocks(int *render_blocks, int *sec_blocks)
{
        int dev = 0;
        hipDeviceProp_t prop;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess)
                e = hipGetDeviceProperties(&prop, dev);
        if (e != hipSuccess)
                return e;
        // the smaller residency of the two render variants (a surplus block
        // only waits, then finds the queues empty)
        const int a = resident_blocks(reinterpret_cast<const void *>(k_render_p<true>), kPersistBlock, prop, &e);
        if (e != hipSuccess)
                return e;
        const int b = resident_blocks(reinterpret_cast<const void *>(k_render_p<false>), kPersistBlock, prop, &e);
        if (e != hipSuccess)
                return e;
        *render_blocks = std::min(a, b);
        int sb = 1 << 30;
        const void *sk[6] = { reinterpret_cast<const void *>(k_secondary_p<false, false, false>),
                              reinterpret_cast<const void *>(k_secondary_p<false, true, false>),
                              reinterpret_cast<const void *>(k_secondary_p<true, false, false>),
                              reinterpret_cast<const void *>(k_secondary_p<true, true, false>),
                              reinterpret_cast<const void *>(k_secondary_p<false, true, true>),
                              reinterpret_cast<const void *>(k_secondary_p<true, true, true>) };
        for (int i = 0; i < 6 && e == hipSuccess; ++i)
                sb = std::min(sb, resident_blocks(sk[i], kSecPBlock, prop, &e));
        *sec_blocks = sb;
        return e;
}

hipError_t launch_render(const RenderParams &p, bool instrumented,
                         hipStream_t st, int *q_waves, int slice_units[8])
{
        *q_waves = 0;
        for (int x = 0; x < 8; ++x)
                slice_units[x] = 0;
        if (p.tiles_this_rank <= 0)
                return hipSuccess;
        const bool w = p.sc.wide_leaves != 0;
        const RenderKind kind = render_kind(p, instrumented);
        if (kind != kRenderGrid) {
                // one resident generation of 4-wave workgroups (<= one per
                // 4 units, a multiple of 8 for the XCD map)
                const int need = (p.tiles_this_rank + 7) & ~7;  // 4 units per tile, 4 waves per block
                // (kCollectiveReserve: room for the RCCL gather of the previous frame)
                // a caller with frames in flight (vrt_scene_set_frames_in_flight)
                // gets 1/grid_div of the resident slots per frame
                const int full = (p.sc.persist_blocks / std::max(1, p.sc.grid_div)) & ~7;
                const int cap = std::max(8, p.nranks > 1 ? full - kCollectiveReserve : full);
                const int g = std::min(cap, need);
                if (kind == kRenderPersistFast) {
                        hipLaunchKernelGGL(k_render_p<true>, dim3(g), dim3(kPersistBlock), 0, st, p);
                        if (hipError_t e = hipGetLastError())
                                return e;
#if VRT_UNIT_DIAG
                        {
                                static int ndump = 0;
                                const size_t nu = std::min<size_t>((size_t)p.tiles_this_rank * 4, kUnitDiagMax);
                                std::vector<uint32_t> d(nu * 4);
                                if (hipStreamSynchronize(st) == hipSuccess &&
                                    hipMemcpyFromSymbol(d.data(), HIP_SYMBOL(g_unit_diag), d.size() * 4) == hipSuccess &&
                                    ndump < 64) {
                                        char name[64];
                                        std::snprintf(name, sizeof name, "gpurun_out/unit_diag_%d.bin", ndump++);
                                        if (FILE *f = std::fopen(name, "wb")) {
                                                std::fwrite(d.data(), 4, d.size(), f);
                                                std::fclose(f);
                                        }
                                        if (VRT_LIGHT_DIAG &&
                                            hipMemcpyFromSymbol(d.data(), HIP_SYMBOL(g_unit_walk), d.size() * 4) == hipSuccess) {
                                                std::snprintf(name, sizeof name, "gpurun_out/unit_walk_%d.bin", ndump - 1);
                                                if (FILE *f = std::fopen(name, "wb")) {
                                                        std::fwrite(d.data(), 4, d.size(), f);
                                                        std::fclose(f);
                                                }
                                        }
                                }
                        }
#endif
                        if (p.test_flags & VRT_TEST_FAIL_LAUNCH)  // test hook: fail between the two launches
                                return hipErrorLaunchFailure;
                        // the deferred pass only when some ray of the frame may
                        // defer, on half the persistent grid, or fewer blocks when
                        // the host's bound says only a few units can be deferred
                        // (each of the grid's waves then takes at most one)
                        const int64_t nd = (p.test_flags & VRT_TEST_FORCE_DEFER) ? INT64_MAX
                                                                                  : camera_defer_bound(p.cam);
                        if (nd > 0) {
                                const int half = std::max(8, (g / 2) & ~7);
                                const int64_t want = ((nd + 3) / 4 + 7) & ~int64_t(7);
                                const int gd = (int)std::min<int64_t>(half, std::max<int64_t>(8, want));
                                hipLaunchKernelGGL(k_render_defer, dim3(gd), dim3(kPersistBlock), 0, st, p);
                        }
                } else {
                        hipLaunchKernelGGL(k_render_p<false>, dim3(g), dim3(kPersistBlock), 0, st, p);
                }
                // failing adds per slice counter: one from every wave of the
                // kPersistHelp XCDs that visit it (g/8 blocks per XCD)
                *q_waves = kPersistHelp * (g / 8) * (kPersistBlock / 64);
                for (int x = 0; x < 8; ++x)
                        slice_units[x] = slice_size(p.tiles_this_rank * 4, x, VRT_SLICE_CHUNK);
                return hipGetLastError();
        }
        // round the grid up to a multiple of 8 (one slot per XCD)
        const int grid = (p.tiles_this_rank * (4) + 7) & ~7;
        void (*kern)(RenderParams) = instrumented ? (w ? k_render<true, true> : k_render<true, false>)
                                                  : (w ? k_render<false, true> : k_render<false, false>);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(kRenderBlock), 0, st, p);
        return hipGetLastError();
}

hipError_t launch_ray_march(const DevScene &sc, const void *d_rays, int64_t n,
                            void *d_hits, hipStream_t st)
{
        if (n <= 0)
                return hipSuccess;
        const int64_t grid = (n + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(sc.wide_leaves ? k_ray_march<true> : k_ray_march<false>, dim3((unsigned)grid),
                           dim3(kBlock), 0, st,
                           sc, static_cast<const float *>(d_rays), n,
                           static_cast<uint32_t *>(d_hits));
        return hipGetLastError();
}

// stbiw__linear_to_rgbe (VRT/stb_image_write.h:601-616) per pixel, the
// per-pixel half of stbi_write_hdr (the scanline RLE stays on the host,
// vrt_hdr.cpp).  Byte-identical to the reference's x86-64 build:
// frexp of the float max component (glibc: NaN / inf keep exponent 0),
// nrm = (m * 256) / max with a correctly rounded divide, and
// (unsigned char)(float) as cvttss2si (out of range / NaN -> INT_MIN).
__device__ __forceinline__ unsigned char cvt_uchar(float f)
{
        const int i = (f >= -2147483648.0f && f < 2147483648.0f) ? (int)f : INT_MIN;
        return (unsigned char)i;
}

__global__ void k_rgbe(const float *__restrict__ img, int64_t npx, int comp,
                       uchar4 *__restrict__ out)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= npx)
                return;
        const float *q = img + i * comp;
        const float r = q[0];
        const float g = comp >= 3 ? q[1] : r;
        const float b = comp >= 3 ? q[2] : r;
        const float m12 = g > b ? g : b;
        const float mx = r > m12 ? r : m12;
        uchar4 o = make_uchar4(0, 0, 0, 0);
        if (!(mx < 1e-32f)) {
                int e = 0;
                float m = mx;
                if (__builtin_isfinite(mx))
                        m = frexpf(mx, &e);
                const float nrm = __fdiv_rn(m * 256.0f, mx);
                o = make_uchar4(cvt_uchar(__fmul_rn(r, nrm)), cvt_uchar(__fmul_rn(g, nrm)),
                                cvt_uchar(__fmul_rn(b, nrm)), (unsigned char)(e + 128));
        }
        out[i] = o;
}

hipError_t launch_rgbe(const float *img, int64_t npx, int comp, uint8_t *out, hipStream_t st)
{
        if (npx <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(k_rgbe, dim3((unsigned)((npx + 255) / 256)), dim3(256), 0, st, img, npx, comp,
                           reinterpret_cast<uchar4 *>(out));
        return hipGetLastError();
}

hipError_t launch_unpack(int nx, int ny, int ntx, int nty, int nranks,
                         int tpr, const float *src, float *dst, hipStream_t st)
{
        const int64_t n = (int64_t)nx * ny;
        if (n <= 0)
                return hipSuccess;
        if (nx % 8 == 0 && ny % 8 == 0 && ntx == nx / 8 && nty == ny / 8 &&
            (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
                const int64_t nq = n * 3 / 4;
                hipLaunchKernelGGL(k_unpack4, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, nx, ny, ntx,
                                   nty, nranks, tpr, reinterpret_cast<const float4 *>(src),
                                   reinterpret_cast<float4 *>(dst));
                return hipGetLastError();
        }
        hipLaunchKernelGGL(k_unpack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           nx, ny, ntx, nty, nranks, tpr, src, dst);
        return hipGetLastError();
}

hipError_t launch_selftest(const double *mt_in, double *mt_out,
                           const float *sat_in, int32_t *sat_out, int64_t n,
                           hipStream_t st)
{
        if (n <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(k_selftest, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                           mt_in, mt_out, sat_in, sat_out, n);
        return hipGetLastError();
}


// ---------------------------------------------------------------------------
// Full trace(): light pass, light-map accumulation in the
// canonical order, cone_trace_init_filter, cone-tracing render.
// ---------------------------------------------------------------------------
// VoxelOctree::illum_d (VRT/voxel_octree.cc:19-20)
__device__ __forceinline__ f3 illum_dir(int i)
{
        const float v = i < 3 ? 1.f : -1.f;
        const int ax = i % 3;
        return mk3(ax == 0 ? v : 0.f, ax == 1 ? v : 0.f, ax == 2 ? v : 0.f);
}

// Grid of the light / trace passes: one one-wave block per work unit,
// rounded up to 8 blocks.  Measured against it and slower: looping blocks
// (a resident grid taking every gridDim.x-th unit, 3-30 % slower for any grid
// size) and blocks of 2 / 4 / 8 consecutive units (light pass -10 / -25 /
// -43 %): the one-block-per-unit launch keeps the most rays in flight.
__host__ __device__ __forceinline__ int trace_vblocks(int tiles)
{
        return (tiles * (4) + 7) & ~7;
}

// XCD-aware block order: block b of nb (a multiple of 8) -> its place in
// the launch's work (blocks b, b + 8, ... run on one XCD and take
// consecutive places: the k_render mapping)
__device__ __forceinline__ int xcd_place(int b, int nb)
{
        return (b & 7) * (nb >> 3) + (b >> 3);
}

// Block b -> work unit with the units dealt to the XCDs in chunks of kC
// consecutive units (chunk j to XCD j % 8), so a dense region of the film
// (a run of heavy units) is shared by all eight XCDs instead of landing on
// one or two of them, as xcd_place's contiguous eighths put it.  kC = 0:
// xcd_place.  Units past the last whole chunk round keep xcd_place's order.
template <int kC>
__device__ __forceinline__ int chunk_place(int b, int nb)
{
        if (kC == 0)
                return xcd_place(b, nb);
        const int x = b & 7, i = b >> 3, per = nb >> 3, full = per / kC * kC;
        if (i >= full)
                return 8 * full + x * (per - full) + (i - full);
        return ((i / kC) * 8 + x) * kC + i % kC;
}
#ifndef VRT_LIGHT_CHUNK
#define VRT_LIGHT_CHUNK 16
#endif
#ifndef VRT_PRIM_CHUNK
#define VRT_PRIM_CHUNK 0
#endif

// 8x8-pixel tile of work unit u and this lane's pixel / sample.  Returns
// false for padding units.
__device__ __forceinline__ bool tile_lane_at(const RenderParams &p, int u, int tid, int &k, int &px, int &py,
                                             int &s, int &lx, int &ly)
{
        constexpr int kQ = 4;  // work units per tile
        if (u >= p.tiles_this_rank * kQ)
                return false;
        k = u / kQ;
        int tx, ty;
        rank_tile(p.ntx, p.nty, p.nranks, p.rank, p.ntx_magic, p.tile_xy, k, tx, ty);
        const int wave = (u % kQ) + (tid >> 6), lane = tid & 63;
        s = lane & 3;
        const int pix = lane >> 2;
        lx = (wave & 1) * 4 + (pix & 3);
        ly = (wave >> 1) * 4 + (pix >> 2);
        px = tx * 8 + lx;
        py = ty * 8 + ly;
        return true;
}
__device__ __forceinline__ bool tile_lane(const RenderParams &p, int u, int &k, int &px, int &py,
                                          int &s, int &lx, int &ly)
{
        return tile_lane_at(p, u, (int)threadIdx.x, k, px, py, s, lx, ly);
}

// Light-pass walks are budgeted: a sample whose walk would pass
// VRT_LIGHT_BUDGET triangle tests is handed (its work unit and lane) to
// k_light_tail, which re-walks it from the root with a group of lanes on
// that one ray (leaf_isect_grp).  The light pass's longest waves are whole
// waves of samples landing in the large leaves under dense geometry (up to
// ~2000 serial triangle tests per lane).
#ifndef VRT_LIGHT_BUDGET
// 768 since round 5: the light map alone builds faster at 256 (round 4's
// choice), but in the whole frame, where the tail runs beside the view's
// primary march, 256 / 512 / 768 / 1,024 / 2,048 give 4.013 / 3.973 / 3.965 /
// 3.962 / 4.17 ms per frame
#define VRT_LIGHT_BUDGET 768
#endif
#ifndef VRT_LIGHT_TAIL_GRID
#define VRT_LIGHT_TAIL_GRID 8192
#endif

__device__ __forceinline__ RayK light_ray(const LightParams &p, int px, int py, int s)
{
        const CamParams &c = p.r.cam;
        const f3 dn = camera_dir(c.s, c.u, c.nf, c.e, c.z, c.nx, c.ny, px, py,
                                 sample_x(s), sample_y(s));
        return make_rayk(mk3(c.origin[0], c.origin[1], c.origin[2]), dn, c.tmin, c.tmax);
}

// one light-map sample record for a hit (m.hit) of sample (px, py, s)
__device__ __forceinline__ void light_record(const LightParams &p, const RayK &r, const MarchResult &m, int px,
                                             int py, int s)
{
        // canonical order: render_mt task t = tx*8 + ty (VRT/camera.h:50-56)
        const int tx = px / p.ptx, ty = py / p.pty;
        const int64_t task = (int64_t)tx * 8 + ty;
        const int64_t key = ((task * p.pty + (py - ty * p.pty)) * p.ptx + (px - tx * p.ptx)) * 4 + s;
        f3 nrm;
        const f3 il = shade_hit(p.r.sc, r, m, nrm);
        const uint32_t j = atomicAdd(p.count, 1u);  // the hit lanes' adds: one atomic per wave
        p.keys[j] = ((uint64_t)m.node << p.kbits) | (uint64_t)key;
        p.vals[j] = j;
        float *o = p.samp + 6 * (int64_t)j;
        o[0] = il.x; o[1] = il.y; o[2] = il.z;
        o[3] = nrm.x; o[4] = nrm.y; o[5] = nrm.z;
}

template <bool kR64>
__device__ __forceinline__ void light_unit(const LightParams &p, uint2 *stk, int u)
{
        const int tid = threadIdx.x;
        int k, px, py, s, lx, ly;
        if (!tile_lane(p.r, u, k, px, py, s, lx, ly))
                return;
        const RayK r = light_ray(p, px, py, s);
        MarchResult m;
#if VRT_LIGHT_DIAG
        const uint64_t dg_t0 = __builtin_amdgcn_s_memtime();
        m.A = m.L = m.T = 0;
#endif
        if (p.r.test_flags & VRT_TEST_LIGHT_TAIL)
                m.deferred = true;  // test hook: every sample to k_light_tail
        else
                ray_march_dispatch<false, kRenderBlock, 1, kR64, VRT_LIGHT_BUDGET>(p.r.sc, r, stk + tid, nullptr,
                                                                                     nullptr, m);
#if VRT_LIGHT_DIAG
        {
                const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memtime() - dg_t0);
                const uint32_t v[8] = { dt, wave_max_u32(m.A), wave_sum_u32(m.A), wave_max_u32(m.L),
                                        wave_sum_u32(m.L), wave_max_u32(m.T), wave_sum_u32(m.T),
                                        wave_sum_u32(m.hit ? 1u : 0u) };
                if (lane_id() < 8 && u < kLightDiagWaves) {
                        uint32_t x = v[0];
#pragma unroll
                        for (int q = 1; q < 8; ++q)
                                x = lane_id() == (uint32_t)q ? v[q] : x;
                        g_light_diag[(size_t)u * 8 + lane_id()] = x;
                }
        }
#endif
        if (m.deferred) {
                const uint32_t j = atomicAdd(p.tail_n, 1u);
                p.tail[j] = (uint32_t)u << 6 | (uint32_t)tid;
                return;
        }
        if (m.hit)
                light_record(p, r, m, px, py, s);
}

#ifndef VRT_LIGHT_WAVES_PER_EU
#define VRT_LIGHT_WAVES_PER_EU 6  // 80 VGPRs (the compiler alone: 98, 4 waves); light map +2 %, round 4
#endif
template <bool kR64>
__global__ __launch_bounds__(kRenderBlock, VRT_LIGHT_WAVES_PER_EU) void k_light(LightParams p)
{
        __shared__ uint2 stk[kStack * kRenderBlock];
        light_unit<kR64>(p, stk, chunk_place<VRT_LIGHT_CHUNK>(blockIdx.x, gridDim.x));
}

// The light pass's deferred samples, one per group of VRT_LIGHT_TAIL_G
// lanes (see VRT_LIGHT_BUDGET): a group walks its sample's ray from the
// root, its lanes alike, with the leaves' records split over them.  Same
// result as the budgeted walk would have reached.
#ifndef VRT_LIGHT_TAIL_G
#define VRT_LIGHT_TAIL_G 8
#endif
#ifndef VRT_TAIL_WAVES_PER_EU
#define VRT_TAIL_WAVES_PER_EU 1  // 1: the compiler's choice
#endif
template <bool kR64>
__global__ __launch_bounds__(64, VRT_TAIL_WAVES_PER_EU) void k_light_tail(LightParams p)
{
        constexpr int kG = VRT_LIGHT_TAIL_G, kR = 64 / kG;  // lanes per sample, samples per wave
        __shared__ uint2 stk[kStack * 64];
        const uint32_t n = *p.tail_n;
        const uint32_t gl = threadIdx.x & (kG - 1);
        for (uint32_t i0 = blockIdx.x * kR; i0 < n; i0 += gridDim.x * kR) {
                const uint32_t i = i0 + threadIdx.x / kG;
                if (i < n) {  // whole groups
                        const uint32_t slot = p.tail[i];
                        int k, px, py, s, lx, ly;
                        tile_lane_at(p.r, (int)(slot >> 6), (int)(slot & 63), k, px, py, s, lx, ly);
                        const RayK r = light_ray(p, px, py, s);
                        MarchResult m;
                        ray_march_dispatch<false, 64, kG, kR64>(p.r.sc, r, stk + threadIdx.x, nullptr, nullptr, m);
                        if (m.hit && gl == 0)
                                light_record(p, r, m, px, py, s);
                }
        }
}

// Permute the per-sample records into the sorted (leaf, canonical) order so
// the serial per-leaf sums below stream contiguous memory.
__global__ __launch_bounds__(256) void k_lm_gather(int64_t n, const uint32_t *__restrict__ vals,
                                                   const float *__restrict__ samp, float *__restrict__ out)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n)
                return;
        const float2 *q = reinterpret_cast<const float2 *>(samp + 6 * (int64_t)vals[i]);
        float2 *o = reinterpret_cast<float2 *>(out + 6 * i);
        o[0] = q[0];
        o[1] = q[1];
        o[2] = q[2];
}

// Start index of every run of equal leaf keys (run order is irrelevant)
// and, per leaf, the end of its run.
__global__ __launch_bounds__(256) void k_lm_segments(int64_t n, const uint64_t *__restrict__ keys, int kbits,
                                                     uint32_t *__restrict__ seg_start, unsigned int *__restrict__ nseg,
                                                     uint32_t *__restrict__ seg_end)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n)
                return;
        const uint64_t leaf = keys[i] >> kbits;
        if (i + 1 == n || (keys[i + 1] >> kbits) != leaf)
                seg_end[leaf] = (uint32_t)(i + 1);
        if (i > 0 && (keys[i - 1] >> kbits) == leaf)
                return;
        seg_start[atomicAdd(nseg, 1u)] = (uint32_t)i;
}

// One 32-lane group per run (stable sort: the run is in canonical sample
// order); lane 3d+c owns the running sum leaf->illum[d][c] and adds
// clamp(dot(illum_d[d], n), 0, 1) * illum[c] sample by sample, from zero
// (VRT/main.cc:90-95).  The 18 sums are independent, so they run side by
// side; each stays a strictly sequential chain.  The run's end is known
// (seg_end), so the samples' loads and coefficients are issued kLmBatch at a
// time ahead of the chain of adds instead of one load round trip per add.
constexpr int kLmBatch = 8;
__global__ __launch_bounds__(256) void k_lm_accum(const float *__restrict__ samp,
                                                  const uint64_t *__restrict__ keys, int kbits,
                                                  const uint32_t *__restrict__ seg_start,
                                                  const unsigned int *__restrict__ nseg,
                                                  const uint32_t *__restrict__ seg_end, LMRec *__restrict__ lm)
{
        const uint32_t seg = blockIdx.x * 8 + (threadIdx.x >> 5);
        const int l = threadIdx.x & 31;
        if (seg >= *nseg || l >= 18)
                return;
        const int d = l / 3, c = l % 3;
        const int64_t i0 = seg_start[seg];
        const uint32_t leaf = (uint32_t)(keys[i0] >> kbits);
        const int64_t i1 = seg_end[leaf];
        const f3 dir = illum_dir(d);
        float acc = 0.f;
        int64_t j = i0;
        for (; j + kLmBatch <= i1; j += kLmBatch) {
                float cf[kLmBatch], v[kLmBatch];
#pragma unroll
                for (int u = 0; u < kLmBatch; ++u) {
                        const float *q = samp + 6 * (j + u);  // gathered into sorted order
                        cf[u] = clampf(dot(dir, mk3(q[3], q[4], q[5])), 0.f, 1.f);
                        v[u] = q[c];
                }
#pragma unroll
                for (int u = 0; u < kLmBatch; ++u)
                        acc = acc + cf[u] * v[u];
        }
        for (; j < i1; ++j) {
                const float *q = samp + 6 * j;
                const float coeff = clampf(dot(dir, mk3(q[3], q[4], q[5])), 0.f, 1.f);
                acc = acc + coeff * q[c];
        }
        lm[leaf].illum[l] = acc;
}

// cone_trace_init_filter, leaf case (VRT/voxel_octree.cc:192-200), run
// first: every leaf's illum starts at zero (k_lm_accum then writes the sums
// of the leaves with hits; an empty leaf has none) and its coverage is set.
// Block 0 also zeroes the build's counters.
__global__ __launch_bounds__(256) void k_lm_leaves(const NodeRec *__restrict__ nodes, int64_t n,
                                                   LMRec *__restrict__ lm, uint32_t *bad, unsigned int *count,
                                                   unsigned int *tail_n, unsigned int *nseg)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i == 0) {
                *bad = 0u;
                *count = 0u;
                *tail_n = 0u;
                *nseg = 0u;
        }
        if (i >= n)
                return;
        const uint32_t a = nodes[i].a;
        if (!(a & kLeafBit))
                return;
        lm[i].cov = (a & ~kLeafBit) == 0 ? 0.f : 1.f;
#pragma unroll
        for (int f = 0; f < 18; ++f)
                lm[i].illum[f] = 0.f;
}

// cone_trace_init_filter, internal case for one BFS level (children in
// order 0..7 summed from zero, then / 8; VRT/voxel_octree.cc:201-213)
__global__ __launch_bounds__(256) void k_lm_level(const NodeRec *__restrict__ nodes, int64_t begin,
                                                  int64_t end, LMRec *__restrict__ lm)
{
        const int64_t i = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= end)
                return;
        const uint32_t a = nodes[i].a;
        if (a & kLeafBit)
                return;
        float cov = 0.f;
        float acc[18];
#pragma unroll
        for (int f = 0; f < 18; ++f)
                acc[f] = 0.f;
        for (int c = 0; c < 8; ++c) {
                const LMRec &ch = lm[a + c];
                cov += ch.cov;
#pragma unroll
                for (int f = 0; f < 18; ++f)
                        acc[f] += ch.illum[f];
        }
#pragma unroll
        for (int f = 0; f < 18; ++f)
                lm[i].illum[f] = acc[f] / 8.0f;
        lm[i].cov = cov / 8.f;
}

// VoxelOctree::compute_illum (VRT/voxel_octree.h:72-82)
__device__ __forceinline__ f3 compute_illum(const LMRec *__restrict__ lm, uint32_t ni, f3 d)
{
        const float4 *q = reinterpret_cast<const float4 *>(lm + ni);
        const float4 q0 = q[0], q1 = q[1], q2 = q[2], q3 = q[3], q4 = q[4];
        const float L[18] = { q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y,
                              q2.z, q2.w, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, q4.z };
        f3 r = mk3(0.f, 0.f, 0.f);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
                float coeff = dot(illum_dir(i), d);
                coeff = clampf(coeff, 0.f, 1.f);
                r = mk3(r.x + coeff * L[3 * i + 0], r.y + coeff * L[3 * i + 1], r.z + coeff * L[3 * i + 2]);
        }
        return r;
}

// (int)log2f(x) for x >= 1 through the host-libm threshold table
__device__ __forceinline__ int split_level_of(float x, const float *up)
{
        const int e = (int)(__float_as_uint(x) >> 23) - 127;
        if (e >= 63)
                return e;  // unreachable for finite scenes (maxdist/mindist < 2^63)
        return x >= up[e] ? e + 1 : e;
}

// Cone-descent record per node (box centre as AABB3D::center computes it,
// child word) and a flag raised when any light-map value is not finite.
__global__ __launch_bounds__(256) void k_lm_aux(const NodeRec *__restrict__ nodes, const LMRec *__restrict__ lm,
                                                int64_t n, float4 *__restrict__ cc, uint32_t *bad)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i >= n)
                return;
        const NodeRec nr = nodes[i];
        cc[i] = make_float4((nr.bmin[0] + nr.bmax[0]) * .5f, (nr.bmin[1] + nr.bmax[1]) * .5f,
                            (nr.bmin[2] + nr.bmax[2]) * .5f, __uint_as_float(nr.a));
        bool ok = __builtin_isfinite(lm[i].cov);
#pragma unroll
        for (int f = 0; f < 18; ++f)
                ok = ok && __builtin_isfinite(lm[i].illum[f]);
        if (!ok)
                atomicOr(bad, 1u);
}

// Fast cone march (finite light map): the same values as cone_march_ref.
// Two exact shortcuts: a node with coverage +0 adds w * illum = +-0 to the
// running sum (w = ... * cov) and transparency * 0 to the opacity, which
// leave them unchanged (the sums start at +0 and never become -0), so its
// illum is not read; and compute_illum's terms with coefficient +0 are +-0
// for finite illum and are skipped the same way.  Descent reads 16-B
// centre/child records.
__device__ __forceinline__ f3 cone_march_fast(const TraceParams &p, f3 o, f3 d)
{
        const float aperture = 0.577350269f, step = .1f, decay = 1.f;
        const f3 nd = -d;
        float co[6];
#pragma unroll
        for (int i = 0; i < 6; ++i)
                co[i] = clampf(dot(illum_dir(i), nd), 0.f, 1.f);
        float dist = p.mindist;
        float opacity = 0.f;
        f3 diffuse = mk3(0.f, 0.f, 0.f);
        // the split level of the current diameter (non-increasing as the
        // diameter grows: TraceParams::split_bound), and its bound
        int level = -1;
        float bound = 0.f;
        for (int guard = 0; dist < p.maxdist && opacity < 1.f && guard < (1 << 16); ++guard) {
                const f3 pt = o + d * dist;
                const float diam = std_max(p.mindist, aperture * 2.f * dist);
                if (p.maxdist < diam)
                        break;
                if (level < 0) {  // first step: the reference's division once
                        level = min(split_level_of(p.maxdist / diam, p.split_up), 63);  // >= 63: below any node
                        bound = p.split_bound[level];
                }
                while (level > 0 && diam > bound) {
                        --level;
                        bound = p.split_bound[level];
                }
                int split = level;
                uint32_t ni = 0;
                float4 c = p.cc[0];
                uint32_t a = __float_as_uint(c.w);
                while (!(a & kLeafBit) && split) {
                        int i = 0;
                        i += (pt.x > c.x ? 4 : 0);
                        i += (pt.y > c.y ? 2 : 0);
                        i += (pt.z > c.z ? 1 : 0);
                        ni = a + (uint32_t)i;
                        c = p.cc[ni];
                        a = __float_as_uint(c.w);
                        split--;
                }
                if (split == 0) {
                        const float cov = p.lm[ni].cov;
                        if (cov != 0.f) {
                                const float *L = p.lm[ni].illum;
                                f3 il = mk3(0.f, 0.f, 0.f);
#pragma unroll
                                for (int i = 0; i < 6; ++i)
                                        if (co[i] != 0.f)
                                                il = mk3(il.x + co[i] * L[3 * i + 0], il.y + co[i] * L[3 * i + 1],
                                                         il.z + co[i] * L[3 * i + 2]);
                                const float transparency = clampf(1.f - opacity, 0.f, 1.f);
                                const float aa = cov * step;
                                const float w = (1.f / (1.f + decay * dist)) * transparency * cov;
                                diffuse = mk3(diffuse.x + w * il.x, diffuse.y + w * il.y, diffuse.z + w * il.z);
                                opacity += transparency * aa;
                        }
                }
                dist += step * diam;
        }
        return diffuse;
}

__device__ __forceinline__ int octant_of(const f3 &pt, const float4 &c)
{
        return (pt.x > c.x ? 4 : 0) + (pt.y > c.y ? 2 : 0) + (pt.z > c.z ? 1 : 0);
}

// cone_march_fast with one memory round trip per descent level and one per
// light-map read (finite light map, every lane's cone having at most one
// non-zero coefficient per axis: the caller checks).  The descent consumes
// each 16-B (centre, child) record in the iteration that loads it (the next
// octant is computed right away, also for a leaf, where it is unused), so
// the record is one load; the root record is loaded once per cone.  A
// light-map read fetches the coverage and, per axis, the illum vector of the
// direction the cone faces (index a if co[a] != 0, else a + 3) together,
// whatever the coverage; the sum over the 6 directions then runs in index
// order 0..5 with the unselected slots adding +0: the terms cone_march_fast
// skips (coefficient +0) and these +0 slots leave il unchanged, since il
// starts at +0 and under round-to-nearest never becomes -0, so the sums are
// bit-identical.
//
// The descent also records the cell of the point it followed -- per
// axis the half-open interval (lo, hi] cut by the centres whose octant
// choice it used (pt > centre: lo, else hi; the octree's cells are nested,
// max/min keep the tightest), a property of the node reached, read from
// TraceParams::cells -- and the next step at the same split level
// whose point lies in that cell makes the same choices at every node of the
// path, so it reuses the node (and whether the descent ended above the split
// level) without descending.  Any other step descends from the root.
//
// The steps come from the cone step table (k_cone_steps): a step's
// distance, split level and distance weight depend on mindist and maxdist
// only, not on the cone, so they are computed once per frame and read here
// with scalar loads; the cone ends at the table's end or at opacity 1, where
// the reference's loop ends.
__device__ __forceinline__ f3 cone_march_axes(const TraceParams &p, f3 o, f3 d, const float co[6], int nsteps)
{
        const float step = .1f;
        const int jx = co[0] != 0.f ? 0 : 3, jy = co[1] != 0.f ? 1 : 4, jz = co[2] != 0.f ? 2 : 5;
        const float cx = co[jx], cy = co[jy], cz = co[jz];
        const float4 c0 = p.cc[0];
        const uint32_t a0 = __float_as_uint(c0.w);
        float opacity = 0.f;
        f3 diffuse = mk3(0.f, 0.f, 0.f);
        // the last descent's cell
        f3 lo = mk3(0.f, 0.f, 0.f), hi = lo;
        int c_level = -1;
        // the last descent's node: its coverage (+0 when the descent ended
        // above the split level: the step adds nothing) and illumination
        float cov = 0.f;
        f3 il = mk3(0.f, 0.f, 0.f);
        // (constant address space, index the same in every active lane: the
        // entries are scalar loads)
        typedef const __attribute__((address_space(4))) float ConstF;
        ConstF *tab = (ConstF *)p.steps;
        for (int k = 0; k < nsteps && opacity < 1.f; ++k) {
                const int ku = __builtin_amdgcn_readfirstlane(k) * 4;
                const float dist = tab[ku], inv = tab[ku + 1];
                const int level = __float_as_int(tab[ku + 2]);
                const f3 pt = o + d * dist;
                // one divergent region per step: the cell test without
                // short-circuit branches (& of the compares)
                const bool same = (level == c_level) & (pt.x > lo.x) & (pt.x <= hi.x) & (pt.y > lo.y) &
                                  (pt.y <= hi.y) & (pt.z > lo.z) & (pt.z <= hi.z);
                if (!same) {
                        int split = level;
                        uint32_t ni = 0, a = a0;
                        int i = octant_of(pt, c0);
                        while (!(a & kLeafBit) && split) {
                                ni = a + (uint32_t)i;
                                const float4 c = p.cc[ni];
                                a = __float_as_uint(c.w);
                                i = octant_of(pt, c);
                                split--;
                        }
                        // the cell of the path (precomputed per node: cone_cells)
                        const float4 l4 = p.cells[2 * ni], h4 = p.cells[2 * ni + 1];
                        lo = mk3(l4.x, l4.y, l4.z);
                        hi = mk3(h4.x, h4.y, h4.z);
                        c_level = level;
                        // the node's light-map entry (a valid node also when the
                        // descent ended at a leaf above the split level, whose
                        // coverage is then taken as +0)
                        const LMRec *R = p.lm + ni;
                        float L[9];
                        float cv = R->cov;
#pragma unroll
                        for (int q = 0; q < 3; ++q) {
                                L[q] = R->illum[3 * jx + q];
                                L[3 + q] = R->illum[3 * jy + q];
                                L[6 + q] = R->illum[3 * jz + q];
                        }
                        cov = split == 0 ? cv : 0.f;
                        const f3 tx = mk3(cx * L[0], cx * L[1], cx * L[2]);
                        const f3 ty = mk3(cy * L[3], cy * L[4], cy * L[5]);
                        const f3 tz = mk3(cz * L[6], cz * L[7], cz * L[8]);
                        const f3 z0 = mk3(0.f, 0.f, 0.f);
                        il = z0;
                        il = il + (jx == 0 ? tx : z0);
                        il = il + (jy == 1 ? ty : z0);
                        il = il + (jz == 2 ? tz : z0);
                        il = il + (jx == 3 ? tx : z0);
                        il = il + (jy == 4 ? ty : z0);
                        il = il + (jz == 5 ? tz : z0);
                }
                // branch-free: with cov = +0 (coverage zero, or no node at the
                // split level) w = +0 and transparency * aa = +0, and w * il is
                // +-0 for the finite il of a finite light map, so diffuse and
                // opacity keep their values bit for bit (they start at +0 and
                // never become -0), exactly as the reference's skipped step
                const float transparency = clampf(1.f - opacity, 0.f, 1.f);
                const float aa = cov * step;
                const float w = inv * transparency * cov;  // inv = 1 / (1 + decay * dist)
                diffuse = mk3(diffuse.x + w * il.x, diffuse.y + w * il.y, diffuse.z + w * il.z);
                opacity += transparency * aa;
        }
        return diffuse;
}

// The cone march's step sequence (cone_trace's loop, VRT/voxel_octree.cc:
// 276-311, with the split level kept by the split_bound cursor): per step
// (dist, 1 / (1 + decay * dist), split level, diam), the same operations as
// cone_march_fast's loop header, up to the step where dist reaches maxdist
// or maxdist < diam.  -1 if longer than kConeSteps.  One lane, launched
// after k_trace_prim (k_cones_film follows on the stream).
__global__ __launch_bounds__(64) void k_cone_steps(TraceParams p)
{
        if (threadIdx.x != 0)
                return;
        const float aperture = 0.577350269f, step = .1f, decay = 1.f;
        float dist = p.mindist;
        int level = -1, n = 0;
        float bound = 0.f;
        for (int guard = 0; dist < p.maxdist && guard < (1 << 16); ++guard) {
                const float diam = std_max(p.mindist, aperture * 2.f * dist);
                if (p.maxdist < diam)
                        break;
                if (level < 0) {
                        level = min(split_level_of(p.maxdist / diam, p.split_up), 63);
                        bound = p.split_bound[level];
                }
                while (level > 0 && diam > bound) {
                        --level;
                        bound = p.split_bound[level];
                }
                if (n == kConeSteps) {
                        n = -1;
                        break;
                }
                p.steps[n++] = make_float4(dist, 1.f / (1.f + decay * dist), __int_as_float(level), diam);
                dist += step * diam;
        }
        *p.nsteps = n;
}

// cone_trace(root, cone, min_voxel_size) (VRT/voxel_octree.cc:276-311)
__device__ __forceinline__ f3 cone_march_ref(const TraceParams &p, f3 o, f3 d);

__device__ __forceinline__ f3 cone_march(const TraceParams &p, f3 o, f3 d)
{
        if (*p.lm_bad == 0u) {
                const f3 nd = -d;
                float co[6];
#pragma unroll
                for (int i = 0; i < 6; ++i)
                        co[i] = clampf(dot(illum_dir(i), nd), 0.f, 1.f);
                const bool twin = (co[0] != 0.f && co[3] != 0.f) || (co[1] != 0.f && co[4] != 0.f) ||
                                  (co[2] != 0.f && co[5] != 0.f);
                const int nsteps = *p.nsteps;
                if (!twin && nsteps >= 0 && nsteps <= kConeSteps)
                        return cone_march_axes(p, o, d, co, nsteps);
                return cone_march_fast(p, o, d);  // a NaN direction (or no step table)
        }
        return cone_march_ref(p, o, d);
}

__device__ __forceinline__ f3 cone_march_ref(const TraceParams &p, f3 o, f3 d)
{
        const float aperture = 0.577350269f, step = .1f, decay = 1.f;
        const NodeRec *__restrict__ nodes = p.r.sc.nodes;
        const f3 nd = -d;
        float dist = p.mindist;
        float opacity = 0.f;
        f3 diffuse = mk3(0.f, 0.f, 0.f);
        // (the host rejects mindist <= 0, which would never terminate; the
        // step cap is a guard only: dist grows >= 11% per step)
        for (int guard = 0; dist < p.maxdist && opacity < 1.f && guard < (1 << 16); ++guard) {
                const f3 pt = o + d * dist;
                const float diam = std_max(p.mindist, aperture * 2.f * dist);
                if (p.maxdist < diam)
                        break;
                int split = split_level_of(p.maxdist / diam, p.split_up);
                uint32_t ni = 0;
                float bmin[3], bmax[3];
                uint32_t a, b;
                load_node(nodes, 0, bmin, bmax, a, b);
                while (!(a & kLeafBit) && split) {
                        const float cx = (bmin[0] + bmax[0]) * .5f;
                        const float cy = (bmin[1] + bmax[1]) * .5f;
                        const float cz = (bmin[2] + bmax[2]) * .5f;
                        int i = 0;
                        i += (pt.x > cx ? 4 : 0);
                        i += (pt.y > cy ? 2 : 0);
                        i += (pt.z > cz ? 1 : 0);
                        ni = a + (uint32_t)i;
                        load_node(nodes, ni, bmin, bmax, a, b);
                        split--;
                }
                if (split == 0) {
                        const f3 il = compute_illum(p.lm, ni, nd);
                        const float transparency = clampf(1.f - opacity, 0.f, 1.f);
                        const float cov = p.lm[ni].cov;
                        const float aa = cov * step;
                        const float w = (1.f / (1.f + decay * dist)) * transparency * cov;
                        diffuse = mk3(diffuse.x + w * il.x, diffuse.y + w * il.y, diffuse.z + w * il.z);
                        opacity += transparency * aa;
                }
                dist += step * diam;
        }
        return diffuse;
}

// cone_trace(root, isect, min_voxel_size) with orthonormal_basis
// (VRT/voxel_octree.cc:256-274, 313-330) over a sample record (hit point in
// rec[0].xyz, normal in rec[1].xyz), the record re-read and the basis remade
// per cone -- the same operations, so the same values (volatile asm keeps the
// compiler from hoisting the record across the marches)
__device__ __forceinline__ f3 cone_trace_rec(const TraceParams &p, const float4 *rec)
{
        const float hx[6] = { 0.000000f, 0.000000f, 0.823639f, 0.509037f, -0.509037f, -0.823639f };
        const float hy[6] = { 0.000000f, 0.866025f, 0.267617f, -0.700629f, -0.700629f, 0.267617f };
        const float hz[6] = { 1.0f, 0.5f, 0.5f, 0.5f, 0.5f, 0.5f };
        const float hw[6] = { 0.25f, 0.15f, 0.15f, 0.15f, 0.15f, 0.15f };
        f3 diffuse = mk3(0.f, 0.f, 0.f);
        for (int i = 0; i < 6; ++i) {
                const float4 *q = rec;
                asm volatile("" : "+v"(q));
                const float4 r0 = q[0], r1 = q[1];
                const f3 hit = mk3(r0.x, r0.y, r0.z), n = mk3(r1.x, r1.y, r1.z);
                const float sg = (0.0f > n.z) ? -1.0f : 1.0f;
                const float a0 = -1.0f / (sg + n.z);
                const float a1 = n.x * n.y * a0;
                const f3 t = mk3(1.0f + sg * n.x * n.x * a0, sg * a1, -sg * n.x);
                const f3 bb = mk3(a1, sg + n.y * n.y * a0, -n.y);
                f3 r = mk3(0.f, 0.f, 0.f);
                r = r + t * hx[i];
                r = r + bb * hy[i];
                r = r + n * hz[i];
                const f3 cd = normalize(r);
                const f3 cm = cone_march(p, hit, cd);
                diffuse = diffuse + cm * hw[i];
        }
        return diffuse;
}


// ---- split trace: primary pass, one lane per (sample, cone), film add ----
// Primary pass: trace()'s ray_march + get_albedo + leaf compute_illum(-d);
// slot = work unit * kRenderBlock + tid.
// The primary pass's walks can be budgeted as the light pass's
// (VRT_LIGHT_BUDGET): a sample past VRT_PRIM_BUDGET triangle tests is
// re-walked by k_trace_prim_tail with a group of lanes, which writes its
// record.  Off by default: the view's long walks are not a few waves'
// tail as the light pass's are, and the re-walks cost more than they save
// (VRT_TEST_PRIM_TAIL still runs the tail path in the tests).
#ifndef VRT_PRIM_BUDGET
#define VRT_PRIM_BUDGET 0  // off: 256 / 128 / 512 measured -11 / -21 / -3.5 % on the render (the view's deferred samples are many)
#endif
__device__ __forceinline__ RayK trace_ray(const TraceParams &p, int px, int py, int s)
{
        const CamParams &c = p.r.cam;
        const f3 dn = camera_dir(c.s, c.u, c.nf, c.e, c.z, c.nx, c.ny, px, py,
                                 sample_x(s), sample_y(s));
        return make_rayk(mk3(c.origin[0], c.origin[1], c.origin[2]), dn, c.tmin, c.tmax);
}

__device__ __forceinline__ void trace_prim_record(const TraceParams &p, const RayK &r, const MarchResult &m,
                                                  int64_t slot)
{
        float4 *o = p.rec + 4 * slot;
        if (m.hit) {
                f3 nrm;
                const f3 albedo = hit_albedo(p.r.sc, m, nrm);
                // the hit leaf and -d: the direct term compute_illum(leaf, -d)
                // is taken in k_cones_film, so this pass never reads the light
                // map and can run while the light map is being built
                const f3 nd = -r.d;
                o[0] = make_float4(m.hp.x, m.hp.y, m.hp.z, 1.f);
                o[1] = make_float4(nrm.x, nrm.y, nrm.z, 0.f);
                o[2] = make_float4(albedo.x, albedo.y, albedo.z, 0.f);
                o[3] = make_float4(__uint_as_float(m.node), nd.x, nd.y, nd.z);
        } else {
                const f3 sk = sky(r.d.y);
                o[0] = make_float4(0.f, 0.f, 0.f, 0.f);
                o[2] = make_float4(sk.x, sk.y, sk.z, 0.f);
        }
}

template <bool kR64>
__device__ __forceinline__ void trace_prim_unit(const TraceParams &p, uint2 *stk, int u)
{
        const int tid = threadIdx.x;
        int k, px, py, s, lx, ly;
        if (!tile_lane(p.r, u, k, px, py, s, lx, ly))
                return;
        const int64_t slot = (int64_t)u * kRenderBlock + tid;
        const RayK r = trace_ray(p, px, py, s);
        MarchResult m;
        if (p.r.test_flags & VRT_TEST_PRIM_TAIL)
                m.deferred = true;  // test hook: every sample to k_trace_prim_tail
        else
                ray_march_dispatch<false, kRenderBlock, 1, kR64, VRT_PRIM_BUDGET>(p.r.sc, r, stk + tid, nullptr,
                                                                                    nullptr, m);
        if (m.deferred) {
                const uint32_t j = atomicAdd(p.tail_n, 1u);
                p.tail[j] = (uint32_t)slot;
                return;
        }
        trace_prim_record(p, r, m, slot);
}

#ifndef VRT_PRIM_WAVES_PER_EU
#define VRT_PRIM_WAVES_PER_EU 1  // 1: the compiler's choice
#endif
template <bool kR64>
__global__ __launch_bounds__(kRenderBlock, VRT_PRIM_WAVES_PER_EU) void k_trace_prim(TraceParams p)
{
        __shared__ uint2 stk[kStack * kRenderBlock];
        trace_prim_unit<kR64>(p, stk, chunk_place<VRT_PRIM_CHUNK>(blockIdx.x, gridDim.x));
}

// The primary pass's deferred samples, one per group of VRT_LIGHT_TAIL_G
// lanes (as k_light_tail): the group re-walks the sample from the root and
// its first lane writes the sample's record.
template <bool kR64>
__global__ __launch_bounds__(64) void k_trace_prim_tail(TraceParams p)
{
        constexpr int kG = VRT_LIGHT_TAIL_G, kR = 64 / kG;
        __shared__ uint2 stk[kStack * 64];
        const uint32_t n = *p.tail_n;
        for (uint32_t i0 = blockIdx.x * kR; i0 < n; i0 += gridDim.x * kR) {
                const uint32_t i = i0 + threadIdx.x / kG;
                if (i < n) {  // whole groups
                        const uint32_t slot = p.tail[i];
                        int k, px, py, s, lx, ly;
                        tile_lane_at(p.r, (int)(slot / kRenderBlock), (int)(slot % kRenderBlock), k, px, py, s, lx,
                                     ly);
                        const RayK r = trace_ray(p, px, py, s);
                        MarchResult m;
                        ray_march_dispatch<false, 64, kG, kR64>(p.r.sc, r, stk + threadIdx.x, nullptr, nullptr, m);
                        if ((threadIdx.x & (kG - 1)) == 0)
                                trace_prim_record(p, r, m, slot);
                }
        }
}

// Cones + film: one wave per work unit of the primary pass (its 64 sample
// slots: 16 pixels x 4 samples, lane = 4 * pixel + sample).  A hit lane
// marches the 6 cones one after the other (the wave marches the same cone of
// 64 neighbouring samples at a time: coherent node reads) and sums them in
// cone order from zero as cone_trace does (VRT/voxel_octree.cc:276-311),
// then trace()'s get_albedo * (indirect + direct) (VRT/main.cc:22-27); a
// miss keeps its sky colour.  The pixel's 4 samples are added in sample order
// with cross-lane reads (Film::add(c * .25f), VRT/main.cc:121) and the
// pixel is written once: each sample record is read once, and no per-cone
// result goes through memory.
#ifndef VRT_CONES_WAVES_PER_EU
#define VRT_CONES_WAVES_PER_EU 8  // 64 VGPRs, 24 B/lane of spill: +1.9 % over 7 waves (70 VGPRs) since the step table and cells (round 5; round 4, before them: 7 waves +9.8 %)
#endif
__global__ __launch_bounds__(64, VRT_CONES_WAVES_PER_EU) void k_cones_film(TraceParams p)
{
        const int u = blockIdx.x;
        constexpr int kQ = 4;
        if (u >= p.r.tiles_this_rank * kQ)
                return;
        const int64_t slot = (int64_t)u * 64 + threadIdx.x;
        f3 col;
        if (p.rec[4 * slot + 0].w != 0.f) {
                // cone_trace with the hit point and normal read from the
                // sample record per cone (L2 hits) and the basis remade per
                // cone -- the same values -- rather than held in registers
                // across the 6 cone marches
                const f3 diffuse = cone_trace_rec(p, p.rec + 4 * slot);
                const float4 r2 = p.rec[4 * slot + 2], r3 = p.rec[4 * slot + 3];
                const f3 direct = compute_illum(p.lm, __float_as_uint(r3.x), mk3(r3.y, r3.z, r3.w));
                const f3 lsum = diffuse + direct;
                col = mk3(r2.x * lsum.x, r2.y * lsum.y, r2.z * lsum.z);
        } else {
                const float4 r2 = p.rec[4 * slot + 2];
                col = mk3(r2.x, r2.y, r2.z);
        }
        // the pixel of this lane, made after the cone marches (not held across them)
        const int lane = threadIdx.x;
        const int k = u / kQ, wave = u % kQ;
        int tx, ty;
        rank_tile(p.r.ntx, p.r.nty, p.r.nranks, p.r.rank, p.r.ntx_magic, p.r.tile_xy, k, tx, ty);
        const int s = lane & 3, pix = lane >> 2;
        const int lx = (wave & 1) * 4 + (pix & 3), ly = (wave >> 1) * 4 + (pix >> 2);
        const int px = tx * 8 + lx, py = ty * 8 + ly;
        const size_t si = ((size_t)py * p.r.cam.nx + px) * 4 + s;
        if (p.r.so.hit)
                p.r.so.hit[si] = p.rec[4 * slot + 0].w != 0.f ? 1 : 0;
        if (p.r.so.rgb) {
                p.r.so.rgb[3 * si + 0] = col.x;
                p.r.so.rgb[3 * si + 1] = col.y;
                p.r.so.rgb[3 * si + 2] = col.z;
        }
        const f3 cq = col * .25f;
        const int l0 = lane & ~3;
        float acc[3] = { 0.0f, 0.0f, 0.0f };
        const float cv[3] = { cq.x, cq.y, cq.z };
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
                for (int q = 0; q < 3; ++q)
                        acc[q] += __shfl(cv[q], l0 + j, 64);
        }
        if (s == 0) {
                float *o;
                if (p.r.image_layout)
                        o = p.r.out + ((size_t)py * p.r.cam.nx + px) * 3;
                else
                        o = p.r.out + ((size_t)k * 64 + ly * 8 + lx) * 3;
                o[0] = acc[0];
                o[1] = acc[1];
                o[2] = acc[2];
        }
}

// VRT_LIGHT_DIAG builds: the per-wave records of the last light pass
hipError_t light_diag_copy(void *host, size_t bytes)
{
#if VRT_LIGHT_DIAG
        return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_light_diag), bytes);
#else
        (void)host;
        (void)bytes;
        return hipErrorNotSupported;
#endif
}

hipError_t launch_light(const LightParams &p, hipStream_t st)
{
        if (p.r.tiles_this_rank <= 0)
                return hipSuccess;
        const int grid = trace_vblocks(p.r.tiles_this_rank);
        hipLaunchKernelGGL(p.r.sc.wide_leaves ? k_light<true> : k_light<false>, dim3(grid), dim3(kRenderBlock), 0, st, p);
        if (VRT_LIGHT_BUDGET > 0 || (p.r.test_flags & VRT_TEST_LIGHT_TAIL))
                hipLaunchKernelGGL(p.r.sc.wide_leaves ? k_light_tail<true> : k_light_tail<false>,
                                   dim3(VRT_LIGHT_TAIL_GRID), dim3(64), 0, st, p);
        return hipGetLastError();
}

hipError_t launch_lm_accum(int64_t n, const uint64_t *keys_sorted, const uint32_t *vals_sorted, int kbits,
                           const float *samp, uint32_t *seg_start, unsigned int *nseg,
                           int64_t max_seg, uint32_t *seg_end, LMRec *lm, hipStream_t st)
{
        if (n <= 0)
                return hipSuccess;
        // samp -> gathered copy directly after it (the caller sizes 2 x 24 B
        // per sample)
        float *sorted = const_cast<float *>(samp) + 6 * n;
        const unsigned g = (unsigned)((n + 255) / 256);
        hipLaunchKernelGGL(k_lm_gather, dim3(g), dim3(256), 0, st, n, vals_sorted, samp, sorted);
        hipLaunchKernelGGL(k_lm_segments, dim3(g), dim3(256), 0, st, n, keys_sorted, kbits, seg_start, nseg, seg_end);
        if (max_seg > 0)
                hipLaunchKernelGGL(k_lm_accum, dim3((unsigned)((max_seg + 7) / 8)), dim3(256), 0, st, sorted,
                                   keys_sorted, kbits, seg_start, nseg, seg_end, lm);
        return hipGetLastError();
}

hipError_t launch_lm_leaves(const NodeRec *nodes, int64_t nnodes, LMRec *lm, uint32_t *bad, unsigned int *count,
                            unsigned int *tail_n, unsigned int *nseg, hipStream_t st)
{
        const unsigned g = (unsigned)std::max<int64_t>(1, (nnodes + 255) / 256);
        hipLaunchKernelGGL(k_lm_leaves, dim3(g), dim3(256), 0, st, nodes, nnodes, lm, bad, count, tail_n, nseg);
        return hipGetLastError();
}

hipError_t launch_lm_level(const NodeRec *nodes, int64_t begin, int64_t end, LMRec *lm, hipStream_t st)
{
        if (end <= begin)
                return hipSuccess;
        hipLaunchKernelGGL(k_lm_level, dim3((unsigned)((end - begin + 255) / 256)), dim3(256), 0, st, nodes, begin,
                           end, lm);
        return hipGetLastError();
}

hipError_t launch_trace(const TraceParams &p, hipStream_t st)
{
        if (p.r.tiles_this_rank <= 0)
                return hipSuccess;
        if (hipError_t e = launch_trace_prim(p, st))
                return e;
        return launch_cones(p, st);
}

// the split trace's two halves: the primary march (no light-map read) and
// the cones + film pass (reads the light map)
hipError_t launch_trace_prim(const TraceParams &p, hipStream_t st)
{
        if (p.r.tiles_this_rank <= 0)
                return hipSuccess;
        const bool tail = VRT_PRIM_BUDGET > 0 || (p.r.test_flags & VRT_TEST_PRIM_TAIL);
        if (tail)
                if (hipError_t e = hipMemsetAsync(p.tail_n, 0, 4, st))
                        return e;
        hipLaunchKernelGGL(p.r.sc.wide_leaves ? k_trace_prim<true> : k_trace_prim<false>,
                           dim3(trace_vblocks(p.r.tiles_this_rank)), dim3(kRenderBlock), 0, st, p);
        if (tail)
                hipLaunchKernelGGL(p.r.sc.wide_leaves ? k_trace_prim_tail<true> : k_trace_prim_tail<false>,
                                   dim3(VRT_LIGHT_TAIL_GRID), dim3(64), 0, st, p);
        if (p.build_steps)
                hipLaunchKernelGGL(k_cone_steps, dim3(1), dim3(64), 0, st, p);
        return hipGetLastError();
}

hipError_t launch_cones(const TraceParams &p, hipStream_t st)
{
        if (p.r.tiles_this_rank <= 0)
                return hipSuccess;
        const int64_t nslots = (int64_t)p.r.tiles_this_rank * 256;
        hipLaunchKernelGGL(k_cones_film, dim3((unsigned)(nslots / 64)), dim3(64), 0, st, p);
        return hipGetLastError();
}

hipError_t launch_lm_aux(const NodeRec *nodes, const LMRec *lm, int64_t n, float4 *cc, uint32_t *bad,
                         hipStream_t st)
{
        if (n <= 0)
                return hipSuccess;
        hipLaunchKernelGGL(k_lm_aux, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nodes, lm, n, cc, bad);
        return hipGetLastError();
}

// The compile-time switches of this kernel build that select a path
// (vrt_build_flag): the tests assert on them, so a build that silently turns
// a path off (e.g. config 5's compaction, VRT_SEC_SPILL_T=0) fails its tests.
bool build_flag(const char *name, int64_t *value)
{
        static const struct {
                const char *name;
                int64_t value;
        } kFlags[] = {
                { "VRT_SEC_SPILL_T", VRT_SEC_SPILL_T },

                { "VRT_SEC_SLICE_CHUNK", VRT_SEC_SLICE_CHUNK },
                { "VRT_SEC_TAKE", VRT_SEC_TAKE },

                { "VRT_SLICE_CHUNK", VRT_SLICE_CHUNK },
                { "VRT_DEAL_BLOCK", VRT_DEAL_BLOCK },
                { "VRT_DEAL_WEIGHT", VRT_DEAL_WEIGHT },
                { "VRT_DEAL_SPAN", VRT_DEAL_SPAN },
                { "VRT_LIGHT_BUDGET", VRT_LIGHT_BUDGET },
                { "VRT_PRIM_BUDGET", VRT_PRIM_BUDGET },
        };
        for (const auto &f : kFlags)
                if (std::strcmp(f.name, name) == 0) {
                        *value = f.value;
                        return true;
                }
        return false;
}

}  // namespace vrt

#if VRT_PHASE_STAMPS
extern "C" __attribute__((visibility("default"))) int vrt_diag_phases(unsigned long long out[24], int reset)
{
        if (hipMemcpyFromSymbol(out, HIP_SYMBOL(vrt::g_phase), sizeof(unsigned long long) * vrt::kPhaseWords) !=
            hipSuccess)
                return -1;
        if (reset) {
                unsigned long long z[vrt::kPhaseWords] = {};
                if (hipMemcpyToSymbol(HIP_SYMBOL(vrt::g_phase), z, sizeof z) != hipSuccess)
                        return -1;
        }
        return 0;
}
#endif
