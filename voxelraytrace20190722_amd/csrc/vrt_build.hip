// vrt_build.hip -- octree build on the GPU.
//
// Same octree as the host build (vrt_host.cpp: build_tree) and as the
// reference's recursive insert()/split() (VRT/voxel_octree.cc:27-75): a node
// at depth < max_depth is split iff some triangle overlaps it and all its
// ancestors (Triangle::is_overlap = triBoxOverlap on the node's exact float
// box, VRT/voxel_octree.cc:486-492); a max-depth leaf lists exactly those
// triangles, in input order.  Level-synchronous on the device:
//   frontier P_l = (triangle, node code, node box) pairs that overlap;
//   k_expand tests the 8 children of every pair (SAT) and appends the
//   overlapping ones to P_{l+1} (wave-aggregated atomics; order is
//   irrelevant because everything below is sorted);
//   internal nodes of level l = sorted unique codes of P_l (hipCUB);
//   leaf lists = sorted (code << 32 | tri) of P_max_depth.
// Then the BFS child-block layout is written top-down one level per launch
// (children boxes from the parent's stored box with split()'s float ops),
// and the content masks bottom-up.  Node boxes, codes, leaf lists and masks
// are identical to the host build (tests/test_gpu.py).
#include <hipcub/hipcub.hpp>

#include "vrt_internal.h"

namespace vrt {

namespace {

struct alignas(16) Pair {
        float mn[3], mx[3];
        uint32_t tri, code;
};
static_assert(sizeof(Pair) == 32, "Pair must be 32 B");

// split() child box (VRT/voxel_octree.cc:30-35)
__device__ __forceinline__ void child_box_dev(const float *pmn, const float *pmx, int i, float *cmn, float *cmx)
{
        const int m[3] = { (i & 4) ? 1 : 0, (i & 2) ? 1 : 0, (i & 1) ? 1 : 0 };
#pragma unroll
        for (int k = 0; k < 3; ++k) {
                const float half = (pmx[k] - pmn[k]) / 2.0f;
                cmn[k] = pmn[k] + (float)m[k] * half;
                cmx[k] = cmn[k] + half;
        }
}

// Triangle::is_overlap (VRT/voxel_octree.cc:486-492)
__device__ __forceinline__ bool overlaps_dev(const float *tri9, const float *mn, const float *mx)
{
        float c[3], h[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
                c[k] = (mn[k] + mx[k]) * .5f;
                h[k] = (mx[k] - mn[k]) / 2.f;
        }
        return tri_box_overlap(c, h, tri9) == 1;
}

// Exclusive prefix of `cnt` over the wave plus one atomicAdd per wave.
__device__ __forceinline__ uint32_t wave_append(uint32_t cnt, unsigned int *counter)
{
        const int lane = threadIdx.x & 63;
        uint32_t incl = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(incl, o, 64);
                if (lane >= o)
                        incl += v;
        }
        uint32_t base = 0;
        if (lane == 63 && incl)
                base = atomicAdd(counter, incl);
        base = __shfl(base, 63, 64);
        return base + incl - cnt;
}

__global__ __launch_bounds__(256) void k_seed(int n, const float *__restrict__ pos, Pair root,
                                              Pair *__restrict__ out, unsigned int *counter)
{
        const int i = blockIdx.x * blockDim.x + threadIdx.x;
        float tri[9];
        bool hit = false;
        if (i < n) {
#pragma unroll
                for (int k = 0; k < 9; ++k)
                        tri[k] = pos[9 * (int64_t)i + k];
                hit = overlaps_dev(tri, root.mn, root.mx);
        }
        const uint32_t at = wave_append(hit ? 1u : 0u, counter);
        if (hit) {
                Pair p = root;
                p.tri = (uint32_t)i;
                p.code = 0;
                out[at] = p;
        }
}

__global__ __launch_bounds__(256) void k_expand(int64_t n, const Pair *__restrict__ in,
                                                const float *__restrict__ pos, uint32_t *__restrict__ codes,
                                                Pair *__restrict__ out, unsigned int *counter)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        uint32_t mask = 0;
        Pair p;
        float cmn[8][3], cmx[8][3];
        if (i < n) {
                p = in[i];
                codes[i] = p.code;
                float tri[9];
                const float *t = pos + 9 * (int64_t)p.tri;
#pragma unroll
                for (int k = 0; k < 9; ++k)
                        tri[k] = t[k];
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                        child_box_dev(p.mn, p.mx, c, cmn[c], cmx[c]);
                        if (overlaps_dev(tri, cmn[c], cmx[c]))
                                mask |= 1u << c;
                }
        }
        uint32_t at = wave_append((uint32_t)__popc(mask), counter);
        if (mask) {
#pragma unroll
                for (int c = 0; c < 8; ++c)
                        if (mask & (1u << c)) {
                                Pair q;
#pragma unroll
                                for (int k = 0; k < 3; ++k) {
                                        q.mn[k] = cmn[c][k];
                                        q.mx[k] = cmx[c][k];
                                }
                                q.tri = p.tri;
                                q.code = (p.code << 3) | (uint32_t)c;
                                out[at++] = q;
                        }
        }
}

__global__ __launch_bounds__(256) void k_leaf_keys(int64_t n, const Pair *__restrict__ in, uint64_t *__restrict__ keys)
{
        const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (i < n)
                keys[i] = ((uint64_t)in[i].code << 32) | in[i].tri;
}

__device__ __forceinline__ uint32_t vox_of_dev(uint32_t code, int depth)
{
        uint32_t ix = 0, iy = 0, iz = 0;
        for (int l = depth - 2; l >= 0; --l) {
                const uint32_t ci = (code >> (3 * l)) & 7u;
                ix = (ix << 1) | ((ci >> 2) & 1u);
                iy = (iy << 1) | ((ci >> 1) & 1u);
                iz = (iz << 1) | (ci & 1u);
        }
        return ix | (iy << 10) | (iz << 20);
}

template <class T>
__device__ __forceinline__ int64_t lower_bound_dev(const T *a, int64_t n, T key)
{
        int64_t lo = 0, hi = n;
        while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (a[mid] < key)
                        lo = mid + 1;
                else
                        hi = mid;
        }
        return lo;
}

struct FlatLevel {
        int level, max_depth;
        int64_t begin, count;     // node index range of this level
        const uint32_t *iall;     // internal codes, level by level, each sorted
        int64_t jg_base;          // global index of this level's first internal node
        int64_t n_int;            // internal nodes at this level
        uint32_t *inode_of;       // global internal index -> node index
        const uint64_t *refs;     // sorted (code << 32 | tri)
        int64_t nrefs;
        float root_mn[3], root_mx[3];
        NodeRec *nodes;
        uint32_t *node_vox;
};

__global__ __launch_bounds__(256) void k_flatten(FlatLevel f)
{
        const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (t >= f.count)
                return;
        const int64_t ni = f.begin + t;
        uint32_t code;
        float mn[3], mx[3];
        if (f.level == 1) {
                code = 0;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                        mn[k] = f.root_mn[k];
                        mx[k] = f.root_mx[k];
                }
        } else {
                const int64_t jp = (ni - 1) >> 3;
                const int c = (int)((ni - 1) & 7);
                const NodeRec &pn = f.nodes[f.inode_of[jp]];
                child_box_dev(pn.bmin, pn.bmax, c, mn, mx);
                code = (f.iall[jp] << 3) | (uint32_t)c;
        }
        NodeRec nr;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
                nr.bmin[k] = mn[k];
                nr.bmax[k] = mx[k];
        }
        nr.b = 0;
        if (f.level < f.max_depth) {
                const uint32_t *I = f.iall + f.jg_base;
                const int64_t r = lower_bound_dev<uint32_t>(I, f.n_int, code);
                if (r < f.n_int && I[r] == code) {
                        const int64_t jg = f.jg_base + r;
                        nr.a = (uint32_t)(1 + 8 * jg);
                        f.inode_of[jg] = (uint32_t)ni;
                } else {
                        nr.a = kLeafBit;  // empty leaf above max depth
                }
        } else {
                const uint64_t k0 = (uint64_t)code << 32;
                const int64_t lo = lower_bound_dev<uint64_t>(f.refs, f.nrefs, k0);
                const int64_t hi = lower_bound_dev<uint64_t>(f.refs, f.nrefs, k0 + (1ull << 32));
                nr.a = kLeafBit | (uint32_t)(hi - lo);
                nr.b = (uint32_t)lo;
        }
        f.nodes[ni] = nr;
        f.node_vox[ni] = vox_of_dev(code, f.level);
}

// content masks of one level, bottom-up (vrt_host.cpp: build_tree)
__global__ __launch_bounds__(256) void k_masks(int64_t begin, int64_t end, NodeRec *__restrict__ nodes,
                                               uint8_t *__restrict__ has)
{
        const int64_t ni = begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (ni >= end)
                return;
        NodeRec &nr = nodes[ni];
        if (nr.a & kLeafBit) {
                has[ni] = (nr.a & ~kLeafBit) ? 1 : 0;
                return;
        }
        uint32_t m = 0;
        for (int c = 0; c < 8; ++c)
                m |= (uint32_t)has[nr.a + c] << c;
        nr.b = m;
        has[ni] = m ? 1 : 0;
}

struct Dev {
        void *p = nullptr;
        ~Dev()
        {
                if (p)
                        (void)hipFree(p);
        }
        hipError_t alloc(size_t n)
        {
                if (p)
                        (void)hipFree(p);
                p = nullptr;
                return hipMalloc(&p, n ? n : 16);
        }
        template <class T>
        T *as() const
        {
                return static_cast<T *>(p);
        }
};

#define BCHK(expr)                                                                           \
        do {                                                                                 \
                hipError_t e_ = (expr);                                                      \
                if (e_ != hipSuccess) {                                                      \
                        *err = std::string(#expr) + ": " + hipGetErrorString(e_);             \
                        return e_;                                                           \
                }                                                                            \
        } while (0)

unsigned grid_of(int64_t n)
{
        return (unsigned)((n + 255) / 256);
}

}  // namespace

hipError_t build_tree_device(int device, const float *pos, int ntri, const float root_mn[3],
                             const float root_mx[3], int D, DeviceBuild *out, std::string *err)
{
        BCHK(hipSetDevice(device));
        hipStream_t st = nullptr;
        hipEvent_t e0, e1;
        BCHK(hipEventCreate(&e0));
        BCHK(hipEventCreate(&e1));
        struct EvGuard {
                hipEvent_t a, b;
                ~EvGuard()
                {
                        (void)hipEventDestroy(a);
                        (void)hipEventDestroy(b);
                }
        } evg{ e0, e1 };
        Dev dpos, cnt, pa, pb, codes, codes_s, uniq, nuniq, temp, iall, keys, keys_s, inode, dnodes, dvox, dhas;
        BCHK(dpos.alloc((size_t)ntri * 36));
        BCHK(hipMemcpy(dpos.p, pos, (size_t)ntri * 36, hipMemcpyHostToDevice));
        BCHK(hipEventRecord(e0, st));
        BCHK(cnt.alloc(16));
        Pair root;
        for (int k = 0; k < 3; ++k) {
                root.mn[k] = root_mn[k];
                root.mx[k] = root_mx[k];
        }
        root.tri = 0;
        root.code = 0;
        // level 1 frontier
        BCHK(pa.alloc((size_t)std::max(1, ntri) * sizeof(Pair)));
        BCHK(hipMemsetAsync(cnt.p, 0, 16, st));
        if (ntri > 0)
                hipLaunchKernelGGL(k_seed, dim3(grid_of(ntri)), dim3(256), 0, st, ntri, dpos.as<float>(), root,
                                   pa.as<Pair>(), cnt.as<unsigned int>());
        BCHK(hipGetLastError());
        unsigned int hn = 0;
        BCHK(hipMemcpy(&hn, cnt.p, 4, hipMemcpyDeviceToHost));
        int64_t n = hn;
        std::vector<uint32_t> h_iall;          // internal codes, level by level
        std::vector<int64_t> n_int(D + 1, 0);  // per level
        int64_t nrefs = 0;
        for (int l = 1; l <= D; ++l) {
                if (l == D) {
                        // leaf lists: sort (code << 32 | tri)
                        nrefs = n;
                        BCHK(keys.alloc((size_t)std::max<int64_t>(1, n) * 8));
                        BCHK(keys_s.alloc((size_t)std::max<int64_t>(1, n) * 8));
                        if (n > 0) {
                                hipLaunchKernelGGL(k_leaf_keys, dim3(grid_of(n)), dim3(256), 0, st, n, pa.as<Pair>(),
                                                   keys.as<uint64_t>());
                                BCHK(hipGetLastError());
                                size_t tb = 0;
                                const int bits = 32 + 3 * (D - 1);
                                BCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, keys.as<uint64_t>(),
                                                                       keys_s.as<uint64_t>(), (int)n, 0, bits, st));
                                BCHK(temp.alloc(tb));
                                BCHK(hipcub::DeviceRadixSort::SortKeys(temp.p, tb, keys.as<uint64_t>(),
                                                                       keys_s.as<uint64_t>(), (int)n, 0, bits, st));
                        }
                        break;
                }
                // expand: codes of this level + next frontier
                BCHK(codes.alloc((size_t)std::max<int64_t>(1, n) * 4));
                BCHK(pb.alloc((size_t)std::max<int64_t>(1, 8 * n) * sizeof(Pair)));
                BCHK(hipMemsetAsync(cnt.p, 0, 16, st));
                if (n > 0)
                        hipLaunchKernelGGL(k_expand, dim3(grid_of(n)), dim3(256), 0, st, n, pa.as<Pair>(),
                                           dpos.as<float>(), codes.as<uint32_t>(), pb.as<Pair>(),
                                           cnt.as<unsigned int>());
                BCHK(hipGetLastError());
                // internal nodes of level l = sorted unique codes
                int64_t nu = 0;
                if (n > 0) {
                        const int bits = std::max(1, 3 * (l - 1));
                        BCHK(codes_s.alloc((size_t)n * 4));
                        BCHK(uniq.alloc((size_t)n * 4));
                        BCHK(nuniq.alloc(8));
                        size_t tb = 0, tb2 = 0;
                        BCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, tb, codes.as<uint32_t>(), codes_s.as<uint32_t>(),
                                                               (int)n, 0, bits, st));
                        BCHK(hipcub::DeviceSelect::Unique(nullptr, tb2, codes_s.as<uint32_t>(), uniq.as<uint32_t>(),
                                                          nuniq.as<int>(), (int)n, st));
                        BCHK(temp.alloc(std::max(tb, tb2)));
                        BCHK(hipcub::DeviceRadixSort::SortKeys(temp.p, tb, codes.as<uint32_t>(), codes_s.as<uint32_t>(),
                                                               (int)n, 0, bits, st));
                        BCHK(hipcub::DeviceSelect::Unique(temp.p, tb2, codes_s.as<uint32_t>(), uniq.as<uint32_t>(),
                                                          nuniq.as<int>(), (int)n, st));
                        int hnu = 0;
                        BCHK(hipMemcpy(&hnu, nuniq.p, 4, hipMemcpyDeviceToHost));
                        nu = hnu;
                        const size_t o = h_iall.size();
                        h_iall.resize(o + (size_t)nu);
                        if (nu)
                                BCHK(hipMemcpy(h_iall.data() + o, uniq.p, (size_t)nu * 4, hipMemcpyDeviceToHost));
                }
                n_int[l] = nu;
                BCHK(hipMemcpy(&hn, cnt.p, 4, hipMemcpyDeviceToHost));
                n = hn;
                std::swap(pa.p, pb.p);
                if (nu == 0)
                        break;  // nothing below this level
        }
        // ---- flatten: level ranges as the host build (root, then 8 children
        // per internal node of the previous level, in code order)
        int64_t ninternal = (int64_t)h_iall.size();
        const int64_t nnodes = 1 + 8 * ninternal;
        out->level_begin.clear();
        BCHK(iall.alloc(std::max<size_t>(1, h_iall.size()) * 4));
        if (!h_iall.empty())
                BCHK(hipMemcpy(iall.p, h_iall.data(), h_iall.size() * 4, hipMemcpyHostToDevice));
        BCHK(inode.alloc(std::max<int64_t>(1, ninternal) * 4));
        BCHK(dnodes.alloc((size_t)nnodes * sizeof(NodeRec)));
        BCHK(dvox.alloc((size_t)nnodes * 4));
        int64_t begin = 0, count = 1, jg_base = 0;
        for (int l = 1; l <= D && count > 0; ++l) {
                out->level_begin.push_back(begin);
                FlatLevel f;
                f.level = l;
                f.max_depth = D;
                f.begin = begin;
                f.count = count;
                f.iall = iall.as<uint32_t>();
                f.jg_base = jg_base;
                f.n_int = l < D ? n_int[l] : 0;
                f.inode_of = inode.as<uint32_t>();
                f.refs = keys_s.as<uint64_t>();
                f.nrefs = nrefs;
                for (int k = 0; k < 3; ++k) {
                        f.root_mn[k] = root_mn[k];
                        f.root_mx[k] = root_mx[k];
                }
                f.nodes = dnodes.as<NodeRec>();
                f.node_vox = dvox.as<uint32_t>();
                hipLaunchKernelGGL(k_flatten, dim3(grid_of(count)), dim3(256), 0, st, f);
                BCHK(hipGetLastError());
                begin += count;
                count = 8 * f.n_int;
                jg_base += f.n_int;
        }
        out->level_begin.push_back(nnodes);
        // content masks bottom-up
        BCHK(dhas.alloc((size_t)nnodes));
        for (int l = (int)out->level_begin.size() - 1; l >= 1; --l) {
                const int64_t b0 = out->level_begin[l - 1], b1 = out->level_begin[l];
                hipLaunchKernelGGL(k_masks, dim3(grid_of(b1 - b0)), dim3(256), 0, st, b0, b1, dnodes.as<NodeRec>(),
                                   dhas.as<uint8_t>());
                BCHK(hipGetLastError());
        }
        BCHK(hipEventRecord(e1, st));
        BCHK(hipEventSynchronize(e1));
        float ms = 0.f;
        BCHK(hipEventElapsedTime(&ms, e0, e1));
        out->device_ms = ms;
        out->ninternal = ninternal;
        out->nodes.resize((size_t)nnodes);
        out->node_vox.resize((size_t)nnodes);
        out->refs.resize((size_t)nrefs);
        BCHK(hipMemcpy(out->nodes.data(), dnodes.p, (size_t)nnodes * sizeof(NodeRec), hipMemcpyDeviceToHost));
        BCHK(hipMemcpy(out->node_vox.data(), dvox.p, (size_t)nnodes * 4, hipMemcpyDeviceToHost));
        if (nrefs)
                BCHK(hipMemcpy(out->refs.data(), keys_s.p, (size_t)nrefs * 8, hipMemcpyDeviceToHost));
        return hipSuccess;
}

// Stable device radix sort of (uint32 key, uint32 value) pairs on the low
// `bits` key bits, for the light-map accumulation (vrt_kernels.hip: leaf
// key, canonical sample index); the same hipCUB / rocPRIM onesweep sort the
// build's frontier uses, so hipCUB's templates compile in this one file.
hipError_t sort_pairs_u64(void *temp, size_t *temp_bytes, const uint64_t *keys_in, uint64_t *keys_out,
                          const uint32_t *vals_in, uint32_t *vals_out, int64_t n, int bits, hipStream_t st)
{
        return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out,
                                                  (int)n, 0, bits, st);
}

}  // namespace vrt
