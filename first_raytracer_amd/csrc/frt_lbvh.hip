// frt_lbvh.hip -- GPU BVH builders over the world
// primitives' boxes, on the device, as fast alternatives to the host SAH builds
// (parallel_bvh_node::create_bvh, parallel_bvh.h:67-175; host: csrc/host/scene.cpp):
// a linear BVH (steps 1-5 below) and PLOC clustering on the same Morton order
// (steps 1-3, then k_ploc_*; SAH-like quality, the default).
//
//   1. centroid bounds       one block reduction + atomics on order-preserving uints
//   2. Morton keys           30-bit (10 bits / axis) centroid code << 32 | prim index
//                            (unique 64-bit keys: equal codes keep prim order)
//   3. radix sort            hipcub::DeviceRadixSort (rocPRIM onepass sort)
//   4. hierarchy             Karras 2012: internal node i covers a key range found
//                            by prefix-length search; children are the two sides
//                            of the range's highest differing bit
//   5. refit                 leaves climb to the root; the second child to arrive
//                            at a node writes its box (atomic arrival counters)
//
// Output: n-1 internal nodes (node 0 = root), children as internal index >= 0
// or ~(sorted leaf position), the internal nodes' boxes, and the sorted
// primitive order.  The host turns that into the frt_scene_view BVH
// (frt_scene_build_bvh_gpu) and the usual upload path (DFS order, leaf
// collapse, BVH4Q) takes it from there.  The tree differs from the
// reference's SAH tree, so hits differ from the reference's only where two
// primitives are hit at exactly the same t (the DFS rank tie rule then follows
// this tree's order).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "frt_lbvh.hpp"

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ uint32_t f2ord(float f)   // monotone float -> uint map
{
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t u)
{
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// boxes: 2 float4 per prim (lo.xyz, hi.xyz)
__global__ __launch_bounds__(kBlock) void k_centroid_bounds(const float4 *__restrict__ box, int n, uint32_t *bounds)
{
    __shared__ float red[6][kBlock];
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const float4 a = box[2 * i], b = box[2 * i + 1];
        const float c[3] = {0.5f * (a.x + b.x), 0.5f * (a.y + b.y), 0.5f * (a.z + b.z)};
        for (int k = 0; k < 3; ++k) { lo[k] = fminf(lo[k], c[k]); hi[k] = fmaxf(hi[k], c[k]); }
    }
    for (int k = 0; k < 3; ++k) { red[k][threadIdx.x] = lo[k]; red[3 + k][threadIdx.x] = hi[k]; }
    __syncthreads();
    for (int s = kBlock / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int k = 0; k < 3; ++k) {
                red[k][threadIdx.x] = fminf(red[k][threadIdx.x], red[k][threadIdx.x + s]);
                red[3 + k][threadIdx.x] = fmaxf(red[3 + k][threadIdx.x], red[3 + k][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int k = 0; k < 3; ++k) {
            atomicMin(&bounds[k], f2ord(red[k][0]));
            atomicMax(&bounds[3 + k], f2ord(red[3 + k][0]));
        }
}

__device__ __forceinline__ uint32_t spread10(uint32_t v)   // 10 bits -> every third bit
{
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ __launch_bounds__(kBlock) void k_morton(const float4 *__restrict__ box, int n, const uint32_t *bounds,
                                                    unsigned long long *keys)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 a = box[2 * i], b = box[2 * i + 1];
    const float c[3] = {0.5f * (a.x + b.x), 0.5f * (a.y + b.y), 0.5f * (a.z + b.z)};
    uint32_t code = 0;
    for (int k = 0; k < 3; ++k) {
        const float lo = ord2f(bounds[k]), hi = ord2f(bounds[3 + k]);
        const float ext = hi - lo;
        float u = ext > 0.0f ? (c[k] - lo) / ext : 0.5f;
        u = fminf(fmaxf(u * 1024.0f, 0.0f), 1023.0f);
        code |= spread10((uint32_t)u) << (2 - k);
    }
    keys[i] = ((unsigned long long)code << 32) | (uint32_t)i;
}

__device__ __forceinline__ int delta(const unsigned long long *k, int n, int i, int j)
{
    if (j < 0 || j >= n) return -1;
    return __clzll(k[i] ^ k[j]);   // keys are unique: 0..63
}

// Karras 2012, "Maximizing parallelism in the construction of BVHs, octrees
// and k-d trees", Fig. 4: internal node i
__global__ __launch_bounds__(kBlock) void k_hierarchy(const unsigned long long *__restrict__ k, int n,
                                                       int *__restrict__ child, int *__restrict__ parent_int,
                                                       int *__restrict__ parent_leaf)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(k, n, i, i - d);
    int lmax = 2;
    while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(k, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int g = i + s * d + min(d, 0);
    const int lo = min(i, j), hi = max(i, j);
    const int left = (lo == g) ? ~g : g, right = (hi == g + 1) ? ~(g + 1) : g + 1;
    child[2 * i] = left;
    child[2 * i + 1] = right;
    if (left < 0) parent_leaf[~left] = i; else parent_int[left] = i;
    if (right < 0) parent_leaf[~right] = i; else parent_int[right] = i;
}

// bottom-up boxes: every leaf climbs; the second arrival at a node has both
// children's boxes and continues, the first stops
__global__ __launch_bounds__(kBlock) void k_refit(const float4 *__restrict__ box, const unsigned long long *__restrict__ k,
                                                   int n, const int *__restrict__ child, const int *__restrict__ parent_int,
                                                   const int *__restrict__ parent_leaf, unsigned *arrive, float4 *node_box)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    int node = parent_leaf[i];
    while (node >= 0) {
        // acq_rel at agent scope: this thread's box stores are released before
        // the count, and the sibling's are visible (L1 invalidated) after it
        if (__hip_atomic_fetch_add(&arrive[node], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 0u)
            return;                                      // the sibling is not done yet
        float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
        for (int side = 0; side < 2; ++side) {
            const int c = child[2 * node + side];
            float4 a, b;
            if (c < 0) {
                const int prim = (int)(uint32_t)k[~c];
                a = box[2 * prim]; b = box[2 * prim + 1];
            } else {
                a = node_box[2 * c];
                b = node_box[2 * c + 1];
            }
            lo = make_float4(fminf(lo.x, a.x), fminf(lo.y, a.y), fminf(lo.z, a.z), 0.0f);
            hi = make_float4(fmaxf(hi.x, b.x), fmaxf(hi.y, b.y), fmaxf(hi.z, b.z), 0.0f);
        }
        node_box[2 * node] = lo;
        node_box[2 * node + 1] = hi;
        node = parent_int[node];
    }
}

// ---- PLOC (Meister & Bittner 2018, "Parallel Locally-Ordered Clustering for
// Bounding Volume Hierarchy Construction") over the Morton-sorted leaves ----
// A cluster = (box, id): id ~p for the leaf at sorted position p, >= 0 for an
// internal node.  Per iteration: every cluster finds, among the kPlocRadius
// clusters on either side in Morton order, the one whose union box has the
// smallest surface area (ties: the lower index); mutual nearest neighbours
// merge into a new internal node (the lower index creates it and keeps the
// slot), and the survivors are compacted in order.  Internal nodes are
// numbered downwards from n-2, so the root (the last merge) is node 0.
#ifndef FRT_EXP_PLOC_R
#define FRT_EXP_PLOC_R 16
#endif
constexpr int kPlocRadius = FRT_EXP_PLOC_R;

__device__ __forceinline__ float union_area(float4 alo, float4 ahi, float4 blo, float4 bhi)
{
    const float dx = fmaxf(ahi.x, bhi.x) - fminf(alo.x, blo.x);
    const float dy = fmaxf(ahi.y, bhi.y) - fminf(alo.y, blo.y);
    const float dz = fmaxf(ahi.z, bhi.z) - fminf(alo.z, blo.z);
    return dx * dy + dy * dz + dz * dx;
}

__global__ __launch_bounds__(kBlock) void k_ploc_init(const float4 *__restrict__ box, const unsigned long long *__restrict__ k,
                                                       int n, float4 *cbox, int *cid)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const int prim = (int)(uint32_t)k[i];
    cbox[2 * i] = box[2 * prim];
    cbox[2 * i + 1] = box[2 * prim + 1];
    cid[i] = ~i;
}

// nearest neighbour within the window; the block's clusters +- radius staged in LDS
__global__ __launch_bounds__(kBlock) void k_ploc_nn(const float4 *__restrict__ cbox, int c, int *__restrict__ nn)
{
    __shared__ float4 slo[kBlock + 2 * kPlocRadius], shi[kBlock + 2 * kPlocRadius];
    const int base = blockIdx.x * kBlock - kPlocRadius;
    for (int t = threadIdx.x; t < kBlock + 2 * kPlocRadius; t += kBlock) {
        const int j = base + t;
        if (j >= 0 && j < c) { slo[t] = cbox[2 * j]; shi[t] = cbox[2 * j + 1]; }
    }
    __syncthreads();
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= c) return;
    const int li = i - base;
    const float4 alo = slo[li], ahi = shi[li];
    float best = INFINITY;
    int bj = -1;
    const int j0 = max(0, i - kPlocRadius), j1 = min(c - 1, i + kPlocRadius);
    for (int j = j0; j <= j1; ++j) {
        if (j == i) continue;
        const float a = union_area(alo, ahi, slo[j - base], shi[j - base]);
        if (a < best) { best = a; bj = j; }           // ascending j: ties keep the lower index
    }
    nn[i] = bj;
}

// survivor / creator flags: mutual pairs merge at the lower index
__global__ __launch_bounds__(kBlock) void k_ploc_flags(const int *__restrict__ nn, int c, int *keep, int *create)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= c) return;
    const int j = nn[i];
    const bool mutual = j >= 0 && nn[j] == i;
    keep[i] = (mutual && i > j) ? 0 : 1;
    create[i] = (mutual && i < j) ? 1 : 0;
}

__global__ __launch_bounds__(kBlock) void k_ploc_merge(const float4 *__restrict__ cbox, const int *__restrict__ cid,
                                                        const int *__restrict__ nn, const int *__restrict__ keep_pos,
                                                        const int *__restrict__ create_pos, const int *__restrict__ keep,
                                                        const int *__restrict__ create, int c, int next_node,
                                                        float4 *__restrict__ obox, int *__restrict__ oid,
                                                        int *__restrict__ child, float4 *__restrict__ node_box)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= c || !keep[i]) return;
    const int o = keep_pos[i];
    if (!create[i]) {
        obox[2 * o] = cbox[2 * i];
        obox[2 * o + 1] = cbox[2 * i + 1];
        oid[o] = cid[i];
        return;
    }
    const int j = nn[i];
    const float4 alo = cbox[2 * i], ahi = cbox[2 * i + 1], blo = cbox[2 * j], bhi = cbox[2 * j + 1];
    const float4 lo = make_float4(fminf(alo.x, blo.x), fminf(alo.y, blo.y), fminf(alo.z, blo.z), 0.0f);
    const float4 hi = make_float4(fmaxf(ahi.x, bhi.x), fmaxf(ahi.y, bhi.y), fmaxf(ahi.z, bhi.z), 0.0f);
    const int node = next_node - create_pos[i];       // numbered downwards: the root is node 0
    child[2 * node] = cid[i];                          // Morton order: the lower index on the left
    child[2 * node + 1] = cid[j];
    node_box[2 * node] = lo;
    node_box[2 * node + 1] = hi;
    obox[2 * o] = lo;
    obox[2 * o + 1] = hi;
    oid[o] = node;
}

// ---- binned SAH, top down, one level of the tree per launch ----
// A task is a node over idx[b, e) (sizes >= 2).  One block per task: box and
// centroid bounds, 32 centroid bins per axis in LDS (ordered-uint min / max
// atomics), the cheapest split N_L A_L + N_R A_R (the host builder's rule,
// csrc/host/scene.cpp SahBuilder), then a stable block-wide partition of the
// range into idx_out.  Children of two or more prims become next-level tasks;
// single prims become leaves (~prim).  Node ids are handed out by an atomic
// counter (their numbering varies, the tree does not).
constexpr int kSahBins = 32;
struct SahTask { int b, e, node; };

__device__ __forceinline__ float4 fmin4(float4 a, float4 b)
{
    return make_float4(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), 0.0f);
}
__device__ __forceinline__ float4 fmax4(float4 a, float4 b)
{
    return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), 0.0f);
}
__device__ __forceinline__ float area3(float4 lo, float4 hi)
{
    const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}
__device__ __forceinline__ float comp(float4 v, int k) { return k == 0 ? v.x : k == 1 ? v.y : v.z; }

__global__ __launch_bounds__(kBlock) void k_sah_level(const float4 *__restrict__ box, const int *__restrict__ idx_in,
                                                       int *__restrict__ idx_out, const SahTask *__restrict__ tasks,
                                                       SahTask *__restrict__ next, int *__restrict__ next_count,
                                                       int *__restrict__ node_counter, int *__restrict__ child,
                                                       float4 *__restrict__ node_box)
{
    __shared__ uint32_t red[6][kBlock];
    __shared__ uint32_t bcnt[3][kSahBins], blo[3][kSahBins][3], bhi[3][kSahBins][3];
    __shared__ uint32_t cmn[3], cmx[3];
    __shared__ float best_cost[3];
    __shared__ int best_bin[3];
    __shared__ int s_axis, s_bin, s_left;
    __shared__ int scan[kBlock];
    const SahTask T = tasks[blockIdx.x];
    const int b = T.b, e = T.e, n = e - b, tid = threadIdx.x;
    // ---- bounds: prims' box union and centroid range ----
    float4 lo = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), hi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
    float4 clo = lo, chi = hi;
    for (int i = b + tid; i < e; i += kBlock) {
        const int p = idx_in[i];
        const float4 a = box[2 * p], z = box[2 * p + 1];
        const float4 c = make_float4(0.5f * (a.x + z.x), 0.5f * (a.y + z.y), 0.5f * (a.z + z.z), 0.0f);
        lo = fmin4(lo, a); hi = fmax4(hi, z); clo = fmin4(clo, c); chi = fmax4(chi, c);
    }
    if (tid < 3) { cmn[tid] = 0xffffffffu; cmx[tid] = 0u; }
    for (int k = 0; k < 3; ++k) { red[k][tid] = f2ord(comp(lo, k)); red[3 + k][tid] = f2ord(comp(hi, k)); }
    __syncthreads();
    for (int k = 0; k < 3; ++k) { atomicMin(&cmn[k], f2ord(comp(clo, k))); atomicMax(&cmx[k], f2ord(comp(chi, k))); }
    for (int st = kBlock / 2; st > 0; st >>= 1) {
        if (tid < st)
            for (int k = 0; k < 3; ++k) {
                red[k][tid] = min(red[k][tid], red[k][tid + st]);
                red[3 + k][tid] = max(red[3 + k][tid], red[3 + k][tid + st]);
            }
        __syncthreads();
    }
    if (tid == 0) {
        node_box[2 * T.node] = make_float4(ord2f(red[0][0]), ord2f(red[1][0]), ord2f(red[2][0]), 0.0f);
        node_box[2 * T.node + 1] = make_float4(ord2f(red[3][0]), ord2f(red[4][0]), ord2f(red[5][0]), 0.0f);
    }
    float cl[3], sc[3];
    for (int k = 0; k < 3; ++k) {
        cl[k] = ord2f(cmn[k]);
        const float ext = ord2f(cmx[k]) - cl[k];
        sc[k] = ext > 0.0f ? (float)kSahBins / ext : 0.0f;
    }
    // ---- bins ----
    if (n > 2) {
        for (int t = tid; t < 3 * kSahBins; t += kBlock) {
            const int k = t / kSahBins, j = t % kSahBins;
            bcnt[k][j] = 0u;
            for (int a = 0; a < 3; ++a) { blo[k][j][a] = 0xffffffffu; bhi[k][j][a] = 0u; }
        }
        __syncthreads();
        for (int i = b + tid; i < e; i += kBlock) {
            const int p = idx_in[i];
            const float4 a = box[2 * p], z = box[2 * p + 1];
            const float c[3] = {0.5f * (a.x + z.x), 0.5f * (a.y + z.y), 0.5f * (a.z + z.z)};
            for (int k = 0; k < 3; ++k) {
                if (sc[k] == 0.0f) continue;
                const int j = min(kSahBins - 1, (int)((c[k] - cl[k]) * sc[k]));
                atomicAdd(&bcnt[k][j], 1u);
                for (int q = 0; q < 3; ++q) {
                    atomicMin(&blo[k][j][q], f2ord(comp(a, q)));
                    atomicMax(&bhi[k][j][q], f2ord(comp(z, q)));
                }
            }
        }
        __syncthreads();
        // ---- the cheapest split per axis (thread k), then over the axes ----
        if (tid < 3) {
            const int k = tid;
            float bc = INFINITY;
            int bj = -1;
            if (sc[k] != 0.0f) {
                float rarea[kSahBins];
                int rcnt[kSahBins];
                float4 rl = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), rh = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
                int c = 0;
                for (int j = kSahBins - 1; j > 0; --j) {
                    if (bcnt[k][j]) {
                        rl = fmin4(rl, make_float4(ord2f(blo[k][j][0]), ord2f(blo[k][j][1]), ord2f(blo[k][j][2]), 0.0f));
                        rh = fmax4(rh, make_float4(ord2f(bhi[k][j][0]), ord2f(bhi[k][j][1]), ord2f(bhi[k][j][2]), 0.0f));
                        c += (int)bcnt[k][j];
                    }
                    rarea[j] = c ? area3(rl, rh) : 0.0f;
                    rcnt[j] = c;
                }
                float4 ll = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), lh = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
                c = 0;
                for (int j = 0; j < kSahBins - 1; ++j) {
                    if (bcnt[k][j]) {
                        ll = fmin4(ll, make_float4(ord2f(blo[k][j][0]), ord2f(blo[k][j][1]), ord2f(blo[k][j][2]), 0.0f));
                        lh = fmax4(lh, make_float4(ord2f(bhi[k][j][0]), ord2f(bhi[k][j][1]), ord2f(bhi[k][j][2]), 0.0f));
                        c += (int)bcnt[k][j];
                    }
                    if (c == 0 || rcnt[j + 1] == 0) continue;
                    const float cost = (float)c * area3(ll, lh) + (float)rcnt[j + 1] * rarea[j + 1];
                    if (cost < bc) { bc = cost; bj = j; }
                }
            }
            best_cost[k] = bc;
            best_bin[k] = bj;
        }
        __syncthreads();
        if (tid == 0) {
            int ax = -1;
            for (int k = 0; k < 3; ++k)
                if (best_bin[k] >= 0 && (ax < 0 || best_cost[k] < best_cost[ax])) ax = k;
            s_axis = ax;
            s_bin = ax >= 0 ? best_bin[ax] : 0;
        }
        __syncthreads();
    } else if (tid == 0) {
        s_axis = -1;
    }
    if (tid == 0) s_left = 0;
    __syncthreads();
    const int ax = s_axis, bin = s_bin;
    // ---- stable partition of [b, e) into idx_out (left: bin <= best bin) ----
    int mid;
    if (ax >= 0) {
        int nl = 0;
        for (int i = b + tid; i < e; i += kBlock) {
            const int p = idx_in[i];
            const float c = 0.5f * (comp(box[2 * p], ax) + comp(box[2 * p + 1], ax));
            nl += min(kSahBins - 1, (int)((c - cl[ax]) * sc[ax])) <= bin ? 1 : 0;
        }
        atomicAdd(&s_left, nl);
        __syncthreads();
        mid = b + s_left;
    } else {
        mid = b + n / 2;
    }
    if (ax >= 0 && mid > b && mid < e) {
        int base_l = b, base_r = mid;
        for (int c0 = b; c0 < e; c0 += kBlock) {
            const int i = c0 + tid;
            int p = 0, f = 0;
            if (i < e) {
                p = idx_in[i];
                const float c = 0.5f * (comp(box[2 * p], ax) + comp(box[2 * p + 1], ax));
                f = min(kSahBins - 1, (int)((c - cl[ax]) * sc[ax])) <= bin ? 1 : 0;
            }
            scan[tid] = f;
            __syncthreads();
            for (int off = 1; off < kBlock; off <<= 1) {          // inclusive scan (Hillis-Steele)
                const int v = tid >= off ? scan[tid - off] : 0;
                __syncthreads();
                scan[tid] += v;
                __syncthreads();
            }
            const int incl = scan[tid], tot = scan[kBlock - 1];
            if (i < e) {
                if (f) idx_out[base_l + incl - 1] = p;
                else idx_out[base_r + (tid - incl)] = p;
            }
            base_l += tot;
            base_r += min(kBlock, e - c0) - tot;
            __syncthreads();
        }
    } else {                                                 // one bin or n <= 2: median split in order
        mid = b + n / 2;
        for (int i = b + tid; i < e; i += kBlock) idx_out[i] = idx_in[i];
    }
    __syncthreads();
    // ---- children ----
    if (tid < 2) {
        const int cb = tid == 0 ? b : mid, ce = tid == 0 ? mid : e;
        int ref;
        if (ce - cb == 1) {
            ref = ~idx_out[cb];
        } else {
            ref = atomicAdd(node_counter, 1);
            const int slot = atomicAdd(next_count, 1);
            next[slot] = SahTask{cb, ce, ref};
        }
        child[2 * T.node + tid] = ref;
    }
}

}  // namespace

namespace frt {

#define LCHK(x)                                                                                     \
    do {                                                                                            \
        const hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); goto done; }   \
    } while (0)

int lbvh_build(hipStream_t st, int n, const float *box6, int32_t *child2, float *node_box6, int32_t *order,
               float *ms, std::string &err, int algo)
{
    int rc = -1;
    float4 *d_box = nullptr, *d_nbox = nullptr;
    unsigned long long *d_keys = nullptr, *d_sorted = nullptr;
    int *d_child = nullptr, *d_pint = nullptr, *d_pleaf = nullptr;
    uint32_t *d_bounds = nullptr;
    unsigned *d_arrive = nullptr;
    void *d_tmp = nullptr;
    size_t tmp_bytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::vector<float4> hbox;
    std::vector<unsigned long long> hkeys;
    const int grid_n = (n + kBlock - 1) / kBlock;
    const uint32_t init[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    if (n < 2) { err = "lbvh_build: needs at least 2 primitives"; return -1; }
    hbox.resize(2 * (size_t)n);
    for (int i = 0; i < n; ++i) {
        hbox[2 * i] = make_float4(box6[6 * i], box6[6 * i + 1], box6[6 * i + 2], 0.0f);
        hbox[2 * i + 1] = make_float4(box6[6 * i + 3], box6[6 * i + 4], box6[6 * i + 5], 0.0f);
    }
    LCHK(hipMalloc(&d_box, sizeof(float4) * 2 * (size_t)n));
    LCHK(hipMalloc(&d_nbox, sizeof(float4) * 2 * (size_t)(n - 1)));
    LCHK(hipMalloc(&d_keys, sizeof(unsigned long long) * (size_t)n));
    LCHK(hipMalloc(&d_sorted, sizeof(unsigned long long) * (size_t)n));
    LCHK(hipMalloc(&d_child, sizeof(int) * 2 * (size_t)(n - 1)));
    LCHK(hipMalloc(&d_pint, sizeof(int) * (size_t)(n - 1)));
    LCHK(hipMalloc(&d_pleaf, sizeof(int) * (size_t)n));
    LCHK(hipMalloc(&d_bounds, sizeof(uint32_t) * 6));
    LCHK(hipMalloc(&d_arrive, sizeof(unsigned) * (size_t)(n - 1)));
    LCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp_bytes, d_keys, d_sorted, n, 0, 64, st));
    LCHK(hipMalloc(&d_tmp, tmp_bytes));
    LCHK(hipMemcpyAsync(d_box, hbox.data(), sizeof(float4) * 2 * (size_t)n, hipMemcpyHostToDevice, st));
    LCHK(hipMemcpyAsync(d_bounds, init, sizeof(init), hipMemcpyHostToDevice, st));
    LCHK(hipMemsetAsync(d_arrive, 0, sizeof(unsigned) * (size_t)(n - 1), st));
    LCHK(hipMemsetAsync(d_pint, 0xff, sizeof(int) * (size_t)(n - 1), st));   // root's parent = -1
    LCHK(hipEventCreate(&e0));
    LCHK(hipEventCreate(&e1));
    LCHK(hipEventRecord(e0, st));
    if (algo == kGpuBvhSah) {
        // top-down binned SAH; leaves are ~prim, order = identity
        int *ia = nullptr, *ib = nullptr, *d_cnt = nullptr;
        SahTask *ta = nullptr, *tb = nullptr;
        int k = 1, level = 0;
        const SahTask root{0, n, 0};
        std::vector<int> iota(n);
        for (int i = 0; i < n; ++i) iota[i] = i;
#define SCHK(x)                                                                                     \
    do {                                                                                            \
        const hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); goto sah_done; } \
    } while (0)
        SCHK(hipMalloc(&ia, sizeof(int) * (size_t)n));
        SCHK(hipMalloc(&ib, sizeof(int) * (size_t)n));
        SCHK(hipMalloc(&ta, sizeof(SahTask) * (size_t)n));
        SCHK(hipMalloc(&tb, sizeof(SahTask) * (size_t)n));
        SCHK(hipMalloc(&d_cnt, sizeof(int) * 2));
        SCHK(hipMemcpyAsync(ia, iota.data(), sizeof(int) * (size_t)n, hipMemcpyHostToDevice, st));
        SCHK(hipMemcpyAsync(ta, &root, sizeof(SahTask), hipMemcpyHostToDevice, st));
        {
            const int one = 1;                                    // node 0 = root, already allocated
            SCHK(hipMemcpyAsync(d_cnt + 1, &one, sizeof(int), hipMemcpyHostToDevice, st));
        }
        while (k > 0) {
            int nk = 0;
            SCHK(hipMemsetAsync(d_cnt, 0, sizeof(int), st));
            k_sah_level<<<k, kBlock, 0, st>>>(d_box, ia, ib, ta, tb, d_cnt, d_cnt + 1, d_child, d_nbox);
            SCHK(hipGetLastError());
            SCHK(hipMemcpyAsync(&nk, d_cnt, sizeof(int), hipMemcpyDeviceToHost, st));
            SCHK(hipStreamSynchronize(st));
            // ranges not split further keep their (final) order in ib; carry them over
            std::swap(ia, ib);
            std::swap(ta, tb);
            k = nk;
            if (++level > 4096) { err = "sah: no progress"; goto sah_done; }
        }
        for (int i = 0; i < n; ++i) order[i] = i;
    sah_done:
        (void)hipFree(ia); (void)hipFree(ib); (void)hipFree(ta); (void)hipFree(tb); (void)hipFree(d_cnt);
#undef SCHK
        if (!err.empty()) goto done;
        goto finished;
    }
    k_centroid_bounds<<<std::min(grid_n, 1024), kBlock, 0, st>>>(d_box, n, d_bounds);
    k_morton<<<grid_n, kBlock, 0, st>>>(d_box, n, d_bounds, d_keys);
    LCHK(hipGetLastError());
    LCHK(hipcub::DeviceRadixSort::SortKeys(d_tmp, tmp_bytes, d_keys, d_sorted, n, 0, 64, st));
    if (algo == kGpuBvhLbvh) {
        k_hierarchy<<<(n - 1 + kBlock - 1) / kBlock, kBlock, 0, st>>>(d_sorted, n, d_child, d_pint, d_pleaf);
        k_refit<<<grid_n, kBlock, 0, st>>>(d_box, d_sorted, n, d_child, d_pint, d_pleaf, d_arrive, d_nbox);
        LCHK(hipGetLastError());
    } else {
        // PLOC: ping-pong cluster arrays; flags and their exclusive scans per iteration
#define PCHK(x)                                                                                     \
    do {                                                                                            \
        const hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); goto ploc_done; } \
    } while (0)
        float4 *cb[2] = {nullptr, nullptr};
        int *ci[2] = {nullptr, nullptr};
        int *nn = nullptr, *keep = nullptr, *create = nullptr, *kpos = nullptr, *cpos = nullptr;
        void *stmp = nullptr;
        size_t stmp_bytes = 0;
        int tail[4];
        int c = n, cur = 0, made = 0;
        PCHK(hipMalloc(&cb[0], sizeof(float4) * 2 * (size_t)n));
        PCHK(hipMalloc(&cb[1], sizeof(float4) * 2 * (size_t)n));
        PCHK(hipMalloc(&ci[0], sizeof(int) * (size_t)n));
        PCHK(hipMalloc(&ci[1], sizeof(int) * (size_t)n));
        PCHK(hipMalloc(&nn, sizeof(int) * (size_t)n));
        PCHK(hipMalloc(&keep, sizeof(int) * (size_t)n));
        PCHK(hipMalloc(&create, sizeof(int) * (size_t)n));
        PCHK(hipMalloc(&kpos, sizeof(int) * (size_t)n));
        PCHK(hipMalloc(&cpos, sizeof(int) * (size_t)n));
        PCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, stmp_bytes, keep, kpos, n, st));
        PCHK(hipMalloc(&stmp, stmp_bytes));
        k_ploc_init<<<grid_n, kBlock, 0, st>>>(d_box, d_sorted, n, cb[0], ci[0]);
        PCHK(hipGetLastError());
        while (c > 1) {
            const int g = (c + kBlock - 1) / kBlock;
            k_ploc_nn<<<g, kBlock, 0, st>>>(cb[cur], c, nn);
            k_ploc_flags<<<g, kBlock, 0, st>>>(nn, c, keep, create);
            PCHK(hipGetLastError());
            PCHK(hipcub::DeviceScan::ExclusiveSum(stmp, stmp_bytes, keep, kpos, c, st));
            PCHK(hipcub::DeviceScan::ExclusiveSum(stmp, stmp_bytes, create, cpos, c, st));
            // survivors and merges of this pass (last element + its flag)
            PCHK(hipMemcpyAsync(&tail[0], kpos + c - 1, sizeof(int), hipMemcpyDeviceToHost, st));
            PCHK(hipMemcpyAsync(&tail[1], keep + c - 1, sizeof(int), hipMemcpyDeviceToHost, st));
            PCHK(hipMemcpyAsync(&tail[2], cpos + c - 1, sizeof(int), hipMemcpyDeviceToHost, st));
            PCHK(hipMemcpyAsync(&tail[3], create + c - 1, sizeof(int), hipMemcpyDeviceToHost, st));
            k_ploc_merge<<<g, kBlock, 0, st>>>(cb[cur], ci[cur], nn, kpos, cpos, keep, create, c, n - 2 - made,
                                               cb[cur ^ 1], ci[cur ^ 1], d_child, d_nbox);
            PCHK(hipGetLastError());
            PCHK(hipStreamSynchronize(st));
            const int c_new = tail[0] + tail[1], merged = tail[2] + tail[3];
            if (merged <= 0 || c_new != c - merged) { err = "ploc: no merge progress"; goto ploc_done; }
            made += merged;
            c = c_new;
            cur ^= 1;
        }
        if (made != n - 1) err = "ploc: wrong node count";
    ploc_done:
        (void)hipFree(cb[0]); (void)hipFree(cb[1]); (void)hipFree(ci[0]); (void)hipFree(ci[1]);
        (void)hipFree(nn); (void)hipFree(keep); (void)hipFree(create); (void)hipFree(kpos); (void)hipFree(cpos);
        (void)hipFree(stmp);
        if (!err.empty()) goto done;
#undef PCHK
    }
finished:
    LCHK(hipEventRecord(e1, st));
    {
        std::vector<float4> nb(2 * (size_t)(n - 1));
        hkeys.resize(n);
        LCHK(hipMemcpyAsync(child2, d_child, sizeof(int) * 2 * (size_t)(n - 1), hipMemcpyDeviceToHost, st));
        LCHK(hipMemcpyAsync(nb.data(), d_nbox, sizeof(float4) * nb.size(), hipMemcpyDeviceToHost, st));
        LCHK(hipMemcpyAsync(hkeys.data(), d_sorted, sizeof(unsigned long long) * (size_t)n, hipMemcpyDeviceToHost, st));
        LCHK(hipStreamSynchronize(st));
        LCHK(hipEventElapsedTime(ms, e0, e1));
        for (int i = 0; i < n - 1; ++i) {
            const float4 a = nb[2 * i], b = nb[2 * i + 1];
            const float v[6] = {a.x, a.y, a.z, b.x, b.y, b.z};
            for (int k = 0; k < 6; ++k) node_box6[6 * i + k] = v[k];
        }
        if (algo != kGpuBvhSah)
            for (int i = 0; i < n; ++i) order[i] = (int32_t)(uint32_t)hkeys[i];
    }
    rc = 0;
done:
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d_box); (void)hipFree(d_nbox); (void)hipFree(d_keys); (void)hipFree(d_sorted);
    (void)hipFree(d_child); (void)hipFree(d_pint); (void)hipFree(d_pleaf); (void)hipFree(d_bounds);
    (void)hipFree(d_arrive); (void)hipFree(d_tmp);
    return rc;
}

}  // namespace frt
