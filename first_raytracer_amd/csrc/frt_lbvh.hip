// frt_lbvh.hip -- GPU BVH builder: a linear BVH over the
// world primitives' boxes, built on the device in four passes, as a fast
// alternative to the reference-topology SAH build (parallel_bvh_node::create_bvh,
// parallel_bvh.h:67-175; host: csrc/host/scene.cpp).
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

}  // namespace

namespace frt {

#define LCHK(x)                                                                                     \
    do {                                                                                            \
        const hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); goto done; }   \
    } while (0)

int lbvh_build(hipStream_t st, int n, const float *box6, int32_t *child2, float *node_box6, int32_t *order,
               float *ms, std::string &err)
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
    k_centroid_bounds<<<std::min(grid_n, 1024), kBlock, 0, st>>>(d_box, n, d_bounds);
    k_morton<<<grid_n, kBlock, 0, st>>>(d_box, n, d_bounds, d_keys);
    LCHK(hipGetLastError());
    LCHK(hipcub::DeviceRadixSort::SortKeys(d_tmp, tmp_bytes, d_keys, d_sorted, n, 0, 64, st));
    k_hierarchy<<<(n - 1 + kBlock - 1) / kBlock, kBlock, 0, st>>>(d_sorted, n, d_child, d_pint, d_pleaf);
    k_refit<<<grid_n, kBlock, 0, st>>>(d_box, d_sorted, n, d_child, d_pint, d_pleaf, d_arrive, d_nbox);
    LCHK(hipGetLastError());
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
