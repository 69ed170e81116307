// frt_render.hip -- MI355X (gfx950) path-tracing integrator: device layout,
// persistent path megakernel, film reduction and the C-ABI of include/frt.h.
//
// One lane owns one path.  Each loop iteration every active lane traces ONE
// ray (camera/extension = closest hit, or shadow = any hit) through the BVH
// with a per-lane LDS stack, then shades.  Lanes whose sample finished start
// the next sample of their work item; lanes whose item finished fetch a new
// one with one wave-aggregated atomic (__ballot + mbcnt compaction).  Work
// items are (tile, sample chunk, 64-pixel block) so a refill hands adjacent
// pixels to the lanes of a wave.  Results are written per (chunk, slot) and
// reduced in a fixed order: the image is deterministic and independent of
// scheduling and of the number of GPUs.
//
// Reference (first_ray/): path::Li path.cpp:4-116, path::Render path.cpp:118-148,
// parallel_bvh_node::hit parallel_bvh.h:39-64, hitable_list::hit
// hitable_list.cpp:4-21, camera::get_ray camera.h:30-35, viewer::add_sample
// viewer.cpp:109-132.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "frt.h"
#include "frt_device.hpp"
#include "frt_path.hpp"
#include "frt_mlt.hpp"
#include "frt_lbvh.hpp"

using namespace frt;

namespace {

constexpr int kBlock = 256;
constexpr size_t kLdsSceneBytes = 16 * 1024;   // LDS plan: 5-6 blocks/CU x (stack + scene) must fit 160 KiB
constexpr size_t kLdsOctBytes = 14 * 1024;     // ... with the octant node copies: 5 x (8 + 10 + 14) KiB
constexpr int kLdsMaxDepth = 16;                // LDS plan: binary stacks of 8 or 16 entries
// float4 slots of the octant plan's nodes in LDS (scene_to_lds): 8 x 3 per
// node for the boxes, then one int2 of child refs per node
__host__ __device__ constexpr int oct_lds_node_slots(int n_nodes) { return 24 * n_nodes + (n_nodes + 1) / 2; }
#ifndef FRT_QUEUE_GRAB
#define FRT_QUEUE_GRAB 64
#endif
constexpr int kQueueGrab = FRT_QUEUE_GRAB;      // path work queue: items a wave takes per atomic (at least)

struct DevWork {
    int nx, ny, spp, max_depth;
    uint32_t seed, s_off;                // frame seed, first global sample index (progressive passes)
    int tile, ntx, shard_index, shard_count;
    int spi, n_chunks;
    uint32_t n_items, n_slots;
    int trav_min;                        // shade when at most this many lanes of a wave still traverse
    int min_desc;                        // leaf postponing: see bvh2_step
    float *partial;                      // [n_chunks][n_slots][3]
    unsigned *counter;                   // work-queue head
    unsigned long long *wave_rays;       // [n_waves][4]: camera, extension, shadow, samples
    uint32_t grab;                       // items a wave takes per queue atomic (at least those it needs)
};

// slot -> pixel inside a tile: 8x8 blocks, row-major inside a block
__device__ __host__ __forceinline__ void slot_to_local(int s, int tile, int &lx, int &ly)
{
    const int b = s >> 6, l = s & 63;
    const int bpr = tile >> 3;
    lx = (b % bpr) * 8 + (l & 7);
    ly = (b / bpr) * 8 + (l >> 3);
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Small scenes (nodes + triangles + shading records + materials, <=
// kLdsSceneBytes) are copied into LDS once per block and traversed there
// (ds_read_b128 instead of L1/L2 round trips).  A wave's ds_read_b128 is
// served 16 lanes at a time from 64 banks: lanes reading distinct elements
// stay conflict-free when the elements' 16-B slots differ mod 16.  48-B
// records do that interleaved ((3 i + k) mod 16: triangles, the octant copies'
// node boxes), which puts every part at an immediate offset of one address;
// 64-B and 32-B records are copied planar (part k of element i at
// [k * count + i]), since interleaved only 4 or 8 slots would be used.
// Octant plan: 8 x n_nodes box records (3 float4), then the n_nodes child ref
// pairs (int2, one set for the 8 copies): 392 B per node instead of 512 B,
// 2 address VALU per node step instead of 5.
// HBM-resident scenes: the interleaved strides flatten_scene uses, as
// constants the compiler folds into the address arithmetic (kernel arguments
// would cost a quarter-rate v_mul_lo_u32 per node / triangle access).
__device__ __forceinline__ void scene_strides_hbm(DevScene &S)
{
    S.node_es = 4; S.node_ps = 1;
    S.node4_es = kNode4Parts; S.node4_ps = 1;
    S.tri_es = 3; S.tri_ps = 1;
    S.sh_es = 2; S.sh_ps = 1;
}

template <int WORLD>
__device__ __forceinline__ void scene_to_lds(DevScene &S, int *lds_base)
{
    // the LDS plans are binary (BVH4Q from LDS was 13 % slower on Cornell and was removed in round 4)
    static_assert(WORLD == FRT_WORLD_BVH || WORLD == kWorldBvh2Oct, "LDS plans hold a binary tree");
    constexpr bool OCT = WORLD == kWorldBvh2Oct;
    float4 *l4 = reinterpret_cast<float4 *>(lds_base);
    const DevScene S0 = S;
    const int nn = OCT ? oct_lds_node_slots(S0.n_nodes) : 4 * S0.n_nodes;
    const int nt = 3 * S0.n_tris, ns = 2 * S0.n_tris, nm = kMatStride * S0.n_mats;
    if constexpr (OCT) {   // node e = o * n_nodes + j, part k < 3 -> [3 e + k]; refs of j -> int2 [j]
        int2 *refs = reinterpret_cast<int2 *>(l4 + 24 * S0.n_nodes);
        for (int i = threadIdx.x; i < 32 * S0.n_nodes; i += kBlock) {
            const int e = i >> 2, k = i & 3;
            const float4 v = S0.nodes_oct[i];
            if (k < 3) l4[3 * e + k] = v;
            else if (e < S0.n_nodes) refs[e] = make_int2(f2i(v.x), f2i(v.y));
        }
        S.node_refs = refs;
    } else {
        for (int i = threadIdx.x; i < nn; i += kBlock) l4[(i & 3) * S0.n_nodes + (i >> 2)] = S0.nodes[i];
    }
    for (int i = threadIdx.x; i < nt; i += kBlock) l4[nn + i] = S0.tris[i];   // interleaved (48 B)
    for (int i = threadIdx.x; i < ns; i += kBlock) l4[nn + nt + (i & 1) * S0.n_tris + (i >> 1)] = S0.tshade[i];
    for (int i = threadIdx.x; i < nm; i += kBlock) l4[nn + nt + ns + i] = S0.mats[i];
    __syncthreads();
    S.nodes = l4;
    S.node_es = 1; S.node_ps = S0.n_nodes;
    S.tris = l4 + nn;
    S.tshade = l4 + nn + nt;
    S.mats = l4 + nn + nt + ns;
    S.tri_es = 3; S.tri_ps = 1;
    S.sh_es = 1; S.sh_ps = S0.n_tris;
}


// the octant node step of each integrator (bvh2_step's STEP): the path kernels
// store the far child without a branch (Cornell +0.4 %); AO and normals keep
// the branches (their rays agree more: Store cost AO 2.4 %, normals 3 %, same
// call, profiles/r05/r05af); PSS-MLT's chain kernel takes kStepSelect
#ifndef FRT_EXP_PATH_STEP
#define FRT_EXP_PATH_STEP kStepStore   // experiment builds vary the path kernels' form
#endif
#ifndef FRT_EXP_MLT_STEP
#define FRT_EXP_MLT_STEP kStepSelect   // ... and the chain kernel's
#endif
template <int KIND> constexpr int kPathStep = KIND == FRT_INTEGRATOR_PATH ? FRT_EXP_PATH_STEP : kStepBranch;
// ------------------------------------------------------------------------
// the persistent path megakernel
// ------------------------------------------------------------------------
// Work-item state of a lane: sample range, slot, chunk, pixel and the chunk's
// radiance sum, in an LDS column (kItemWords x kBlock ints after the traversal
// stack).  It is touched once per sample; as VGPRs it stayed live -- and
// spilled to scratch -- across every traversal and shading phase (spilled
// VGPRs at the register cap: cornell_1m 51 -> 24, Cornell 31 -> 6; same-call
// A/B +4.5 % / +1 %).
// (9 words -- the pixel index derived -- fit a 6th octant block per CU: 229.4 vs 229.1 ms at a
// 6-wave cap, 230.5 vs 230.2 at 5, profiles/r05/r05l; not kept)
// (7 words -- the end and the pixel coordinates derived -- measured 1 % slower on Cornell and
// +-0 on cornell_1m, also with the 4-wide plan's LDS stack grown to 15 entries: profiles/r06/r06i)
constexpr int kItemWords = 10;
enum { kIsCur, kIsEnd, kIsSlot, kIsChunk, kIsPix, kIsPx, kIsPy, kIsAcc };   // kIsAcc..+2: r, g, b
struct ItemState {
    int *b;      // the lane's column
    __device__ int get(int k) const { return b[k * kBlock]; }
    __device__ void set(int k, int x) const { b[k * kBlock] = x; }
};

// R: float (the product kernels) or double (the fp64 kernels, DESIGN.md
// "Precision": list worlds under FRT_PRECISION_AUTO, every plan under _FP64)
template <int STACK, int WORLD, bool LDS_SCENE, int WAVES = 1, int MATS = kMatsNone,
          int KIND = FRT_INTEGRATOR_PATH, typename R = float>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) void path_megakernel(
    const DevScene S0, const DevWork W)
{
    // [STACK][kBlock] stack, [kItemWords][kBlock] item state, then the scene
    extern __shared__ __attribute__((aligned(16))) int lds_mem[];
    int *stk = lds_mem + threadIdx.x;                                 // one LDS column per lane
    constexpr int kStackInts = WORLD != FRT_WORLD_LIST ? STACK * kBlock : 0;
    constexpr int kItemInts = kItemWords * kBlock;
    DevScene S = S0;
    if constexpr (LDS_SCENE) scene_to_lds<WORLD>(S, lds_mem + kStackInts + kItemInts);
    else scene_strides_hbm(S);
    const int lane = threadIdx.x & 63;
    const int T2 = W.tile * W.tile;

    // work-item state
    bool have_item = false, exhausted = false, active = false;
    // the wave's own item range [q_cur, q_end) from its last queue atomic (wave-uniform)
    uint32_t q_cur = 0, q_end = 0;
    const ItemState I{lds_mem + kStackInts + (int)threadIdx.x};
    PathState<R> P;
    // ray in flight: tracing = traversal steps remain; pending = finished, not yet shaded
    Trav<R> T;
    bool tracing = false, pending = false;
    int ovf[kOverflow<WORLD>];
    // ray counters are wave-uniform (SGPRs): popcounts of per-iteration ballots
    unsigned long long n_cam = 0, n_ext = 0, n_sh = 0, n_smp = 0;
    // HBM plans of the lambertian path kernels keep less per-lane state across
    // the traversal steps: the sample's radiance goes into the item's LDS sum
    // as it is found (NEE after a shadow ray, emission, environment), the RNG
    // key is re-derived from the item at shading, t_max from the ray kind.
    // cornell_1m +1.2 % (spilled VGPRs 26 -> 14); on the LDS plan it costs
    // 0.3 % (same-call A/B, profiles/r03/samecall/lean_*.jsonl).  The material
    // kernels keep the full state (DESIGN.md "Register-cap hazard"), and so do
    // the fp64 kernels (their per-sample sum stays fp64 until the sample ends).
    // The flushes round each contribution into the fp32 item sum, so a lean
    // plan's film equals the per-sample plans' to fp32 rounding, not bit for
    // bit (tests/test_gpu_parity.py::test_lean_plan_rounding).
    constexpr bool kLean = !LDS_SCENE && MATS == kMatsNone && KIND == FRT_INTEGRATOR_PATH && !kIsF64<R>;
    auto flush_L = [&]() {
        I.set(kIsAcc + 0, f2i(i2f(I.get(kIsAcc + 0)) + (float)P.L.x));
        I.set(kIsAcc + 1, f2i(i2f(I.get(kIsAcc + 1)) + (float)P.L.y));
        I.set(kIsAcc + 2, f2i(i2f(I.get(kIsAcc + 2)) + (float)P.L.z));
        P.L = zero3<R>();
    };
    auto ray_tmax = [&]() -> R {
        if constexpr (kLean) return P.shadow ? R(1) - Cst<R>::shadow_eps : Cst<R>::tmax;
        else return P.rtmax;
    };

    unsigned long long diag_t0 = FRT_DIAG_CLOCK();
    for (;;) {
        FRT_DIAG_TICK(6);
        // ---- traversal: steps (descend to a leaf, test it) of every lane's ray,
        // until at most trav_min lanes are still traversing.  Lanes whose ray is
        // done wait here only while the rest of the wave needs few more steps;
        // then they shade together while the stragglers keep their state.
        for (;;) {
            bool shadow_done = false;
            if (tracing) FRT_DIAG_TICK(3);
            // (LDS-resident binary plans: no leaf postponing, compiled out)
            if (tracing && trav_step_world<WORLD, kBlock, STACK, kPathStep<KIND>>(T, S, P.ro, P.rd, P.shadow, stk, ovf,
                                                                       LDS_SCENE && (WORLD == FRT_WORLD_BVH || WORLD == kWorldBvh2Oct)
                                                                           ? 0 : W.min_desc)) {
                if (KIND == FRT_INTEGRATOR_PATH && P.shadow) {   // finish the shadow ray here, keep traversing
                    if (path_after_shadow<MATS>(P, T.h.prim < 0)) {
                        if constexpr (kLean) flush_L();
                        shadow_done = true;
                        tracing = trav_begin_world<WORLD>(T, S, P.ro, P.rd, ray_tmax());
                        pending = !tracing;
                    } else {                                      // path ended (P.term): shade finishes it
                        tracing = false;
                        pending = true;
                    }
                } else {
                    tracing = false;
                    pending = true;
                }
            }
            n_ext += __popcll(__ballot(shadow_done));
            if (__popcll(__ballot(tracing)) <= W.trav_min) break;
        }
        // ---- shade the finished rays ----
        const unsigned long long diag_t1 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(16, diag_t1 - diag_t0);
        uint32_t ne = 0, ns = 0;
        bool next_ray = false;
        if (pending) {
            FRT_DIAG_TICK(4);
            pending = false;
            if constexpr (kLean)
                P.key = rng_key(W.seed, (uint32_t)I.get(kIsPix), (uint32_t)(I.get(kIsCur) - 1) + W.s_off);
            const bool done = shade_kind<KIND, MATS>(P, S, T.h, W.max_depth, ne, ns);
            if (done || kLean) flush_L();   // fp32 chunk sums in either precision
            active = !done;
            next_ray = !done;
        }
        n_ext += __popcll(__ballot(ne != 0));
        n_sh += __popcll(__ballot(ns != 0));
        const unsigned long long diag_t2 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(17, diag_t2 - diag_t1);
        // ---- retire a finished item: its chunk sum goes to its own slot ----
        if (!active && have_item && I.get(kIsCur) >= I.get(kIsEnd)) {
            float *dst = W.partial + 3ull * ((size_t)(uint32_t)I.get(kIsChunk) * W.n_slots + (uint32_t)I.get(kIsSlot));
            dst[0] = i2f(I.get(kIsAcc + 0)); dst[1] = i2f(I.get(kIsAcc + 1)); dst[2] = i2f(I.get(kIsAcc + 2));
            have_item = false;
        }
        // ---- wave-aggregated refill, lanes ranked by mbcnt: items come from the
        // wave's own range first; when it runs short, one atomic takes
        // max(grab, still needed) more.  With one atomic per refill every wave
        // of the grid queued on one counter: AO (1.5 rays a sample) took 72.5 ms
        // at 1080p 512 spp, 31.9 ms with 64 items a grab; Cornell path +1.0 %,
        // cornell_1m +1.6 %; 256 a grab lengthens the frame's tail
        // (profiles/r03/samecall/grab_*.jsonl).  Items are disjoint and each
        // (chunk, slot) sum has one writer, so the film does not depend on it. ----
        const bool need = !active && !have_item && !exhausted;
        const uint64_t m = __ballot(need);
        if (m) {
            const uint32_t nm = (uint32_t)__popcll(m), r = lane_rank(m);
            const uint32_t left = q_end - q_cur;
            uint32_t w;
            if (nm <= left) {
                w = q_cur + r;
                q_cur += nm;
            } else {
                const uint32_t take = max(W.grab, nm - left);
                const int leader = __ffsll((unsigned long long)m) - 1;
                uint32_t base = 0;
                if (lane == leader) base = atomicAdd(W.counter, take);
                base = __shfl(base, leader);
                w = r < left ? q_cur + r : base + (r - left);
                q_cur = base + (nm - left);
                q_end = base + take;
            }
            if (need) {
                if (w >= W.n_items) {
                    exhausted = true;
                } else {
                    const uint32_t s = w % (uint32_t)T2;
                    const uint32_t q = w / (uint32_t)T2;
                    const uint32_t chunk = q % (uint32_t)W.n_chunks;
                    const uint32_t t_ord = q / (uint32_t)W.n_chunks;
                    const int tile_id = W.shard_index + (int)t_ord * W.shard_count;
                    int lx, ly;
                    slot_to_local((int)s, W.tile, lx, ly);
                    const int px = (tile_id % W.ntx) * W.tile + lx;
                    const int py = (tile_id / W.ntx) * W.tile + ly;
                    if (px < W.nx && py < W.ny) {   // padding slots of edge tiles carry no work
                        have_item = true;
                        const int s_cur = (int)chunk * W.spi;
                        I.set(kIsCur, s_cur);
                        I.set(kIsSlot, (int)(t_ord * (uint32_t)T2 + s));
                        I.set(kIsChunk, (int)chunk);
                        I.set(kIsPix, py * W.nx + px);
                        I.set(kIsEnd, min(W.spp, s_cur + W.spi));
                        I.set(kIsPx, px);
                        I.set(kIsPy, py);
                        I.set(kIsAcc + 0, 0); I.set(kIsAcc + 1, 0); I.set(kIsAcc + 2, 0);
                    }
                }
            }
        }
        // ---- next camera sample of the item ----
        const bool start = !active && have_item && I.get(kIsCur) < I.get(kIsEnd);
        if (start) {
            const int s_cur = I.get(kIsCur);
            path_begin(P, S, I.get(kIsPx), I.get(kIsPy), W.nx, W.ny, W.seed, (uint32_t)I.get(kIsPix),
                       (uint32_t)s_cur + W.s_off);
            I.set(kIsCur, s_cur + 1);
            active = true;
            next_ray = true;
        }
        const unsigned long long started = __popcll(__ballot(start));
        n_cam += started;
        n_smp += started;
        // ---- set up the next ray's traversal (a scene miss is finished at once) ----
        if (next_ray) {
            tracing = trav_begin_world<WORLD>(T, S, P.ro, P.rd, ray_tmax());
            pending = !tracing;
        }
        diag_t0 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(18, diag_t0 - diag_t2);
        if (__ballot(active || !exhausted) == 0) break;
    }
    // per-wave ray counters, no atomics: lane 0 writes the wave's sums
    const unsigned long long c[4] = {n_cam, n_ext, n_sh, n_smp};
    if (lane == 0) {
        const size_t wv = ((size_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
        for (int k = 0; k < 4; ++k) W.wave_rays[4 * wv + k] = c[k];
    }
}


// ------------------------------------------------------------------------
// ray queries (frt_trace_device): a buffer of rays through the same
// resumable traversal, Scene::world->hit (path.cpp:10, 50; parallel_bvh.h:39-64,
// hitable_list.cpp:4-21) batched.  Persistent; a lane whose ray is done takes
// the next ray at once, so the wave's lanes stay busy until the buffer runs
// dry.  Rays come from a wave-local chunk (kTraceChunk rays taken with one
// atomic); a global atomic per refill put its latency on every traversal
// step (4 Grays/s on camera rays: profiles/r03/r03e_trace_atomic_per_step.jsonl).
// ------------------------------------------------------------------------
constexpr uint32_t kTraceChunk = 256;   // rays a wave takes from the buffer with one atomic
// the context's queue words: [0] the render / PSS-MLT work queue, [kTraceCounterWord] the ray-query queue
constexpr size_t kCounterBytes = 256;
constexpr int kTraceCounterWord = 32;   // 128 B after the render queue's word
struct DevRays {
    const float4 *ray;       // 2 per ray: (origin, t_max) | (direction, flags: bit 0 = any-hit)
    float4 *hit;             // 1 per ray: (t, u, v, prim ref of the scene view as int bits; -1 = miss)
    uint32_t n;
    int min_desc;            // leaf postponing (bvh2_step)
    unsigned *counter;       // ray-queue head
};
template <int STACK, int WORLD, bool LDS_SCENE, int WAVES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES))) void trace_kernel(
    const DevScene S0, const DevRays R)
{
    extern __shared__ __attribute__((aligned(16))) int lds_mem[];
    int *stk = lds_mem + threadIdx.x;                                 // one LDS column per lane
    constexpr int kStackInts = WORLD != FRT_WORLD_LIST ? STACK * kBlock : 0;
    DevScene S = S0;
    if constexpr (LDS_SCENE) scene_to_lds<WORLD>(S, lds_mem + kStackInts);
    else scene_strides_hbm(S);
    const int lane = threadIdx.x & 63;
    Trav<float> T;
    int ovf[kOverflow<WORLD>];
    f3 o = mk3(0, 0, 0), d = mk3(0, 0, 1);
    bool anyhit = false, tracing = false, exhausted = false;
    uint32_t id = 0;
    auto finish = [&]() {
        const int p = T.h.prim;
        const int ref = (p < 0 || (p & FRT_PRIM_SPHERE)) ? p : S.tri_view[p];
        R.hit[id] = make_float4(T.h.t, T.h.u, T.h.v, i2f(ref));
    };
    // Each lane holds the NEXT ray of its queue in registers (loaded while the
    // current one traverses), so a lane that finishes starts its next ray
    // without waiting on memory.
    uint32_t chunk_next = 0, chunk_end = 0;                          // wave-uniform
    float4 na = make_float4(0, 0, 0, 0), nb = make_float4(0, 0, 0, 0);
    uint32_t nid = 0;
    bool have_next = false;
    for (;;) {
        if (!tracing && have_next) {                                  // start the prefetched ray
            id = nid;
            o = xyz(na);
            d = xyz(nb);
            anyhit = (f2i(nb.w) & 1) != 0;
            have_next = false;
            tracing = trav_begin_world<WORLD>(T, S, o, d, na.w);
            if (!tracing) finish();                                   // the ray misses the scene box
        }
        const bool need = !have_next && !exhausted;
        const uint64_t m = __ballot(need);
        if (m) {
            // the wave's lanes without a queued ray take the rest of its chunk,
            // then a new chunk (one atomic per kTraceChunk rays) once it runs short
            const uint32_t want = (uint32_t)__popcll(m), left = chunk_end - chunk_next;
            uint32_t fresh = 0xffffffffu;
            if (left < want && chunk_end < R.n) {
                uint32_t b0 = 0;
                if (lane == 0) b0 = atomicAdd(R.counter, kTraceChunk);
                fresh = __builtin_amdgcn_readfirstlane(__shfl(b0, 0));
            }
            const uint32_t rank = lane_rank(m);
            const uint32_t w = rank < left ? chunk_next + rank : (fresh == 0xffffffffu ? 0xffffffffu : fresh + (rank - left));
            if (left >= want) {
                chunk_next += want;
            } else if (fresh != 0xffffffffu) {
                chunk_next = fresh + (want - left);
                chunk_end = fresh + kTraceChunk;
            } else {
                chunk_next = chunk_end;
            }
            if (need) {
                if (w >= R.n) {
                    exhausted = true;
                } else {
                    nid = w;
                    na = R.ray[2 * (size_t)w];
                    nb = R.ray[2 * (size_t)w + 1];
                    have_next = true;
                }
            }
        }
        if (__ballot(tracing || have_next) == 0) break;
        if (tracing && trav_step_world<WORLD, kBlock, STACK>(T, S, o, d, anyhit, stk, ovf,
                                                             LDS_SCENE && (WORLD == FRT_WORLD_BVH || WORLD == kWorldBvh2Oct) ? 0 : R.min_desc)) {
            tracing = false;
            finish();
        }
    }
}

// film: slot mean = sum over chunks (fixed order) * (1/spp)  (viewer.cpp:111)
__global__ void film_reduce(const float *__restrict__ partial, float *__restrict__ out, uint32_t n_slots,
                            int n_chunks, int spp, int tile, int ntx, int shard_index, int shard_count, int nx, int ny)
{
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const int T2 = tile * tile;
    const int t_ord = (int)(s / (uint32_t)T2), sl = (int)(s % (uint32_t)T2);
    const int tile_id = shard_index + t_ord * shard_count;
    int lx, ly;
    slot_to_local(sl, tile, lx, ly);
    const int px = (tile_id % ntx) * tile + lx, py = (tile_id / ntx) * tile + ly;
    float r = 0.0f, g = 0.0f, b = 0.0f;
    if (px < nx && py < ny) {
        for (int c = 0; c < n_chunks; ++c) {
            const float *q = partial + 3ull * ((size_t)c * n_slots + s);
            r += q[0]; g += q[1]; b += q[2];
        }
        const float k = 1.0f / (float)spp;
        r *= k; g *= k; b *= k;
    }
    out[3ull * s + 0] = r;
    out[3ull * s + 1] = g;
    out[3ull * s + 2] = b;
}

// frt_render_multi: the gathered slot buffers of n shards (shard r at
// gathered[r * max_slots * 3]) into the device film, (y*nx+x)*3
__global__ void scatter_shards(const float *__restrict__ gathered, float *__restrict__ film, uint32_t max_slots,
                               int n, int tile, int ntx, int nx, int ny)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (uint64_t)max_slots * (uint64_t)n) return;
    const int r = (int)(i / max_slots);
    const uint32_t s = (uint32_t)(i % max_slots);
    const int T2 = tile * tile;
    const int tile_id = r + (int)(s / (uint32_t)T2) * n;
    int lx, ly;
    slot_to_local((int)(s % (uint32_t)T2), tile, lx, ly);
    const int px = (tile_id % ntx) * tile + lx, py = (tile_id / ntx) * tile + ly;
    if (px >= nx || py >= ny) return;                // padding slots, slots past a short shard's end
    const size_t d = 3 * ((size_t)py * nx + px);
    film[d + 0] = gathered[3 * i + 0];
    film[d + 1] = gathered[3 * i + 1];
    film[d + 2] = gathered[3 * i + 2];
}

// ------------------------------------------------------------------------
// PSS-MLT (pssmlt.cpp:301-365)
// ------------------------------------------------------------------------
// chain state columns (ItemState over kChainWords words): step count, chain
// index, the current state's film position, scalar contribution, pending
// weight and colour
constexpr int kChainWords = 9;
enum { kCsT, kCsC, kCsX, kCsY, kCsSc, kCsW, kCsCc };   // kCsCc..+2: r, g, b
struct MltWork {
    int nx, ny;
    uint32_t seed;
    int shard_index, shard_count;
    uint32_t n_local;                    // chains of this shard: global c = shard_index + j * shard_count
    uint64_t steps;                      // mutations per chain
    float b, scale, s2p, logp;           // normaliser, nx*ny/ns, pixel-dim perturb constants
    int trav_min;                        // see path_megakernel / trav_min()
    int min_desc;                        // leaf postponing: see bvh2_step
    float *U;                            // [n_local][kMltRow] current primary samples + fingerprint (frt_mlt.hpp)
    unsigned long long *film;            // [nx*ny*3] splat accumulation, fixed point (kSplatFix)
    unsigned *counter;
    unsigned long long *wave_rays;
};

template <int WORLD, int STACK>
__device__ __forceinline__ Hit<float> trace_any(const DevScene &S, const PathState<float> &P, int *stk)
{
    return trace<WORLD, kBlock, STACK>(S, P.ro, P.rd, P.rtmax, P.shadow, stk);
}

// bootstrap: sc of n_init independent eye paths (pssmlt.cpp:303-312); the host
// sums them in a fixed order
template <int STACK, int WORLD, bool MATS>
__global__ __launch_bounds__(kBlock) void mlt_bootstrap(const DevScene S0, int nx, int ny, uint32_t seed, int n_init,
                                                        float *sc)
{
    DevScene S = S0;
    scene_strides_hbm(S);
    extern __shared__ __attribute__((aligned(16))) int lds_mem[];
    int *stk = lds_mem + threadIdx.x;
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n_init) return;
    PrndSource src{nullptr, 0, 0, rng_key(seed ^ kMltBootSalt, (uint32_t)i, 0u), 0u, true, 0.0f, 0.0f};
    MltPath M;
    mlt_begin(M, S, src, nx, ny);
    uint32_t ne = 0, ns = 0;
    for (;;) {
        if (mlt_beyond(M)) { M.P.L = M.P.L + M.P.beta * S.env; break; }
        const Hit<float> h = trace_any<WORLD, STACK>(S, M.P, stk);
        if (mlt_shade<MATS>(M, S, h, src, ne, ns)) break;
    }
    sc[i] = fmaxf(fmaxf(M.P.L.x, M.P.L.y), M.P.L.z);
}

// Splats (AccumulatePathContribution, pssmlt.cpp) add into a fixed-point film:
// a splat is rounded to a multiple of 2^-kSplatFix and added with a 64-bit
// integer atomic.  Integer sums do not depend on the order the chains' atomics
// land in, so the film is bit-reproducible run to run (float atomics were
// not).  Splats are >= 0 (scale, weights and radiance are); the quantum
// 2^-36 = 1.5e-11 is far below fp32's resolution of the pixel values, and a
// signed 64-bit pixel holds up to 2^27 before it wraps.  A splat that is not a
// finite value in [0, 2^27) is dropped (the reference's pixel would turn NaN /
// Inf there; none occurs in the test scenes).  mlt_film_to_float converts once
// at the end.
constexpr int kSplatFix = 36;
__device__ __forceinline__ void mlt_splat(const MltWork &W, float x, float y, f3 c, float w)
{
    const int pix = mlt_pixel(x, y, W.nx, W.ny);
    if (pix < 0) return;
    const float k = W.scale * w;
    const double q = (double)(1ull << kSplatFix), lim = 9.2233720368547758e18;   // 2^63
    const double v[3] = {(double)(k * c.x) * q, (double)(k * c.y) * q, (double)(k * c.z) * q};
    if (!(v[0] >= 0.0 && v[0] < lim && v[1] >= 0.0 && v[1] < lim && v[2] >= 0.0 && v[2] < lim)) return;
    unsigned long long *f = W.film + 3 * (size_t)pix;
    atomicAdd(f + 0, (unsigned long long)__double2ll_rn(v[0]));
    atomicAdd(f + 1, (unsigned long long)__double2ll_rn(v[1]));
    atomicAdd(f + 2, (unsigned long long)__double2ll_rn(v[2]));
}
__global__ void mlt_film_to_float(const unsigned long long *__restrict__ acc, float *__restrict__ film, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) film[i] = (float)((double)(long long)acc[i] * (1.0 / (double)(1ull << kSplatFix)));
}

// one lane = one chain tracing the rays of its current eye path (initial
// state, then one proposal per mutation); traversal steps interleave with
// shading as in path_megakernel
#ifndef FRT_EXP_MLT_WAVES
#define FRT_EXP_MLT_WAVES 4      // register cap of the chain kernel: 4 waves/SIMD.  Round 1 measured 5
#endif                           // +17 % over the compiler's own allocation (profiles/r01_expmlt1.txt);
                                 // round 4's kernel: 4 waves 690.8 ms, 5 waves 700.5, 6 waves 783.9
                                 // (same call, profiles/r04/r04g); experiment builds vary it
template <int STACK, int WORLD, bool LDS_SCENE, bool MATS>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(FRT_EXP_MLT_WAVES))) void mlt_megakernel(
    const DevScene S0, const MltWork W)
{
    // [STACK][kBlock] stack, [kChainWords][kBlock] chain state, then the scene
    extern __shared__ __attribute__((aligned(16))) int lds_mem[];
    int *stk = lds_mem + threadIdx.x;
    constexpr int kStackInts = WORLD != FRT_WORLD_LIST ? STACK * kBlock : 0;
    DevScene S = S0;
    if constexpr (LDS_SCENE) scene_to_lds<WORLD>(S, lds_mem + kStackInts + kChainWords * kBlock);
    else scene_strides_hbm(S);
    const int lane = threadIdx.x & 63;
    bool have = false, exhausted = false, init = false, large = false;
    // the chain's current state (touched once per proposal) in an LDS column,
    // as the path kernel's work item (ItemState)
    const ItemState C{lds_mem + kStackInts + (int)threadIdx.x};
    uint32_t j = 0;
    RngKey key{0, 0};
    MltPath M;
    uint32_t n_cam = 0, n_ext = 0, n_sh = 0, n_smp = 0;

    auto source = [&]() {
        PrndSource src{W.U, W.n_local, j, key, 2u, init || large, W.s2p, W.logp};
        return src;
    };
    // ray in flight, as in path_megakernel: tracing = traversal steps remain;
    // pending = finished (or the path went beyond MaxPathLength), not yet shaded
    Trav<float> T;
    bool tracing = false, pending = false, beyond = false;
    int ovf[kOverflow<WORLD>];
    // diagnostic build (FRT_DIAG, tools/diag_phases.py --integrator pssmlt): lane
    // counts of the traversal (pairs 1, 2, 7 in bvh2_step), step loop (3),
    // shading (4), accept / reject (5), outer loop (6); cycles of the step loop
    // (16), shading (17), accept / reject + splats (19), row materialisation
    // (20), queue + next proposal (18)
    unsigned long long diag_t0 = FRT_DIAG_CLOCK();
    for (;;) {
        FRT_DIAG_TICK(6);
        // ---- traversal steps until at most trav_min lanes still traverse ----
        for (;;) {
            bool ext = false;
            if (tracing) FRT_DIAG_TICK(3);
            if (tracing && trav_step_world<WORLD, kBlock, STACK, FRT_EXP_MLT_STEP>(T, S, M.P.ro, M.P.rd, M.P.shadow, stk, ovf,
                                                                 LDS_SCENE ? 0 : W.min_desc)) {   // LDS plans: compiled out
                if (M.P.shadow) {               // finish the shadow ray here (mlt_shade's shadow branch)
                    if (!path_after_shadow<(MATS ? kMatsAll : kMatsNone)>(M.P, T.h.prim < 0)) {   // path ended (P.term)
                        tracing = false;
                        pending = true;
                    } else if (mlt_beyond(M)) {
                        beyond = true;
                        tracing = false;
                        pending = true;
                    } else {
                        ext = true;
                        tracing = trav_begin_world<WORLD>(T, S, M.P.ro, M.P.rd, M.P.rtmax);
                        pending = !tracing;
                    }
                } else {
                    tracing = false;
                    pending = true;
                }
            }
            if (ext) ++n_ext;                   // per-lane counters, reduced at the end
            if (__popcll(__ballot(tracing)) <= W.trav_min) break;
        }
        bool next_ray = false, done = false;
        const unsigned long long diag_t1 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(16, diag_t1 - diag_t0);
        if (pending) {
            FRT_DIAG_TICK(4);
            pending = false;
            if (beyond) {                               // pssmlt.cpp:151, :276
                M.P.L = M.P.L + M.P.beta * S.env;
                beyond = false;
                done = true;
            } else {
                uint32_t ne = 0, ns = 0;
                done = mlt_shade<MATS>(M, S, T.h, source(), ne, ns);
                n_ext += ne; n_sh += ns;
                next_ray = !done;
            }
        }
        // accept / reject (per lane); the accepted proposal's row is written below
        const unsigned long long diag_t2 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(17, diag_t2 - diag_t1);
        bool mat = false, mat_fresh = false, setup_next = false;
        RngKey mat_key = key;
        if (done) {
            FRT_DIAG_TICK(5);
            const f3 L = M.P.L;
            const float sc = fmaxf(fmaxf(L.x, L.y), L.z);
            float cx = i2f(C.get(kCsX)), cy = i2f(C.get(kCsY)), csc = i2f(C.get(kCsSc)), cw = i2f(C.get(kCsW));
            f3 cc = mk3(i2f(C.get(kCsCc)), i2f(C.get(kCsCc + 1)), i2f(C.get(kCsCc + 2)));
            uint32_t t = (uint32_t)C.get(kCsT);
            bool moved = false;
            if (init) {                                 // current = initial state, materialised
                mat = true; mat_fresh = true;
                cx = M.x; cy = M.y; cc = L; csc = sc;
                moved = true;
                init = false;
            } else {                                    // pssmlt.cpp:200-209
                float a = 1.0f;
                if (csc > 0.0f) a = fmaxf(fminf(1.0f, sc / csc), 0.0f);
                if (sc > 0.0f) mlt_splat(W, M.x, M.y, L, (a + (large ? 1.0f : 0.0f)) / (sc / W.b + kMltLargeStep));
                if (csc > 0.0f) cw += (1.0f - a) / (csc / W.b + kMltLargeStep);
                if (rng_u(key, 1) <= a) {               // accept: splat the old state's weight, move
                    if (csc > 0.0f && cw != 0.0f) mlt_splat(W, cx, cy, cc, cw);
                    uint2 *fp = reinterpret_cast<uint2 *>(W.U + (size_t)j * kMltRow + kMltFp);
                    uint2 f = *fp;                      // trajectory fingerprint: (accepts, sum of 1-based steps)
                    f.x += 1u; f.y += t + 1u;
                    *fp = f;
                    cw = 0.0f;
                    mat = true; mat_fresh = large;
                    cx = M.x; cy = M.y; cc = L; csc = sc;
                    moved = true;
                }
                ++t;
                ++n_smp;
            }
            if ((uint64_t)t >= W.steps) {               // chain finished
                if (csc > 0.0f && cw != 0.0f) mlt_splat(W, cx, cy, cc, cw);
                have = false;
            } else {
                setup_next = true;
                C.set(kCsT, (int)t);
                C.set(kCsW, f2i(cw));
                if (moved) {
                    C.set(kCsX, f2i(cx)); C.set(kCsY, f2i(cy)); C.set(kCsSc, f2i(csc));
                    C.set(kCsCc, f2i(cc.x)); C.set(kCsCc + 1, f2i(cc.y)); C.set(kCsCc + 2, f2i(cc.z));
                }
            }
        }
        // ---- materialise accepted proposals: the rows of the wave's n accepted
        // chains as one flat range of n * 92 elements over the 64 lanes
        // (element e: chain rank e / 92, dimension e % 92).  A ds_permute first
        // moves the r-th accepted chain's (row, key, fresh) to lane r (the other
        // lanes fill lanes n..63, so it is a permutation).  Coalesced along each
        // row; only the last trip has idle lanes (one chain at a time left 28 of
        // 64 lanes idle on every second trip).  The whole wave is active here. ----
        const unsigned long long diag_t3 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(19, diag_t3 - diag_t2);
        if (const uint64_t mm = __ballot(mat)) {
            const uint32_t n = (uint32_t)__popcll(mm);
            const int dst = 4 * (int)(mat ? lane_rank(mm) : n + lane_rank(~mm));   // byte address of the target lane
            const uint32_t rj = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)(j | (mat_fresh ? 0x80000000u : 0u)));
            const uint32_t rk0 = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)mat_key.k0);
            const uint32_t rk1 = (uint32_t)__builtin_amdgcn_ds_permute(dst, (int)mat_key.k1);
            const uint32_t total = n * (uint32_t)kMltDims;
            for (uint32_t e0 = 0; e0 < total; e0 += 64) {
                const uint32_t e = e0 + (uint32_t)lane;
                const uint32_t r = min(e / (uint32_t)kMltDims, n - 1u);
                const uint32_t jl = (uint32_t)__shfl((int)rj, (int)r);   // every lane active: sources are lanes < n
                const RngKey kl{(uint32_t)__shfl((int)rk0, (int)r), (uint32_t)__shfl((int)rk1, (int)r)};
                if (e < total) {
                    const int d = (int)(e - r * (uint32_t)kMltDims);
                    float *row = W.U + (size_t)(jl & 0x7fffffffu) * kMltRow;   // j < 2^31: bit 31 = fresh
                    const float u = rng_u(kl, 2u + (uint32_t)d);
                    row[d] = (jl >> 31) ? u : mlt_mutate(row[d], u, d, W.s2p, W.logp);
                }
            }
        }
        const unsigned long long diag_t4 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(20, diag_t4 - diag_t3);
        if (setup_next) {                               // next proposal reads the new state
            key = rng_key(W.seed ^ kMltChainSalt, (uint32_t)C.get(kCsC), (uint32_t)C.get(kCsT) + 1u);
            large = rng_u(key, 0) < kMltLargeStep;      // large_step vs mutate (pssmlt.cpp:187-196)
            mlt_begin(M, S, source(), W.nx, W.ny);
            ++n_cam;
            next_ray = true;
        }
        // ---- chains from the queue, one atomic per wave ----
        const bool need = !have && !exhausted;
        const uint64_t m = __ballot(need);
        if (m) {
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(W.counter, (unsigned)__popcll(m));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t w = base + lane_rank(m);
                if (w >= W.n_local) {
                    exhausted = true;
                } else {
                    have = true;
                    init = true;
                    j = w;
                    *reinterpret_cast<uint2 *>(W.U + (size_t)w * kMltRow + kMltFp) = make_uint2(0u, 0u);
                    const uint32_t c = (uint32_t)W.shard_index + w * (uint32_t)W.shard_count;
                    C.set(kCsC, (int)c);
                    C.set(kCsT, 0);
                    C.set(kCsW, 0);
                    C.set(kCsSc, 0);
                    key = rng_key(W.seed ^ kMltChainSalt, c, 0u);   // initial state: TMarkovChain(s)
                    mlt_begin(M, S, source(), W.nx, W.ny);
                    ++n_cam;
                    next_ray = true;
                }
            }
        }
        // ---- next ray of the eye path ----
        if (next_ray) {
            if (mlt_beyond(M)) {
                beyond = true;
                pending = true;
            } else {
                tracing = trav_begin_world<WORLD>(T, S, M.P.ro, M.P.rd, M.P.rtmax);
                pending = !tracing;
            }
        }
        diag_t0 = FRT_DIAG_CLOCK();
        FRT_DIAG_CYC(18, diag_t0 - diag_t4);
        if (__ballot(have || !exhausted) == 0) break;
    }
    unsigned long long cnt[4] = {n_cam, n_ext, n_sh, n_smp};
    for (int k = 0; k < 4; ++k)
        for (int off = 32; off > 0; off >>= 1) cnt[k] += __shfl_xor(cnt[k], off);
    if (lane == 0) {
        const size_t wv = ((size_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
        for (int k = 0; k < 4; ++k) W.wave_rays[4 * wv + k] = cnt[k];
    }
}

}  // namespace

#if defined(FRT_DIAG) && !defined(FRT_TU_MATS)
__device__ unsigned long long *frt::frt_diag;
#endif

// ==========================================================================
// host side
// ==========================================================================
struct frt_ctx {
    int device = -1;
    int n_cu = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string err;
    // scene
    bool have_scene = false;
    DevScene S{};
    int world_kind = 0, stack_needed = 0;
    bool has_bvh4 = false;        // nodes4 holds the 4-wide BVH4Q
    int depth4 = 0;               // levels of that wide tree
    int n_tris = 0, n_spheres = 0, n_list = 0;
    bool has_spec_mats = false;   // a non-lambertian scattering material or a texture: MATS kernels
    int mats = kMatsNone;         // kMats* mask of the scene's material set (pick_launcher)
    bool has_metal = false;       // ao::Li cannot sample metal (constant_pdf::generate throws, pdf.h:195-198)
    size_t scene_lds_bytes = 0;                         // LDS copy with the binary nodes
    size_t scene_lds_bytes_oct = 0;                     // ... with the 8 octant copies of the binary nodes
    int precision = FRT_PRECISION_AUTO;                 // frt_set_precision
    bool has_f64 = false;                               // the scene's fp64 records are in HBM
    double last_mlt_b = 0.0;
    uint64_t mlt_rows = 0;        // chains whose state rows the last PSS-MLT render left in `partial`
    std::vector<void *> scene_bufs;
    // workspace
    float *partial = nullptr; size_t partial_bytes = 0;
    unsigned *counter = nullptr;
    unsigned long long *wave_rays = nullptr; size_t wave_rays_n = 0;
    float *slots_out = nullptr; size_t slots_out_bytes = 0;
    unsigned long long *splat = nullptr; size_t splat_bytes = 0;   // PSS-MLT fixed-point splat film
    // frt_render_multi on this context as shard 0: RCCL communicators over the
    // member devices (one per member, cached while the device list is the
    // same), the gather buffer and the device film
    std::vector<int> comm_devs;
    std::vector<ncclComm_t> comms;
    float *gather = nullptr; size_t gather_bytes = 0;
    float *film_dev = nullptr; size_t film_dev_bytes = 0;
};

// ---- launch plans ----
// Shared by the two translation units of the library: this file, and
// frt_render_mats.hip, which includes it with FRT_TU_MATS defined and holds
// every kernel compiled with a material set (MATS != kMatsNone: the path
// kernels of specular / textured scenes, AO, the fp64 kernels of such scenes,
// PSS-MLT on them).  That unit is compiled with the basic SGPR register
// allocator (Makefile): under the default greedy allocator these kernels
// have given the oracle's ray counts with wrong radiance at some register
// caps, in every failing source state on record, and the basic SGPR (or
// VGPR) allocator removed every such failure at an equal or larger spill
// count (DESIGN.md "Register-cap hazard").  The lambertian kernels (the
// bench configurations) stay on the greedy allocator.
static bool bvh4_stack_fits(int depth4, int lds_entries) { return 3 * depth4 <= lds_entries + kBvh4Overflow; }
struct Launcher {
    const void *fn = nullptr;
    size_t lds = 0;
    int stack = 0;
    int waves = 0;
    bool lds_scene = false;
    bool wide = false;      // 4-wide quantized BVH
    bool f64 = false;       // the fp64 kernel
    size_t scene_lds = 0;   // scene bytes the plan loads into LDS (octant copies or planar tree), 0 = HBM
};
template <int STACK, int WORLD, bool LDS, int WAVES = 1, int MATS = kMatsNone,
          int KIND = FRT_INTEGRATOR_PATH, typename R = float>
static Launcher make_launcher(size_t scene_bytes)
{
    Launcher L;
    L.fn = reinterpret_cast<const void *>(&path_megakernel<STACK, WORLD, LDS, WAVES, MATS, KIND, R>);
    L.f64 = kIsF64<R>;
    L.lds = (WORLD != FRT_WORLD_LIST ? (size_t)STACK * kBlock * sizeof(int) : 0) +
            (size_t)kItemWords * kBlock * sizeof(int) + (LDS ? scene_bytes : 0);
    L.scene_lds = LDS ? scene_bytes : 0;
    L.stack = STACK;
    L.waves = WAVES > 1 ? WAVES : 0;
    L.lds_scene = LDS;
    L.wide = WORLD == kWorldBvh4;
    return L;
}
#ifndef FRT_EXP_W6
#define FRT_EXP_W6 6   // experiment builds: the register cap behind the "6 waves" plans
#endif
#ifndef FRT_EXP_W7
#define FRT_EXP_W7 7   // experiment builds: the register cap behind the 4-wide "7 waves" plan
#endif
template <int STACK, bool LDS, int WORLD = FRT_WORLD_BVH, int MATS = kMatsNone>
static Launcher bvh_launcher(int waves, size_t sb)
{
    // Every material set has a 6-wave build again (round 3).  Under the greedy
    // register allocator the material kernels have compiled, at some caps, to
    // kernels with the oracle's ray counts and wrong radiance; they now come
    // from frt_render_mats.hip, built with the basic SGPR allocator, which
    // removed every such failure on record (DESIGN.md "Register-cap hazard";
    // test_register_caps_agree checks every cap and plan).  The defaults stay
    // 4 / 5 waves for the specular sets (faster than 6:
    // profiles/r02/r02_ab_sphere_hbm_mats.jsonl).
    if constexpr (MATS == kMatsNone && WORLD == kWorldBvh4)   // the lambertian 4-wide HBM plan (round 5)
        if (waves == 7) return make_launcher<STACK, WORLD, LDS, FRT_EXP_W7, MATS>(sb);
    if (waves == 6) return make_launcher<STACK, WORLD, LDS, FRT_EXP_W6, MATS>(sb);
    if (waves == 5) return make_launcher<STACK, WORLD, LDS, 5, MATS>(sb);
    if constexpr (MATS != kMatsNone) {
        if (waves == 4) return make_launcher<STACK, WORLD, LDS, 4, MATS>(sb);
        if (waves == 3) return make_launcher<STACK, WORLD, LDS, 3, MATS>(sb);
    }
    return make_launcher<STACK, WORLD, LDS, 1, MATS>(sb);
}
#ifndef FRT_EXP_BVH4_LSTACK
#define FRT_EXP_BVH4_LSTACK 12
#endif
// LDS entries of the 4-wide stack; deeper ones go to scratch.  12 since round 5
// (was 16): 12 KiB of stack + 10 KiB of item state a block let 7 blocks share a
// CU's 160 KiB, and the lambertian 4-wide kernel runs 7 waves/SIMD (72 VGPRs,
// no spills since the SLP vectorizer is off): cornell_1m 360.3 -> 344.3 ms
// (+4.6 %, same call, profiles/r05/r05i/ab_m.jsonl)
constexpr int kBvh4LdsStack = FRT_EXP_BVH4_LSTACK;
// Two more units for the lambertian kernels of the octant LDS plan, each under
// the machine scheduling strategy that measured fastest for it (same call, two
// alternations): frt_render_lds.hip holds the path kernels (C2) under
// max-memory-clause (Makefile LDSFLAGS; Cornell 229.4 / 229.7 -> 227.5 / 227.5
// ms, profiles/r06/r06f), frt_render_chain.hip the PSS-MLT chain kernels (C5)
// under iterative-maxocc (CHAINFLAGS; 576.8 / 576.1 -> 570.6 / 571.6 ms against
// max-memory-clause, profiles/r06/r06h).  The 4-wide HBM kernel (cornell_1m)
// loses under every other strategy (max-memory-clause 1.6 %, iterative ones
// 9-26 %), so it stays in the main unit on the default one.  Diagnostic builds
// (FRT_DIAG: their counters are a device global of the main unit) keep these
// kernels in the main unit.
#if (defined(FRT_DIAG) && !defined(FRT_TU_LDS) && !defined(FRT_TU_CHAIN)) || defined(FRT_EXP_NO_LDS_SPLIT)
constexpr bool kSplitLds = false;
#else
constexpr bool kSplitLds = true;
#endif
namespace frt_lds {
int path_oct(int stack, int waves, size_t scene_bytes, Launcher &L);
int mlt_oct(int stack, const void **boot, const void **chains);
}  // namespace frt_lds

// MATS: the material set the kernel is compiled for (kMats* mask, frt_path.hpp)
template <int MATS>
static int pick_launcher_t(const frt_ctx *c, int flags, Launcher &L)
{
    if (c->world_kind == FRT_WORLD_LIST) { L = make_launcher<16, FRT_WORLD_LIST, false, 1, MATS>(0); return FRT_OK; }
    const int d = c->stack_needed;
    const size_t sb = c->scene_lds_bytes;
    const bool lds = d < kLdsMaxDepth && sb <= kLdsSceneBytes && !(flags & FRT_FLAG_NO_LDS_SCENE);
    // register cap: waves/SIMD the compiler must fit (its spills land in the
    // shading code, not the traversal loops).  Measured (profiles/r01_ab_perf3.jsonl):
    // 5 waves best for LDS-resident scenes, 6 for HBM-resident ones.  The
    // material kernels (MATS) in LDS run 15-21 % faster on the compiler's own
    // allocation than under the 5-wave cap (profiles/r01d_perf_mats.jsonl).
    // Material kernels: textures alone cost about the lambertian kernel's
    // registers (117 vs 111 VGPRs uncapped; the compiler's 4 waves are best),
    // the specular branch 152, the rough conductor lobes 170 -- capped at 4
    // waves/SIMD (128 VGPRs; a few spills in the specular shading) they run
    // +40 % over the compiler's 2-wave allocation (same-call A/B,
    // profiles/r02/r02_mats*.jsonl).
    // (The lambertian LDS kernel fits 111 VGPRs without spills since its work-
    // item state moved to LDS; the compiler's 4 waves win 2 % at 64 spp but lose
    // 10 % at the bench's 512 spp -- 337 vs 307 ms, same call --, so the cap stays:
    // profiles/r02/r02_ab_cornell_knobs.jsonl, r02_ab_cornell_512spp.jsonl.)
    int waves = (MATS & kMatsSpecAny) ? (lds ? 4 : 5) : MATS == kMatsTex && lds ? 0 : lds ? 5 : 6;
    // the lambertian 4-wide HBM plan: 7 waves (round 5; the binary HBM fallback keeps 6)
    const bool wide = !lds && c->has_bvh4 && !(flags & FRT_FLAG_BVH2) && bvh4_stack_fits(c->depth4, kBvh4LdsStack);
    if (MATS == kMatsNone && wide) waves = 7;
    if constexpr (MATS != kMatsNone) {   // FRT_MATS_WAVES: register cap of the material kernels (tuning knob, not part of the C-ABI)
        const char *e = std::getenv("FRT_MATS_WAVES");
        if (e) waves = std::atoi(e);
    }
    if (flags & FRT_FLAG_WAVES4) waves = 0;   // the compiler's own allocation (~120 VGPRs, 4 waves)
    if (flags & FRT_FLAG_WAVES5) waves = 5;
    if (flags & FRT_FLAG_WAVES6) waves = 6;
    // (Measured and removed A/B plans, DESIGN.md section 5: lockstep brute force over tiny
    // scenes, 4-wide nodes from LDS, speculative traversal, an 8-wide HBM tree.)
    // HBM-resident scenes: the 4-wide quantized BVH (half the bytes per box test)
    if (wide) {
        L = bvh_launcher<kBvh4LdsStack, false, kWorldBvh4, MATS>(waves, 0);
        return FRT_OK;
    }
    // LDS-resident binary tree: the per-octant node copies when they fit
    const bool oct = lds && !(flags & FRT_FLAG_NO_OCT) && c->scene_lds_bytes_oct <= kLdsOctBytes;
    if (oct) {
        if constexpr (MATS == kMatsNone && kSplitLds) {   // the third unit's kernels (frt_lds)
            return frt_lds::path_oct(d < 8 ? 8 : 16, waves, c->scene_lds_bytes_oct, L);
        } else {
            L = d < 8 ? bvh_launcher<8, true, kWorldBvh2Oct, MATS>(waves, c->scene_lds_bytes_oct)
                      : bvh_launcher<16, true, kWorldBvh2Oct, MATS>(waves, c->scene_lds_bytes_oct);
            return FRT_OK;
        }
    }
    if (d < 8) L = lds ? bvh_launcher<8, true, FRT_WORLD_BVH, MATS>(waves, sb)
                       : bvh_launcher<8, false, FRT_WORLD_BVH, MATS>(waves, 0);
    else if (d < 16) L = lds ? bvh_launcher<16, true, FRT_WORLD_BVH, MATS>(waves, sb)
                             : bvh_launcher<16, false, FRT_WORLD_BVH, MATS>(waves, 0);
    else if (d < 24) L = bvh_launcher<24, false, FRT_WORLD_BVH, MATS>(waves, 0);
    else if (d < 32) L = bvh_launcher<32, false, FRT_WORLD_BVH, MATS>(waves, 0);
    else if (d < 64) L = make_launcher<64, FRT_WORLD_BVH, false, 1, MATS>(0);
    else return FRT_E_UNSUPPORTED;
    return FRT_OK;
}
// AO / normals: the default plans only (LDS-resident binary BVH, HBM 4-wide or
// binary), register caps as for path; ao keeps the specular generate() code.
template <int KIND>
static int pick_launcher_kind(const frt_ctx *c, int flags, Launcher &L)
{
    constexpr int M = KIND == FRT_INTEGRATOR_AO ? kMatsAll : kMatsNone;
    if (c->world_kind == FRT_WORLD_LIST) { L = make_launcher<16, FRT_WORLD_LIST, false, 1, M, KIND>(0); return FRT_OK; }
    const int d = c->stack_needed;
    const size_t sb = c->scene_lds_bytes;
    const bool lds = d < kLdsMaxDepth && sb <= kLdsSceneBytes && !(flags & FRT_FLAG_NO_LDS_SCENE);
    const bool oct = lds && !(flags & FRT_FLAG_NO_OCT) && c->scene_lds_bytes_oct <= kLdsOctBytes;
    if (oct) {
        L = d < 8 ? make_launcher<8, kWorldBvh2Oct, true, 5, M, KIND>(c->scene_lds_bytes_oct)
                  : make_launcher<16, kWorldBvh2Oct, true, 5, M, KIND>(c->scene_lds_bytes_oct);
    } else if (lds) {
        L = d < 8 ? make_launcher<8, FRT_WORLD_BVH, true, 5, M, KIND>(sb)
                  : make_launcher<16, FRT_WORLD_BVH, true, 5, M, KIND>(sb);
    } else if (c->has_bvh4 && !(flags & FRT_FLAG_BVH2) && bvh4_stack_fits(c->depth4, kBvh4LdsStack)) {
        L = make_launcher<kBvh4LdsStack, kWorldBvh4, false, 6, M, KIND>(0);
    } else if (d < 16) {
        L = make_launcher<16, FRT_WORLD_BVH, false, 6, M, KIND>(0);
    } else if (d < 32) {
        L = make_launcher<32, FRT_WORLD_BVH, false, 6, M, KIND>(0);
    } else if (d < 64) {
        L = make_launcher<64, FRT_WORLD_BVH, false, 1, M, KIND>(0);
    } else {
        return FRT_E_UNSUPPORTED;
    }
    return FRT_OK;
}
// fp64 kernels (path only; DESIGN.md "Precision"): the list world with the
// scene's material set, or the binary tree from HBM with every material
// compiled in (the debugging build; no register cap, stack 32 or 64)
#ifndef FRT_EXP_F64_LIST_WAVES
#define FRT_EXP_F64_LIST_WAVES 1   // experiment builds: register cap of the fp64 list kernels (1 = the compiler's own)
#endif
template <int MATS>
static int pick_launcher_f64_t(const frt_ctx *c, Launcher &L)
{
    if (c->world_kind == FRT_WORLD_LIST) {
        // (a 2-wave register cap changed nothing: profiles/r03/r03c_ab_veach_listbox_f64waves.jsonl)
        L = make_launcher<16, FRT_WORLD_LIST, false, FRT_EXP_F64_LIST_WAVES, MATS, FRT_INTEGRATOR_PATH, double>(0);
        return FRT_OK;
    }
    const int d = c->stack_needed;
    if (d < 32) L = make_launcher<32, FRT_WORLD_BVH, false, 1, kMatsAll, FRT_INTEGRATOR_PATH, double>(0);
    else if (d < 64) L = make_launcher<64, FRT_WORLD_BVH, false, 1, kMatsAll, FRT_INTEGRATOR_PATH, double>(0);
    else return FRT_E_UNSUPPORTED;
    return FRT_OK;
}
template <int STACK, int WORLD, bool LDS, bool MATS>
static void mlt_kernels_t(const void **boot, const void **chains)
{
    *boot = reinterpret_cast<const void *>(&mlt_bootstrap<STACK, WORLD, MATS>);
    *chains = reinterpret_cast<const void *>(&mlt_megakernel<STACK, WORLD, LDS, MATS>);
}

// the material unit's entry points (frt_render_mats.hip)
namespace frt_mats {
// path (KIND = FRT_INTEGRATOR_PATH, fp32), fp64 path (f64) or AO: the plan for
// the scene's material set c->mats (!= kMatsNone)
int pick(const frt_ctx *c, int integrator, int flags, bool f64, Launcher &L);
// PSS-MLT with the material branch, for the (stack, world, lds) plans of render_mlt
int mlt(int stack, int world, bool lds, const void **boot, const void **chains);
}  // namespace frt_mats

#if defined(FRT_TU_LDS)
int frt_lds::path_oct(int stack, int waves, size_t scene_bytes, Launcher &L)
{
    if (stack == 8) L = bvh_launcher<8, true, kWorldBvh2Oct, kMatsNone>(waves, scene_bytes);
    else if (stack == 16) L = bvh_launcher<16, true, kWorldBvh2Oct, kMatsNone>(waves, scene_bytes);
    else return FRT_E_UNSUPPORTED;
    return FRT_OK;
}
#elif defined(FRT_TU_CHAIN)
int frt_lds::mlt_oct(int stack, const void **boot, const void **chains)
{
    if (stack == 8) mlt_kernels_t<8, kWorldBvh2Oct, true, false>(boot, chains);
    else if (stack == 16) mlt_kernels_t<16, kWorldBvh2Oct, true, false>(boot, chains);
    else return FRT_E_UNSUPPORTED;
    return FRT_OK;
}
#elif defined(FRT_TU_MATS)
int frt_mats::pick(const frt_ctx *c, int integrator, int flags, bool f64, Launcher &L)
{
    if (integrator == FRT_INTEGRATOR_AO) return pick_launcher_kind<FRT_INTEGRATOR_AO>(c, flags, L);
    if (f64) {
        switch (c->mats) {
        case kMatsNone: return pick_launcher_f64_t<kMatsNone>(c, L);   // BVH worlds: kMatsAll kernels
        case kMatsTex: return pick_launcher_f64_t<kMatsTex>(c, L);
        case kMatsSpec: return pick_launcher_f64_t<kMatsSpec>(c, L);   // veach_mis (C3): phong plates
        case kMatsSpec | kMatsTex: return pick_launcher_f64_t<kMatsSpec | kMatsTex>(c, L);
        default: return pick_launcher_f64_t<kMatsAll>(c, L);
        }
    }
    switch (c->mats) {   // the smallest kernel covering the scene's materials
    case kMatsTex: return pick_launcher_t<kMatsTex>(c, flags, L);
    case kMatsSpec:
    case kMatsSpec | kMatsTex: return pick_launcher_t<kMatsSpec | kMatsTex>(c, flags, L);
    default: return pick_launcher_t<kMatsAll>(c, flags, L);
    }
}
int frt_mats::mlt(int stack, int world, bool lds, const void **boot, const void **chains)
{
    if (world == FRT_WORLD_LIST) mlt_kernels_t<16, FRT_WORLD_LIST, false, true>(boot, chains);
    else if (world == kWorldBvh4) mlt_kernels_t<kBvh4LdsStack, kWorldBvh4, false, true>(boot, chains);
    else if (world == kWorldBvh2Oct && stack == 8) mlt_kernels_t<8, kWorldBvh2Oct, true, true>(boot, chains);
    else if (world == kWorldBvh2Oct && stack == 16) mlt_kernels_t<16, kWorldBvh2Oct, true, true>(boot, chains);
    else if (lds && stack == 8) mlt_kernels_t<8, FRT_WORLD_BVH, true, true>(boot, chains);
    else if (lds && stack == 16) mlt_kernels_t<16, FRT_WORLD_BVH, true, true>(boot, chains);
    else if (!lds && stack == 16) mlt_kernels_t<16, FRT_WORLD_BVH, false, true>(boot, chains);
    else if (!lds && stack == 32) mlt_kernels_t<32, FRT_WORLD_BVH, false, true>(boot, chains);
    else if (!lds && stack == 64) mlt_kernels_t<64, FRT_WORLD_BVH, false, true>(boot, chains);
    else return FRT_E_UNSUPPORTED;
    return FRT_OK;
}
#else   // the main unit: everything else


static void free_comms(frt_ctx *c)
{
    for (ncclComm_t m : c->comms) (void)ncclCommDestroy(m);
    c->comms.clear();
    c->comm_devs.clear();
}

static int set_err(frt_ctx *c, int code, const std::string &m)
{
    if (c) c->err = m;
    return code;
}
#define HIPCHK(ctx, x)                                                                             \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess)                                                                      \
            return set_err(ctx, FRT_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_));       \
    } while (0)

extern "C" int frt_get_abi_version(void) { return FRT_ABI_VERSION; }

extern "C" int frt_create(int hip_device, frt_ctx **out)
{
    if (!out) return FRT_E_INVALID;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return FRT_E_NO_DEVICE;
    if (hip_device < 0 || hip_device >= n) return FRT_E_NO_DEVICE;
    frt_ctx *c = new frt_ctx();
    c->device = hip_device;
    if (hipSetDevice(hip_device) != hipSuccess) { delete c; return FRT_E_HIP; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, hip_device) != hipSuccess) { delete c; return FRT_E_HIP; }
    if (std::string(prop.gcnArchName).rfind("gfx950", 0) != 0) {
        fprintf(stderr, "frt: device %d is %s, not gfx950\n", hip_device, prop.gcnArchName);
        delete c;
        return FRT_E_NO_DEVICE;
    }
    c->n_cu = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipMalloc(&c->counter, kCounterBytes) != hipSuccess) {
        delete c;
        return FRT_E_HIP;
    }
    *out = c;
    return FRT_OK;
}

static void free_scene(frt_ctx *c)
{
    for (void *p : c->scene_bufs) (void)hipFree(p);
    c->scene_bufs.clear();
    c->have_scene = false;
}

extern "C" int frt_destroy(frt_ctx *c)
{
    if (!c) return FRT_E_INVALID;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    free_scene(c);
    if (c->partial) (void)hipFree(c->partial);
    if (c->counter) (void)hipFree(c->counter);
    if (c->wave_rays) (void)hipFree(c->wave_rays);
    if (c->slots_out) (void)hipFree(c->slots_out);
    if (c->splat) (void)hipFree(c->splat);
    free_comms(c);
    if (c->gather) (void)hipFree(c->gather);
    if (c->film_dev) (void)hipFree(c->film_dev);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return FRT_OK;
}

extern "C" const char *frt_last_error(const frt_ctx *c) { return c ? c->err.c_str() : "null context"; }

// Precision of the context's kernels (DESIGN.md "Precision"): read by the
// next frt_upload_scene (which then also uploads the fp64 records) and by
// every render.
extern "C" int frt_set_precision(frt_ctx *c, int precision)
{
    if (!c) return FRT_E_INVALID;
    if (precision != FRT_PRECISION_AUTO && precision != FRT_PRECISION_FP32 && precision != FRT_PRECISION_FP64)
        return set_err(c, FRT_E_INVALID, "precision must be FRT_PRECISION_AUTO, _FP32 or _FP64");
    c->precision = precision;
    return FRT_OK;
}

// GPU BVH build on this context's device and stream (frt_lbvh.hip); called
// by frt_scene_build_bvh_gpu (csrc/host/scene.cpp).  Internal to libfrt.so.
extern "C" int frt_internal_lbvh(frt_ctx *c, int n, const float *box6, int32_t *child2, float *node_box6,
                                 int32_t *order, double *ms, int algo)
{
    if (!c || n < 2 || !box6 || !child2 || !node_box6 || !order) return FRT_E_INVALID;
    if (algo != FRT_GPU_BVH_PLOC && algo != FRT_GPU_BVH_LBVH && algo != FRT_GPU_BVH_SAH)
        return set_err(c, FRT_E_INVALID, "unknown GPU BVH builder");
    HIPCHK(c, hipSetDevice(c->device));
    float dev_ms = 0.0f;
    std::string err;
    if (frt::lbvh_build(c->stream, n, box6, child2, node_box6, order, &dev_ms, err,
                        algo == FRT_GPU_BVH_LBVH ? frt::kGpuBvhLbvh
                        : algo == FRT_GPU_BVH_SAH ? frt::kGpuBvhSah : frt::kGpuBvhPloc) != 0)
        return set_err(c, FRT_E_HIP, err);
    if (ms) *ms = dev_ms;
    return FRT_OK;
}

// ---- scene flattening: DFS order, fp32 conversion with outward-rounded boxes ----
static inline float round_down(double x)
{
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
}
static inline float round_up(double x)
{
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}

// host image of the device scene (DESIGN.md "Data layout")
struct FlatScene {
    std::vector<float4> nodes, tris, tshade, tnorm, spheres, mats, tuv;
    std::vector<float4> texels;   // image_texture texels (rgb, -), all images back to back
    std::vector<uint4> nodes4;   // 4-wide quantized BVH
    std::vector<float4> nodes_oct;   // 8 octant copies of `nodes` (DevScene::nodes_oct), LDS plan scenes only
    std::vector<double4> tris64, tshade64, tnorm64, spheres64;   // fp64 records (DevScene::tris64 ...)
    bool has4 = false;           // nodes4 / root4 usable
    int root4 = 0, depth4 = 0;
    std::vector<int> smat, lights, list;
    std::vector<int> tri_view;      // device triangle id -> scene-view triangle (DevScene::tri_view)
    DevScene meta{};     // scalars + camera; pointers filled by the consumer
    int depth = 0;
};

// Shading starts when at most this many lanes of a wave still traverse
// (0 = every ray of the wave finishes first).  Per plan and integrator, at the
// bench's 1080p / 512 spp (same call, profiles/r02/r02_ab_trav_min_512spp.txt):
// path 28 from LDS (Cornell 308.0 -> 301.4 ms; 12 was round 1's 64-spp
// optimum, profiles/r01_ab_perf6.jsonl) and 40 from HBM (cornell_1m 863.5 ->
// 857.3 ms); PSS-MLT and AO keep 12 / 32 (28 costs them 4-5 %).  Round 4's
// cheaper LDS node loop moved the LDS path optimum to 20 (Cornell 245.3 ->
// 242.5 ms; 16 / 24: 243.4 / 243.7; profiles/r04/r04{h,i}/ab_*.jsonl).
// FRT_TRAV_MIN overrides (tuning knob of this library, not part of the C-ABI).
static int trav_min(bool lds_scene, bool path = false)
{
    const char *e = std::getenv("FRT_TRAV_MIN");
    const int v = e ? std::atoi(e)
                    : path ? (lds_scene ? kTravMinLdsPath : kTravMinHbmPath) : (lds_scene ? kTravMinLds : kTravMinHbm);
    return std::min(std::max(v, 0), 63);
}

// Leaf postponing (bvh2_step): a wave's descent stops once fewer than this
// many of its lanes still descend.  0 = every lane reaches its leaf first.
// HBM plans 12 since round 4 (cornell_1m 512 spp 767.5 -> 760.9 ms over 8, 16:
// 761.6, same call, profiles/r04/r04n; confirmed 765.4 -> 759.2 in r04o).
// FRT_MIN_DESC overrides (tuning knob, not part of the C-ABI).
static int min_desc(bool lds_scene)
{
    const char *e = std::getenv("FRT_MIN_DESC");
    const int v = e ? std::atoi(e) : (lds_scene ? kMinDescLds : kMinDescHbm);
    return std::min(std::max(v, 0), 64);
}

// Triangles per leaf: FRT_LEAF_SIZE overrides (1 = the reference's one-prim
// leaves), else 0 = by plan (see flatten_scene).  A tuning knob of this
// library, not part of the C-ABI.
static int leaf_size_override()
{
    const char *e = std::getenv("FRT_LEAF_SIZE");
    return e ? std::min(std::max(std::atoi(e), 1), kLeafMax) : 0;
}

// Multi-triangle leaves: every subtree of the DFS-ordered binary tree holding
// only triangles, at most `leaf_max` of them, becomes one leaf.  Its triangles
// are the contiguous device ids [first, first + count) (device id = DFS rank).
// The closest hit over triangles is the lexicographic minimum of (t, DFS rank)
// whatever the visit order (the tie rule in trace_bvh), and the parent's box
// already bounds the subtree, so hits are unchanged -- only node visits drop.
static void collapse_leaves(FlatScene &F, int leaf_max)
{
    const int nn = (int)(F.nodes.size() / 4);
    if (leaf_max <= 1 || nn == 0) return;
    auto child = [&](int i, int side) { return f2i(side ? F.nodes[4 * i + 3].y : F.nodes[4 * i + 3].x); };
    // subtree triangle count / first device id / holds a sphere; children follow parents in pre-order
    std::vector<int> cnt(nn, 0), first(nn, INT32_MAX);
    std::vector<char> sph(nn, 0);
    for (int i = nn - 1; i >= 0; --i)
        for (int side = 0; side < 2; ++side) {
            const int c = child(i, side);
            if (c >= 0) {
                cnt[i] += cnt[c]; first[i] = std::min(first[i], first[c]); sph[i] |= sph[c];
            } else if (~c & FRT_PRIM_SPHERE) {
                sph[i] = 1;
            } else {
                cnt[i] += 1; first[i] = std::min(first[i], ~c);
            }
        }
    std::vector<float4> out;
    out.reserve(F.nodes.size());
    int depth = 0;
    // pre-order rebuild; (old node, slot in `out` of the parent's child ref or -1, level)
    struct Item { int old, parent_slot, side, lvl; };
    std::vector<Item> st{{0, -1, 0, 1}};
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        const int me = (int)(out.size() / 4);
        if (it.parent_slot >= 0) {
            float4 &r = out[it.parent_slot];
            (it.side ? r.y : r.x) = i2f(me);
        }
        depth = std::max(depth, it.lvl);
        for (int k = 0; k < 4; ++k) out.push_back(F.nodes[4 * it.old + k]);
        const int slot = 4 * me + 3;
        for (int side = 1; side >= 0; --side) {
            const int c = child(it.old, side);
            if (c < 0) continue;                                  // leaf ref kept as is
            if (!sph[c] && cnt[c] <= leaf_max) {
                float4 &r = out[slot];
                (side ? r.y : r.x) = i2f(~(first[c] | ((cnt[c] - 1) << kLeafCountShift)));
            } else {
                st.push_back({c, slot, side, it.lvl + 1});
            }
        }
    }
    F.nodes.swap(out);
    F.depth = depth;
}

// 4-wide quantized BVH (DESIGN.md "BVH4Q") from the binary tree after
// collapse_leaves: each 4-wide node takes the descendants of its binary node
// that minimise the summed box area of the 4-wide nodes below it (an exact
// dynamic programme over the binary tree, after Ylitie, Karras & Laine 2017;
// round 5, replacing "open the interior child of largest area until four":
// cornell_1m +0.4 %, 23 % fewer nodes).  Child boxes are the binary tree's padded fp32 boxes quantized to 8
// bits per plane on a per-node power-of-two grid, rounded outward.  Nodes in
// depth-first pre-order (a node's first interior child follows it; sibling
// blocks and a breadth-first order measured the same).
// Returns false (no BVH4; the binary tree is used) when a node's grid would
// overflow the slab arithmetic.
static bool build_bvh4(FlatScene &F, int root_ref)
{
    F.nodes4.clear();
    F.depth4 = 0;
    F.root4 = root_ref;
    const int nn = (int)(F.nodes.size() / 4);
    if (nn == 0 || root_ref < 0) return true;
    struct Child { float lo[3], hi[3]; int ref; };
    auto kids = [&](int i, Child *out) {
        const float4 a = F.nodes[4 * i], b = F.nodes[4 * i + 1], c = F.nodes[4 * i + 2], r = F.nodes[4 * i + 3];
        out[0] = Child{{a.x, a.y, a.z}, {a.w, b.x, b.y}, f2i(r.x)};
        out[1] = Child{{b.z, b.w, c.x}, {c.y, c.z, c.w}, f2i(r.y)};
    };
    auto area = [](const Child &c) {
        const double dx = (double)c.hi[0] - c.lo[0], dy = (double)c.hi[1] - c.lo[1], dz = (double)c.hi[2] - c.lo[2];
        return dx * dy + dy * dz + dz * dx;
    };
    // empty slots: the inverted box q_lo = 255 > q_hi = 0 on every axis,
    // which the near / far slab test rejects -- except on a node so small
    // against its distance from the ray origin that each axis' planes round
    // to one value (then a real child's hit has tn == tf and must stay a hit,
    // so the test cannot reject it either; ADVICE r2,
    // test_bvh4_tiny_far_nodes).  Their ref is a one-primitive leaf of the
    // scene's first primitive: a spurious visit re-tests a real primitive,
    // which cannot change a closest hit (same t, same DFS rank) or an any-hit
    // answer, and needs no per-child ref compare in the node loop (that
    // compare cost 2 % on cornell_1m).
    const uint32_t empty_ref = (uint32_t)~(F.tris.empty() ? FRT_PRIM_SPHERE : 0);
    // Area-optimal collapse: per binary node n, T[n] = the summed box area of the
    // 4-wide nodes that represent n's subtree when n takes one slot (n becomes a
    // node), D[n][j] the least such sum when n's subtree fills at most j slots of
    // its parent (n opened); the leaves are fixed, so the sum of node areas is
    // the whole SAH difference between two collapses.  Children follow parents
    // in pre-order, so one backward sweep fills the tables.
    std::vector<double> T(nn, 0.0), D(5 * (size_t)nn, 0.0);
    std::vector<signed char> split(5 * (size_t)nn, 1);
    auto slot_cost = [&](const Child &c, int k) {   // c in at most k slots
        if (c.ref < 0) return 0.0;
        return k >= 2 ? std::min(T[c.ref], D[5 * (size_t)c.ref + k]) : T[c.ref];
    };
    {
        std::vector<double> own(nn, 0.0);   // a node's own box area, from its parent's record
        for (int i = 0; i < nn; ++i) {
            Child two[2];
            kids(i, two);
            for (int s = 0; s < 2; ++s) if (two[s].ref >= 0) own[two[s].ref] = area(two[s]);
        }
        for (int i = nn - 1; i >= 0; --i) {
            Child two[2];
            kids(i, two);
            for (int j = 2; j <= 4; ++j) {
                double best = 1e300;
                for (int k = 1; k < j; ++k) {
                    const double v = slot_cost(two[0], k) + slot_cost(two[1], j - k);
                    if (v < best) { best = v; split[5 * (size_t)i + j] = (signed char)k; }
                }
                D[5 * (size_t)i + j] = best;
            }
            T[i] = own[i] + D[5 * (size_t)i + 4];
        }
    }
    std::function<void(const Child &, int, Child *, int &)> gather = [&](const Child &c, int k, Child *out, int &n) {
        if (c.ref < 0 || k < 2 || !(D[5 * (size_t)c.ref + k] < T[c.ref])) { out[n++] = c; return; }
        Child two[2];
        kids(c.ref, two);
        const int kl = split[5 * (size_t)c.ref + k];
        gather(two[0], kl, out, n);
        gather(two[1], k - kl, out, n);
    };
    struct Item { int bin, parent, slot, lvl; };   // binary node, wide parent (-1 root), child slot, level
    std::vector<Item> st{{root_ref, -1, 0, 1}};
    while (!st.empty()) {
        const Item it = st.back();
        st.pop_back();
        const int me = (int)(F.nodes4.size() / kNode4Parts);
        if (it.parent >= 0) {
            uint4 &r = F.nodes4[(size_t)kNode4Parts * it.parent + 1];
            (it.slot == 0 ? r.x : it.slot == 1 ? r.y : it.slot == 2 ? r.z : r.w) = (uint32_t)me;
        }
        F.depth4 = std::max(F.depth4, it.lvl);
        Child ch[4], two[2];   // slots in left-to-right order
        int n = 0;
        kids(it.bin, two);
        const int kl = split[5 * (size_t)it.bin + 4];
        gather(two[0], kl, ch, n);
        gather(two[1], 4 - kl, ch, n);
        // per-axis grid: origin = min child lo, step 2^e with every plane within 255 steps
        float org[3];
        int ex[3];
        uint32_t qlo[3] = {0, 0, 0}, qhi[3] = {0, 0, 0};
        for (int a = 0; a < 3; ++a) {
            float lo = ch[0].lo[a], hi = ch[0].hi[a];
            for (int k = 1; k < n; ++k) { lo = std::min(lo, ch[k].lo[a]); hi = std::max(hi, ch[k].hi[a]); }
            org[a] = lo;
            const double ext = (double)hi - (double)lo;
            int e = -126;
            if (ext > 0.0) {
                std::frexp(ext / 255.0, &e);            // ext / 255 <= 2^e
                e = std::max(e, -126);
                while (e > -126 && std::ldexp(255.0, e - 1) >= ext) --e;
            }
            if (e > 20) return false;                  // 2^e / |d| must stay finite (|1/d| <= 1e30)
            if (e < -100) return false;                // 2^e / |d| must stay a normal float for the empty-slot
                                                       // test (padded boxes are never this thin)
            ex[a] = e;
            for (int s = 0; s < 4; ++s) {
                double ql = 255.0, qh = 0.0;           // empty slot: the inverted box
                if (s < n) {
                    const Child &c = ch[s];
                    ql = std::floor(((double)c.lo[a] - lo) / std::ldexp(1.0, e));
                    qh = std::ceil(((double)c.hi[a] - lo) / std::ldexp(1.0, e));
                    ql = std::min(std::max(ql, 0.0), 255.0);
                    qh = std::min(std::max(qh, 0.0), 255.0);
                    // outward: the decoded plane must enclose the fp32 box (exact in double)
                    while (ql > 0.0 && (double)lo + ql * std::ldexp(1.0, e) > (double)c.lo[a]) ql -= 1.0;
                    while (qh < 255.0 && (double)lo + qh * std::ldexp(1.0, e) < (double)c.hi[a]) qh += 1.0;
                }
                qlo[a] |= (uint32_t)ql << (8 * s);
                qhi[a] |= (uint32_t)qh << (8 * s);
            }
        }
        uint32_t refs[4];
        for (int s = 0; s < 4; ++s) refs[s] = s < n ? (uint32_t)ch[s].ref : empty_ref;
        F.nodes4.resize((size_t)(me + 1) * kNode4Parts);
        uint4 *out = F.nodes4.data() + (size_t)me * kNode4Parts;
        out[0] = make_uint4((uint32_t)f2i(org[0]), (uint32_t)f2i(org[1]), (uint32_t)f2i(org[2]),
                            ((uint32_t)ex[0] & 0xffu) | (((uint32_t)ex[1] & 0xffu) << 8) | (((uint32_t)ex[2] & 0xffu) << 16));
        out[1] = make_uint4(refs[0], refs[1], refs[2], refs[3]);
        out[2] = make_uint4(qlo[0], qhi[0], qlo[1], qhi[1]);
        out[3] = make_uint4(qlo[2], qhi[2], 0u, 0u);
        for (int s = n - 1; s >= 0; --s)               // pre-order: the first slot next
            if (ch[s].ref >= 0) st.push_back({ch[s].ref, me, s, it.lvl + 1});
    }
    F.root4 = 0;
    return true;
}

// f64: also build the fp64 records of the fp64 kernels (DESIGN.md "Precision")
static int flatten_scene(const frt_scene_view *sv, FlatScene &F, std::string &err, bool f64)
{
    auto fail = [&](int code, const std::string &m) { err = m; return code; };
    const int nt = sv->n_tris, ns = sv->n_spheres, nm = sv->n_materials;
    if (nt < 0 || ns < 0 || nm <= 0 || !sv->materials || (nt > 0 && (!sv->tri_v || !sv->tri_material || !sv->tri_inv_area)))
        return fail(FRT_E_INVALID, "scene view: missing triangle arrays or materials");
    if (ns > 0 && (!sv->sphere || !sv->sphere_material)) return fail(FRT_E_INVALID, "scene view: missing sphere arrays");
    for (int i = 0; i < nm; ++i) {
        const int t = sv->materials[i].type;
        if (t != FRT_MAT_LAMBERTIAN && t != FRT_MAT_DIFFUSE_LIGHT && t != FRT_MAT_MODIFIED_PHONG &&
            t != FRT_MAT_METAL && t != FRT_MAT_DIELECTRIC && t != FRT_MAT_ROUGH_CONDUCTOR)
            return fail(FRT_E_UNSUPPORTED, "material type " + std::to_string(t) + " is not supported");
        const int tex = sv->materials[i].texture;
        if (tex != FRT_TEX_CONSTANT && tex != FRT_TEX_CHECKER && tex != FRT_TEX_IMAGE)
            return fail(FRT_E_INVALID, "material texture must be FRT_TEX_CONSTANT, FRT_TEX_CHECKER or FRT_TEX_IMAGE");
        if (tex != FRT_TEX_CONSTANT && (t == FRT_MAT_DIFFUSE_LIGHT || t == FRT_MAT_METAL))
            return fail(FRT_E_UNSUPPORTED, "checker / image textures apply to lambertian / modified_phong / dielectric / "
                                           "rough_conductor colours");
        if (tex == FRT_TEX_IMAGE) {
            const int k = sv->materials[i].image;
            if (k < 0 || k >= sv->n_images || !sv->images)
                return fail(FRT_E_INVALID, "material image index out of range");
            const frt_image &im = sv->images[k];
            if (im.nx <= 0 || im.ny <= 0 || !im.data || (im.format != FRT_IMAGE_SRGB8 && im.format != FRT_IMAGE_F32))
                return fail(FRT_E_INVALID, "scene view: bad image");
        }
        if (t == FRT_MAT_ROUGH_CONDUCTOR &&
            (!(sv->materials[i].alpha > 0.0) || (sv->materials[i].distribution != FRT_DIST_GGX &&
                                                  sv->materials[i].distribution != FRT_DIST_BECKMANN)))
            return fail(FRT_E_INVALID, "rough_conductor needs alpha > 0 and a GGX / Beckmann distribution");
    }
    auto valid_ref = [&](int ref) {
        if (ref < 0) return false;
        if (ref & FRT_PRIM_SPHERE) return (ref & ~FRT_PRIM_SPHERE) < ns;
        return ref < nt;
    };
    auto prim_box = [&](int ref, double *lo, double *hi) {
        if (ref & FRT_PRIM_SPHERE) {
            const double *q = &sv->sphere[4 * (ref & ~FRT_PRIM_SPHERE)];
            for (int k = 0; k < 3; ++k) { lo[k] = q[k] - q[3]; hi[k] = q[k] + q[3]; }
        } else {
            const double *v = &sv->tri_v[9 * ref];
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(std::min(v[k], v[3 + k]), v[6 + k]);
                hi[k] = std::max(std::max(v[k], v[3 + k]), v[6 + k]);
            }
        }
    };
    std::vector<int> tri_order;            // device id -> view triangle
    std::vector<int> tri_dev(nt, -1);      // view triangle -> device id
    DevScene &S = F.meta;
    S = DevScene{};
    if (sv->world_kind == FRT_WORLD_BVH) {
        const int nn = sv->n_nodes;
        if (nn < 0 || (nn > 0 && (!sv->node_box || !sv->node_child)))
            return fail(FRT_E_INVALID, "scene view: missing BVH arrays");
        if (sv->root >= nn || (sv->root >= 0 && nn == 0)) return fail(FRT_E_INVALID, "scene view: bad root");
        double rlo[3], rhi[3];
        if (sv->root < 0) {
            if (!valid_ref(~sv->root)) return fail(FRT_E_INVALID, "scene view: bad root prim");
            prim_box(~sv->root, rlo, rhi);
        } else {
            for (int k = 0; k < 3; ++k) { rlo[k] = sv->node_box[6 * sv->root + k]; rhi[k] = sv->node_box[6 * sv->root + 3 + k]; }
        }
        double scale = 1.0;   // conservative box padding relative to the scene extent
        for (int k = 0; k < 3; ++k) scale = std::max(scale, std::max(std::fabs(rlo[k]), std::fabs(rhi[k])));
        const double pad = 4e-6 * scale;
        auto padded = [&](const double *lo, const double *hi, float *flo, float *fhi) {
            for (int k = 0; k < 3; ++k) { flo[k] = round_down(lo[k] - pad); fhi[k] = round_up(hi[k] + pad); }
        };
        padded(rlo, rhi, S.root_lo, S.root_hi);
        S.ao_tmax = (float)((rhi[1] - rlo[1]) * 0.50f);   // ao.cpp:19-21 (unpadded root box, fp64)
        std::vector<int> new_id(std::max(nn, 1), -1), order;
        order.reserve(nn);
        // left-first DFS: node ids in pre-order, triangle leaves numbered in visit order
        std::vector<std::pair<int, int>> st;   // (child ref, level)
        st.push_back({sv->root, 1});
        while (!st.empty()) {
            const auto [x, lvl] = st.back();
            st.pop_back();
            if (x >= 0) {
                if (x >= nn || new_id[x] >= 0) return fail(FRT_E_INVALID, "scene view: BVH is not a tree");
                new_id[x] = (int)order.size();
                order.push_back(x);
                F.depth = std::max(F.depth, lvl);
                st.push_back({sv->node_child[2 * x + 1], lvl + 1});
                st.push_back({sv->node_child[2 * x], lvl + 1});
            } else {
                const int ref = ~x;
                if (!valid_ref(ref)) return fail(FRT_E_INVALID, "scene view: bad leaf prim");
                if (!(ref & FRT_PRIM_SPHERE)) {
                    if (tri_dev[ref] >= 0) return fail(FRT_E_INVALID, "scene view: triangle in two leaves");
                    tri_dev[ref] = (int)tri_order.size();
                    tri_order.push_back(ref);
                }
            }
        }
        F.nodes.resize(4 * order.size());
        for (size_t i = 0; i < order.size(); ++i) {
            const int x = order[i];
            float cb[2][6];
            int cref[2];
            for (int side = 0; side < 2; ++side) {
                const int ch = sv->node_child[2 * x + side];
                double lo[3], hi[3];
                if (ch >= 0) {
                    for (int k = 0; k < 3; ++k) { lo[k] = sv->node_box[6 * ch + k]; hi[k] = sv->node_box[6 * ch + 3 + k]; }
                    cref[side] = new_id[ch];
                } else {
                    const int ref = ~ch;
                    prim_box(ref, lo, hi);
                    cref[side] = ~((ref & FRT_PRIM_SPHERE) ? ref : tri_dev[ref]);
                }
                padded(lo, hi, &cb[side][0], &cb[side][3]);
            }
            F.nodes[4 * i + 0] = make_float4(cb[0][0], cb[0][1], cb[0][2], cb[0][3]);
            F.nodes[4 * i + 1] = make_float4(cb[0][4], cb[0][5], cb[1][0], cb[1][1]);
            F.nodes[4 * i + 2] = make_float4(cb[1][2], cb[1][3], cb[1][4], cb[1][5]);
            F.nodes[4 * i + 3] = make_float4(i2f(cref[0]), i2f(cref[1]), 0.0f, 0.0f);
        }
        if (nt >= kLeafIndexLimit) return fail(FRT_E_INVALID, "scene view: too many triangles");
        // leaf size by plan (profiles/r01_leaf_ab.txt; re-checked at 512 spp in
        // profiles/r02/r02z_ab_leaf_512spp.txt): 2 triangles when the scene
        // fits the LDS plan (Cornell +6 % over 4), else 4 (cornell_1m: +11 % over 2)
        const int forced = leaf_size_override();
        if (forced) {
            collapse_leaves(F, forced);
        } else {
            const std::vector<float4> binary = F.nodes;
            const int depth = F.depth;
            collapse_leaves(F, kLeafSmallScene);
            const size_t bytes = sizeof(float4) * (F.nodes.size() + 5 * (size_t)nt + 2 * (size_t)nm);
            if (bytes > kLdsSceneBytes || F.depth >= kLdsMaxDepth) {
                F.nodes = binary;
                F.depth = depth;
                collapse_leaves(F, kLeafDefault);
            }
        }
        for (int i = 0; i < nt; ++i)   // triangles outside the tree: trailing ids, never intersected
            if (tri_dev[i] < 0) { tri_dev[i] = (int)tri_order.size(); tri_order.push_back(i); }
    } else if (sv->world_kind == FRT_WORLD_LIST) {
        S.ao_spheres_only = 1;                              // ao.cpp:21 t_max is NaN (ao_shade)
        if (sv->n_list < 0 || (sv->n_list > 0 && !sv->list)) return fail(FRT_E_INVALID, "scene view: bad list");
        for (int i = 0; i < nt; ++i) { tri_dev[i] = i; tri_order.push_back(i); }
        for (int i = 0; i < sv->n_list; ++i)
            if (!valid_ref(sv->list[i])) return fail(FRT_E_INVALID, "scene view: bad list entry");
    } else {
        return fail(FRT_E_INVALID, "scene view: unknown world kind");
    }
    auto dev_ref = [&](int ref) { return (ref & FRT_PRIM_SPHERE) ? ref : tri_dev[ref]; };
    F.tri_view = tri_order;

    // triangles in device order: v0 | e1 | e2 with the edges taken in fp64 (triangle.h:58-60)
    bool any_smooth = false;
    for (int i = 0; i < nt; ++i)
        if (sv->tri_geometry_normal && !sv->tri_geometry_normal[i]) any_smooth = true;
    if (any_smooth && !sv->tri_n) return fail(FRT_E_INVALID, "scene view: smooth triangles without normals");
    F.tris.resize(3 * (size_t)nt);
    F.tshade.resize(2 * (size_t)nt);
    if (any_smooth) F.tnorm.resize(3 * (size_t)nt);
    if (f64) {
        F.tris64.resize(3 * (size_t)nt);
        F.tshade64.resize(nt);
        if (any_smooth) F.tnorm64.resize(3 * (size_t)nt);
    }
    for (int d = 0; d < nt; ++d) {
        const int i = tri_order[d];
        const double *v = &sv->tri_v[9 * i];
        const double e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
        const double e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        double ng[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double l = std::sqrt(ng[0] * ng[0] + ng[1] * ng[1] + ng[2] * ng[2]);
        for (int k = 0; k < 3; ++k) ng[k] = ng[k] / l;   // unit_vector(cross(e1, e2)), triangle.h:101
        F.tris[3 * d + 0] = make_float4((float)v[0], (float)v[1], (float)v[2], 0.0f);
        F.tris[3 * d + 1] = make_float4((float)e1[0], (float)e1[1], (float)e1[2], 0.0f);
        F.tris[3 * d + 2] = make_float4((float)e2[0], (float)e2[1], (float)e2[2], 0.0f);
        const int mat = sv->tri_material[i];
        if (mat < 0 || mat >= nm) return fail(FRT_E_INVALID, "scene view: bad triangle material");
        const int geo = sv->tri_geometry_normal ? (sv->tri_geometry_normal[i] ? 1 : 0) : 1;
        F.tshade[2 * d + 0] = make_float4((float)ng[0], (float)ng[1], (float)ng[2], (float)sv->tri_inv_area[i]);
        F.tshade[2 * d + 1] = make_float4(i2f(mat), i2f(geo), 0.0f, 0.0f);
        if (any_smooth)
            for (int k = 0; k < 3; ++k)
                F.tnorm[3 * d + k] = make_float4((float)sv->tri_n[9 * i + 3 * k], (float)sv->tri_n[9 * i + 3 * k + 1],
                                                 (float)sv->tri_n[9 * i + 3 * k + 2], 0.0f);
        if (f64) {
            F.tris64[3 * d + 0] = make_double4(v[0], v[1], v[2], 0.0);
            F.tris64[3 * d + 1] = make_double4(e1[0], e1[1], e1[2], 0.0);
            F.tris64[3 * d + 2] = make_double4(e2[0], e2[1], e2[2], 0.0);
            F.tshade64[d] = make_double4(ng[0], ng[1], ng[2], sv->tri_inv_area[i]);
            if (any_smooth)
                for (int k = 0; k < 3; ++k)
                    F.tnorm64[3 * d + k] = make_double4(sv->tri_n[9 * i + 3 * k], sv->tri_n[9 * i + 3 * k + 1],
                                                        sv->tri_n[9 * i + 3 * k + 2], 0.0);
        }
    }
    // texture coordinates, only when a material is textured (in HBM; read at textured hits)
    bool any_tex = false;
    for (int i = 0; i < nm; ++i) any_tex |= sv->materials[i].texture != FRT_TEX_CONSTANT;
    if (any_tex) {
        F.tuv.assign(2 * (size_t)std::max(nt, 1), make_float4(0.0f, 0.0f, 0.0f, 0.0f));
        if (sv->tri_uv)
            for (int d = 0; d < nt; ++d) {
                const double *q = &sv->tri_uv[6 * tri_order[d]];
                F.tuv[2 * d] = make_float4((float)q[0], (float)q[1], (float)q[2], (float)q[3]);
                F.tuv[2 * d + 1] = make_float4((float)q[4], (float)q[5], 0.0f, 0.0f);
            }
    }
    F.spheres.resize(ns);
    F.smat.resize(ns);
    if (f64) F.spheres64.resize(ns);
    for (int k = 0; k < ns; ++k) {
        const double *q = &sv->sphere[4 * k];
        F.spheres[k] = make_float4((float)q[0], (float)q[1], (float)q[2], (float)q[3]);
        if (f64) F.spheres64[k] = make_double4(q[0], q[1], q[2], q[3]);
        F.smat[k] = sv->sphere_material[k];
        if (F.smat[k] < 0 || F.smat[k] >= nm) return fail(FRT_E_INVALID, "scene view: bad sphere material");
    }
    // image_texture texels: the reference's value per texel (texture.h:76-87: the float of an
    // HDR image, FromSrgb(byte / 255.0) in double otherwise, util.h:62-66) rounded to fp32
    std::vector<int> image_off(std::max(sv->n_images, 0), -1);
    for (int i = 0; i < nm; ++i) {
        if (sv->materials[i].texture != FRT_TEX_IMAGE) continue;
        const int k = sv->materials[i].image;
        if (image_off[k] >= 0) continue;
        const frt_image &im = sv->images[k];
        const size_t n = (size_t)im.nx * im.ny;
        if (F.texels.size() + n > (size_t)INT32_MAX) return fail(FRT_E_UNSUPPORTED, "images larger than 2^31 texels");
        image_off[k] = (int)F.texels.size();
        auto srgb = [](double v) { return v <= 0.04045 ? v * (1.0 / 12.92) : std::pow((v + 0.055) * (1.0 / 1.055), 2.4); };
        for (size_t q = 0; q < n; ++q) {
            double c[3];
            for (int ch = 0; ch < 3; ++ch)
                c[ch] = im.format == FRT_IMAGE_F32 ? (double)static_cast<const float *>(im.data)[3 * q + ch]
                                                   : srgb(static_cast<const uint8_t *>(im.data)[3 * q + ch] / 255.0);
            F.texels.push_back(make_float4((float)c[0], (float)c[1], (float)c[2], 0.0f));
        }
    }
    F.mats.assign(kMatStride * (size_t)nm, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (int i = 0; i < nm; ++i) {
        const frt_material &m = sv->materials[i];
        float4 *d = &F.mats[kMatStride * i];
        auto f4 = [](const double *v, float w) { return make_float4((float)v[0], (float)v[1], (float)v[2], w); };
        // m0 = (albedo | kd | metal albedo | rough eta, type); m1 = (emit, -) for lights,
        // (ks, exponent | ior | alpha) otherwise; m2 = (rough k, distribution)
        d[0] = f4(m.type == FRT_MAT_ROUGH_CONDUCTOR ? m.eta : m.albedo, i2f(m.type));
        if (m.type == FRT_MAT_DIFFUSE_LIGHT) d[1] = f4(m.emit, 0.0f);
        else d[1] = f4(m.specular, (float)(m.type == FRT_MAT_MODIFIED_PHONG ? m.exponent
                                           : m.type == FRT_MAT_DIELECTRIC ? m.ior : m.alpha));
        d[2] = f4(m.k, i2f(m.distribution));
        d[3] = f4(m.tex_odd, i2f(m.texture));
        d[4] = make_float4((float)m.tex_scale[0], (float)m.tex_scale[1], 0.0f, 0.0f);
        if (m.texture == FRT_TEX_IMAGE)   // (nx, ny, first texel)
            d[4] = make_float4(i2f(sv->images[m.image].nx), i2f(sv->images[m.image].ny), i2f(image_off[m.image]), 0.0f);
    }
    if (sv->n_lights < 0 || (sv->n_lights > 0 && !sv->lights)) return fail(FRT_E_INVALID, "scene view: bad lights");
    F.lights.resize(sv->n_lights);
    for (int i = 0; i < sv->n_lights; ++i) {
        if (!valid_ref(sv->lights[i])) return fail(FRT_E_INVALID, "scene view: bad light");
        F.lights[i] = dev_ref(sv->lights[i]);
    }
    F.list.resize(sv->world_kind == FRT_WORLD_LIST ? sv->n_list : 0);
    for (size_t i = 0; i < F.list.size(); ++i) F.list[i] = dev_ref(sv->list[i]);

    // octant copies of the binary nodes: child boxes as (near xyz, far xyz).
    // Only the LDS binary plan reads them, and only when they fit its budget
    // (pick_launcher_t): larger scenes get none (8x the node array otherwise).
    const size_t oct_bytes = sizeof(float4) * (oct_lds_node_slots((int)(F.nodes.size() / 4)) + F.tris.size() +
                                               F.tshade.size() + F.mats.size());
    if (sv->world_kind == FRT_WORLD_BVH && F.depth < kLdsMaxDepth && oct_bytes <= kLdsOctBytes)
        F.nodes_oct.resize(8 * F.nodes.size());
    for (int o = 0; o < 8 && !F.nodes_oct.empty(); ++o)
        for (size_t i = 0; i < F.nodes.size() / 4; ++i) {
            const float4 *n = &F.nodes[4 * i];
            const float b0[6] = {n[0].x, n[0].y, n[0].z, n[0].w, n[1].x, n[1].y};
            const float b1[6] = {n[1].z, n[1].w, n[2].x, n[2].y, n[2].z, n[2].w};
            float q[12];
            for (int a = 0; a < 3; ++a) {
                const bool neg = (o >> a) & 1;
                q[a] = neg ? b0[3 + a] : b0[a];
                q[3 + a] = neg ? b0[a] : b0[3 + a];
                q[6 + a] = neg ? b1[3 + a] : b1[a];
                q[9 + a] = neg ? b1[a] : b1[3 + a];
            }
            float4 *d = &F.nodes_oct[(size_t)o * F.nodes.size() + 4 * i];
            d[0] = make_float4(q[0], q[1], q[2], q[3]);
            d[1] = make_float4(q[4], q[5], q[6], q[7]);
            d[2] = make_float4(q[8], q[9], q[10], q[11]);
            d[3] = n[3];
        }
    S.root = (sv->world_kind == FRT_WORLD_BVH) ? ((sv->root >= 0) ? 0 : ~dev_ref(~sv->root)) : 0;
    F.has4 = sv->world_kind == FRT_WORLD_BVH && build_bvh4(F, S.root);
    if (!F.has4) F.nodes4.clear();
    S.root4 = F.has4 ? F.root4 : S.root;
    S.n_lights = sv->n_lights;
    S.n_list = (int)F.list.size();
    S.n_nodes = (int)(F.nodes.size() / 4);
    S.n_tris = nt;
    S.n_mats = nm;
    S.n_nodes4 = (int)(F.nodes4.size() / kNode4Parts);
    S.node_es = 4; S.node_ps = 1;
    S.node4_es = kNode4Parts; S.node4_ps = 1;
    S.tri_es = 3; S.tri_ps = 1;
    S.sh_es = 2; S.sh_ps = 1;
    S.world_kind = sv->world_kind;
    auto f3d = [](const double *x) { return mk3((float)x[0], (float)x[1], (float)x[2]); };
    S.cam_o = f3d(sv->cam_origin); S.cam_llc = f3d(sv->cam_lower_left);
    S.cam_h = f3d(sv->cam_horizontal); S.cam_v = f3d(sv->cam_vertical);
    S.cam_u = f3d(sv->cam_u); S.cam_vv = f3d(sv->cam_v);
    S.lens_r = (float)sv->cam_lens_radius;
    S.cam_w = f3d(sv->cam_w);
    S.cam_half_height = (float)sv->cam_half_height;
    S.env = f3d(sv->env_color);
    auto d3d = [](const double *x) { return d3{x[0], x[1], x[2]}; };
    S.cam64_o = d3d(sv->cam_origin); S.cam64_llc = d3d(sv->cam_lower_left);
    S.cam64_h = d3d(sv->cam_horizontal); S.cam64_v = d3d(sv->cam_vertical);
    S.cam64_u = d3d(sv->cam_u); S.cam64_vv = d3d(sv->cam_v);
    S.lens_r64 = sv->cam_lens_radius;
    return FRT_OK;
}

template <typename T, typename P>
static int upload_vec(frt_ctx *c, const std::vector<T> &v, P *dst)
{
    void *p = nullptr;
    const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    HIPCHK(c, hipMalloc(&p, bytes));
    c->scene_bufs.push_back(p);
    if (!v.empty()) HIPCHK(c, hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    *dst = (P)p;
    return FRT_OK;
}

extern "C" int frt_upload_scene(frt_ctx *c, const frt_scene_view *sv)
{
    if (!c || !sv) return FRT_E_INVALID;
    HIPCHK(c, hipSetDevice(c->device));
    FlatScene F;
    std::string err;
    // fp64 records when this context's precision can pick the fp64 kernels for the scene
    const bool want_f64 = c->precision == FRT_PRECISION_FP64 ||
                          (c->precision == FRT_PRECISION_AUTO && sv->world_kind == FRT_WORLD_LIST);
    const int frc = flatten_scene(sv, F, err, want_f64);
    if (frc != FRT_OK) return set_err(c, frc, err);
    free_scene(c);
    c->S = F.meta;
    DevScene &S = c->S;
    int rc;
    if ((rc = upload_vec(c, F.nodes, &S.nodes)) || (rc = upload_vec(c, F.nodes4, &S.nodes4)) ||
        (rc = upload_vec(c, F.nodes_oct, &S.nodes_oct)) ||
        (rc = upload_vec(c, F.tris, &S.tris)) ||
        (rc = upload_vec(c, F.tshade, &S.tshade)) || (rc = upload_vec(c, F.tnorm, &S.tnorm)) ||
        (rc = upload_vec(c, F.tuv, &S.tuv)) || (rc = upload_vec(c, F.texels, &S.texels)) ||
        (rc = upload_vec(c, F.spheres, &S.spheres)) || (rc = upload_vec(c, F.smat, &S.sphere_mat)) ||
        (rc = upload_vec(c, F.mats, &S.mats)) || (rc = upload_vec(c, F.lights, &S.lights)) ||
        (rc = upload_vec(c, F.list, &S.list)) || (rc = upload_vec(c, F.tri_view, &S.tri_view)))
        return rc;
    S.tris64 = nullptr; S.tshade64 = nullptr; S.tnorm64 = nullptr; S.spheres64 = nullptr;
    if (want_f64 && ((rc = upload_vec(c, F.tris64, &S.tris64)) || (rc = upload_vec(c, F.tshade64, &S.tshade64)) ||
                     (rc = upload_vec(c, F.tnorm64, &S.tnorm64)) || (rc = upload_vec(c, F.spheres64, &S.spheres64))))
        return rc;
    c->world_kind = S.world_kind;
    c->stack_needed = F.depth;
    c->has_bvh4 = F.has4;
    c->n_tris = S.n_tris;
    c->n_spheres = (int)F.spheres.size();
    c->n_list = S.n_list;
    c->has_spec_mats = false;
    c->has_metal = false;
    c->mats = kMatsNone;
    for (int i = 0; i < sv->n_materials; ++i) {
        const int t = sv->materials[i].type;
        if (t == FRT_MAT_MODIFIED_PHONG || t == FRT_MAT_METAL || t == FRT_MAT_DIELECTRIC) c->mats |= kMatsSpec;
        if (t == FRT_MAT_ROUGH_CONDUCTOR) c->mats |= kMatsRough;
        if (sv->materials[i].texture != FRT_TEX_CONSTANT) c->mats |= kMatsTex;
        if (t == FRT_MAT_METAL) c->has_metal = true;
    }
    c->has_spec_mats = c->mats != kMatsNone;
    c->depth4 = F.depth4;
    c->scene_lds_bytes = sizeof(float4) * (F.nodes.size() + F.tris.size() + F.tshade.size() + F.mats.size());
    c->scene_lds_bytes_oct = F.nodes_oct.empty() ? SIZE_MAX
                             : sizeof(float4) * (oct_lds_node_slots(S.n_nodes) + F.tris.size() + F.tshade.size() +
                                                 F.mats.size());
    c->has_f64 = want_f64;
    c->have_scene = true;
    return FRT_OK;
}

// 4-wide traversal holds at most 3 pending siblings per level of the path
constexpr int kSelftestStack = 8;   // small, so the host self-test exercises the overflow entries

// host image of the flattened scene as the kernels see it (HBM strides)
static DevScene host_scene(const FlatScene &F)
{
    DevScene S = F.meta;
    S.nodes = F.nodes.data(); S.nodes4 = F.nodes4.data(); S.nodes_oct = F.nodes_oct.data();
    S.tris = F.tris.data(); S.tshade = F.tshade.data(); S.tnorm = F.tnorm.data();
    S.tuv = F.tuv.data(); S.texels = F.texels.data();
    S.spheres = F.spheres.data(); S.sphere_mat = F.smat.data(); S.mats = F.mats.data();
    S.lights = F.lights.data(); S.list = F.list.data(); S.tri_view = F.tri_view.data();
    S.tris64 = F.tris64.data(); S.tshade64 = F.tshade64.data(); S.tnorm64 = F.tnorm64.data();
    S.spheres64 = F.spheres64.data();
    return S;
}

// the self-test's per-pixel loop in precision R (fp64: the binary tree or the list)
template <typename R>
static void selftest_pixels(const DevScene &S, const FlatScene &F, const frt_render_params *p, const int32_t *pixels,
                            int npix, bool wide, std::vector<int> &stack, float *out_rgb, uint64_t cnt[3])
{
    uint32_t n_ext = 0, n_sh = 0;
    for (int i = 0; i < npix; ++i) {
        const int pix = pixels[i];
        const int px = pix % p->nx, py = pix / p->nx;
        V3<R> acc = zero3<R>();
        for (int smp = 0; smp < p->spp; ++smp) {
            PathState<R> P;
            path_begin(P, S, px, py, p->nx, p->ny, p->seed, (uint32_t)pix, (uint32_t)(smp + p->sample_offset));
            ++cnt[0];
            for (;;) {
                Hit<R> h;
                if (S.world_kind == FRT_WORLD_LIST) {
                    h = trace<FRT_WORLD_LIST, 1>(S, P.ro, P.rd, P.rtmax, P.shadow, stack.data());
                } else if constexpr (!kIsF64<R>) {
                    h = wide ? trace<kWorldBvh4, 1, kSelftestStack>(S, P.ro, P.rd, P.rtmax, P.shadow, stack.data())
                             : trace<FRT_WORLD_BVH, 1>(S, P.ro, P.rd, P.rtmax, P.shadow, stack.data());
                } else {
                    h = trace<FRT_WORLD_BVH, 1>(S, P.ro, P.rd, P.rtmax, P.shadow, stack.data());
                }
                n_ext = n_sh = 0;
                const bool done = p->integrator == FRT_INTEGRATOR_AO ? ao_shade(P, S, h, n_sh)
                                  : p->integrator == FRT_INTEGRATOR_NORMALS ? normals_shade(P, S, h)
                                  : path_shade(P, S, h, p->max_depth, n_ext, n_sh);
                cnt[1] += n_ext; cnt[2] += n_sh;
                if (done) break;
            }
            acc = acc + P.L;
        }
        const R k = R(1) / (R)p->spp;
        out_rgb[3 * i] = (float)(acc.x * k); out_rgb[3 * i + 1] = (float)(acc.y * k); out_rgb[3 * i + 2] = (float)(acc.z * k);
    }
}

// Self-test hook (CPU-only unit tests): runs frt_path.hpp -- the code the
// megakernel runs per lane -- on the host over the flattened scene, in fp32 or
// (FRT_FLAG_FP64) in fp64.  Not a render path: frt_render / frt_render_device
// never call it.
extern "C" int frt_selftest_path_host(const frt_scene_view *sv, const frt_render_params *p, const int32_t *pixels,
                                      int npix, float *out_rgb, frt_stats *st)
{
    if (!sv || !p || !pixels || !out_rgb || npix < 0 || p->spp <= 0 || p->nx <= 0 || p->ny <= 0) return FRT_E_INVALID;
    for (int i = 0; i < npix; ++i)
        if (pixels[i] < 0 || pixels[i] >= p->nx * p->ny) return FRT_E_INVALID;
    const bool f64 = (p->flags & FRT_FLAG_FP64) != 0;
    FlatScene F;
    std::string err;
    const int rc = flatten_scene(sv, F, err, f64);
    if (rc != FRT_OK) return rc;
    if (p->integrator == FRT_INTEGRATOR_AO)
        for (int i = 0; i < sv->n_materials; ++i)
            if (sv->materials[i].type == FRT_MAT_METAL) return FRT_E_UNSUPPORTED;
    const DevScene S = host_scene(F);
    std::vector<int> stack(std::max(F.depth + 1, kSelftestStack));
    const bool wide = !f64 && S.world_kind == FRT_WORLD_BVH && F.has4 && !(p->flags & FRT_FLAG_BVH2) &&
                      bvh4_stack_fits(F.depth4, kSelftestStack);
    uint64_t cnt[3] = {0, 0, 0};   // camera, extension, shadow
    if (f64) selftest_pixels<double>(S, F, p, pixels, npix, wide, stack, out_rgb, cnt);
    else selftest_pixels<float>(S, F, p, pixels, npix, wide, stack, out_rgb, cnt);
    if (st) {
        memset(st, 0, sizeof(*st));
        st->camera_rays = cnt[0]; st->extension_rays = cnt[1]; st->shadow_rays = cnt[2];
        st->samples = cnt[0]; st->pixels = (uint64_t)npix;
        st->stack_entries = wide ? (uint32_t)kSelftestStack : (uint32_t)stack.size();
        st->bvh_depth = (uint32_t)(wide ? F.depth4 : F.depth);   // which tree was traversed
        st->fp64 = f64 ? 1u : 0u;
    }
    return FRT_OK;
}


// Self-test hook: n PSS-MLT bootstrap eye paths (fresh primary samples from the
// bootstrap stream) through frt_mlt.hpp on the host; out6[i] = x, y, r, g, b, sc.
extern "C" int frt_selftest_mlt_paths_host(const frt_scene_view *sv, int nx, int ny, uint32_t seed, int n,
                                           float *out6)
{
    if (!sv || !out6 || n < 0 || nx <= 0 || ny <= 0) return FRT_E_INVALID;
    FlatScene F;
    std::string err;
    const int rc = flatten_scene(sv, F, err, false);
    if (rc != FRT_OK) return rc;
    const DevScene S = host_scene(F);
    std::vector<int> stack(std::max(F.depth + 1, 1));
    for (int i = 0; i < n; ++i) {
        PrndSource src{nullptr, 0, 0, rng_key(seed ^ kMltBootSalt, (uint32_t)i, 0u), 0u, true, 0.0f, 0.0f};
        MltPath M;
        mlt_begin(M, S, src, nx, ny);
        uint32_t ne = 0, ns = 0;
        for (;;) {
            if (mlt_beyond(M)) { M.P.L = M.P.L + M.P.beta * S.env; break; }
            const Hit<float> h = (S.world_kind == FRT_WORLD_LIST)
                              ? trace<FRT_WORLD_LIST, 1>(S, M.P.ro, M.P.rd, M.P.rtmax, M.P.shadow, stack.data())
                              : trace<FRT_WORLD_BVH, 1>(S, M.P.ro, M.P.rd, M.P.rtmax, M.P.shadow, stack.data());
            if (mlt_shade(M, S, h, src, ne, ns)) break;
        }
        const f3 L = M.P.L;
        float *o = &out6[6 * (size_t)i];
        o[0] = M.x; o[1] = M.y; o[2] = L.x; o[3] = L.y; o[4] = L.z; o[5] = fmaxf(fmaxf(L.x, L.y), L.z);
    }
    return FRT_OK;
}

// ---- shard geometry ----
static int eff_tile(const frt_render_params *p) { return p->tile_size > 0 ? p->tile_size : 32; }
constexpr int kRetiredFlags = 32 | 64 | 128;   // frt.h: the round-4 plans measured slower and removed
static bool params_ok(const frt_render_params *p)
{
    const int T = eff_tile(p);
    if (!(p && p->nx > 0 && p->ny > 0 && p->spp > 0 && (T % 8) == 0 && T <= 256 && p->shard_count >= 1 &&
          p->shard_index >= 0 && p->shard_index < p->shard_count && p->max_depth >= -1 && p->max_depth < 100000))
        return false;
    if (p->sample_offset < 0 || (int64_t)p->sample_offset + p->spp > (int64_t)0xffffffffLL) return false;
    if ((int64_t)p->nx * p->ny > (int64_t)INT32_MAX) return false;   // pixel indices are int32 (frt_shard_slots)
    if (p->flags & kRetiredFlags) return false;         // removed A/B plans: fail loudly, not silently
    if (p->integrator == FRT_INTEGRATOR_PATH || p->integrator == FRT_INTEGRATOR_AO ||
        p->integrator == FRT_INTEGRATOR_NORMALS)
        return true;
    return p->integrator == FRT_INTEGRATOR_PSSMLT && p->mlt_chains > 0 && p->mlt_bootstrap > 0 &&
           p->sample_offset == 0;
}
static int my_tiles(const frt_render_params *p)
{
    const int T = eff_tile(p);
    const int ntiles = ((p->nx + T - 1) / T) * ((p->ny + T - 1) / T);
    if (p->shard_index >= ntiles) return 0;
    return (ntiles - 1 - p->shard_index) / p->shard_count + 1;
}
extern "C" int64_t frt_shard_slot_count(const frt_render_params *p)
{
    if (!params_ok(p)) return FRT_E_INVALID;
    if (p->integrator == FRT_INTEGRATOR_PSSMLT) return (int64_t)p->nx * p->ny;   // whole film per shard
    const int T = eff_tile(p);
    return (int64_t)my_tiles(p) * T * T;
}
extern "C" int frt_shard_slots(const frt_render_params *p, int32_t *slot_pixel)
{
    if (!params_ok(p) || !slot_pixel) return FRT_E_INVALID;
    if (p->integrator == FRT_INTEGRATOR_PSSMLT) {
        for (int64_t i = 0; i < (int64_t)p->nx * p->ny; ++i) slot_pixel[i] = (int32_t)i;
        return FRT_OK;
    }
    const int T = eff_tile(p), ntx = (p->nx + T - 1) / T;
    const int nmt = my_tiles(p);
    for (int t = 0; t < nmt; ++t) {
        const int tile_id = p->shard_index + t * p->shard_count;
        for (int s = 0; s < T * T; ++s) {
            int lx, ly;
            slot_to_local(s, T, lx, ly);
            const int px = (tile_id % ntx) * T + lx, py = (tile_id / ntx) * T + ly;
            slot_pixel[(size_t)t * T * T + s] = (px < p->nx && py < p->ny) ? py * p->nx + px : -1;
        }
    }
    return FRT_OK;
}


// does this render run the fp64 kernels?  FRT_FLAG_FP64 / _FP32 override the
// context's precision for one call (A/B)
static bool use_f64(const frt_ctx *c, const frt_render_params *p)
{
    if (p->integrator != FRT_INTEGRATOR_PATH || (p->flags & FRT_FLAG_FP32)) return false;
    if (p->flags & FRT_FLAG_FP64) return true;
    return c->precision == FRT_PRECISION_FP64 || (c->precision == FRT_PRECISION_AUTO && c->world_kind == FRT_WORLD_LIST);
}
static int pick_launcher(const frt_ctx *c, int integrator, int flags, Launcher &L, bool f64)
{
    if (f64 && !c->has_f64) return FRT_E_INVALID;
    if (integrator == FRT_INTEGRATOR_NORMALS) return pick_launcher_kind<FRT_INTEGRATOR_NORMALS>(c, flags, L);
    if (integrator == FRT_INTEGRATOR_AO || c->mats != kMatsNone || (f64 && c->world_kind != FRT_WORLD_LIST))
        return frt_mats::pick(c, integrator, flags, f64, L);   // every kernel with a material set
    if (f64) {   // a lambertian list world (BVH worlds' fp64 kernels carry every material: the other unit)
        L = make_launcher<16, FRT_WORLD_LIST, false, 1, kMatsNone, FRT_INTEGRATOR_PATH, double>(0);
        return FRT_OK;
    }
    return pick_launcher_t<kMatsNone>(c, flags, L);
}


// ---- ray queries: trace_kernel plans (the path plans' residency rules) ----
struct TraceLauncher {
    const void *fn = nullptr;
    size_t lds = 0;
    int waves = 0;
    bool lds_scene = false;
    size_t scene_lds = 0;   // as Launcher::scene_lds
};
template <int STACK, int WORLD, bool LDS, int WAVES>
static TraceLauncher make_trace(size_t scene_bytes)
{
    TraceLauncher L;
    L.fn = reinterpret_cast<const void *>(&trace_kernel<STACK, WORLD, LDS, WAVES>);
    L.lds = (WORLD != FRT_WORLD_LIST ? (size_t)STACK * kBlock * sizeof(int) : 0) + (LDS ? scene_bytes : 0);
    L.scene_lds = LDS ? scene_bytes : 0;
    L.waves = WAVES;
    L.lds_scene = LDS;
    return L;
}
// register cap of the ray-query kernel: FRT_TRACE_WAVES (6 / 8 / 10; A/B knob, not part of the C-ABI)
template <int STACK, int WORLD, bool LDS>
static TraceLauncher trace_waves(size_t sb)
{
    const char *e = std::getenv("FRT_TRACE_WAVES");
    const int w = e ? std::atoi(e) : 8;
    if (w == 6) return make_trace<STACK, WORLD, LDS, 6>(sb);
    if (w == 10) return make_trace<STACK, WORLD, LDS, 10>(sb);
    return make_trace<STACK, WORLD, LDS, 8>(sb);
}
static int pick_trace(const frt_ctx *c, int flags, TraceLauncher &L)
{
    if (c->world_kind == FRT_WORLD_LIST) { L = make_trace<16, FRT_WORLD_LIST, false, 8>(0); return FRT_OK; }
    const int d = c->stack_needed;
    const bool lds = d < kLdsMaxDepth && c->scene_lds_bytes <= kLdsSceneBytes && !(flags & FRT_FLAG_NO_LDS_SCENE);
    if (lds && !(flags & FRT_FLAG_NO_OCT) && c->scene_lds_bytes_oct <= kLdsOctBytes) {
        L = d < 8 ? trace_waves<8, kWorldBvh2Oct, true>(c->scene_lds_bytes_oct)
                  : trace_waves<16, kWorldBvh2Oct, true>(c->scene_lds_bytes_oct);
    } else if (lds) {
        L = d < 8 ? make_trace<8, FRT_WORLD_BVH, true, 8>(c->scene_lds_bytes)
                  : make_trace<16, FRT_WORLD_BVH, true, 8>(c->scene_lds_bytes);
    } else if (c->has_bvh4 && !(flags & FRT_FLAG_BVH2) && bvh4_stack_fits(c->depth4, kBvh4LdsStack)) {
        L = trace_waves<kBvh4LdsStack, kWorldBvh4, false>(0);
    } else if (d < 16) {
        L = make_trace<16, FRT_WORLD_BVH, false, 8>(0);
    } else if (d < 32) {
        L = make_trace<32, FRT_WORLD_BVH, false, 8>(0);
    } else if (d < 64) {
        L = make_trace<64, FRT_WORLD_BVH, false, 1>(0);
    } else {
        return FRT_E_UNSUPPORTED;
    }
    return FRT_OK;
}

// Batched Scene::world->hit (include/frt.h frt_trace_device)
extern "C" int frt_trace_device(frt_ctx *c, const float *rays, int64_t n, float *hits, int flags, void *hip_stream,
                                frt_stats *st)
{
    const auto t_start = std::chrono::steady_clock::now();
    if (!c || n < 0 || (n > 0 && (!rays || !hits))) return FRT_E_INVALID;
    if (!c->have_scene) return set_err(c, FRT_E_NO_SCENE, "no scene uploaded");
    HIPCHK(c, hipSetDevice(c->device));
    hipStream_t stream = hip_stream ? (hipStream_t)hip_stream : c->stream;
    TraceLauncher L;
    if (pick_trace(c, flags, L) != FRT_OK) return set_err(c, FRT_E_UNSUPPORTED, "BVH deeper than 63 levels");
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, L.fn, kBlock, L.lds) != hipSuccess || bpc <= 0) bpc = 1;
    const int64_t want = std::max<int64_t>(1, (n + kBlock - 1) / kBlock);
    const int grid = (int)std::min<int64_t>((int64_t)c->n_cu * bpc, want);
    // the 32-bit ray-queue head runs past n by up to one chunk per wave
    // (render_impl has the same headroom check)
    if (n + (int64_t)(grid * kBlock / 64) * kTraceChunk >= (int64_t)0xffffffffLL)
        return set_err(c, FRT_E_UNSUPPORTED, "frt_trace_device: too many rays for one call (2^32 - 1 less the queue headroom)");
    DevRays R{};
    R.ray = reinterpret_cast<const float4 *>(rays);
    R.hit = reinterpret_cast<float4 *>(hits);
    R.n = (uint32_t)n;
    R.min_desc = min_desc(L.lds_scene);
    // its own queue word, a cache line away from the render queue's: a trace and
    // a render of one context on two streams do not share a queue head
    R.counter = c->counter + kTraceCounterWord;
    HIPCHK(c, hipMemsetAsync(R.counter, 0, sizeof(unsigned), stream));
    HIPCHK(c, hipEventRecord(c->ev0, stream));
    if (n > 0) {
        DevScene Sarg = c->S;
        void *args[] = {&Sarg, &R};
        const hipError_t le = hipLaunchKernel(L.fn, dim3(grid), dim3(kBlock), args, L.lds, stream);
        if (le != hipSuccess) return set_err(c, FRT_E_HIP, std::string("trace_kernel launch: ") + hipGetErrorString(le));
    }
    HIPCHK(c, hipEventRecord(c->ev1, stream));
    HIPCHK(c, hipStreamSynchronize(stream));
    float ms = 0.0f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
    if (st) {
        memset(st, 0, sizeof(*st));
        st->camera_rays = (uint64_t)n;
        st->kernel_ms = ms;
        st->scene_in_lds = L.lds_scene ? 1u : 0u;
        st->waves_cap = (uint32_t)L.waves;
        st->scene_bytes = L.lds_scene ? L.scene_lds : c->scene_lds_bytes;   // what this plan reads
        st->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    return FRT_OK;
}

// ---- PSS-MLT render: bootstrap b, then the chain megakernel splatting into dev_film ----
// PSS-MLT kernels of a plan: the material branch from the material unit
template <int STACK, int WORLD, bool LDS = false>
static void mlt_kernels(bool mats, const void **boot, const void **chains)
{
    if (mats) frt_mats::mlt(STACK, WORLD, LDS, boot, chains);
    else if constexpr (WORLD == kWorldBvh2Oct && kSplitLds) frt_lds::mlt_oct(STACK, boot, chains);
    else mlt_kernels_t<STACK, WORLD, LDS, false>(boot, chains);
}

#if defined(FRT_DIAG)
// diagnostic builds only: the per-phase counters of the last path or PSS-MLT
// render, one kDiagSlots row per wave on the device, summed over waves here
static unsigned long long g_diag_sum[kDiagSlots];
static unsigned long long *g_diag_buf = nullptr;
static size_t g_diag_n = 0;
static int diag_begin(frt_ctx *c, size_t n_waves, hipStream_t st)
{
    if (g_diag_n < n_waves * kDiagSlots) {
        if (g_diag_buf) HIPCHK(c, hipFree(g_diag_buf));
        g_diag_n = n_waves * kDiagSlots;
        HIPCHK(c, hipMalloc(&g_diag_buf, g_diag_n * sizeof(unsigned long long)));
    }
    HIPCHK(c, hipMemsetAsync(g_diag_buf, 0, g_diag_n * sizeof(unsigned long long), st));
    HIPCHK(c, hipMemcpyToSymbolAsync(HIP_SYMBOL(frt::frt_diag), &g_diag_buf, sizeof(g_diag_buf), 0,
                                     hipMemcpyHostToDevice, st));
    return FRT_OK;
}
static int diag_end(frt_ctx *c, size_t n_waves)
{
    std::vector<unsigned long long> dv(n_waves * kDiagSlots);
    HIPCHK(c, hipMemcpy(dv.data(), g_diag_buf, dv.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    for (int k = 0; k < kDiagSlots; ++k) g_diag_sum[k] = 0;
    for (size_t w = 0; w < n_waves; ++w)
        for (int k = 0; k < kDiagSlots; ++k) g_diag_sum[k] += dv[w * kDiagSlots + k];
    return FRT_OK;
}
extern "C" int frt_diag_read(unsigned long long *out)
{
    for (int k = 0; k < kDiagSlots; ++k) out[k] = g_diag_sum[k];
    return kDiagSlots;
}
#endif

static int render_mlt(frt_ctx *c, const frt_render_params *p, float *dev_film, hipStream_t st, frt_stats *stats)
{
    const auto t_start = std::chrono::steady_clock::now();
    int stack;
    const void *kboot = nullptr, *kchain = nullptr;
    const int d = c->stack_needed;
    const bool lds_scene = c->world_kind == FRT_WORLD_BVH && d < kLdsMaxDepth && c->scene_lds_bytes <= kLdsSceneBytes &&
                           !(p->flags & FRT_FLAG_NO_LDS_SCENE);
    // the octant node copies when they fit, as the path kernels (round 5: the chain kernel used the planar tree)
    const bool oct = lds_scene && !(p->flags & FRT_FLAG_NO_OCT) && c->scene_lds_bytes_oct <= kLdsOctBytes;
    if (c->world_kind == FRT_WORLD_LIST) { stack = 0; mlt_kernels<16, FRT_WORLD_LIST>(c->has_spec_mats, &kboot, &kchain); }
    else if (!lds_scene && c->has_bvh4 && !(p->flags & FRT_FLAG_BVH2) && bvh4_stack_fits(c->depth4, kBvh4LdsStack)) {
        stack = kBvh4LdsStack;
        mlt_kernels<kBvh4LdsStack, kWorldBvh4>(c->has_spec_mats, &kboot, &kchain);
    }
    else if (oct && d < 8) { stack = 8; mlt_kernels<8, kWorldBvh2Oct, true>(c->has_spec_mats, &kboot, &kchain); }
    else if (oct) { stack = 16; mlt_kernels<16, kWorldBvh2Oct, true>(c->has_spec_mats, &kboot, &kchain); }
    else if (lds_scene && d < 8) { stack = 8; mlt_kernels<8, FRT_WORLD_BVH, true>(c->has_spec_mats, &kboot, &kchain); }
    else if (lds_scene) { stack = 16; mlt_kernels<16, FRT_WORLD_BVH, true>(c->has_spec_mats, &kboot, &kchain); }
    else if (d < 16) { stack = 16; mlt_kernels<16, FRT_WORLD_BVH>(c->has_spec_mats, &kboot, &kchain); }
    else if (d < 32) { stack = 32; mlt_kernels<32, FRT_WORLD_BVH>(c->has_spec_mats, &kboot, &kchain); }
    else if (d < 64) { stack = 64; mlt_kernels<64, FRT_WORLD_BVH>(c->has_spec_mats, &kboot, &kchain); }
    else return set_err(c, FRT_E_UNSUPPORTED, "BVH deeper than 63 levels");
    const size_t lds_boot = (size_t)stack * kBlock * sizeof(int);
    const size_t lds = lds_boot + (size_t)kChainWords * kBlock * sizeof(int) +
                       (oct ? c->scene_lds_bytes_oct : lds_scene ? c->scene_lds_bytes : 0);
    const uint32_t n_chains = (uint32_t)p->mlt_chains;
    const uint32_t n_local = (n_chains > (uint32_t)p->shard_index)
                                 ? (n_chains - 1 - (uint32_t)p->shard_index) / (uint32_t)p->shard_count + 1 : 0;
    const uint64_t total = (uint64_t)p->spp * (uint64_t)p->nx * (uint64_t)p->ny;   // viewer ns
    const uint64_t steps = total / n_chains;                                       // samples_per_thread
    if (steps >= 0xffffffffULL) return set_err(c, FRT_E_UNSUPPORTED, "pssmlt: more than 2^32 - 1 mutations per chain");
    // bootstrap normaliser (identical on every shard: same streams, fixed-order host sum)
    const int n_init = p->mlt_bootstrap;
    const size_t need = std::max<size_t>((size_t)n_init * sizeof(float), (size_t)kMltRow * n_local * sizeof(float));
    if (need > c->partial_bytes) {
        if (c->partial) HIPCHK(c, hipFree(c->partial));
        c->partial = nullptr;
        HIPCHK(c, hipMalloc(&c->partial, need));
        c->partial_bytes = need;
    }
#if defined(FRT_DIAG)
    // the bootstrap's traversal ticks too: a diagnostic buffer for its grid (zeroed again before the chains)
    if (const int drc = diag_begin(c, (size_t)(n_init + kBlock - 1) / kBlock * (kBlock / 64), st)) return drc;
#endif
    {
        int nx = p->nx, ny = p->ny, ni = n_init;
        uint32_t seed = p->seed;
        float *sc = c->partial;
        DevScene Sarg = c->S;
        void *args[] = {&Sarg, &nx, &ny, &seed, &ni, &sc};
        HIPCHK(c, hipLaunchKernel(kboot, dim3((n_init + kBlock - 1) / kBlock), dim3(kBlock), args, lds_boot, st));
    }
    std::vector<float> sc(n_init);
    HIPCHK(c, hipMemcpyAsync(sc.data(), c->partial, n_init * sizeof(float), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    double b = 0.0;
    for (float v : sc) b += v;
    b /= n_init;
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kchain, kBlock, lds) != hipSuccess || bpc <= 0) bpc = 1;
    const int grid = std::max(1, std::min<int>(c->n_cu * bpc, (int)((n_local + kBlock - 1) / kBlock)));
    const size_t n_waves = (size_t)grid * kBlock / 64;
    if (n_waves > c->wave_rays_n) {
        if (c->wave_rays) HIPCHK(c, hipFree(c->wave_rays));
        c->wave_rays = nullptr;
        HIPCHK(c, hipMalloc(&c->wave_rays, n_waves * 4 * sizeof(unsigned long long)));
        c->wave_rays_n = n_waves;
    }
    MltWork W{};
    W.nx = p->nx; W.ny = p->ny; W.seed = p->seed;
    W.shard_index = p->shard_index; W.shard_count = p->shard_count;
    W.n_local = n_local; W.steps = steps;
    W.b = (float)b;
    W.scale = (float)((double)p->nx * p->ny / ((double)steps * (double)n_chains));   // AccumulatePathContribution
    W.s2p = 0.1f;
    W.logp = (float)std::log((double)0.1f / (2.0 / (double)(p->nx + p->ny)));
    const size_t n_film = (size_t)p->nx * p->ny * 3;
    if (n_film * sizeof(unsigned long long) > c->splat_bytes) {
        if (c->splat) HIPCHK(c, hipFree(c->splat));
        c->splat = nullptr;
        HIPCHK(c, hipMalloc(&c->splat, n_film * sizeof(unsigned long long)));
        c->splat_bytes = n_film * sizeof(unsigned long long);
    }
    W.U = c->partial; W.film = c->splat; W.counter = c->counter; W.wave_rays = c->wave_rays;
    W.trav_min = trav_min(lds_scene);
    W.min_desc = min_desc(lds_scene);
    HIPCHK(c, hipMemsetAsync(c->splat, 0, n_film * sizeof(unsigned long long), st));
    HIPCHK(c, hipMemsetAsync(c->counter, 0, 64, st));
#if defined(FRT_DIAG)
    if (const int drc = diag_begin(c, n_waves, st)) return drc;
#endif
    HIPCHK(c, hipEventRecord(c->ev0, st));
    if (n_local > 0 && steps > 0) {
        DevScene Sarg = c->S;
        void *args[] = {&Sarg, &W};
        HIPCHK(c, hipLaunchKernel(kchain, dim3(grid), dim3(kBlock), args, lds, st));
    }
    HIPCHK(c, hipEventRecord(c->ev1, st));
    mlt_film_to_float<<<dim3((unsigned)((n_film + kBlock - 1) / kBlock)), dim3(kBlock), 0, st>>>(c->splat, dev_film, n_film);
    HIPCHK(c, hipGetLastError());
    std::vector<unsigned long long> wr(n_waves * 4, 0);
    if (n_local > 0 && steps > 0)
        HIPCHK(c, hipMemcpyAsync(wr.data(), c->wave_rays, wr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    float ms = 0.0f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
#if defined(FRT_DIAG)
    if (const int drc = diag_end(c, n_waves)) return drc;
#endif
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (size_t w = 0; w < n_waves; ++w) {
            stats->camera_rays += wr[4 * w]; stats->extension_rays += wr[4 * w + 1];
            stats->shadow_rays += wr[4 * w + 2]; stats->samples += wr[4 * w + 3];
        }
        stats->pixels = (uint64_t)p->nx * p->ny;
        stats->work_items = n_local;
        stats->scene_in_lds = lds_scene ? 1u : 0u;
        stats->stack_entries = (uint32_t)stack;
        stats->bvh_depth = (uint32_t)c->stack_needed;
        // the LDS copy the chain kernel loads (the octant node copies on that plan)
        stats->scene_bytes = oct ? c->scene_lds_bytes_oct : c->scene_lds_bytes;
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
    }
    c->last_mlt_b = b;
    c->mlt_rows = (n_local > 0 && steps > 0) ? n_local : 0;
    return FRT_OK;
}

// The chain states of the last PSS-MLT render (test / diagnostic read-back):
// local chains [first, first + n) of that render's shard, chain c = shard_index
// + j * shard_count.  u_out (n x 92): final primary samples; fp_out (n x 2): the
// trajectory fingerprint (accepted proposals, sum of the accepted steps' 1-based
// indices mod 2^32), which ora_mlt_render_shard computes the same way.
extern "C" int frt_mlt_chain_state(frt_ctx *c, uint64_t first, uint64_t n, float *u_out, uint32_t *fp_out)
{
    if (!c) return FRT_E_INVALID;
    if (c->mlt_rows == 0 || first + n > c->mlt_rows || first + n < first)
        return set_err(c, FRT_E_INVALID, "frt_mlt_chain_state: no such chains in the last PSS-MLT render");
    if (n == 0) return FRT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    std::vector<float> rows(n * kMltRow);
    HIPCHK(c, hipMemcpy(rows.data(), c->partial + first * kMltRow, rows.size() * sizeof(float), hipMemcpyDeviceToHost));
    for (uint64_t k = 0; k < n; ++k) {
        if (u_out) memcpy(u_out + k * kMltDims, rows.data() + k * kMltRow, kMltDims * sizeof(float));
        if (fp_out) memcpy(fp_out + 2 * k, rows.data() + k * kMltRow + kMltFp, 2 * sizeof(uint32_t));
    }
    return FRT_OK;
}


// Work granule of a path / AO / normals render: the frame's samples cut into
// n_chunks chunks of spi samples (the last one shorter), k = n_chunks chosen
// for at least about 40 items per resident lane and at most `target` samples
// an item (about 150 rays: path 24, AO 96, normals 128).  With one queue
// atomic per refill the first rule alone was best (Cornell 512 spp at 5-6
// chunks, profiles/r03/samecall/spi_*.jsonl); with 64-item grabs smaller items
// pay: Cornell 512 spp 289.7 ms at 6 chunks, 281.9 at 23 (flat from 16 to 64
// chunks), cornell_1m 824.1 -> 810.0 ms, while AO stays best at 6 chunks (1.5
// rays a sample; profiles/r03/samecall/grab64_spi_*.jsonl).  The target rule
// grows k with spp, so it is capped at kMaxItemsPerLane items per resident
// lane: the (chunk, slot) partial sums, 12 B an item, stay below
// kMaxItemsPerLane x the resident lanes x 12 B (~1.8 GB on MI355X) at any spp,
// and frames of any spp fit the 32-bit queue.  FRT_SPI_TARGET overrides the target (0:
// the first rule alone; A/B knob).  spi_req > 0: the caller's samples per item.
// Round 4: the chunks are the whole frame's for every shard count (films
// identical at any N), so at N = 8 a shard has an eighth of the items.  Path
// items of 8 samples under a cap of 384 items per lane (1080p 512 spp: 57 / 64
// chunks, partial sums 1.4 / 1.6 GB) keep ~40 items per lane in an eighth:
// predicted 8-way speedup of the render Cornell 6.79 -> 7.37, cornell_1m
// 6.64 -> 7.20 (shards timed alone, tools/shard_balance.py); at N = 1 Cornell
// +0.5 %, cornell_1m -0.4 % time (profiles/r04/r04g).
constexpr double kMaxItemsPerLane = 384.0;
static void work_granule(int integrator, int spp, uint64_t n_slots, long long lanes, int spi_req, int &spi,
                         int &n_chunks)
{
    spi = spi_req;
    if (spi <= 0) {
        const char *tgt = std::getenv("FRT_SPI_TARGET");
        const int target = tgt ? std::atoi(tgt)
                               : integrator == FRT_INTEGRATOR_PATH ? 8 : integrator == FRT_INTEGRATOR_AO ? 96 : 128;
        const double slots = std::max((double)n_slots, 1.0);
        const double k_lanes = std::max(1.0, std::round(40.0 * (double)lanes / slots));
        double k = k_lanes;
        if (target > 0) {
            const double k_cap = std::max(k_lanes, std::floor(kMaxItemsPerLane * (double)lanes / slots));
            k = std::max(k, std::min(std::ceil((double)spp / (double)target), k_cap));
        }
        spi = (int)std::ceil((double)spp / k);
    }
    spi = std::max(1, std::min(spi, spp));
    n_chunks = (spp + spi - 1) / spi;
}
// the granule rule for host tests (CPU): internal to libfrt.so, not in include/frt.h
extern "C" int frt_internal_work_granule(int integrator, int spp, int64_t n_slots, int64_t lanes, int spi_req,
                                         int *spi, int *n_chunks)
{
    if (spp <= 0 || n_slots < 0 || lanes <= 0 || !spi || !n_chunks) return FRT_E_INVALID;
    work_granule(integrator, spp, (uint64_t)n_slots, (long long)lanes, spi_req, *spi, *n_chunks);
    return FRT_OK;
}

static int render_impl(frt_ctx *c, const frt_render_params *p, float *dev_slots, hipStream_t st, frt_stats *stats)
{
    const auto t_start = std::chrono::steady_clock::now();
    if (!c || !p) return FRT_E_INVALID;
    if (!params_ok(p)) return set_err(c, FRT_E_INVALID, "bad render params");
    if (!c->have_scene) return set_err(c, FRT_E_NO_SCENE, "no scene uploaded");
    HIPCHK(c, hipSetDevice(c->device));
    c->mlt_rows = 0;                                   // `partial` is about to be reused
    if (p->integrator == FRT_INTEGRATOR_PSSMLT) return render_mlt(c, p, dev_slots, st, stats);
    if (p->integrator == FRT_INTEGRATOR_AO && c->has_metal)   // ao::Li -> constant_pdf::generate throws (pdf.h:195-198)
        return set_err(c, FRT_E_UNSUPPORTED, "ao integrator: metal has no sampling pdf (constant_pdf::generate)");
    const int T = eff_tile(p);
    const int nmt = my_tiles(p);
    // 32-bit slot indices: params_ok caps the frame at 2^31 - 1 pixels, so a shard's padded
    // slots stay below 2^32 (checked, not assumed: a wrap would render nothing)
    const uint64_t n_slots64 = (uint64_t)nmt * T * T;
    if (n_slots64 >= 0xffffffffULL) return set_err(c, FRT_E_UNSUPPORTED, "frame too large for one call: shard it");
    const uint32_t n_slots = (uint32_t)n_slots64;
    // kernel variant: stack depth, world kind, LDS-resident scene
    Launcher L;
    const bool f64 = use_f64(c, p);
    const int prc = pick_launcher(c, p->integrator, p->flags, L, f64);
    if (prc == FRT_E_INVALID)
        return set_err(c, prc, "fp64 render of a scene uploaded without fp64 records: frt_set_precision(FRT_PRECISION_FP64) "
                               "before frt_upload_scene");
    if (prc != FRT_OK) return set_err(c, FRT_E_UNSUPPORTED, "BVH deeper than 63 levels");
    int bpc = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, L.fn, kBlock, L.lds) != hipSuccess || bpc <= 0) bpc = 1;
    const int grid = c->n_cu * bpc;
    const long long lanes = (long long)grid * kBlock;
    // the granule follows the whole frame's slots, not the shard's: every
    // shard cuts its pixels' samples into the same chunks, so the per-pixel
    // sums (and the film) are byte-identical for any shard count
    // (tools/shard_balance.py: N = 8 of the bench frame still balances)
    const int n_tiles_frame = ((p->nx + T - 1) / T) * ((p->ny + T - 1) / T);
    int spi = 0, n_chunks = 0;
    work_granule(p->integrator, p->spp, (uint64_t)n_tiles_frame * T * T, lanes, p->samples_per_item, spi, n_chunks);
    const unsigned long long n_items = (unsigned long long)n_slots * n_chunks;
    // queue grab: items a wave takes per atomic (FRT_GRAB: A/B knob, not part of the C-ABI)
    const char *gb = std::getenv("FRT_GRAB");
    const uint32_t grab = (uint32_t)std::min(std::max(gb ? std::atoi(gb) : kQueueGrab, 1), 4096);
    // the counter runs past n_items by at most one grab per wave
    if (n_items + (unsigned long long)(lanes / 64) * (grab + 64) >= 0xffffffffULL)
        return set_err(c, FRT_E_UNSUPPORTED, "frame too large for one call: shard it");
    // workspace
    const size_t pbytes = std::max<size_t>((size_t)n_chunks * n_slots * 3 * sizeof(float), 16);
    if (pbytes > c->partial_bytes) {
        if (c->partial) HIPCHK(c, hipFree(c->partial));
        c->partial = nullptr;
        HIPCHK(c, hipMalloc(&c->partial, pbytes));
        c->partial_bytes = pbytes;
    }
    const size_t n_waves = (size_t)grid * kBlock / 64;
    if (n_waves > c->wave_rays_n) {
        if (c->wave_rays) HIPCHK(c, hipFree(c->wave_rays));
        c->wave_rays = nullptr;
        HIPCHK(c, hipMalloc(&c->wave_rays, n_waves * 4 * sizeof(unsigned long long)));
        c->wave_rays_n = n_waves;
    }
    DevWork W{};
    W.nx = p->nx; W.ny = p->ny; W.spp = p->spp; W.max_depth = p->max_depth; W.seed = p->seed;
    W.s_off = (uint32_t)p->sample_offset;
    W.tile = T; W.ntx = (p->nx + T - 1) / T; W.shard_index = p->shard_index; W.shard_count = p->shard_count;
    W.spi = spi; W.n_chunks = n_chunks; W.n_items = (uint32_t)n_items; W.n_slots = n_slots;
    W.grab = grab;
    W.partial = c->partial; W.counter = c->counter; W.wave_rays = c->wave_rays;
    W.trav_min = trav_min(L.lds_scene, p->integrator == FRT_INTEGRATOR_PATH);
    W.min_desc = min_desc(L.lds_scene);

    HIPCHK(c, hipMemsetAsync(c->counter, 0, 64, st));
#if defined(FRT_DIAG)
    if (const int drc = diag_begin(c, n_waves, st)) return drc;
#endif
    HIPCHK(c, hipEventRecord(c->ev0, st));
    DevScene Sarg = c->S;
    void *args[] = {&Sarg, &W};
    const hipError_t le = hipLaunchKernel(L.fn, dim3(grid), dim3(kBlock), args, L.lds, st);
    if (le != hipSuccess) return set_err(c, FRT_E_HIP, std::string("path_megakernel launch: ") + hipGetErrorString(le));
    HIPCHK(c, hipEventRecord(c->ev1, st));
    if (n_slots > 0) {
        hipLaunchKernelGGL(film_reduce, dim3((n_slots + 255) / 256), dim3(256), 0, st, c->partial, dev_slots, n_slots,
                           n_chunks, p->spp, T, W.ntx, p->shard_index, p->shard_count, p->nx, p->ny);
        HIPCHK(c, hipGetLastError());
    }
    std::vector<unsigned long long> wr(n_waves * 4);
    HIPCHK(c, hipMemcpyAsync(wr.data(), c->wave_rays, wr.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    float ms = 0.0f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
#if defined(FRT_DIAG)
    if (const int drc = diag_end(c, n_waves)) return drc;
#endif
    if (stats) {
        memset(stats, 0, sizeof(*stats));
        for (size_t w = 0; w < n_waves; ++w) {
            stats->camera_rays += wr[4 * w]; stats->extension_rays += wr[4 * w + 1];
            stats->shadow_rays += wr[4 * w + 2]; stats->samples += wr[4 * w + 3];
        }
        uint64_t px = 0;
        for (int t = 0; t < nmt; ++t) {
            const int tile_id = p->shard_index + t * p->shard_count;
            const int tx = tile_id % W.ntx, ty = tile_id / W.ntx;
            px += (uint64_t)std::max(0, std::min(T, p->nx - tx * T)) * std::max(0, std::min(T, p->ny - ty * T));
        }
        stats->pixels = px;
        stats->work_items = n_items;
        stats->scene_in_lds = L.lds_scene ? 1u : 0u;
        stats->waves_cap = (uint32_t)L.waves;
        stats->stack_entries = (uint32_t)L.stack;
        stats->bvh_depth = (uint32_t)(L.wide ? c->depth4 : c->stack_needed);
        stats->scene_bytes = L.lds_scene ? L.scene_lds : c->scene_lds_bytes;   // what this plan reads
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        stats->fp64 = L.f64 ? 1u : 0u;
    }
    return FRT_OK;
}

extern "C" int frt_render_device(frt_ctx *c, const frt_render_params *p, float *slots_rgb, void *hip_stream, frt_stats *st)
{
    if (!c || !slots_rgb) return FRT_E_INVALID;
    return render_impl(c, p, slots_rgb, hip_stream ? (hipStream_t)hip_stream : c->stream, st);
}

extern "C" int frt_render(frt_ctx *c, const frt_render_params *p, float *film_rgb, frt_stats *st)
{
    if (!c || !film_rgb) return FRT_E_INVALID;
    if (!params_ok(p)) return set_err(c, FRT_E_INVALID, "bad render params");
    const int64_t ns = frt_shard_slot_count(p);
    HIPCHK(c, hipSetDevice(c->device));
    const size_t bytes = std::max<size_t>((size_t)ns * 3 * sizeof(float), 16);
    if (bytes > c->slots_out_bytes) {
        if (c->slots_out) HIPCHK(c, hipFree(c->slots_out));
        c->slots_out = nullptr;
        HIPCHK(c, hipMalloc(&c->slots_out, bytes));
        c->slots_out_bytes = bytes;
    }
    const int rc = render_impl(c, p, c->slots_out, c->stream, st);
    if (rc != FRT_OK) return rc;
    std::vector<float> host((size_t)ns * 3);
    std::vector<int32_t> map((size_t)ns);
    HIPCHK(c, hipMemcpy(host.data(), c->slots_out, host.size() * sizeof(float), hipMemcpyDeviceToHost));
    if (p->integrator == FRT_INTEGRATOR_PSSMLT) {   // splat film of this shard: accumulate
        for (size_t i = 0; i < host.size(); ++i) film_rgb[i] += host[i];
        return FRT_OK;
    }
    frt_shard_slots(p, map.data());
    for (int64_t s = 0; s < ns; ++s) {
        const int32_t px = map[s];
        if (px < 0) continue;
        film_rgb[3 * (size_t)px + 0] = host[3 * s + 0];
        film_rgb[3 * (size_t)px + 1] = host[3 * s + 1];
        film_rgb[3 * (size_t)px + 2] = host[3 * s + 2];
    }
    return FRT_OK;
}

// device buffer of at least `bytes` (grown, never shrunk)
static int ensure_buf(frt_ctx *c, float **buf, size_t *have, size_t bytes)
{
    if (bytes <= *have) return FRT_OK;
    if (*buf) HIPCHK(c, hipFree(*buf));
    *buf = nullptr;
    *have = 0;
    HIPCHK(c, hipMalloc(buf, bytes));
    *have = bytes;
    return FRT_OK;
}

#define NCCLCHK(ctx, x)                                                                            \
    do {                                                                                           \
        ncclResult_t r_ = (x);                                                                     \
        if (r_ != ncclSuccess)                                                                     \
            return set_err(ctx, FRT_E_HIP, std::string(#x) + ": " + ncclGetErrorString(r_));      \
    } while (0)

// One process, n GPUs (SURVEY 8(b) frt_render_multi; what frt::path_gpu does
// in C++; the reference's task graph over rows, path.cpp:118-148).  Context i
// renders shard (i, n) -- tiles i, i + n, ... -- into its own HBM slot buffer
// on its own host thread (frt_render_device), then the buffers move device to
// device to context 0's GPU:
//   * every context on its own device: RCCL, one communicator per device
//     (ncclCommInitAll, cached on ctxs[0]), a grouped ncclSend / ncclRecv of
//     each shard's slots to rank 0 over xGMI (PSS-MLT: ncclReduce, sum);
//   * contexts sharing a device (RCCL takes one rank per device):
//     hipMemcpyPeerAsync into the same gather buffer (PSS-MLT: summed in
//     order 0..n-1 by film_add).
// Context 0 scatters the gathered slots into a device film and copies it to
// film_rgb once.  Path shards cover every pixel, so film_rgb is overwritten;
// PSS-MLT adds the summed splat film to film_rgb (as frt_render does).
// Stats: ray and sample counts summed, kernel_ms / total_ms the slowest shard's.
__global__ void film_add(float *__restrict__ dst, const float *__restrict__ src, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] += src[i];
}

extern "C" int frt_render_multi(frt_ctx **ctxs, int n, const frt_render_params *p, float *film_rgb, frt_stats *st)
{
    if (!ctxs || n <= 0 || !p || !film_rgb) return FRT_E_INVALID;
    for (int i = 0; i < n; ++i)
        if (!ctxs[i]) return FRT_E_INVALID;
    frt_ctx *c0 = ctxs[0];
    if (!params_ok(p) || p->shard_count != 1 || p->shard_index != 0)
        return set_err(c0, FRT_E_INVALID, "frt_render_multi: params must describe the whole frame (shard 0 of 1)");
    const auto t_start = std::chrono::steady_clock::now();
    const bool mlt = p->integrator == FRT_INTEGRATOR_PSSMLT;
    const size_t film_n = (size_t)p->nx * p->ny * 3;
    // per-shard slot buffers (the largest shard's size: RCCL moves equal counts)
    int64_t max_slots = 0;
    for (int i = 0; i < n; ++i) {
        frt_render_params q = *p;
        q.shard_index = i;
        q.shard_count = n;
        max_slots = std::max<int64_t>(max_slots, frt_shard_slot_count(&q));
    }
    const size_t shard_floats = (size_t)max_slots * 3;
    for (int i = 0; i < n; ++i) {
        HIPCHK(ctxs[i], hipSetDevice(ctxs[i]->device));
        const int rc = ensure_buf(ctxs[i], &ctxs[i]->slots_out, &ctxs[i]->slots_out_bytes,
                                  std::max<size_t>(shard_floats * sizeof(float), 16));
        if (rc != FRT_OK) return rc;
    }
    std::vector<frt_stats> sts(n);
    std::vector<int> rcs(n, FRT_OK);
    auto work = [&](int i) {
        frt_render_params q = *p;
        q.shard_index = i;
        q.shard_count = n;
        rcs[i] = render_impl(ctxs[i], &q, ctxs[i]->slots_out, ctxs[i]->stream, &sts[i]);
    };
    std::vector<std::thread> th;
    for (int i = 1; i < n; ++i) th.emplace_back(work, i);
    work(0);
    for (auto &t : th) t.join();
    for (int i = 0; i < n; ++i)
        if (rcs[i] != FRT_OK) {
            if (i != 0) set_err(c0, rcs[i], std::string("shard ") + std::to_string(i) + ": " + ctxs[i]->err);
            return rcs[i];
        }
    // ---- device-to-device exchange to context 0 ----
    std::vector<int> devs(n);
    bool distinct = true;
    for (int i = 0; i < n; ++i) {
        devs[i] = ctxs[i]->device;
        for (int j = 0; j < i; ++j) distinct &= devs[j] != devs[i];
    }
    HIPCHK(c0, hipSetDevice(c0->device));
    int rc = ensure_buf(c0, &c0->gather, &c0->gather_bytes, std::max<size_t>((size_t)n * shard_floats * sizeof(float), 16));
    if (rc == FRT_OK) rc = ensure_buf(c0, &c0->film_dev, &c0->film_dev_bytes, std::max<size_t>(film_n * sizeof(float), 16));
    if (rc != FRT_OK) return rc;
    if (distinct) {
        if (c0->comm_devs != devs) {
            free_comms(c0);
            c0->comms.resize(n);
            NCCLCHK(c0, ncclCommInitAll(c0->comms.data(), n, devs.data()));
            c0->comm_devs = devs;
        }
        NCCLCHK(c0, ncclGroupStart());
        for (int i = 0; i < n; ++i) {
            if (mlt) {          // the shard films summed on rank 0
                NCCLCHK(c0, ncclReduce(ctxs[i]->slots_out, i == 0 ? c0->film_dev : ctxs[i]->slots_out, film_n,
                                       ncclFloat, ncclSum, 0, c0->comms[i], ctxs[i]->stream));
            } else {            // shard i's slots -> gather[i]
                NCCLCHK(c0, ncclSend(ctxs[i]->slots_out, shard_floats, ncclFloat, 0, c0->comms[i], ctxs[i]->stream));
                NCCLCHK(c0, ncclRecv(c0->gather + (size_t)i * shard_floats, shard_floats, ncclFloat, i, c0->comms[0],
                                     c0->stream));
            }
        }
        NCCLCHK(c0, ncclGroupEnd());
        for (int i = 1; i < n; ++i) {   // rank 0's stream waits for the senders' streams
            HIPCHK(ctxs[i], hipSetDevice(ctxs[i]->device));
            HIPCHK(ctxs[i], hipStreamSynchronize(ctxs[i]->stream));
        }
        HIPCHK(c0, hipSetDevice(c0->device));
    } else {
        for (int i = 0; i < n; ++i) {
            HIPCHK(c0, hipMemcpyPeerAsync(c0->gather + (size_t)i * shard_floats, c0->device, ctxs[i]->slots_out,
                                          ctxs[i]->device, shard_floats * sizeof(float), c0->stream));
        }
        if (mlt) {
            HIPCHK(c0, hipMemsetAsync(c0->film_dev, 0, film_n * sizeof(float), c0->stream));
            for (int i = 0; i < n; ++i) {
                hipLaunchKernelGGL(film_add, dim3((unsigned)((film_n + 255) / 256)), dim3(256), 0, c0->stream,
                                   c0->film_dev, c0->gather + (size_t)i * shard_floats, film_n);
                HIPCHK(c0, hipGetLastError());
            }
        }
    }
    if (!mlt) {
        const int T = eff_tile(p);
        const uint64_t total = (uint64_t)n * (uint64_t)max_slots;
        hipLaunchKernelGGL(scatter_shards, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, c0->stream,
                           c0->gather, c0->film_dev, (uint32_t)max_slots, n, T, (p->nx + T - 1) / T, p->nx, p->ny);
        HIPCHK(c0, hipGetLastError());
    }
    if (mlt) {
        std::vector<float> host(film_n);
        HIPCHK(c0, hipMemcpyAsync(host.data(), c0->film_dev, film_n * sizeof(float), hipMemcpyDeviceToHost, c0->stream));
        HIPCHK(c0, hipStreamSynchronize(c0->stream));
        for (size_t k = 0; k < film_n; ++k) film_rgb[k] += host[k];
    } else {
        HIPCHK(c0, hipMemcpyAsync(film_rgb, c0->film_dev, film_n * sizeof(float), hipMemcpyDeviceToHost, c0->stream));
        HIPCHK(c0, hipStreamSynchronize(c0->stream));
    }
    if (st) {
        frt_stats a = sts[0];
        for (int i = 1; i < n; ++i) {
            a.camera_rays += sts[i].camera_rays; a.extension_rays += sts[i].extension_rays;
            a.shadow_rays += sts[i].shadow_rays; a.samples += sts[i].samples;
            a.pixels += mlt ? 0 : sts[i].pixels; a.work_items += sts[i].work_items;
            a.kernel_ms = std::max(a.kernel_ms, sts[i].kernel_ms);
        }
        a.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
        *st = a;
    }
    return FRT_OK;
}

#endif  // FRT_TU_LDS / FRT_TU_CHAIN / FRT_TU_MATS / main unit
