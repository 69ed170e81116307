// frt_path.hpp -- per-path logic of the integrator, __host__ __device__ so the
// HIP megakernel and the host self-test (frt_selftest_path_host) run the very
// same code.  Templated on the scalar type R like frt_device.hpp: float for
// the product kernels, double for the fp64 kernels (DESIGN.md "Precision").
// Restates (first_ray/ is fp64):
//   path::Li                  path.cpp:4-116 (iterative: one ray per step)
//   parallel_bvh_node::hit    parallel_bvh.h:39-64 (ordered stack traversal)
//   hitable_list::hit         hitable_list.cpp:4-21
//   triangle / sphere sample_direct + pdf_direct_sampling
//                             triangle.h:139-175, sphere.h:64-107
//   lambertian, diffuse_light material.h:50-73, 179-192
//   camera::get_ray           camera.h:30-35
#pragma once
#include "frt.h"
#include "frt_device.hpp"

namespace frt {

FRT_HD int f2i(float f) { return __builtin_bit_cast(int, f); }
FRT_HD float i2f(int i) { return __builtin_bit_cast(float, i); }
// materials: kMatStride float4 per material (frt_upload_scene packs them):
// m0 = (albedo | kd | metal albedo | rough eta, type), m1 = (emit | ks,
// exponent | ior | alpha), m2 = (rough k, distribution), m3 = (checker tex1
// colour, texture kind), m4 = (u_scale, v_scale, -, -)
constexpr int kMatStride = 5;
FRT_HD float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
// true if the predicate holds on any active lane of the wave (the host self-test is one lane)
FRT_HD bool wave_any(bool x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __ballot(x) != 0;
#else
    return x;
#endif
}

// number of active lanes of the wave for which x holds (host self-test: one lane)
FRT_HD int wave_count(bool x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __popcll(__ballot(x));
#else
    return x ? 1 : 0;
#endif
}

// Diagnostic build only (`make exp NAME=diag DEFS=-DFRT_DIAG`): per-phase
// lane occupancy.  FRT_DIAG_TICK(k) adds, for the executing wave, one trip and
// the number of active lanes to counter pair k of the wave's slot in
// frt_diag (read back by frt_diag_read); FRT_DIAG_CYC(k, c) adds cycles.
// Kernels launched without a buffer (frt_diag null: ray queries) count nothing;
// a launch's grid must fit the buffer the host sized for it (diag_begin).
// Compiled out of every product build.
#if defined(FRT_DIAG)
constexpr int kDiagSlots = 24;
extern __device__ unsigned long long *frt_diag;
#endif
#if defined(FRT_DIAG) && defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ unsigned long long *diag_slot()
{
    return frt_diag + (size_t)((blockIdx.x * blockDim.x + threadIdx.x) >> 6) * kDiagSlots;
}
#define FRT_DIAG_TICK(k)                                                                \
    do {                                                                                \
        const uint64_t m_ = __ballot(1);                                                \
        if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)m_) - 1 && frt_diag) { \
            unsigned long long *d_ = diag_slot();                                       \
            d_[2 * (k)] += 1;                                                           \
            d_[2 * (k) + 1] += __popcll(m_);                                            \
        }                                                                               \
    } while (0)
#define FRT_DIAG_CYC(k, c)                                                              \
    do {                                                                                \
        const uint64_t m_ = __ballot(1);                                                \
        if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)m_) - 1 && frt_diag) diag_slot()[k] += (c); \
    } while (0)
#define FRT_DIAG_CLOCK() ((unsigned long long)clock64())
#else
#define FRT_DIAG_TICK(k) do {} while (0)
#define FRT_DIAG_CYC(k, c) do {} while (0)
#define FRT_DIAG_CLOCK() 0ull
#endif

constexpr int kSentinel = 0x7fffffff;   // "stack empty"; never a node index
constexpr int kStepBranch = 0, kStepStore = 1, kStepSelect = 2;   // bvh2_step's node-visit forms
constexpr int kWorldBvh4 = 2;           // internal world kind: 4-wide quantized BVH
constexpr int kWorldBvh2Oct = 4;        // internal world kind: binary nodes from LDS, one copy per ray octant
#ifndef FRT_EXP_BVH4_OVF
#define FRT_EXP_BVH4_OVF 44             // experiment builds vary it
#endif
constexpr int kBvh4Overflow = FRT_EXP_BVH4_OVF;   // private stack entries after the LDS ones: with the 12 LDS
                                        // entries, 4-wide trees to depth 18 (3 pending siblings a level)
template <int WORLD> constexpr int kOverflow = WORLD == kWorldBvh4 ? kBvh4Overflow : 1;

// device scene (fp32, HBM-resident; DESIGN.md "Data layout")
struct DevScene {
    const float4 *nodes;     // 4 x float4 per interior node: child0 box | child1 box | (child0, child1) refs
    const float4 *tris;      // 3 x float4 per triangle: v0 | e1 | e2 (48 B), DFS leaf order
    const float4 *tshade;    // 2 x float4 per triangle: (n_geo, inv_area) | (mat, geo, -, -)
    const float4 *tnorm;     // 3 x float4 per triangle: vertex normals (smooth shading only)
    const float4 *spheres;   // (centre, radius)
    const int *sphere_mat;
    const float4 *mats;      // kMatStride x float4 per material (see kMatStride)
    const float4 *tuv;       // 2 x float4 per triangle: (uv0, uv1) | (uv2, -): texture coordinates (textured scenes)
    const float4 *texels;    // image_texture texels (rgb, -) of every image, in HBM
    const int *lights;       // device prim refs
    const int *list;         // device prim refs (list worlds)
    const int *tri_view;     // device triangle id -> scene-view triangle index (ray queries, frt_trace_device)
    const uint4 *nodes4;     // 4 x uint4 per 4-wide node (HBM-resident scenes; DESIGN.md "BVH4Q")
    const float4 *nodes_oct; // 8 copies of `nodes`, copy o with each child box as (near xyz, far xyz) for
                             // rays of octant o (bit a set: 1/d_a < 0); LDS plans copy them (kWorldBvh2Oct)
    const int2 *node_refs;   // kWorldBvh2Oct in LDS: the (child0, child1) refs of node j, shared by the
                             // 8 copies, whose records there hold only the two boxes (3 float4, 48 B)
    // fp64 records of the fp64 kernels (null when the context uploaded none,
    // frt_set_precision): the same device order as tris / tshade / tnorm /
    // spheres, in the reference's doubles (edges taken in fp64, triangle.h:58-60)
    const double4 *tris64;   // 3 per triangle: v0 | e1 | e2
    const double4 *tshade64; // (n_geo, inv_area) per triangle
    const double4 *tnorm64;  // 3 per triangle: vertex normals (smooth shading only)
    const double4 *spheres64;// (centre, radius)
    int root;                // node index, or ~prim for a single-leaf world
    int root4;               // 4-wide root node, or the same leaf ref as root
    int n_lights, n_list, world_kind;
    int n_nodes, n_tris, n_mats;
    // element i, part k of nodes / tris / tshade lives at [i * es + k * ps]:
    // interleaved in HBM (es = parts, ps = 1).  In LDS the layout keeps lanes
    // that read distinct elements on distinct bank slots: 48-B records
    // (triangles, octant node boxes: es = 3) do so interleaved, 64-B and 32-B
    // ones (binary nodes, shading records) planar (es = 1, ps = count).
    int node_es, node_ps, tri_es, tri_ps, sh_es, sh_ps, node4_es, node4_ps;
    int n_nodes4;
    float root_lo[3], root_hi[3];
    float ao_tmax;           // ao.cpp:21 world box height * 0.5
    int ao_spheres_only;     // list world: ao.cpp's t_max is NaN (see ao_shade)
    f3 cam_o, cam_llc, cam_h, cam_v, cam_u, cam_vv, cam_w;
    float lens_r, cam_half_height;
    d3 cam64_o, cam64_llc, cam64_h, cam64_v, cam64_u, cam64_vv;   // the constructed camera in fp64
    double lens_r64;
    f3 env;
};

template <typename R> struct Hit {
    int prim;     // device prim ref, -1 = miss
    R t, u, v;
};

// BVH leaf ref ~x: x = FRT_PRIM_SPHERE | k, or first triangle | (count - 1) << kLeafCountShift
// (count - 1 in bits 27..29 below the sphere flag: up to 8 triangles, 2^27 triangles per scene)
constexpr int kLeafCountShift = 27, kLeafIndexMask = (1 << kLeafCountShift) - 1, kLeafIndexLimit = 1 << kLeafCountShift;
constexpr int kLeafMax = 8, kLeafDefault = 4, kLeafSmallScene = 2;
constexpr int kTravMinLds = 12, kTravMinHbm = 32;           // PSS-MLT, AO, normals: see trav_min()
constexpr int kTravMinLdsPath = 20, kTravMinHbmPath = 40;   // path::Li
constexpr int kMinDescLds = 0, kMinDescHbm = 12;    // leaf postponing: see min_desc()

FRT_HD float4 node_part(const DevScene &S, int i, int k) { return S.nodes[i * S.node_es + k * S.node_ps]; }
FRT_HD uint4 node4_part(const DevScene &S, int i, int k) { return S.nodes4[i * S.node4_es + k * S.node4_ps]; }
// (BVH4Q child planes as exact fp16 for v_fma_mix_f32 -- one instruction per
// plane instead of a byte convert and an FMA, 80-B nodes -- measured round 5:
// node loop 166 -> 149 VALU, cornell_1m 386.3 -> 394.7 ms; not kept,
// profiles/r05/r05f/ab_m.jsonl)
constexpr int kNode4Parts = 4;
FRT_HD float4 tri_part(const DevScene &S, int i, int k) { return S.tris[i * S.tri_es + k * S.tri_ps]; }
FRT_HD float4 shade_part(const DevScene &S, int i, int k) { return S.tshade[i * S.sh_es + k * S.sh_ps]; }

// geometry records in the kernel's precision: the fp32 arrays (LDS or HBM
// strides) or the fp64 ones
template <typename R> FRT_HD V3<R> tri_vec(const DevScene &S, int i, int k)   // v0 | e1 | e2
{
    if constexpr (kIsF64<R>) return xyz(S.tris64[3 * i + k]);
    else return xyz(tri_part(S, i, k));
}
template <typename R> FRT_HD void sphere_get(const DevScene &S, int k, V3<R> &c, R &r)
{
    if constexpr (kIsF64<R>) { const double4 q = S.spheres64[k]; c = xyz(q); r = q.w; }
    else { const float4 q = S.spheres[k]; c = xyz(q); r = q.w; }
}
template <typename R> FRT_HD V3<R> geo_normal(const DevScene &S, int i)
{
    if constexpr (kIsF64<R>) return xyz(S.tshade64[i]);
    else return xyz(shade_part(S, i, 0));
}
template <typename R> FRT_HD R inv_area(const DevScene &S, int i)
{
    if constexpr (kIsF64<R>) return S.tshade64[i].w;
    else return shade_part(S, i, 0).w;
}
template <typename R> FRT_HD V3<R> vert_normal(const DevScene &S, int i, int k)
{
    if constexpr (kIsF64<R>) return xyz(S.tnorm64[3 * i + k]);
    else return xyz(S.tnorm[3 * i + k]);
}
// the constant environment colour (material.h:219-232) in the kernel's precision
template <typename R> FRT_HD V3<R> env_of(const DevScene &S) { return V3<R>{R(S.env.x), R(S.env.y), R(S.env.z)}; }
template <typename R> struct CamView { V3<R> o, llc, h, v, u, vv; R lens_r; };
template <typename R> FRT_HD CamView<R> cam_view(const DevScene &S)
{
    if constexpr (kIsF64<R>) return CamView<R>{S.cam64_o, S.cam64_llc, S.cam64_h, S.cam64_v, S.cam64_u, S.cam64_vv, S.lens_r64};
    else return CamView<R>{S.cam_o, S.cam_llc, S.cam_h, S.cam_v, S.cam_u, S.cam_vv, S.lens_r};
}

template <bool STRAIGHT = false, typename R>
FRT_HD R prim_t(const DevScene &S, int ref, V3<R> o, V3<R> d, R tmin, R tmax, R &u, R &v)
{
    if (ref & FRT_PRIM_SPHERE) {
        V3<R> c;
        R r;
        sphere_get(S, ref & ~FRT_PRIM_SPHERE, c, r);
        u = v = R(0);
        return sphere_intersect(o, d, c, r, tmin, tmax);
    }
    const V3<R> a = tri_vec<R>(S, ref, 0), b = tri_vec<R>(S, ref, 1), c = tri_vec<R>(S, ref, 2);
    return tri_intersect<STRAIGHT>(o, d, a, b, c, tmin, tmax, u, v);
}

// Leaf ~node: one sphere, or triangles [first, first + count) (collapse_leaves;
// the reference's leaves hold one prim, parallel_bvh.h:129-149).  Updates the
// closest hit with the DFS-rank tie rule; true = any-hit query satisfied.
template <bool STRAIGHT = false, typename R>   // STRAIGHT: see tri_intersect
FRT_HD bool leaf_hit(const DevScene &S, int lref, V3<R> o, V3<R> d, R tmin, bool anyhit, Hit<R> &h)
{
    if constexpr (STRAIGHT) {   // 4-wide traversal: one loop for both kinds (-1.1 % on cornell_1m split, r04d)
        const bool is_sph = (lref & FRT_PRIM_SPHERE) != 0;
        const int first = is_sph ? lref : (lref & kLeafIndexMask);
        const int count = is_sph ? 1 : (lref >> kLeafCountShift) + 1;
        for (int k = 0; k < count; ++k) {
            FRT_DIAG_TICK(1);
            const int ref = first + k;
            R u, v;
            const R t = prim_t<STRAIGHT>(S, ref, o, d, tmin, h.t, u, v);
            if (t > R(0) && ((t < h.t) || (h.prim >= 0 && (is_sph || ref < h.prim)))) {
                h.prim = ref; h.t = t; h.u = u; h.v = v;
                if (anyhit) return true;
            }
        }
        return false;
    }
    if (lref & FRT_PRIM_SPHERE) {   // a sphere leaf (one sphere)
        FRT_DIAG_TICK(1);
        R u, v;
        const R t = prim_t(S, lref, o, d, tmin, h.t, u, v);
        if (t > R(0) && ((t < h.t) || h.prim >= 0)) {
            h.prim = lref; h.t = t; h.u = u; h.v = v;
            return anyhit;
        }
        return false;
    }
    // triangles [first, first + count): no sphere test in the loop.  A hit has
    // t <= h.t (tri_intersect's t_max); at t == h.t the lower DFS rank wins,
    // and a triangle rank is below every sphere ref and never below -1 (no hit)
    const int first = lref & kLeafIndexMask;
    const int count = (lref >> kLeafCountShift) + 1;
    for (int k = 0; k < count; ++k) {
        FRT_DIAG_TICK(1);
        const int ref = first + k;
        R u, v;
        const V3<R> a = tri_vec<R>(S, ref, 0), b = tri_vec<R>(S, ref, 1), c = tri_vec<R>(S, ref, 2);
        const R t = tri_intersect<STRAIGHT>(o, d, a, b, c, tmin, h.t, u, v);
        if (t > R(0) && ((t < h.t) || ref < h.prim)) {
            h.prim = ref; h.t = t; h.u = u; h.v = v;
            if (anyhit) return true;
        }
    }
    return false;
}

// parallel_bvh_node::hit as an ordered stack traversal.  Closest hit keeps the
// reference's answer: minimum t, exact ties to the leaf that comes first in
// the left-first DFS (device triangle ids ARE that order).  Boxes are padded
// outward, so culling never removes a hit.
//
// The traversal is resumable: Trav holds a ray's whole traversal state, and
// one bvh*_step call descends to the next leaf and tests it.  The megakernel
// interleaves steps of many rays with shading (path_megakernel); trace_bvh /
// trace_bvh4 run the steps back to back.  Stack entry k lives at
// stk[k * STRIDE] (LDS column per lane on the GPU, a plain array on the
// host); the 4-wide traversal continues in `ovf` (private / scratch) after
// LSTACK entries.
template <typename R> struct Trav {
    SlabRay<R> sr;
    R tmin;
    int node, sp;
    Hit<R> h;
};

// t_min of a BVH query: EPSILON * max(1, |o|_inf) (parallel_bvh.h:46-51)
template <typename R> FRT_HD R bvh_tmin(V3<R> o)
{
    return Cst<R>::eps * vmax(R(1), vmax(vabs(o.x), vmax(vabs(o.y), vabs(o.z))));
}

// Root box with the unscaled EPSILON (parallel_bvh.h:43), then bvh_tmin.
// False: the ray misses the scene (T.h is the miss record).
template <typename R> FRT_HD bool trav_begin(Trav<R> &T, const DevScene &S, int root, V3<R> o, V3<R> d, R tmax)
{
    T.h = Hit<R>{-1, tmax, R(0), R(0)};
    T.sp = 0;
    T.node = root;
    T.sr = slab_ray(o, d);
    T.tmin = bvh_tmin(o);
    return slab_entry<R>(S.root_lo[0], S.root_lo[1], S.root_lo[2], S.root_hi[0], S.root_hi[1], S.root_hi[2], T.sr,
                         Cst<R>::eps, tmax) != R(__builtin_inff());
}

// binary nodes: descend to a leaf, test it.  True when the query is finished.
// min_desc > 0 (the megakernel's leaf postponing): the descent stops for the
// whole wave once fewer than min_desc of its lanes are still descending; those
// lanes keep their node and stack and resume on the next step, while the lanes
// that reached a leaf test it now.  A wave then no longer runs its node loop
// for as many trips as its slowest lane needs to reach a leaf.
// STEP (octant plan): how a node visit updates node / stack.  kStepBranch:
// push, descend or pop as branches.  kStepStore: the far child is written to
// the slot above the top on every visit (the stack keeps it only when both
// children were hit), the pop keeps its branch.  kStepSelect: also the entry
// below the top is read on every visit, and node / sp come from selects -- no
// branch in the loop body.  The octant plan's stack has more slots than the
// tree has levels (d < STACK), so the slot above the top is always inside the
// lane's column.  Cornell (path): Store +0.4 %, Select -0.9 %; PSS-MLT: Select
// +1.1 %, Store -0.2 %; AO / normals: Store -2.4 % / -3 % (same call, two
// alternations, profiles/r05/r05z, r05af; the Cornell kernel issued 0.48 SALU
// per VALU instruction with the branches, r05y).
// OCT (kWorldBvh2Oct): S.nodes holds the 8 octant copies; the ray's copy
// stores every child box as (near xyz, far xyz) for its direction signs, so a
// box costs 6 FMAs and two 3-way max / min instead of also sorting each
// slab's two distances (the same values: lo <= hi and 1/d has the octant's
// sign, so the near plane's distance is the smaller one).
// (Speculative traversal -- a lane that reaches a leaf parks it and keeps
// descending while other lanes of its wave have none yet, Aila & Laine 2009 --
// was measured on both plans and removed: +1 % on cornell_1m in round 1,
// -0.4 % on Cornell and -14 % on cornell_1m at 512 spp in round 3, DESIGN.md.)
template <int STRIDE, bool OCT = false, int STEP = kStepBranch, typename R>
FRT_HD bool bvh2_step(Trav<R> &T, const DevScene &S, V3<R> o, V3<R> d, bool anyhit, int *stk, int min_desc = 0)
{
    int node = T.node, sp = T.sp;
    DevScene Sn = S;
    if constexpr (OCT) {   // the ray's copy: n_nodes 48-B box records (scene_to_lds)
        const int oct = (T.sr.invd.x < R(0) ? 1 : 0) | (T.sr.invd.y < R(0) ? 2 : 0) | (T.sr.invd.z < R(0) ? 4 : 0);
        Sn.nodes = S.nodes + oct * 3 * S.n_nodes;
    }
    // (a branch-free body -- speculative stack-top read, predicated push -- was
    // 4.5 % slower on Cornell: profiles/r01_exp1_branchy.txt)
    // (OCT: t_best held finite -- a ray query may pass t_max = +inf -- so that
    // slab_nf's tn <= tf is the hit test)
    // (a node-or-leaf loop -- Aila & Laine's "if-if": each trip visits a node or
    // tests a leaf until the lane's query is done -- was 60 % slower on Cornell
    // and 50 % on PSS-MLT than this descend-then-test step: profiles/r05/r05d)
    const R tmin = T.tmin, tbest = OCT ? vmin(T.h.t, Cst<R>::tmax) : T.h.t;
    while ((unsigned)node < (unsigned)kSentinel) {   // interior node
        FRT_DIAG_TICK(2);
        R t0, t1;
        int c0, c1;
        bool h0, h1;
        if constexpr (OCT) {   // one address: the record's parts and the refs at immediate offsets
            const float4 *rec = Sn.nodes + u24mul(node, 3);   // 32-bit mad (node < 2^24)
            const float4 n0 = rec[0], n1 = rec[1], n2 = rec[2];
            const int2 cr = S.node_refs[node];
            R f0, f1;
            slab_nf<R>(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, T.sr, tmin, tbest, t0, f0);
            slab_nf<R>(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, T.sr, tmin, tbest, t1, f1);
            h0 = t0 <= f0; h1 = t1 <= f1;
            c0 = cr.x; c1 = cr.y;
            // (the 12 plane distances as 6 v_pk_fma_f32 over same-axis plane pairs: 19 VALU
            // per node instead of 25 and 4 fewer spills, yet Cornell 237.3 -> 241.8 ms, and
            // the 4-wide test's pairs 385 -> 396 ms on cornell_1m: profiles/r04/r04o.  Packed
            // f32 is no throughput lever on gfx950, MI355X_MICROARCH.md's issue-cost table.)
        } else {
            const float4 n0 = node_part(Sn, node, 0), n1 = node_part(Sn, node, 1);
            const float4 n2 = node_part(Sn, node, 2), n3 = node_part(Sn, node, 3);
            t0 = slab_entry<R>(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, T.sr, tmin, tbest);
            t1 = slab_entry<R>(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, T.sr, tmin, tbest);
            h0 = t0 != R(__builtin_inff()); h1 = t1 != R(__builtin_inff());
            c0 = f2i(n3.x); c1 = f2i(n3.y);
        }
        if constexpr (OCT && STEP == kStepSelect) {   // no branches: store above the top, read below it
            const bool first0 = h0 && (!h1 || t0 <= t1);
            const int nr = first0 ? c0 : c1, fr = first0 ? c1 : c0;
            const int below = stk[(sp > 0 ? sp - 1 : 0) * STRIDE];
            stk[sp * STRIDE] = fr;                 // the slot above the top: kept only when pushed
            const bool both = h0 && h1, any = h0 || h1;
            node = any ? nr : (sp > 0 ? below : kSentinel);
            sp += both ? 1 : (!any && sp > 0 ? -1 : 0);
        } else if constexpr (OCT && STEP == kStepStore) {   // the store without a branch, the pop with one
            const bool first0 = h0 && (!h1 || t0 <= t1);
            const int nr = first0 ? c0 : c1, fr = first0 ? c1 : c0;
            stk[sp * STRIDE] = fr;
            sp += (h0 && h1) ? 1 : 0;
            if (h0 || h1) node = nr;
            else node = (sp > 0) ? stk[--sp * STRIDE] : kSentinel;
        } else if (h0 && h1) {
            const bool first0 = t0 <= t1;
            stk[sp * STRIDE] = first0 ? c1 : c0;
            ++sp;
            node = first0 ? c0 : c1;
        } else if (h0) {
            node = c0;
        } else if (h1) {
            node = c1;
        } else {
            node = (sp > 0) ? stk[--sp * STRIDE] : kSentinel;
        }
        if (min_desc > 0 && wave_count((unsigned)node < (unsigned)kSentinel) < min_desc) break;
    }
    if ((unsigned)node < (unsigned)kSentinel) {          // postponed: still descending
        T.node = node;
        T.sp = sp;
        return false;
    }
    bool done = node == kSentinel || leaf_hit(S, ~node, o, d, T.tmin, anyhit, T.h);
    if (!done) {
        node = (sp > 0) ? stk[--sp * STRIDE] : kSentinel;
        done = node == kSentinel;
    }
    T.node = node;
    T.sp = sp;
    return done;
}

// The same query over the 4-wide quantized BVH (flatten_scene's build_bvh4):
// node = 64 B: (frame origin xyz, exponent bytes) | 4 child refs |
// 8-bit child box planes lo_x hi_x lo_y hi_y | lo_z hi_z.  A child plane is
// origin + q * 2^e; the slab test runs on the ray transformed per node
// (t = q * (2^e / d) + (origin - o) / d), so a plane costs one convert and
// one FMA.  Quantised planes round outward and the boxes keep their padding,
// so culling stays conservative and the hit equals the binary traversal's
// bit for bit (the (t, DFS rank) minimum does not depend on visit order).
// fp32 only: the fp64 kernels traverse the binary tree.
template <int STRIDE, int LSTACK>
FRT_HD bool bvh4_step(Trav<float> &T, const DevScene &S, f3 o, f3 d, bool anyhit, int *stk, int *ovf, int min_desc = 0)
{
    int node = T.node, sp = T.sp;
    // Entries below LSTACK live in the lane's LDS column, deeper ones in `ovf`
    // (scratch).  A wave-uniform test keeps the common case on plain LDS
    // accesses: a per-lane select between the two would make the compiler
    // branch per push and pop through a generic (flat) pointer.
    auto push = [&](int v) {
        if (!wave_any(sp >= LSTACK)) {
            stk[sp * STRIDE] = v;
        } else {
            if (sp < LSTACK) stk[sp * STRIDE] = v;
            else ovf[sp - LSTACK] = v;
        }
        ++sp;
    };
    auto pop = [&]() -> int {
        if (sp == 0) return kSentinel;
        --sp;
        if (!wave_any(sp >= LSTACK)) return stk[sp * STRIDE];
        return sp < LSTACK ? stk[sp * STRIDE] : ovf[sp - LSTACK];
    };
    while ((unsigned)node < (unsigned)kSentinel) {
        FRT_DIAG_TICK(0);
        const uint4 w0 = node4_part(S, node, 0), w1 = node4_part(S, node, 1);
        const uint4 w2 = node4_part(S, node, 2), w3 = node4_part(S, node, 3);
        const SlabRay<float> &sr = T.sr;
        // plane scale 2^e / d per axis: e is a signed byte (v_bfe_i32 + v_ldexp_f32; the same value as
        // the float 2^e times 1/d, which is exact in the normal range build_bvh4 keeps)
        const float ax = ldexpf(sr.invd.x, (int)(int8_t)(w0.w & 0xffu)), bx = fmaf(u2f(w0.x), sr.invd.x, sr.oinv.x);
        const float ay = ldexpf(sr.invd.y, (int)(int8_t)((w0.w >> 8) & 0xffu)), by = fmaf(u2f(w0.y), sr.invd.y, sr.oinv.y);
        const float az = ldexpf(sr.invd.z, (int)(int8_t)((w0.w >> 16) & 0xffu)), bz = fmaf(u2f(w0.z), sr.invd.z, sr.oinv.z);
        // near / far plane words per axis by the ray's direction sign: a
        // negative 1/d turns the hi plane into the entry plane.  Per child this
        // replaces the per-axis min / max of the two plane distances (the same
        // values: q_lo <= q_hi and the scale a has the sign of 1/d).  Empty
        // slots are the inverted box q_lo = 255 > q_hi = 0 with a harmless ref
        // (build_bvh4), so they need no test here.
        const bool sx = sr.invd.x < 0.0f, sy = sr.invd.y < 0.0f, sz = sr.invd.z < 0.0f;
        float t[4];
        int c[4] = {(int)w1.x, (int)w1.y, (int)w1.z, (int)w1.w};
        const uint32_t xn = sx ? w2.y : w2.x, xf = sx ? w2.x : w2.y;
        const uint32_t yn = sy ? w2.w : w2.z, yf = sy ? w2.z : w2.w;
        const uint32_t zn = sz ? w3.y : w3.x, zf = sz ? w3.x : w3.y;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int sh = 8 * i;
            const float txn = fmaf((float)((xn >> sh) & 0xffu), ax, bx), txf = fmaf((float)((xf >> sh) & 0xffu), ax, bx);
            const float tyn = fmaf((float)((yn >> sh) & 0xffu), ay, by), tyf = fmaf((float)((yf >> sh) & 0xffu), ay, by);
            const float tzn = fmaf((float)((zn >> sh) & 0xffu), az, bz), tzf = fmaf((float)((zf >> sh) & 0xffu), az, bz);
            const float tn = smax(smax(txn, tyn), smax(tzn, T.tmin));   // v_maximum3 (slab_entry)
            const float tf = smin(smin(txf, tyf), smin(tzf, T.h.t));
            t[i] = (tf < tn) ? __builtin_inff() : tn;
        }
        // nearest first: sorting network on (t, child), as selects (no branches)
        auto cx = [&](int i, int j) {
            const bool sw = t[j] < t[i];
            const float ti = sw ? t[j] : t[i], tj = sw ? t[i] : t[j];
            const int ci = sw ? c[j] : c[i], cj = sw ? c[i] : c[j];
            t[i] = ti; t[j] = tj; c[i] = ci; c[j] = cj;
        };
        // (nearest-only ordering, the rest unsorted, was 5.6 % slower on 1M: profiles/r01_exp2.txt)
        cx(0, 1); cx(2, 3); cx(0, 2); cx(1, 3); cx(1, 2);
        // hit children are sorted first; the far ones go on the stack, farthest first
        if (!wave_any(sp > LSTACK - 3)) {               // wave-uniform: every push stays in LDS
            // (unconditional writes above the top with sp advanced by the hits: cornell_1m
            // 343.5 -> 347.2 ms, profiles/r05/r05o; not kept)
            if (t[3] != __builtin_inff()) stk[sp++ * STRIDE] = c[3];
            if (t[2] != __builtin_inff()) stk[sp++ * STRIDE] = c[2];
            if (t[1] != __builtin_inff()) stk[sp++ * STRIDE] = c[1];
        } else {
            if (t[3] != __builtin_inff()) push(c[3]);
            if (t[2] != __builtin_inff()) push(c[2]);
            if (t[1] != __builtin_inff()) push(c[1]);
        }
        node = (t[0] != __builtin_inff()) ? c[0] : pop();
        if (min_desc > 0 && wave_count((unsigned)node < (unsigned)kSentinel) < min_desc) break;
    }
    if ((unsigned)node < (unsigned)kSentinel) {          // postponed (min_desc): still descending
        T.node = node;
        T.sp = sp;
        return false;
    }
    bool done = node == kSentinel || leaf_hit<true>(S, ~node, o, d, T.tmin, anyhit, T.h);
    if (!done) {
        node = pop();
        done = node == kSentinel;
    }
    T.node = node;
    T.sp = sp;
    return done;
}

template <int STRIDE, typename R>
FRT_HD Hit<R> trace_bvh(const DevScene &S, V3<R> o, V3<R> d, R tmax, bool anyhit, int *stk)
{
    Trav<R> T;
    if (trav_begin(T, S, S.root, o, d, tmax))
        while (!bvh2_step<STRIDE>(T, S, o, d, anyhit, stk)) {}
    return T.h;
}

template <int STRIDE, int LSTACK, int OVF>
FRT_HD Hit<float> trace_bvh4(const DevScene &S, f3 o, f3 d, float tmax, bool anyhit, int *stk)
{
    Trav<float> T;
    int ovf[OVF];
    if (trav_begin(T, S, S.root4, o, d, tmax))
        while (!bvh4_step<STRIDE, LSTACK>(T, S, o, d, anyhit, stk, ovf)) {}
    return T.h;
}

// hitable_list::hit: in list order, triangles strict '<', spheres inclusive (sphere.h:34).
// (A per-prim fp32 box test before the primitive test was 12-15 % slower on
// veach_mis in both precisions -- its big plates and floor pass their boxes:
// profiles/r03/r03c_ab_veach_listbox_f64waves.jsonl.)
template <typename R> FRT_HD Hit<R> trace_list(const DevScene &S, V3<R> o, V3<R> d, R tmax, bool anyhit)
{
    Hit<R> h{-1, tmax, R(0), R(0)};
    for (int i = 0; i < S.n_list; ++i) {
#if defined(__HIP_DEVICE_COMPILE__)   // every lane tests the same entry: a scalar load
        const int ref = frt_uniform(((const __attribute__((address_space(4))) int *)S.list)[frt_uniform(i)]);
#else
        const int ref = S.list[i];
#endif
        R u, v;
#if defined(__HIP_DEVICE_COMPILE__)
        // fp64 (C3): the uniform entry's records through the constant address space as
        // indexed base pointers, so that the compiler reads them with scalar loads (the
        // entry, the sphere and all three vertex records; the form matters -- an offset
        // pointer left v0 and the sphere as vector loads).  veach 256 spp, same call:
        // 201.7 / 201.4 ms -> 187.2 / 187.2 with the vertex records v1 / v2 scalar
        // (profiles/r05/r05aj), -> 174.9 / 174.8 with every load scalar (r05am)
        R t;
        if constexpr (kIsF64<R>) {
            typedef const __attribute__((address_space(4))) double4 *cptr;
            if (ref & FRT_PRIM_SPHERE) {
                const cptr sb = (cptr)S.spheres64;
                const double4 q = sb[ref & ~FRT_PRIM_SPHERE];
                u = v = R(0);
                t = sphere_intersect(o, d, xyz(q), q.w, Cst<R>::eps, h.t);
            } else {
                const cptr tb = (cptr)S.tris64;
                const double4 a = tb[3 * ref], b = tb[3 * ref + 1], c = tb[3 * ref + 2];
                t = tri_intersect(o, d, xyz(a), xyz(b), xyz(c), Cst<R>::eps, h.t, u, v);
            }
        } else {   // fp32 list kernels: the same scalar loads of the fp32 records
            typedef const __attribute__((address_space(4))) float4 *cptr;
            if (ref & FRT_PRIM_SPHERE) {
                const cptr sb = (cptr)S.spheres;
                const float4 q = sb[ref & ~FRT_PRIM_SPHERE];
                u = v = R(0);
                t = sphere_intersect(o, d, xyz(q), q.w, Cst<R>::eps, h.t);
            } else {
                const cptr tb = (cptr)S.tris;
                const float4 a = tb[ref * S.tri_es], b = tb[ref * S.tri_es + S.tri_ps], c = tb[ref * S.tri_es + 2 * S.tri_ps];
                t = tri_intersect(o, d, xyz(a), xyz(b), xyz(c), Cst<R>::eps, h.t, u, v);
            }
        }
#else
        const R t = prim_t(S, ref, o, d, Cst<R>::eps, h.t, u, v);
#endif
        if (t > R(0) && ((ref & FRT_PRIM_SPHERE) || t < h.t)) {
            h.prim = ref; h.t = t; h.u = u; h.v = v;
            if (anyhit) return h;
        }
    }
    return h;
}

template <int WORLD, int STRIDE, int STACK = 0, typename R>
FRT_HD Hit<R> trace(const DevScene &S, V3<R> o, V3<R> d, R tmax, bool anyhit, int *stk)
{
    if constexpr (WORLD == FRT_WORLD_LIST) return trace_list(S, o, d, tmax, anyhit);
    else if constexpr (WORLD == kWorldBvh4) return trace_bvh4<STRIDE, STACK, kBvh4Overflow>(S, o, d, tmax, anyhit, stk);
    else return trace_bvh<STRIDE>(S, o, d, tmax, anyhit, stk);
}

// resumable form of trace<> (path_megakernel): begin, then steps until true
template <int WORLD, typename R>
FRT_HD bool trav_begin_world(Trav<R> &T, const DevScene &S, V3<R> o, V3<R> d, R tmax)
{
    if constexpr (WORLD == FRT_WORLD_LIST) {
        T.h = Hit<R>{-1, tmax, R(0), R(0)};
        return true;
    } else {
        return trav_begin(T, S, WORLD == kWorldBvh4 ? S.root4 : S.root, o, d, tmax);
    }
}
template <int WORLD, int STRIDE, int STACK, int STEP = kStepBranch, typename R>
FRT_HD bool trav_step_world(Trav<R> &T, const DevScene &S, V3<R> o, V3<R> d, bool anyhit, int *stk, int *ovf,
                            int min_desc = 0)
{
    // 4-wide (HBM-resident scenes): the slab ray and t_min again from (o, d)
    // (the values trav_begin set), so that they are not live across the
    // megakernel's shading phases (spilled VGPRs 81 -> 36 at the 6-wave cap;
    // cornell_1m +2.8 %, same-call A/B).  The binary LDS plan keeps them.
    if constexpr (WORLD == kWorldBvh4) {
        static_assert(!kIsF64<R>, "the fp64 kernels traverse the binary tree");
        T.sr = slab_ray(o, d);
        T.tmin = bvh_tmin(o);
    }
    if constexpr (WORLD == FRT_WORLD_LIST) {
        T.h = trace_list(S, o, d, T.h.t, anyhit);
        return true;
    } else if constexpr (WORLD == kWorldBvh4) {
        return bvh4_step<STRIDE, STACK>(T, S, o, d, anyhit, stk, ovf, min_desc);
    } else {
        return bvh2_step<STRIDE, WORLD == kWorldBvh2Oct, STEP>(T, S, o, d, anyhit, stk, min_desc);
    }
}

// hit record of a primitive: shading normal + material
template <typename R>
FRT_HD void prim_shade(const DevScene &S, int ref, V3<R> ro, V3<R> p, R u, R v, V3<R> &n, int &mat)
{
    if (ref & FRT_PRIM_SPHERE) {                               // sphere.h:47-50
        const int k = ref & ~FRT_PRIM_SPHERE;
        V3<R> c;
        R r;
        sphere_get(S, k, c, r);
        n = rcp(r) * (p - c);
        if (len2(ro - c) < r * r) n = -n;                      // origin inside: flip
        mat = S.sphere_mat[k];
        return;
    }
    const float4 s1 = shade_part(S, ref, 1);
    mat = f2i(s1.x);
    if (f2i(s1.y)) {                                           // use_geometry_normals (triangle.h:100-101)
        n = geo_normal<R>(S, ref);
    } else {                                                   // triangle.h:103
        const V3<R> n0 = vert_normal<R>(S, ref, 0), n1 = vert_normal<R>(S, ref, 1), n2 = vert_normal<R>(S, ref, 2);
        n = normalize((R(1) - u - v) * n0 + u * n1 + v * n2);
    }
}

// pdf_direct_sampling with the record's (p, t, normal) and direction
template <typename R>
FRT_HD R prim_pdf(const DevScene &S, int ref, V3<R> rec_p, R rec_t, V3<R> rec_n, V3<R> to_light)
{
    if (!(ref & FRT_PRIM_SPHERE)) return inv_area<R>(S, ref);    // triangle.h:139-144
    V3<R> c;                                                     // sphere.h:64-78
    R r;
    sphere_get(S, ref & ~FRT_PRIM_SPHERE, c, r);
    const V3<R> o = rec_p - rec_t * to_light;
    const V3<R> dir = c - o;
    const R d2 = len2(dir);
    const R r2 = r * r;
    if (d2 <= r2) return rcp(R(4) * Cst<R>::pi * r2);
    const R cos_max = fsqrt(R(1) - fdiv(r2, d2));
    const R solid = R(2) * Cst<R>::pi * (R(1) - cos_max);
    return fdiv(rcp(solid) * vabs(dot(to_light, rec_n)), d2);
}

// sample_direct: returns to_light (unnormalised, as the reference), light normal, material
template <typename R>
FRT_HD V3<R> prim_sample(const DevScene &S, int ref, V3<R> o, R u0, R u1, V3<R> &ln, int &lmat)
{
    if (ref & FRT_PRIM_SPHERE) {                                   // sphere.h:80-107
        const int k = ref & ~FRT_PRIM_SPHERE;
        V3<R> c;
        R r;
        sphere_get(S, k, c, r);
        lmat = S.sphere_mat[k];
        const V3<R> direction = c - o;
        const R d2 = len2(direction);
        if (d2 <= r * r) {
            const V3<R> p = c + r * uniform_sphere(u0, u1);
            ln = normalize(c - p);
            return p - o;
        }
        const Onb<R> uvw = onb_from_w(direction);                  // unnormalised axis, as the reference
        const V3<R> p = onb_local(uvw, random_to_sphere(r, d2, u0, u1));
        ln = normalize(p);
        return p;
    }
    const V3<R> a = tri_vec<R>(S, ref, 0), b = tri_vec<R>(S, ref, 1), c = tri_vec<R>(S, ref, 2);   // triangle.h:145-175
    const R su0 = fsqrt(u0);
    const R b0 = R(1) - su0;
    const R b1 = u1 * su0;
    const V3<R> lp = a + b0 * b + b1 * c;                          // (1-b0-b1) v0 + b0 v1 + b1 v2
    const float4 s1 = shade_part(S, ref, 1);
    lmat = f2i(s1.x);
    if (f2i(s1.y)) {
        ln = geo_normal<R>(S, ref);
    } else {
        const V3<R> n0 = vert_normal<R>(S, ref, 0), n1 = vert_normal<R>(S, ref, 1), n2 = vert_normal<R>(S, ref, 2);
        ln = normalize((R(1) - b0 - b1) * n0 + b0 * n1 + b1 * n2);
    }
    return lp - o;
}

// Material sets a kernel is compiled for (the MATS template mask): the
// lambertian / diffuse_light core is always there; kMatsTex adds checker
// textures, kMatsSpec the specular branch for modified_phong, metal and
// dielectric, kMatsRough the rough conductor lobes (erf / erfinv, GGX slopes,
// conductor Fresnel) -- the register-hungry part.  A scene runs the smallest
// kernel covering its materials (frt_upload_scene).
constexpr int kMatsNone = 0, kMatsTex = 1, kMatsSpec = 2, kMatsRough = 4, kMatsAll = 7;
constexpr int kMatsSpecAny = kMatsSpec | kMatsRough;

// ---- textures (texture.h:30-49), MATS kernels only ----
// (int)x as the reference's x86-64 build computes it (cvttsd2si): NaN and
// out-of-range give INT_MIN
template <typename R> FRT_HD int x86_trunc(R x)
{
    if (!(x > R(-2147483649.0f) && x < R(2147483648.0f))) return (int)0x80000000;
    return (int)x;
}
FRT_HD int imodulo2(int a) { const int r = a % 2; return r < 0 ? r + 2 : r; }   // util.h:125-128
FRT_HD float vatan2(float y, float x) { return atan2f(y, x); }
FRT_HD double vatan2(double y, double x) { return atan2(y, x); }
FRT_HD float vasin(float x) { return asinf(x); }
FRT_HD double vasin(double x) { return asin(x); }
// hit texture coordinates: get_sphere_uv(p - centre) (hitable.h:15-21; the
// offset is not normalised, as in sphere.h:52) or the OBJ vt interpolated
// with the barycentrics (triangle.h:105-107)
template <typename R> FRT_HD void prim_uv(const DevScene &S, int ref, V3<R> p, R u, R v, R &tu, R &tv)
{
    if (ref & FRT_PRIM_SPHERE) {
        V3<R> c;
        R r;
        sphere_get(S, ref & ~FRT_PRIM_SPHERE, c, r);
        const V3<R> q = p - c;
        const R phi = vatan2(q.z, q.x), theta = vasin(q.y);
        tu = R(1) - (phi + Cst<R>::pi) / (R(2) * Cst<R>::pi);
        tv = (theta + R(0.5f) * Cst<R>::pi) / Cst<R>::pi;
        return;
    }
    const float4 a = S.tuv[2 * ref], b = S.tuv[2 * ref + 1];
    const R w = R(1) - u - v;
    tu = (w * R(a.x) + u * R(a.z)) + v * R(b.x);
    tv = (w * R(a.y) + u * R(a.w)) + v * R(b.y);
}
// checker_texture::value: the material's textured colour (m0 for lambertian /
// modified_phong, m1 for dielectric / rough_conductor) becomes tex1 where
// x * y == 1 (texture.h:37-41)
FRT_HD int imodulo(int a, int b) { const int r = a % b; return r < 0 ? r + b : r; }   // util.h:125-128
// image_texture::value (texture.h:59-88): the nearest texel at (u nx, v ny) in
// stb's row order, indices outside [0, n] wrapped, n clamped to n - 1; the
// texels hold the reference's linear value (FromSrgb(byte / 255) or the HDR
// float) per texel, so only the index arithmetic runs here (fp32: a texel edge
// can round to the neighbour, as the checker's cell edges do)
template <typename R> FRT_HD f3 image_texel(const DevScene &S, float4 m4, R tu, R tv)
{
    const int nx = f2i(m4.x), ny = f2i(m4.y);
    int i = x86_trunc(tu * (R)nx), j = x86_trunc(tv * (R)ny);
    if (i < 0 || i > nx) i = imodulo(i, nx);
    if (j < 0 || j > ny) j = imodulo(j, ny);
    if (i == nx) i = nx - 1;
    if (j == ny) j = ny - 1;
    return xyz(S.texels[f2i(m4.z) + j * nx + i]);
}
template <typename R>
FRT_HD void apply_texture(const DevScene &S, int mat, int mtype, int ref, V3<R> p, R u, R v, float4 &m0, float4 &m1)
{
    const float4 m3 = S.mats[kMatStride * mat + 3];
    const int tex = f2i(m3.w);
    if (tex == FRT_TEX_CONSTANT) return;
    const float4 m4 = S.mats[kMatStride * mat + 4];
    R tu, tv;
    prim_uv(S, ref, p, u, v, tu, tv);
    f3 c;
    if (tex == FRT_TEX_IMAGE) {
        c = image_texel(S, m4, tu, tv);
    } else {
        const int x = 2 * imodulo2(x86_trunc(tu * R(m4.x) * R(2))) - 1, y = 2 * imodulo2(x86_trunc(tv * R(m4.y) * R(2))) - 1;
        if (x * y != 1) return;
        c = xyz(m3);
    }
    if (mtype == FRT_MAT_LAMBERTIAN || mtype == FRT_MAT_MODIFIED_PHONG) { m0.x = c.x; m0.y = c.y; m0.z = c.z; }
    else { m1.x = c.x; m1.y = c.y; m1.z = c.z; }
}

// ---------------------------------------------------------------------------
// one path as a state machine: begin() makes the camera ray, shade() consumes
// the hit of the ray just traced and sets up the next one (shadow first,
// then the extension ray) or finishes the path.
// ---------------------------------------------------------------------------
template <typename R> struct PathState {
    V3<R> ro, rd;         // ray to trace next
    R rtmax;
    bool shadow;          // any-hit query
    bool term;            // the path ends after this shadow ray (zero bsdf pdf)
    V3<R> beta, L;        // throughput, radiance of this sample
    V3<R> nee;            // NEE contribution if the shadow ray is unoccluded
    V3<R> nxt_d;          // extension direction after the shadow ray
    V3<R> nxt_o;          // its origin when it differs from the shadow ray's (specular kernels only)
    V3<R> prev_p;         // previous hit point (MIS distance, path.cpp:25)
    R prev_pdf;           // bsdf pdf of the previous bounce
    bool prev_spec;       // previous bounce was modified_phong / metal / dielectric: no MIS on light hits
    int depth;
    RngKey key;
};

// path.cpp:129-136 + camera.h:30-35 (+ util.h:21-41 thin lens)
template <typename R>
FRT_HD void path_begin(PathState<R> &P, const DevScene &S, int px, int py, int nx, int ny, uint32_t seed,
                       uint32_t pixel, uint32_t sample)
{
    P.key = rng_key(seed, pixel, sample);
    const CamView<R> cam = cam_view<R>(S);
    const R u = fdiv((R)px + rng_r<R>(P.key, 0), (R)nx);
    const R v = fdiv((R)py + rng_r<R>(P.key, 1), (R)ny);
    V3<R> off = zero3<R>();
    if (cam.lens_r != R(0)) {
        const R a = rng_r<R>(P.key, 2) * R(2) - R(1), b = rng_r<R>(P.key, 3) * R(2) - R(1);
        R rx = R(0), ry = R(0);
        if (a != R(0) || b != R(0)) {
            R r, phi;
            if (a * a > b * b) { r = a; phi = (Cst<R>::pi / R(4)) * (b / a); }
            else { r = b; phi = (Cst<R>::pi / R(2)) - (Cst<R>::pi / R(4)) * (a / b); }
            rx = r * vcos(phi); ry = r * vsin(phi);
        }
        off = (cam.lens_r * rx) * cam.u + (cam.lens_r * ry) * cam.vv;
    }
    P.ro = cam.o + off;
    P.rd = ((cam.llc + u * cam.h + v * cam.v) - cam.o) - off;
    P.rtmax = Cst<R>::tmax;
    P.shadow = false;
    P.term = false;
    P.depth = 0;
    P.beta = V3<R>{R(1), R(1), R(1)};
    P.L = zero3<R>();
    P.prev_pdf = R(0);
    P.prev_p = zero3<R>();
    P.prev_spec = false;
}

// Shadow ray done (path.cpp:50-77): add the NEE term if unoccluded, then the
// extension ray.  The megakernel runs this inside its traversal loop, so
// shading phases only see closest-hit results.  Lambertian bounces leave from
// the NEE origin (p + eps n); specular ones may leave from the other side
// (path.cpp:91-93), so the specular kernels carry the origin (MATS).
// Returns false when the path ends here: its scattered direction had pdf 0,
// so the reference returns 0 for the vertex after tracing the shadow ray
// (path.cpp:45-77 run before :87-90 / :103-106) -- the ray is traced and
// counted like the reference's, its NEE term dropped.
template <int MATS = kMatsAll, typename R>
FRT_HD bool path_after_shadow(PathState<R> &P, bool unoccluded)
{
    P.shadow = false;
    if (P.term) return false;
    if (unoccluded) P.L = P.L + P.nee;
    if constexpr ((MATS & kMatsSpecAny) != 0) P.ro = P.nxt_o;
    P.rd = P.nxt_d; P.rtmax = Cst<R>::tmax;
    ++P.depth;
    return true;
}

// The specular materials of path.cpp:78-95 behind one interface (the
// oracle's spec_generate / spec_value / spec_eval): modified_phong, metal,
// dielectric, rough_conductor.
struct SpecMat {
    int type;
    float4 m0, m1, m2;
};
FRT_HD SpecMat spec_mat(const DevScene &S, int mat, int type, float4 m0, float4 m1)
{
    SpecMat M{type, m0, m1, make_float4(0.0f, 0.0f, 0.0f, 0.0f)};
    if (type == FRT_MAT_ROUGH_CONDUCTOR) M.m2 = S.mats[kMatStride * mat + 2];
    return M;
}
// scatter's direction from the get3d sample (material.h:83-88, 117-119, 139-145,
// 262-268) and srec.sampled_pdf (-1 unless the rough conductor sets it)
// MATS without kMatsRough: the scene has no rough conductor, its lobes are
// not compiled (the switch's default is then metal's).
template <int MATS = kMatsAll, typename R>
FRT_HD V3<R> spec_generate(const SpecMat &M, V3<R> n, V3<R> wi, R s0, R s1, R &sampled_pdf)
{
    sampled_pdf = R(-1);
    switch (M.type) {
    case FRT_MAT_MODIFIED_PHONG: return cosine_power_generate(n, wi, R(M.m1.w), s0, s1);
    case FRT_MAT_DIELECTRIC: return dielectric_generate(n, wi, R(M.m1.w), s0);
    case FRT_MAT_METAL: return reflect(-wi, n);          // reflect(unit(r_in.d), n); -wi = unit(r_in.d)
    default:
        if constexpr ((MATS & kMatsRough) != 0)
            return normalize(rough_generate(n, wi, R(M.m1.w), f2i(M.m2.w), s0, s1, sampled_pdf));
        return reflect(-wi, n);
    }
}
template <int MATS = kMatsAll, typename R>
FRT_HD R spec_value(const SpecMat &M, V3<R> n, V3<R> wi, V3<R> wo)     // srec.pdf_ptr->value
{
    switch (M.type) {
    case FRT_MAT_MODIFIED_PHONG: return cosine_power_value(n, wi, R(M.m1.w), wo);
    case FRT_MAT_DIELECTRIC: return dielectric_value(n, wi, R(M.m1.w), wo);
    case FRT_MAT_METAL: return R(1);                     // constant_pdf(1) (pdf.h:186-201)
    default:
        if constexpr ((MATS & kMatsRough) != 0) return rough_value(n, wi, R(M.m1.w), f2i(M.m2.w), wo);
        return R(1);
    }
}
template <int MATS = kMatsAll, typename R>
FRT_HD V3<R> spec_eval(const SpecMat &M, V3<R> n, V3<R> wi, V3<R> wo)          // eval_bsdf
{
    switch (M.type) {
    case FRT_MAT_MODIFIED_PHONG: return phong_eval(rgb<R>(M.m0), rgb<R>(M.m1), R(M.m1.w), n, wi, wo);
    case FRT_MAT_DIELECTRIC: return dielectric_eval(rgb<R>(M.m1), R(M.m1.w), n, wi, wo);
    case FRT_MAT_METAL: return rgb<R>(M.m0);
    default:
        if constexpr ((MATS & kMatsRough) != 0)
            return rough_eval(rgb<R>(M.m0), rgb<R>(M.m2), rgb<R>(M.m1), R(M.m1.w), f2i(M.m2.w), n, wi, wo);
        return rgb<R>(M.m0);
    }
}
FRT_HD bool mat_is_specular(int t)
{
    return t == FRT_MAT_MODIFIED_PHONG || t == FRT_MAT_METAL || t == FRT_MAT_DIELECTRIC || t == FRT_MAT_ROUGH_CONDUCTOR;
}
// light hits after these return Le unweighted (path.cpp:18-22)
FRT_HD bool mat_no_mis(int t) { return t == FRT_MAT_MODIFIED_PHONG || t == FRT_MAT_METAL || t == FRT_MAT_DIELECTRIC; }

// Returns true when the path is finished (P.L is the sample's radiance).
// MATS = false compiles the lambertian / diffuse_light scenes' kernel: the
// specular branch is dead code there (it would cost registers and code size).
template <int MATS = kMatsAll, typename R>
FRT_HD bool path_shade(PathState<R> &P, const DevScene &S, const Hit<R> &h, int max_depth, uint32_t &n_ext, uint32_t &n_sh)
{
    if (P.shadow) {
        if (!path_after_shadow<MATS>(P, h.prim < 0)) return true;
        ++n_ext;
        return false;
    }
    if (P.term) return true;                            // finished in the traversal loop
    if (h.prim < 0) {                                   // path.cpp:115 environment
        P.L = P.L + P.beta * env_of<R>(S);
        return true;
    }
    const V3<R> p = P.ro + h.t * P.rd;
    V3<R> n;
    int mat;
    prim_shade(S, h.prim, P.ro, p, h.u, h.v, n, mat);
    float4 m0 = S.mats[kMatStride * mat], m1 = S.mats[kMatStride * mat + 1];
    const int mtype = f2i(m0.w);
    if constexpr ((MATS & kMatsTex) != 0) apply_texture(S, mat, mtype, h.prim, p, h.u, h.v, m0, m1);
    // diffuse_light::emitted is one-sided (material.h:184-190)
    if (mtype == FRT_MAT_DIFFUSE_LIGHT && dot(n, P.rd) < R(0)) {
        const V3<R> Le = rgb<R>(m1);
        if (P.depth == 0 || P.prev_spec) {
            P.L = P.L + P.beta * Le;                    // path.cpp:16-22 (camera ray / after phong, metal, dielectric)
        } else {                                        // path.cpp:24-31: MIS against the bsdf sample
            const R cos_wo = dot(n, -normalize(P.rd));
            R d2 = len2(p - P.prev_p);
            if (d2 <= Cst<R>::eps) d2 = Cst<R>::eps;
            const R light_pdf = fdiv(prim_pdf(S, h.prim, p, h.t, n, P.rd) * d2, vabs(cos_wo));
            P.L = P.L + mi_weight(P.prev_pdf, light_pdf) * (P.beta * Le);
        }
        return true;
    }
    const bool lamb = mtype == FRT_MAT_LAMBERTIAN, spec = (MATS & kMatsSpecAny) && mat_is_specular(mtype);
    if (!(lamb || spec) || P.depth > max_depth) return true;   // no scatter: Le (= 0)
    const bool diel = (MATS & kMatsSpec) && mtype == FRT_MAT_DIELECTRIC;
    const uint32_t base = dim_bounce(P.depth);
    // The scattered direction first: a zero pdf returns 0 for this vertex,
    // dropping its NEE too (path.cpp:84-86, 103-106) -- after the reference has
    // traced the shadow ray, so that ray is still traced (P.term).
    V3<R> wo, beta_next;
    R pdf;
    const V3<R> wi = -normalize(P.rd);                  // hrec.wi (triangle.h:108, sphere.h:47)
    SpecMat M{};
    if (!(MATS & kMatsSpecAny) || lamb) {               // cosine_pdf (path.cpp:96-110)
        const Onb<R> uvw = onb_from_w(n);
        wo = onb_local(uvw, cosine_direction(rng_r<R>(P.key, base + 6), rng_r<R>(P.key, base + 7)));
        const R cw = dot(n, normalize(wo));
        pdf = vmax(cw, R(0)) * Cst<R>::inv_pi;
        beta_next = fdiv(vabs(cw), pdf) * (P.beta * (Cst<R>::inv_pi * rgb<R>(m0)));   // lambertian::eval_bsdf
    } else {                                            // specular branch (path.cpp:78-95); the
        M = spec_mat(S, mat, mtype, m0, m1);            // scatter sample is get3d's (base + 0, 1)
        R sampled;
        wo = spec_generate<MATS>(M, n, wi, rng_r<R>(P.key, base + 0), rng_r<R>(P.key, base + 1), sampled);
        pdf = spec_value<MATS>(M, n, wi, wo);
        if (sampled > R(0)) pdf = sampled;              // path.cpp:82
        const V3<R> bsdf = spec_eval<MATS>(M, n, wi, wo);
        beta_next = P.beta * (rcp(pdf) * bsdf);
    }
    // Lambertian-only kernels (MATS = false) never see pdf 0: the cosine lobe's
    // z = sqrt(1 - r0) >= 2^-12 (r0 < 1 - 2^-24), far above the rounding of
    // dot(n, wo); the constant lets the compiler drop the state.
    // NEE's light pick (path.cpp:39-40)
    const int nl = S.n_lights;
    int idx = (int)(rng_r<R>(P.key, base + 3) * (R)nl);
    if (idx == nl) idx -= 1;
    const bool nee = idx >= 0 && !diel;
    P.term = (MATS & kMatsSpecAny) && pdf == R(0);
    if (P.term && !nee) return true;
    // origin of the next ray: off the surface on the side it leaves (path.cpp:91-93, 99)
    const V3<R> nee_o = p + Cst<R>::eps * n;
    const V3<R> origin = (!(MATS & kMatsSpecAny) || lamb || dot(n, wo) > R(0)) ? nee_o : p - Cst<R>::eps * n;
    P.nxt_d = wo;
    if constexpr ((MATS & kMatsSpecAny) != 0) P.nxt_o = origin;
    // next-event estimation (path.cpp:38-77); not from dielectrics (path.cpp:40)
    if (nee) {
        const int lref = S.lights[idx];
        V3<R> ln;
        int lmat;
        const V3<R> tl = prim_sample(S, lref, nee_o, rng_r<R>(P.key, base + 4), rng_r<R>(P.key, base + 5), ln, lmat);
        const R dist2 = len2(tl);
        const V3<R> tu = rlen(tl) * tl;
        const R cos_wi = dot(n, tu);
        const R cos_lo = dot(ln, -tu);
        P.nee = zero3<R>();
        if (cos_lo != R(0)) {
            const R light_pdf = fdiv(prim_pdf(S, lref, p, h.t, n, tu) * dist2, vabs(cos_lo));
            // eval_bsdf toward the light; only the non-specular bsdf gets the cosine (path.cpp:61-62)
            const bool l = !(MATS & kMatsSpecAny) || lamb;
            const V3<R> f = l ? cos_wi * (Cst<R>::inv_pi * rgb<R>(m0)) : spec_eval<MATS>(M, n, wi, tu);
            const R bsdf_pdf = l ? vmax(cos_wi, R(0)) * Cst<R>::inv_pi : spec_value<MATS>(M, n, wi, tu);
            const R wgt = mi_weight(light_pdf, bsdf_pdf);
            const float4 lm0 = S.mats[kMatStride * lmat], lm1 = S.mats[kMatStride * lmat + 1];
            if (f2i(lm0.w) == FRT_MAT_DIFFUSE_LIGHT && dot(ln, tu) < R(0))
                P.nee = fdiv(wgt, light_pdf) * (P.beta * (rgb<R>(lm1) * f));
        }
        P.ro = nee_o; P.rd = tl; P.rtmax = R(1) - Cst<R>::shadow_eps;
        P.shadow = true;
        ++n_sh;
    }
    P.prev_spec = (MATS & kMatsSpec) && mat_no_mis(mtype);
    P.beta = beta_next;
    P.prev_p = p;
    P.prev_pdf = pdf;
    if (!P.shadow) {
        P.ro = origin; P.rd = wo; P.rtmax = Cst<R>::tmax;
        ++P.depth; ++n_ext;
    }
    return false;
}

// ---- the reference's other integrators on the same traversal ----

// ao::Li (ao.cpp:4-27).  Camera hit on a scattering material: one
// visibility ray from the hit point (no offset, ao.cpp:15) along the
// material pdf's generate() -- dims dim_bounce(0) + 6, 7 -- up to
// S.ao_tmax (half the world box height, ao.cpp:19-21); occluded -> 0,
// otherwise, and for misses and lights, the environment.  The visibility
// ray is an any-hit query traced like path's shadow rays.  List worlds
// have no box (hitable_list::bounding_box returns before assigning it,
// hitable_list.cpp:27-29: t_max is NaN): only spheres can occlude there
// (sphere.h's `t > t_max` test passes NaN, triangle.h's `t < t_max` does
// not), answered here with a loop over the list's spheres.
template <int MATS = kMatsAll, typename R>
FRT_HD bool ao_shade(PathState<R> &P, const DevScene &S, const Hit<R> &h, uint32_t &n_sh)
{
    const V3<R> env = env_of<R>(S);
    if (P.shadow) {                                     // visibility ray done
        P.L = h.prim < 0 ? env : zero3<R>();
        return true;
    }
    P.L = env;
    if (h.prim < 0) return true;
    const V3<R> p = P.ro + h.t * P.rd;
    V3<R> n;
    int mat;
    prim_shade(S, h.prim, P.ro, p, h.u, h.v, n, mat);
    const float4 m0 = S.mats[kMatStride * mat], m1 = S.mats[kMatStride * mat + 1];
    const int mtype = f2i(m0.w);
    const uint32_t base = dim_bounce(0);
    const R u0 = rng_r<R>(P.key, base + 6), u1 = rng_r<R>(P.key, base + 7);
    V3<R> wo;
    if (mtype == FRT_MAT_LAMBERTIAN) {
        wo = onb_local(onb_from_w(n), cosine_direction(u0, u1));
    } else if ((MATS & kMatsSpec) && mtype == FRT_MAT_MODIFIED_PHONG) {
        wo = cosine_power_generate(n, -normalize(P.rd), R(m1.w), u0, u1);
    } else if ((MATS & kMatsSpec) && mtype == FRT_MAT_DIELECTRIC) {
        wo = dielectric_generate(n, -normalize(P.rd), R(m1.w), u0);
    } else if ((MATS & kMatsRough) && mtype == FRT_MAT_ROUGH_CONDUCTOR) {   // pdf.h:465-482 (metal: refused at launch)
        const float4 m2 = S.mats[kMatStride * mat + 2];
        R unused;
        if constexpr ((MATS & kMatsRough) != 0) wo = rough_generate(n, -normalize(P.rd), R(m1.w), f2i(m2.w), u0, u1, unused);
    } else {
        return true;                                    // no scatter (diffuse_light)
    }
    ++n_sh;
    if (S.ao_spheres_only) {
        for (int i = 0; i < S.n_list; ++i) {
            const int ref = S.list[i];
            if (!(ref & FRT_PRIM_SPHERE)) continue;
            V3<R> c;
            R r;
            sphere_get(S, ref & ~FRT_PRIM_SPHERE, c, r);
            if (sphere_intersect(p, wo, c, r, Cst<R>::eps, Cst<R>::tmax) > R(0)) {
                P.L = zero3<R>();
                break;
            }
        }
        return true;
    }
    P.ro = p; P.rd = wo; P.rtmax = R(S.ao_tmax);
    P.shadow = true;
    return false;
}

// normals_renderer::Li (debug_renderer.h:8-17): the shading normal of the
// camera hit, the environment on a miss.
template <typename R> FRT_HD bool normals_shade(PathState<R> &P, const DevScene &S, const Hit<R> &h)
{
    if (h.prim < 0) {
        P.L = env_of<R>(S);
        return true;
    }
    const V3<R> p = P.ro + h.t * P.rd;
    V3<R> n;
    int mat;
    prim_shade(S, h.prim, P.ro, p, h.u, h.v, n, mat);
    P.L = n;
    return true;
}

// integrator dispatch of the megakernel / self-test (KIND = FRT_INTEGRATOR_*)
template <int KIND, int MATS, typename R>
FRT_HD bool shade_kind(PathState<R> &P, const DevScene &S, const Hit<R> &h, int max_depth, uint32_t &n_ext, uint32_t &n_sh)
{
    if constexpr (KIND == FRT_INTEGRATOR_AO) return ao_shade<MATS>(P, S, h, n_sh);
    else if constexpr (KIND == FRT_INTEGRATOR_NORMALS) return normals_shade(P, S, h);
    else return path_shade<MATS>(P, S, h, max_depth, n_ext, n_sh);
}

}  // namespace frt
