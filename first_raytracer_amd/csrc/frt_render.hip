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

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "frt.h"
#include "frt_device.hpp"

using namespace frt;

namespace {

constexpr int kBlock = 256;
constexpr int kSentinel = 0x7fffffff;

// ------------------------------------------------------------------------
// device scene (fp32, HBM-resident; DESIGN.md "Data layout")
// ------------------------------------------------------------------------
struct DevScene {
    const float4 *__restrict__ nodes;    // 4 x float4 per interior node (child boxes + child refs), DFS order
    const float4 *__restrict__ tris;     // 3 x float4 per triangle: v0 | e1 | e2 (48 B), DFS leaf order
    const float4 *__restrict__ tshade;   // 2 x float4 per triangle: (n_geo, inv_area) | (mat, geo, -, -)
    const float4 *__restrict__ tnorm;    // 3 x float4 per triangle: vertex normals (smooth shading only)
    const float4 *__restrict__ spheres;  // (centre, radius)
    const int *__restrict__ sphere_mat;
    const float4 *__restrict__ mats;     // 2 x float4 per material: (albedo, type) | (emit, -)
    const int *__restrict__ lights;      // device prim refs
    const int *__restrict__ list;        // device prim refs (list worlds)
    int root;                            // node index, or ~prim for a single-leaf world
    int n_lights, n_list, world_kind;
    float root_lo[3], root_hi[3];
    f3 cam_o, cam_llc, cam_h, cam_v, cam_u, cam_vv;
    float lens_r;
    f3 env;
};

struct DevWork {
    int nx, ny, spp, max_depth;
    uint32_t seed;
    int tile, ntx, shard_index, shard_count;
    int spi, n_chunks;
    uint32_t n_items, n_slots;
    float *partial;                      // [n_chunks][n_slots][3]
    unsigned *counter;                   // work-queue head
    unsigned long long *wave_rays;       // [n_waves][4]: camera, extension, shadow, samples
};

struct Hit {
    int prim;     // device prim ref, -1 = miss
    float t, u, v;
};

// slot -> pixel inside a tile: 8x8 blocks, row-major inside a block
__device__ __host__ __forceinline__ void slot_to_local(int s, int tile, int &lx, int &ly)
{
    const int b = s >> 6, l = s & 63;
    const int bpr = tile >> 3;
    lx = (b % bpr) * 8 + (l & 7);
    ly = (b / bpr) * 8 + (l >> 3);
}

// ------------------------------------------------------------------------
// primitive tests
// ------------------------------------------------------------------------
__device__ __forceinline__ float prim_t(const DevScene &S, int ref, f3 o, f3 d, float tmin, float tmax,
                                        float &u, float &v)
{
    if (ref & FRT_PRIM_SPHERE) {
        const float4 sp = S.spheres[ref & ~FRT_PRIM_SPHERE];
        u = v = 0.0f;
        return sphere_intersect(o, d, xyz(sp), sp.w, tmin, tmax);
    }
    const float4 a = S.tris[3 * ref], b = S.tris[3 * ref + 1], c = S.tris[3 * ref + 2];
    return tri_intersect(o, d, xyz(a), xyz(b), xyz(c), tmin, tmax, u, v);
}

// parallel_bvh_node::hit restated as an ordered stack traversal.  Closest hit
// keeps the reference's answer: the minimum t, exact ties going to the leaf
// that comes first in the left-first DFS (device triangle ids ARE that order).
template <int STACK>
__device__ Hit trace_bvh(const DevScene &S, f3 o, f3 d, float tmax, bool anyhit, int *stk)
{
    Hit h{-1, tmax, 0.0f, 0.0f};
    const f3 invd = safe_inv(d);
    // root box tested with the unscaled EPSILON (parallel_bvh.h:43,46-51)
    if (slab_entry(S.root_lo[0], S.root_lo[1], S.root_lo[2], S.root_hi[0], S.root_hi[1], S.root_hi[2], o, invd,
                   kEps, tmax) == __builtin_inff())
        return h;
    const float tmin = kEps * fmaxf(1.0f, fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z))));
    int node = S.root;
    int sp = 0;
    for (;;) {
        while (node >= 0) {
            const float4 n0 = S.nodes[4 * node], n1 = S.nodes[4 * node + 1];
            const float4 n2 = S.nodes[4 * node + 2], n3 = S.nodes[4 * node + 3];
            const float t0 = slab_entry(n0.x, n0.y, n0.z, n0.w, n1.x, n1.y, o, invd, tmin, h.t);
            const float t1 = slab_entry(n1.z, n1.w, n2.x, n2.y, n2.z, n2.w, o, invd, tmin, h.t);
            const int c0 = __float_as_int(n3.x), c1 = __float_as_int(n3.y);
            const bool h0 = t0 != __builtin_inff(), h1 = t1 != __builtin_inff();
            if (h0 && h1) {
                const bool first0 = t0 <= t1;
                stk[sp * kBlock] = first0 ? c1 : c0;
                ++sp;
                node = first0 ? c0 : c1;
            } else if (h0) {
                node = c0;
            } else if (h1) {
                node = c1;
            } else {
                node = (sp > 0) ? stk[--sp * kBlock] : kSentinel;
            }
        }
        if (node == kSentinel) break;
        // leaf: one primitive (parallel_bvh.h:129-149 single-prim leaves)
        const int ref = ~node;
        float u, v;
        const float t = prim_t(S, ref, o, d, tmin, h.t, u, v);
        if (t > 0.0f) {
            const bool better = (t < h.t) || (h.prim >= 0 && (ref & FRT_PRIM_SPHERE ? true : ref < h.prim));
            if (better) {
                h.prim = ref; h.t = t; h.u = u; h.v = v;
                if (anyhit) return h;
            }
        }
        node = (sp > 0) ? stk[--sp * kBlock] : kSentinel;
        if (node == kSentinel) break;
    }
    return h;
}

// hitable_list::hit: linear, triangles strict '<', spheres inclusive (sphere.h:34)
__device__ Hit trace_list(const DevScene &S, f3 o, f3 d, float tmax, bool anyhit)
{
    Hit h{-1, tmax, 0.0f, 0.0f};
    for (int i = 0; i < S.n_list; ++i) {
        const int ref = S.list[i];
        float u, v;
        const float t = prim_t(S, ref, o, d, kEps, h.t, u, v);
        if (t > 0.0f && ((ref & FRT_PRIM_SPHERE) || t < h.t)) {
            h.prim = ref; h.t = t; h.u = u; h.v = v;
            if (anyhit) return h;
        }
    }
    return h;
}

template <int STACK, int WORLD>
__device__ __forceinline__ Hit trace(const DevScene &S, f3 o, f3 d, float tmax, bool anyhit, int *stk)
{
    if constexpr (WORLD == FRT_WORLD_LIST) return trace_list(S, o, d, tmax, anyhit);
    else return trace_bvh<STACK>(S, o, d, tmax, anyhit, stk);
}

// shading record of a primitive hit: normal + material
__device__ __forceinline__ void prim_shade(const DevScene &S, int ref, f3 p, float u, float v, f3 &n, int &mat)
{
    if (ref & FRT_PRIM_SPHERE) {                               // sphere.h:47-50
        const int k = ref & ~FRT_PRIM_SPHERE;
        const float4 sp = S.spheres[k];
        n = (1.0f / sp.w) * (p - xyz(sp));       // inside flip: caller (needs the ray origin)
        mat = S.sphere_mat[k];
        return;
    }
    const float4 s0 = S.tshade[2 * ref], s1 = S.tshade[2 * ref + 1];
    mat = __float_as_int(s1.x);
    if (__float_as_int(s1.y)) {                                // use_geometry_normals (triangle.h:100-101)
        n = xyz(s0);
    } else {                                                   // triangle.h:103
        const f3 n0 = xyz(S.tnorm[3 * ref]), n1 = xyz(S.tnorm[3 * ref + 1]), n2 = xyz(S.tnorm[3 * ref + 2]);
        n = normalize((1.0f - u - v) * n0 + u * n1 + v * n2);
    }
}

// pdf_direct_sampling: triangle.h:139-144 (inv_area); sphere.h:64-78 with the
// record's (p, t, normal) and the given direction
__device__ __forceinline__ float prim_pdf(const DevScene &S, int ref, f3 rec_p, float rec_t, f3 rec_n, f3 to_light)
{
    if (!(ref & FRT_PRIM_SPHERE)) return S.tshade[2 * ref].w;
    const float4 sp = S.spheres[ref & ~FRT_PRIM_SPHERE];
    const f3 o = rec_p - rec_t * to_light;
    const f3 dir = xyz(sp) - o;
    const float d2 = len2(dir);
    const float r2 = sp.w * sp.w;
    if (d2 <= r2) return 1.0f / (4.0f * kPi * r2);
    const float cos_max = sqrtf(1.0f - r2 / d2);
    const float solid = 2.0f * kPi * (1.0f - cos_max);
    return (1.0f / solid) * fabsf(dot(to_light, rec_n)) / d2;
}

// sample_direct: triangle.h:145-175, sphere.h:80-107.  Returns to_light
// (unnormalised, as the reference), light normal and material.
__device__ __forceinline__ f3 prim_sample(const DevScene &S, int ref, f3 o, float u0, float u1, f3 &ln, int &lmat)
{
    if (ref & FRT_PRIM_SPHERE) {
        const int k = ref & ~FRT_PRIM_SPHERE;
        const float4 sp = S.spheres[k];
        const f3 c = xyz(sp);
        lmat = S.sphere_mat[k];
        const f3 direction = c - o;
        const float d2 = len2(direction);
        if (d2 <= sp.w * sp.w) {
            const f3 p = c + sp.w * uniform_sphere(u0, u1);
            ln = normalize(c - p);
            return p - o;
        }
        const Onb uvw = onb_from_w(direction);
        const f3 p = onb_local(uvw, random_to_sphere(sp.w, d2, u0, u1));
        ln = normalize(p);
        return p;
    }
    const float4 a = S.tris[3 * ref], b = S.tris[3 * ref + 1], c = S.tris[3 * ref + 2];
    const float su0 = sqrtf(u0);
    const float b0 = 1.0f - su0;
    const float b1 = u1 * su0;
    const f3 lp = xyz(a) + b0 * xyz(b) + b1 * xyz(c);            // (1-b0-b1) v0 + b0 v1 + b1 v2
    const float4 s0 = S.tshade[2 * ref], s1 = S.tshade[2 * ref + 1];
    lmat = __float_as_int(s1.x);
    if (__float_as_int(s1.y)) {
        ln = xyz(s0);
    } else {
        const f3 n0 = xyz(S.tnorm[3 * ref]), n1 = xyz(S.tnorm[3 * ref + 1]), n2 = xyz(S.tnorm[3 * ref + 2]);
        ln = normalize((1.0f - b0 - b1) * n0 + b0 * n1 + b1 * n2);
    }
    return lp - o;
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// ------------------------------------------------------------------------
// the persistent path megakernel
// ------------------------------------------------------------------------
template <int STACK, int WORLD>
__global__ __launch_bounds__(kBlock) void path_megakernel(const DevScene S, const DevWork W)
{
    extern __shared__ int lds_stack[];       // [STACK][kBlock]
    int *stk = lds_stack + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const int T2 = W.tile * W.tile;

    // work-item state
    bool have_item = false, exhausted = false;
    int s_cur = 0, s_end = 0;
    uint32_t slot = 0, chunk = 0, pix = 0;
    int px = 0, py = 0;
    f3 acc = mk3(0, 0, 0);
    // path state
    bool active = false, shadow = false;
    f3 ro = mk3(0, 0, 0), rd = mk3(0, 0, 1);
    float rtmax = kTMaxClosest;
    f3 beta = mk3(1, 1, 1), L = mk3(0, 0, 0), nee = mk3(0, 0, 0);
    f3 nxt_o = mk3(0, 0, 0), nxt_d = mk3(0, 0, 1), prev_p = mk3(0, 0, 0);
    float prev_pdf = 0.0f;
    int depth = 0;
    RngKey key{0, 0};
    unsigned long long n_cam = 0, n_ext = 0, n_sh = 0, n_smp = 0;

    for (;;) {
        // ---- retire a finished item ----
        if (!active && have_item && s_cur >= s_end) {
            float *dst = W.partial + 3ull * ((size_t)chunk * W.n_slots + slot);
            dst[0] = acc.x; dst[1] = acc.y; dst[2] = acc.z;
            have_item = false;
        }
        // ---- wave-aggregated refill (one atomic per wave) ----
        const bool need = !active && !have_item && !exhausted;
        const uint64_t m = __ballot(need);
        if (m) {
            const int leader = __ffsll((unsigned long long)m) - 1;
            uint32_t base = 0;
            if (lane == leader) base = atomicAdd(W.counter, (unsigned)__popcll(m));
            base = __shfl(base, leader);
            if (need) {
                const uint32_t w = base + lane_rank(m);
                if (w >= W.n_items) {
                    exhausted = true;
                } else {
                    const uint32_t s = w % (uint32_t)T2;
                    const uint32_t q = w / (uint32_t)T2;
                    chunk = q % (uint32_t)W.n_chunks;
                    const uint32_t t_ord = q / (uint32_t)W.n_chunks;
                    const int tile_id = W.shard_index + (int)t_ord * W.shard_count;
                    int lx, ly;
                    slot_to_local((int)s, W.tile, lx, ly);
                    px = (tile_id % W.ntx) * W.tile + lx;
                    py = (tile_id / W.ntx) * W.tile + ly;
                    slot = t_ord * (uint32_t)T2 + s;
                    if (px < W.nx && py < W.ny) {
                        have_item = true;
                        pix = (uint32_t)py * (uint32_t)W.nx + (uint32_t)px;
                        s_cur = (int)chunk * W.spi;
                        s_end = min(W.spp, s_cur + W.spi);
                        acc = mk3(0, 0, 0);
                    }
                }
            }
        }
        // ---- start the next camera sample (path.cpp:129-136, camera.h:30-35) ----
        if (!active && have_item && s_cur < s_end) {
            key = rng_key(W.seed, pix, (uint32_t)s_cur);
            ++s_cur;
            const float u = ((float)px + rng_u(key, 0)) / (float)W.nx;
            const float v = ((float)py + rng_u(key, 1)) / (float)W.ny;
            f3 off = mk3(0, 0, 0);
            if (S.lens_r != 0.0f) {                         // util.h:21-41 concentric disk
                const float a = rng_u(key, 2) * 2.0f - 1.0f, b = rng_u(key, 3) * 2.0f - 1.0f;
                float rx = 0.0f, ry = 0.0f;
                if (a != 0.0f || b != 0.0f) {
                    float r, phi;
                    if (a * a > b * b) { r = a; phi = (kPi / 4.0f) * (b / a); }
                    else { r = b; phi = (kPi / 2.0f) - (kPi / 4.0f) * (a / b); }
                    rx = r * cosf(phi); ry = r * sinf(phi);
                }
                off = (S.lens_r * rx) * S.cam_u + (S.lens_r * ry) * S.cam_vv;
            }
            ro = S.cam_o + off;
            rd = ((S.cam_llc + u * S.cam_h + v * S.cam_v) - S.cam_o) - off;
            rtmax = kTMaxClosest;
            shadow = false;
            depth = 0;
            beta = mk3(1, 1, 1);
            L = mk3(0, 0, 0);
            active = true;
            ++n_cam; ++n_smp;
        }
        if (__ballot(active) == 0) {
            if (__ballot(!exhausted) == 0) break;
            continue;
        }
        if (!active) continue;

        // ---- trace one ray ----
        const Hit h = trace<STACK, WORLD>(S, ro, rd, rtmax, shadow, stk);

        // ---- shade ----
        bool finish = false;
        if (shadow) {
            if (h.prim < 0) L = L + nee;                // path.cpp:50-77, unoccluded
            shadow = false;
            ro = nxt_o; rd = nxt_d; rtmax = kTMaxClosest;
            ++depth; ++n_ext;
        } else if (h.prim < 0) {
            L = L + beta * S.env;                       // path.cpp:115 environment
            finish = true;
        } else {
            const f3 p = ro + h.t * rd;
            f3 n; int mat;
            prim_shade(S, h.prim, p, h.u, h.v, n, mat);
            if ((h.prim & FRT_PRIM_SPHERE) && len2(ro - xyz(S.spheres[h.prim & ~FRT_PRIM_SPHERE])) <
                    S.spheres[h.prim & ~FRT_PRIM_SPHERE].w * S.spheres[h.prim & ~FRT_PRIM_SPHERE].w)
                n = -n;                                 // sphere.h:48-49
            const float4 m0 = S.mats[2 * mat], m1 = S.mats[2 * mat + 1];
            const int mtype = __float_as_int(m0.w);
            // diffuse_light::emitted, one-sided (material.h:184-190)
            const f3 Le = (mtype == FRT_MAT_DIFFUSE_LIGHT && dot(n, rd) < 0.0f) ? xyz(m1) : mk3(0, 0, 0);
            if (nonzero(Le)) {
                if (depth == 0) {
                    L = L + beta * Le;                  // path.cpp:16-22
                } else {                                // path.cpp:24-31 MIS vs the bsdf sample
                    const float cos_wo = dot(n, -normalize(rd));
                    float d2 = len2(p - prev_p);
                    if (d2 <= kEps) d2 = kEps;
                    const float light_pdf = prim_pdf(S, h.prim, p, h.t, n, rd) * d2 / fabsf(cos_wo);
                    L = L + mi_weight(prev_pdf, light_pdf) * (beta * Le);
                }
                finish = true;
            } else if (mtype == FRT_MAT_LAMBERTIAN && depth <= W.max_depth) {
                const uint32_t base = dim_bounce(depth);
                // bsdf sample first: a zero pdf drops this vertex's NEE too (path.cpp:96-106)
                const Onb uvw = onb_from_w(n);
                const f3 wo = onb_local(uvw, cosine_direction(rng_u(key, base + 6), rng_u(key, base + 7)));
                const float cw = dot(n, normalize(wo));
                const float pdf = fmaxf(cw, 0.0f) * kInvPi;
                if (pdf == 0.0f) {
                    finish = true;
                } else {
                    const f3 f = kInvPi * xyz(m0);      // lambertian::eval_bsdf (material.h:62-65)
                    const f3 beta_next = (fabsf(cw) / pdf) * (beta * f);
                    nxt_o = p + kEps * n;
                    nxt_d = wo;
                    // next-event estimation (path.cpp:38-77)
                    const int nl = S.n_lights;
                    int idx = (int)(rng_u(key, base + 3) * (float)nl);
                    if (idx == nl) idx -= 1;
                    if (idx >= 0) {
                        const int lref = S.lights[idx];
                        f3 ln; int lmat;
                        const f3 origin = p + kEps * n;
                        const f3 tl = prim_sample(S, lref, origin, rng_u(key, base + 4), rng_u(key, base + 5), ln, lmat);
                        const float dist2 = len2(tl);
                        const f3 tu = rlen(tl) * tl;
                        const float cos_wi = dot(n, tu);
                        const float cos_lo = dot(ln, -tu);
                        nee = mk3(0, 0, 0);
                        if (cos_lo != 0.0f) {
                            const float light_pdf = prim_pdf(S, lref, p, h.t, n, tu) * dist2 / fabsf(cos_lo);
                            const float bsdf_pdf = fmaxf(cos_wi, 0.0f) * kInvPi;
                            const float wgt = mi_weight(light_pdf, bsdf_pdf);
                            const float4 lm0 = S.mats[2 * lmat], lm1 = S.mats[2 * lmat + 1];
                            const bool emits = __float_as_int(lm0.w) == FRT_MAT_DIFFUSE_LIGHT && dot(ln, tu) < 0.0f;
                            if (emits) nee = (wgt / light_pdf * cos_wi) * (beta * (xyz(lm1) * f));
                        }
                        ro = origin; rd = tl; rtmax = 1.0f - kShadowEps;
                        shadow = true;
                        ++n_sh;
                    }
                    beta = beta_next;
                    prev_p = p;
                    prev_pdf = pdf;
                    if (!shadow) {
                        ro = nxt_o; rd = nxt_d; rtmax = kTMaxClosest;
                        ++depth; ++n_ext;
                    }
                }
            } else {
                finish = true;                          // light seen from behind, or depth cap
            }
        }
        if (finish) {
            acc = acc + L;
            active = false;
        }
    }
    // per-wave ray counters (no atomics): lane 0 writes the wave's sums
    for (int off = 32; off > 0; off >>= 1) {
        n_cam += __shfl_xor(n_cam, off);
        n_ext += __shfl_xor(n_ext, off);
        n_sh += __shfl_xor(n_sh, off);
        n_smp += __shfl_xor(n_smp, off);
    }
    if (lane == 0) {
        const size_t wv = ((size_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
        W.wave_rays[4 * wv + 0] = n_cam;
        W.wave_rays[4 * wv + 1] = n_ext;
        W.wave_rays[4 * wv + 2] = n_sh;
        W.wave_rays[4 * wv + 3] = n_smp;
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

}  // namespace

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
    std::vector<void *> scene_bufs;
    // workspace
    float *partial = nullptr; size_t partial_bytes = 0;
    unsigned *counter = nullptr;
    unsigned long long *wave_rays = nullptr; size_t wave_rays_n = 0;
    float *slots_out = nullptr; size_t slots_out_bytes = 0;
};

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
        hipMalloc(&c->counter, 64) != hipSuccess) {
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
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
    return FRT_OK;
}

extern "C" const char *frt_last_error(const frt_ctx *c) { return c ? c->err.c_str() : "null context"; }

// ---- scene upload: DFS flattening + fp32 conversion with outward rounding ----
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

static inline float bits_f(int x)
{
    float f;
    memcpy(&f, &x, 4);
    return f;
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
    const int nt = sv->n_tris, ns = sv->n_spheres, nm = sv->n_materials;
    if (nt < 0 || ns < 0 || nm <= 0 || (nt > 0 && (!sv->tri_v || !sv->tri_material || !sv->tri_inv_area)))
        return set_err(c, FRT_E_INVALID, "scene view: missing triangle arrays or materials");
    if (ns > 0 && (!sv->sphere || !sv->sphere_material))
        return set_err(c, FRT_E_INVALID, "scene view: missing sphere arrays");
    for (int i = 0; i < nm; ++i)
        if (sv->materials[i].type != FRT_MAT_LAMBERTIAN && sv->materials[i].type != FRT_MAT_DIFFUSE_LIGHT)
            return set_err(c, FRT_E_UNSUPPORTED, "material type " + std::to_string(sv->materials[i].type) +
                                                     " is outside the hot path (lambertian/diffuse_light only)");
    auto valid_ref = [&](int ref) {
        if (ref & FRT_PRIM_SPHERE) return (ref & ~FRT_PRIM_SPHERE) < ns;
        return ref >= 0 && ref < nt;
    };
    // world
    std::vector<int> tri_order;                     // device id -> view triangle
    std::vector<int> tri_dev(nt, -1);               // view triangle -> device id
    std::vector<float4> nodes;
    int depth = 0;
    double rlo[3] = {0, 0, 0}, rhi[3] = {0, 0, 0};
    auto prim_box = [&](int ref, double *lo, double *hi) {
        if (ref & FRT_PRIM_SPHERE) {
            const double *s = &sv->sphere[4 * (ref & ~FRT_PRIM_SPHERE)];
            for (int k = 0; k < 3; ++k) { lo[k] = s[k] - s[3]; hi[k] = s[k] + s[3]; }
        } else {
            const double *v = &sv->tri_v[9 * ref];
            for (int k = 0; k < 3; ++k) {
                lo[k] = std::min(std::min(v[k], v[3 + k]), v[6 + k]);
                hi[k] = std::max(std::max(v[k], v[3 + k]), v[6 + k]);
            }
        }
    };
    double scale = 1.0;
    if (sv->world_kind == FRT_WORLD_BVH) {
        const int nn = sv->n_nodes;
        if (nn < 0 || (nn > 0 && (!sv->node_box || !sv->node_child)))
            return set_err(c, FRT_E_INVALID, "scene view: missing BVH arrays");
        if (nn == 0 && sv->root >= 0) return set_err(c, FRT_E_INVALID, "scene view: empty BVH");
        if (sv->root >= nn) return set_err(c, FRT_E_INVALID, "scene view: bad root");
        // scene scale for the conservative box padding
        if (nn > 0) {
            const double *b = &sv->node_box[6 * sv->root];
            for (int k = 0; k < 3; ++k) scale = std::max(scale, std::max(std::fabs(b[k]), std::fabs(b[3 + k])));
        }
        const double pad = 4e-6 * scale;
        auto padded = [&](const double *lo, const double *hi, float *flo, float *fhi) {
            for (int k = 0; k < 3; ++k) { flo[k] = round_down(lo[k] - pad); fhi[k] = round_up(hi[k] + pad); }
        };
        // left-first DFS: node ids in pre-order, triangle leaves numbered in visit order
        std::vector<int> new_id(std::max(nn, 1), -1);
        std::vector<int> order;
        order.reserve(nn);
        if (sv->root < 0) {
            const int ref = ~sv->root;
            if (!valid_ref(ref)) return set_err(c, FRT_E_INVALID, "scene view: bad root prim");
            if (!(ref & FRT_PRIM_SPHERE)) { tri_dev[ref] = 0; tri_order.push_back(ref); }
            double lo[3], hi[3];
            prim_box(ref, lo, hi);
            for (int k = 0; k < 3; ++k) { rlo[k] = lo[k]; rhi[k] = hi[k]; }
        } else {
            std::vector<std::pair<int, int>> st;   // (child ref, level)
            st.push_back({sv->root, 1});
            while (!st.empty()) {
                auto [x, lvl] = st.back();
                st.pop_back();
                if (x >= 0) {
                    if (x >= nn || new_id[x] >= 0) return set_err(c, FRT_E_INVALID, "scene view: BVH is not a tree");
                    new_id[x] = (int)order.size();
                    order.push_back(x);
                    depth = std::max(depth, lvl);
                    st.push_back({sv->node_child[2 * x + 1], lvl + 1});
                    st.push_back({sv->node_child[2 * x], lvl + 1});
                } else {
                    const int ref = ~x;
                    if (!valid_ref(ref)) return set_err(c, FRT_E_INVALID, "scene view: bad leaf prim");
                    if (!(ref & FRT_PRIM_SPHERE)) {
                        if (tri_dev[ref] >= 0) return set_err(c, FRT_E_INVALID, "scene view: triangle in two leaves");
                        tri_dev[ref] = (int)tri_order.size();
                        tri_order.push_back(ref);
                    }
                }
            }
            nodes.resize(4 * order.size());
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
                        const int dref = (ref & FRT_PRIM_SPHERE) ? ref : tri_dev[ref];
                        cref[side] = ~dref;
                    }
                    padded(lo, hi, &cb[side][0], &cb[side][3]);
                }
                nodes[4 * i + 0] = make_float4(cb[0][0], cb[0][1], cb[0][2], cb[0][3]);
                nodes[4 * i + 1] = make_float4(cb[0][4], cb[0][5], cb[1][0], cb[1][1]);
                nodes[4 * i + 2] = make_float4(cb[1][2], cb[1][3], cb[1][4], cb[1][5]);
                nodes[4 * i + 3] = make_float4(bits_f(cref[0]), bits_f(cref[1]), 0.0f, 0.0f);
            }
            for (int k = 0; k < 3; ++k) { rlo[k] = sv->node_box[6 * sv->root + k]; rhi[k] = sv->node_box[6 * sv->root + 3 + k]; }
        }
        float flo[3], fhi[3];
        padded(rlo, rhi, flo, fhi);
        for (int k = 0; k < 3; ++k) { c->S.root_lo[k] = flo[k]; c->S.root_hi[k] = fhi[k]; }
        // triangles outside the tree keep trailing ids (never intersected)
        for (int i = 0; i < nt; ++i)
            if (tri_dev[i] < 0) { tri_dev[i] = (int)tri_order.size(); tri_order.push_back(i); }
    } else if (sv->world_kind == FRT_WORLD_LIST) {
        if (sv->n_list < 0 || (sv->n_list > 0 && !sv->list)) return set_err(c, FRT_E_INVALID, "scene view: bad list");
        for (int i = 0; i < nt; ++i) { tri_dev[i] = i; tri_order.push_back(i); }
        for (int i = 0; i < sv->n_list; ++i)
            if (!valid_ref(sv->list[i])) return set_err(c, FRT_E_INVALID, "scene view: bad list entry");
    } else {
        return set_err(c, FRT_E_INVALID, "scene view: unknown world kind");
    }

    // triangles in device order
    std::vector<float4> tris(3 * (size_t)nt), tshade(2 * (size_t)nt), tnorm;
    bool any_smooth = false;
    for (int i = 0; i < nt; ++i)
        if (sv->tri_geometry_normal && !sv->tri_geometry_normal[i]) any_smooth = true;
    if (any_smooth && !sv->tri_n) return set_err(c, FRT_E_INVALID, "scene view: smooth triangles without normals");
    if (any_smooth) tnorm.resize(3 * (size_t)nt);
    for (int d = 0; d < nt; ++d) {
        const int i = tri_order[d];
        const double *v = &sv->tri_v[9 * i];
        const double e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
        const double e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        double ng[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const double l = std::sqrt(ng[0] * ng[0] + ng[1] * ng[1] + ng[2] * ng[2]);
        for (int k = 0; k < 3; ++k) ng[k] = ng[k] / l;
        tris[3 * d + 0] = make_float4((float)v[0], (float)v[1], (float)v[2], 0.0f);
        tris[3 * d + 1] = make_float4((float)e1[0], (float)e1[1], (float)e1[2], 0.0f);
        tris[3 * d + 2] = make_float4((float)e2[0], (float)e2[1], (float)e2[2], 0.0f);
        const int mat = sv->tri_material[i];
        if (mat < 0 || mat >= nm) return set_err(c, FRT_E_INVALID, "scene view: bad triangle material");
        const int geo = sv->tri_geometry_normal ? (sv->tri_geometry_normal[i] ? 1 : 0) : 1;
        tshade[2 * d + 0] = make_float4((float)ng[0], (float)ng[1], (float)ng[2], (float)sv->tri_inv_area[i]);
        tshade[2 * d + 1] = make_float4(bits_f(mat), bits_f(geo), 0.0f, 0.0f);
        if (any_smooth)
            for (int k = 0; k < 3; ++k)
                tnorm[3 * d + k] = make_float4((float)sv->tri_n[9 * i + 3 * k], (float)sv->tri_n[9 * i + 3 * k + 1],
                                               (float)sv->tri_n[9 * i + 3 * k + 2], 0.0f);
    }
    std::vector<float4> spheres(ns);
    std::vector<int> smat(ns);
    for (int k = 0; k < ns; ++k) {
        const double *s = &sv->sphere[4 * k];
        spheres[k] = make_float4((float)s[0], (float)s[1], (float)s[2], (float)s[3]);
        smat[k] = sv->sphere_material[k];
        if (smat[k] < 0 || smat[k] >= nm) return set_err(c, FRT_E_INVALID, "scene view: bad sphere material");
    }
    std::vector<float4> mats(2 * (size_t)nm);
    for (int i = 0; i < nm; ++i) {
        const frt_material &m = sv->materials[i];
        mats[2 * i] = make_float4((float)m.albedo[0], (float)m.albedo[1], (float)m.albedo[2], bits_f(m.type));
        mats[2 * i + 1] = make_float4((float)m.emit[0], (float)m.emit[1], (float)m.emit[2], 0.0f);
    }
    auto dev_ref = [&](int ref) { return (ref & FRT_PRIM_SPHERE) ? ref : tri_dev[ref]; };
    std::vector<int> lights(std::max(sv->n_lights, 0)), list(std::max(sv->n_list, 0));
    for (int i = 0; i < sv->n_lights; ++i) {
        if (!valid_ref(sv->lights[i])) return set_err(c, FRT_E_INVALID, "scene view: bad light");
        lights[i] = dev_ref(sv->lights[i]);
    }
    for (int i = 0; i < (int)list.size(); ++i) list[i] = dev_ref(sv->list[i]);

    free_scene(c);
    DevScene &S = c->S;
    int rc;
    if ((rc = upload_vec(c, nodes, &S.nodes)) || (rc = upload_vec(c, tris, &S.tris)) ||
        (rc = upload_vec(c, tshade, &S.tshade)) || (rc = upload_vec(c, tnorm, &S.tnorm)) ||
        (rc = upload_vec(c, spheres, &S.spheres)) || (rc = upload_vec(c, smat, &S.sphere_mat)) ||
        (rc = upload_vec(c, mats, &S.mats)) || (rc = upload_vec(c, lights, &S.lights)) ||
        (rc = upload_vec(c, list, &S.list)))
        return rc;
    S.root = (sv->world_kind == FRT_WORLD_BVH) ? ((sv->root >= 0) ? 0 : ~dev_ref(~sv->root)) : 0;
    S.n_lights = sv->n_lights;
    S.n_list = (int)list.size();
    S.world_kind = sv->world_kind;
    auto f3d = [](const double *x) { return mk3((float)x[0], (float)x[1], (float)x[2]); };
    S.cam_o = f3d(sv->cam_origin); S.cam_llc = f3d(sv->cam_lower_left);
    S.cam_h = f3d(sv->cam_horizontal); S.cam_v = f3d(sv->cam_vertical);
    S.cam_u = f3d(sv->cam_u); S.cam_vv = f3d(sv->cam_v);
    S.lens_r = (float)sv->cam_lens_radius;
    S.env = f3d(sv->env_color);
    c->world_kind = sv->world_kind;
    c->stack_needed = depth;
    c->have_scene = true;
    return FRT_OK;
}

// ---- shard geometry ----
static int eff_tile(const frt_render_params *p) { return p->tile_size > 0 ? p->tile_size : 32; }
static bool params_ok(const frt_render_params *p)
{
    const int T = eff_tile(p);
    return p && p->nx > 0 && p->ny > 0 && p->spp > 0 && (T % 8) == 0 && T <= 256 && p->shard_count >= 1 &&
           p->shard_index >= 0 && p->shard_index < p->shard_count && p->max_depth >= -1 && p->max_depth < 100000 &&
           p->integrator == FRT_INTEGRATOR_PATH;
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
    const int T = eff_tile(p);
    return (int64_t)my_tiles(p) * T * T;
}
extern "C" int frt_shard_slots(const frt_render_params *p, int32_t *slot_pixel)
{
    if (!params_ok(p) || !slot_pixel) return FRT_E_INVALID;
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

template <int STACK, int WORLD>
static hipError_t launch_path(frt_ctx *c, const DevWork &W, int grid, hipStream_t st)
{
    const size_t lds = (WORLD == FRT_WORLD_BVH) ? (size_t)STACK * kBlock * sizeof(int) : 0;
    hipLaunchKernelGGL((path_megakernel<STACK, WORLD>), dim3(grid), dim3(kBlock), lds, st, c->S, W);
    return hipGetLastError();
}
template <int STACK, int WORLD>
static int occupancy(int *blocks)
{
    const size_t lds = (WORLD == FRT_WORLD_BVH) ? (size_t)STACK * kBlock * sizeof(int) : 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, path_megakernel<STACK, WORLD>, kBlock, lds) ==
                   hipSuccess ? 0 : -1;
}

static int render_impl(frt_ctx *c, const frt_render_params *p, float *dev_slots, hipStream_t st, frt_stats *stats)
{
    const auto t_start = std::chrono::steady_clock::now();
    if (!c || !p) return FRT_E_INVALID;
    if (!params_ok(p)) return set_err(c, FRT_E_INVALID, "bad render params");
    if (!c->have_scene) return set_err(c, FRT_E_NO_SCENE, "no scene uploaded");
    HIPCHK(c, hipSetDevice(c->device));
    const int T = eff_tile(p);
    const int nmt = my_tiles(p);
    const uint32_t n_slots = (uint32_t)nmt * T * T;
    // kernel variant by stack depth
    int stack = 16;
    if (c->world_kind == FRT_WORLD_BVH) {
        if (c->stack_needed < 16) stack = 16;
        else if (c->stack_needed < 32) stack = 32;
        else if (c->stack_needed < 64) stack = 64;
        else return set_err(c, FRT_E_UNSUPPORTED, "BVH deeper than 63 levels");
    }
    int bpc = 0;
    int oc;
    if (c->world_kind == FRT_WORLD_LIST) oc = occupancy<16, FRT_WORLD_LIST>(&bpc);
    else if (stack == 16) oc = occupancy<16, FRT_WORLD_BVH>(&bpc);
    else if (stack == 32) oc = occupancy<32, FRT_WORLD_BVH>(&bpc);
    else oc = occupancy<64, FRT_WORLD_BVH>(&bpc);
    if (oc != 0 || bpc <= 0) bpc = 1;
    const int grid = c->n_cu * bpc;
    const long long lanes = (long long)grid * kBlock;
    // work granule: aim for >= 16 items per resident lane
    int spi = p->samples_per_item;
    if (spi <= 0) {
        const double want_items = 16.0 * (double)lanes;
        spi = (int)std::floor((double)p->spp * (double)n_slots / std::max(want_items, 1.0));
        spi = std::max(1, std::min(spi, p->spp));
    }
    spi = std::min(spi, p->spp);
    const int n_chunks = (p->spp + spi - 1) / spi;
    const unsigned long long n_items = (unsigned long long)n_slots * n_chunks;
    if (n_items >= 0xffffffffULL) return set_err(c, FRT_E_UNSUPPORTED, "frame too large for one call: shard it");
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
    W.tile = T; W.ntx = (p->nx + T - 1) / T; W.shard_index = p->shard_index; W.shard_count = p->shard_count;
    W.spi = spi; W.n_chunks = n_chunks; W.n_items = (uint32_t)n_items; W.n_slots = n_slots;
    W.partial = c->partial; W.counter = c->counter; W.wave_rays = c->wave_rays;

    HIPCHK(c, hipMemsetAsync(c->counter, 0, 64, st));
    HIPCHK(c, hipEventRecord(c->ev0, st));
    hipError_t le;
    if (c->world_kind == FRT_WORLD_LIST) le = launch_path<16, FRT_WORLD_LIST>(c, W, grid, st);
    else if (stack == 16) le = launch_path<16, FRT_WORLD_BVH>(c, W, grid, st);
    else if (stack == 32) le = launch_path<32, FRT_WORLD_BVH>(c, W, grid, st);
    else le = launch_path<64, FRT_WORLD_BVH>(c, W, grid, st);
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
        stats->kernel_ms = ms;
        stats->total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
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
