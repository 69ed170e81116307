// frt_mlt.hpp -- PSS-MLT (Kelemen et al.) restated from first_ray/pssmlt.cpp
// for the GPU: one lane = one Markov chain.  __host__ __device__ like
// frt_path.hpp (the host self-test runs the same code).
//
//   pssmlt::Li              pssmlt.cpp:147-277 (depth <= 10, prnd offsets, MIS t^2)
//   GenerateEyePath         pssmlt.cpp:105-144 (pixel mapping generalised to nx, ny)
//   perturb / mutate        pssmlt.cpp:6-17, 62-73
//   Render (chain loop)     pssmlt.cpp:301-365, AccumulatePathContribution :19-38
//
// Primary samples: a chain's current state u[0..91] lives in HBM chain-major,
// U[chain][dim] (one 384-B row per chain, kMltRow).  A proposal is never stored: its
// dimension d is computed when the path reads it -- a fresh uniform on a large
// step, else perturb(U[c][d], r) -- and written back for all 92 dimensions
// only when the proposal is accepted (by the whole wave, one chain's row at a
// time: mlt_megakernel).  Random numbers follow DESIGN.md "PSS-MLT streams".
#pragma once
#include "frt_path.hpp"

namespace frt {

constexpr int kMltMaxPath = 10;                              // MaxPathLength (pssmlt.h:11)
constexpr int kMltDims = 4 + (kMltMaxPath + 1) * 8;          // 92 prnds a path can read
// U row stride: the 92 primary samples, then the chain's trajectory
// fingerprint (word 92: accepted proposals, word 93: sum of the accepted steps'
// 1-based indices mod 2^32; ora_mlt_render_shard keeps the same) and 2 pad
// words: 384 B = three 128-B lines per row
constexpr int kMltRow = 96;
constexpr int kMltFp = kMltDims;
constexpr float kMltLargeStep = 0.3f;                        // LargeStepProb (pssmlt.h:13)
constexpr uint32_t kMltChainSalt = 0x3C6EF372U, kMltBootSalt = 0xB5297A4DU;

// perturb (pssmlt.cpp:6-17) with log(s2/s1) precomputed.  The two halves as
// selects around one exp (the same operations and values as the branches,
// whose FMA the compiler formed as s2 * e + value and -s2 * e + value; as
// branches a wave ran both halves, two v_exp_f32 and the exec-mask bookkeeping)
FRT_HD float mlt_perturb(float value, float s2, float log_ratio, float r)
{
    const bool up = r < 0.5f;
    const float rr = up ? r * 2.0f : (r - 0.5f) * 2.0f;
    const float e = fexp(-log_ratio * rr);
    float result = fmaf(up ? s2 : -s2, e, value);
    if (up && result > 1.0f) result -= 1.0f;
    if (!up && result < 0.0f) result += 1.0f;
    return result;
}

// small-step mutation of dimension d (pixel dims 0, 1 use s1 = 2/(nx+ny), s2 = 0.1)
FRT_HD float mlt_mutate(float cur, float r, int d, float s2p, float logp)
{
    if (d < 2) return mlt_perturb(cur, s2p, logp, r);
    return mlt_perturb(cur, 1.0f / 64.0f, 2.77258872223978123767f /* log(16) */, r);
}

// Source of primary samples for one eye path.
struct PrndSource {
    const float *U;        // chain states [n_chains][dim] (null: bootstrap / fresh)
    uint32_t n_chains, chain;
    RngKey key;            // step key (chain, step) or bootstrap key
    uint32_t dim0;         // first RNG dimension holding prnd 0
    bool fresh;            // large step / initial state / bootstrap: uniform from the key
    float s2p, logp;       // pixel dims (0,1): s1 = 2/(nx+ny), s2 = 0.1f
    FRT_HD float get(int d) const
    {
        const float r = rng_u(key, dim0 + (uint32_t)d);
        if (fresh) return r;
        return mlt_mutate(U[(size_t)chain * kMltRow + d], r, d, s2p, logp);
    }
    // The chain's current values of dims [d0, d0 + 4 N) in N 16-B loads issued
    // together (d0 % 4 == 0), for at().  One per
    // dimension, each behind the previous dimension's hash and mutation,
    // exposed the load latency once per primary sample.  Fresh sources read none.
    // (d0 % 4 == 0 and rows of 96 floats: 16-B aligned)
    template <int N> FRT_HD void fetch(int d0, float4 (&c)[N]) const
    {
        if (fresh) return;
        const float4 *row = reinterpret_cast<const float4 *>(U + (size_t)chain * kMltRow + d0);
        for (int k = 0; k < N; ++k) c[k] = row[k];
    }
    // get(d) with the current value already fetched
    FRT_HD float at(int d, float cur) const
    {
        const float r = rng_u(key, dim0 + (uint32_t)d);
        if (fresh) return r;
        return mlt_mutate(cur, r, d, s2p, logp);
    }
};
FRT_HD float f4_at(const float4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

struct MltPath {
    PathState<float> P;    // ro, rd, rtmax, shadow, beta, L, nee, nxt_d, depth, prev_spec (prev_p unused)
    int off;               // PathRndsOffset
    float x, y;            // film position of the eye ray (GenerateEyePath)
};

// GenerateEyePath, first half: camera ray from prnds 0..3 and its film position
// (pssmlt.cpp:115-138 with PixelWidth/Height = nx/ny, dist = ny/(2 half_height)).
FRT_HD void mlt_begin(MltPath &M, const DevScene &S, const PrndSource &src, int nx, int ny)
{
    float4 c[1] = {make_float4(0.0f, 0.0f, 0.0f, 0.0f)};
    src.fetch<1>(0, c);
    const float s = src.at(0, c[0].x), t = src.at(1, c[0].y), l0 = src.at(2, c[0].z), l1 = src.at(3, c[0].w);
    f3 off = mk3(0, 0, 0);
    if (S.lens_r != 0.0f) {
        const float a = l0 * 2.0f - 1.0f, b = l1 * 2.0f - 1.0f;
        float rx = 0.0f, ry = 0.0f;
        if (a != 0.0f || b != 0.0f) {
            float r, phi;
            if (a * a > b * b) { r = a; phi = (kPi / 4.0f) * (b / a); }
            else { r = b; phi = (kPi / 2.0f) - (kPi / 4.0f) * (a / b); }
            rx = r * cosf(phi); ry = r * sinf(phi);
        }
        off = (S.lens_r * rx) * S.cam_u + (S.lens_r * ry) * S.cam_vv;
    }
    PathState<float> &P = M.P;
    P.ro = S.cam_o + off;
    P.rd = ((S.cam_llc + s * S.cam_h + t * S.cam_v) - S.cam_o) - off;
    P.rtmax = kTMaxClosest;
    P.shadow = false;
    P.term = false;
    P.depth = 0;
    P.beta = mk3(1, 1, 1);
    P.L = mk3(0, 0, 0);
    P.prev_pdf = 0.0f;
    P.prev_spec = false;
    M.off = 4;
    const f3 dir = normalize(P.rd);
    const float dist = (float)ny / (2.0f * S.cam_half_height);
    const f3 center = S.cam_o + dist * S.cam_w;
    const f3 pos = (S.cam_o + fdiv(dist, dot(dir, S.cam_w)) * dir) - center;
    M.x = -dot(S.cam_u, pos) + (float)nx * 0.5f;
    M.y = -dot(S.cam_vv, pos) + (float)ny * 0.5f;
}

// True when the next ray would be at depth > MaxPathLength: the reference does
// not trace it and returns the environment (pssmlt.cpp:151, :276).
FRT_HD bool mlt_beyond(const MltPath &M) { return !M.P.shadow && M.P.depth > kMltMaxPath; }

// pssmlt::Li, one hit at a time.  Returns true when the path is finished.
template <bool MATS = true>   // false: lambertian / diffuse_light scenes (see path_shade)
FRT_HD bool mlt_shade(MltPath &M, const DevScene &S, const Hit<float> &h, const PrndSource &src, uint32_t &n_ext,
                      uint32_t &n_sh)
{
    PathState<float> &P = M.P;
    if (P.shadow) {
        if (!path_after_shadow<(MATS ? kMatsAll : kMatsNone)>(P, h.prim < 0)) return true;
        if (P.depth <= kMltMaxPath) ++n_ext;
        return false;
    }
    if (P.term) return true;                            // finished in the traversal loop
    if (h.prim < 0) {
        P.L = P.L + P.beta * S.env;
        return true;
    }
    const f3 p = P.ro + h.t * P.rd;
    f3 n;
    int mat;
    prim_shade(S, h.prim, P.ro, p, h.u, h.v, n, mat);
    float4 m0 = S.mats[kMatStride * mat], m1 = S.mats[kMatStride * mat + 1];
    const int mtype = f2i(m0.w);
    if constexpr (MATS) apply_texture(S, mat, mtype, h.prim, p, h.u, h.v, m0, m1);
    // this vertex's primary samples, dims v0 + k (lambertian-only kernels: v0 =
    // 4 + 8 * vertex, so the 8 dims are two aligned float4; with specular
    // vertices, which consume 6, each is read on its own)
    const int v0 = M.off;
    float4 cur[2] = {make_float4(0.0f, 0.0f, 0.0f, 0.0f), make_float4(0.0f, 0.0f, 0.0f, 0.0f)};
    if constexpr (!MATS) src.fetch<2>(v0, cur);
    auto pr = [&](int k) -> float {
        if constexpr (!MATS) return src.at(v0 + k, f4_at(cur[k >> 2], k & 3));
        else return src.get(v0 + k);
    };
    const float sc0 = pr(0), sc1 = pr(1);               // scatter rnd (pssmlt.cpp:159-163)
    M.off += 3;                                         // consumed at every hit
    if (mtype == FRT_MAT_DIFFUSE_LIGHT && dot(n, P.rd) < 0.0f) {
        const f3 Le = xyz(m1);
        if (P.depth == 0 || P.prev_spec) {
            P.L = P.L + P.beta * Le;
        } else {                                        // pssmlt.cpp:175-184: distance^2 = t^2
            const float cos_wo = dot(n, -normalize(P.rd));
            float d2 = h.t * h.t;
            if (d2 <= kEps) d2 = kEps;
            const float light_pdf = fdiv(prim_pdf(S, h.prim, p, h.t, n, P.rd) * d2, fabsf(cos_wo));
            P.L = P.L + mi_weight(P.prev_pdf, light_pdf) * (P.beta * Le);
        }
        return true;
    }
    const bool lamb = mtype == FRT_MAT_LAMBERTIAN, spec = MATS && mat_is_specular(mtype),
               diel = MATS && mtype == FRT_MAT_DIELECTRIC;
    if (!(lamb || spec)) return true;                   // diffuse_light seen from behind
    const f3 wi = -normalize(P.rd);
    // NEE prnds (pssmlt.cpp:190-195); the bsdf prnds follow only for the diffuse branch
    const float rnd0 = pr(3), rnd1 = pr(4), rnd2 = pr(5);   // = M.off + 0, 1, 2
    M.off += 3;
    f3 wo, beta_next;
    float pdf;
    SpecMat SM{};
    if (!MATS || lamb) {
        const float b0 = pr(6), b1 = pr(7);             // = M.off + 0, 1
        M.off += 2;
        const Onb<float> uvw = onb_from_w(n);
        wo = onb_local(uvw, cosine_direction(b0, b1));
        const float cw = dot(n, normalize(wo));
        pdf = fmaxf(cw, 0.0f) * kInvPi;                 // pdf 0: the vertex returns 0 (pssmlt.cpp:261-264)
        beta_next = fdiv(fabsf(cw), pdf) * (P.beta * (kInvPi * xyz(m0)));
    } else {                                            // pssmlt.cpp:232-249
        SM = spec_mat(S, mat, mtype, m0, m1);
        float sampled;
        wo = spec_generate<kMatsAll>(SM, n, wi, sc0, sc1, sampled);
        pdf = spec_value<kMatsAll>(SM, n, wi, wo);
        if (sampled > 0.0f) pdf = sampled;
        const f3 bsdf = spec_eval<kMatsAll>(SM, n, wi, wo);
        beta_next = P.beta * (rcp(pdf) * bsdf);
    }
    // a zero pdf ends the path after the shadow ray the reference traces first (P.term)
    const int nl = S.n_lights;
    int idx = (int)(rnd0 * (float)nl);
    if (idx == nl) idx -= 1;
    // Lambertian-only kernels (MATS = false) never see pdf 0: the cosine lobe's
    // z = sqrt(1 - r0) >= 2^-12 (r0 < 1 - 2^-24), far above the rounding of
    // dot(n, wo); the constant lets the compiler drop the state.
    P.term = MATS && pdf == 0.0f;
    if (P.term && !(idx >= 0 && !diel)) return true;
    const f3 nee_o = p + kEps * n;
    const f3 origin = (!MATS || lamb || dot(n, wo) > 0.0f) ? nee_o : p - kEps * n;   // hrec.p moved off (:243, :253)
    P.nxt_d = wo;
    if constexpr (MATS) P.nxt_o = origin;
    if (idx >= 0 && !diel) {
        const int lref = S.lights[idx];
        f3 ln;
        int lmat;
        const f3 tl = prim_sample(S, lref, nee_o, rnd1, rnd2, ln, lmat);
        const float dist2 = len2(tl);
        const f3 tu = rlen(tl) * tl;
        const float cos_wi = dot(n, tu);
        const float cos_lo = dot(ln, -tu);
        P.nee = mk3(0, 0, 0);
        if (cos_lo != 0.0f) {
            const float light_pdf = fdiv(prim_pdf(S, lref, p, h.t, n, tu) * dist2, fabsf(cos_lo));
            const bool l = !MATS || lamb;
            const f3 f = l ? cos_wi * (kInvPi * xyz(m0)) : spec_eval<kMatsAll>(SM, n, wi, tu);
            const float bsdf_pdf = l ? fmaxf(cos_wi, 0.0f) * kInvPi : spec_value<kMatsAll>(SM, n, wi, tu);
            const float wgt = mi_weight(light_pdf, bsdf_pdf);
            const float4 lm0 = S.mats[kMatStride * lmat], lm1 = S.mats[kMatStride * lmat + 1];
            if (f2i(lm0.w) == FRT_MAT_DIFFUSE_LIGHT && dot(ln, tu) < 0.0f)
                P.nee = fdiv(wgt, light_pdf) * (P.beta * (xyz(lm1) * f));
        }
        P.ro = nee_o; P.rd = tl; P.rtmax = 1.0f - kShadowEps;
        P.shadow = true;
        ++n_sh;
    }
    P.beta = beta_next;
    P.prev_pdf = pdf;
    P.prev_spec = MATS && mat_no_mis(mtype);
    if (!P.shadow) {
        P.ro = origin; P.rd = wo; P.rtmax = kTMaxClosest;
        ++P.depth;
        if (P.depth <= kMltMaxPath) ++n_ext;
    }
    return false;
}

// AccumulatePathContribution target pixel (pssmlt.cpp:19-31); -1 if off film
FRT_HD int mlt_pixel(float x, float y, int nx, int ny)
{
    const int ix = (int)x, iy = (int)y;
    if (ix < 0 || ix >= nx || iy < 0 || iy >= ny) return -1;
    return iy * nx + ix;
}

}  // namespace frt
