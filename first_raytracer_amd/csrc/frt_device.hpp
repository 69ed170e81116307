// frt_device.hpp -- fp32 device math shared by the path megakernel.
// All functions are __host__ __device__ so the same code can be compiled for
// the host-side self tests (frt_selftest_* in frt_render.hip).
//
// Reference semantics restated (fp64 there, fp32 here), first_ray/:
//   aabb::hit           aabb.h:14-31       (slab test, NaN-tolerant)
//   triangle::hit       triangle.h:69-118  (Moller-Trumbore)
//   sphere::hit         sphere.h:26-56
//   onb::build_from_w   onb.h:18-30
//   hemisphere_to_cosine_direction pdf.h:13-23, cosine_pdf pdf.h:80-97
//   miWeight            util.h:55-60
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define FRT_HD __host__ __device__ __forceinline__

namespace frt {

constexpr float kEps = 1e-4f;              // util.h:10 EPSILON
constexpr float kShadowEps = 1e-3f;        // util.h:11 SHADOW_EPSILON
constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.318309886183790671538f;
constexpr float kTMaxClosest = 3.40282347e+38f;   // FLT_MAX (path.cpp:10)

struct f3 { float x, y, z; };
FRT_HD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
FRT_HD f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
FRT_HD f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
FRT_HD f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
FRT_HD f3 operator*(float t, f3 v) { return f3{t * v.x, t * v.y, t * v.z}; }
FRT_HD f3 operator-(f3 v) { return f3{-v.x, -v.y, -v.z}; }
FRT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
FRT_HD f3 cross(f3 a, f3 b) { return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
FRT_HD float len2(f3 v) { return dot(v, v); }
FRT_HD bool nonzero(f3 v) { return v.x != 0.0f || v.y != 0.0f || v.z != 0.0f; }
FRT_HD f3 xyz(float4 v) { return f3{v.x, v.y, v.z}; }

// ---------------------------------------------------------------------------
// RNG stream spec (identical to oracle/frt_oracle.c rng_make/rng_u)
// ---------------------------------------------------------------------------
FRT_HD uint32_t mix32(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
struct RngKey { uint32_t k0, k1; };
FRT_HD RngKey rng_key(uint32_t seed, uint32_t pixel, uint32_t sample)
{
    const uint32_t a = mix32(seed ^ 0x2545F491U);
    RngKey k;
    k.k0 = mix32(mix32(a ^ pixel) + sample * 0x9E3779B9U);
    k.k1 = mix32(mix32(a + pixel * 0x632BE5ABU) ^ (sample * 0x85157AF5U + 0x5851F42DU));
    return k;
}
// uniform in [0,1) with 24 bits: exact in fp32 and fp64
FRT_HD float rng_u(RngKey k, uint32_t dim)
{
    const uint32_t h = mix32(mix32(k.k0 ^ (dim * 0x85EBCA77U + 0xC2B2AE3DU)) + k.k1);
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}
// dimension layout: camera 0..3; bounce d: base 4 + 8d (+3 light pick,
// +4..5 light sample, +6..7 bsdf direction; +0..2 reserved for get3d)
FRT_HD uint32_t dim_bounce(int depth) { return 4u + 8u * (uint32_t)depth; }

// ---------------------------------------------------------------------------
// geometry
// ---------------------------------------------------------------------------
// Hardware transcendental units on the GPU (v_rcp / v_rsq / v_sqrt / v_sin /
// v_cos / v_exp, ~1 ulp), libm on the host (self-test build).  The IEEE
// sequences they replace (div_scale/fmas/fixup, denormal-scaled sqrt, sin/cos
// range reduction) dominated the shading code; the parity gate is RMSE 1e-3
// against the fp64 oracle, and the device results stay bit-identical across
// kernel variants (same instructions everywhere).  -DFRT_EXP_IEEE_MATH builds
// the IEEE versions (6 % slower on Cornell, 11 % on 1M: profiles/r01_exp2.txt).
FRT_HD float rcp(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
FRT_HD float fdiv(float a, float b) { return a * rcp(b); }
FRT_HD float fsqrt(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
FRT_HD float frsqrt(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_rsqf(x);
#else
    return 1.0f / sqrtf(x);
#endif
}
// sin / cos of 2*pi*r for r in [0, 1) (v_sin_f32 / v_cos_f32 take revolutions)
FRT_HD void sincos_2pi(float r, float &s, float &c)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    s = __builtin_amdgcn_sinf(r);
    c = __builtin_amdgcn_cosf(r);
#else
    sincosf(2.0f * 3.14159265358979323846f * r, &s, &c);
#endif
}
// e^x for moderate |x| (PSS-MLT perturbation: x in [-8, 0])
FRT_HD float fexp(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_exp2f(x * 1.44269504088896340736f);
#else
    return expf(x);
#endif
}
// ln x, x^y (x > 0) on the hardware log2 / exp2 (v_log_f32 / v_exp_f32)
FRT_HD float flog(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_logf(x) * 0.69314718055994530942f;
#else
    return logf(x);
#endif
}
FRT_HD float fpow(float x, float y)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#else
    return powf(x, y);
#endif
}
FRT_HD float rlen(f3 v) { return frsqrt(len2(v)); }
FRT_HD f3 normalize(f3 v) { return rlen(v) * v; }

// Ray prepared for slab tests: t = lo * invd + oinv with oinv = -o * invd
// (one FMA per slab plane).  Zero direction components are nudged to
// +-1e-30 so no 0*inf NaN can arise; the reference's NaN-tolerant compare
// (aabb.h:24-25) keeps the interval unchanged in that case, and so does this
// (the near-parallel slab spans +-huge).  Device boxes are padded outward, so
// neither the nudge nor the FMA rounding can cull a hit.
struct SlabRay { f3 invd, oinv; };
FRT_HD SlabRay slab_ray(f3 o, f3 d)
{
    const float tiny = 1e-30f;
    const float dx = fabsf(d.x) > tiny ? d.x : copysignf(tiny, d.x);
    const float dy = fabsf(d.y) > tiny ? d.y : copysignf(tiny, d.y);
    const float dz = fabsf(d.z) > tiny ? d.z : copysignf(tiny, d.z);
    SlabRay r;
    r.invd = f3{rcp(dx), rcp(dy), rcp(dz)};
    r.oinv = f3{-o.x * r.invd.x, -o.y * r.invd.y, -o.z * r.invd.z};
    return r;
}
// slab test of a box against [tmin, tmax]; returns entry distance or +inf on
// miss (aabb.h:14-31: the reference's per-axis early exit decides the same).
FRT_HD float slab_entry(float lox, float loy, float loz, float hix, float hiy, float hiz, const SlabRay &r,
                        float tmin, float tmax)
{
    const float tx0 = fmaf(lox, r.invd.x, r.oinv.x), tx1 = fmaf(hix, r.invd.x, r.oinv.x);
    const float ty0 = fmaf(loy, r.invd.y, r.oinv.y), ty1 = fmaf(hiy, r.invd.y, r.oinv.y);
    const float tz0 = fmaf(loz, r.invd.z, r.oinv.z), tz1 = fmaf(hiz, r.invd.z, r.oinv.z);
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), tmin));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    return (tf < tn) ? __builtin_inff() : tn;
}

// the same test on a box stored as (near, far) planes for the ray's octant
// (bvh2_step OCT): bit-identical to slab_entry on the (lo, hi) box
FRT_HD float slab_entry_nf(float nx, float ny, float nz, float fx, float fy, float fz, const SlabRay &r,
                           float tmin, float tmax)
{
    const float tn = fmaxf(fmaxf(fmaf(nx, r.invd.x, r.oinv.x), fmaf(ny, r.invd.y, r.oinv.y)),
                           fmaxf(fmaf(nz, r.invd.z, r.oinv.z), tmin));
    const float tf = fminf(fminf(fmaf(fx, r.invd.x, r.oinv.x), fmaf(fy, r.invd.y, r.oinv.y)),
                           fminf(fmaf(fz, r.invd.z, r.oinv.z), tmax));
    return (tf < tn) ? __builtin_inff() : tn;
}

// Moller-Trumbore (triangle.h:69-118): returns t, or -1 on miss.  Accepts
// t in (tmin, tmax] -- the caller resolves t == tmax with the DFS rank tie rule.
FRT_HD float tri_intersect(f3 o, f3 d, f3 v0, f3 e1, f3 e2, float tmin, float tmax, float &u, float &v)
{
    const f3 h = cross(d, e2);
    const float a = dot(e1, h);
    if (a == 0.0f) return -1.0f;
    const float f = rcp(a);
    const f3 s = o - v0;
    u = f * dot(s, h);
    if (u < 0.0f || u > 1.0f) return -1.0f;
    const f3 q = cross(s, e1);
    v = f * dot(d, q);
    if (!(v >= 0.0f && u + v <= 1.0f)) return -1.0f;
    const float t = f * dot(e2, q);
    return (t > tmin && t <= tmax) ? t : -1.0f;
}

// sphere::hit (sphere.h:26-56): returns t or -1; accepts t in [tmin, tmax].
// The discriminant b^2 - a(|oc|^2 - r^2) loses ~|oc|^2/r^2 ulps to
// cancellation in fp32 (veach's r = 0.03 lights at distance 15: a 2 % error,
// which blurs the silhouette the fp64 reference draws sharply).  It is formed
// instead as a(r^2 - |oc - (b/a) d|^2) from the ray's perpendicular offset,
// which keeps the error relative to r^2 (Hearn-Baker form); same roots.
FRT_HD float sphere_intersect(f3 o, f3 d, f3 c, float r, float tmin, float tmax)
{
    const f3 oc = o - c;
    const float a = dot(d, d);
    const float b = dot(oc, d);
    const float ia = rcp(a);
    const f3 l = oc - (b * ia) * d;
    float disc = a * (r * r - dot(l, l));
    if (!(disc >= 0.0f)) return -1.0f;
    disc = fsqrt(disc);
    float t = (-b - disc) * ia;
    if (t < tmin) t = (-b + disc) * ia;
    if (t < tmin || t > tmax) return -1.0f;
    return t;
}

// onb::build_from_w (onb.h:18-30) + fromLocal
struct Onb { f3 u, v, w; };
FRT_HD Onb onb_from_w(f3 n)
{
    Onb b;
    b.w = n;
    if (fabsf(n.x) > fabsf(n.y)) {
        const float inv = frsqrt(n.x * n.x + n.z * n.z);
        b.v = f3{n.z * inv, 0.0f, -n.x * inv};
    } else {
        const float inv = frsqrt(n.y * n.y + n.z * n.z);
        b.v = f3{0.0f, n.z * inv, -n.y * inv};
    }
    b.u = cross(b.v, b.w);
    return b;
}
FRT_HD f3 onb_local(const Onb &b, f3 a) { return a.x * b.u + a.y * b.v + a.z * b.w; }

// pdf.h:13-23
FRT_HD f3 cosine_direction(float r0, float r1)
{
    const float r = fsqrt(r0);
    float sp, cp;
    sincos_2pi(r1, sp, cp);                       // phi = 2 pi r1
    return f3{r * cp, r * sp, fsqrt(1.0f - r0)};
}
// pdf.h:38-44
FRT_HD f3 uniform_sphere(float u0, float u1)
{
    const float z = 1.0f - 2.0f * u0;
    const float r = fsqrt(fmaxf(0.0f, 1.0f - z * z));
    float sp, cp;
    sincos_2pi(u1, sp, cp);
    return f3{r * cp, r * sp, z};
}
// pdf.h:46-56
FRT_HD f3 random_to_sphere(float radius, float dist2, float r1, float r2)
{
    const float z = 1.0f + r2 * (fsqrt(1.0f - fdiv(radius * radius, dist2)) - 1.0f);
    float sp, cp;
    sincos_2pi(r1, sp, cp);
    const float s = fsqrt(1.0f - z * z);
    return f3{cp * s, sp * s, z};
}
// x^y for x in [0, 1], y > 0 (phong lobes): exp2(y log2 x) on the hardware units
FRT_HD float fpow01(float x, float y)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#else
    return powf(x, y);
#endif
}

// ---- specular materials (material.h:75-171, pdf.h:99-184, util.h:73-117) ----
constexpr float kDeltaEps = 1e-3f;                               // util.h:12 DELTA_EPSILON
FRT_HD f3 reflect(f3 v, f3 n) { return normalize(v - (2.0f * dot(v, n)) * n); }   // util.h:73-76
FRT_HD f3 refract(f3 wi, f3 n, float eta, float cos_t)                            // util.h:79-84
{
    if (cos_t < 0.0f) eta = rcp(eta);
    return normalize((dot(wi, n) * eta + cos_t) * n - eta * wi);
}
FRT_HD float fresnel_dielectric(float cos_i, float &cos_t_out, float eta)       // util.h:86-117
{
    if (eta == 1.0f) { cos_t_out = -cos_i; return 0.0f; }
    const float scale = (cos_i > 0.0f) ? rcp(eta) : eta;
    const float cos_t2 = 1.0f - (1.0f - cos_i * cos_i) * (scale * scale);
    if (cos_t2 <= 0.0f) { cos_t_out = 0.0f; return 1.0f; }      // total internal reflection
    const float ci = fabsf(cos_i), ct = fsqrt(cos_t2);
    const float rs = fdiv(ci - eta * ct, ci + eta * ct);
    const float rp = fdiv(eta * ci - ct, eta * ci + ct);
    cos_t_out = (cos_i > 0.0f) ? -ct : ct;
    return 0.5f * (rs * rs + rp * rp);
}
// cosine_power_pdf (pdf.h:99-136); the onb's w is the shading normal
FRT_HD float cosine_power_value(f3 n, f3 wi, float e, f3 wo)
{
    if (dot(n, wo) <= 0.0f || dot(n, wi) <= 0.0f) return 0.0f;
    const float alpha = fmaxf(0.0f, dot(reflect(-wi, n), wo));
    return fpow01(alpha, e) * (e + 1.0f) * (0.5f * kInvPi);
}
FRT_HD f3 cosine_power_generate(f3 n, f3 wi, float e, float s0, float s1)
{
    const f3 r = reflect(-wi, n);
    const float sin_a = fsqrt(1.0f - fpow01(s1, fdiv(2.0f, e + 1.0f)));
    const float cos_a = fpow01(s1, rcp(e + 1.0f));
    float sp, cp;
    sincos_2pi(s0, sp, cp);
    return onb_local(onb_from_w(r), f3{sin_a * cp, sin_a * sp, cos_a});
}
// modified_phong::eval_bsdf (material.h:92-100), cosine included
FRT_HD f3 phong_eval(f3 kd, f3 ks, float e, f3 n, f3 wi, f3 wo)
{
    const float alpha = fmaxf(0.0f, dot(normalize(reflect(-wi, n)), wo));
    const f3 result = kInvPi * kd + ((e + 2.0f) * (0.5f * kInvPi) * fpow01(alpha, e)) * ks;
    return dot(n, wo) * result;
}
// dielectric_pdf (pdf.h:138-184) and dielectric::eval_bsdf (material.h:146-171)
FRT_HD float dielectric_value(f3 n, f3 wi, float ior, f3 wo)
{
    float cos_t;
    const float F = fresnel_dielectric(dot(wi, n), cos_t, ior);
    if (dot(wi, n) * dot(wo, n) >= 0.0f)
        return (fabsf(dot(reflect(-wi, n), wo) - 1.0f) > kDeltaEps) ? 0.0f : F;
    return (fabsf(dot(refract(wi, n, ior, cos_t), wo) - 1.0f) > kDeltaEps) ? 0.0f : 1.0f - F;
}
FRT_HD f3 dielectric_generate(f3 n, f3 wi, float ior, float s0)
{
    float cos_t;
    const float F = fresnel_dielectric(dot(wi, n), cos_t, ior);
    return (s0 <= F) ? reflect(-wi, n) : refract(wi, n, ior, cos_t);
}
FRT_HD f3 dielectric_eval(f3 ks, float ior, f3 n, f3 wi, f3 wo)
{
    float cos_t;
    const float F = fresnel_dielectric(dot(wi, n), cos_t, ior);
    if (dot(wi, n) * dot(wo, n) >= 0.0f) {
        if (fabsf(dot(reflect(-wi, n), wo) - 1.0f) > kDeltaEps) return f3{0.0f, 0.0f, 0.0f};
        return F * ks;
    }
    if (fabsf(dot(refract(wi, n, ior, cos_t), wo) - 1.0f) > kDeltaEps) return f3{0.0f, 0.0f, 0.0f};
    const float factor = cos_t < 0.0f ? rcp(ior) : ior;
    return (factor * factor * (1.0f - F)) * ks;
}

// ---- rough_conductor (material.h:246-315), roughconductor_pdf (pdf.h:231-486,
//      pdf.cpp:5-12), microfacet.h; isotropic alpha.  fp32 restatement of the
//      oracle's rough_* functions (oracle/frt_oracle.c) on the hardware
//      transcendentals (rcp, sqrt, rsq, exp2, log2, sin / cos in revolutions)
//      like the rest of the shading code; only acos stays libm.  The OCML
//      tan / pow / atan2 / sin / cos and IEEE divisions of round 1 made this the
//      register-hungriest part of the material kernels. ----
constexpr int kDistGgx = 0, kDistBeckmann = 1;
FRT_HD float safe_sqrtf(float v) { const float r = fsqrt(v); return (0.0f < r) ? r : 0.0f; }   // util.h:43-46 (NaN -> 0)
FRT_HD f3 onb_to_local(const Onb &b, f3 a) { return f3{dot(a, b.u), dot(a, b.v), dot(a, b.w)}; }
// microfacet::fresnelConductorExact (microfacet.h:8-31), one channel
FRT_HD float fresnel_conductor1(float cos_i, float eta, float k)
{
    const float c2 = cos_i * cos_i, s2 = 1.0f - c2, s4 = s2 * s2;
    const float temp1 = eta * eta - k * k - s2;
    const float a2pb2 = safe_sqrtf(temp1 * temp1 + 4.0f * (k * k * eta * eta));
    const float a = safe_sqrtf(0.5f * (a2pb2 + temp1));
    const float term1 = a2pb2 + c2, term2 = (2.0f * cos_i) * a;
    const float rs2 = fdiv(term1 - term2, term1 + term2);
    const float term3 = c2 * a2pb2 + s4, term4 = s2 * term2;
    const float rp2 = rs2 * fdiv(term3 - term4, term3 + term4);
    return 0.5f * (rp2 + rs2);
}
// microfacet::smithG1 (microfacet.h:48-88)
FRT_HD float smith_g1(f3 v, f3 m, f3 n, float alpha, int dist)
{
    const float cos_t = dot(n, v);
    if (dot(v, m) * cos_t <= 0.0f) return 0.0f;
    const float temp = 1.0f - cos_t * cos_t;
    if (temp <= 0.0f) return 1.0f;
    const float tan_t = fdiv(fsqrt(temp), cos_t);
    if (dist == kDistBeckmann) {
        const float a = rcp(alpha * tan_t);
        if (a >= 1.6f) return 1.0f;
        const float a2 = a * a;
        return fdiv(3.535f * a + 2.181f * a2, 1.0f + 2.276f * a + 2.577f * a2);
    }
    const float root = alpha * tan_t;
    return fdiv(2.0f, 1.0f + fsqrt(1.0f + root * root));          // hypot2(1, root) (util.h:239-254)
}
// microfacet::eval (microfacet.h:90-135)
FRT_HD float microfacet_d(f3 m, f3 n, float alpha, int dist)
{
    const f3 ml = onb_to_local(onb_from_w(n), m);
    const float cos_t = ml.z;
    if (cos_t <= 0.0f) return 0.0f;
    const float c2 = cos_t * cos_t, a2 = alpha * alpha;
    const float be = fdiv(fdiv(ml.x * ml.x, a2) + fdiv(ml.y * ml.y, a2), c2);
    float r;
    if (dist == kDistBeckmann) {
        r = fdiv(fexp(-be), kPi * a2 * c2 * c2);
    } else {
        const float root = (1.0f + be) * c2;
        r = rcp(kPi * a2 * root * root);
    }
    return (r * cos_t < 1e-20f) ? 0.0f : r;
}
// util.h:185-236
FRT_HD float erfinv_f(float x)
{
    float w = -flog((1.0f - x) * (1.0f + x)), p;
    if (w < 5.0f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = 3.43273939e-07f + p * w;
        p = -3.5233877e-06f + p * w;
        p = -4.39150654e-06f + p * w;
        p = 0.00021858087f + p * w;
        p = -0.00125372503f + p * w;
        p = -0.00417768164f + p * w;
        p = 0.246640727f + p * w;
        p = 1.50140941f + p * w;
    } else {
        w = fsqrt(w) - 3.0f;
        p = -0.000200214257f;
        p = 0.000100950558f + p * w;
        p = 0.00134934322f + p * w;
        p = -0.00367342844f + p * w;
        p = 0.00573950773f + p * w;
        p = -0.0076224613f + p * w;
        p = 0.00943887047f + p * w;
        p = 1.00167406f + p * w;
        p = 2.83297682f + p * w;
    }
    return p * x;
}
FRT_HD float erf_f(float x)
{
    const float sign = copysignf(1.0f, x);
    x = fabsf(x);
    const float t = rcp(1.0f + 0.3275911f * x);
    const float y = 1.0f - (((((1.061405429f * t - 1.453152027f) * t) + 1.421413741f) * t - 0.284496736f) * t +
                            0.254829592f) * t * fexp(-x * x);
    return sign * y;
}
// roughconductor_pdf::sampleVisible11 (pdf.h:280-397)
// theta_i enters as cos / sin (cos_t = ws.z, sin_t = sqrt((1 - z)(1 + z)));
// normal: the reference's theta_i < 1e-4 test, which in fp32 holds exactly
// when rough_generate left theta at 0 (ws.z >= 0.99999: acos of anything
// below that is >= 4.5e-3).  tan(theta_i) = sin / cos, as tan(acos z) is;
// theta_i itself only for the Beckmann fit, so GGX lanes run no acos.
FRT_HD void sample_visible11(bool normal, float cos_t, float sin_t, float sx, float sy, int dist, float &slx, float &sly)
{
    const float kSqrtPiInv = 0.564189583547756287f;
    if (normal) {                                               // normal incidence
        const float r = (dist == kDistBeckmann) ? fsqrt(-flog(1.0f - sx)) : safe_sqrtf(fdiv(sx, 1.0f - sx));
        float sp, cp;
        sincos_2pi(sy, sp, cp);                                 // phi = 2 pi sy
        slx = r * cp; sly = r * sp;
        return;
    }
    const float tan_t = fdiv(sin_t, cos_t);
    if (dist == kDistBeckmann) {
        const float theta_i = acosf(cos_t);
        const float cot_t = rcp(tan_t);
        float a = -1.0f, c = erf_f(cot_t);
        const float sample_x = fmaxf(sx, 1e-6f);
        const float fit = 1.0f + theta_i * (-0.876f + theta_i * (0.4265f - 0.0594f * theta_i));
        float b = c - (1.0f + c) * fpow(1.0f - sample_x, fit);
        const float norm = rcp(1.0f + c + kSqrtPiInv * tan_t * fexp(-cot_t * cot_t));
        for (int it = 1; it < 10; ++it) {
            if (!(b >= a && b <= c)) b = 0.5f * (a + c);
            const float inv_erf = erfinv_f(b);
            const float value = norm * (1.0f + b + kSqrtPiInv * tan_t * fexp(-inv_erf * inv_erf)) - sample_x;
            const float deriv = norm * (1.0f - inv_erf * tan_t);
            if (fabsf(value) < 1e-5f) break;
            if (value > 0.0f) c = b; else a = b;
            b -= fdiv(value, deriv);
        }
        slx = erfinv_f(b);
        sly = erfinv_f(2.0f * fmaxf(sy, 1e-6f) - 1.0f);
        return;
    }
    const float a = rcp(tan_t);
    const float g1 = fdiv(2.0f, 1.0f + safe_sqrtf(1.0f + rcp(a * a)));
    float A = fdiv(2.0f * sx, g1) - 1.0f;
    if (fabsf(A) == 1.0f) A -= copysignf(1.0f, A) * kEps;
    const float tmp = rcp(A * A - 1.0f);
    const float B = tan_t;
    const float D = safe_sqrtf(B * B * tmp * tmp - (A * A - B * B) * tmp);
    const float s1 = B * tmp - D, s2 = B * tmp + D;
    slx = (A < 0.0f || s2 > a) ? s1 : s2;
    float S;
    if (sy > 0.5f) { S = 1.0f; sy = 2.0f * (sy - 0.5f); }
    else { S = -1.0f; sy = 2.0f * (0.5f - sy); }
    const float z = fdiv(sy * (sy * (sy * -0.365728915865723f + 0.790235037209296f) - 0.424965825137544f) +
                             0.000152998850436920f,
                         sy * (sy * (sy * (sy * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) + 1.0f) -
                             0.539825872510702f);
    sly = S * z * fsqrt(1.0f + slx * slx);
}
// roughconductor_pdf::generate (pdf.h:409-482, pdf.cpp:5-12): wo, and the
// sampled pdf (pdfVisible / (4 wo.m)) that path.cpp:82 prefers when > 0
FRT_HD f3 rough_generate(f3 n, f3 wi, float alpha, int dist, float s0, float s1, float &sampled_pdf)
{
    const Onb uvw = onb_from_w(n);
    const f3 wl = onb_to_local(uvw, wi);
    f3 ws = f3{alpha * wl.x, alpha * wl.y, wl.z};
    ws = frsqrt(len2(ws)) * ws;
    // theta = acos(ws.z) (0 at and above 0.99999), phi = atan2(ws.y, ws.x): sin / cos phi as
    // ws.y / r, ws.x / r; sample_visible11 takes theta as cos / sin
    const bool normal = !(ws.z < 0.99999f);
    float sp = 0.0f, cp = 1.0f;
    if (!normal) {
        const float rr = ws.x * ws.x + ws.y * ws.y;
        if (rr > 0.0f) { const float ir = frsqrt(rr); sp = ws.y * ir; cp = ws.x * ir; }
    }
    float slx, sly;
    sample_visible11(normal, ws.z, fsqrt((1.0f - ws.z) * (1.0f + ws.z)), s0, s1, dist, slx, sly);
    if (!(fabsf(slx) <= 3.40282347e+38f)) slx = 0.0f;             // !std::isfinite
    const float rx = (cp * slx - sp * sly) * alpha, ry = (sp * slx + cp * sly) * alpha;
    const float nrm = frsqrt(rx * rx + ry * ry + 1.0f);
    const f3 ml = f3{-rx * nrm, -ry * nrm, nrm};
    const f3 mw = onb_local(uvw, ml);
    float pdf = 0.0f;
    if (wl.z != 0.0f)
        pdf = fdiv(smith_g1(onb_local(uvw, wl), mw, n, alpha, dist) * fabsf(dot(wl, ml)) * microfacet_d(mw, n, alpha, dist),
                   fabsf(wl.z));
    const f3 wo = reflect(-wi, mw);
    sampled_pdf = fdiv(pdf, 4.0f * dot(wo, mw));
    return wo;
}
// roughconductor_pdf::value (pdf.h:237-250)
FRT_HD float rough_value(f3 n, f3 wi, float alpha, int dist, f3 wo)
{
    if (dot(n, wo) <= 0.0f || dot(n, wi) <= 0.0f) return 0.0f;
    const f3 H = normalize(wo + wi);
    return fdiv(microfacet_d(H, n, alpha, dist) * smith_g1(wi, H, n, alpha, dist), 4.0f * dot(wi, n));
}
// rough_conductor::eval_bsdf (material.h:277-307); no cosine (is_specular)
FRT_HD f3 rough_eval(f3 eta, f3 k, f3 spec, float alpha, int dist, f3 n, f3 wi, f3 wo)
{
    const float cos_wi = dot(wi, n);
    if (cos_wi <= 0.0f || dot(wo, n) <= 0.0f) return f3{0.0f, 0.0f, 0.0f};
    const f3 H = normalize(wo + wi);
    const float D = microfacet_d(H, n, alpha, dist);
    if (D == 0.0f) return f3{0.0f, 0.0f, 0.0f};
    const float c = dot(wi, H);
    const f3 F = f3{fresnel_conductor1(c, eta.x, k.x), fresnel_conductor1(c, eta.y, k.y),
                    fresnel_conductor1(c, eta.z, k.z)} * spec;
    const float G = smith_g1(wi, H, n, alpha, dist) * smith_g1(wo, H, n, alpha, dist);
    return fdiv(D * G, 4.0f * cos_wi) * F;
}

// util.h:55-60
FRT_HD float mi_weight(float p1, float p2)
{
    p1 *= p1;
    p2 *= p2;
    return fdiv(p1, p1 + p2);
}

}  // namespace frt
