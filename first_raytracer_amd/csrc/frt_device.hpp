// frt_device.hpp -- device math shared by the path megakernel, templated on
// the scalar type R: float for the product kernels, double for the fp64
// kernels ("fp32 on the GPU, with an fp64 compile option for
// debugging parity"; DESIGN.md "Precision").  All functions are
// __host__ __device__ so the same code also runs in the host self tests
// (frt_selftest_* in frt_render.hip).
//
// Reference semantics restated (fp64 there), first_ray/:
//   aabb::hit           aabb.h:14-31       (slab test, NaN-tolerant)
//   triangle::hit       triangle.h:69-118  (Moller-Trumbore)
//   sphere::hit         sphere.h:26-56
//   onb::build_from_w   onb.h:18-30
//   hemisphere_to_cosine_direction pdf.h:13-23, cosine_pdf pdf.h:80-97
//   miWeight            util.h:55-60
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#define FRT_HD __host__ __device__ __forceinline__

namespace frt {

constexpr float kEps = 1e-4f;              // util.h:10 EPSILON
constexpr float kShadowEps = 1e-3f;        // util.h:11 SHADOW_EPSILON
constexpr float kPi = 3.14159265358979323846f;
constexpr float kInvPi = 0.318309886183790671538f;
constexpr float kTMaxClosest = 3.40282347e+38f;   // FLT_MAX (path.cpp:10)

// Per-precision constants.  The double set keeps the reference's values:
// EPSILON is the double 1e-4 (util.h:10) while SHADOW_EPSILON and
// DELTA_EPSILON are float literals widened to double (util.h:11-12).
template <typename R> struct Cst;
template <> struct Cst<float> {
    static constexpr float eps = kEps, shadow_eps = kShadowEps, delta_eps = 1e-3f;
    static constexpr float pi = kPi, inv_pi = kInvPi, tmax = kTMaxClosest;
};
template <> struct Cst<double> {
    static constexpr double eps = 1e-4, shadow_eps = (double)1e-3f, delta_eps = (double)1e-3f;
    static constexpr double pi = 3.14159265358979323846, inv_pi = 0.318309886183790671538;
    static constexpr double tmax = (double)kTMaxClosest;
};
template <typename R> constexpr bool kIsF64 = std::is_same<R, double>::value;

template <typename R> struct V3 { R x, y, z; };
using f3 = V3<float>;
using d3 = V3<double>;
FRT_HD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
template <typename R> FRT_HD V3<R> zero3() { return V3<R>{R(0), R(0), R(0)}; }
template <typename R> FRT_HD V3<R> operator+(V3<R> a, V3<R> b) { return V3<R>{a.x + b.x, a.y + b.y, a.z + b.z}; }
template <typename R> FRT_HD V3<R> operator-(V3<R> a, V3<R> b) { return V3<R>{a.x - b.x, a.y - b.y, a.z - b.z}; }
template <typename R> FRT_HD V3<R> operator*(V3<R> a, V3<R> b) { return V3<R>{a.x * b.x, a.y * b.y, a.z * b.z}; }
template <typename R> FRT_HD V3<R> operator*(R t, V3<R> v) { return V3<R>{t * v.x, t * v.y, t * v.z}; }
template <typename R> FRT_HD V3<R> operator-(V3<R> v) { return V3<R>{-v.x, -v.y, -v.z}; }
template <typename R> FRT_HD R dot(V3<R> a, V3<R> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename R> FRT_HD V3<R> cross(V3<R> a, V3<R> b)
{
    return V3<R>{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
template <typename R> FRT_HD R len2(V3<R> v) { return dot(v, v); }
template <typename R> FRT_HD bool nonzero(V3<R> v) { return v.x != R(0) || v.y != R(0) || v.z != R(0); }
FRT_HD f3 xyz(float4 v) { return f3{v.x, v.y, v.z}; }
FRT_HD d3 xyz(double4 v) { return d3{v.x, v.y, v.z}; }
// an fp32 record (material colour, padded box) in the kernel's precision
template <typename R> FRT_HD V3<R> rgb(float4 v) { return V3<R>{R(v.x), R(v.y), R(v.z)}; }

// min / max / abs / fma / copysign of either precision (the float forms are
// the fminf / fmaxf ... the fp32 kernels have always used)
// max / min for the slab tests, whose operands are never NaN (directions are
// nudged off zero, slab_ray): gfx950's NaN-propagating v_maximum3 / v_minimum3
// take them as they are, where fmaxf / fminf (IEEE maxNum) first quiet every
// operand that is not the result of arithmetic in the same block -- t_min and
// t_best, once per node.  Equal results for non-NaN operands, so the same hits.
FRT_HD float smax(float a, float b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_elementwise_maximum(a, b);
#else
    return fmaxf(a, b);
#endif
}
FRT_HD float smin(float a, float b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_elementwise_minimum(a, b);
#else
    return fminf(a, b);
#endif
}
// a * b for 0 <= a, b < 2^24 as one full-rate v_mul_u32_u24 (an int index times
// a constant became a 64-bit v_mad_u64_u32 in the LDS address)
FRT_HD int u24mul(int a, int b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (int)__umul24((unsigned)a, (unsigned)b);
#else
    return a * b;
#endif
}
FRT_HD double smax(double a, double b) { return fmax(a, b); }
FRT_HD double smin(double a, double b) { return fmin(a, b); }
FRT_HD float vmin(float a, float b) { return fminf(a, b); }
FRT_HD double vmin(double a, double b) { return fmin(a, b); }
FRT_HD float vmax(float a, float b) { return fmaxf(a, b); }
FRT_HD double vmax(double a, double b) { return fmax(a, b); }
FRT_HD float vabs(float a) { return fabsf(a); }
FRT_HD double vabs(double a) { return fabs(a); }
FRT_HD float vfma(float a, float b, float c) { return fmaf(a, b, c); }
FRT_HD double vfma(double a, double b, double c) { return fma(a, b, c); }
FRT_HD float vcopysign(float a, float b) { return copysignf(a, b); }
FRT_HD double vcopysign(double a, double b) { return copysign(a, b); }
FRT_HD float vacos(float a) { return acosf(a); }
FRT_HD double vacos(double a) { return acos(a); }
FRT_HD float vcos(float a) { return cosf(a); }
FRT_HD double vcos(double a) { return cos(a); }
FRT_HD float vsin(float a) { return sinf(a); }
FRT_HD double vsin(double a) { return sin(a); }

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
// uniform in [0,1) with 24 bits: exact in fp32 and fp64.  One mix32 round
// per dimension over the (pixel, sample) key, which is itself two rounds
// deep; a second round per dimension (rounds 1-3) cost Cornell 1.9 % and the
// PSS-MLT chain kernel 3 % (two quarter-rate multiplies per random number;
// same-call timing builds, profiles/r04/r04{k,m}).
FRT_HD float rng_u(RngKey k, uint32_t dim)
{
    const uint32_t h = mix32((k.k0 ^ (dim * 0x85EBCA77U + 0xC2B2AE3DU)) + k.k1);
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}
template <typename R> FRT_HD R rng_r(RngKey k, uint32_t dim) { return R(rng_u(k, dim)); }
// dimension layout: camera 0..3; bounce d: base 4 + 8d (+3 light pick,
// +4..5 light sample, +6..7 bsdf direction; +0..2 reserved for get3d)
FRT_HD uint32_t dim_bounce(int depth) { return 4u + 8u * (uint32_t)depth; }

// ---------------------------------------------------------------------------
// geometry
// ---------------------------------------------------------------------------
// fp32: hardware transcendental units on the GPU (v_rcp / v_rsq / v_sqrt /
// v_sin / v_cos / v_exp, ~1 ulp), libm on the host (self-test build).  The
// IEEE sequences they replace (div_scale/fmas/fixup, denormal-scaled sqrt,
// sin/cos range reduction) dominated the shading code; the parity gate is RMSE
// 1e-3 against the fp64 oracle, and the device results stay bit-identical
// across kernel variants (same instructions everywhere).  -DFRT_EXP_IEEE_MATH
// builds the IEEE versions (6 % slower on Cornell, 11 % on 1M:
// profiles/r01_exp2.txt).  fp64: the IEEE double operations and OCML
// (correctly rounded division and sqrt), as the reference's libm.
FRT_HD float rcp(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
FRT_HD double rcp(double x) { return 1.0 / x; }
FRT_HD float fdiv(float a, float b) { return a * rcp(b); }
FRT_HD double fdiv(double a, double b) { return a / b; }
FRT_HD float fsqrt(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
FRT_HD double fsqrt(double x) { return sqrt(x); }
FRT_HD float frsqrt(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_rsqf(x);
#else
    return 1.0f / sqrtf(x);
#endif
}
FRT_HD double frsqrt(double x) { return 1.0 / sqrt(x); }
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
FRT_HD void sincos_2pi(double r, double &s, double &c) { sincos(2.0 * Cst<double>::pi * r, &s, &c); }
// e^x for moderate |x| (PSS-MLT perturbation: x in [-8, 0])
FRT_HD float fexp(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_exp2f(x * 1.44269504088896340736f);
#else
    return expf(x);
#endif
}
FRT_HD double fexp(double x) { return exp(x); }
// ln x, x^y (x > 0) on the hardware log2 / exp2 (v_log_f32 / v_exp_f32)
FRT_HD float flog(float x)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_logf(x) * 0.69314718055994530942f;
#else
    return logf(x);
#endif
}
FRT_HD double flog(double x) { return log(x); }
FRT_HD float fpow(float x, float y)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#else
    return powf(x, y);
#endif
}
FRT_HD double fpow(double x, double y) { return pow(x, y); }
template <typename R> FRT_HD R rlen(V3<R> v) { return frsqrt(len2(v)); }
template <typename R> FRT_HD V3<R> normalize(V3<R> v) { return rlen(v) * v; }

// Ray prepared for slab tests: t = lo * invd + oinv with oinv = -o * invd
// (one FMA per slab plane).  Zero direction components are nudged to
// +-1e-30 so no 0*inf NaN can arise; the reference's NaN-tolerant compare
// (aabb.h:24-25) keeps the interval unchanged in that case, and so does this
// (the near-parallel slab spans +-huge).  Device boxes are padded outward, so
// neither the nudge nor the FMA rounding can cull a hit.
// a value every active lane holds, moved into a scalar register (plain on the host)
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ int frt_uniform(int x) { return __builtin_amdgcn_readfirstlane(x); }
#else
inline int frt_uniform(int x) { return x; }
#endif
template <typename R> struct SlabRay { V3<R> invd, oinv; };
template <typename R> FRT_HD SlabRay<R> slab_ray(V3<R> o, V3<R> d)
{
    const R tiny = R(1e-30f);
    const R dx = vabs(d.x) > tiny ? d.x : vcopysign(tiny, d.x);
    const R dy = vabs(d.y) > tiny ? d.y : vcopysign(tiny, d.y);
    const R dz = vabs(d.z) > tiny ? d.z : vcopysign(tiny, d.z);
    SlabRay<R> r;
    r.invd = V3<R>{rcp(dx), rcp(dy), rcp(dz)};
    r.oinv = V3<R>{-o.x * r.invd.x, -o.y * r.invd.y, -o.z * r.invd.z};
    return r;
}
// slab test of a box against [tmin, tmax]; returns entry distance or +inf on
// miss (aabb.h:14-31: the reference's per-axis early exit decides the same).
// The box planes are the padded fp32 boxes in either precision.
template <typename R>
FRT_HD R slab_entry(R lox, R loy, R loz, R hix, R hiy, R hiz, const SlabRay<R> &r, R tmin, R tmax)
{
    const R tx0 = vfma(lox, r.invd.x, r.oinv.x), tx1 = vfma(hix, r.invd.x, r.oinv.x);
    const R ty0 = vfma(loy, r.invd.y, r.oinv.y), ty1 = vfma(hiy, r.invd.y, r.oinv.y);
    const R tz0 = vfma(loz, r.invd.z, r.oinv.z), tz1 = vfma(hiz, r.invd.z, r.oinv.z);
    const R tn = smax(smax(smin(tx0, tx1), smin(ty0, ty1)), smax(smin(tz0, tz1), tmin));
    const R tf = smin(smin(smax(tx0, tx1), smax(ty0, ty1)), smin(smax(tz0, tz1), tmax));
    return (tf < tn) ? R(__builtin_inff()) : tn;
}

// the same test on a box stored as (near, far) planes for the ray's octant
// (bvh2_step OCT): bit-identical to slab_entry on the (lo, hi) box
template <typename R>
FRT_HD R slab_entry_nf(R nx, R ny, R nz, R fx, R fy, R fz, const SlabRay<R> &r, R tmin, R tmax)
{
    const R tn = smax(smax(vfma(nx, r.invd.x, r.oinv.x), vfma(ny, r.invd.y, r.oinv.y)),
                      smax(vfma(nz, r.invd.z, r.oinv.z), tmin));
    const R tf = smin(smin(vfma(fx, r.invd.x, r.oinv.x), vfma(fy, r.invd.y, r.oinv.y)),
                      smin(vfma(fz, r.invd.z, r.oinv.z), tmax));
    return (tf < tn) ? R(__builtin_inff()) : tn;
}
// ... as the interval itself: the box is hit iff tn <= tf, the same decision
// as slab_entry_nf's for a finite tmax (then tf is finite, so tn <= tf rules
// out tn = +inf), without the select to +inf and the compare against it
template <typename R>
FRT_HD void slab_nf(R nx, R ny, R nz, R fx, R fy, R fz, const SlabRay<R> &r, R tmin, R tmax, R &tn, R &tf)
{
    tn = smax(smax(vfma(nx, r.invd.x, r.oinv.x), vfma(ny, r.invd.y, r.oinv.y)), smax(vfma(nz, r.invd.z, r.oinv.z), tmin));
    tf = smin(smin(vfma(fx, r.invd.x, r.oinv.x), vfma(fy, r.invd.y, r.oinv.y)), smin(vfma(fz, r.invd.z, r.oinv.z), tmax));
}

// Moller-Trumbore (triangle.h:69-118): returns t, or -1 on miss.  Accepts
// t in (tmin, tmax] -- the caller resolves t == tmax with the DFS rank tie rule.
// STRAIGHT (fp32): straight-line code, the same values and decisions.  In a
// wave the early outs only skip work when every lane fails together; as
// branches they cost exec-mask bookkeeping and a branch per test.  Measured
// per plan (same call, profiles/r04/r04c): cornell_1m's 4-wide HBM plan
// +4.4 %, Cornell's LDS plan -2.4 % -- so only the 4-wide traversal uses it.
template <bool STRAIGHT = false, typename R>
FRT_HD R tri_intersect(V3<R> o, V3<R> d, V3<R> v0, V3<R> e1, V3<R> e2, R tmin, R tmax, R &u, R &v)
{
    if constexpr (STRAIGHT && !kIsF64<R>) {
        const V3<R> h = cross(d, e2);
        const R a = dot(e1, h);
        const R f = rcp(a);
        const V3<R> s = o - v0;
        u = f * dot(s, h);
        const V3<R> q = cross(s, e1);
        v = f * dot(d, q);
        const R t = f * dot(e2, q);
        const bool ok = a != R(0) && !(u < R(0) || u > R(1)) && v >= R(0) && u + v <= R(1) && t > tmin && t <= tmax;
        return ok ? t : R(-1);
    }
    const V3<R> h = cross(d, e2);
    const R a = dot(e1, h);
    if (a == R(0)) return R(-1);
    const R f = rcp(a);
    const V3<R> s = o - v0;
    u = f * dot(s, h);
    if (u < R(0) || u > R(1)) return R(-1);
    const V3<R> q = cross(s, e1);
    v = f * dot(d, q);
    if (!(v >= R(0) && u + v <= R(1))) return R(-1);
    const R t = f * dot(e2, q);
    return (t > tmin && t <= tmax) ? t : R(-1);
}

// sphere::hit (sphere.h:26-56): returns t or -1; accepts t in [tmin, tmax].
// The discriminant b^2 - a(|oc|^2 - r^2) loses ~|oc|^2/r^2 ulps to
// cancellation in fp32 (veach's r = 0.03 lights at distance 15: a 2 % error,
// which blurs the silhouette the fp64 reference draws sharply).  It is formed
// instead as a(r^2 - |oc - (b/a) d|^2) from the ray's perpendicular offset,
// which keeps the error relative to r^2 (Hearn-Baker form); same roots.
template <typename R> FRT_HD R sphere_intersect(V3<R> o, V3<R> d, V3<R> c, R r, R tmin, R tmax)
{
    const V3<R> oc = o - c;
    const R a = dot(d, d);
    const R b = dot(oc, d);
    const R ia = rcp(a);
    const V3<R> l = oc - (b * ia) * d;
    R disc = a * (r * r - dot(l, l));
    if (!(disc >= R(0))) return R(-1);
    disc = fsqrt(disc);
    R t = (-b - disc) * ia;
    if (t < tmin) t = (-b + disc) * ia;
    if (t < tmin || t > tmax) return R(-1);
    return t;
}

// onb::build_from_w (onb.h:18-30) + fromLocal
template <typename R> struct Onb { V3<R> u, v, w; };
template <typename R> FRT_HD Onb<R> onb_from_w(V3<R> n)
{
    Onb<R> b;
    b.w = n;
    if (vabs(n.x) > vabs(n.y)) {
        const R inv = frsqrt(n.x * n.x + n.z * n.z);
        b.v = V3<R>{n.z * inv, R(0), -n.x * inv};
    } else {
        const R inv = frsqrt(n.y * n.y + n.z * n.z);
        b.v = V3<R>{R(0), n.z * inv, -n.y * inv};
    }
    b.u = cross(b.v, b.w);
    return b;
}
template <typename R> FRT_HD V3<R> onb_local(const Onb<R> &b, V3<R> a) { return a.x * b.u + a.y * b.v + a.z * b.w; }

// pdf.h:13-23
template <typename R> FRT_HD V3<R> cosine_direction(R r0, R r1)
{
    const R r = fsqrt(r0);
    R sp, cp;
    sincos_2pi(r1, sp, cp);                       // phi = 2 pi r1
    return V3<R>{r * cp, r * sp, fsqrt(R(1) - r0)};
}
// pdf.h:38-44
template <typename R> FRT_HD V3<R> uniform_sphere(R u0, R u1)
{
    const R z = R(1) - R(2) * u0;
    const R r = fsqrt(vmax(R(0), R(1) - z * z));
    R sp, cp;
    sincos_2pi(u1, sp, cp);
    return V3<R>{r * cp, r * sp, z};
}
// pdf.h:46-56
template <typename R> FRT_HD V3<R> random_to_sphere(R radius, R dist2, R r1, R r2)
{
    const R z = R(1) + r2 * (fsqrt(R(1) - fdiv(radius * radius, dist2)) - R(1));
    R sp, cp;
    sincos_2pi(r1, sp, cp);
    const R s = fsqrt(R(1) - z * z);
    return V3<R>{cp * s, sp * s, z};
}
// x^y for x in [0, 1], y >= 0 (phong lobes): exp2(y log2 x) on the hardware
// units; y = 0 gives 1 for every x, std::pow's answer (0^0 = 1; the MTL
// default Ns is 0, so veach_mi's plates have y = 0 and see alpha = 0 often --
// exp2(0 * -inf) would be NaN)
FRT_HD float fpow01(float x, float y)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    return y == 0.0f ? 1.0f : __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#else
    return powf(x, y);
#endif
}
FRT_HD double fpow01(double x, double y) { return pow(x, y); }
// x^y for x in [0, 1], y >= 0 where the result only weights radiance (the
// phong lobe's pdf value and eval_bsdf; never a direction): the fp32 form as
// fpow01.  In the fp64 kernels, for y <= 64: log2 of the double's mantissa m
// on the fp32 unit with m's fp32 rounding residual carried to first order, the
// exponent kept exact, and 2^(y log2 x) rebuilt in double range.  What is left
// is v_log_f32's error, ~2^-22 absolute in log2 m, times y: relative error
// <= 64 * 2^-22 * ln 2 ~ 1.1e-5 at y = 64, 1.7e-7 at y = 1 (without
// the bound, Ns 1000-1024 reached ~1e-4).  No underflow before double's, so
// pdf == 0, which ends a path (path.cpp:84-86), comes out exactly where the
// double pow gives 0.  y = 0 gives 1 and x = 0 gives 0 (std::pow's values);
// larger exponents take OCML's double pow, as the host replay and the
// reference do.  The directions
// (cosine_power_generate) keep the double pow: they decide what the next ray
// hits.
FRT_HD float fpow01_w(float x, float y) { return fpow01(x, y); }
FRT_HD double fpow01_w(double x, double y)
{
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FRT_EXP_IEEE_MATH)
    if (y == 0.0) return 1.0;                                 // pow(x, 0) = 1 for every x (veach's plates: Ns 0)
    if (!(x > 0.0)) return x == 0.0 ? 0.0 : pow(x, y);
    if (y > 64.0) return pow(x, y);
    int k;
    const double m = frexp(x, &k);                            // x = m 2^k, m in [0.5, 1)
    const float mf = (float)m;
    const double lm = (double)__builtin_amdgcn_logf(mf) + (m - (double)mf) * (1.4426950408889634 / (double)mf);
    const double l = y * (lm + (double)k);                    // y log2 x
    if (l < -1100.0) return 0.0;
    const double li = floor(l);
    return ldexp((double)__builtin_amdgcn_exp2f((float)(l - li)), (int)li);
#else
    return pow(x, y);
#endif
}

// ---- specular materials (material.h:75-171, pdf.h:99-184, util.h:73-117) ----
template <typename R> FRT_HD V3<R> reflect(V3<R> v, V3<R> n) { return normalize(v - (R(2) * dot(v, n)) * n); }   // util.h:73-76
template <typename R> FRT_HD V3<R> refract(V3<R> wi, V3<R> n, R eta, R cos_t)                                    // util.h:79-84
{
    if (cos_t < R(0)) eta = rcp(eta);
    return normalize((dot(wi, n) * eta + cos_t) * n - eta * wi);
}
template <typename R> FRT_HD R fresnel_dielectric(R cos_i, R &cos_t_out, R eta)                                  // util.h:86-117
{
    if (eta == R(1)) { cos_t_out = -cos_i; return R(0); }
    const R scale = (cos_i > R(0)) ? rcp(eta) : eta;
    const R cos_t2 = R(1) - (R(1) - cos_i * cos_i) * (scale * scale);
    if (cos_t2 <= R(0)) { cos_t_out = R(0); return R(1); }      // total internal reflection
    const R ci = vabs(cos_i), ct = fsqrt(cos_t2);
    const R rs = fdiv(ci - eta * ct, ci + eta * ct);
    const R rp = fdiv(eta * ci - ct, eta * ci + ct);
    cos_t_out = (cos_i > R(0)) ? -ct : ct;
    return R(0.5f) * (rs * rs + rp * rp);
}
// cosine_power_pdf (pdf.h:99-136); the onb's w is the shading normal
template <typename R> FRT_HD R cosine_power_value(V3<R> n, V3<R> wi, R e, V3<R> wo)
{
    if (dot(n, wo) <= R(0) || dot(n, wi) <= R(0)) return R(0);
    const R alpha = vmax(R(0), dot(reflect(-wi, n), wo));
    return fpow01_w(alpha, e) * (e + R(1)) * (R(0.5f) * Cst<R>::inv_pi);
}
template <typename R> FRT_HD V3<R> cosine_power_generate(V3<R> n, V3<R> wi, R e, R s0, R s1)
{
    const V3<R> r = reflect(-wi, n);
    const R sin_a = fsqrt(R(1) - fpow01(s1, fdiv(R(2), e + R(1))));
    const R cos_a = fpow01(s1, rcp(e + R(1)));
    R sp, cp;
    sincos_2pi(s0, sp, cp);
    return onb_local(onb_from_w(r), V3<R>{sin_a * cp, sin_a * sp, cos_a});
}
// modified_phong::eval_bsdf (material.h:92-100), cosine included
template <typename R> FRT_HD V3<R> phong_eval(V3<R> kd, V3<R> ks, R e, V3<R> n, V3<R> wi, V3<R> wo)
{
    const R alpha = vmax(R(0), dot(normalize(reflect(-wi, n)), wo));
    const V3<R> result = Cst<R>::inv_pi * kd + ((e + R(2)) * (R(0.5f) * Cst<R>::inv_pi) * fpow01_w(alpha, e)) * ks;
    return dot(n, wo) * result;
}
// dielectric_pdf (pdf.h:138-184) and dielectric::eval_bsdf (material.h:146-171)
template <typename R> FRT_HD R dielectric_value(V3<R> n, V3<R> wi, R ior, V3<R> wo)
{
    R cos_t;
    const R F = fresnel_dielectric(dot(wi, n), cos_t, ior);
    if (dot(wi, n) * dot(wo, n) >= R(0))
        return (vabs(dot(reflect(-wi, n), wo) - R(1)) > Cst<R>::delta_eps) ? R(0) : F;
    return (vabs(dot(refract(wi, n, ior, cos_t), wo) - R(1)) > Cst<R>::delta_eps) ? R(0) : R(1) - F;
}
template <typename R> FRT_HD V3<R> dielectric_generate(V3<R> n, V3<R> wi, R ior, R s0)
{
    R cos_t;
    const R F = fresnel_dielectric(dot(wi, n), cos_t, ior);
    return (s0 <= F) ? reflect(-wi, n) : refract(wi, n, ior, cos_t);
}
template <typename R> FRT_HD V3<R> dielectric_eval(V3<R> ks, R ior, V3<R> n, V3<R> wi, V3<R> wo)
{
    R cos_t;
    const R F = fresnel_dielectric(dot(wi, n), cos_t, ior);
    if (dot(wi, n) * dot(wo, n) >= R(0)) {
        if (vabs(dot(reflect(-wi, n), wo) - R(1)) > Cst<R>::delta_eps) return zero3<R>();
        return F * ks;
    }
    if (vabs(dot(refract(wi, n, ior, cos_t), wo) - R(1)) > Cst<R>::delta_eps) return zero3<R>();
    const R factor = cos_t < R(0) ? rcp(ior) : ior;
    return (factor * factor * (R(1) - F)) * ks;
}

// ---- rough_conductor (material.h:246-315), roughconductor_pdf (pdf.h:231-486,
//      pdf.cpp:5-12), microfacet.h; isotropic alpha.  Restatement of the
//      oracle's rough_* functions (oracle/frt_oracle.c); in fp32 on the
//      hardware transcendentals (rcp, sqrt, rsq, exp2, log2, sin / cos in
//      revolutions) like the rest of the shading code, only acos stays libm.
//      The OCML tan / pow / atan2 / sin / cos and IEEE divisions of round 1
//      made this the register-hungriest part of the material kernels.  The
//      fitted polynomials keep their fp32 coefficients in both precisions. ----
constexpr int kDistGgx = 0, kDistBeckmann = 1;
template <typename R> FRT_HD R safe_sqrtf(R v) { const R r = fsqrt(v); return (R(0) < r) ? r : R(0); }   // util.h:43-46 (NaN -> 0)
template <typename R> FRT_HD V3<R> onb_to_local(const Onb<R> &b, V3<R> a) { return V3<R>{dot(a, b.u), dot(a, b.v), dot(a, b.w)}; }
// microfacet::fresnelConductorExact (microfacet.h:8-31), one channel
template <typename R> FRT_HD R fresnel_conductor1(R cos_i, R eta, R k)
{
    const R c2 = cos_i * cos_i, s2 = R(1) - c2, s4 = s2 * s2;
    const R temp1 = eta * eta - k * k - s2;
    const R a2pb2 = safe_sqrtf(temp1 * temp1 + R(4) * (k * k * eta * eta));
    const R a = safe_sqrtf(R(0.5f) * (a2pb2 + temp1));
    const R term1 = a2pb2 + c2, term2 = (R(2) * cos_i) * a;
    const R rs2 = fdiv(term1 - term2, term1 + term2);
    const R term3 = c2 * a2pb2 + s4, term4 = s2 * term2;
    const R rp2 = rs2 * fdiv(term3 - term4, term3 + term4);
    return R(0.5f) * (rp2 + rs2);
}
// microfacet::smithG1 (microfacet.h:48-88)
template <typename R> FRT_HD R smith_g1(V3<R> v, V3<R> m, V3<R> n, R alpha, int dist)
{
    const R cos_t = dot(n, v);
    if (dot(v, m) * cos_t <= R(0)) return R(0);
    const R temp = R(1) - cos_t * cos_t;
    if (temp <= R(0)) return R(1);
    const R tan_t = fdiv(fsqrt(temp), cos_t);
    if (dist == kDistBeckmann) {
        const R a = rcp(alpha * tan_t);
        if (a >= R(1.6f)) return R(1);
        const R a2 = a * a;
        return fdiv(R(3.535f) * a + R(2.181f) * a2, R(1) + R(2.276f) * a + R(2.577f) * a2);
    }
    const R root = alpha * tan_t;
    return fdiv(R(2), R(1) + fsqrt(R(1) + root * root));          // hypot2(1, root) (util.h:239-254)
}
// microfacet::eval (microfacet.h:90-135)
template <typename R> FRT_HD R microfacet_d(V3<R> m, V3<R> n, R alpha, int dist)
{
    const V3<R> ml = onb_to_local(onb_from_w(n), m);
    const R cos_t = ml.z;
    if (cos_t <= R(0)) return R(0);
    const R c2 = cos_t * cos_t, a2 = alpha * alpha;
    const R be = fdiv(fdiv(ml.x * ml.x, a2) + fdiv(ml.y * ml.y, a2), c2);
    R r;
    if (dist == kDistBeckmann) {
        r = fdiv(fexp(-be), Cst<R>::pi * a2 * c2 * c2);
    } else {
        const R root = (R(1) + be) * c2;
        r = rcp(Cst<R>::pi * a2 * root * root);
    }
    return (r * cos_t < R(1e-20f)) ? R(0) : r;
}
// util.h:185-236
template <typename R> FRT_HD R erfinv_f(R x)
{
    R w = -flog((R(1) - x) * (R(1) + x)), p;
    if (w < R(5)) {
        w = w - R(2.5f);
        p = R(2.81022636e-08f);
        p = R(3.43273939e-07f) + p * w;
        p = R(-3.5233877e-06f) + p * w;
        p = R(-4.39150654e-06f) + p * w;
        p = R(0.00021858087f) + p * w;
        p = R(-0.00125372503f) + p * w;
        p = R(-0.00417768164f) + p * w;
        p = R(0.246640727f) + p * w;
        p = R(1.50140941f) + p * w;
    } else {
        w = fsqrt(w) - R(3);
        p = R(-0.000200214257f);
        p = R(0.000100950558f) + p * w;
        p = R(0.00134934322f) + p * w;
        p = R(-0.00367342844f) + p * w;
        p = R(0.00573950773f) + p * w;
        p = R(-0.0076224613f) + p * w;
        p = R(0.00943887047f) + p * w;
        p = R(1.00167406f) + p * w;
        p = R(2.83297682f) + p * w;
    }
    return p * x;
}
template <typename R> FRT_HD R erf_f(R x)
{
    const R sign = vcopysign(R(1), x);
    x = vabs(x);
    const R t = rcp(R(1) + R(0.3275911f) * x);
    const R y = R(1) - (((((R(1.061405429f) * t - R(1.453152027f)) * t) + R(1.421413741f)) * t - R(0.284496736f)) * t +
                        R(0.254829592f)) * t * fexp(-x * x);
    return sign * y;
}
// roughconductor_pdf::sampleVisible11 (pdf.h:280-397)
// theta_i enters as cos / sin (cos_t = ws.z, sin_t = sqrt((1 - z)(1 + z)));
// normal: the reference's theta_i < 1e-4 test, which in fp32 holds exactly
// when rough_generate left theta at 0 (ws.z >= 0.99999: acos of anything
// below that is >= 4.5e-3).  tan(theta_i) = sin / cos, as tan(acos z) is;
// theta_i itself only for the Beckmann fit, so GGX lanes run no acos.
template <typename R>
FRT_HD void sample_visible11(bool normal, R cos_t, R sin_t, R sx, R sy, int dist, R &slx, R &sly)
{
    const R kSqrtPiInv = R(0.564189583547756287f);
    if (normal) {                                               // normal incidence
        const R r = (dist == kDistBeckmann) ? fsqrt(-flog(R(1) - sx)) : safe_sqrtf(fdiv(sx, R(1) - sx));
        R sp, cp;
        sincos_2pi(sy, sp, cp);                                 // phi = 2 pi sy
        slx = r * cp; sly = r * sp;
        return;
    }
    const R tan_t = fdiv(sin_t, cos_t);
    if (dist == kDistBeckmann) {
        const R theta_i = vacos(cos_t);
        const R cot_t = rcp(tan_t);
        R a = R(-1), c = erf_f(cot_t);
        const R sample_x = vmax(sx, R(1e-6f));
        const R fit = R(1) + theta_i * (R(-0.876f) + theta_i * (R(0.4265f) - R(0.0594f) * theta_i));
        R b = c - (R(1) + c) * fpow(R(1) - sample_x, fit);
        const R norm = rcp(R(1) + c + kSqrtPiInv * tan_t * fexp(-cot_t * cot_t));
        for (int it = 1; it < 10; ++it) {
            if (!(b >= a && b <= c)) b = R(0.5f) * (a + c);
            const R inv_erf = erfinv_f(b);
            const R value = norm * (R(1) + b + kSqrtPiInv * tan_t * fexp(-inv_erf * inv_erf)) - sample_x;
            const R deriv = norm * (R(1) - inv_erf * tan_t);
            if (vabs(value) < R(1e-5f)) break;
            if (value > R(0)) c = b; else a = b;
            b -= fdiv(value, deriv);
        }
        slx = erfinv_f(b);
        sly = erfinv_f(R(2) * vmax(sy, R(1e-6f)) - R(1));
        return;
    }
    const R a = rcp(tan_t);
    const R g1 = fdiv(R(2), R(1) + safe_sqrtf(R(1) + rcp(a * a)));
    R A = fdiv(R(2) * sx, g1) - R(1);
    if (vabs(A) == R(1)) A -= vcopysign(R(1), A) * Cst<R>::eps;
    const R tmp = rcp(A * A - R(1));
    const R B = tan_t;
    const R D = safe_sqrtf(B * B * tmp * tmp - (A * A - B * B) * tmp);
    const R s1 = B * tmp - D, s2 = B * tmp + D;
    slx = (A < R(0) || s2 > a) ? s1 : s2;
    R S;
    if (sy > R(0.5f)) { S = R(1); sy = R(2) * (sy - R(0.5f)); }
    else { S = R(-1); sy = R(2) * (R(0.5f) - sy); }
    const R z = fdiv(sy * (sy * (sy * R(-0.365728915865723f) + R(0.790235037209296f)) - R(0.424965825137544f)) +
                         R(0.000152998850436920f),
                     sy * (sy * (sy * (sy * R(0.169507819808272f) - R(0.397203533833404f)) - R(0.232500544458471f)) + R(1)) -
                         R(0.539825872510702f));
    sly = S * z * fsqrt(R(1) + slx * slx);
}
// roughconductor_pdf::generate (pdf.h:409-482, pdf.cpp:5-12): wo, and the
// sampled pdf (pdfVisible / (4 wo.m)) that path.cpp:82 prefers when > 0
template <typename R> FRT_HD V3<R> rough_generate(V3<R> n, V3<R> wi, R alpha, int dist, R s0, R s1, R &sampled_pdf)
{
    const Onb<R> uvw = onb_from_w(n);
    const V3<R> wl = onb_to_local(uvw, wi);
    V3<R> ws = V3<R>{alpha * wl.x, alpha * wl.y, wl.z};
    ws = frsqrt(len2(ws)) * ws;
    // theta = acos(ws.z) (0 at and above 0.99999), phi = atan2(ws.y, ws.x): sin / cos phi as
    // ws.y / r, ws.x / r; sample_visible11 takes theta as cos / sin
    const bool normal = !(ws.z < R(0.99999f));
    R sp = R(0), cp = R(1);
    if (!normal) {
        const R rr = ws.x * ws.x + ws.y * ws.y;
        if (rr > R(0)) { const R ir = frsqrt(rr); sp = ws.y * ir; cp = ws.x * ir; }
    }
    R slx, sly;
    sample_visible11(normal, ws.z, fsqrt((R(1) - ws.z) * (R(1) + ws.z)), s0, s1, dist, slx, sly);
    if (!(vabs(slx) <= R(3.40282347e+38f))) slx = R(0);          // !std::isfinite
    const R rx = (cp * slx - sp * sly) * alpha, ry = (sp * slx + cp * sly) * alpha;
    const R nrm = frsqrt(rx * rx + ry * ry + R(1));
    const V3<R> ml = V3<R>{-rx * nrm, -ry * nrm, nrm};
    const V3<R> mw = onb_local(uvw, ml);
    R pdf = R(0);
    if (wl.z != R(0))
        pdf = fdiv(smith_g1(onb_local(uvw, wl), mw, n, alpha, dist) * vabs(dot(wl, ml)) * microfacet_d(mw, n, alpha, dist),
                   vabs(wl.z));
    const V3<R> wo = reflect(-wi, mw);
    sampled_pdf = fdiv(pdf, R(4) * dot(wo, mw));
    return wo;
}
// roughconductor_pdf::value (pdf.h:237-250)
template <typename R> FRT_HD R rough_value(V3<R> n, V3<R> wi, R alpha, int dist, V3<R> wo)
{
    if (dot(n, wo) <= R(0) || dot(n, wi) <= R(0)) return R(0);
    const V3<R> H = normalize(wo + wi);
    return fdiv(microfacet_d(H, n, alpha, dist) * smith_g1(wi, H, n, alpha, dist), R(4) * dot(wi, n));
}
// rough_conductor::eval_bsdf (material.h:277-307); no cosine (is_specular)
template <typename R>
FRT_HD V3<R> rough_eval(V3<R> eta, V3<R> k, V3<R> spec, R alpha, int dist, V3<R> n, V3<R> wi, V3<R> wo)
{
    const R cos_wi = dot(wi, n);
    if (cos_wi <= R(0) || dot(wo, n) <= R(0)) return zero3<R>();
    const V3<R> H = normalize(wo + wi);
    const R D = microfacet_d(H, n, alpha, dist);
    if (D == R(0)) return zero3<R>();
    const R c = dot(wi, H);
    const V3<R> F = V3<R>{fresnel_conductor1(c, eta.x, k.x), fresnel_conductor1(c, eta.y, k.y),
                          fresnel_conductor1(c, eta.z, k.z)} * spec;
    const R G = smith_g1(wi, H, n, alpha, dist) * smith_g1(wo, H, n, alpha, dist);
    return fdiv(D * G, R(4) * cos_wi) * F;
}

// util.h:55-60
template <typename R> FRT_HD R mi_weight(R p1, R p2)
{
    p1 *= p1;
    p2 *= p2;
    return fdiv(p1, p1 + p2);
}

}  // namespace frt
