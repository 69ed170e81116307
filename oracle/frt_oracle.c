/*
 * frt_oracle.c -- TEST INFRASTRUCTURE ONLY.  See frt_oracle.h.
 *
 * fp64 CPU restatement of jammm/first_raytracer's path::Li hot path.  Every
 * arithmetic expression keeps the reference's operand order so the component
 * functions are bit-identical to the reference's own code (pinned by
 * tests/golden/kat_*.json, produced by oracle/_ref/ref_kat built from the
 * reference sources).  File:line citations are relative to
 * /root/reference/first_ray/.
 *
 * Build: see oracle/Makefile (gcc -O2 -ffp-contract=off, no -march: the
 * reference's x86-64 doubles are not FMA-contracted either).
 */
#define _GNU_SOURCE
#include "frt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* util.h:10-12 */
static const double EPSILON = 1e-4;
static const double SHADOW_EPSILON = (double)1e-3f;

/* ------------------------------------------------------------------------ */
/* RNG stream spec (DESIGN.md "RNG stream spec"; identical in csrc/frt_device.hpp) */
/* ------------------------------------------------------------------------ */
static inline uint32_t mix32(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
typedef struct { uint32_t k0, k1; } rng_key;
static inline rng_key rng_make(uint32_t seed, uint32_t pixel, uint32_t sample)
{
    uint32_t a = mix32(seed ^ 0x2545F491U);
    rng_key k;
    k.k0 = mix32(mix32(a ^ pixel) + sample * 0x9E3779B9U);
    k.k1 = mix32(mix32(a + pixel * 0x632BE5ABU) ^ (sample * 0x85157AF5U + 0x5851F42DU));
    return k;
}
static inline double rng_u(rng_key k, uint32_t dim)
{
    uint32_t h = mix32((k.k0 ^ (dim * 0x85EBCA77U + 0xC2B2AE3DU)) + k.k1);   /* one round per dimension (round 4) */
    return (double)(h >> 8) * (1.0 / 16777216.0);
}
double ora_rng_uniform(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t dim)
{
    return rng_u(rng_make(seed, pixel, sample), dim);
}
/* dimension layout: camera 0..3 (path.cpp:131-133); bounce at depth d uses
 * base = 4 + 8 d: scatter get3d +0..2 (path.cpp:36), light pick get1d +3
 * (path.cpp:39), light sample get2d +4..5 (path.cpp:45), bsdf get2d +6..7
 * (path.cpp:99). */
#define DIM_BOUNCE(d) (4u + 8u * (uint32_t)(d))

/* ------------------------------------------------------------------------ */
/* Vector3f (geometry.h:297-547), fp64                                       */
/* ------------------------------------------------------------------------ */
typedef struct { double e[3]; } v3;
static inline v3 mk(double x, double y, double z) { v3 r; r.e[0] = x; r.e[1] = y; r.e[2] = z; return r; }
static inline v3 vadd(v3 a, v3 b) { return mk(a.e[0] + b.e[0], a.e[1] + b.e[1], a.e[2] + b.e[2]); }
static inline v3 vsub(v3 a, v3 b) { return mk(a.e[0] - b.e[0], a.e[1] - b.e[1], a.e[2] - b.e[2]); }
static inline v3 vmul(v3 a, v3 b) { return mk(a.e[0] * b.e[0], a.e[1] * b.e[1], a.e[2] * b.e[2]); }
static inline v3 smul(double t, v3 v) { return mk(t * v.e[0], t * v.e[1], t * v.e[2]); }  /* t*v and v*t */
static inline v3 sdiv(v3 v, double t) { return mk(v.e[0] / t, v.e[1] / t, v.e[2] / t); }  /* v / t      */
static inline v3 vneg(v3 v) { return mk(-v.e[0], -v.e[1], -v.e[2]); }
static inline double dot(v3 a, v3 b) { return a.e[0] * b.e[0] + a.e[1] * b.e[1] + a.e[2] * b.e[2]; }
static inline v3 cross(v3 a, v3 b)
{
    return mk((a.e[1] * b.e[2]) - (a.e[2] * b.e[1]),
              (a.e[2] * b.e[0]) - (a.e[0] * b.e[2]),
              (a.e[0] * b.e[1]) - (a.e[1] * b.e[0]));
}
static inline double vlen(v3 v) { return sqrt(v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]); }
static inline double vlen2(v3 v) { return v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]; }
static inline v3 unit(v3 v) { return sdiv(v, vlen(v)); }                       /* geometry.h:468 */
static inline v3 make_unit(v3 v)                                             /* geometry.h:372 */
{
    double k = 1.0 / sqrt(v.e[0] * v.e[0] + v.e[1] * v.e[1] + v.e[2] * v.e[2]);
    return mk(v.e[0] * k, v.e[1] * k, v.e[2] * k);
}
static inline v3 vscale_inplace(v3 v, double t) { return mk(v.e[0] * t, v.e[1] * t, v.e[2] * t); } /* *= t */
static inline v3 vdiv_inplace(v3 v, double t)                                /* /= t: *= 1/t */
{
    double k = 1.0 / t;
    return mk(v.e[0] * k, v.e[1] * k, v.e[2] * k);
}
static inline v3 vload(const double *p) { return mk(p[0], p[1], p[2]); }
static inline void vstore(double *p, v3 v) { p[0] = v.e[0]; p[1] = v.e[1]; p[2] = v.e[2]; }
static inline double std_max(double a, double b) { return (a < b) ? b : a; }   /* std::max */

/* util.h:55-60 */
static inline double miWeight(double pdf1, double pdf2)
{
    pdf1 *= pdf1;
    pdf2 *= pdf2;
    return pdf1 / (pdf1 + pdf2);
}
/* util.h:62-66 */
static inline double FromSrgb(double v)
{
    if (v <= 0.04045) return v * (1.0 / 12.92);
    return pow((v + 0.055) * (1.0 / 1.055), 2.4);
}

/* ------------------------------------------------------------------------ */
/* ray / aabb / onb                                                         */
/* ------------------------------------------------------------------------ */
typedef struct { v3 o, d; } ray;
static inline v3 ray_at(const ray *r, double t) { return vadd(r->o, smul(t, r->d)); } /* ray.h:13 */

typedef struct { v3 min, max, size; } aabb;                                   /* aabb.h:6-68 */
static inline aabb aabb_mk(v3 lo, v3 hi) { aabb b; b.min = lo; b.max = hi; b.size = vsub(hi, lo); return b; }
static inline int aabb_hit(const aabb *b, const ray *r, double tmin, double tmax) /* aabb.h:14-31 */
{
    for (int i = 0; i < 3; ++i) {
        double invD = 1.0 / r->d.e[i];
        double t0 = (b->min.e[i] - r->o.e[i]) * invD;
        double t1 = (b->max.e[i] - r->o.e[i]) * invD;
        if (invD < 0.0) { double tt = t0; t0 = t1; t1 = tt; }
        tmin = t0 > tmin ? t0 : tmin;
        tmax = t1 < tmax ? t1 : tmax;
        if (tmax < tmin) return 0;
    }
    return 1;
}
static inline int aabb_longest_axis(const aabb *b)                           /* aabb.h:33-43 */
{
    int axis = 0;
    if (b->size.e[1] > b->size.e[0]) axis = 1;
    else if (b->size.e[2] > b->size.e[0]) axis = 2;
    return axis;
}
static inline double aabb_area(const aabb *b)                                /* aabb.h:46-49 */
{
    return 2 * ((b->size.e[0] * b->size.e[1]) + (b->size.e[1] * b->size.e[2]) + (b->size.e[0] * b->size.e[2]));
}
static inline aabb surrounding_box(aabb b0, aabb b1)                         /* aabb.h:57-68 */
{
    v3 small = mk(fmin(b0.min.e[0], b1.min.e[0]), fmin(b0.min.e[1], b1.min.e[1]), fmin(b0.min.e[2], b1.min.e[2]));
    v3 big = mk(fmax(b0.max.e[0], b1.max.e[0]), fmax(b0.max.e[1], b1.max.e[1]), fmax(b0.max.e[2], b1.max.e[2]));
    return aabb_mk(small, big);
}

typedef struct { v3 axis[3]; } onb;                                          /* onb.h:6-33 */
static inline onb onb_from_w(v3 n)
{
    onb b;
    b.axis[2] = n;
    if (fabs(n.e[0]) > fabs(n.e[1])) {
        double invLen = 1.0 / sqrt(n.e[0] * n.e[0] + n.e[2] * n.e[2]);
        b.axis[1] = mk(n.e[2] * invLen, (double)0.0f, -n.e[0] * invLen);
    } else {
        double invLen = 1.0 / sqrt(n.e[1] * n.e[1] + n.e[2] * n.e[2]);
        b.axis[1] = mk(0.0, n.e[2] * invLen, -n.e[1] * invLen);
    }
    b.axis[0] = cross(b.axis[1], b.axis[2]);
    return b;
}
static inline v3 onb_from_local(const onb *b, v3 a)                          /* onb.h:16 */
{
    return vadd(vadd(smul(a.e[0], b->axis[0]), smul(a.e[1], b->axis[1])), smul(a.e[2], b->axis[2]));
}

/* pdf.h:13-23 */
static inline v3 hemisphere_to_cosine_direction(double r0, double r1)
{
    const double r = sqrt(r0);
    const double phi = 2 * (double)M_PI * r1;
    const double x = r * cos(phi);
    const double y = r * sin(phi);
    return mk(x, y, sqrt(1 - r0));
}
/* pdf.h:38-44 */
static inline v3 uniform_sample_sphere(double u0, double u1)
{
    const double z = 1 - 2 * u0;
    const double r = sqrt(std_max((double)0, (double)1 - z * z));
    const double phi = 2 * (double)M_PI * u1;
    return mk(r * cos(phi), r * sin(phi), z);
}
/* pdf.h:46-56 */
static inline v3 random_to_sphere(double radius, double distance_squared, double r1, double r2)
{
    double z = 1 + r2 * (sqrt(1 - radius * radius / distance_squared) - 1);
    double phi = 2 * (double)M_PI * r1;
    double x = cos(phi) * sqrt(1 - z * z);
    double y = sin(phi) * sqrt(1 - z * z);
    return mk(x, y, z);
}
/* cosine_pdf (pdf.h:80-97): value uses uvw.w() == the normal */
static inline double cosine_pdf_value(v3 w, v3 direction)
{
    double c = dot(w, unit(direction));
    double cosine = (c < 0.0) ? 0.0 : c;   /* std::max<double>(c, 0.0) */
    return cosine / (double)M_PI;
}

enum { MAT_LAMBERT = 0, MAT_LIGHT = 1, MAT_PHONG = 2, MAT_METAL = 3, MAT_DIELECTRIC = 4,
       MAT_ROUGH = 5 };                                                      /* = FRT_MAT_* */
enum { DIST_GGX = 0, DIST_BECKMANN = 1 };                                     /* util.h:48-52 */
/* albedo: lambertian / modified_phong diffuse / metal albedo; ks: specular
 * reflectance (phong, dielectric, rough_conductor's constant texture) */
typedef struct {
    int type; v3 albedo; v3 emit; double ks[3], ior, shininess; int dist; double alpha; v3 eta, k;
    int tex; v3 tex_odd; double tex_scale[2];   /* checker_texture (texture.h:30-49) of the textured colour */
    int image;                                   /* image_texture (texture.h:51-95): scene image index */
} material;
enum { TEX_CONSTANT = 0, TEX_CHECKER = 1, TEX_IMAGE = 2 };
/* image_texture's decoded image: nx*ny*3 texel values, linear (FromSrgb(byte / 255)
 * for 8-bit images, the floats of an HDR image) */
typedef struct { int nx, ny; double *rgb; } ora_image;

/* ---- specular materials (material.h:75-171, pdf.h:99-184, util.h:73-117) ---- */
static const double DELTA_EPSILON = 1e-3f;                                   /* util.h:12 */
static inline v3 ref_reflect(v3 v, v3 n)                                     /* util.h:73-76 */
{
    return unit(vsub(v, smul(2 * dot(v, n), n)));
}
static inline v3 ref_refract(v3 wi, v3 n, double eta, double cosThetaT)      /* util.h:79-84 */
{
    if (cosThetaT < 0) eta = 1 / eta;
    return unit(vsub(smul(dot(wi, n) * eta + cosThetaT, n), smul(eta, wi)));
}
static inline double fresnelDielectricExt(double cosThetaI_, double *cosThetaT_, double eta)   /* util.h:86-117 */
{
    if (eta == 1) { *cosThetaT_ = -cosThetaI_; return 0.0; }
    double scale = (cosThetaI_ > 0) ? 1 / eta : eta,
           cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0) { *cosThetaT_ = 0.0; return 1.0; }
    double cosThetaI = fabs(cosThetaI_);
    double cosThetaT = sqrt(cosThetaTSqr);
    double Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    double Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    *cosThetaT_ = (cosThetaI_ > 0) ? -cosThetaT : cosThetaT;
    return 0.5 * (Rs * Rs + Rp * Rp);
}
/* cosine_power_pdf (pdf.h:99-136); uvw.w() is the normal, wi = hrec.wi */
static inline double cosine_power_value(v3 n, v3 wi, double e, v3 wo)
{
    if (dot(n, wo) <= 0 || dot(n, wi) <= 0) return 0.0;
    const double alpha = std_max(0.0, dot(ref_reflect(vneg(wi), n), wo));
    const double specular_pdf = pow(alpha, e);
    return specular_pdf * (e + 1.0) / (2 * (double)M_PI);
}
static inline v3 cosine_power_generate(v3 n, v3 wi, double e, double s0, double s1)
{
    v3 R = ref_reflect(vneg(wi), n);
    double sinAlpha = sqrt(1 - pow(s1, 2 / (e + 1)));
    double cosAlpha = pow(s1, 1 / (e + 1));
    double phi = (2.0 * M_PI) * s0;
    v3 localDir = mk(sinAlpha * cos(phi), sinAlpha * sin(phi), cosAlpha);
    onb b = onb_from_w(R);
    return onb_from_local(&b, localDir);
}
/* modified_phong::eval_bsdf (material.h:92-100), cosine included */
static inline v3 phong_eval(v3 kd, const double ks[3], double e, v3 n, v3 wi, v3 wo)
{
    const v3 reflected = unit(ref_reflect(vneg(wi), n));
    const double alpha = std_max(0.0, dot(reflected, wo));
    const double k = (e + 2) / (2 * M_PI), pw = pow(alpha, e);
    const v3 spec = mk(ks[0] * k * pw, ks[1] * k * pw, ks[2] * k * pw);
    const v3 result = vadd(sdiv(kd, M_PI), spec);
    return smul(dot(n, wo), result);
}
/* dielectric_pdf (pdf.h:138-184) */
static inline double dielectric_value(v3 n, v3 wi, double ior, v3 wo)
{
    double cosThetaT;
    double F = fresnelDielectricExt(dot(wi, n), &cosThetaT, ior);
    if (dot(wi, n) * dot(wo, n) >= 0) {
        if (fabs(dot(ref_reflect(vneg(wi), n), wo) - 1) > DELTA_EPSILON) return 0.0;
        return F;
    }
    if (fabs(dot(ref_refract(wi, n, ior, cosThetaT), wo) - 1) > DELTA_EPSILON) return 0.0;
    return 1.0 - F;
}
static inline v3 dielectric_generate(v3 n, v3 wi, double ior, double s0)
{
    double cosThetaT;
    double F = fresnelDielectricExt(dot(wi, n), &cosThetaT, ior);
    if (s0 <= F) return ref_reflect(vneg(wi), n);
    return ref_refract(wi, n, ior, cosThetaT);
}
/* dielectric::eval_bsdf (material.h:146-171) */
static inline v3 dielectric_eval(const double ks[3], double ior, v3 n, v3 wi, v3 wo)
{
    double cosThetaT;
    double F = fresnelDielectricExt(dot(wi, n), &cosThetaT, ior);
    if (dot(wi, n) * dot(wo, n) >= 0) {
        if (fabs(dot(ref_reflect(vneg(wi), n), wo) - 1) > DELTA_EPSILON) return mk(0.0, 0.0, 0.0);
        return mk(ks[0] * F, ks[1] * F, ks[2] * F);
    }
    if (fabs(dot(ref_refract(wi, n, ior, cosThetaT), wo) - 1) > DELTA_EPSILON) return mk(0.0, 0.0, 0.0);
    double factor = cosThetaT < 0 ? (1.0 / ior) : (ior);
    return mk(ks[0] * factor * factor * (1 - F), ks[1] * factor * factor * (1 - F), ks[2] * factor * factor * (1 - F));
}

/* ---- metal (material.h:110-130) ---- */
/* metal::scatter: reflect(unit(r_in.d), n) (util.h:73-76); constant_pdf(1)
 * (pdf.h:186-201); eval_bsdf = albedo */

/* ---- rough_conductor (material.h:246-315), roughconductor_pdf (pdf.h:231-486,
 *      pdf.cpp:5-12), microfacet.h; isotropic (alphaU = alphaV = alpha) ---- */
static inline double safe_sqrt1(double v) { return std_max(0.0, sqrt(v)); }       /* util.h:43-46 */
static inline v3 safe_sqrt3(v3 v)                                                 /* geometry.h:451-460 */
{
    return mk(std_max(0.0, sqrt(v.e[0])), std_max(0.0, sqrt(v.e[1])), std_max(0.0, sqrt(v.e[2])));
}
static inline v3 vdiv(v3 a, v3 b) { return mk(a.e[0] / b.e[0], a.e[1] / b.e[1], a.e[2] / b.e[2]); }
static inline v3 vsplat(double x) { return mk(x, x, x); }
static inline double hypot2(double a, double b)                                   /* util.h:239-254 */
{
    double r;
    if (fabs(a) > fabs(b)) { r = b / a; r = fabs(a) * sqrt(1.0 + r * r); }
    else if (b != 0.0) { r = a / b; r = fabs(b) * sqrt(1.0 + r * r); }
    else r = 0.0;
    return r;
}
static inline double erfinv(double x)                                             /* util.h:185-214 */
{
    double w = -log(((double)1 - x) * ((double)1 + x));
    double p;
    if (w < (double)5) {
        w = w - (double)2.5;
        p = (double)2.81022636e-08;
        p = (double)3.43273939e-07 + p * w;
        p = (double)-3.5233877e-06 + p * w;
        p = (double)-4.39150654e-06 + p * w;
        p = (double)0.00021858087 + p * w;
        p = (double)-0.00125372503 + p * w;
        p = (double)-0.00417768164 + p * w;
        p = (double)0.246640727 + p * w;
        p = (double)1.50140941 + p * w;
    } else {
        w = sqrt(w) - (double)3;
        p = (double)-0.000200214257;
        p = (double)0.000100950558 + p * w;
        p = (double)0.00134934322 + p * w;
        p = (double)-0.00367342844 + p * w;
        p = (double)0.00573950773 + p * w;
        p = (double)-0.0076224613 + p * w;
        p = (double)0.00943887047 + p * w;
        p = (double)1.00167406 + p * w;
        p = (double)2.83297682 + p * w;
    }
    return p * x;
}
static inline double erf_(double x)                                               /* util.h:216-236 */
{
    const double a1 = 0.254829592, a2 = -0.284496736, a3 = 1.421413741, a4 = -1.453152027, a5 = 1.061405429,
                 pp = 0.3275911;
    const double sign = copysignf(1.0f, (float)x);
    x = fabs(x);
    const double t = 1.0 / (1.0 + pp * x);
    const double y = 1.0 - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * exp(-x * x);
    return sign * y;
}
/* util.h:139-148: sincos of a double through sinf / cosf.  (Under _GNU_SOURCE,
 * util.h:134-136 makes sincos(double) call itself and never return; this is
 * the reference's other configuration, see oracle/ref_kat_conductor.cpp.) */
static inline void sincos_f(double theta, double *sn, double *cs)
{
    *sn = sinf((float)theta);
    *cs = cosf((float)theta);
}
static inline v3 onb_to_local(const onb *b, v3 a)                                 /* onb.h:17 */
{
    return mk(dot(a, b->axis[0]), dot(a, b->axis[1]), dot(a, b->axis[2]));
}
/* microfacet::fresnelConductorExact (microfacet.h:8-31) */
static inline v3 fresnel_conductor_exact(double cosThetaI, v3 eta, v3 k)
{
    const double cosThetaI2 = cosThetaI * cosThetaI, sinThetaI2 = 1 - cosThetaI2, sinThetaI4 = sinThetaI2 * sinThetaI2;
    const v3 temp1 = vsub(vsub(vmul(eta, eta), vmul(k, k)), vsplat(sinThetaI2));
    const v3 a2pb2 = safe_sqrt3(vadd(vmul(temp1, temp1), smul(4, vmul(vmul(vmul(k, k), eta), eta))));
    const v3 a = safe_sqrt3(smul(0.5, vadd(a2pb2, temp1)));
    const v3 term1 = vadd(a2pb2, vsplat(cosThetaI2)), term2 = smul(2 * cosThetaI, a);
    const v3 Rs2 = vdiv(vsub(term1, term2), vadd(term1, term2));
    const v3 term3 = vadd(smul(cosThetaI2, a2pb2), vsplat(sinThetaI4)), term4 = smul(sinThetaI2, term2);
    const v3 Rp2 = vdiv(vmul(Rs2, vsub(term3, term4)), vadd(term3, term4));
    return smul(0.5, vadd(Rp2, Rs2));
}
/* microfacet::smithG1 (microfacet.h:48-88); projectRoughness returns alpha
 * for the isotropic case (microfacet.h:33-46) */
static inline double smith_g1(v3 v, v3 m, v3 n, double alpha, int dist)
{
    const double cosTheta = dot(n, v);
    if (dot(v, m) * cosTheta <= 0) return 0.0;
    const double temp = 1 - (cosTheta * cosTheta);
    if (temp <= 0.0) return 1.0;
    const double tanTheta = sqrt(temp) / cosTheta;
    if (dist == DIST_BECKMANN) {
        const double a = 1.0 / (alpha * tanTheta);
        if (a >= 1.6f) return 1.0;
        const double aSqr = a * a;
        return ((double)3.535f * a + (double)2.181f * aSqr) / (1.0 + (double)2.276f * a + (double)2.577f * aSqr);
    }
    const double root = alpha * tanTheta;
    return 2.0 / (1.0 + hypot2(1.0, root));
}
/* microfacet::eval (microfacet.h:90-135) */
static inline double microfacet_d(v3 m, v3 n, double alpha, int dist)
{
    const onb b = onb_from_w(n);
    const v3 ml = onb_to_local(&b, m);
    const double cosTheta = ml.e[2];
    if (cosTheta <= 0) return 0.0;
    const double cosTheta2 = cosTheta * cosTheta;
    const double be = ((ml.e[0] * ml.e[0]) / (alpha * alpha) + (ml.e[1] * ml.e[1]) / (alpha * alpha)) / cosTheta2;
    double result;
    if (dist == DIST_BECKMANN) {
        result = exp(-be) / (M_PI * alpha * alpha * cosTheta2 * cosTheta2);
    } else {
        const double root = ((double)1 + be) * cosTheta2;
        result = (double)1 / (M_PI * alpha * alpha * root * root);
    }
    if (result * cosTheta < (double)1e-20f) result = 0;
    return result;
}
/* roughconductor_pdf::sampleVisible11 (pdf.h:280-397) */
static void sample_visible11(double thetaI, double sx, double sy, int dist, double *slope_x, double *slope_y)
{
    const double SQRT_PI_INV = 1 / sqrt(M_PI);
    if (dist == DIST_BECKMANN) {
        if (thetaI < 1e-4f) {
            double sinPhi, cosPhi;
            const double r = sqrt(-log(1.0 - sx));
            sincos_f(2 * M_PI * sy, &sinPhi, &cosPhi);
            *slope_x = r * cosPhi; *slope_y = r * sinPhi;
            return;
        }
        const double tanThetaI = tan(thetaI), cotThetaI = 1 / tanThetaI;
        double a = -1, c = erf_(cotThetaI);
        const double sample_x = std_max(sx, (double)1e-6f);
        const double fit = 1 + thetaI * ((double)-0.876f + thetaI * ((double)0.4265f - (double)0.0594f * thetaI));
        double b = c - (1 + c) * pow(1 - sample_x, fit);
        const double normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * exp(-cotThetaI * cotThetaI));
        int it = 0;
        while (++it < 10) {
            if (!(b >= a && b <= c)) b = 0.5 * (a + c);
            const double invErf = erfinv(b);
            const double value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * exp(-invErf * invErf)) - sample_x;
            const double derivative = normalization * (1 - invErf * tanThetaI);
            if (fabs(value) < 1e-5f) break;
            if (value > 0) c = b; else a = b;
            b -= value / derivative;
        }
        *slope_x = erfinv(b);
        *slope_y = erfinv(2.0 * std_max(sy, (double)1e-6f) - 1.0);
        return;
    }
    if (thetaI < 1e-4f) {
        double sinPhi, cosPhi;
        const double r = safe_sqrt1(sx / (1 - sx));
        sincos_f(2 * M_PI * sy, &sinPhi, &cosPhi);
        *slope_x = r * cosPhi; *slope_y = r * sinPhi;
        return;
    }
    const double tanThetaI = tan(thetaI);
    const double a = 1 / tanThetaI;
    const double G1 = 2.0 / (1.0 + safe_sqrt1(1.0 + 1.0 / (a * a)));
    double A = 2.0 * sx / G1 - 1.0;
    if (fabs(A) == 1) A -= (double)copysignf(1.0f, (float)A) * EPSILON;
    const double tmp = 1.0 / (A * A - 1.0);
    const double B = tanThetaI;
    const double D = safe_sqrt1(B * B * tmp * tmp - (A * A - B * B) * tmp);
    const double slope_x_1 = B * tmp - D, slope_x_2 = B * tmp + D;
    *slope_x = (A < 0.0 || slope_x_2 > 1.0 / tanThetaI) ? slope_x_1 : slope_x_2;
    double S;
    if (sy > 0.5) { S = 1.0; sy = 2.0 * (sy - 0.5); }
    else { S = -1.0; sy = 2.0 * (0.5 - sy); }
    const double z = (sy * (sy * (sy * (-(double)0.365728915865723) + (double)0.790235037209296) -
                            (double)0.424965825137544) + (double)0.000152998850436920) /
                     (sy * (sy * (sy * (sy * (double)0.169507819808272 - (double)0.397203533833404) -
                                  (double)0.232500544458471) + (double)1) - (double)0.539825872510702);
    *slope_y = S * z * sqrt(1.0 + *slope_x * *slope_x);
}
/* roughconductor_pdf::sampleVisible (pdf.h:409-455), local frame */
static v3 sample_visible(v3 wi_l, double sx, double sy, double alpha, int dist)
{
    const v3 wi = unit(mk(alpha * wi_l.e[0], alpha * wi_l.e[1], wi_l.e[2]));
    double theta = 0, phi = 0;
    if (wi.e[2] < (double)0.99999) {
        theta = acos(wi.e[2]);
        phi = atan2(wi.e[1], wi.e[0]);
    }
    double sinPhi, cosPhi;
    sincos_f(phi, &sinPhi, &cosPhi);
    double slx, sly;
    sample_visible11(theta, sx, sy, dist, &slx, &sly);
    if (!isfinite(slx)) slx = 0.0;
    const double rx = cosPhi * slx - sinPhi * sly, ry = sinPhi * slx + cosPhi * sly;
    slx = rx * alpha;
    sly = ry * alpha;
    const double normalization = (double)1 / sqrt(slx * slx + sly * sly + (double)1.0);
    return mk(-slx * normalization, -sly * normalization, normalization);
}
/* roughconductor_pdf::pdfVisible (pdf.cpp:5-12) */
static inline double pdf_visible(const onb *uvw, v3 wi_l, v3 m_l, v3 n, double alpha, int dist)
{
    const double cosTheta = wi_l.e[2];
    if (cosTheta == 0) return 0.0;
    const v3 mw = onb_from_local(uvw, m_l);
    return smith_g1(onb_from_local(uvw, wi_l), mw, n, alpha, dist) * fabs(dot(wi_l, m_l)) *
           microfacet_d(mw, n, alpha, dist) / fabs(cosTheta);
}
/* roughconductor_pdf::generate (pdf.h:465-482): wo and srec.sampled_pdf */
static v3 rough_generate(v3 n, v3 wi, double alpha, int dist, double s0, double s1, double *sampled_pdf)
{
    const onb uvw = onb_from_w(n);
    const v3 wi_l = onb_to_local(&uvw, wi);
    const v3 m = sample_visible(wi_l, s0, s1, alpha, dist);
    double pdf = pdf_visible(&uvw, wi_l, m, n, alpha, dist);
    const v3 mw = onb_from_local(&uvw, m);
    const v3 wo = ref_reflect(vneg(wi), mw);
    pdf /= 4.0 * dot(wo, mw);
    *sampled_pdf = pdf;
    return wo;
}
/* roughconductor_pdf::value (pdf.h:237-250) */
static inline double rough_value(v3 n, v3 wi, double alpha, int dist, v3 wo)
{
    if (dot(n, wo) <= 0 || dot(n, wi) <= 0) return 0.0;
    const v3 H = unit(vadd(wo, wi));
    const double e = microfacet_d(H, n, alpha, dist);
    return e * smith_g1(wi, H, n, alpha, dist) / (4.0 * dot(wi, n));
}
/* rough_conductor::eval_bsdf (material.h:277-307) */
static inline v3 rough_eval(const material *m, v3 n, v3 wi, v3 wo)
{
    const double cosWi = dot(wi, n);
    if (cosWi <= 0 || dot(wo, n) <= 0) return mk(0.0, 0.0, 0.0);
    const v3 H = unit(vadd(wo, wi));
    const double D = microfacet_d(H, n, m->alpha, m->dist);
    if (D == 0) return mk(0.0, 0.0, 0.0);
    const v3 F = vmul(fresnel_conductor_exact(dot(wi, H), m->eta, m->k), vload(m->ks));
    const double G = smith_g1(wi, H, n, m->alpha, m->dist) * smith_g1(wo, H, n, m->alpha, m->dist);
    const double model = D * G / (4.0 * cosWi);
    return smul(model, F);
}

/* ---- the specular materials behind one interface (path.cpp:78-95) ---- */
static inline int mat_scatters(int t)
{
    return t == MAT_LAMBERT || t == MAT_PHONG || t == MAT_METAL || t == MAT_DIELECTRIC || t == MAT_ROUGH;
}
/* light hits after these return Le unweighted (path.cpp:18-22, pssmlt.cpp:168-172) */
static inline int mat_no_mis(int t) { return t == MAT_PHONG || t == MAT_METAL || t == MAT_DIELECTRIC; }
/* scatter's direction (srec.specular_ray.d) from the get3d sample, and srec.sampled_pdf */
static inline v3 spec_generate(const material *m, v3 n, v3 wi, v3 rd, double s0, double s1, double *sampled_pdf)
{
    *sampled_pdf = -1.0;                                   /* scatter_record ctor (pdf.h:69) */
    switch (m->type) {
    case MAT_PHONG: return cosine_power_generate(n, wi, m->shininess, s0, s1);
    case MAT_DIELECTRIC: return dielectric_generate(n, wi, m->ior, s0);
    case MAT_METAL: return ref_reflect(unit(rd), n);       /* reflect(unit(r_in.d), n) */
    default: return unit(rough_generate(n, wi, m->alpha, m->dist, s0, s1, sampled_pdf));
    }
}
static inline double spec_value(const material *m, v3 n, v3 wi, v3 wo)   /* srec.pdf_ptr->value */
{
    switch (m->type) {
    case MAT_PHONG: return cosine_power_value(n, wi, m->shininess, wo);
    case MAT_DIELECTRIC: return dielectric_value(n, wi, m->ior, wo);
    case MAT_METAL: return 1.0;
    default: return rough_value(n, wi, m->alpha, m->dist, wo);
    }
}
static inline v3 spec_eval(const material *m, v3 n, v3 wi, v3 wo)        /* eval_bsdf */
{
    switch (m->type) {
    case MAT_PHONG: return phong_eval(m->albedo, m->ks, m->shininess, n, wi, wo);
    case MAT_DIELECTRIC: return dielectric_eval(m->ks, m->ior, n, wi, wo);
    case MAT_METAL: return m->albedo;
    default: return rough_eval(m, n, wi, wo);
    }
}

/* util.h:21-41 */
static inline void random_in_unit_disk(double s0, double s1, double *ox, double *oy)
{
    double a = s0 * 2.0 - 1.0, b = s1 * 2.0 - 1.0;
    if (a == 0.0 && b == 0.0) { *ox = 0.0; *oy = 0.0; return; }
    double a2 = a * a, b2 = b * b, phi, r;
    if (a2 > b2) { r = a; phi = (M_PI / 4.0) * (b / a); }
    else { r = b; phi = (M_PI / 2.0) - (M_PI / 4.0) * (a / b); }
    double cosphi = cos(phi), sinphi = sin(phi);
    *ox = r * cosphi; *oy = r * sinphi;
}

/* ------------------------------------------------------------------------ */
/* camera (camera.h:10-35)                                                  */
/* ------------------------------------------------------------------------ */
typedef struct { v3 origin, llc, horizontal, vertical, u, v, w; double lens_radius, half_height; } camera;
static camera camera_mk(v3 lookfrom, v3 lookat, v3 vup, double vfov, double aspect, double aperture, double focus_dist)
{
    camera c;
    c.lens_radius = aperture / 2;
    double theta = vfov * (double)M_PI / 180.0;
    double half_height = tan(theta / 2);
    double half_width = aspect * half_height;
    c.half_height = half_height;
    c.origin = lookfrom;
    c.w = unit(vsub(lookfrom, lookat));
    c.u = unit(cross(vup, c.w));
    c.v = cross(c.w, c.u);
    c.llc = vsub(vsub(vsub(c.origin, smul(half_width * focus_dist, c.u)), smul(half_height * focus_dist, c.v)),
                 smul(focus_dist, c.w));
    c.horizontal = smul(2 * half_width * focus_dist, c.u);
    c.vertical = smul(2 * half_height * focus_dist, c.v);
    return c;
}
static inline ray camera_get_ray(const camera *c, double s, double t, double l0, double l1)
{
    double rx, ry;
    if (c->lens_radius == 0) { rx = c->lens_radius; ry = c->lens_radius; }
    else { random_in_unit_disk(l0, l1, &rx, &ry); rx = c->lens_radius * rx; ry = c->lens_radius * ry; }
    v3 offset = vadd(smul(rx, c->u), smul(ry, c->v));
    ray r;
    r.o = vadd(c->origin, offset);
    r.d = vsub(vsub(vadd(vadd(c->llc, smul(s, c->horizontal)), smul(t, c->vertical)), c->origin), offset);
    return r;
}

/* ------------------------------------------------------------------------ */
/* scene                                                                    */
/* ------------------------------------------------------------------------ */

typedef struct {
    v3 v0, v1, v2, e1, e2;      /* triangle.h:58-66 (edges from the fp64 vertices) */
    v3 n0, n1, n2;              /* vertex normals (mesh->normals)                  */
    double uv[6];               /* mesh->uv of v0, v1, v2 (0 without vt)            */
    double inv_area;            /* 1/(0.5 |e1 x e2| nTriangles_of_mesh)            */
    int mat, geo;               /* material, use_geometry_normals                  */
} tri;
typedef struct { v3 c; double r; int mat; } sphere;

typedef struct { aabb box; int32_t left, right; } bnode;                     /* child<0: ~prim_ref */

#define REF_SPHERE (1 << 30)
enum { WORLD_BVH = 0, WORLD_LIST = 1 };

struct ora_scene {
    tri *tris; int ntris;
    sphere *sph; int nsph;
    material *mats; int nmats;
    int world_kind;
    bnode *nodes; int nnodes; int32_t root;   /* root >= 0 node, < 0 single prim leaf */
    int32_t *list; int nlist;                 /* prim refs, list worlds         */
    int32_t *lights; int nlights;             /* prim refs (Scene::lights)       */
    camera cam;
    v3 env;
    int bvh_depth;
    ora_image *images; int nimages;
};

typedef struct {
    double t;
    v3 p, normal;
    int32_t obj;     /* prim ref */
    int mat;
    double tu, tv;   /* hrec.u, hrec.v: texture coordinates (triangle.h:105-107, sphere.h:52) */
} hit_record;

/* (int)x as x86-64's cvttsd2si computes it: NaN and out-of-range give INT_MIN
 * (the C++ conversion is undefined there; checker_texture hits it through
 * get_sphere_uv's NaN on large spheres) */
static inline int x86_trunc(double x)
{
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return (int)x;
}
static inline int imodulo(int a, int b) { int r = a % b; return (r < 0) ? r + b : r; }   /* util.h:125-128 */
/* checker_texture::value (texture.h:35-44): 1 -> tex1 (odd), 0 -> tex0 */
static inline int checker_odd(double u, double v, double us, double vs)
{
    const int x = 2 * imodulo(x86_trunc(u * us * 2), 2) - 1, y = 2 * imodulo(x86_trunc(v * vs * 2), 2) - 1;
    return x * y == 1;
}
/* the hit's material with its texture evaluated: lambertian albedo,
 * modified_phong diffuse_reflectance, dielectric / rough_conductor specular */
/* image_texture::value (texture.h:59-88): nearest texel, out-of-range indices
 * wrapped (util.h:125-128 modulo), the upper edge clamped */
static v3 image_value(const ora_image *img, double u, double v)
{
    const int nx = img->nx, ny = img->ny;
    int i = x86_trunc(u * nx), j = x86_trunc(v * ny);
    if (i < 0 || i > nx) i = imodulo(i, nx);
    if (j < 0 || j > ny) j = imodulo(j, ny);
    if (i == nx) i = nx - 1;
    if (j == ny) j = ny - 1;
    return vload(img->rgb + 3 * ((size_t)j * nx + i));
}
static const material *mat_at(const ora_scene *s, const hit_record *h, material *tmp)
{
    const material *m = &s->mats[h->mat];
    if (m->tex == TEX_IMAGE) {
        *tmp = *m;
        const v3 c = image_value(&s->images[m->image], h->tu, h->tv);
        if (m->type == MAT_LAMBERT || m->type == MAT_PHONG) tmp->albedo = c;
        else vstore(tmp->ks, c);
        return tmp;
    }
    if (m->tex != TEX_CHECKER) return m;
    *tmp = *m;
    if (checker_odd(h->tu, h->tv, m->tex_scale[0], m->tex_scale[1])) {
        if (m->type == MAT_LAMBERT || m->type == MAT_PHONG) tmp->albedo = m->tex_odd;
        else vstore(tmp->ks, m->tex_odd);
    }
    return tmp;
}


/* triangle::hit (triangle.h:69-118) */
static int tri_hit(const tri *tr, const ray *r, double t_min, double t_max, hit_record *hrec, double *uo, double *vo)
{
    double a, f, u, v;
    const v3 h = cross(r->d, tr->e2);
    a = dot(tr->e1, h);
    if (a == 0) return 0;
    f = 1.0 / a;
    v3 s = vsub(r->o, tr->v0);
    u = f * dot(s, h);
    if (u < 0.0 || u > 1.0) return 0;
    v3 q = cross(s, tr->e1);
    v = f * dot(r->d, q);
    if (v >= 0.0 && u + v <= 1.0) {
        double t = f * dot(tr->e2, q);
        if (t > t_min && t < t_max) {
            hrec->t = t;
            hrec->p = ray_at(r, t);
            if (tr->geo)
                hrec->normal = unit(cross(tr->e1, tr->e2));
            else
                hrec->normal = unit(vadd(vadd(smul((1 - u - v), tr->n0), smul(u, tr->n1)), smul(v, tr->n2)));
            hrec->mat = tr->mat;
            /* uvhit = (1-u-v) uv0 + u uv1 + v uv2 (triangle.h:105) */
            hrec->tu = ((1 - u - v) * tr->uv[0] + u * tr->uv[2]) + v * tr->uv[4];
            hrec->tv = ((1 - u - v) * tr->uv[1] + u * tr->uv[3]) + v * tr->uv[5];
            if (uo) { *uo = u; *vo = v; }
            return 1;
        }
    }
    return 0;
}
/* sphere::hit (sphere.h:26-56) */
static int sphere_hit(const sphere *sp, const ray *r, double t_min, double t_max, hit_record *rec)
{
    v3 oc = vsub(r->o, sp->c);
    const double a = dot(r->d, r->d);
    const double b = dot(oc, r->d);
    const double c = dot(oc, oc) - sp->r * sp->r;
    double discriminant = b * b - a * c;
    if (discriminant >= 0.0) {
        discriminant = sqrt(discriminant);
        double t = (-b - discriminant) / a;
        if (t < t_min) t = (-b + discriminant) / a;
        if (t < t_min || t > t_max) return 0;
        rec->t = t;
        rec->p = ray_at(r, rec->t);
        rec->normal = sdiv(vsub(rec->p, sp->c), sp->r);
        if (vlen2(vsub(r->o, sp->c)) < sp->r * sp->r) rec->normal = vneg(rec->normal);
        rec->mat = sp->mat;
        /* get_sphere_uv(rec.p - center) (hitable.h:15-21): the offset is not
         * normalised, so asin sees |y| > 1 (NaN) on spheres of radius > 1 */
        const v3 q = vsub(rec->p, sp->c);
        const double phi = atan2(q.e[2], q.e[0]), theta = asin(q.e[1]);
        rec->tu = 1 - (phi + M_PI) / (2 * M_PI);
        rec->tv = (theta + M_PI / 2) / M_PI;
        return 1;
    }
    return 0;
}

static inline aabb prim_box(const ora_scene *s, int32_t ref)
{
    if (ref & REF_SPHERE) {                                                  /* sphere.h:58-62 */
        const sphere *sp = &s->sph[ref & ~REF_SPHERE];
        v3 rr = mk(sp->r, sp->r, sp->r);
        return aabb_mk(vsub(sp->c, rr), vadd(sp->c, rr));
    }
    const tri *t = &s->tris[ref];                                            /* triangle.h:120-137 */
    v3 mn = mk(fmin(fmin(t->v0.e[0], t->v1.e[0]), t->v2.e[0]),
               fmin(fmin(t->v0.e[1], t->v1.e[1]), t->v2.e[1]),
               fmin(fmin(t->v0.e[2], t->v1.e[2]), t->v2.e[2]));
    v3 mx = mk(fmax(fmax(t->v0.e[0], t->v1.e[0]), t->v2.e[0]),
               fmax(fmax(t->v0.e[1], t->v1.e[1]), t->v2.e[1]),
               fmax(fmax(t->v0.e[2], t->v1.e[2]), t->v2.e[2]));
    return aabb_mk(mn, mx);
}

static inline int prim_hit(const ora_scene *s, int32_t ref, const ray *r, double tmin, double tmax,
                           hit_record *rec, ora_counters *cnt)
{
    int ok;
    if (ref & REF_SPHERE) {
        cnt->sphere_tests++;
        ok = sphere_hit(&s->sph[ref & ~REF_SPHERE], r, tmin, tmax, rec);
    } else {
        cnt->tri_tests++;
        ok = tri_hit(&s->tris[ref], r, tmin, tmax, rec, NULL, NULL);
    }
    if (ok) rec->obj = ref;
    return ok;
}

/* parallel_bvh_node::hit (parallel_bvh.h:39-64) */
static int bvh_hit(const ora_scene *s, int32_t node, const ray *r, double t_min, double t_max,
                   hit_record *rec, ora_counters *cnt)
{
    if (node < 0) return prim_hit(s, ~node, r, t_min, t_max, rec, cnt);
    const bnode *nd = &s->nodes[node];
    cnt->node_visits++;
    if (aabb_hit(&nd->box, r, t_min, t_max)) {
        cnt->box_passes++;
        double ray_min_t = t_min;
        if (ray_min_t == EPSILON)
            ray_min_t *= std_max(std_max(std_max(fabs(r->o.e[0]), fabs(r->o.e[1])), fabs(r->o.e[2])), EPSILON);
        if (ray_min_t > t_min) t_min = ray_min_t;
        if (bvh_hit(s, nd->left, r, t_min, t_max, rec, cnt)) {
            bvh_hit(s, nd->right, r, t_min, rec->t, rec, cnt);
            return 1;
        }
        return bvh_hit(s, nd->right, r, t_min, t_max, rec, cnt);
    }
    return 0;
}
/* hitable_list::hit (hitable_list.cpp:4-21) */
static int list_hit(const ora_scene *s, const ray *r, double t_min, double t_max, hit_record *rec, ora_counters *cnt)
{
    hit_record temp;
    int hit_anything = 0;
    double closest = t_max;
    for (int i = 0; i < s->nlist; ++i) {
        if (prim_hit(s, s->list[i], r, t_min, closest, &temp, cnt)) {
            hit_anything = 1;
            closest = temp.t;
            *rec = temp;
        }
    }
    return hit_anything;
}
static inline int world_hit(const ora_scene *s, const ray *r, double t_min, double t_max, hit_record *rec,
                            ora_counters *cnt)
{
    if (s->world_kind == WORLD_LIST) return list_hit(s, r, t_min, t_max, rec, cnt);
    return bvh_hit(s, s->root, r, t_min, t_max, rec, cnt);
}

/* pdf_direct_sampling: triangle.h:139-144; sphere.h:64-78 */
static double prim_pdf_direct(const ora_scene *s, int32_t ref, const hit_record *lrec, v3 to_light)
{
    if (!(ref & REF_SPHERE)) return s->tris[ref].inv_area;
    const sphere *sp = &s->sph[ref & ~REF_SPHERE];
    ray rr; rr.o = lrec->p; rr.d = to_light;
    const v3 o = ray_at(&rr, -lrec->t);
    const v3 direction = vsub(sp->c, o);
    const double distance_squared = vlen2(direction);
    const double radius_squared = sp->r * sp->r;
    if (distance_squared <= radius_squared) return 1 / (4 * M_PI * sp->r * sp->r);
    const double cos_theta_max = sqrt(1 - radius_squared / vlen2(direction));
    const double solid_angle = 2 * M_PI * (1 - cos_theta_max);
    return (1 / solid_angle) * fabs(dot(to_light, lrec->normal)) / vlen2(direction);
}
/* sample_direct: triangle.h:145-175; sphere.h:80-107.  Fills lrec (t, p, normal, mat, obj). */
static v3 prim_sample_direct(const ora_scene *s, int32_t ref, hit_record *rec, v3 o, double u0, double u1)
{
    if (!(ref & REF_SPHERE)) {
        const tri *t = &s->tris[ref];
        double su0 = sqrt(u0);
        double b0 = 1 - su0;
        double b1 = u1 * su0;
        v3 random_point = vadd(vadd(smul((1 - b0 - b1), t->v0), smul(b0, t->v1)), smul(b1, t->v2));
        rec->t = 1.0;
        rec->p = random_point;
        if (t->geo) rec->normal = unit(cross(t->e1, t->e2));
        else rec->normal = unit(vadd(vadd(smul((1 - b0 - b1), t->n0), smul(b0, t->n1)), smul(b1, t->n2)));
        rec->mat = t->mat;
        rec->obj = ref;
        return vsub(random_point, o);
    }
    const sphere *sp = &s->sph[ref & ~REF_SPHERE];
    const v3 direction = vsub(sp->c, o);
    const double distance_squared = vlen2(direction);
    onb uvw = onb_from_w(direction);
    if (distance_squared <= sp->r * sp->r) {
        v3 p = vadd(sp->c, smul(sp->r, uniform_sample_sphere(u0, u1)));
        rec->p = p;
        rec->mat = sp->mat;
        rec->normal = unit(vsub(sp->c, p));
        rec->obj = ref;
        return vsub(p, o);
    }
    v3 p = onb_from_local(&uvw, random_to_sphere(sp->r, distance_squared, u0, u1));
    rec->mat = sp->mat;
    rec->normal = unit(p);
    rec->obj = ref;
    return p;
}
/* diffuse_light::emitted (material.h:184-190); other materials emit 0 */
static inline v3 mat_emitted(const ora_scene *s, int mat, v3 d, v3 normal)
{
    const material *m = &s->mats[mat];
    if (m->type == MAT_LIGHT && dot(normal, d) < 0) return m->emit;
    return mk(0, 0, 0);
}
/* hitable_list::pick_sample (hitable_list.cpp:64-70) */
static inline int pick_sample(double sample, int list_size)
{
    int index = (int)(sample * list_size);
    if (index == list_size) index -= 1;
    return index;
}

typedef struct { const ora_scene *s; rng_key key; ora_counters *cnt; int max_depth; } li_ctx;   /* max_depth: 33 in path.cpp:36 */

/* path::Li (path.cpp:4-116), recursive like the reference so the
 * association order of every product/sum matches.  Materials: lambertian,
 * diffuse_light, modified_phong and dielectric (the ones mesh_loader.cpp:59-112
 * creates); the specular branch is path.cpp:78-95. */
static v3 Li(li_ctx *c, const ray *r, int depth, const hit_record *prev, double prev_bsdf_pdf)
{
    const ora_scene *s = c->s;
    hit_record hrec;
    if (depth == 0) c->cnt->camera_rays++; else c->cnt->extension_rays++;
    if (world_hit(s, r, EPSILON, FLT_MAX, &hrec, c->cnt)) {
        v3 Le = mat_emitted(s, hrec.mat, r->d, hrec.normal);
        if ((Le.e[0] != 0.0) || (Le.e[1] != 0.0) || (Le.e[2] != 0.0)) {
            if (depth == 0 || mat_no_mis(s->mats[prev->mat].type))
                return Le;
            const double cos_wo = dot(hrec.normal, vneg(unit(r->d)));
            double distance_squared = vlen2(vsub(hrec.p, prev->p));
            if (distance_squared <= EPSILON) distance_squared = EPSILON;
            double surface_bsdf_pdf = prev_bsdf_pdf;
            const double light_pdf = prim_pdf_direct(s, hrec.obj, &hrec, r->d) * distance_squared / fabs(cos_wo);
            const double weight = miWeight(surface_bsdf_pdf, light_pdf);
            return smul(weight, Le);
        }
        material mtex;
        const material *m = mat_at(s, &hrec, &mtex);
        /* lambertian / modified_phong / dielectric::scatter succeed; diffuse_light's fails (material.h) */
        if (depth <= c->max_depth && mat_scatters(m->type)) {
            const uint32_t base = DIM_BOUNCE(depth);
            const int specular = m->type != MAT_LAMBERT;
            const v3 wi = vneg(unit(r->d));                   /* hrec.wi (triangle.h:108, sphere.h:47) */
            /* scatter's get3d sample: the specular direction (material.h:83-88, 117-119, 139-145, 262-268) */
            v3 spec_dir = mk(0, 0, 0);
            double sampled_pdf = -1.0;
            if (specular)
                spec_dir = spec_generate(m, hrec.normal, wi, r->d, rng_u(c->key, base + 0), rng_u(c->key, base + 1),
                                         &sampled_pdf);
            const int index = pick_sample(rng_u(c->key, base + 3), s->nlights);
            if (index >= 0 && m->type != MAT_DIELECTRIC) {
                hit_record lrec;
                v3 offset_origin = vadd(hrec.p, smul(EPSILON, hrec.normal));
                v3 to_light = prim_sample_direct(s, s->lights[index], &lrec, offset_origin,
                                                 rng_u(c->key, base + 4), rng_u(c->key, base + 5));
                const double dist_to_light = vlen(to_light);
                ray shadow; shadow.o = offset_origin; shadow.d = to_light;
                c->cnt->shadow_rays++;
                if (!world_hit(s, &shadow, EPSILON, 1 - SHADOW_EPSILON, &lrec, c->cnt)) {
                    to_light = make_unit(to_light);
                    shadow.d = to_light;
                    v3 surface_bsdf = specular ? spec_eval(m, hrec.normal, wi, to_light) : sdiv(m->albedo, M_PI);
                    const double cos_wi = dot(hrec.normal, unit(to_light));
                    const double cos_wo = dot(lrec.normal, vneg(unit(to_light)));
                    if (cos_wo != 0) {
                        double distance_squared = dist_to_light * dist_to_light;
                        if (!specular) surface_bsdf = vscale_inplace(surface_bsdf, cos_wi);
                        const double light_pdf = prim_pdf_direct(s, s->lights[index], &hrec, to_light)
                                                 * distance_squared / fabs(cos_wo);
                        const double surface_bsdf_pdf =
                            specular ? spec_value(m, hrec.normal, wi, to_light) : cosine_pdf_value(hrec.normal, to_light);
                        const double weight = miWeight(light_pdf, surface_bsdf_pdf);
                        v3 em = mat_emitted(s, lrec.mat, shadow.d, lrec.normal);
                        Le = vadd(Le, sdiv(smul(weight, vmul(em, surface_bsdf)), light_pdf));
                    }
                }
            }
            if (specular) {                                   /* path.cpp:78-95 */
                double surface_bsdf_pdf = spec_value(m, hrec.normal, wi, spec_dir);
                if (sampled_pdf > 0.0) surface_bsdf_pdf = sampled_pdf;
                const v3 surface_bsdf = spec_eval(m, hrec.normal, wi, spec_dir);
                if (surface_bsdf_pdf == 0) return mk(0, 0, 0);
                const int outside = dot(hrec.normal, spec_dir) > 0;
                ray sr;
                sr.o = outside ? vadd(hrec.p, smul(EPSILON, hrec.normal)) : vsub(hrec.p, smul(EPSILON, hrec.normal));
                sr.d = spec_dir;
                v3 li = Li(c, &sr, depth + 1, &hrec, surface_bsdf_pdf);
                return vadd(Le, sdiv(vmul(surface_bsdf, li), surface_bsdf_pdf));
            }
            /* diffuse bounce (path.cpp:96-110) */
            onb uvw = onb_from_w(hrec.normal);
            ray wo;
            wo.o = vadd(hrec.p, smul(EPSILON, hrec.normal));
            wo.d = onb_from_local(&uvw, hemisphere_to_cosine_direction(rng_u(c->key, base + 6),
                                                                        rng_u(c->key, base + 7)));
            const double surface_bsdf_pdf = cosine_pdf_value(hrec.normal, wo.d);
            const v3 surface_bsdf = sdiv(m->albedo, M_PI);
            if (surface_bsdf_pdf == 0) return mk(0, 0, 0);
            const double cos_wo = fabs(dot(hrec.normal, unit(wo.d)));
            v3 li = Li(c, &wo, depth + 1, &hrec, surface_bsdf_pdf);
            return vadd(Le, sdiv(smul(cos_wo, vmul(surface_bsdf, li)), surface_bsdf_pdf));
        }
        return Le;
    }
    /* environment_map::eval with a constant texture (material.h:219-232) */
    return s->env;
}

/* scene->world->bounding_box (ao.cpp:19-21): the root node's box
 * (parallel_bvh.h:33-37), a lone primitive's box, or -- hitable_list
 * (hitable_list.cpp:23-31) returns before assigning when its first element
 * reports a box -- the default aabb, whose Vector3 members are quiet NaNs
 * (geometry.h:345-348). */
static double world_box_size_y(const ora_scene *s)
{
    if (s->world_kind == WORLD_LIST) return NAN;
    const aabb b = s->root >= 0 ? s->nodes[s->root].box : prim_box(s, ~s->root);
    return b.size.e[1];
}

/* ao::Li (ao.cpp:4-27).  The camera hit's material scatters (lambertian,
 * modified_phong, dielectric) -> one visibility ray from hrec.p (no offset)
 * along the scattering pdf's generate(get2d()) up to t_max = half the world
 * box height; occluded -> 0, otherwise (and for misses / lights) the
 * environment.  RNG: the get2d is dims DIM_BOUNCE(0) + 6, 7 (the scatter's
 * get3d has no effect on the result). */
static v3 ao_Li(li_ctx *c, const ray *r)
{
    const ora_scene *s = c->s;
    hit_record hrec;
    c->cnt->camera_rays++;
    if (world_hit(s, r, EPSILON, FLT_MAX, &hrec, c->cnt)) {
        const material *m = &s->mats[hrec.mat];
        if (mat_scatters(m->type)) {                            /* (metal: rejected up front) */
            const uint32_t base = DIM_BOUNCE(0);
            const double u0 = rng_u(c->key, base + 6), u1 = rng_u(c->key, base + 7);
            const v3 wi = vneg(unit(r->d));
            v3 dir;
            if (m->type == MAT_LAMBERT) {                       /* cosine_pdf::generate (pdf.h:91-94) */
                onb uvw = onb_from_w(hrec.normal);
                dir = onb_from_local(&uvw, hemisphere_to_cosine_direction(u0, u1));
            } else if (m->type == MAT_PHONG) {                  /* cosine_power_pdf::generate (pdf.h:115-132) */
                dir = cosine_power_generate(hrec.normal, wi, m->shininess, u0, u1);
            } else if (m->type == MAT_DIELECTRIC) {             /* dielectric_pdf::generate (pdf.h:164-178) */
                dir = dielectric_generate(hrec.normal, wi, m->ior, u0);
            } else {                                            /* roughconductor_pdf::generate (pdf.h:465-482) */
                double unused;
                dir = rough_generate(hrec.normal, wi, m->alpha, m->dist, u0, u1, &unused);
            }
            ray shadow; shadow.o = hrec.p; shadow.d = dir;
            const double t_max = world_box_size_y(s) * 0.50f;
            c->cnt->shadow_rays++;
            if (world_hit(s, &shadow, EPSILON, t_max, &hrec, c->cnt)) return mk(0.0, 0.0, 0.0);
        }
    }
    return s->env;
}

/* normals_renderer::Li (debug_renderer.h:8-17): the hit's shading normal, else the environment */
static v3 normals_Li(li_ctx *c, const ray *r)
{
    hit_record hrec;
    c->cnt->camera_rays++;
    if (world_hit(c->s, r, EPSILON, FLT_MAX, &hrec, c->cnt)) return hrec.normal;
    return c->s->env;
}

/* one pixel, path.cpp:120-143 (loop over s, add_sample divides by ns: *= 1/ns);
 * ao.h:15-38 and debug_renderer.h:19-45 are the same loop around their Li */
static void render_pixel(const ora_scene *s, int kind, int nx, int ny, int spp, uint32_t seed, int max_depth, int x,
                         int y, double *out, ora_counters *cnt)
{
    v3 col = mk(0.0, 0.0, 0.0);
    const uint32_t pixel = (uint32_t)y * (uint32_t)nx + (uint32_t)x;
    for (int smp = 0; smp < spp; ++smp) {
        li_ctx c; c.s = s; c.cnt = cnt; c.key = rng_make(seed, pixel, (uint32_t)smp); c.max_depth = max_depth;
        double u = (double)(x + rng_u(c.key, 0)) / (double)nx;
        double v = (double)(y + rng_u(c.key, 1)) / (double)ny;
        ray r = camera_get_ray(&s->cam, u, v, rng_u(c.key, 2), rng_u(c.key, 3));
        hit_record h; memset(&h, 0, sizeof(h)); h.mat = 0;
        v3 sample = kind == ORA_INTEGRATOR_AO        ? ao_Li(&c, &r)
                  : kind == ORA_INTEGRATOR_NORMALS ? normals_Li(&c, &r)
                                                   : Li(&c, &r, 0, &h, 0.0);
        col = vadd(col, sample);
        cnt->samples++;
    }
    col = vdiv_inplace(col, (double)spp);
    vstore(out, col);
}

typedef struct {
    const ora_scene *s; int kind, nx, ny, spp, max_depth; uint32_t seed;
    const int32_t *pixels; int npix; int tid, nth;
    double *out; ora_counters cnt;
} job;
static void *render_worker(void *arg)
{
    job *j = (job *)arg;
    memset(&j->cnt, 0, sizeof(j->cnt));
    for (int i = j->tid; i < j->npix; i += j->nth) {
        int p = j->pixels[i];
        render_pixel(j->s, j->kind, j->nx, j->ny, j->spp, j->seed, j->max_depth, p % j->nx, p / j->nx,
                     &j->out[3 * (size_t)i], &j->cnt);
    }
    return NULL;
}
int ora_render(const ora_scene *s, int nx, int ny, int spp, uint32_t seed, const int32_t *pixels, int npix,
               int nthreads, double *out_rgb, ora_counters *cnt)
{
    return ora_render_integrator(s, ORA_INTEGRATOR_PATH, nx, ny, spp, seed, pixels, npix, nthreads, out_rgb, cnt);
}
int ora_render_integrator(const ora_scene *s, int kind, int nx, int ny, int spp, uint32_t seed,
                          const int32_t *pixels, int npix, int nthreads, double *out_rgb, ora_counters *cnt)
{
    return ora_render_depth(s, kind, nx, ny, spp, seed, 33, pixels, npix, nthreads, out_rgb, cnt);
}
/* the same with path::Li's depth cap as a parameter (33 in path.cpp:36; the PSS-MLT
 * comparison uses pssmlt's MaxPathLength 10, pssmlt.h) */
int ora_render_depth(const ora_scene *s, int kind, int nx, int ny, int spp, uint32_t seed, int max_depth,
                     const int32_t *pixels, int npix, int nthreads, double *out_rgb, ora_counters *cnt)
{
    if (!s || nx <= 0 || ny <= 0 || spp <= 0 || npix < 0) return -1;
    if (kind != ORA_INTEGRATOR_PATH && kind != ORA_INTEGRATOR_AO && kind != ORA_INTEGRATOR_NORMALS) return -3;
    /* ao::Li calls srec.pdf_ptr->generate, which metal's constant_pdf throws on (pdf.h:195-198) */
    if (kind == ORA_INTEGRATOR_AO)
        for (int i = 0; i < s->nmats; ++i) if (s->mats[i].type == MAT_METAL) return -4;
    for (int i = 0; i < npix; ++i)
        if (pixels[i] < 0 || pixels[i] >= nx * ny) return -2;
    if (nthreads < 1) nthreads = 1;
    job *jobs = (job *)calloc((size_t)nthreads, sizeof(job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t].s = s; jobs[t].kind = kind; jobs[t].nx = nx; jobs[t].ny = ny; jobs[t].spp = spp; jobs[t].seed = seed;
        jobs[t].max_depth = max_depth;
        jobs[t].pixels = pixels; jobs[t].npix = npix; jobs[t].tid = t; jobs[t].nth = nthreads; jobs[t].out = out_rgb;
        if (nthreads > 1) pthread_create(&th[t], NULL, render_worker, &jobs[t]);
    }
    if (nthreads == 1) render_worker(&jobs[0]);
    ora_counters tot; memset(&tot, 0, sizeof(tot));
    for (int t = 0; t < nthreads; ++t) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        tot.node_visits += jobs[t].cnt.node_visits; tot.box_passes += jobs[t].cnt.box_passes;
        tot.tri_tests += jobs[t].cnt.tri_tests; tot.sphere_tests += jobs[t].cnt.sphere_tests;
        tot.camera_rays += jobs[t].cnt.camera_rays; tot.extension_rays += jobs[t].cnt.extension_rays;
        tot.shadow_rays += jobs[t].cnt.shadow_rays; tot.samples += jobs[t].cnt.samples;
    }
    if (cnt) *cnt = tot;
    free(jobs); free(th);
    return 0;
}

int ora_world_hit(const ora_scene *s, const double *o, const double *d, double tmin, double tmax,
                  double *t_out, int32_t *prim_out, ora_counters *cnt)
{
    ora_counters local; memset(&local, 0, sizeof(local));
    ray r; r.o = vload(o); r.d = vload(d);
    hit_record h;
    int ok = world_hit(s, &r, tmin, tmax, &h, cnt ? cnt : &local);
    if (ok) { *t_out = h.t; *prim_out = h.obj; } else { *t_out = 0; *prim_out = -1; }
    return ok;
}


/* ------------------------------------------------------------------------ */
/* PSS-MLT (pssmlt.cpp:6-365, pssmlt.h:9-18), Kelemen et al.; chains and the */
/* bootstrap draw from the counter RNG (DESIGN.md "PSS-MLT streams").        */
/* ------------------------------------------------------------------------ */
#define MLT_MAX_PATH 10                       /* MaxPathLength */
#define MLT_DIMS (4 + (MLT_MAX_PATH + 1) * 8) /* prnds a path can read: 92 */
static const double MLT_LARGE_STEP_PROB = (double)0.3f;

typedef struct { double x, y; v3 c; double sc; } mlt_contrib;   /* PathContribution */

typedef struct { const double *prnds; int off; int depth; hit_record prev; double prev_pdf; ora_counters *cnt; } mlt_state;

/* pssmlt::Li (pssmlt.cpp:147-277) */
static v3 mlt_Li(const ora_scene *s, const ray *r, mlt_state *st)
{
    hit_record hrec;
    if (st->depth == 0) st->cnt->camera_rays++; else if (st->depth <= MLT_MAX_PATH) st->cnt->extension_rays++;
    if (st->depth <= MLT_MAX_PATH && world_hit(s, r, EPSILON, FLT_MAX, &hrec, st->cnt)) {
        v3 Le = mat_emitted(s, hrec.mat, r->d, hrec.normal);
        const double rnd_s0 = st->prnds[st->off + 0], rnd_s1 = st->prnds[st->off + 1];   /* scatter rnd */
        st->off += 3;
        if ((Le.e[0] != 0.0) || (Le.e[1] != 0.0) || (Le.e[2] != 0.0)) {
            if (st->depth == 0 || mat_no_mis(s->mats[st->prev.mat].type))
                return Le;
            const double cos_wo = dot(hrec.normal, vneg(unit(r->d)));
            double distance_squared = hrec.t * hrec.t;
            if (distance_squared <= EPSILON) distance_squared = EPSILON;
            const double light_pdf = prim_pdf_direct(s, hrec.obj, &hrec, r->d) * distance_squared / fabs(cos_wo);
            const double weight = miWeight(st->prev_pdf, light_pdf);
            return smul(weight, Le);
        }
        material mtex;
        const material *m = mat_at(s, &hrec, &mtex);
        if (mat_scatters(m->type)) {
            const int specular = m->type != MAT_LAMBERT;
            const v3 wi = vneg(unit(r->d));
            v3 spec_dir = mk(0, 0, 0);
            double sampled_pdf = -1.0;
            if (specular) spec_dir = spec_generate(m, hrec.normal, wi, r->d, rnd_s0, rnd_s1, &sampled_pdf);
            const double rnd0 = st->prnds[st->off + 0], rnd1 = st->prnds[st->off + 1], rnd2 = st->prnds[st->off + 2];
            st->off += 3;
            const int index = pick_sample(rnd0, s->nlights);
            if (index >= 0 && m->type != MAT_DIELECTRIC) {
                hit_record lrec;
                v3 offset_origin = vadd(hrec.p, smul(EPSILON, hrec.normal));
                v3 to_light = prim_sample_direct(s, s->lights[index], &lrec, offset_origin, rnd1, rnd2);
                const double dist_to_light = vlen(to_light);
                ray shadow; shadow.o = offset_origin; shadow.d = to_light;
                st->cnt->shadow_rays++;
                if (!world_hit(s, &shadow, EPSILON, 1 - SHADOW_EPSILON, &lrec, st->cnt)) {
                    to_light = make_unit(to_light);
                    shadow.d = to_light;
                    v3 surface_bsdf = specular ? spec_eval(m, hrec.normal, wi, to_light) : sdiv(m->albedo, M_PI);
                    const double cos_wi = dot(hrec.normal, unit(to_light));
                    const double cos_wo = dot(lrec.normal, vneg(unit(to_light)));
                    if (cos_wo != 0) {
                        double distance_squared = dist_to_light * dist_to_light;
                        if (!specular) surface_bsdf = vscale_inplace(surface_bsdf, cos_wi);
                        const double light_pdf = prim_pdf_direct(s, s->lights[index], &hrec, to_light)
                                                 * distance_squared / fabs(cos_wo);
                        const double surface_bsdf_pdf =
                            specular ? spec_value(m, hrec.normal, wi, to_light) : cosine_pdf_value(hrec.normal, to_light);
                        const double weight = miWeight(light_pdf, surface_bsdf_pdf);
                        v3 em = mat_emitted(s, lrec.mat, shadow.d, lrec.normal);
                        Le = vadd(Le, sdiv(smul(weight, vmul(em, surface_bsdf)), light_pdf));
                    }
                }
            }
            if (specular) {                                   /* pssmlt.cpp:232-249 */
                double surface_bsdf_pdf = spec_value(m, hrec.normal, wi, spec_dir);
                if (sampled_pdf > 0.0) surface_bsdf_pdf = sampled_pdf;
                const v3 surface_bsdf = spec_eval(m, hrec.normal, wi, spec_dir);
                if (surface_bsdf_pdf == 0) return mk(0, 0, 0);
                const int outside = dot(hrec.normal, spec_dir) > 0;
                ray sr;
                sr.o = outside ? vadd(hrec.p, smul(EPSILON, hrec.normal)) : vsub(hrec.p, smul(EPSILON, hrec.normal));
                sr.d = spec_dir;
                st->depth += 1;
                st->prev_pdf = surface_bsdf_pdf;
                st->prev = hrec;
                v3 li = mlt_Li(s, &sr, st);
                return vadd(Le, sdiv(vmul(surface_bsdf, li), surface_bsdf_pdf));
            }
            /* diffuse bounce: hrec.p is moved off the surface first (pssmlt.cpp:253) */
            hrec.p = vadd(hrec.p, smul(EPSILON, hrec.normal));
            const double r0 = st->prnds[st->off + 0], r1 = st->prnds[st->off + 1];
            st->off += 2;
            onb uvw = onb_from_w(hrec.normal);
            ray wo; wo.o = hrec.p;
            wo.d = onb_from_local(&uvw, hemisphere_to_cosine_direction(r0, r1));
            const double surface_bsdf_pdf = cosine_pdf_value(hrec.normal, wo.d);
            const v3 surface_bsdf = sdiv(m->albedo, M_PI);
            if (surface_bsdf_pdf == 0) return mk(0, 0, 0);
            const double cos_wo = fabs(dot(hrec.normal, unit(wo.d)));
            st->depth += 1;
            st->prev_pdf = surface_bsdf_pdf;
            st->prev = hrec;
            v3 li = mlt_Li(s, &wo, st);
            return vadd(Le, sdiv(smul(cos_wo, vmul(surface_bsdf, li)), surface_bsdf_pdf));
        }
        return Le;
    }
    return s->env;
}

/* GenerateEyePath (pssmlt.cpp:105-144) with PixelWidth/Height and
 * camera::dist = PixelHeight/(2 half_height) generalised to the film size. */
static mlt_contrib mlt_eye_path(const ora_scene *s, const double *prnds, int nx, int ny, ora_counters *cnt)
{
    const camera *cam = &s->cam;
    ray r = camera_get_ray(cam, prnds[0], prnds[1], prnds[2], prnds[3]);
    const v3 dir = unit(r.d);
    mlt_state st; memset(&st, 0, sizeof st);
    st.prnds = prnds; st.off = 4; st.depth = 0; st.prev_pdf = 0.0; st.cnt = cnt;
    mlt_contrib pc;
    pc.c = mlt_Li(s, &r, &st);
    pc.sc = std_max(std_max(pc.c.e[0], pc.c.e[1]), pc.c.e[2]);
    const double dist = (double)ny / (2 * cam->half_height);
    const v3 center = vadd(cam->origin, smul(dist, cam->w));
    const v3 pos = vsub(vadd(cam->origin, smul(dist / dot(dir, cam->w), dir)), center);
    pc.x = -dot(cam->u, pos) + (nx * 0.5);
    pc.y = -dot(cam->v, pos) + (ny * 0.5);
    return pc;
}

/* perturb (pssmlt.cpp:6-17) */
static inline double mlt_perturb(double value, double s1, double s2, double r)
{
    double result;
    if (r < 0.5) {
        r = r * 2.0;
        result = value + s2 * exp(-log(s2 / s1) * r); if (result > 1.0) result -= 1.0;
    } else {
        r = (r - 0.5) * 2.0;
        result = value - s2 * exp(-log(s2 / s1) * r); if (result < 0.0) result += 1.0;
    }
    return result;
}

typedef struct {
    const ora_scene *s; int nx, ny; uint32_t seed; double b, scale;
    int j0, j1, shard_index, shard_count; long long steps;    /* chains c = shard_index + j * shard_count */
    double *film; ora_counters cnt;
    uint32_t *fp; double *u;                                 /* per local chain: fingerprint, final state */
} mlt_job;

static void mlt_splat(double *film, int nx, int ny, const mlt_contrib *pc, double w, double scale)
{
    if (pc->sc == 0) return;                                   /* AccumulatePathContribution */
    const int ix = (int)pc->x, iy = (int)pc->y;
    if (ix < 0 || ix >= nx || iy < 0 || iy >= ny) return;
    const v3 c = smul(w, pc->c);
    for (int k = 0; k < 3; ++k) film[((size_t)ix + (size_t)iy * nx) * 3 + k] += scale * c.e[k];
}

static void *mlt_worker(void *arg)
{
    mlt_job *j = (mlt_job *)arg;
    double cur[MLT_DIMS], prop[MLT_DIMS];
    const double s1p = 2.0 / (double)(j->nx + j->ny), s2p = (double)0.1f;
    memset(&j->cnt, 0, sizeof j->cnt);
    for (int jl = j->j0; jl < j->j1; ++jl) {
        const int c = j->shard_index + jl * j->shard_count;
        uint32_t n_acc = 0, acc_sum = 0;                     /* chain fingerprint (see ora_mlt_render_shard) */
        rng_key k0 = rng_make(j->seed ^ 0x3C6EF372U, (uint32_t)c, 0u);
        for (int d = 0; d < MLT_DIMS; ++d) cur[d] = rng_u(k0, (uint32_t)(2 + d));
        mlt_contrib C = mlt_eye_path(j->s, cur, j->nx, j->ny, &j->cnt);
        for (long long t = 0; t < j->steps; ++t) {
            rng_key k = rng_make(j->seed ^ 0x3C6EF372U, (uint32_t)c, (uint32_t)(t + 1));
            double large;
            if (rng_u(k, 0) < MLT_LARGE_STEP_PROB) {
                for (int d = 0; d < MLT_DIMS; ++d) prop[d] = rng_u(k, (uint32_t)(2 + d));
                large = 1.0;
            } else {
                prop[0] = mlt_perturb(cur[0], s1p, s2p, rng_u(k, 2));
                prop[1] = mlt_perturb(cur[1], s1p, s2p, rng_u(k, 3));
                for (int d = 2; d < MLT_DIMS; ++d) prop[d] = mlt_perturb(cur[d], 1.0 / 1024.0, 1.0 / 64.0, rng_u(k, (uint32_t)(2 + d)));
                large = 0.0;
            }
            mlt_contrib P = mlt_eye_path(j->s, prop, j->nx, j->ny, &j->cnt);
            j->cnt.samples++;
            double a = 1.0;
            if (C.sc > 0.0) { a = P.sc / C.sc; a = a < 1.0 ? a : 1.0; a = a > 0.0 ? a : 0.0; }
            if (P.sc > 0.0) mlt_splat(j->film, j->nx, j->ny, &P, (a + large) / (P.sc / j->b + MLT_LARGE_STEP_PROB), j->scale);
            if (C.sc > 0.0) mlt_splat(j->film, j->nx, j->ny, &C, (1.0 - a) / (C.sc / j->b + MLT_LARGE_STEP_PROB), j->scale);
            if (rng_u(k, 1) <= a) {
                memcpy(cur, prop, sizeof cur); C = P;
                n_acc += 1u; acc_sum += (uint32_t)(t + 1);
            }
        }
        if (j->fp) { j->fp[2 * (size_t)jl] = n_acc; j->fp[2 * (size_t)jl + 1] = acc_sum; }
        if (j->u) memcpy(j->u + (size_t)jl * MLT_DIMS, cur, sizeof cur);
    }
    return NULL;
}

/* bootstrap normaliser b (pssmlt.cpp:303-312): mean scalar contribution of
 * n_init independent paths */
double ora_mlt_bootstrap(const ora_scene *s, int nx, int ny, uint32_t seed, int n_init)
{
    double prnds[MLT_DIMS];
    ora_counters cnt; memset(&cnt, 0, sizeof cnt);
    double b = 0.0;
    for (int i = 0; i < n_init; ++i) {
        rng_key k = rng_make(seed ^ 0xB5297A4DU, (uint32_t)i, 0u);
        for (int d = 0; d < MLT_DIMS; ++d) prnds[d] = rng_u(k, (uint32_t)d);
        b += mlt_eye_path(s, prnds, nx, ny, &cnt).sc;
    }
    return b / n_init;
}

/* pssmlt::Render (pssmlt.cpp:301-365) for the chains of one shard: of
 * n_chains chains of `steps` mutations each, the n_local chains
 * c = shard_index + j * shard_count (j = 0, 1, ...), the GPU's shard rule
 * (frt_render.hip MltWork).  film (nx*ny*3, zeroed by the caller) receives
 * their splats scaled by nx*ny/(n_chains*steps) as AccumulatePathContribution
 * does with ns, so the shard films of all shards sum to the full render.
 * Per local chain j (optional): fp[2j] = accepted proposals, fp[2j+1] = the
 * sum of the accepted steps' 1-based indices mod 2^32 -- the trajectory's
 * fingerprint, which the GPU keeps too -- and u[92 j ..] = its final state. */
int ora_mlt_render_shard(const ora_scene *s, int nx, int ny, uint32_t seed, int n_init, int n_chains, long long steps,
                         int shard_index, int shard_count, int nthreads, double *film, double *b_out,
                         ora_counters *cnt, uint32_t *fp, double *u)
{
    if (!s || nx <= 0 || ny <= 0 || n_chains <= 0 || steps <= 0 || n_init <= 0) return -1;
    if (shard_count < 1 || shard_index < 0 || shard_index >= shard_count) return -1;
    const int n_local = shard_index < n_chains ? (n_chains - 1 - shard_index) / shard_count + 1 : 0;
    const double b = ora_mlt_bootstrap(s, nx, ny, seed, n_init);
    if (b_out) *b_out = b;
    if (cnt) memset(cnt, 0, sizeof *cnt);
    if (n_local == 0) return 0;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > n_local) nthreads = n_local;
    mlt_job *jobs = (mlt_job *)calloc((size_t)nthreads, sizeof(mlt_job));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    double **films = (double **)calloc((size_t)nthreads, sizeof(double *));
    const double scale = (double)nx * ny / ((double)n_chains * (double)steps);
    for (int t = 0; t < nthreads; ++t) {
        films[t] = (double *)calloc((size_t)nx * ny * 3, sizeof(double));
        jobs[t].s = s; jobs[t].nx = nx; jobs[t].ny = ny; jobs[t].seed = seed; jobs[t].b = b; jobs[t].scale = scale;
        jobs[t].j0 = (int)((long long)n_local * t / nthreads); jobs[t].j1 = (int)((long long)n_local * (t + 1) / nthreads);
        jobs[t].shard_index = shard_index; jobs[t].shard_count = shard_count;
        jobs[t].steps = steps; jobs[t].film = films[t]; jobs[t].fp = fp; jobs[t].u = u;
        pthread_create(&th[t], NULL, mlt_worker, &jobs[t]);
    }
    ora_counters tot; memset(&tot, 0, sizeof tot);
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        for (size_t i = 0; i < (size_t)nx * ny * 3; ++i) film[i] += films[t][i];
        free(films[t]);
        tot.node_visits += jobs[t].cnt.node_visits; tot.tri_tests += jobs[t].cnt.tri_tests;
        tot.sphere_tests += jobs[t].cnt.sphere_tests; tot.camera_rays += jobs[t].cnt.camera_rays;
        tot.extension_rays += jobs[t].cnt.extension_rays; tot.shadow_rays += jobs[t].cnt.shadow_rays;
        tot.samples += jobs[t].cnt.samples; tot.box_passes += jobs[t].cnt.box_passes;
    }
    if (cnt) *cnt = tot;
    free(jobs); free(th); free(films);
    return 0;
}

/* every chain (shard 0 of 1) */
int ora_mlt_render(const ora_scene *s, int nx, int ny, uint32_t seed, int n_init, int n_chains, long long steps,
                   int nthreads, double *film, double *b_out, ora_counters *cnt)
{
    return ora_mlt_render_shard(s, nx, ny, seed, n_init, n_chains, steps, 0, 1, nthreads, film, b_out, cnt, NULL, NULL);
}

/* one PSS-MLT eye path for given primary samples (92 doubles): out x, y, r, g, b, sc */
void ora_mlt_eye_path(const ora_scene *s, int nx, int ny, const double *prnds, double *out6)
{
    ora_counters cnt; memset(&cnt, 0, sizeof cnt);
    mlt_contrib pc = mlt_eye_path(s, prnds, nx, ny, &cnt);
    out6[0] = pc.x; out6[1] = pc.y; vstore(out6 + 2, pc.c); out6[5] = pc.sc;
}

/* ------------------------------------------------------------------------ */
/* BVH build: parallel_bvh_node ctor (parallel_bvh.h:67-160) with glibc      */
/* qsort and the bvh.h:6-55 comparators.  Subtrees are built depth-first,    */
/* the left child first, exactly like the sequential taskflow schedule.      */
/* ------------------------------------------------------------------------ */
typedef struct { const ora_scene *s; int axis; } cmp_ctx;
static int box_cmp(const void *a, const void *b, void *arg)
{
    const cmp_ctx *c = (const cmp_ctx *)arg;
    aabb bl = prim_box(c->s, *(const int32_t *)a);
    aabb br = prim_box(c->s, *(const int32_t *)b);
    if (bl.min.e[c->axis] - br.min.e[c->axis] < 0.0) return -1;
    return 1;
}
typedef struct { aabb *boxes; double *left_area, *right_area; } bscratch;

static int32_t build_rec(ora_scene *s, int32_t *l, int n, int g_index, bscratch *g, int depth)
{
    if (depth > s->bvh_depth) s->bvh_depth = depth;
    int32_t me = s->nnodes++;
    aabb *boxes = g->boxes + g_index;
    double *left_area = g->left_area + g_index;
    double *right_area = g->right_area + g_index;

    aabb main_box = prim_box(s, l[0]);
    for (int i = 1; i < n; ++i) {
        aabb nb = prim_box(s, l[i]);
        main_box = surrounding_box(nb, main_box);
    }
    cmp_ctx cc; cc.s = s; cc.axis = aabb_longest_axis(&main_box);
    qsort_r(l, (size_t)n, sizeof(int32_t), box_cmp, &cc);
    for (int i = 0; i < n; ++i) boxes[i] = prim_box(s, l[i]);
    left_area[0] = aabb_area(&boxes[0]);
    aabb left_box = boxes[0];
    for (int i = 1; i < n - 1; ++i) { left_box = surrounding_box(left_box, boxes[i]); left_area[i] = aabb_area(&left_box); }
    right_area[n - 1] = aabb_area(&boxes[n - 1]);
    aabb right_box = boxes[n - 1];
    for (int i = n - 2; i > 0; --i) { right_box = surrounding_box(right_box, boxes[i]); right_area[i] = aabb_area(&right_box); }
    double min_SAH = FLT_MAX;
    int min_idx = 0;
    for (int i = 0; i < n - 1; ++i) {
        double SAH = i * left_area[i] + (n - i - 1) * right_area[i + 1];
        if (SAH < min_SAH) { min_idx = i; min_SAH = SAH; }
    }
    s->nodes[me].box = main_box;
    int32_t left, right;
    if (min_idx == 0) left = ~l[0];
    else left = build_rec(s, l, min_idx + 1, g_index, g, depth + 1);
    if (min_idx == n - 2) right = ~l[min_idx + 1];
    else right = build_rec(s, l + min_idx + 1, n - min_idx - 1, g_index + min_idx + 1, g, depth + 1);
    s->nodes[me].left = left;
    s->nodes[me].right = right;
    return me;
}
static int build_bvh(ora_scene *s, int32_t *prims, int n)
{
    s->nodes = (bnode *)calloc((size_t)(n > 1 ? n - 1 : 1), sizeof(bnode));
    s->nnodes = 0; s->bvh_depth = 0;
    if (n <= 0) return -1;
    if (n == 1) { s->root = ~prims[0]; return 0; }   /* the reference reads an uninitialised index here */
    bscratch g;
    g.boxes = (aabb *)malloc(sizeof(aabb) * (size_t)n);
    g.left_area = (double *)malloc(sizeof(double) * (size_t)n);
    g.right_area = (double *)malloc(sizeof(double) * (size_t)n);
    s->root = build_rec(s, prims, n, 0, &g, 1);
    free(g.boxes); free(g.left_area); free(g.right_area);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* OBJ/MTL ingest: Assimp 5.0.1 ObjFileParser + post-processing restated     */
/* (mesh split per object/material, fast_atoreal_move float parsing, quad   */
/* triangulation, GenSmoothNormals for meshes without vn), then             */
/* mesh_loader.cpp:59-112 material mapping.  Assimp is absent: parity at    */
/* this boundary is "unpinned" (SURVEY.md 8(c)).                             */
/* ------------------------------------------------------------------------ */
static const double fast_atof_table[16] = {
    0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001,
    0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001, 0.000000000000001};
static uint64_t strtoul10_64(const char *in, const char **out, unsigned *max_inout)
{
    unsigned cur = 0;
    uint64_t value = 0;
    while (*in >= '0' && *in <= '9') {
        const uint64_t new_value = (value * 10) + (uint64_t)(*in - '0');
        if (new_value < value) break;   /* overflow: Assimp throws; keep value */
        value = new_value;
        ++in; ++cur;
        if (max_inout && *max_inout == cur) {
            while (*in >= '0' && *in <= '9') ++in;
            break;
        }
    }
    if (out) *out = in;
    if (max_inout) *max_inout = cur;
    return value;
}
static const char *fast_atof_float(const char *c, float *outv)
{
    float f = 0;
    int inv = (*c == '-');
    if (inv || *c == '+') ++c;
    if (!((*c >= '0' && *c <= '9') || ((*c == '.' || *c == ',') && c[1] >= '0' && c[1] <= '9'))) {
        *outv = 0; return c;
    }
    if (!(*c == '.' || *c == ',')) f = (float)strtoul10_64(c, &c, NULL);
    if ((*c == '.' || *c == ',') && c[1] >= '0' && c[1] <= '9') {
        ++c;
        unsigned diff = 15;  /* AI_FAST_ATOF_RELAVANT_DECIMALS */
        double pl = (double)strtoul10_64(c, &c, &diff);
        pl *= fast_atof_table[diff];
        f += (float)pl;
    } else if (*c == '.') {
        ++c;
    }
    if (*c == 'e' || *c == 'E') {
        ++c;
        int einv = (*c == '-');
        if (einv || *c == '+') ++c;
        float ex = (float)strtoul10_64(c, &c, NULL);
        if (einv) ex = -ex;
        f *= powf(10.0f, ex);
    }
    if (inv) f = -f;
    *outv = f;
    return c;
}
float ora_kat_atof(const char *s) { float f; fast_atof_float(s, &f); return f; }

typedef struct { char name[128]; float kd[3], ks[3], ke[3]; float d, ni, ns; int has_kd; } mtl;
typedef struct { int mtl; int nfaces; int *faces; int cap; int *tfaces; } omesh;   /* faces: v idx + vn idx; tfaces: vt idx */

typedef struct {
    float *v; int nv, capv;              /* positions */
    float *vn; int nvn, capvn;           /* normals (vn) */
    float *vt; int nvt, capvt;           /* texture coordinates (vt: u, v) */
    mtl *mats; int nmats;
    omesh *meshes; int nmeshes, capm;
    int *fv_n;                            /* per triangle corner: normal index or -1 (parallel to faces) */
} objdata;

static void trim(char *s)
{
    size_t n = strlen(s);
    while (n && (s[n - 1] == '\n' || s[n - 1] == '\r' || s[n - 1] == ' ' || s[n - 1] == '\t')) s[--n] = 0;
}
static int load_mtl(const char *path, objdata *od)
{
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char line[1024];
    mtl *cur = NULL;
    while (fgets(line, sizeof line, f)) {
        char *p = line;
        while (*p == ' ' || *p == '\t') ++p;
        trim(p);
        if (!strncmp(p, "newmtl", 6)) {
            od->mats = (mtl *)realloc(od->mats, sizeof(mtl) * (size_t)(od->nmats + 1));
            cur = &od->mats[od->nmats++];
            memset(cur, 0, sizeof(*cur));
            const char *nm = p + 6; while (*nm == ' ' || *nm == '\t') ++nm;
            snprintf(cur->name, sizeof cur->name, "%s", nm);
            cur->kd[0] = cur->kd[1] = cur->kd[2] = 0.6f;  /* ObjFile::Material defaults */
            cur->d = 1.0f; cur->ni = 1.0f;
            continue;
        }
        if (!cur) continue;
        const char *q;
        float *dst = NULL; int n3 = 0;
        if (p[0] == 'K' && p[1] == 'd' && (p[2] == ' ' || p[2] == '\t')) { dst = cur->kd; n3 = 1; cur->has_kd = 1; }
        else if (p[0] == 'K' && p[1] == 's' && (p[2] == ' ' || p[2] == '\t')) { dst = cur->ks; n3 = 1; }
        else if (p[0] == 'K' && p[1] == 'e' && (p[2] == ' ' || p[2] == '\t')) { dst = cur->ke; n3 = 1; }
        else if (p[0] == 'd' && (p[1] == ' ' || p[1] == '\t')) dst = &cur->d;
        else if (p[0] == 'N' && p[1] == 'i') dst = &cur->ni;
        else if (p[0] == 'N' && p[1] == 's') dst = &cur->ns;
        else if (p[0] == 'T' && p[1] == 'r') { q = p + 2; while (*q == ' ' || *q == '\t') ++q; float tr; fast_atof_float(q, &tr); cur->d = 1.0f - tr; continue; }
        if (!dst) continue;
        q = p + (n3 ? 2 : (p[0] == 'd' ? 1 : 2));
        for (int k = 0; k < (n3 ? 3 : 1); ++k) {
            while (*q == ' ' || *q == '\t') ++q;
            q = fast_atof_float(q, &dst[k]);
        }
    }
    fclose(f);
    return 0;
}
static int find_mtl(const objdata *od, const char *name)
{
    for (int i = 0; i < od->nmats; ++i) if (!strcmp(od->mats[i].name, name)) return i;
    return -1;
}
static omesh *new_mesh(objdata *od, int mtl_idx)
{
    if (od->nmeshes == od->capm) { od->capm = od->capm ? 2 * od->capm : 16; od->meshes = (omesh *)realloc(od->meshes, sizeof(omesh) * (size_t)od->capm); }
    omesh *m = &od->meshes[od->nmeshes++];
    memset(m, 0, sizeof(*m));
    m->mtl = mtl_idx;
    return m;
}
static void mesh_push(omesh *m, int a, int b, int c, int na, int nb, int nc, int ta, int tb, int tc)
{
    if (m->nfaces == m->cap) {
        m->cap = m->cap ? 2 * m->cap : 64;
        m->faces = (int *)realloc(m->faces, sizeof(int) * 6 * (size_t)m->cap);
        m->tfaces = (int *)realloc(m->tfaces, sizeof(int) * 3 * (size_t)m->cap);
    }
    int *t = &m->tfaces[3 * m->nfaces];
    int *f = &m->faces[6 * m->nfaces++];
    f[0] = a; f[1] = b; f[2] = c; f[3] = na; f[4] = nb; f[5] = nc;
    t[0] = ta; t[1] = tb; t[2] = tc;
}
static inline void fsub3(const float *a, const float *b, float *o) { o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2]; }
static inline void fdivs3(float *v, float f)   /* aiVector3t::operator/= */
{
    if (f == 1.0f) return;
    const float invF = 1.0f / f;
    v[0] *= invF; v[1] *= invF; v[2] *= invF;
}
static inline void fnorm3(float *v)   /* aiVector3D::Normalize */
{
    fdivs3(v, sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]));
}
static inline float fdot3(const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

/* TriangulateProcess quad rule: fan from the concave vertex (or 0). */
static int quad_start(const objdata *od, const int *vi)
{
    for (int i = 0; i < 4; ++i) {
        const float *v0 = &od->v[3 * vi[(i + 3) % 4]], *v1 = &od->v[3 * vi[(i + 2) % 4]];
        const float *v2 = &od->v[3 * vi[(i + 1) % 4]], *v = &od->v[3 * vi[i]];
        float left[3], diag[3], right[3];
        fsub3(v0, v, left); fsub3(v1, v, diag); fsub3(v2, v, right);
        fnorm3(left); fnorm3(diag); fnorm3(right);
        const float angle = acosf(fdot3(left, diag)) + acosf(fdot3(right, diag));
        if (angle > (float)M_PI) return i;
    }
    return 0;
}

static int parse_obj(const char *path, objdata *od)
{
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    char line[4096];
    omesh *cur = NULL;
    int cur_mtl = -2;          /* -2: no material selected yet (NoMaterial) */
    int cur_has_obj = 0;
    char group[512] = "";
    while (fgets(line, sizeof line, f)) {
        char *p = line;
        while (*p == ' ' || *p == '\t') ++p;
        trim(p);
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            if (od->nv == od->capv) { od->capv = od->capv ? 2 * od->capv : 1024; od->v = (float *)realloc(od->v, sizeof(float) * 3 * (size_t)od->capv); }
            const char *q = p + 1;
            for (int k = 0; k < 3; ++k) { while (*q == ' ' || *q == '\t') ++q; q = fast_atof_float(q, &od->v[3 * od->nv + k]); }
            od->nv++;
        } else if (p[0] == 'v' && p[1] == 'n') {
            if (od->nvn == od->capvn) { od->capvn = od->capvn ? 2 * od->capvn : 1024; od->vn = (float *)realloc(od->vn, sizeof(float) * 3 * (size_t)od->capvn); }
            const char *q = p + 2;
            for (int k = 0; k < 3; ++k) { while (*q == ' ' || *q == '\t') ++q; q = fast_atof_float(q, &od->vn[3 * od->nvn + k]); }
            od->nvn++;
        } else if (p[0] == 'v' && p[1] == 't') {
            if (od->nvt == od->capvt) { od->capvt = od->capvt ? 2 * od->capvt : 1024; od->vt = (float *)realloc(od->vt, sizeof(float) * 2 * (size_t)od->capvt); }
            const char *q = p + 2;
            for (int k = 0; k < 2; ++k) { while (*q == ' ' || *q == '\t') ++q; q = fast_atof_float(q, &od->vt[2 * od->nvt + k]); }
            od->nvt++;
        } else if (!strncmp(p, "mtllib", 6)) {
            const char *nm = p + 6; while (*nm == ' ' || *nm == '\t') ++nm;
            char dir[2048]; snprintf(dir, sizeof dir, "%s", path);
            char *slash = strrchr(dir, '/');
            char full[4096];
            if (slash) { slash[1] = 0; snprintf(full, sizeof full, "%s%s", dir, nm); } else snprintf(full, sizeof full, "%s", nm);
            load_mtl(full, od);
        } else if ((p[0] == 'g' || p[0] == 'o') && (p[1] == ' ' || p[1] == '\t' || p[1] == 0)) {
            /* ObjFileParser::getGroupName/createObject: a new group name starts a new
             * object + mesh inheriting the current material */
            const char *nm = p + 1; while (*nm == ' ' || *nm == '\t') ++nm;
            if (cur && !strcmp(nm, group)) continue;
            snprintf(group, sizeof group, "%s", nm);
            cur = new_mesh(od, cur_mtl);
            cur_has_obj = 1;
        } else if (!strncmp(p, "usemtl", 6)) {
            const char *nm = p + 6; while (*nm == ' ' || *nm == '\t') ++nm;
            int idx = find_mtl(od, nm);
            if (idx < 0) {  /* unknown name: Assimp creates a named default material */
                od->mats = (mtl *)realloc(od->mats, sizeof(mtl) * (size_t)(od->nmats + 1));
                mtl *m = &od->mats[od->nmats];
                memset(m, 0, sizeof(*m));
                snprintf(m->name, sizeof m->name, "%s", nm);
                m->kd[0] = m->kd[1] = m->kd[2] = 0.6f; m->d = 1.0f; m->ni = 1.0f;
                idx = od->nmats++;
            }
            if (idx == cur_mtl && cur) continue;   /* same material: ignored */
            cur_mtl = idx;
            if (!cur) { cur = new_mesh(od, cur_mtl); cur_has_obj = 1; continue; }
            if (cur->mtl != -2 && cur->mtl != idx && cur->nfaces > 0) cur = new_mesh(od, cur_mtl);  /* needsNewMesh */
            else cur->mtl = idx;
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            if (!cur) { cur = new_mesh(od, cur_mtl); cur_has_obj = 1; }
            int vi[64], ni[64], ti[64], nvtx = 0;
            const char *q = p + 1;
            while (*q && nvtx < 64) {
                while (*q == ' ' || *q == '\t') ++q;
                if (!*q) break;
                long a = strtol(q, (char **)&q, 10), nn = 0, tt = 0;
                if (*q == '/') {
                    ++q;
                    if (*q != '/') tt = strtol(q, (char **)&q, 10);
                    if (*q == '/') { ++q; nn = strtol(q, (char **)&q, 10); }
                }
                while (*q && *q != ' ' && *q != '\t') ++q;
                vi[nvtx] = (int)(a < 0 ? od->nv + a : a - 1);
                ni[nvtx] = nn == 0 ? -1 : (int)(nn < 0 ? od->nvn + nn : nn - 1);
                ti[nvtx] = tt == 0 ? -1 : (int)(tt < 0 ? od->nvt + tt : tt - 1);
                nvtx++;
            }
            if (nvtx == 3) mesh_push(cur, vi[0], vi[1], vi[2], ni[0], ni[1], ni[2], ti[0], ti[1], ti[2]);
            else if (nvtx == 4) {
                int s0 = quad_start(od, vi);
                int o[4] = {s0, (s0 + 1) % 4, (s0 + 2) % 4, (s0 + 3) % 4};
                mesh_push(cur, vi[o[0]], vi[o[1]], vi[o[2]], ni[o[0]], ni[o[1]], ni[o[2]], ti[o[0]], ti[o[1]], ti[o[2]]);
                mesh_push(cur, vi[o[0]], vi[o[2]], vi[o[3]], ni[o[0]], ni[o[2]], ni[o[3]], ti[o[0]], ti[o[2]], ti[o[3]]);
            } else if (nvtx > 4) {
                for (int k = 1; k + 1 < nvtx; ++k)
                    mesh_push(cur, vi[0], vi[k], vi[k + 1], ni[0], ni[k], ni[k + 1], ti[0], ti[k], ti[k + 1]);
            }
        }
    }
    (void)cur_has_obj;
    fclose(f);
    return 0;
}

/* GenVertexNormalsProcess with the default 175 degree limit: every corner
 * gets the normalised sum of the face normals of all corners at (nearly) the
 * same position inside the mesh. */
static void smooth_normals(const objdata *od, const omesh *m, float *cn /* 9 per face */)
{
    int nc = 3 * m->nfaces;
    float *fnrm = (float *)malloc(sizeof(float) * 3 * (size_t)m->nfaces);
    float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
    for (int fi = 0; fi < m->nfaces; ++fi) {
        const int *f = &m->faces[6 * fi];
        const float *a = &od->v[3 * f[0]], *b = &od->v[3 * f[1]], *c = &od->v[3 * f[2]];
        float e1[3], e2[3];
        fsub3(b, a, e1); fsub3(c, a, e2);
        float n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        float l = sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (l > 0.0f) fdivs3(n, l);   /* NormalizeSafe */
        memcpy(&fnrm[3 * fi], n, sizeof n);
        for (int k = 0; k < 3; ++k) {
            const float *v = &od->v[3 * f[k]];
            for (int d = 0; d < 3; ++d) { if (v[d] < lo[d]) lo[d] = v[d]; if (v[d] > hi[d]) hi[d] = v[d]; }
        }
    }
    float dd[3] = {hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]};
    float eps = sqrtf(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]) * 1e-4f;
    float eps2 = eps * eps;
    for (int i = 0; i < nc; ++i) {
        const float *pi = &od->v[3 * m->faces[6 * (i / 3) + (i % 3)]];
        float acc[3] = {0, 0, 0};
        for (int j = 0; j < nc; ++j) {
            const float *pj = &od->v[3 * m->faces[6 * (j / 3) + (j % 3)]];
            float d3[3]; fsub3(pj, pi, d3);
            if (d3[0] * d3[0] + d3[1] * d3[1] + d3[2] * d3[2] < eps2) {
                acc[0] += fnrm[3 * (j / 3)]; acc[1] += fnrm[3 * (j / 3) + 1]; acc[2] += fnrm[3 * (j / 3) + 2];
            }
        }
        float l = sqrtf(acc[0] * acc[0] + acc[1] * acc[1] + acc[2] * acc[2]);
        if (l > 0.0f) fdivs3(acc, l);
        memcpy(&cn[3 * i], acc, sizeof acc);
    }
    free(fnrm);
}

/* Matrix4x4 (geometry.h:919-1065): point transform with the w divide
 * (:966-983), Gauss-Jordan inverse with full pivoting (Matrix::invert,
 * :857-907) and normal_transform = inverse-transpose product (:830-838). */
static inline v3 mat4_point(const double *m, v3 v)
{
    const double x = m[0] * v.e[0] + m[1] * v.e[1] + m[2] * v.e[2] + m[3];
    const double y = m[4] * v.e[0] + m[5] * v.e[1] + m[6] * v.e[2] + m[7];
    const double z = m[8] * v.e[0] + m[9] * v.e[1] + m[10] * v.e[2] + m[11];
    const double w = m[12] * v.e[0] + m[13] * v.e[1] + m[14] * v.e[2] + m[15];
    if (w == 1.0) return mk(x, y, z);
    return sdiv(mk(x, y, z), w);
}
static inline v3 mat4_normal(const double *inv, v3 v)
{
    return mk(inv[0] * v.e[0] + inv[4] * v.e[1] + inv[8] * v.e[2],
              inv[1] * v.e[0] + inv[5] * v.e[1] + inv[9] * v.e[2],
              inv[2] * v.e[0] + inv[6] * v.e[1] + inv[10] * v.e[2]);
}
static int mat4_invert(const double *src, double *t)
{
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    memcpy(t, src, 16 * sizeof(double));
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        double big = 0;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < 4; k++) {
                    if (ipiv[k] == 0) {
                        if (fabs(t[4 * j + k]) >= big) { big = fabs(t[4 * j + k]); irow = j; icol = k; }
                    } else if (ipiv[k] > 1) {
                        return 0;
                    }
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) { double x = t[4 * irow + k]; t[4 * irow + k] = t[4 * icol + k]; t[4 * icol + k] = x; }
        indxr[i] = irow; indxc[i] = icol;
        if (t[4 * icol + icol] == 0) return 0;
        const double pivinv = 1.0 / t[4 * icol + icol];
        t[4 * icol + icol] = 1.0;
        for (int j = 0; j < 4; j++) t[4 * icol + j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j != icol) {
                const double save = t[4 * j + icol];
                t[4 * j + icol] = 0;
                for (int k = 0; k < 4; k++) t[4 * j + k] -= t[4 * icol + k] * save;
            }
        }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) {
                double x = t[4 * k + indxr[j]]; t[4 * k + indxr[j]] = t[4 * k + indxc[j]]; t[4 * k + indxc[j]] = x;
            }
    return 1;
}

/* material from the 26-double description of ora_scene_add_obj / _add_sphere */
static material material_from_desc(const double *d)
{
    material m; memset(&m, 0, sizeof(m));
    m.type = (int)d[0];
    m.albedo = vload(d + 1); m.emit = vload(d + 4);
    m.ks[0] = d[7]; m.ks[1] = d[8]; m.ks[2] = d[9];
    m.shininess = d[10]; m.ior = d[11]; m.dist = (int)d[12]; m.alpha = d[13];
    m.eta = vload(d + 14); m.k = vload(d + 17);
    m.tex = (int)d[20]; m.tex_odd = vload(d + 21); m.tex_scale[0] = d[24]; m.tex_scale[1] = d[25];
    if (m.tex == TEX_IMAGE) m.image = (int)d[26];   /* the description is 27 doubles then */
    return m;
}

static int add_obj_x(ora_scene *s, const char *path, int geo, int32_t **lights, int *nlights,
                     const double *to_world, const double *bsdf);
/* create_triangle_mesh (triangle.cpp:9-23) + mesh_loader material mapping */
static int add_obj(ora_scene *s, const char *path, int geo, int32_t **lights, int *nlights)
{
    return add_obj_x(s, path, geo, lights, nlights, NULL, NULL);
}
/* ... and its (file, toWorld, bsdf) overload (triangle.cpp:26-60): every mesh
 * of the file takes `bsdf` when given; vertices go through toWorld, normals
 * through its inverse transpose. */
static int add_obj_x(ora_scene *s, const char *path, int geo, int32_t **lights, int *nlights,
                     const double *to_world, const double *bsdf)
{
    double inv[16];
    if (to_world && !mat4_invert(to_world, inv)) return -2;
    int shared_mat = -1;
    objdata od; memset(&od, 0, sizeof(od));
    if (parse_obj(path, &od) != 0) return -1;
    for (int mi = 0; mi < od.nmeshes; ++mi) {
        omesh *m = &od.meshes[mi];
        if (m->nfaces == 0) continue;   /* Assimp drops empty meshes */
        /* material (mesh_loader.cpp:59-112) */
        material mat; memset(&mat, 0, sizeof(mat));
        const mtl *mt = (m->mtl >= 0) ? &od.mats[m->mtl] : NULL;
        if (!mt) {
            mat.type = MAT_LAMBERT; mat.albedo = mk(0.5, 0.5, 0.5);
        } else if (mt->ke[0] != 0 || mt->ke[1] != 0 || mt->ke[2] != 0) {
            mat.type = MAT_LIGHT; mat.emit = mk(mt->ke[0], mt->ke[1], mt->ke[2]);
        } else if (mt->ks[0] != 0 || mt->ks[1] != 0 || mt->ks[2] != 0) {
            mat.type = (mt->d < 1.0f) ? MAT_DIELECTRIC : MAT_PHONG;
            mat.albedo = mk(FromSrgb(mt->kd[0]), FromSrgb(mt->kd[1]), FromSrgb(mt->kd[2]));
            mat.ks[0] = FromSrgb(mt->ks[0]); mat.ks[1] = FromSrgb(mt->ks[1]); mat.ks[2] = FromSrgb(mt->ks[2]);
            mat.ior = mt->ni; mat.shininess = mt->ns;
        } else {
            mat.type = MAT_LAMBERT;
            mat.albedo = mk(FromSrgb(mt->kd[0]), FromSrgb(mt->kd[1]), FromSrgb(mt->kd[2]));
        }
        int mat_idx;
        if (bsdf) {                                     /* mesh->mat.reset(bsdf): one material for all */
            if (shared_mat < 0) {
                s->mats = (material *)realloc(s->mats, sizeof(material) * (size_t)(s->nmats + 1));
                s->mats[s->nmats] = material_from_desc(bsdf);
                shared_mat = s->nmats++;
            }
            mat_idx = shared_mat;
            mat = s->mats[mat_idx];
        } else {
            s->mats = (material *)realloc(s->mats, sizeof(material) * (size_t)(s->nmats + 1));
            s->mats[s->nmats] = mat;
            mat_idx = s->nmats++;
        }
        /* normals: vn when every corner has one, else GenSmoothNormals */
        int has_vn = 1;
        for (int fi = 0; fi < m->nfaces && has_vn; ++fi)
            for (int k = 0; k < 3; ++k) if (m->faces[6 * fi + 3 + k] < 0) has_vn = 0;
        float *cn = (float *)malloc(sizeof(float) * 9 * (size_t)m->nfaces);
        if (has_vn) {
            for (int fi = 0; fi < m->nfaces; ++fi)
                for (int k = 0; k < 3; ++k) memcpy(&cn[9 * fi + 3 * k], &od.vn[3 * m->faces[6 * fi + 3 + k]], 3 * sizeof(float));
        } else if (!geo) {
            smooth_normals(&od, m, cn);
        } else {
            memset(cn, 0, sizeof(float) * 9 * (size_t)m->nfaces);
        }
        /* texture coordinates (mesh_loader.cpp:34-38) when every corner has a vt;
         * without them the reference leaves uv uninitialised -- here 0 */
        int has_vt = od.nvt > 0;
        for (int c = 0; c < 3 * m->nfaces && has_vt; ++c)
            if (m->tfaces[c] < 0 || m->tfaces[c] >= od.nvt) has_vt = 0;
        s->tris = (tri *)realloc(s->tris, sizeof(tri) * (size_t)(s->ntris + m->nfaces));
        for (int fi = 0; fi < m->nfaces; ++fi) {
            tri *t = &s->tris[s->ntris + fi];
            const int *f = &m->faces[6 * fi];
            for (int k = 0; k < 3; ++k)
                for (int d = 0; d < 2; ++d) t->uv[2 * k + d] = has_vt ? (double)od.vt[2 * m->tfaces[3 * fi + k] + d] : 0.0;
            t->v0 = mk(od.v[3 * f[0]], od.v[3 * f[0] + 1], od.v[3 * f[0] + 2]);
            t->v1 = mk(od.v[3 * f[1]], od.v[3 * f[1] + 1], od.v[3 * f[1] + 2]);
            t->v2 = mk(od.v[3 * f[2]], od.v[3 * f[2] + 1], od.v[3 * f[2] + 2]);
            t->n0 = mk(cn[9 * fi], cn[9 * fi + 1], cn[9 * fi + 2]);
            t->n1 = mk(cn[9 * fi + 3], cn[9 * fi + 4], cn[9 * fi + 5]);
            t->n2 = mk(cn[9 * fi + 6], cn[9 * fi + 7], cn[9 * fi + 8]);
            if (to_world) {
                t->v0 = mat4_point(to_world, t->v0); t->v1 = mat4_point(to_world, t->v1); t->v2 = mat4_point(to_world, t->v2);
                t->n0 = mat4_normal(inv, t->n0); t->n1 = mat4_normal(inv, t->n1); t->n2 = mat4_normal(inv, t->n2);
            }
            t->e1 = vsub(t->v1, t->v0);
            t->e2 = vsub(t->v2, t->v0);
            t->inv_area = 1 / (0.5 * vlen(cross(t->e1, t->e2)) * m->nfaces);
            t->mat = mat_idx;
            t->geo = geo;
            if (mat.type == MAT_LIGHT) {
                *lights = (int32_t *)realloc(*lights, sizeof(int32_t) * (size_t)(*nlights + 1));
                (*lights)[(*nlights)++] = s->ntris + fi;
            }
        }
        s->ntris += m->nfaces;
        free(cn);
    }
    for (int i = 0; i < od.nmeshes; ++i) { free(od.meshes[i].faces); free(od.meshes[i].tfaces); }
    free(od.meshes); free(od.v); free(od.vn); free(od.vt); free(od.mats);
    return 0;
}

static int add_material(ora_scene *s, int type, v3 albedo, v3 emit)
{
    s->mats = (material *)realloc(s->mats, sizeof(material) * (size_t)(s->nmats + 1));
    memset(&s->mats[s->nmats], 0, sizeof(material));
    s->mats[s->nmats].type = type; s->mats[s->nmats].albedo = albedo; s->mats[s->nmats].emit = emit;
    return s->nmats++;
}
static int add_sphere(ora_scene *s, v3 c, double r, int mat)
{
    s->sph = (sphere *)realloc(s->sph, sizeof(sphere) * (size_t)(s->nsph + 1));
    s->sph[s->nsph].c = c; s->sph[s->nsph].r = r; s->sph[s->nsph].mat = mat;
    return s->nsph++;
}

int ora_load_scene(const char *kind, const char *obj_path, double aspect, ora_scene **out)
{
    ora_scene *s = (ora_scene *)calloc(1, sizeof(ora_scene));
    int32_t *lights = NULL; int nlights = 0;
    s->env = mk(0.0, 0.0, 0.0);
    if (!strcmp(kind, "cornell_box_obj") || !strcmp(kind, "obj_geo") || !strcmp(kind, "obj_smooth")) {
        /* main.cpp:222-252 */
        if (add_obj(s, obj_path, strcmp(kind, "obj_smooth") != 0, &lights, &nlights) != 0) { free(s); return -1; }
        s->world_kind = WORLD_BVH;
        int32_t *prims = (int32_t *)malloc(sizeof(int32_t) * (size_t)s->ntris);
        for (int i = 0; i < s->ntris; ++i) prims[i] = i;
        build_bvh(s, prims, s->ntris);
        free(prims);
        s->cam = camera_mk(mk(0, 1, (double)3.9f), mk(0, 1, 0), mk(0, 1, 0), 40.0, aspect, 0.0, 10.0);
    } else if (!strcmp(kind, "veach_mis")) {
        /* main.cpp:281-314: list world = mesh triangles + 5 spheres; lights = mesh
         * emitters + 5 separate (identical) sphere objects; black env. */
        if (add_obj(s, obj_path, 0, &lights, &nlights) != 0) { free(s); return -1; }
        const double cx[5] = {10, (double)-1.25f, (double)-3.75f, (double)1.25f, (double)3.75f};
        const double cy[5] = {10, 0, 0, 0, 0};
        const double cz[5] = {4, 0, 0, 0, 0};
        const double rad[5] = {0.5, (double)0.1f, (double)0.03333f, (double)0.3f, (double)0.9f};
        const double em[5] = {800, 100, (double)901.803f, (double)11.1111f, 1.23457};
        s->world_kind = WORLD_LIST;
        s->nlist = s->ntris + 5;
        s->list = (int32_t *)malloc(sizeof(int32_t) * (size_t)s->nlist);
        for (int i = 0; i < s->ntris; ++i) s->list[i] = i;
        for (int k = 0; k < 5; ++k) {
            int m = add_material(s, MAT_LIGHT, mk(0, 0, 0), mk(em[k], em[k], em[k]));
            s->list[s->ntris + k] = REF_SPHERE | add_sphere(s, mk(cx[k], cy[k], cz[k]), rad[k], m);
        }
        for (int k = 0; k < 5; ++k) {
            int m = add_material(s, MAT_LIGHT, mk(0, 0, 0), mk(em[k], em[k], em[k]));
            int id = add_sphere(s, mk(cx[k], cy[k], cz[k]), rad[k], m);
            lights = (int32_t *)realloc(lights, sizeof(int32_t) * (size_t)(nlights + 1));
            lights[nlights++] = REF_SPHERE | id;
        }
        s->cam = camera_mk(mk(0, 2, 15), mk(0, -2, 2.5), mk(0, 1, 0), 28.0, aspect, 0.0, 50.0);
    } else {
        free(s);
        return -3;
    }
    s->lights = lights; s->nlights = nlights;
    *out = s;
    return 0;
}

/* ---- incremental construction: what main.cpp's scene functions do with
 *      create_triangle_mesh / new sphere / camera / create_bvh ---- */
int ora_scene_new(ora_scene **out)
{
    ora_scene *s = (ora_scene *)calloc(1, sizeof(ora_scene));
    if (!s) return -1;
    s->env = mk(0.0, 0.0, 0.0);
    s->nodes = NULL; s->nnodes = 0; s->root = 0;
    *out = s;
    return 0;
}
/* world prims in insertion order; kept in `list` until ora_scene_finish */
static void push_world(ora_scene *s, int32_t ref)
{
    s->list = (int32_t *)realloc(s->list, sizeof(int32_t) * (size_t)(s->nlist + 1));
    s->list[s->nlist++] = ref;
}
int ora_scene_add_obj(ora_scene *s, const char *obj_path, const double *to_world16, const double *bsdf20,
                      int use_geometry_normals)
{
    const int t0 = s->ntris;
    const int rc = add_obj_x(s, obj_path, use_geometry_normals, &s->lights, &s->nlights, to_world16, bsdf20);
    if (rc != 0) return rc == -2 ? -2 : -1;
    for (int i = t0; i < s->ntris; ++i) push_world(s, i);
    return 0;
}
/* where: 1 = the world list, 2 = Scene::lights (a separate sphere object, as
 * veach_mis and random_scene do), 3 = both (one object) */
int ora_scene_add_sphere(ora_scene *s, const double *c, double r, const double *mat20, int where)
{
    s->mats = (material *)realloc(s->mats, sizeof(material) * (size_t)(s->nmats + 1));
    s->mats[s->nmats] = material_from_desc(mat20);
    const int m = s->nmats++;
    const int id = add_sphere(s, vload(c), r, m);
    if (where & 1) push_world(s, REF_SPHERE | id);
    if (where & 2) {
        s->lights = (int32_t *)realloc(s->lights, sizeof(int32_t) * (size_t)(s->nlights + 1));
        s->lights[s->nlights++] = REF_SPHERE | id;
    }
    return 0;
}
void ora_scene_set_camera(ora_scene *s, const double *from, const double *at, const double *vup, double vfov,
                          double aspect, double aperture, double focus)
{
    s->cam = camera_mk(vload(from), vload(at), vload(vup), vfov, aspect, aperture, focus);
}
/* world_kind 0: parallel_bvh_node::create_bvh over the world prims in
 * insertion order; 1: hitable_list */
int ora_scene_finish(ora_scene *s, int world_kind)
{
    s->world_kind = world_kind;
    if (world_kind == WORLD_BVH) {
        if (s->nlist > 0) build_bvh(s, s->list, s->nlist);
        free(s->list); s->list = NULL; s->nlist = 0;
    }
    return 0;
}
void ora_free_scene(ora_scene *s)
{
    if (!s) return;
    for (int i = 0; i < s->nimages; ++i) free(s->images[i].rgb);
    free(s->images);
    free(s->tris); free(s->sph); free(s->mats); free(s->nodes); free(s->list); free(s->lights); free(s);
}
/* util.h:62-66 */
static double from_srgb(double v)
{
    if (v <= 0.04045) return v * (1.0 / 12.92);
    return pow((v + 0.055) * (1.0 / 1.055), 2.4);
}
/* image_texture's image as stb decodes it (rows as given, 3 channels): format 0 =
 * 8-bit (texel FromSrgb(x / 255.0), texture.h:82-84), 1 = floats (the HDR branch) */
int ora_scene_add_image(ora_scene *s, int nx, int ny, int format, const void *data, int *index)
{
    if (!s || nx <= 0 || ny <= 0 || !data || (format != 0 && format != 1)) return -1;
    ora_image *im = (ora_image *)realloc(s->images, (size_t)(s->nimages + 1) * sizeof(ora_image));
    if (!im) return -1;
    s->images = im;
    const size_t n = (size_t)nx * ny * 3;
    double *rgb = (double *)malloc(n * sizeof(double));
    if (!rgb) return -1;
    for (size_t k = 0; k < n; ++k)
        rgb[k] = format == 0 ? from_srgb(((const uint8_t *)data)[k] / 255.0) : (double)((const float *)data)[k];
    s->images[s->nimages] = (ora_image){nx, ny, rgb};
    *index = s->nimages++;
    return 0;
}
/* Test hooks (pinned by the image KATs of oracle/ref_kat.cpp):
 * image_texture::value on an image given as stb decodes it, and the direction
 * -> (u, v) map of environment_map::eval (material.h:219-232). */
int ora_image_lookup(int nx, int ny, int format, const void *data, double u, double v, double *out3)
{
    if (nx <= 0 || ny <= 0 || !data || !out3 || (format != 0 && format != 1)) return -1;
    const size_t n = (size_t)nx * ny * 3;
    double *rgb = (double *)malloc(n * sizeof(double));
    if (!rgb) return -1;
    for (size_t k = 0; k < n; ++k)
        rgb[k] = format == 0 ? from_srgb(((const uint8_t *)data)[k] / 255.0) : (double)((const float *)data)[k];
    const ora_image img = {nx, ny, rgb};
    vstore(out3, image_value(&img, u, v));
    free(rgb);
    return 0;
}
void ora_env_uv(const double *d, double *u, double *v)
{
    const v3 direction = unit(vload(d));
    double phi = atan2(direction.e[0], -direction.e[2]);
    double theta = acos(direction.e[1]);
    phi = (phi < 0) ? (phi + M_PI * 2) : phi;
    theta = (theta < 0) ? (theta + M_PI) : theta;
    *u = phi / (2.0 * M_PI);
    *v = theta / (M_PI);
}

/* Scene::env_map with another constant texture (material.h:206-232); the
 * reference scenes' environment is black, so AO / normals tests set one. */
void ora_scene_set_env(ora_scene *s, const double *rgb) { s->env = vload(rgb); }
double ora_scene_ao_tmax(const ora_scene *s) { return world_box_size_y(s) * 0.50f; }
void ora_scene_get_info(const ora_scene *s, ora_scene_info *info)
{
    info->n_tris = s->ntris; info->n_spheres = s->nsph; info->n_materials = s->nmats;
    info->n_lights = s->nlights; info->n_nodes = s->nnodes; info->world_kind = s->world_kind;
    info->n_list = s->nlist; info->bvh_depth = s->bvh_depth;
}
/* nodes were allocated in pre-order (left subtree first) = left-first DFS order */
int ora_scene_export_bvh(const ora_scene *s, double *boxes, int32_t *left, int32_t *right)
{
    for (int i = 0; i < s->nnodes; ++i) {
        vstore(&boxes[6 * i], s->nodes[i].box.min);
        vstore(&boxes[6 * i + 3], s->nodes[i].box.max);
        left[i] = s->nodes[i].left; right[i] = s->nodes[i].right;
    }
    return s->nnodes;
}
int ora_scene_export_tris(const ora_scene *s, double *v9, int32_t *mat)
{
    for (int i = 0; i < s->ntris; ++i) {
        vstore(&v9[9 * i], s->tris[i].v0); vstore(&v9[9 * i + 3], s->tris[i].v1); vstore(&v9[9 * i + 6], s->tris[i].v2);
        mat[i] = s->tris[i].mat;
    }
    return s->ntris;
}


/* camera as constructed (camera.h:10-28): origin, llc, horizontal, vertical, u, v, lens_radius (19 doubles) */
void ora_scene_export_camera(const ora_scene *s, double *out19)
{
    vstore(out19, s->cam.origin); vstore(out19 + 3, s->cam.llc); vstore(out19 + 6, s->cam.horizontal);
    vstore(out19 + 9, s->cam.vertical); vstore(out19 + 12, s->cam.u); vstore(out19 + 15, s->cam.v);
    out19[18] = s->cam.lens_radius;
}
/* lights (prim refs) and materials (type, albedo[3], emit[3] -> 7 doubles each) */
int ora_scene_export_lights(const ora_scene *s, int32_t *refs)
{
    for (int i = 0; i < s->nlights; ++i) refs[i] = s->lights[i];
    return s->nlights;
}
int ora_scene_export_materials(const ora_scene *s, double *out26)
{
    for (int i = 0; i < s->nmats; ++i) {
        double *o = out26 + 26 * i;
        o[0] = s->mats[i].type;
        vstore(o + 1, s->mats[i].albedo); vstore(o + 4, s->mats[i].emit);
        o[7] = s->mats[i].ks[0]; o[8] = s->mats[i].ks[1]; o[9] = s->mats[i].ks[2];
        o[10] = s->mats[i].shininess; o[11] = s->mats[i].ior;
        o[12] = s->mats[i].dist; o[13] = s->mats[i].alpha;
        vstore(o + 14, s->mats[i].eta); vstore(o + 17, s->mats[i].k);
        o[20] = s->mats[i].tex; vstore(o + 21, s->mats[i].tex_odd);
        o[24] = s->mats[i].tex_scale[0]; o[25] = s->mats[i].tex_scale[1];
    }
    return s->nmats;
}

/* ------------------------------------------------------------------------ */
/* known-answer entry points                                                */
/* ------------------------------------------------------------------------ */
static tri kat_tri(const double *v9, const double *n9, int geo, int nmesh)
{
    tri t; memset(&t, 0, sizeof t);
    t.v0 = vload(v9); t.v1 = vload(v9 + 3); t.v2 = vload(v9 + 6);
    if (n9) { t.n0 = vload(n9); t.n1 = vload(n9 + 3); t.n2 = vload(n9 + 6); }
    t.e1 = vsub(t.v1, t.v0); t.e2 = vsub(t.v2, t.v0);
    t.inv_area = 1 / (0.5 * vlen(cross(t.e1, t.e2)) * nmesh);
    t.geo = geo;
    return t;
}
int ora_kat_tri_hit(const double *v9, const double *n9, int geo, const double *o, const double *d,
                    double tmin, double tmax, double *out)
{
    tri t = kat_tri(v9, n9, geo, 1);
    ray r; r.o = vload(o); r.d = vload(d);
    hit_record h; double u = 0, v = 0;
    int ok = tri_hit(&t, &r, tmin, tmax, &h, &u, &v);
    memset(out, 0, sizeof(double) * 10);
    out[0] = ok;
    if (ok) { out[1] = h.t; vstore(out + 2, h.p); vstore(out + 5, h.normal); out[8] = u; out[9] = v; }
    return ok;
}
int ora_kat_sphere_hit(const double *c, double r, const double *o, const double *d, double tmin, double tmax, double *out)
{
    sphere sp; sp.c = vload(c); sp.r = r; sp.mat = 0;
    ray ry; ry.o = vload(o); ry.d = vload(d);
    hit_record h;
    int ok = sphere_hit(&sp, &ry, tmin, tmax, &h);
    memset(out, 0, sizeof(double) * 8);
    out[0] = ok;
    if (ok) { out[1] = h.t; vstore(out + 2, h.p); vstore(out + 5, h.normal); }
    return ok;
}
/* KAT: hit texture coordinates and checker_texture::value's pick (texture.h:35-44):
 * out4 = ok, u, v, odd; t_max = (double)FLT_MAX as in the reference harness */
int ora_kat_texture_sphere(const double *c, double r, const double *o, const double *d, double us, double vs,
                           double *out4)
{
    sphere sp; sp.c = vload(c); sp.r = r; sp.mat = 0;
    ray ry; ry.o = vload(o); ry.d = vload(d);
    hit_record h;
    const int ok = sphere_hit(&sp, &ry, 1e-4, (double)3.40282347e+38f, &h);
    memset(out4, 0, sizeof(double) * 4);
    out4[0] = ok;
    if (ok) { out4[1] = h.tu; out4[2] = h.tv; out4[3] = checker_odd(h.tu, h.tv, us, vs); }
    return ok;
}
int ora_kat_texture_tri(const double *v9, const double *uv6, const double *o, const double *d, double us, double vs,
                        double *out4)
{
    tri t = kat_tri(v9, NULL, 1, 1);
    memcpy(t.uv, uv6, sizeof(double) * 6);
    ray r; r.o = vload(o); r.d = vload(d);
    hit_record h;
    const int ok = tri_hit(&t, &r, 1e-4, (double)3.40282347e+38f, &h, NULL, NULL);
    memset(out4, 0, sizeof(double) * 4);
    out4[0] = ok;
    if (ok) { out4[1] = h.tu; out4[2] = h.tv; out4[3] = checker_odd(h.tu, h.tv, us, vs); }
    return ok;
}
int ora_kat_aabb_hit(const double *lo, const double *hi, const double *o, const double *d, double tmin, double tmax)
{
    aabb b = aabb_mk(vload(lo), vload(hi));
    ray r; r.o = vload(o); r.d = vload(d);
    return aabb_hit(&b, &r, tmin, tmax);
}
void ora_kat_camera(const double *from, const double *at, const double *vup, double vfov, double aspect,
                    double aperture, double focus, double s, double t, const double *smp, double *out6)
{
    camera c = camera_mk(vload(from), vload(at), vload(vup), vfov, aspect, aperture, focus);
    ray r = camera_get_ray(&c, s, t, smp[0], smp[1]);
    vstore(out6, r.o); vstore(out6 + 3, r.d);
}
void ora_kat_cosine(const double *n, const double *smp, double *out4)
{
    onb b = onb_from_w(vload(n));
    v3 d = onb_from_local(&b, hemisphere_to_cosine_direction(smp[0], smp[1]));
    vstore(out4, d);
    out4[3] = cosine_pdf_value(vload(n), d);
}
/* specular KATs (ref_kat.cpp kat_specular) */
void ora_kat_fresnel(const double *n, const double *wi, double eta, double *out8)
{
    double cosT = 0;
    const double F = fresnelDielectricExt(dot(vload(wi), vload(n)), &cosT, eta);
    out8[0] = F; out8[1] = cosT;
    vstore(out8 + 2, ref_reflect(vneg(vload(wi)), vload(n)));
    vstore(out8 + 5, ref_refract(vload(wi), vload(n), eta, cosT));
}
void ora_kat_phong(const double *n, const double *wi, double e, double s0, double s1, const double *wo,
                   const double *kd, const double *ks, double *out11)
{
    const v3 N = vload(n), WI = vload(wi), WO = vload(wo);
    const v3 d = cosine_power_generate(N, WI, e, s0, s1);
    vstore(out11, d);
    out11[3] = cosine_power_value(N, WI, e, d);
    out11[4] = cosine_power_value(N, WI, e, WO);
    vstore(out11 + 5, phong_eval(vload(kd), ks, e, N, WI, d));
    vstore(out11 + 8, phong_eval(vload(kd), ks, e, N, WI, WO));
}
void ora_kat_dielectric(const double *n, const double *wi, double ior, double u0, const double *wo, const double *ks,
                        double *out12)
{
    const v3 N = vload(n), WI = vload(wi), WO = vload(wo);
    const v3 d = dielectric_generate(N, WI, ior, u0);
    double cosT = 0;
    const double F = fresnelDielectricExt(dot(WI, N), &cosT, ior);
    vstore(out12, d);
    out12[3] = (u0 <= F) ? 1.0 : (cosT < 0 ? ior : (1.0 / ior));   /* srec.eta (pdf.h:171-181) */
    out12[4] = dielectric_value(N, WI, ior, d);
    out12[5] = dielectric_value(N, WI, ior, WO);
    vstore(out12 + 6, dielectric_eval(ks, ior, N, WI, d));
    vstore(out12 + 9, dielectric_eval(ks, ior, N, WI, WO));
}
void ora_kat_metal(const double *n, const double *wi, const double *albedo, const double *wo, double *out7)
{
    material m; memset(&m, 0, sizeof m);
    m.type = MAT_METAL; m.albedo = vload(albedo);
    const v3 N = vload(n), WI = vload(wi), WO = vload(wo);
    double sp;
    vstore(out7, spec_generate(&m, N, WI, vneg(WI), 0.0, 0.0, &sp));   /* r_in = ray(0, -wi) */
    out7[3] = spec_value(&m, N, WI, WO);
    vstore(out7 + 4, spec_eval(&m, N, WI, WO));
}
/* rough_conductor: out = generate() dir[3], sampled_pdf, value(unit(dir)), value(wo),
 * eval_bsdf(unit(dir))[3], eval_bsdf(wo)[3] */
void ora_kat_conductor(const double *n, const double *wi, int ggx, double alpha, const double *eta, const double *k,
                       const double *spec, double s0, double s1, const double *wo, double *out12)
{
    material m; memset(&m, 0, sizeof m);
    m.type = MAT_ROUGH; m.alpha = alpha; m.dist = ggx ? DIST_GGX : DIST_BECKMANN;
    m.eta = vload(eta); m.k = vload(k); m.ks[0] = spec[0]; m.ks[1] = spec[1]; m.ks[2] = spec[2];
    const v3 N = vload(n), WI = vload(wi), WO = vload(wo);
    double sp;
    const v3 d = rough_generate(N, WI, alpha, m.dist, s0, s1, &sp);
    const v3 du = unit(d);
    vstore(out12, d);
    out12[3] = sp;
    out12[4] = rough_value(N, WI, alpha, m.dist, du);
    out12[5] = rough_value(N, WI, alpha, m.dist, WO);
    vstore(out12 + 6, rough_eval(&m, N, WI, du));
    vstore(out12 + 9, rough_eval(&m, N, WI, WO));
}
void ora_kat_tri_sample(const double *v9, const double *n9, int geo, int n_tris_in_mesh, const double *o,
                        const double *smp, double *out10)
{
    ora_scene s; memset(&s, 0, sizeof s);
    tri t = kat_tri(v9, n9, geo, n_tris_in_mesh);
    s.tris = &t; s.ntris = 1;
    hit_record rec;
    v3 tl = prim_sample_direct(&s, 0, &rec, vload(o), smp[0], smp[1]);
    vstore(out10, rec.p); vstore(out10 + 3, rec.normal); vstore(out10 + 6, tl);
    out10[9] = prim_pdf_direct(&s, 0, &rec, tl);
}
void ora_kat_sphere_sample(const double *c, double r, const double *o, const double *smp, double *out7)
{
    ora_scene s; memset(&s, 0, sizeof s);
    sphere sp; sp.c = vload(c); sp.r = r; sp.mat = 0;
    s.sph = &sp; s.nsph = 1;
    hit_record rec; memset(&rec, 0, sizeof rec);
    v3 tl = prim_sample_direct(&s, REF_SPHERE, &rec, vload(o), smp[0], smp[1]);
    vstore(out7, tl); vstore(out7 + 3, rec.normal);
    /* pdf_direct_sampling(lrec, to_light) as evaluated at a BSDF hit: lrec.p = o + 1*tl, t = 1 */
    hit_record l2; l2.t = 1.0; l2.p = vadd(vload(o), tl); l2.normal = rec.normal;
    out7[6] = prim_pdf_direct(&s, REF_SPHERE, &l2, tl);
}
double ora_kat_miweight(double a, double b) { return miWeight(a, b); }
double ora_kat_fromsrgb(double v) { return FromSrgb(v); }
int ora_kat_pick(double u, int n) { return pick_sample(u, n); }
static int key_cmp(const void *a, const void *b, void *arg)
{
    const double *k = (const double *)arg;
    if (k[*(const int32_t *)a] - k[*(const int32_t *)b] < 0.0) return -1;
    return 1;
}
void ora_kat_sort(const double *keys, int n, int32_t *perm_out)
{
    for (int i = 0; i < n; ++i) perm_out[i] = i;
    qsort_r(perm_out, (size_t)n, sizeof(int32_t), key_cmp, (void *)keys);
}


/* hitable_list::hit over ntri triangles (9 doubles each, geometric normals)
 * followed by nsph spheres (c[3], r): out = hit, winner index, t */
void ora_kat_list_hit(int ntri, int nsph, const double *geom, const double *o, const double *d, double *out3)
{
    ora_scene s; memset(&s, 0, sizeof s);
    s.tris = (tri *)calloc((size_t)ntri + 1, sizeof(tri));
    s.sph = (sphere *)calloc((size_t)nsph + 1, sizeof(sphere));
    s.list = (int32_t *)calloc((size_t)(ntri + nsph) + 1, sizeof(int32_t));
    for (int i = 0; i < ntri; ++i) { s.tris[i] = kat_tri(geom + 9 * i, NULL, 1, 1); s.list[i] = i; }
    for (int k = 0; k < nsph; ++k) {
        const double *g = geom + 9 * ntri + 4 * k;
        s.sph[k].c = vload(g); s.sph[k].r = g[3];
        s.list[ntri + k] = REF_SPHERE | k;
    }
    s.ntris = ntri; s.nsph = nsph; s.nlist = ntri + nsph; s.world_kind = WORLD_LIST;
    ray r; r.o = vload(o); r.d = vload(d);
    hit_record h; ora_counters cnt; memset(&cnt, 0, sizeof cnt);
    int ok = world_hit(&s, &r, EPSILON, FLT_MAX, &h, &cnt);
    out3[0] = ok; out3[1] = -1; out3[2] = 0;
    if (ok) {
        out3[1] = (h.obj & REF_SPHERE) ? ntri + (h.obj & ~REF_SPHERE) : h.obj;
        out3[2] = h.t;
    }
    free(s.tris); free(s.sph); free(s.list);
}

/* image_pfm::save_image (image.h:89-118): "PF\n<w> <h>\n-1\n" + float rows y=0..h-1 */
/* viewer::add_sample's display bytes (viewer.cpp:115-117) */
void ora_tonemap_u8(const double *rgb, long n, uint8_t *out)
{
    for (long i = 0; i < n; ++i) out[i] = (uint8_t)(int)(pow(1 - exp(-rgb[i]), 1 / 2.2) * 255 + .5);
}
int ora_write_pfm(const char *path, int nx, int ny, const double *rgb)
{
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    fprintf(f, "PF\n%d %d\n-1\n", nx, ny);
    for (int i = 0; i < nx * ny * 3; ++i) { float v = (float)rgb[i]; fwrite(&v, sizeof v, 1, f); }
    fclose(f);
    return 0;
}
