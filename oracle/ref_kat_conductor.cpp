// ref_kat_conductor.cpp -- TEST INFRASTRUCTURE (see ref_kat.cpp).  Known
// answers for metal and rough_conductor, computed by the reference's own
// classes (material.h:110-130, 246-315; pdf.h:231-486; pdf.cpp:5-12;
// microfacet.h).
//
// Built as its own program because of util.h:130-143: under _GNU_SOURCE
// (always defined by g++/libstdc++) the reference's
// `inline void sincos(double, double*, double*) { sincos(theta, sin, cos); }`
// calls itself, so roughconductor_pdf::sampleVisible (pdf.h:422) never
// returns on Linux.  The reference's other configuration (util.h:139-148, the
// Visual Studio builds, vs19/) computes sinf/cosf of the angle.  This file
// selects that configuration by including the standard headers first and then
// undefining _GNU_SOURCE before the reference headers, so util.h takes its
// #else branch; nothing else in the reference depends on the macro.
#include <cmath>
#include <math.h>
#include <random>
#include <array>
#include <memory>
#include <iostream>
#include <fstream>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <cfloat>
#include <cassert>
#include <string>
#include <vector>
#include <algorithm>
#include <cctype>
#include <thread>
#include <atomic>
#include <mutex>
#undef _GNU_SOURCE
#include "material.h"

static uint64_t g_state = 0x7654321ULL;
static uint64_t next_u64()
{
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static double urand() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }
static double srand2(double a) { return (urand() * 2 - 1) * a; }
static void p(double v) { printf(" %a", v); }
static void pv(const Vector3f &v) { p(v[0]); p(v[1]); p(v[2]); }
static void bar() { printf(" |"); }
static void rand_unit(double *n)
{
    Vector3f v(srand2(1), srand2(1), srand2(1));
    v = unit_vector(v);
    n[0] = v[0]; n[1] = v[1]; n[2] = v[2];
}

// metal (material.h:110-130) and rough_conductor + roughconductor_pdf
// (material.h:246-315, pdf.h:231-486, pdf.cpp:5-12, microfacet.h): the
// visible-normal sample, its sampled_pdf, value() and eval_bsdf() toward the
// sample and toward an independent direction, for GGX and Beckmann.
static void kat_conductor(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        double n[3], w[3], x[3];
        rand_unit(n);
        rand_unit(w);
        rand_unit(x);
        Vector3f nv(n[0], n[1], n[2]), wi(w[0], w[1], w[2]), wo(x[0], x[1], x[2]);
        if (c % 8 != 7 && dot(nv, wi) < 0) wi = -wi;          // mostly from outside
        if (c % 2 == 0 && dot(nv, wo) < 0) wo = -wo;
        hit_record h;
        h.normal = nv; h.wi = wi; h.p = Vector3f(0, 0, 0);
        ray r_in(Vector3f(0, 0, 0), -wi);
        // metal::scatter / eval_bsdf
        const Vector3f alb(urand(), urand(), urand());
        metal me(alb);
        scatter_record ms(h);
        me.scatter(r_in, h, ms, Vector3f(urand(), urand(), urand()));
        printf("metal"); pv(nv); pv(wi); pv(alb); bar();
        pv(ms.specular_ray.direction()); p(ms.pdf_ptr->value(h, wo)); pv(me.eval_bsdf(r_in, h, wo)); printf("\n");
        // rough_conductor
        const int ggx = c % 2;
        const double alpha = (double)(float)(0.02 + 0.5 * urand());
        const Vector3f eta((float)(0.2 + 4 * urand()), (float)(0.2 + 4 * urand()), (float)(0.2 + 4 * urand()));
        const Vector3f k((float)(1 + 9 * urand()), (float)(1 + 9 * urand()), (float)(1 + 9 * urand()));
        const Vector3f spec(urand(), urand(), urand());
        rough_conductor rc(alpha, 1.0, eta, k, new constant_texture(spec), ggx ? "GGX" : "beckmann");
        roughconductor_pdf pdf(r_in, nv, alpha, alpha, ggx ? microfacet_distributions::ggx : microfacet_distributions::beckmann);
        scatter_record srec(h);
        const double s0 = urand(), s1 = urand();
        Vector3f d = pdf.generate(Vector2f(s0, s1), srec);
        printf("conductor"); pv(nv); pv(wi); p(ggx); p(alpha); pv(eta); pv(k); pv(spec); p(s0); p(s1); pv(wo); bar();
        pv(d); p(srec.sampled_pdf); p(pdf.value(h, unit_vector(d))); p(pdf.value(h, wo));
        pv(rc.eval_bsdf(r_in, h, unit_vector(d))); pv(rc.eval_bsdf(r_in, h, wo));
        printf("\n");
    }
}

int main(int argc, char **argv)
{
    const int n = (argc > 1) ? atoi(argv[1]) : 200;
    kat_conductor(n);
    return 0;
}
