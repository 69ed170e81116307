// ref_kat.cpp -- TEST INFRASTRUCTURE.  Known-answer generator built FROM THE
// REFERENCE'S OWN SOURCES (compiled where they lie under /root/reference, see
// oracle/Makefile target `ref`; output only into oracle/_ref/).  It drives the
// reference's component code on deterministic inputs and prints every input
// and output as a C99 hex float, one case per line:
//     <kind> <in...> | <out...>
// oracle/gen_golden.py turns the lines into tests/golden/kat_*.json; the
// tests then check the C restatement (oracle/frt_oracle.c) bit for bit.
//
// Nothing here restates reference logic: every output is computed by the
// reference's own classes (triangle.h, sphere.h, aabb.h, camera.h, pdf.h,
// onb.h, util.h, hitable_list.cpp, bvh.h comparators + glibc qsort,
// image.h image_pfm).  path.cpp / parallel_bvh.h / viewer.cpp / mesh_loader.cpp
// need cpp-taskflow, GLFW/GLEW and Assimp, which this image lacks, so they are
// not built (DESIGN.md "Oracle").
#include "triangle.h"
#include "sphere.h"
#include "camera.h"
#include "pdf.h"
#include "bvh.h"
#include "hitable_list.h"
#include "image.h"
#include "material.h"

#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>
#include <memory>

static uint64_t g_state = 0x1234567ULL;
static uint64_t next_u64()
{
    uint64_t z = (g_state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
static double urand() { return (double)(next_u64() >> 11) * (1.0 / 9007199254740992.0); }
static double srand2(double a) { return (urand() * 2 - 1) * a; }
// coordinates on a float grid (what the OBJ path delivers): float -> double
static double fgrid(double a) { return (double)(float)srand2(a); }

static void p(double v) { printf(" %a", v); }
static void pv(const Vector3f &v) { p(v[0]); p(v[1]); p(v[2]); }
static void bar() { printf(" |"); }

static std::shared_ptr<triangle_mesh> make_mesh(const double *v9, const double *n9, bool geo, int ntris)
{
    // 3 vertices per triangle, all triangles identical copies (only triangle 0 is queried)
    Vector3f *vv = new Vector3f[3 * ntris];
    Vector3f *nn = new Vector3f[3 * ntris];
    Vector2f *uv = new Vector2f[3 * ntris];
    std::vector<int> idx;
    for (int t = 0; t < ntris; ++t)
        for (int k = 0; k < 3; ++k) {
            vv[3 * t + k] = Vector3f(v9[3 * k], v9[3 * k + 1], v9[3 * k + 2]);
            nn[3 * t + k] = n9 ? Vector3f(n9[3 * k], n9[3 * k + 1], n9[3 * k + 2]) : Vector3f(0, 0, 1);
            uv[3 * t + k] = Vector2f(0, 0);
            idx.push_back(3 * t + k);
        }
    std::unique_ptr<material> mat = std::make_unique<lambertian>(new constant_texture(Vector3f(0.5, 0.5, 0.5)));
    return std::make_shared<triangle_mesh>(ntris, 3 * ntris, vv, idx.data(), nn, uv, std::move(mat), geo, "kat", true);
}

static void rand_tri(double *v9)
{
    for (int i = 0; i < 9; ++i) v9[i] = fgrid(2.0);
}
static void rand_unit(double *n)
{
    Vector3f v(srand2(1), srand2(1), srand2(1));
    v = unit_vector(v);
    n[0] = v[0]; n[1] = v[1]; n[2] = v[2];
}

static void kat_tri_hit(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        double v9[9], n9[9];
        rand_tri(v9);
        for (int k = 0; k < 3; ++k) rand_unit(n9 + 3 * k);
        const bool geo = (c % 2) == 0;
        auto mesh = make_mesh(v9, n9, geo, 1);
        triangle tr(mesh, 0);
        // ray aimed at a random barycentric point (some outside the triangle)
        double a = urand() * 1.4 - 0.2, b = urand() * 1.4 - 0.2;
        Vector3f target = (1 - a - b) * Vector3f(v9[0], v9[1], v9[2]) + a * Vector3f(v9[3], v9[4], v9[5]) + b * Vector3f(v9[6], v9[7], v9[8]);
        Vector3f o(fgrid(4), fgrid(4), fgrid(4));
        Vector3f d = target - o;
        if (c % 3 == 1) d = unit_vector(d);
        double tmin = (c % 5 == 0) ? 1e-4 : urand() * 0.5;
        double tmax = (c % 7 == 0) ? urand() * 1.5 : (double)FLT_MAX;
        hit_record h;
        bool ok = tr.hit(ray(o, d), tmin, tmax, h);
        printf("tri_hit");
        for (double x : v9) p(x);
        for (double x : n9) p(x);
        p(geo ? 1 : 0); pv(o); pv(d); p(tmin); p(tmax);
        bar();
        p(ok ? 1 : 0);
        if (ok) { p(h.t); pv(h.p); pv(h.normal); p(h.uv.x); p(h.uv.y); }
        else for (int i = 0; i < 9; ++i) p(0);
        printf("\n");
    }
}

static void kat_sphere_hit(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        Vector3f cen(fgrid(3), fgrid(3), fgrid(3));
        double r = (double)(float)(0.05 + urand());
        sphere sp(cen, r, nullptr);
        Vector3f o = (c % 4 == 0) ? cen + Vector3f(srand2(r * 0.5), srand2(r * 0.5), srand2(r * 0.5))
                                  : Vector3f(fgrid(6), fgrid(6), fgrid(6));
        Vector3f target = cen + Vector3f(srand2(1.5 * r), srand2(1.5 * r), srand2(1.5 * r));
        Vector3f d = target - o;
        if (c % 3 == 1) d = unit_vector(d);
        double tmin = 1e-4, tmax = (c % 5 == 0) ? urand() : (double)FLT_MAX;
        hit_record h;
        bool ok = sp.hit(ray(o, d), tmin, tmax, h);
        printf("sphere_hit"); pv(cen); p(r); pv(o); pv(d); p(tmin); p(tmax); bar();
        p(ok ? 1 : 0);
        if (ok) { p(h.t); pv(h.p); pv(h.normal); } else for (int i = 0; i < 7; ++i) p(0);
        printf("\n");
    }
}

static void kat_aabb(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        Vector3f lo(fgrid(2), fgrid(2), fgrid(2));
        Vector3f hi = lo + Vector3f((double)(float)urand(), (double)(float)urand(), (double)(float)urand());
        if (c % 6 == 0) hi[c % 3] = lo[c % 3];   // flat box
        aabb b(lo, hi);
        Vector3f o(fgrid(4), fgrid(4), fgrid(4));
        Vector3f tgt = lo + Vector3f(urand() * 1.4 - 0.2, urand() * 1.4 - 0.2, urand() * 1.4 - 0.2) * (hi - lo);
        Vector3f d = tgt - o;
        if (c % 5 == 0) d[c % 3] = 0.0;          // axis-parallel: inf / NaN slabs
        double tmin = 1e-4, tmax = (c % 4 == 0) ? urand() : (double)FLT_MAX;
        bool ok = b.hit(ray(o, d), tmin, tmax);
        printf("aabb_hit"); pv(lo); pv(hi); pv(o); pv(d); p(tmin); p(tmax); bar(); p(ok ? 1 : 0);
        p(b.longest_axis()); p(b.area());
        printf("\n");
    }
}

static void kat_camera(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        Vector3f from, at;
        double vfov, aspect, aperture, focus;
        if (c == 0) { from = Vector3f(0, 1, 3.9f); at = Vector3f(0, 1, 0); vfov = 40; aspect = 1920.0 / 1080.0; aperture = 0; focus = 10; }
        else if (c == 1) { from = Vector3f(0, 2, 15); at = Vector3f(0, -2, 2.5); vfov = 28; aspect = 1920.0 / 1080.0; aperture = 0; focus = 50; }
        else {
            from = Vector3f(fgrid(5), fgrid(5), fgrid(5)); at = Vector3f(fgrid(1), fgrid(1), fgrid(1));
            vfov = 20 + 60 * urand(); aspect = 0.5 + urand() * 1.5; aperture = (c % 2) ? 0.0 : urand() * 0.2; focus = 1 + 20 * urand();
        }
        camera cam(from, at, Vector3f(0, 1, 0), vfov, aspect, aperture, focus);
        double s = urand(), t = urand(), l0 = urand(), l1 = urand();
        ray r = cam.get_ray(s, t, Vector2f(l0, l1));
        printf("camera"); pv(from); pv(at); p(vfov); p(aspect); p(aperture); p(focus); p(s); p(t); p(l0); p(l1); bar();
        pv(r.o); pv(r.d); printf("\n");
    }
}

static void kat_cosine(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        double n[3];
        rand_unit(n);
        if (c < 6) { n[0] = n[1] = n[2] = 0; n[c % 3] = (c < 3) ? 1 : -1; }
        Vector3f nv(n[0], n[1], n[2]);
        cosine_pdf pdf(nv);
        hit_record h;
        scatter_record srec(h);
        double s0 = urand(), s1 = urand();
        Vector3f d = pdf.generate(Vector2f(s0, s1), srec);
        double val = pdf.value(h, d);
        printf("cosine"); pv(nv); p(s0); p(s1); bar(); pv(d); p(val); printf("\n");
    }
}

static void kat_tri_sample(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        double v9[9], n9[9];
        rand_tri(v9);
        for (int k = 0; k < 3; ++k) rand_unit(n9 + 3 * k);
        const bool geo = (c % 2) == 0;
        const int ntris = 1 + (c % 3);
        auto mesh = make_mesh(v9, n9, geo, ntris);
        triangle tr(mesh, 0);
        Vector3f o(fgrid(4), fgrid(4), fgrid(4));
        double s0 = urand(), s1 = urand();
        hit_record rec;
        Vector3f tl = tr.sample_direct(rec, o, Vector2f(s0, s1));
        double pdfv = tr.pdf_direct_sampling(rec, tl);
        printf("tri_sample");
        for (double x : v9) p(x);
        for (double x : n9) p(x);
        p(geo ? 1 : 0); p(ntris); pv(o); p(s0); p(s1); bar();
        pv(rec.p); pv(rec.normal); pv(tl); p(pdfv); printf("\n");
    }
}

static void kat_sphere_sample(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        Vector3f cen(fgrid(3), fgrid(3), fgrid(3));
        double r = (double)(float)(0.05 + urand());
        sphere sp(cen, r, nullptr);
        Vector3f o = (c % 5 == 0) ? cen + Vector3f(srand2(r * 0.5), srand2(r * 0.5), srand2(r * 0.5))
                                  : Vector3f(fgrid(8), fgrid(8), fgrid(8));
        double s0 = urand(), s1 = urand();
        hit_record rec;
        Vector3f tl = sp.sample_direct(rec, o, Vector2f(s0, s1));
        hit_record l2;
        l2.t = 1.0; l2.p = o + tl; l2.normal = rec.normal;
        double pdfv = sp.pdf_direct_sampling(l2, tl);
        printf("sphere_sample"); pv(cen); p(r); pv(o); p(s0); p(s1); bar(); pv(tl); pv(rec.normal); p(pdfv); printf("\n");
    }
}

static void kat_scalar(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        double a = urand() * 10, b = urand() * 10;
        if (c == 0) b = 0;
        printf("miweight"); p(a); p(b); bar(); p(miWeight(a, b)); printf("\n");
        double v = (double)(float)urand();
        if (c < 3) v = (double)(float)(0.04045 * (0.5 + 0.5 * c));
        printf("fromsrgb"); p(v); bar(); p(FromSrgb(v)); printf("\n");
        int n = c % 7;
        double u = (c % 11 == 0) ? 1.0 - 1e-17 : urand();
        std::vector<hitable *> items(n, nullptr);
        hitable_list hl(items, n);
        printf("pick"); p(u); p(n); bar(); p(hl.pick_sample(u)); printf("\n");
    }
}

// glibc qsort + bvh.h comparator over triangles whose box.min.x are the keys (with ties)
static void kat_sort(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        int n = 2 + (int)(next_u64() % 40);
        std::vector<double> keys(n);
        for (int i = 0; i < n; ++i) keys[i] = (double)(int)(urand() * 6) * 0.25;   // many ties
        std::vector<std::shared_ptr<triangle_mesh>> meshes;
        std::vector<std::unique_ptr<triangle>> tris;
        std::vector<hitable *> l;
        for (int i = 0; i < n; ++i) {
            double v9[9] = {keys[i], 0, 0, keys[i] + 1, 0, 0, keys[i] + 0.5, 1, 0};
            meshes.push_back(make_mesh(v9, nullptr, true, 1));
            tris.push_back(std::make_unique<triangle>(meshes.back(), 0));
            l.push_back(tris.back().get());
        }
        std::vector<hitable *> sorted = l;
        qsort(sorted.data(), n, sizeof(hitable *), box_x_compare);
        printf("sort"); p(n); for (double k : keys) p(k); bar();
        for (int i = 0; i < n; ++i) {
            int idx = 0;
            while (l[idx] != sorted[i]) ++idx;
            p(idx);
        }
        printf("\n");
    }
}

// hitable_list::hit over triangles (with exact duplicates) and spheres: winner index + t
static void kat_list_hit(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        int ntri = 3 + (int)(next_u64() % 4), nsph = 2;
        std::vector<double> geom;
        std::vector<std::shared_ptr<triangle_mesh>> meshes;
        std::vector<std::unique_ptr<hitable>> objs;
        std::vector<hitable *> l;
        double base[9];
        rand_tri(base);
        for (int i = 0; i < ntri; ++i) {
            double v9[9];
            if (i % 2 == 1) for (int k = 0; k < 9; ++k) v9[k] = base[k];   // duplicates -> exact ties
            else rand_tri(v9);
            meshes.push_back(make_mesh(v9, nullptr, true, 1));
            objs.push_back(std::make_unique<triangle>(meshes.back(), 0));
            l.push_back(objs.back().get());
            for (double x : v9) geom.push_back(x);
        }
        for (int k = 0; k < nsph; ++k) {
            Vector3f cen(fgrid(2), fgrid(2), fgrid(2));
            double r = (double)(float)(0.2 + urand() * 0.5);
            objs.push_back(std::make_unique<sphere>(cen, r, nullptr));
            l.push_back(objs.back().get());
            geom.push_back(cen[0]); geom.push_back(cen[1]); geom.push_back(cen[2]); geom.push_back(r);
        }
        hitable_list hl(l, (int)l.size());
        Vector3f tgt = (1.0 / 3) * (Vector3f(base[0], base[1], base[2]) + Vector3f(base[3], base[4], base[5]) + Vector3f(base[6], base[7], base[8]));
        Vector3f o(fgrid(5), fgrid(5), fgrid(5));
        Vector3f d = tgt - o + Vector3f(srand2(0.3), srand2(0.3), srand2(0.3));
        hit_record h;
        bool ok = hl.hit(ray(o, d), 1e-4, FLT_MAX, h);
        int win = -1;
        if (ok) for (size_t i = 0; i < l.size(); ++i) if (h.obj == l[i]) win = (int)i;
        printf("list_hit"); p(ntri); p(nsph); for (double x : geom) p(x); pv(o); pv(d); bar();
        p(ok ? 1 : 0); p(win); p(ok ? h.t : 0.0); printf("\n");
    }
}

// image_pfm::save_image byte layout (image.h:89-118).  Writes to $HOME/<name>.
// specular materials: util.h reflect / refract / fresnelDielectricExt,
// cosine_power_pdf + modified_phong::eval_bsdf, dielectric_pdf + dielectric::eval_bsdf
static void kat_specular(int ncases)
{
    for (int c = 0; c < ncases; ++c) {
        double n[3], w[3];
        rand_unit(n);
        rand_unit(w);
        Vector3f nv(n[0], n[1], n[2]), wi(w[0], w[1], w[2]);
        if (c % 4 == 0 && dot(nv, wi) < 0) wi = -wi;         // mostly from outside
        // reflect / fresnel / refract
        const double eta = (c % 9 == 0) ? 1.0 : (double)(float)(1.05 + 1.5 * urand());
        double cosT = 0;
        const double F = fresnelDielectricExt(dot(wi, nv), cosT, eta);
        Vector3f rfl = reflect(-wi, nv);
        Vector3f rfr = refract(wi, nv, eta, cosT);
        printf("fresnel"); pv(nv); pv(wi); p(eta); bar(); p(F); p(cosT); pv(rfl); pv(rfr); printf("\n");
        // cosine_power_pdf + modified_phong
        const double e = (c % 3 == 0) ? 1024.0 : (double)(float)(1 + 200 * urand());
        hit_record h;
        h.normal = nv; h.wi = wi; h.p = Vector3f(0, 0, 0);
        ray r_in(Vector3f(0, 0, 0), -wi);
        cosine_power_pdf cpp(r_in, nv, e);
        scatter_record srec(h);
        const double s0 = urand(), s1 = urand();
        Vector3f d = cpp.generate(Vector2f(s0, s1), srec);
        double dr[3];
        rand_unit(dr);
        Vector3f wo(dr[0], dr[1], dr[2]);
        const Vector3f kd(urand(), urand(), urand()), ks(urand(), urand(), urand());
        modified_phong ph(new constant_texture(kd), new constant_texture(ks), e);
        printf("phong"); pv(nv); pv(wi); p(e); p(s0); p(s1); pv(wo); pv(kd); pv(ks); bar();
        pv(d); p(cpp.value(h, d)); p(cpp.value(h, wo)); pv(ph.eval_bsdf(r_in, h, d)); pv(ph.eval_bsdf(r_in, h, wo));
        printf("\n");
        // dielectric_pdf + dielectric
        const double ior = (c % 7 == 0) ? 1.0 : (double)(float)(1.1 + 1.5 * urand());
        dielectric_pdf dp(nv, ior);
        scatter_record srec2(h);
        const double u0 = (c % 5 == 0) ? 0.999999 : urand();
        Vector3f dd = dp.generate(Vector2f(u0, 0.5), srec2);
        dielectric de(ior, new constant_texture(ks), new constant_texture(Vector3f(1.0, 1.0, 1.0)));
        printf("dielectric"); pv(nv); pv(wi); p(ior); p(u0); pv(wo); pv(ks); bar();
        pv(dd); p(srec2.eta); p(dp.value(h, dd)); p(dp.value(h, wo)); pv(de.eval_bsdf(r_in, h, dd)); pv(de.eval_bsdf(r_in, h, wo));
        printf("\n");
    }
}

// checker_texture::value at sphere and triangle hits: the hit's texture
// coordinates (get_sphere_uv, the interpolated OBJ vt) and the colour picked
static void kat_texture(int ncases)
{
    const Vector3f c0(0.125, 0.25, 0.375), c1(0.625, 0.75, 0.875);
    for (int c = 0; c < ncases; ++c) {
        const double scales[5] = {1, 2, 5, 10, (double)(float)(0.5 + 20 * urand())};
        const double us = scales[c % 5], vs = scales[(c / 5) % 5];
        checker_texture tex(new constant_texture(c0), new constant_texture(c1), us, vs);
        hit_record h;
        bool ok;
        if (c % 2 == 0) {
            Vector3f cen(fgrid(3), fgrid(3), fgrid(3));
            // radii above 1 put |p - centre|.y past 1: asin's NaN, (int)NaN
            double r = (double)(float)(c % 8 == 0 ? 1.0 + 2 * urand() : 0.05 + 0.95 * urand());
            sphere sp(cen, r, nullptr);
            Vector3f o(fgrid(6), fgrid(6), fgrid(6));
            Vector3f d = cen + Vector3f(srand2(r), srand2(r), srand2(r)) - o;
            ok = sp.hit(ray(o, d), 1e-4, (double)FLT_MAX, h);
            printf("tex_sphere"); pv(cen); p(r); pv(o); pv(d); p(us); p(vs); bar();
        } else {
            double v9[9], uv6[6];
            rand_tri(v9);
            for (double &x : uv6) x = fgrid(2);
            Vector3f *vv = new Vector3f[3];
            Vector3f *nn = new Vector3f[3];
            Vector2f *uv = new Vector2f[3];
            int idx[3] = {0, 1, 2};
            for (int k = 0; k < 3; ++k) {
                vv[k] = Vector3f(v9[3 * k], v9[3 * k + 1], v9[3 * k + 2]);
                nn[k] = Vector3f(0, 0, 1);
                uv[k] = Vector2f(uv6[2 * k], uv6[2 * k + 1]);
            }
            auto mesh = std::make_shared<triangle_mesh>(1, 3, vv, idx, nn, uv,
                std::make_unique<lambertian>(new constant_texture(c0)), true, "kat", true);
            triangle tr(mesh, 0);
            double a = urand() * 0.9 + 0.05, b = urand() * (0.95 - a);
            Vector3f target = (1 - a - b) * vv[0] + a * vv[1] + b * vv[2];
            Vector3f o(fgrid(4), fgrid(4), fgrid(4));
            ok = tr.hit(ray(o, target - o), 1e-4, (double)FLT_MAX, h);
            printf("tex_tri");
            for (double x : v9) p(x);
            for (double x : uv6) p(x);
            pv(o); pv(target - o); p(us); p(vs); bar();
        }
        p(ok ? 1 : 0);
        if (ok) {
            const Vector3f col = tex.value(h);
            p(h.u); p(h.v); p(col[0] == c1[0] ? 1 : 0);
        } else for (int i = 0; i < 3; ++i) p(0);
        printf("\n");
    }
}

// image_texture::value (texture.h:59-95) on the reference's own `image`
// (image.h / image.cpp, stb vendored): u, v -> the texel it returns.  The
// queries cover the wrap (u < 0, u > 1) and the upper-edge clamp (u = 1).
static void img_query(const char *kind, const image_texture &tex, double u, double v)
{
    hit_record h;
    h.u = u;
    h.v = v;
    const Vector3f c = tex.value(h);
    printf("%s", kind); p(u); p(v); bar(); pv(c); printf("\n");
}
static double edge_coord(int i, int n, int k)   // lands in texel i (k = 0) or wraps to it (k = +-1, +-2)
{
    return ((double)i + 0.25 + 0.5 * urand()) / n + k;
}
static void kat_image(const char *hdr_path)
{
    // 8-bit image through image(unsigned char *, nx, ny, nn) (image.h:25).  That
    // constructor leaves `type` unset, so the harness sets it to an LDR format:
    // the FromSrgb(byte / 255.0) branch (texture.h:82-84)
    const int nx = 5, ny = 3;
    static unsigned char bytes[nx * ny * 3];
    for (int i = 0; i < nx * ny * 3; ++i) bytes[i] = (unsigned char)(next_u64() & 0xff);
    bytes[0] = 0; bytes[1] = 10; bytes[2] = 255;                // the sRGB curve's linear segment and 1.0
    printf("img_ldr_data"); p(nx); p(ny); for (unsigned char b : bytes) p(b); bar(); printf("\n");
    {
        auto img = std::make_unique<image>(bytes, nx, ny, 3);
        img->type = formats::STBI_PNG;
        image_texture tex(std::move(img));
        for (int c = 0; c < 60; ++c)
            img_query("img_ldr", tex, edge_coord((int)(next_u64() % nx), nx, (int)(next_u64() % 5) - 2),
                      edge_coord((int)(next_u64() % ny), ny, (int)(next_u64() % 5) - 2));
        img_query("img_ldr", tex, 1.0, 1.0);                    // i == nx, j == ny: clamped
        img_query("img_ldr", tex, 0.0, 0.0);
        img_query("img_ldr", tex, -1.0, 2.0);
        img_query("img_ldr", tex, -0.1 / nx, -0.1 / ny);        // truncates to 0
        tex.img.release();                                       // the harness owns `bytes`
    }
    // HDR branch (texture.h:74-79) on an in-memory float image, and
    // environment_map::eval (material.h:219-232) over the same texture
    const int hx = 7, hy = 5;
    static float hdr[hx * hy * 3];
    for (float &f : hdr) f = (float)(urand() * 4.0);
    printf("img_hdr_data"); p(hx); p(hy); for (float f : hdr) p(f); bar(); printf("\n");
    {
        auto img = std::make_unique<image>(nullptr, hx, hy, 3);
        img->type = formats::STBI_HDR;
        img->dataf = hdr;
        image_texture tex(std::move(img));
        for (int c = 0; c < 60; ++c)
            img_query("img_hdr", tex, edge_coord((int)(next_u64() % hx), hx, (int)(next_u64() % 5) - 2),
                      edge_coord((int)(next_u64() % hy), hy, (int)(next_u64() % 5) - 2));
        img_query("img_hdr", tex, 1.0, 1.0);
        tex.img.release();
        auto img2 = std::make_unique<image>(nullptr, hx, hy, 3);
        img2->type = formats::STBI_HDR;
        img2->dataf = hdr;
        environment_map env(std::make_unique<image_texture>(std::move(img2)));
        for (int c = 0; c < 120; ++c) {
            Vector3f d(srand2(1), srand2(1), srand2(1));
            if (c < 6) d = Vector3f(c == 0 ? 1 : c == 1 ? -1 : 0, c == 2 ? 1 : c == 3 ? -1 : 0, c == 4 ? 1 : c == 5 ? -1 : 0);
            hit_record h;
            const Vector3f e = env.eval(ray(Vector3f(0, 0, 0), d), h, 0);
            printf("env_img"); pv(d); bar(); pv(e); printf("\n");
        }
        static_cast<image_texture *>(env.env_map_tex.get())->img.release();
    }
    // data/test.hdr through image(file, STBI_HDR) (image.cpp:11-17): the
    // texels of a window -- 5 x 5 around the texel of highest local contrast plus the first
    // and last columns / rows -- read with image_texture::value(x, y)
    // (texture.h:90-95), and value(u, v) queries that land in the window
    // directly or through the wrap (k = +1 maps back to texel i; k = -1 to
    // i + 1, as (int) truncates toward zero) and the u = v = 1 clamp
    auto img = std::make_unique<image>(hdr_path, formats::STBI_HDR);
    const int fx = img->nx, fy = img->ny;
    int bx = 2, by = 2;
    float best = -1.0f;
    for (int y = 2; y < fy - 3; ++y)
        for (int x = 2; x < fx - 3; ++x) {
            const float *t = &img->dataf[3 * ((size_t)y * fx + x)], *r = t + 3, *d = t + 3 * (size_t)fx;
            float g = 0.0f;   // local contrast: distinct texels in the window
            for (int ch = 0; ch < 3; ++ch) g += std::fabs(t[ch] - r[ch]) + std::fabs(t[ch] - d[ch]);
            if (g > best) { best = g; bx = x; by = y; }
        }
    image_texture tex(std::move(img));
    std::vector<int> cols = {0, 1, fx - 1}, rows = {0, 1, fy - 1};
    for (int k = -2; k <= 3; ++k) { cols.push_back(bx + k); rows.push_back(by + k); }
    for (int x : cols)
        for (int y : rows) {
            const Vector3f c = tex.value(x, y);
            printf("hdr_file_texel"); p(fx); p(fy); p(x); p(y); bar(); pv(c); printf("\n");
        }
    for (int c = 0; c < 80; ++c) {
        const int i = bx - 2 + (int)(next_u64() % 5), j = by - 2 + (int)(next_u64() % 5);
        img_query("hdr_file", tex, edge_coord(i, fx, (int)(next_u64() % 3) - 1), edge_coord(j, fy, (int)(next_u64() % 3) - 1));
    }
    img_query("hdr_file", tex, 1.0, 1.0);
    img_query("hdr_file", tex, 0.0, 0.0);
}

static void kat_pfm()
{
    const int nx = 3, ny = 2, nn = 3;
    double data[nx * ny * nn];
    for (int i = 0; i < nx * ny * nn; ++i) data[i] = 0.1 * i + 1.0 / 3.0;
    image_pfm(data, nx, ny, nn).save_image("kat_ref.pfm");
    printf("pfm"); p(nx); p(ny); for (double x : data) p(x); bar(); printf(" kat_ref.pfm\n");
}

int main(int argc, char **argv)
{
    const int n = (argc > 1) ? atoi(argv[1]) : 200;
    kat_tri_hit(n);
    kat_sphere_hit(n);
    kat_aabb(n);
    kat_camera(n / 4);
    kat_cosine(n / 2);
    kat_tri_sample(n / 2);
    kat_sphere_sample(n / 2);
    kat_scalar(n / 2);
    kat_sort(n / 4);
    kat_list_hit(n / 2);
    kat_specular(n);
    kat_texture(n);
    kat_pfm();
    kat_image(argc > 2 ? argv[2] : "/root/reference/first_ray/data/test.hdr");
    return 0;
}
