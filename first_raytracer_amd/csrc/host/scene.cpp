// scene.cpp -- native host-side scene pipeline behind include/frt.h:
//   * OBJ/MTL ingest with the semantics of mesh_loader::load_obj
//     (first_ray/mesh_loader.cpp:5-162) on top of Assimp 5.0.1's OBJ import
//     (object/material mesh split, fast_atoreal_move parsing, quad
//     triangulation, GenSmoothNormals) -- Assimp is absent from this image,
//     its behaviour is restated ("unpinned at the Assimp boundary");
//   * create_triangle_mesh (triangle.cpp:9-23): one triangle per face,
//     emissive meshes feed Scene::lights;
//   * parallel_bvh_node::create_bvh (parallel_bvh.h:67-175): the SAH split
//     rule with glibc's merge-sort qsort order (bvh.h:6-55 comparators),
//     built with std::thread subtrees instead of taskflow subflows;
//   * scene constructors cornell_box_obj (main.cpp:222-252) and veach_mis
//     (main.cpp:281-314), camera (camera.h:10-28);
//   * the cornell_1m tessellation generator and the PFM writer (image.h:89-118).
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <new>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "frt.h"

namespace {

constexpr double kPi = 3.14159265358979323846;

struct V3 {
    double x = 0, y = 0, z = 0;
};
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator*(double t, V3 v) { return {t * v.x, t * v.y, t * v.z}; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double length(V3 v) { return std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
inline V3 unit(V3 v)
{
    const double l = length(v);
    return {v.x / l, v.y / l, v.z / l};
}

// ---------------------------------------------------------------------------
// Assimp fast_atoreal_move<float> (restated): integer part -> float, up to 15
// fractional digits as an integer scaled by a double table, added in float.
// ---------------------------------------------------------------------------
const double kAtofTable[16] = {0.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001,
                               0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001,
                               0.000000000000001};
uint64_t strtoul10_64(const char *in, const char **out, unsigned *max_inout)
{
    unsigned cur = 0;
    uint64_t value = 0;
    while (*in >= '0' && *in <= '9') {
        const uint64_t nv = value * 10 + (uint64_t)(*in - '0');
        if (nv < value) break;
        value = nv;
        ++in;
        ++cur;
        if (max_inout && *max_inout == cur) {
            while (*in >= '0' && *in <= '9') ++in;
            break;
        }
    }
    if (out) *out = in;
    if (max_inout) *max_inout = cur;
    return value;
}
const char *parse_float(const char *c, float &out)
{
    float f = 0.0f;
    const bool inv = (*c == '-');
    if (inv || *c == '+') ++c;
    if (!((*c >= '0' && *c <= '9') || ((*c == '.' || *c == ',') && c[1] >= '0' && c[1] <= '9'))) {
        out = 0.0f;
        return c;
    }
    if (!(*c == '.' || *c == ',')) f = (float)strtoul10_64(c, &c, nullptr);
    if ((*c == '.' || *c == ',') && c[1] >= '0' && c[1] <= '9') {
        ++c;
        unsigned diff = 15;
        double pl = (double)strtoul10_64(c, &c, &diff);
        pl *= kAtofTable[diff];
        f += (float)pl;
    } else if (*c == '.') {
        ++c;
    }
    if (*c == 'e' || *c == 'E') {
        ++c;
        const bool einv = (*c == '-');
        if (einv || *c == '+') ++c;
        float ex = (float)strtoul10_64(c, &c, nullptr);
        if (einv) ex = -ex;
        f *= std::pow(10.0f, ex);
    }
    out = inv ? -f : f;
    return c;
}
inline const char *skip_ws(const char *p)
{
    while (*p == ' ' || *p == '\t') ++p;
    return p;
}

struct Mtl {
    std::string name;
    float kd[3] = {0.6f, 0.6f, 0.6f}, ks[3] = {0, 0, 0}, ke[3] = {0, 0, 0};
    float d = 1.0f, ni = 1.0f, ns = 0.0f;
};
struct ObjMesh {
    int mtl = -2;  // -2: no material
    std::vector<int> v;   // 3 per face
    std::vector<int> vn;  // 3 per face (-1 = none)
    std::vector<int> vt;  // 3 per face (-1 = none)
};
struct ObjData {
    std::vector<float> v, vn, vt;   // vt: 2 per texture vertex (u, v)
    std::vector<Mtl> mats;
    std::vector<ObjMesh> meshes;
};

std::string dir_of(const std::string &path)
{
    const size_t s = path.find_last_of('/');
    return s == std::string::npos ? std::string() : path.substr(0, s + 1);
}
std::string rstrip(std::string s)
{
    while (!s.empty() && (s.back() == '\n' || s.back() == '\r' || s.back() == ' ' || s.back() == '\t')) s.pop_back();
    return s;
}

bool load_mtl(const std::string &path, ObjData &od)
{
    std::ifstream f(path);
    if (!f) return false;
    std::string line;
    Mtl *cur = nullptr;
    while (std::getline(f, line)) {
        line = rstrip(line);
        const char *p = skip_ws(line.c_str());
        if (!strncmp(p, "newmtl", 6)) {
            od.mats.emplace_back();
            cur = &od.mats.back();
            cur->name = skip_ws(p + 6);
            continue;
        }
        if (!cur) continue;
        float *dst = nullptr;
        int n = 1;
        const char *q = nullptr;
        if (p[0] == 'K' && (p[2] == ' ' || p[2] == '\t')) {
            if (p[1] == 'd') dst = cur->kd;
            else if (p[1] == 's') dst = cur->ks;
            else if (p[1] == 'e') dst = cur->ke;
            n = 3;
            q = p + 2;
        } else if (p[0] == 'd' && (p[1] == ' ' || p[1] == '\t')) {
            dst = &cur->d; q = p + 1;
        } else if (p[0] == 'N' && p[1] == 'i') {
            dst = &cur->ni; q = p + 2;
        } else if (p[0] == 'N' && p[1] == 's') {
            dst = &cur->ns; q = p + 2;
        } else if (p[0] == 'T' && p[1] == 'r') {
            float tr;
            parse_float(skip_ws(p + 2), tr);
            cur->d = 1.0f - tr;
            continue;
        }
        if (!dst) continue;
        for (int k = 0; k < n; ++k) q = parse_float(skip_ws(q), dst[k]);
    }
    return true;
}

inline void fdivs(float *v, float f)  // aiVector3t::operator/=
{
    if (f == 1.0f) return;
    const float inv = 1.0f / f;
    v[0] *= inv; v[1] *= inv; v[2] *= inv;
}

// TriangulateProcess: a quad is fanned from its concave vertex (or vertex 0)
int quad_start(const ObjData &od, const int *vi)
{
    for (int i = 0; i < 4; ++i) {
        const float *v0 = &od.v[3 * vi[(i + 3) % 4]], *v1 = &od.v[3 * vi[(i + 2) % 4]];
        const float *v2 = &od.v[3 * vi[(i + 1) % 4]], *v = &od.v[3 * vi[i]];
        float l[3] = {v0[0] - v[0], v0[1] - v[1], v0[2] - v[2]};
        float dg[3] = {v1[0] - v[0], v1[1] - v[1], v1[2] - v[2]};
        float r[3] = {v2[0] - v[0], v2[1] - v[1], v2[2] - v[2]};
        fdivs(l, std::sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]));
        fdivs(dg, std::sqrt(dg[0] * dg[0] + dg[1] * dg[1] + dg[2] * dg[2]));
        fdivs(r, std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]));
        const float angle = std::acos(l[0] * dg[0] + l[1] * dg[1] + l[2] * dg[2]) +
                            std::acos(r[0] * dg[0] + r[1] * dg[1] + r[2] * dg[2]);
        if (angle > (float)kPi) return i;
    }
    return 0;
}

bool parse_obj(const std::string &path, ObjData &od)
{
    std::ifstream f(path);
    if (!f) return false;
    std::string line, group;
    ObjMesh *cur = nullptr;
    int cur_mtl = -2;
    bool any_group = false;
    auto new_mesh = [&](int m) {
        od.meshes.emplace_back();
        od.meshes.back().mtl = m;
        return &od.meshes.back();
    };
    while (std::getline(f, line)) {
        const char *p = skip_ws(line.c_str());
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            const char *q = p + 1;
            for (int k = 0; k < 3; ++k) {
                float x;
                q = parse_float(skip_ws(q), x);
                od.v.push_back(x);
            }
        } else if (p[0] == 'v' && p[1] == 'n') {
            const char *q = p + 2;
            for (int k = 0; k < 3; ++k) {
                float x;
                q = parse_float(skip_ws(q), x);
                od.vn.push_back(x);
            }
        } else if (p[0] == 'v' && p[1] == 't') {
            const char *q = p + 2;
            for (int k = 0; k < 2; ++k) {       // u, v (Assimp keeps a third component; uv uses two)
                float x;
                q = parse_float(skip_ws(q), x);
                od.vt.push_back(x);
            }
        } else if (!strncmp(p, "mtllib", 6)) {
            load_mtl(dir_of(path) + rstrip(skip_ws(p + 6)), od);
        } else if ((p[0] == 'g' || p[0] == 'o') && (p[1] == ' ' || p[1] == '\t' || p[1] == 0 || p[1] == '\r')) {
            // ObjFileParser: a new group name starts a new object whose first mesh inherits the material
            const std::string nm = rstrip(skip_ws(p + 1));
            if (cur && any_group && nm == group) continue;
            group = nm;
            any_group = true;
            cur = new_mesh(cur_mtl);
        } else if (!strncmp(p, "usemtl", 6)) {
            const std::string nm = rstrip(skip_ws(p + 6));
            int idx = -1;
            for (size_t i = 0; i < od.mats.size(); ++i)
                if (od.mats[i].name == nm) idx = (int)i;
            if (idx < 0) {  // unknown: a named default material
                od.mats.emplace_back();
                od.mats.back().name = nm;
                idx = (int)od.mats.size() - 1;
            }
            if (idx == cur_mtl && cur) continue;
            cur_mtl = idx;
            if (!cur) {
                cur = new_mesh(cur_mtl);
                continue;
            }
            if (cur->mtl != -2 && cur->mtl != idx && !cur->v.empty()) cur = new_mesh(cur_mtl);  // needsNewMesh
            else cur->mtl = idx;
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            if (!cur) cur = new_mesh(cur_mtl);
            int vi[64], ni[64], ti[64], nv = 0;
            const char *q = p + 1;
            const int nverts = (int)(od.v.size() / 3), nnorm = (int)(od.vn.size() / 3), ntex = (int)(od.vt.size() / 2);
            while (*q && nv < 64) {
                q = skip_ws(q);
                if (!*q || *q == '\r' || *q == '\n') break;
                char *e;
                long a = strtol(q, &e, 10);
                q = e;
                long nn = 0, tt = 0;
                if (*q == '/') {
                    ++q;
                    if (*q != '/') { tt = strtol(q, &e, 10); q = e; }
                    if (*q == '/') { ++q; nn = strtol(q, &e, 10); q = e; }
                }
                while (*q && *q != ' ' && *q != '\t') ++q;
                vi[nv] = (int)(a < 0 ? nverts + a : a - 1);
                ni[nv] = nn == 0 ? -1 : (int)(nn < 0 ? nnorm + nn : nn - 1);
                ti[nv] = tt == 0 ? -1 : (int)(tt < 0 ? ntex + tt : tt - 1);
                ++nv;
            }
            auto push = [&](int a, int b, int c) {
                cur->v.insert(cur->v.end(), {vi[a], vi[b], vi[c]});
                cur->vn.insert(cur->vn.end(), {ni[a], ni[b], ni[c]});
                cur->vt.insert(cur->vt.end(), {ti[a], ti[b], ti[c]});
            };
            if (nv == 3) {
                push(0, 1, 2);
            } else if (nv == 4) {
                const int s = quad_start(od, vi);
                push(s, (s + 1) % 4, (s + 2) % 4);
                push(s, (s + 2) % 4, (s + 3) % 4);
            } else if (nv > 4) {
                for (int k = 1; k + 1 < nv; ++k) push(0, k, k + 1);
            }
        }
    }
    return true;
}

// GenVertexNormalsProcess, default 175 degree limit: every corner gets the
// normalised sum of the face normals of all corners within epsilon of it.
void smooth_normals(const ObjData &od, const ObjMesh &m, std::vector<float> &cn)
{
    const size_t nf = m.v.size() / 3, nc = m.v.size();
    std::vector<float> fn(3 * nf);
    float lo[3] = {1e30f, 1e30f, 1e30f}, hi[3] = {-1e30f, -1e30f, -1e30f};
    for (size_t f = 0; f < nf; ++f) {
        const float *a = &od.v[3 * m.v[3 * f]], *b = &od.v[3 * m.v[3 * f + 1]], *c = &od.v[3 * m.v[3 * f + 2]];
        const float e1[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
        const float e2[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
        float n[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]};
        const float l = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        if (l > 0.0f) fdivs(n, l);
        memcpy(&fn[3 * f], n, sizeof n);
        for (int k = 0; k < 3; ++k) {
            const float *v = &od.v[3 * m.v[3 * f + k]];
            for (int d = 0; d < 3; ++d) { lo[d] = std::min(lo[d], v[d]); hi[d] = std::max(hi[d], v[d]); }
        }
    }
    const float dd[3] = {hi[0] - lo[0], hi[1] - lo[1], hi[2] - lo[2]};
    const float eps = std::sqrt(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]) * 1e-4f;
    const float eps2 = eps * eps;
    // grid hashing with cell = eps (neighbour cells searched)
    const float cell = eps > 0.0f ? eps : 1.0f;
    auto key = [&](int64_t ix, int64_t iy, int64_t iz) {
        return (uint64_t)(ix * 73856093LL) ^ (uint64_t)(iy * 19349663LL) ^ (uint64_t)(iz * 83492791LL);
    };
    std::unordered_multimap<uint64_t, size_t> grid;
    grid.reserve(nc * 2);
    auto cell_of = [&](const float *v, int64_t *c3) {
        for (int d = 0; d < 3; ++d) c3[d] = (int64_t)std::floor((v[d] - lo[d]) / cell);
    };
    for (size_t i = 0; i < nc; ++i) {
        int64_t c3[3];
        cell_of(&od.v[3 * m.v[i]], c3);
        grid.emplace(key(c3[0], c3[1], c3[2]), i);
    }
    cn.assign(3 * nc, 0.0f);
    std::vector<size_t> found;
    for (size_t i = 0; i < nc; ++i) {
        const float *pi = &od.v[3 * m.v[i]];
        int64_t c3[3];
        cell_of(pi, c3);
        found.clear();
        for (int dx = -1; dx <= 1; ++dx)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dz = -1; dz <= 1; ++dz) {
                    auto r = grid.equal_range(key(c3[0] + dx, c3[1] + dy, c3[2] + dz));
                    for (auto it = r.first; it != r.second; ++it) {
                        const float *pj = &od.v[3 * m.v[it->second]];
                        const float d3[3] = {pj[0] - pi[0], pj[1] - pi[1], pj[2] - pi[2]};
                        if (d3[0] * d3[0] + d3[1] * d3[1] + d3[2] * d3[2] < eps2) found.push_back(it->second);
                    }
                }
        std::sort(found.begin(), found.end());
        found.erase(std::unique(found.begin(), found.end()), found.end());
        float acc[3] = {0, 0, 0};
        for (size_t j : found) {
            acc[0] += fn[3 * (j / 3)];
            acc[1] += fn[3 * (j / 3) + 1];
            acc[2] += fn[3 * (j / 3) + 2];
        }
        const float l = std::sqrt(acc[0] * acc[0] + acc[1] * acc[1] + acc[2] * acc[2]);
        if (l > 0.0f) fdivs(acc, l);
        memcpy(&cn[3 * i], acc, sizeof acc);
    }
}

inline double from_srgb(double v)  // util.h:62-66
{
    if (v <= 0.04045) return v * (1.0 / 12.92);
    return std::pow((v + 0.055) * (1.0 / 1.055), 2.4);
}

}  // namespace

// ---------------------------------------------------------------------------
// host scene
// ---------------------------------------------------------------------------
struct frt_host_scene {
    std::vector<double> tri_v, tri_n, tri_inv_area, tri_uv;
    std::vector<int32_t> tri_mat;
    std::vector<uint8_t> tri_geo;
    std::vector<double> sphere;
    std::vector<int32_t> sphere_mat;
    std::vector<frt_material> mats;
    std::vector<double> node_box;
    std::vector<int32_t> node_child;
    int32_t root = 0;
    int32_t world_kind = FRT_WORLD_BVH;
    std::vector<int32_t> list, lights;
    std::vector<int32_t> world;   // world prims in insertion order (frt_scene_add_*)
    double cam[7][3] = {};   // origin, llc, horizontal, vertical, u, v, w
    double lens_radius = 0, half_height = 0;
    double env[3] = {0, 0, 0};
    std::vector<frt_image> images;                    // data points into image_data
    std::vector<std::vector<uint8_t>> image_data;
    int bvh_depth = 0;
    double load_ms = 0, build_ms = 0;
    bool finished = true;    // false between frt_scene_new and frt_scene_finish

    int add_material(int type, V3 albedo, V3 emit, V3 specular = {}, double exponent = 0, double ior = 0)
    {
        frt_material m{};
        m.type = type;
        m.albedo[0] = albedo.x; m.albedo[1] = albedo.y; m.albedo[2] = albedo.z;
        m.emit[0] = emit.x; m.emit[1] = emit.y; m.emit[2] = emit.z;
        m.specular[0] = specular.x; m.specular[1] = specular.y; m.specular[2] = specular.z;
        m.exponent = exponent;
        m.ior = ior;
        mats.push_back(m);
        return (int)mats.size() - 1;
    }
    int add_sphere(V3 c, double r, int mat)
    {
        sphere.insert(sphere.end(), {c.x, c.y, c.z, r});
        sphere_mat.push_back(mat);
        return (int)sphere_mat.size() - 1;
    }
    void set_camera(V3 lookfrom, V3 lookat, V3 vup, double vfov, double aspect, double aperture, double focus)
    {
        // camera.h:10-28 (fp64, same operation order)
        lens_radius = aperture / 2;
        const double theta = vfov * kPi / 180.0;
        const double hh = std::tan(theta / 2);
        const double hw = aspect * hh;
        const V3 w = unit(lookfrom - lookat);
        const V3 u = unit(cross(vup, w));
        const V3 v = cross(w, u);
        const V3 llc = ((lookfrom - (hw * focus) * u) - (hh * focus) * v) - focus * w;
        const V3 h = (2 * hw * focus) * u;
        const V3 vv = (2 * hh * focus) * v;
        const V3 all[7] = {lookfrom, llc, h, vv, u, v, w};
        for (int i = 0; i < 7; ++i) { cam[i][0] = all[i].x; cam[i][1] = all[i].y; cam[i][2] = all[i].z; }
        half_height = hh;
    }
};

namespace {

// Matrix4x4 (geometry.h:919-1065), row-major double[16]: point transform with
// the w divide (:966-983), Gauss-Jordan inverse with full pivoting
// (Matrix::invert, :857-907), normal_transform = inverse-transpose product (:830-838)
V3 mat4_point(const double *m, const double *v)
{
    const double x = m[0] * v[0] + m[1] * v[1] + m[2] * v[2] + m[3];
    const double y = m[4] * v[0] + m[5] * v[1] + m[6] * v[2] + m[7];
    const double z = m[8] * v[0] + m[9] * v[1] + m[10] * v[2] + m[11];
    const double w = m[12] * v[0] + m[13] * v[1] + m[14] * v[2] + m[15];
    if (w == 1.0) return {x, y, z};
    return {x / w, y / w, z / w};
}
V3 mat4_normal(const double *inv, const double *v)
{
    return {inv[0] * v[0] + inv[4] * v[1] + inv[8] * v[2], inv[1] * v[0] + inv[5] * v[1] + inv[9] * v[2],
            inv[2] * v[0] + inv[6] * v[1] + inv[10] * v[2]};
}
bool mat4_invert(const double *src, double *t)
{
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    memcpy(t, src, 16 * sizeof(double));
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        double big = 0;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] == 1) continue;
            for (int k = 0; k < 4; k++) {
                if (ipiv[k] == 0) {
                    if (std::fabs(t[4 * j + k]) >= big) { big = std::fabs(t[4 * j + k]); irow = j; icol = k; }
                } else if (ipiv[k] > 1) {
                    return false;
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(t[4 * irow + k], t[4 * icol + k]);
        indxr[i] = irow;
        indxc[i] = icol;
        if (t[4 * icol + icol] == 0) return false;
        const double pivinv = 1.0 / t[4 * icol + icol];
        t[4 * icol + icol] = 1.0;
        for (int j = 0; j < 4; j++) t[4 * icol + j] *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j == icol) continue;
            const double save = t[4 * j + icol];
            t[4 * j + icol] = 0;
            for (int k = 0; k < 4; k++) t[4 * j + k] -= t[4 * icol + k] * save;
        }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) std::swap(t[4 * k + indxr[j]], t[4 * k + indxc[j]]);
    return true;
}

// mesh_loader::load_obj + create_triangle_mesh (triangle.cpp:9-23), and its
// (file, toWorld, bsdf) overload (triangle.cpp:26-60): every mesh of the file
// takes `bsdf` when given (one material object for all of them), vertices go
// through toWorld and normals through its inverse transpose.  Emissive meshes
// join Scene::lights.  Returns FRT_OK, FRT_E_IO or FRT_E_INVALID (singular matrix).
int add_obj(frt_host_scene &s, const std::string &path, bool geo, const double *to_world = nullptr,
            const frt_material *bsdf = nullptr)
{
    double inv[16];
    if (to_world && !mat4_invert(to_world, inv)) return FRT_E_INVALID;
    ObjData od;
    if (!parse_obj(path, od)) return FRT_E_IO;
    int shared_mat = -1;
    for (const ObjMesh &m : od.meshes) {
        const size_t nf = m.v.size() / 3;
        if (nf == 0) continue;  // Assimp drops empty meshes
        const Mtl *mt = (m.mtl >= 0) ? &od.mats[m.mtl] : nullptr;
        int type;
        V3 albedo, emit, spec;
        double exponent = 0, ior = 0;
        if (!mt) {  // DefaultMaterial -> lambertian 0.5 (mesh_loader.cpp:107-111)
            type = FRT_MAT_LAMBERTIAN;
            albedo = {0.5, 0.5, 0.5};
        } else if (mt->ke[0] != 0 || mt->ke[1] != 0 || mt->ke[2] != 0) {
            type = FRT_MAT_DIFFUSE_LIGHT;
            emit = {mt->ke[0], mt->ke[1], mt->ke[2]};
        } else if (mt->ks[0] != 0 || mt->ks[1] != 0 || mt->ks[2] != 0) {
            // opacity < 1: dielectric(Ni, FromSrgb(Ks), 1); else modified_phong(FromSrgb(Kd), FromSrgb(Ks), Ns)
            // (mesh_loader.cpp:78-100)
            type = (mt->d < 1.0f) ? FRT_MAT_DIELECTRIC : FRT_MAT_MODIFIED_PHONG;
            albedo = {from_srgb(mt->kd[0]), from_srgb(mt->kd[1]), from_srgb(mt->kd[2])};
            spec = {from_srgb(mt->ks[0]), from_srgb(mt->ks[1]), from_srgb(mt->ks[2])};
            exponent = mt->ns;
            ior = mt->ni;
        } else {
            type = FRT_MAT_LAMBERTIAN;
            albedo = {from_srgb(mt->kd[0]), from_srgb(mt->kd[1]), from_srgb(mt->kd[2])};
        }
        int mat;
        if (bsdf) {                                   // mesh->mat.reset(bsdf)
            if (shared_mat < 0) {
                s.mats.push_back(*bsdf);
                shared_mat = (int)s.mats.size() - 1;
            }
            mat = shared_mat;
            type = bsdf->type;
        } else {
            mat = s.add_material(type, albedo, emit, spec, exponent, ior);
        }
        bool has_vn = true;
        for (int x : m.vn) if (x < 0) { has_vn = false; break; }
        std::vector<float> cn;
        if (has_vn) {
            cn.resize(3 * m.vn.size());
            for (size_t i = 0; i < m.vn.size(); ++i) memcpy(&cn[3 * i], &od.vn[3 * m.vn[i]], 3 * sizeof(float));
        } else if (!geo) {
            smooth_normals(od, m, cn);
        } else {
            cn.assign(3 * m.v.size(), 0.0f);
        }
        // texture coordinates (mesh_loader.cpp:34-38) when every corner has a vt;
        // without them the reference leaves uv uninitialised -- here 0
        bool has_vt = !od.vt.empty();
        for (int x : m.vt) if (x < 0 || 2 * (size_t)x + 1 >= od.vt.size()) { has_vt = false; break; }
        const int base = (int)s.tri_mat.size();
        for (size_t f = 0; f < nf; ++f) {
            for (int k = 0; k < 3; ++k)
                for (int d = 0; d < 2; ++d) s.tri_uv.push_back(has_vt ? (double)od.vt[2 * m.vt[3 * f + k] + d] : 0.0);
            double v[9], n[9];
            for (int k = 0; k < 3; ++k)
                for (int d = 0; d < 3; ++d) {
                    v[3 * k + d] = od.v[3 * m.v[3 * f + k] + d];
                    n[3 * k + d] = cn[3 * (3 * f + k) + d];
                }
            if (to_world) {
                for (int k = 0; k < 3; ++k) {
                    const V3 pv = mat4_point(to_world, v + 3 * k), nv = mat4_normal(inv, n + 3 * k);
                    v[3 * k] = pv.x; v[3 * k + 1] = pv.y; v[3 * k + 2] = pv.z;
                    n[3 * k] = nv.x; n[3 * k + 1] = nv.y; n[3 * k + 2] = nv.z;
                }
            }
            s.tri_v.insert(s.tri_v.end(), v, v + 9);
            s.tri_n.insert(s.tri_n.end(), n, n + 9);
            const V3 e1{v[3] - v[0], v[4] - v[1], v[5] - v[2]}, e2{v[6] - v[0], v[7] - v[1], v[8] - v[2]};
            s.tri_inv_area.push_back(1 / (0.5 * length(cross(e1, e2)) * (double)nf));  // triangle.h:65
            s.tri_mat.push_back(mat);
            s.tri_geo.push_back(geo ? 1 : 0);
            if (type == FRT_MAT_DIFFUSE_LIGHT) s.lights.push_back(base + (int)f);
            s.world.push_back(base + (int)f);
        }
    }
    return FRT_OK;
}

// ---------------------------------------------------------------------------
// parallel_bvh_node construction (parallel_bvh.h:67-160)
// ---------------------------------------------------------------------------
struct Box {
    double lo[3], hi[3];
};
inline double box_area(const Box &b)  // aabb.h:46-49 (size = max - min)
{
    const double sx = b.hi[0] - b.lo[0], sy = b.hi[1] - b.lo[1], sz = b.hi[2] - b.lo[2];
    return 2 * ((sx * sy) + (sy * sz) + (sx * sz));
}
inline Box surround(const Box &a, const Box &b)  // aabb.h:57-68
{
    Box r;
    for (int k = 0; k < 3; ++k) { r.lo[k] = std::fmin(a.lo[k], b.lo[k]); r.hi[k] = std::fmax(a.hi[k], b.hi[k]); }
    return r;
}
inline int longest_axis(const Box &b)  // aabb.h:33-43
{
    const double sx = b.hi[0] - b.lo[0], sy = b.hi[1] - b.lo[1], sz = b.hi[2] - b.lo[2];
    if (sy > sx) return 1;
    if (sz > sx) return 2;
    return 0;
}

struct Builder {
    const std::vector<Box> &pbox;          // per primitive-ref slot
    std::vector<double> node_box;
    std::vector<int32_t> node_child;
    std::atomic<int> n_nodes{0};
    std::atomic<int> max_depth{0};
    std::vector<int32_t> refs;             // slot -> prim ref

    explicit Builder(const std::vector<Box> &b) : pbox(b) {}

    // glibc msort_with_tmp (stdlib/msort.c) with the bvh.h comparator:
    // cmp(a,b) = (key[a] - key[b] < 0) ? -1 : 1; "<= 0" takes from the left run.
    static void msort(int32_t *b, size_t n, int32_t *tmp, const Box *boxes, int axis)
    {
        if (n <= 1) return;
        const size_t n1 = n / 2, n2 = n - n1;
        int32_t *b1 = b, *b2 = b + n1;
        msort(b1, n1, tmp, boxes, axis);
        msort(b2, n2, tmp, boxes, axis);
        size_t i = n1, j = n2;
        int32_t *t = tmp;
        while (i > 0 && j > 0) {
            if (boxes[*b1].lo[axis] - boxes[*b2].lo[axis] < 0.0) { *t++ = *b1++; --i; }
            else { *t++ = *b2++; --j; }
        }
        if (i > 0) memcpy(t, b1, i * sizeof(int32_t));
        memcpy(b, tmp, (n - j) * sizeof(int32_t));
    }

    int32_t build(int32_t *l, int n, int depth)
    {
        int md = max_depth.load();
        while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
        const int me = n_nodes.fetch_add(1);
        const Box *B = pbox.data();
        Box main_box = B[l[0]];
        for (int i = 1; i < n; ++i) main_box = surround(B[l[i]], main_box);
        const int axis = longest_axis(main_box);
        std::vector<int32_t> tmp(n);
        msort(l, (size_t)n, tmp.data(), B, axis);
        std::vector<double> left_area(n), right_area(n);
        left_area[0] = box_area(B[l[0]]);
        Box lb = B[l[0]];
        for (int i = 1; i < n - 1; ++i) { lb = surround(lb, B[l[i]]); left_area[i] = box_area(lb); }
        right_area[n - 1] = box_area(B[l[n - 1]]);
        Box rb = B[l[n - 1]];
        for (int i = n - 2; i > 0; --i) { rb = surround(rb, B[l[i]]); right_area[i] = box_area(rb); }
        double min_sah = 3.40282346638528859812e+38;  // FLT_MAX
        int idx = 0;
        for (int i = 0; i < n - 1; ++i) {
            const double sah = i * left_area[i] + (n - i - 1) * right_area[i + 1];
            if (sah < min_sah) { idx = i; min_sah = sah; }
        }
        tmp.clear(); tmp.shrink_to_fit();
        left_area.clear(); left_area.shrink_to_fit();
        right_area.clear(); right_area.shrink_to_fit();
        int32_t left = 0, right = 0;
        auto do_left = [&] { left = (idx == 0) ? ~l[0] : build(l, idx + 1, depth + 1); };
        auto do_right = [&] { right = (idx == n - 2) ? ~l[idx + 1] : build(l + idx + 1, n - idx - 1, depth + 1); };
        if (n > 65536 && depth < 6) {  // large subtrees on their own thread (taskflow subflows in the reference)
            std::thread th(do_left);
            do_right();
            th.join();
        } else {
            do_left();
            do_right();
        }
        for (int k = 0; k < 3; ++k) { node_box[6 * me + k] = main_box.lo[k]; node_box[6 * me + 3 + k] = main_box.hi[k]; }
        node_child[2 * me] = left;
        node_child[2 * me + 1] = right;
        return me;
    }
};

// leaves hold the slot index; map slots back to prim refs afterwards
void build_bvh(frt_host_scene &s, const std::vector<int32_t> &prims)
{
    const int n = (int)prims.size();
    std::vector<Box> boxes(n);
    for (int i = 0; i < n; ++i) {
        const int ref = prims[i];
        Box &b = boxes[i];
        if (ref & FRT_PRIM_SPHERE) {
            const double *sp = &s.sphere[4 * (ref & ~FRT_PRIM_SPHERE)];
            for (int k = 0; k < 3; ++k) { b.lo[k] = sp[k] - sp[3]; b.hi[k] = sp[k] + sp[3]; }
        } else {
            const double *v = &s.tri_v[9 * ref];
            for (int k = 0; k < 3; ++k) {  // triangle.h:120-137
                b.lo[k] = std::fmin(std::fmin(v[k], v[3 + k]), v[6 + k]);
                b.hi[k] = std::fmax(std::fmax(v[k], v[3 + k]), v[6 + k]);
            }
        }
    }
    s.node_box.clear();
    s.node_child.clear();
    if (n == 0) { s.root = 0; return; }
    if (n == 1) { s.root = ~prims[0]; s.bvh_depth = 0; return; }
    Builder b(boxes);
    b.node_box.assign(6 * (size_t)(n - 1), 0.0);
    b.node_child.assign(2 * (size_t)(n - 1), 0);
    std::vector<int32_t> slots(n);
    for (int i = 0; i < n; ++i) slots[i] = i;
    const int root = b.build(slots.data(), n, 1);
    for (auto &c : b.node_child)
        if (c < 0) c = ~prims[~c];
    s.node_box = std::move(b.node_box);
    s.node_child = std::move(b.node_child);
    s.root = root;
    s.bvh_depth = b.max_depth.load();
}


// ---------------------------------------------------------------------------
// Binned SAH builder (frt_scene_build_bvh_sah): 32 centroid bins on each axis,
// cost N_L A_L + N_R A_R, single-primitive leaves (the upload collapses
// subtrees of <= 4 triangles).  A higher-quality tree than both the
// reference's sweep (sorted by box minimum) and the GPU LBVH, at host cost.
// ---------------------------------------------------------------------------
struct SahBuilder {
    const std::vector<Box> &box;
    std::vector<double> cen;                 // 3 per prim slot
    std::vector<int32_t> idx;                // prim slots, partitioned in place
    std::vector<double> node_box;
    std::vector<int32_t> node_child;
    std::atomic<int> n_nodes{0}, max_depth{0};
    // centroid bins per axis: 32 (8-128 measured 1-2 % apart on the GPU,
    // profiles/r01d_ab_sah_bins.txt).  A build-time constant, so no stray
    // environment can change the tree (and with it which of two exactly tied
    // hits a ray reports); experiment builds set FRT_EXP_SAH_BINS.
#ifndef FRT_EXP_SAH_BINS
#define FRT_EXP_SAH_BINS 32
#endif
    static constexpr int kMaxBins = FRT_EXP_SAH_BINS;
    static constexpr int bins = FRT_EXP_SAH_BINS;

    explicit SahBuilder(const std::vector<Box> &b) : box(b), cen(3 * b.size()), idx(b.size())
    {
        for (size_t i = 0; i < b.size(); ++i) {
            idx[i] = (int32_t)i;
            for (int k = 0; k < 3; ++k) cen[3 * i + k] = 0.5 * (b[i].lo[k] + b[i].hi[k]);
        }
        node_box.assign(6 * (b.size() - 1), 0.0);
        node_child.assign(2 * (b.size() - 1), 0);
    }
    // node over idx[b, e); returns its index (nodes numbered in creation order)
    int32_t build(int b, int e, int depth)
    {
        int md = max_depth.load();
        while (depth > md && !max_depth.compare_exchange_weak(md, depth)) {}
        const int me = n_nodes.fetch_add(1);
        Box nb = box[idx[b]];
        double clo[3], chi[3];
        for (int k = 0; k < 3; ++k) clo[k] = chi[k] = cen[3 * idx[b] + k];
        for (int i = b + 1; i < e; ++i) {
            nb = surround(nb, box[idx[i]]);
            for (int k = 0; k < 3; ++k) {
                clo[k] = std::fmin(clo[k], cen[3 * idx[i] + k]);
                chi[k] = std::fmax(chi[k], cen[3 * idx[i] + k]);
            }
        }
        const int n = e - b;
        int mid = b + n / 2;
        if (n > 2) {
            const int kBins = bins;
            double best = INFINITY;
            int best_axis = -1, best_bin = 0;
            for (int axis = 0; axis < 3; ++axis) {
                const double ext = chi[axis] - clo[axis];
                if (!(ext > 0)) continue;
                Box bb[kMaxBins];
                int cnt[kMaxBins] = {};
                const double sc = kBins / ext;
                for (int i = b; i < e; ++i) {
                    const int bi = std::min(kBins - 1, (int)((cen[3 * idx[i] + axis] - clo[axis]) * sc));
                    bb[bi] = cnt[bi]++ ? surround(bb[bi], box[idx[i]]) : box[idx[i]];
                }
                double right_area[kMaxBins];
                int right_cnt[kMaxBins];
                Box acc{};
                int c = 0;
                for (int i = kBins - 1; i > 0; --i) {
                    if (cnt[i]) { acc = c ? surround(acc, bb[i]) : bb[i]; c += cnt[i]; }
                    right_area[i] = c ? box_area(acc) : 0.0;
                    right_cnt[i] = c;
                }
                c = 0;
                for (int i = 0; i < kBins - 1; ++i) {
                    if (cnt[i]) { acc = c ? surround(acc, bb[i]) : bb[i]; c += cnt[i]; }
                    if (c == 0 || right_cnt[i + 1] == 0) continue;
                    const double cost = c * box_area(acc) + right_cnt[i + 1] * right_area[i + 1];
                    if (cost < best) { best = cost; best_axis = axis; best_bin = i; }
                }
            }
            if (best_axis >= 0) {
                const double sc = kBins / (chi[best_axis] - clo[best_axis]);
                int32_t *m = std::partition(idx.data() + b, idx.data() + e, [&](int32_t p) {
                    return std::min(kBins - 1, (int)((cen[3 * p + best_axis] - clo[best_axis]) * sc)) <= best_bin;
                });
                mid = (int)(m - idx.data());
            }
            if (mid == b || mid == e) mid = b + n / 2;     // all centroids in one bin: median split
        }
        int32_t left = 0, right = 0;
        auto do_left = [&] { left = (mid - b == 1) ? ~idx[b] : build(b, mid, depth + 1); };
        auto do_right = [&] { right = (e - mid == 1) ? ~idx[mid] : build(mid, e, depth + 1); };
        if (n > 65536 && depth < 6) {
            std::thread th(do_left);
            do_right();
            th.join();
        } else {
            do_left();
            do_right();
        }
        for (int k = 0; k < 3; ++k) { node_box[6 * me + k] = nb.lo[k]; node_box[6 * me + 3 + k] = nb.hi[k]; }
        node_child[2 * me] = left;
        node_child[2 * me + 1] = right;
        return me;
    }
};

}  // namespace

extern "C" int frt_scene_create(const char *kind, const char *obj_path, double aspect, frt_host_scene **out)
{
    if (!kind || !obj_path || !out) return FRT_E_INVALID;
    *out = nullptr;
    auto s = std::make_unique<frt_host_scene>();
    const std::string k = kind;
    const auto t0 = std::chrono::steady_clock::now();
    if (k == "cornell_box_obj" || k == "obj_geo" || k == "obj_smooth") {
        if (const int rc = add_obj(*s, obj_path, k != "obj_smooth")) return rc;
        s->world_kind = FRT_WORLD_BVH;
        s->set_camera({0, 1, (double)3.9f}, {0, 1, 0}, {0, 1, 0}, 40.0, aspect, 0.0, 10.0);  // main.cpp:236-242
    } else if (k == "veach_mis") {
        if (const int rc = add_obj(*s, obj_path, false)) return rc;
        // main.cpp:292-302: five emissive spheres in the world list, and five
        // separate identical sphere objects in Scene::lights
        const double cx[5] = {10, (double)-1.25f, (double)-3.75f, (double)1.25f, (double)3.75f};
        const double cy[5] = {10, 0, 0, 0, 0}, cz[5] = {4, 0, 0, 0, 0};
        const double rad[5] = {0.5, (double)0.1f, (double)0.03333f, (double)0.3f, (double)0.9f};
        const double em[5] = {800, 100, (double)901.803f, (double)11.1111f, 1.23457};
        s->world_kind = FRT_WORLD_LIST;
        for (int i = 0; i < (int)s->tri_mat.size(); ++i) s->list.push_back(i);
        std::vector<int32_t> light_refs;
        for (int j = 0; j < 5; ++j) {
            const int m = s->add_material(FRT_MAT_DIFFUSE_LIGHT, {}, {em[j], em[j], em[j]});
            s->list.push_back(FRT_PRIM_SPHERE | s->add_sphere({cx[j], cy[j], cz[j]}, rad[j], m));
        }
        for (int j = 0; j < 5; ++j) {
            const int m = s->add_material(FRT_MAT_DIFFUSE_LIGHT, {}, {em[j], em[j], em[j]});
            s->lights.push_back(FRT_PRIM_SPHERE | s->add_sphere({cx[j], cy[j], cz[j]}, rad[j], m));
        }
        s->set_camera({0, 2, 15}, {0, -2, 2.5}, {0, 1, 0}, 28.0, aspect, 0.0, 50.0);
    } else {
        return FRT_E_INVALID;
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (s->world_kind == FRT_WORLD_BVH) {
        std::vector<int32_t> prims(s->tri_mat.size());
        for (size_t i = 0; i < prims.size(); ++i) prims[i] = (int32_t)i;
        build_bvh(*s, prims);
    }
    const auto t2 = std::chrono::steady_clock::now();
    s->load_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    s->build_ms = std::chrono::duration<double, std::milli>(t2 - t1).count();
    *out = s.release();
    return FRT_OK;
}

// ---- incremental construction (what main.cpp's scene functions do) ----
extern "C" int frt_scene_new(frt_host_scene **out)
{
    if (!out) return FRT_E_INVALID;
    *out = new (std::nothrow) frt_host_scene();
    if (!*out) return FRT_E_INVALID;
    (*out)->finished = false;
    return FRT_OK;
}

static bool material_ok(const frt_material *m, const frt_host_scene *s = nullptr)
{
    if (!m) return false;
    if (m->texture == FRT_TEX_IMAGE) {
        if (m->image < 0 || (s && m->image >= (int)s->images.size())) return false;
    } else if (m->texture != FRT_TEX_CONSTANT && m->texture != FRT_TEX_CHECKER) {
        return false;
    }
    switch (m->type) {
    case FRT_MAT_LAMBERTIAN: case FRT_MAT_DIFFUSE_LIGHT: case FRT_MAT_MODIFIED_PHONG: case FRT_MAT_METAL:
    case FRT_MAT_DIELECTRIC: return true;
    case FRT_MAT_ROUGH_CONDUCTOR:
        return m->alpha > 0.0 && (m->distribution == FRT_DIST_GGX || m->distribution == FRT_DIST_BECKMANN);
    default: return false;
    }
}

extern "C" int frt_scene_add_obj(frt_host_scene *s, const char *obj_path, const double *to_world16,
                                 const frt_material *bsdf, int use_geometry_normals)
{
    if (!s || !obj_path || s->finished || (bsdf && !material_ok(bsdf, s))) return FRT_E_INVALID;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = add_obj(*s, obj_path, use_geometry_normals != 0, to_world16, bsdf);
    s->load_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

extern "C" int frt_scene_add_sphere(frt_host_scene *s, const double *center, double radius, const frt_material *m,
                                    int where)
{
    if (!s || !center || s->finished || !material_ok(m, s) || !(where & FRT_SPHERE_BOTH)) return FRT_E_INVALID;
    s->mats.push_back(*m);
    const int id = s->add_sphere({center[0], center[1], center[2]}, radius, (int)s->mats.size() - 1);
    if (where & FRT_SPHERE_WORLD) s->world.push_back(FRT_PRIM_SPHERE | id);
    if (where & FRT_SPHERE_LIGHTS) s->lights.push_back(FRT_PRIM_SPHERE | id);
    return FRT_OK;
}

extern "C" int frt_scene_set_camera(frt_host_scene *s, const double *lookfrom, const double *lookat, const double *vup,
                                    double vfov, double aspect, double aperture, double focus_dist)
{
    if (!s || !lookfrom || !lookat || !vup) return FRT_E_INVALID;
    s->set_camera({lookfrom[0], lookfrom[1], lookfrom[2]}, {lookat[0], lookat[1], lookat[2]}, {vup[0], vup[1], vup[2]},
                  vfov, aspect, aperture, focus_dist);
    return FRT_OK;
}

extern "C" int frt_scene_set_env(frt_host_scene *s, const double *rgb)
{
    if (!s || !rgb) return FRT_E_INVALID;
    for (int k = 0; k < 3; ++k) s->env[k] = rgb[k];
    return FRT_OK;
}

// image_texture's image (texture.h:51-95), copied: stb's decoded rows as given
extern "C" int frt_scene_add_image(frt_host_scene *s, const frt_image *img, int *index)
{
    if (!s || !img || !index || s->finished || img->nx <= 0 || img->ny <= 0 || !img->data ||
        (img->format != FRT_IMAGE_SRGB8 && img->format != FRT_IMAGE_F32))
        return FRT_E_INVALID;
    const size_t n = (size_t)img->nx * img->ny * 3 * (img->format == FRT_IMAGE_F32 ? sizeof(float) : 1);
    const uint8_t *src = static_cast<const uint8_t *>(img->data);
    s->image_data.emplace_back(src, src + n);
    frt_image c = *img;
    c.data = s->image_data.back().data();
    s->images.push_back(c);
    *index = (int)s->images.size() - 1;
    return FRT_OK;
}

extern "C" int frt_scene_finish(frt_host_scene *s, int world_kind)
{
    if (!s || s->finished || (world_kind != FRT_WORLD_BVH && world_kind != FRT_WORLD_LIST) || s->world.empty())
        return FRT_E_INVALID;
    const auto t0 = std::chrono::steady_clock::now();
    s->world_kind = world_kind;
    if (world_kind == FRT_WORLD_BVH) build_bvh(*s, s->world);
    else s->list = s->world;
    s->finished = true;
    s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return FRT_OK;
}

extern "C" int frt_scene_build_bvh_sah(frt_host_scene *s)
{
    if (!s || !s->finished) return FRT_E_INVALID;
    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<int32_t> prims = (s->world_kind == FRT_WORLD_LIST) ? s->list : s->world;
    const int n = (int)prims.size();
    if (n == 0) return FRT_E_INVALID;
    if (n == 1) {
        s->node_box.clear(); s->node_child.clear(); s->root = ~prims[0]; s->bvh_depth = 0;
    } else {
        std::vector<Box> boxes(n);
        for (int i = 0; i < n; ++i) {
            const int ref = prims[i];
            Box &b = boxes[i];
            if (ref & FRT_PRIM_SPHERE) {
                const double *sp = &s->sphere[4 * (ref & ~FRT_PRIM_SPHERE)];
                for (int k = 0; k < 3; ++k) { b.lo[k] = sp[k] - sp[3]; b.hi[k] = sp[k] + sp[3]; }
            } else {
                const double *v = &s->tri_v[9 * ref];
                for (int k = 0; k < 3; ++k) {
                    b.lo[k] = std::fmin(std::fmin(v[k], v[3 + k]), v[6 + k]);
                    b.hi[k] = std::fmax(std::fmax(v[k], v[3 + k]), v[6 + k]);
                }
            }
        }
        SahBuilder B(boxes);
        const int root = B.build(0, n, 1);
        for (auto &c : B.node_child)
            if (c < 0) c = ~prims[~c];
        s->node_box = std::move(B.node_box);
        s->node_child = std::move(B.node_child);
        s->root = root;
        s->bvh_depth = B.max_depth.load();
    }
    s->world_kind = FRT_WORLD_BVH;
    s->list.clear();
    s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return FRT_OK;
}

// ---- GPU BVH build (frt_lbvh.hip through the context's device) ----
extern "C" int frt_internal_lbvh(frt_ctx *c, int n, const float *box6, int32_t *child2, float *node_box6,
                                 int32_t *order, double *ms, int algo);

static inline float f_down(double x)
{
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
}
static inline float f_up(double x)
{
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}

extern "C" int frt_scene_build_bvh_gpu(frt_host_scene *s, frt_ctx *ctx, double *device_ms)
{
    return frt_scene_build_bvh_gpu_algo(s, ctx, FRT_GPU_BVH_SAH, device_ms);
}

extern "C" int frt_scene_build_bvh_gpu_algo(frt_host_scene *s, frt_ctx *ctx, int algo, double *device_ms)
{
    if (!s || !ctx || !s->finished) return FRT_E_INVALID;
    const auto t0 = std::chrono::steady_clock::now();
    const std::vector<int32_t> prims = (s->world_kind == FRT_WORLD_LIST) ? s->list : s->world;
    const int n = (int)prims.size();
    if (n == 0) return FRT_E_INVALID;
    std::vector<double> nbox;
    std::vector<int32_t> nchild;
    int32_t root = 0;
    double ms = 0.0;
    if (n == 1) {
        root = ~prims[0];
    } else {
        // fp32 boxes rounded outward: they contain the fp64 primitives, so the
        // tree's boxes do too (flatten_scene pads them again for the fp32 rays)
        std::vector<float> box6(6 * (size_t)n);
        for (int i = 0; i < n; ++i) {
            const int ref = prims[i];
            double lo[3], hi[3];
            if (ref & FRT_PRIM_SPHERE) {
                const double *q = &s->sphere[4 * (ref & ~FRT_PRIM_SPHERE)];
                for (int k = 0; k < 3; ++k) { lo[k] = q[k] - q[3]; hi[k] = q[k] + q[3]; }
            } else {
                const double *v = &s->tri_v[9 * ref];
                for (int k = 0; k < 3; ++k) {
                    lo[k] = std::fmin(std::fmin(v[k], v[3 + k]), v[6 + k]);
                    hi[k] = std::fmax(std::fmax(v[k], v[3 + k]), v[6 + k]);
                }
            }
            for (int k = 0; k < 3; ++k) { box6[6 * i + k] = f_down(lo[k]); box6[6 * i + 3 + k] = f_up(hi[k]); }
        }
        std::vector<int32_t> child2(2 * (size_t)(n - 1)), order(n);
        std::vector<float> nb6(6 * (size_t)(n - 1));
        const int rc = frt_internal_lbvh(ctx, n, box6.data(), child2.data(), nb6.data(), order.data(), &ms, algo);
        if (rc != FRT_OK) return rc;
        nbox.assign(nb6.begin(), nb6.end());
        nchild.resize(child2.size());
        for (size_t i = 0; i < child2.size(); ++i) {
            const int c = child2[i];
            if (c < 0 && (~c >= n || order[~c] < 0 || order[~c] >= n)) return FRT_E_HIP;
            if (c >= n - 1) return FRT_E_HIP;
            nchild[i] = c >= 0 ? c : ~prims[order[~c]];
        }
    }
    // depth of the new tree (levels of interior nodes on the longest path)
    int depth = 0;
    if (root >= 0 && !nchild.empty()) {
        std::vector<std::pair<int, int>> st{{0, 1}};
        size_t visited = 0;
        while (!st.empty()) {
            const auto [node, d] = st.back();
            st.pop_back();
            if (++visited > nchild.size()) return FRT_E_HIP;   // not a tree
            depth = std::max(depth, d);
            for (int side = 0; side < 2; ++side)
                if (nchild[2 * node + side] >= 0) st.push_back({nchild[2 * node + side], d + 1});
        }
    }
    s->node_box = std::move(nbox);
    s->node_child = std::move(nchild);
    s->root = root;
    s->bvh_depth = depth;
    s->world_kind = FRT_WORLD_BVH;
    s->list.clear();
    s->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (device_ms) *device_ms = ms;
    return FRT_OK;
}

extern "C" int frt_scene_view_get(const frt_host_scene *s, frt_scene_view *v)
{
    if (!s || !v || !s->finished) return FRT_E_INVALID;
    memset(v, 0, sizeof(*v));
    v->world_kind = s->world_kind;
    v->n_tris = (int32_t)s->tri_mat.size();
    v->tri_v = s->tri_v.data();
    v->tri_n = s->tri_n.data();
    v->tri_material = s->tri_mat.data();
    v->tri_geometry_normal = s->tri_geo.data();
    v->tri_inv_area = s->tri_inv_area.data();
    v->tri_uv = s->tri_uv.empty() ? nullptr : s->tri_uv.data();
    v->n_spheres = (int32_t)s->sphere_mat.size();
    v->sphere = s->sphere.data();
    v->sphere_material = s->sphere_mat.data();
    v->n_materials = (int32_t)s->mats.size();
    v->materials = s->mats.data();
    v->n_nodes = (int32_t)(s->node_child.size() / 2);
    v->root = s->root;
    v->node_box = s->node_box.data();
    v->node_child = s->node_child.data();
    v->n_list = (int32_t)s->list.size();
    v->list = s->list.data();
    v->n_lights = (int32_t)s->lights.size();
    v->lights = s->lights.data();
    for (int k = 0; k < 3; ++k) {
        v->cam_origin[k] = s->cam[0][k];
        v->cam_lower_left[k] = s->cam[1][k];
        v->cam_horizontal[k] = s->cam[2][k];
        v->cam_vertical[k] = s->cam[3][k];
        v->cam_u[k] = s->cam[4][k];
        v->cam_v[k] = s->cam[5][k];
        v->cam_w[k] = s->cam[6][k];
        v->env_color[k] = s->env[k];
    }
    v->cam_lens_radius = s->lens_radius;
    v->cam_half_height = s->half_height;
    v->n_images = (int32_t)s->images.size();
    v->images = s->images.empty() ? nullptr : s->images.data();
    return FRT_OK;
}

extern "C" int frt_scene_info(const frt_host_scene *s, frt_host_scene_info *info)
{
    if (!s || !info) return FRT_E_INVALID;
    info->n_tris = (int32_t)s->tri_mat.size();
    info->n_spheres = (int32_t)s->sphere_mat.size();
    info->n_materials = (int32_t)s->mats.size();
    info->n_lights = (int32_t)s->lights.size();
    info->n_nodes = (int32_t)(s->node_child.size() / 2);
    info->world_kind = s->world_kind;
    info->n_list = (int32_t)s->list.size();
    info->bvh_depth = s->bvh_depth;
    info->load_ms = s->load_ms;
    info->build_ms = s->build_ms;
    return FRT_OK;
}

extern "C" void frt_scene_destroy(frt_host_scene *s) { delete s; }

// ---------------------------------------------------------------------------
// cornell_1m generator: non-emissive quads -> k x k cells
// ---------------------------------------------------------------------------
extern "C" int frt_write_tessellated_obj(const char *src_obj, int k, const char *dst_obj)
{
    if (!src_obj || !dst_obj || k < 1) return FRT_E_INVALID;
    std::ifstream in(src_obj);
    if (!in) return FRT_E_IO;
    std::string dst = dst_obj;
    std::string mtl_dst = dst.substr(0, dst.size() >= 4 ? dst.size() - 4 : dst.size()) + ".mtl";
    // find and copy the material library next to the output
    std::vector<std::string> lines;
    std::string line, mtllib;
    while (std::getline(in, line)) {
        lines.push_back(line);
        const char *p = skip_ws(line.c_str());
        if (!strncmp(p, "mtllib", 6)) mtllib = rstrip(skip_ws(p + 6));
    }
    std::map<std::string, bool> emissive;
    if (!mtllib.empty()) {
        ObjData od;
        load_mtl(dir_of(src_obj) + mtllib, od);
        for (auto &m : od.mats) emissive[m.name] = (m.ke[0] != 0 || m.ke[1] != 0 || m.ke[2] != 0);
        std::ifstream mi(dir_of(src_obj) + mtllib, std::ios::binary);
        std::ofstream mo(mtl_dst, std::ios::binary);
        if (!mi || !mo) return FRT_E_IO;
        mo << mi.rdbuf();
    }
    FILE *f = fopen(dst_obj, "w");
    if (!f) return FRT_E_IO;
    const size_t slash = mtl_dst.find_last_of('/');
    fprintf(f, "# cornell-shaped tessellation (k=%d) of %s\nmtllib %s\n", k, src_obj,
            (slash == std::string::npos ? mtl_dst : mtl_dst.substr(slash + 1)).c_str());
    std::vector<std::string> vtok;  // raw vertex tokens of the source (positions)
    std::string cur_mtl;
    long long written = 0;
    for (const std::string &ln : lines) {
        const char *p = skip_ws(ln.c_str());
        if (p[0] == 'v' && (p[1] == ' ' || p[1] == '\t')) {
            vtok.push_back(rstrip(skip_ws(p + 1)));
        } else if (!strncmp(p, "usemtl", 6)) {
            cur_mtl = rstrip(skip_ws(p + 6));
            fprintf(f, "%s\n", rstrip(p).c_str());
        } else if ((p[0] == 'g' || p[0] == 'o') && (p[1] == ' ' || p[1] == '\t')) {
            fprintf(f, "%s\n", rstrip(p).c_str());
        } else if (p[0] == 'f' && (p[1] == ' ' || p[1] == '\t')) {
            std::istringstream ss(p + 1);
            std::vector<long> idx;
            std::string t;
            while (ss >> t) idx.push_back(std::stol(t));
            const long nv = (long)vtok.size();
            std::vector<std::array<double, 3>> P;
            for (long a : idx) {
                const long i = a < 0 ? nv + a : a - 1;
                float x, y, z;
                const char *q = vtok[i].c_str();
                q = parse_float(skip_ws(q), x);
                q = parse_float(skip_ws(q), y);
                parse_float(skip_ws(q), z);
                P.push_back({x, y, z});
            }
            const bool keep = emissive.count(cur_mtl) && emissive[cur_mtl];
            if (P.size() != 4 || keep || k == 1) {  // lights (and non-quads) stay as they are
                for (auto &pt : P) fprintf(f, "v %.9g %.9g %.9g\n", pt[0], pt[1], pt[2]);
                fprintf(f, "f");
                for (size_t i = 0; i < P.size(); ++i) fprintf(f, " %ld", (long)i - (long)P.size());
                fprintf(f, "\n");
                continue;
            }
            // bilinear grid (k+1)^2 over p0..p3, cells as quads (fanned like the source quads)
            for (int j = 0; j <= k; ++j)
                for (int i = 0; i <= k; ++i) {
                    const double s = (double)i / k, tt = (double)j / k;
                    double q[3];
                    for (int d = 0; d < 3; ++d)
                        q[d] = (1 - s) * (1 - tt) * P[0][d] + s * (1 - tt) * P[1][d] + s * tt * P[2][d] + (1 - s) * tt * P[3][d];
                    fprintf(f, "v %.9g %.9g %.9g\n", q[0], q[1], q[2]);
                }
            const long nvert = (long)(k + 1) * (k + 1);
            for (int j = 0; j < k; ++j)
                for (int i = 0; i < k; ++i) {
                    const long a = j * (k + 1) + i, b = a + 1, c = a + (k + 1) + 1, d = a + (k + 1);
                    fprintf(f, "f %ld %ld %ld %ld\n", a - nvert, b - nvert, c - nvert, d - nvert);
                    ++written;
                }
        }
    }
    fclose(f);
    (void)written;
    return FRT_OK;
}

extern "C" int frt_write_pfm(const char *path, int nx, int ny, const float *rgb)
{
    if (!path || !rgb || nx <= 0 || ny <= 0) return FRT_E_INVALID;
    FILE *f = fopen(path, "wb");
    if (!f) return FRT_E_IO;
    fprintf(f, "PF\n%d %d\n-1\n", nx, ny);
    const size_t n = (size_t)nx * ny * 3;
    const bool ok = fwrite(rgb, sizeof(float), n, f) == n;
    fclose(f);
    return ok ? FRT_OK : FRT_E_IO;
}
