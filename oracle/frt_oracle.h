/*
 * frt_oracle.h -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement, in plain C and fp64, of jammm/first_raytracer's hot path
 * (`path::Li`, first_ray/path.cpp:4-116) together with everything it reaches:
 * camera (camera.h:10-35), parallel_bvh traversal + SAH build
 * (parallel_bvh.h:39-175, bvh.h:6-55), triangle / sphere / aabb / list
 * queries, lambertian + diffuse_light + constant environment, cosine pdf,
 * onb, MIS weights, the OBJ/MTL ingest semantics of mesh_loader.cpp:5-162
 * (Assimp 5.0.1 behaviour restated) and the film / PFM output
 * (viewer.cpp:109-132, image.h:89-118).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product path (first_raytracer_amd/, libfrt.so)
 * never links or calls it.
 *
 * The reference draws std::mt19937 per thread (sampler.h:17-34, path.cpp:122)
 * and cannot be replayed; the restatement and the HIP kernels instead share
 * the counter-based RNG specified in DESIGN.md ("RNG stream spec").
 */
#ifndef FRT_ORACLE_H
#define FRT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ora_scene ora_scene;

typedef struct ora_counters {
    /* reference-algorithm counters (Scene.h:18-22 semantics, 64-bit) */
    uint64_t node_visits;     /* parallel_bvh_node::hit calls (parallel_bvh.h:41) */
    uint64_t box_passes;      /* passed node box tests (parallel_bvh.h:45)        */
    uint64_t tri_tests;       /* triangle::hit calls (triangle.h:71)              */
    uint64_t sphere_tests;    /* sphere::hit calls                                */
    /* top-level scene queries = "rays" (path.cpp:10 and :50)                     */
    uint64_t camera_rays;
    uint64_t extension_rays;
    uint64_t shadow_rays;
    uint64_t samples;
} ora_counters;

typedef struct ora_scene_info {
    int32_t n_tris, n_spheres, n_materials, n_lights, n_nodes, world_kind, n_list;
    int32_t bvh_depth;
} ora_scene_info;

/* Scene constructors (main.cpp:222-252 cornell_box_obj, main.cpp:281-314 veach_mis).
 * `kind`: "cornell_box_obj" | "veach_mis" | "obj_geo" | "obj_smooth".
 * For obj_* the camera is the cornell one.  Returns 0 on success. */
int  ora_load_scene(const char *kind, const char *obj_path, double aspect, ora_scene **out);
void ora_free_scene(ora_scene *s);
void ora_scene_get_info(const ora_scene *s, ora_scene_info *info);

/* Incremental construction (main.cpp's scene functions).  Materials are 26
 * doubles: type (FRT_MAT_* values: 0 lambertian, 1 diffuse_light,
 * 2 modified_phong, 3 metal, 4 dielectric, 5 rough_conductor), albedo[3],
 * emit[3], ks[3] (specular reflectance), shininess, ior, distribution
 * (0 GGX, 1 Beckmann), alpha, eta[3], k[3], texture (0 constant, 1 checker
 * of the textured colour and tex_odd), tex_odd[3], u_scale, v_scale. */
int  ora_scene_new(ora_scene **out);
/* create_triangle_mesh(file, toWorld, bsdf, lights, geo) (triangle.cpp:26-60);
 * to_world16 row-major or NULL (identity), bsdf20 NULL = the file's MTL materials.
 * Returns -1 on I/O error, -2 for a singular matrix. */
int  ora_scene_add_obj(ora_scene *s, const char *obj_path, const double *to_world16, const double *bsdf26,
                       int use_geometry_normals);
/* where: 1 world list, 2 Scene::lights, 3 both */
int  ora_scene_add_sphere(ora_scene *s, const double *c, double r, const double *mat26, int where);
void ora_scene_set_camera(ora_scene *s, const double *from, const double *at, const double *vup, double vfov,
                          double aspect, double aperture, double focus);
/* world_kind 0: create_bvh over the world prims in insertion order, 1: hitable_list */
int  ora_scene_finish(ora_scene *s, int world_kind);

/* Flattened export of the reference-topology BVH in left-first DFS order:
 * node i: box lo[3],hi[3] (6 doubles), left, right (child >= 0 = node index,
 * child < 0 = ~prim_ref).  prim_ref: triangle t -> t, sphere k -> (1<<30)|k. */
int  ora_scene_export_bvh(const ora_scene *s, double *boxes, int32_t *left, int32_t *right);
/* triangles: 9 doubles (v0,v1,v2) each; materials per triangle */
int  ora_scene_export_tris(const ora_scene *s, double *v9, int32_t *mat);

void ora_scene_export_camera(const ora_scene *s, double *out19);
int  ora_scene_export_lights(const ora_scene *s, int32_t *refs);
int  ora_scene_export_materials(const ora_scene *s, double *out26);   /* the 26-double description */

/* Render pixels (linear index y*nx+x, y=0 bottom row) with `spp` samples each,
 * frame seed `seed`, on `nthreads` threads.  out_rgb[3*i..] = mean radiance
 * (viewer::add_sample semantics).  Returns 0 on success. */
int  ora_render(const ora_scene *s, int nx, int ny, int spp, uint32_t seed,
                const int32_t *pixels, int npix, int nthreads,
                double *out_rgb, ora_counters *cnt);

/* The same with the integrator chosen: ORA_INTEGRATOR_PATH (path.cpp:4-116),
 * _AO (ao.cpp:4-27) or _NORMALS (debug_renderer.h:8-17).  Values = FRT_INTEGRATOR_*. */
enum { ORA_INTEGRATOR_PATH = 0, ORA_INTEGRATOR_AO = 2, ORA_INTEGRATOR_NORMALS = 3 };
int  ora_render_integrator(const ora_scene *s, int integrator, int nx, int ny, int spp, uint32_t seed,
                           const int32_t *pixels, int npix, int nthreads, double *out_rgb, ora_counters *cnt);
/* ... and with path::Li's depth cap (33 in path.cpp:36; MaxPathLength 10 for the
 * PSS-MLT comparison) */
int  ora_render_depth(const ora_scene *s, int integrator, int nx, int ny, int spp, uint32_t seed, int max_depth,
                      const int32_t *pixels, int npix, int nthreads, double *out_rgb, ora_counters *cnt);
/* constant environment colour (the reference scenes use black) */
void ora_scene_set_env(ora_scene *s, const double *rgb);
/* image_texture's decoded image (format 0: nx*ny*3 bytes, sRGB; 1: floats); *index
 * = its material description entry d[26] (d[20] = 2) */
int ora_scene_add_image(ora_scene *s, int nx, int ny, int format, const void *data, int *index);
/* test hooks: image_texture::value (format 0 = 8-bit sRGB bytes, 1 = floats)
 * and environment_map::eval's direction -> (u, v) */
int ora_image_lookup(int nx, int ny, int format, const void *data, double u, double v, double *out3);
void ora_env_uv(const double *d, double *u, double *v);
/* ao.cpp:21 t_max = world bounding box height * 0.5 (NaN for list worlds) */
double ora_scene_ao_tmax(const ora_scene *s);

/* PSS-MLT (pssmlt.cpp): bootstrap b, full render (splat film, caller-zeroed),
 * and a single eye path for given primary samples (92 doubles -> x, y, rgb, sc). */
double ora_mlt_bootstrap(const ora_scene *s, int nx, int ny, uint32_t seed, int n_init);
int  ora_mlt_render(const ora_scene *s, int nx, int ny, uint32_t seed, int n_init, int n_chains, long long steps,
                    int nthreads, double *film, double *b_out, ora_counters *cnt);
/* the chains c = shard_index + j * shard_count of an n_chains render (the GPU's
 * shard rule); per local chain, optionally: fp[2j] = accepted proposals,
 * fp[2j+1] = sum of the accepted steps' 1-based indices mod 2^32, u[92 j ..]
 * = final state */
int  ora_mlt_render_shard(const ora_scene *s, int nx, int ny, uint32_t seed, int n_init, int n_chains, long long steps,
                          int shard_index, int shard_count, int nthreads, double *film, double *b_out,
                          ora_counters *cnt, uint32_t *fp, double *u);
void ora_mlt_eye_path(const ora_scene *s, int nx, int ny, const double *prnds, double *out6);

/* Single query of the world (closest or any hit) with reference counters. */
int  ora_world_hit(const ora_scene *s, const double *o, const double *d, double tmin, double tmax,
                   double *t_out, int32_t *prim_out, ora_counters *cnt);

/* RNG stream spec (shared with the HIP kernels). */
double   ora_rng_uniform(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t dim);

/* ---- component known-answer entry points (checked against oracle/_ref) ---- */
/* tri: 9 doubles v0 v1 v2; geo=1 geometric normal, else normals n9.
 * out: hit, t, p[3], normal[3], u, v  (10 doubles) */
int  ora_kat_tri_hit(const double *v9, const double *n9, int geo, const double *o, const double *d,
                     double tmin, double tmax, double *out);
/* sphere c[3], r; out: hit, t, p[3], normal[3] */
int  ora_kat_sphere_hit(const double *c, double r, const double *o, const double *d,
                        double tmin, double tmax, double *out);
/* hit texture coordinates + checker_texture::value's pick; out4: ok, u, v, odd */
int  ora_kat_texture_sphere(const double *c, double r, const double *o, const double *d, double us, double vs,
                            double *out4);
int  ora_kat_texture_tri(const double *v9, const double *uv6, const double *o, const double *d, double us,
                         double vs, double *out4);
/* out: 1/0 */
int  ora_kat_aabb_hit(const double *lo, const double *hi, const double *o, const double *d,
                      double tmin, double tmax);
/* camera: lookfrom, lookat, vup, vfov, aspect, aperture, focus, s, t, sample2 -> o[3], d[3] */
void ora_kat_camera(const double *from, const double *at, const double *vup, double vfov, double aspect,
                    double aperture, double focus, double s, double t, const double *smp, double *out6);
/* cosine pdf around unit normal n: generate(sample2) -> dir[3], value(dir) */
void ora_kat_cosine(const double *n, const double *smp, double *out4);
void ora_kat_fresnel(const double *n, const double *wi, double eta, double *out8);
void ora_kat_phong(const double *n, const double *wi, double e, double s0, double s1, const double *wo,
                   const double *kd, const double *ks, double *out11);
void ora_kat_dielectric(const double *n, const double *wi, double ior, double u0, const double *wo, const double *ks,
                        double *out12);
/* metal (material.h:110-130): out reflect dir[3], constant pdf value, eval_bsdf[3] */
void ora_kat_metal(const double *n, const double *wi, const double *albedo, const double *wo, double *out7);
/* rough_conductor + roughconductor_pdf (material.h:246-315, pdf.h:231-486): ggx = 1 GGX, 0 Beckmann;
 * out: generate dir[3], sampled_pdf, value(unit dir), value(wo), eval(unit dir)[3], eval(wo)[3] */
void ora_kat_conductor(const double *n, const double *wi, int ggx, double alpha, const double *eta, const double *k,
                       const double *spec, double s0, double s1, const double *wo, double *out12);
/* triangle sample_direct from o: out p[3], normal[3], to_light[3], pdf */
void ora_kat_tri_sample(const double *v9, const double *n9, int geo, int n_tris_in_mesh, const double *o,
                        const double *smp, double *out10);
/* sphere sample_direct + pdf_direct_sampling: out to_light[3], rec.normal[3], pdf(of lrec=...)  */
void ora_kat_sphere_sample(const double *c, double r, const double *o, const double *smp, double *out7);
double ora_kat_miweight(double a, double b);
double ora_kat_fromsrgb(double v);
float  ora_kat_atof(const char *s);
int    ora_kat_pick(double u, int n);
/* glibc-qsort ordering with the reference comparator (bvh.h:6-55) on keys */
void   ora_kat_sort(const double *keys, int n, int32_t *perm_out);

void   ora_kat_list_hit(int ntri, int nsph, const double *geom, const double *o, const double *d, double *out3);

/* viewer::add_sample's display bytes (viewer.cpp:115-117), n values */
void ora_tonemap_u8(const double *rgb, long n, uint8_t *out);

/* PFM writer with image_pfm::save_image byte layout (image.h:89-118). */
int  ora_write_pfm(const char *path, int nx, int ny, const double *rgb);

#ifdef __cplusplus
}
#endif
#endif
