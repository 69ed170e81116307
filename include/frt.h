/*
 * frt.h -- C-ABI of the MI355X path-tracing integrator (the drop-in boundary).
 *
 * Replaces, for one GPU, the work the reference enqueues in
 *   path::Render(Scene*, viewer*, tf::Taskflow&)         first_ray/path.cpp:118-148
 *   path::Li(ray, Scene*, depth, prev_hrec, pdf, sampler) first_ray/path.cpp:4-116
 * as driven by renderer<path>::Render                    first_ray/integrator.h:14-46
 * and writes the film that viewer::add_sample fills       first_ray/viewer.cpp:109-132.
 *
 * The caller flattens its Scene (Scene.h:10-26) once into an frt_scene_view
 * (plain host arrays, fp64 like the reference's Vector3f), uploads it, and
 * renders tiles of the frame.  No torch / HIP C++ types cross this boundary;
 * a hip stream is passed as an opaque pointer.  See INTEGRATION.md for the
 * reference-side `path_gpu` binding.
 *
 * Errors: every call returns 0 on success or a negative FRT_E* code;
 * frt_last_error(ctx) describes the last failure (the reference throws
 * std::runtime_error, e.g. triangle.cpp:34, image.h:102; the C++ host
 * wrapper include/frt_integrator.hpp converts codes back into exceptions).
 */
#ifndef FRT_H
#define FRT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FRT_ABI_VERSION 9

enum {
    FRT_OK = 0,
    FRT_E_INVALID = -1,      /* bad argument / malformed scene view        */
    FRT_E_HIP = -2,          /* HIP runtime failure (message in last_error) */
    FRT_E_NO_SCENE = -3,     /* frt_render before frt_upload_scene          */
    FRT_E_UNSUPPORTED = -4,  /* material/feature outside the hot path       */
    FRT_E_IO = -5,           /* file could not be read / written            */
    FRT_E_NO_DEVICE = -6     /* no gfx950 device / bad device index         */
};

enum { FRT_WORLD_BVH = 0, FRT_WORLD_LIST = 1 };          /* parallel_bvh_node | hitable_list */
enum { FRT_MAT_LAMBERTIAN = 0,      /* material.h:50-73                                  */
       FRT_MAT_DIFFUSE_LIGHT = 1,   /* material.h:179-192                                */
       FRT_MAT_MODIFIED_PHONG = 2,  /* material.h:75-108 + cosine_power_pdf (pdf.h:99)   */
       FRT_MAT_METAL = 3,           /* material.h:110-130 + constant_pdf (pdf.h:186)     */
       FRT_MAT_DIELECTRIC = 4,      /* material.h:133-177 + dielectric_pdf (pdf.h:138)   */
       FRT_MAT_ROUGH_CONDUCTOR = 5 };/* material.h:246-315 + roughconductor_pdf (pdf.h:231) */
enum { FRT_DIST_GGX = 0, FRT_DIST_BECKMANN = 1 };   /* microfacet_distributions (util.h:48-52) */
enum { FRT_INTEGRATOR_PATH = 0,     /* path::Li           path.h:8-18, path.cpp:4-116      */
       FRT_INTEGRATOR_PSSMLT = 1,   /* pssmlt             pssmlt.h:29-76                   */
       FRT_INTEGRATOR_AO = 2,       /* ao::Li             ao.h:8-43, ao.cpp:4-27           */
       FRT_INTEGRATOR_NORMALS = 3   /* normals_renderer   debug_renderer.h:6-50            */ };
enum { FRT_FLAG_NO_LDS_SCENE = 1,      /* render_params.flags: keep small scenes in HBM/L2 (A/B timing)  */
       FRT_FLAG_WAVES5 = 2,            /* register cap for 5 waves/SIMD (A/B timing)                     */
       FRT_FLAG_WAVES6 = 4,            /* register cap for 6 waves/SIMD (A/B timing)                     */
       FRT_FLAG_WAVES4 = 8,            /* the compiler's own allocation, ~4 waves/SIMD (A/B timing)      */
       FRT_FLAG_BVH2 = 16,             /* binary nodes for HBM-resident scenes (A/B timing, self-test)   */
       /* 32, 64, 128: retired A/B plans (4-wide nodes from LDS, lockstep brute force,
          speculative traversal), measured slower and removed in round 4; FRT_E_INVALID since round 5 */
       FRT_FLAG_NO_OCT = 256,          /* LDS binary plan without the per-octant node copies (A/B timing) */
       FRT_FLAG_FP64 = 512,            /* path: the fp64 kernel for this call (self-test: fp64 host replay) */
       FRT_FLAG_FP32 = 1024 };         /* path: the fp32 kernels even where the precision picks fp64      */

/* Kernel precision (frt_set_precision).  The reference computes in fp64
 * (geometry.h:351).  FRT_PRECISION_AUTO: fp64 for list worlds (hitable_list,
 * e.g. veach_mis: a few primitives, and lights small enough -- r = 0.033 --
 * that fp32 rounding moves samples onto or off them), fp32 for BVH worlds.
 * FRT_PRECISION_FP64: every path render in fp64 (the binary tree from HBM:
 * the debugging build SURVEY 8(a) names).  FRT_PRECISION_FP32: fp32 only.
 * AO, normals and PSS-MLT always run in fp32. */
enum { FRT_PRECISION_AUTO = 0, FRT_PRECISION_FP32 = 1, FRT_PRECISION_FP64 = 2 };

/* primitive reference: triangle t -> t ; sphere k -> FRT_PRIM_SPHERE | k */
#define FRT_PRIM_SPHERE (1 << 30)

typedef struct frt_material {
    int32_t type;            /* FRT_MAT_*                                                 */
    int32_t distribution;    /* rough_conductor: FRT_DIST_GGX / FRT_DIST_BECKMANN         */
    double albedo[3];        /* lambertian albedo / modified_phong diffuse_reflectance /
                                metal albedo                                              */
    double emit[3];          /* diffuse_light: constant_texture colour                    */
    double specular[3];      /* modified_phong / dielectric / rough_conductor:
                                specular_reflectance (constant texture)                   */
    double exponent;         /* modified_phong: specular_exponent                         */
    double ior;              /* dielectric: ref_idx                                       */
    double alpha;            /* rough_conductor: roughness (alphaU = alphaV)              */
    double eta[3], k[3];     /* rough_conductor: complex IOR (fresnelConductorExact)      */
    /* The material's texture (lambertian albedo, modified_phong diffuse_reflectance,
     * dielectric / rough_conductor specular_reflectance): FRT_TEX_CONSTANT uses the
     * colour field above; FRT_TEX_CHECKER (checker_texture, texture.h:30-49) of two
     * constants -- that field as tex0 and tex_odd as tex1 -- at u_scale, v_scale,
     * looked up at the hit's uv (sphere: get_sphere_uv, hitable.h:15-21; triangle:
     * interpolated OBJ vt, triangle.h:105-107).  FRT_TEX_IMAGE (image_texture,
     * texture.h:51-95): the scene view's image `image`, nearest texel at (u nx, v ny)
     * with the reference's wrap / clamp. */
    int32_t texture;
    int32_t image;           /* FRT_TEX_IMAGE: index into frt_scene_view.images      */
    double tex_odd[3];
    double tex_scale[2];
} frt_material;
enum { FRT_TEX_CONSTANT = 0, FRT_TEX_CHECKER = 1, FRT_TEX_IMAGE = 2 };

/* A decoded image for image_texture (texture.h:51-95; the reference's `image`,
 * image.h, as stb_image returns it: rows top to bottom, 3 channels).
 * FRT_IMAGE_SRGB8: nx*ny*3 bytes, the texel is FromSrgb(byte / 255) (util.h:62-66);
 * FRT_IMAGE_F32: nx*ny*3 floats used as they are (the STBI_HDR branch). */
enum { FRT_IMAGE_SRGB8 = 0, FRT_IMAGE_F32 = 1 };
typedef struct frt_image {
    int32_t nx, ny;
    int32_t format;          /* FRT_IMAGE_*                                               */
    int32_t reserved;
    const void *data;
} frt_image;

typedef struct frt_scene_view {
    int32_t world_kind;                 /* FRT_WORLD_BVH or FRT_WORLD_LIST              */
    /* triangles (triangle.h:55-66, one entry per `triangle` object) */
    int32_t n_tris;
    const double *tri_v;                /* 9 per tri: v0, v1, v2                        */
    const double *tri_n;                /* 9 per tri: vertex normals, or NULL           */
    const int32_t *tri_material;        /* index into materials                         */
    const uint8_t *tri_geometry_normal; /* use_geometry_normals per tri, NULL = all 1   */
    const double *tri_inv_area;         /* 1/(0.5|e1 x e2| nTriangles_of_mesh)           */
    /* spheres (sphere.h:8-24) */
    int32_t n_spheres;
    const double *sphere;               /* 4 per sphere: centre, radius                 */
    const int32_t *sphere_material;
    /* materials */
    int32_t n_materials;
    const frt_material *materials;
    /* BVH world: the parallel_bvh_node tree (parallel_bvh.h:8-27) */
    int32_t n_nodes;
    int32_t root;                       /* node index, or ~prim_ref for a 1-prim world  */
    const double *node_box;             /* 6 per node: min, max                         */
    const int32_t *node_child;          /* 2 per node: left, right; >=0 node, <0 ~prim  */
    /* list world (hitable_list, hitable_list.cpp:4-21) */
    int32_t n_list;
    const int32_t *list;                /* prim refs in list order                      */
    /* Scene::lights (hitable_list of emitters) */
    int32_t n_lights;
    const int32_t *lights;              /* prim refs                                    */
    /* camera (camera.h:10-28), already constructed */
    double cam_origin[3], cam_lower_left[3], cam_horizontal[3], cam_vertical[3];
    double cam_u[3], cam_v[3];
    double cam_lens_radius;
    /* environment_map with a constant texture (material.h:206-232) */
    double env_color[3];
    /* camera w axis and half_height (camera.h:18-26): PSS-MLT's screen mapping
     * (pssmlt.cpp:134-138) needs them; half_height = 256 / camera::dist */
    double cam_w[3];
    double cam_half_height;
    /* texture coordinates: 6 per tri (uv of v0, v1, v2, the OBJ's vt), or NULL = 0 */
    const double *tri_uv;
    /* images of FRT_TEX_IMAGE materials (ABI 7) */
    int32_t n_images;
    const frt_image *images;
} frt_scene_view;

typedef struct frt_render_params {
    int32_t nx, ny;          /* film size (viewer nx, ny); nx * ny <= 2^31 - 1 (int32 pixel
                              * indices), larger frames fail with FRT_E_INVALID             */
    int32_t spp;             /* samples per pixel (viewer ns)                              */
    uint32_t seed;           /* frame seed of the counter RNG (DESIGN.md "RNG stream spec") */
    int32_t max_depth;       /* scatter while depth <= max_depth; reference: 33 (path.cpp:36) */
    int32_t integrator;      /* FRT_INTEGRATOR_*                                           */
    int32_t tile_size;       /* square tiles, multiple of 8; 0 = 32                        */
    int32_t shard_index;     /* this call renders tiles t with t % shard_count == index    */
    int32_t shard_count;     /* 1 = whole frame                                            */
    int32_t samples_per_item;/* work granule in samples; 0 = automatic                     */
    int32_t flags;           /* FRT_FLAG_* bits, 0 = defaults                              */
    /* PSS-MLT only: spp = mutations per pixel (total = spp*nx*ny, the reference's
     * ns), split over mlt_chains chains (chain c runs in shard c % shard_count);
     * mlt_bootstrap = paths for the normaliser b (pssmlt.h:12 N_Init = 10000). */
    int32_t mlt_chains;
    int32_t mlt_bootstrap;
    /* progressive rendering (path / AO / normals): this call renders samples
     * [sample_offset, sample_offset + spp) of every pixel -- the RNG streams
     * are keyed by the global sample index, so passes of 64 + 64 + ... samples
     * average to the film of one call with their total (frt_film_accumulate). */
    int32_t sample_offset;
} frt_render_params;

typedef struct frt_stats {
    uint64_t camera_rays;    /* top-level scene queries, path.cpp:10 at depth 0 */
    uint64_t extension_rays; /* path.cpp:10 at depth > 0                        */
    uint64_t shadow_rays;    /* path.cpp:50                                     */
    uint64_t samples;
    uint64_t pixels;
    uint64_t work_items;
    double kernel_ms;        /* path megakernel, HIP events on its stream       */
    double total_ms;         /* whole call                                      */
    /* launch configuration of the megakernel (measurement reporting) */
    uint32_t scene_in_lds;   /* 1: nodes/triangles/materials were read from LDS */
    uint32_t waves_cap;      /* register cap in waves/SIMD, 0 = compiler's own  */
    uint32_t stack_entries;  /* per-lane LDS traversal stack                    */
    uint32_t bvh_depth;      /* levels of the device BVH (after leaf collapse)  */
    uint64_t scene_bytes;    /* scene bytes the plan reads: its LDS copy when   */
                             /* scene_in_lds (the octant node copies on that    */
                             /* plan), else nodes + triangles + shading records */
                             /* + materials in HBM                              */
    uint32_t fp64;           /* 1: the fp64 kernel ran (ABI 8)                  */
    uint32_t reserved;
} frt_stats;

int frt_get_abi_version(void);

/* ---- context: one per GPU, not thread-safe ---- */
typedef struct frt_ctx frt_ctx;
int frt_create(int hip_device, frt_ctx **out);
int frt_destroy(frt_ctx *ctx);
const char *frt_last_error(const frt_ctx *ctx);
/* FRT_PRECISION_*; read by the next frt_upload_scene (fp64 records are
 * uploaded only when the precision can select the fp64 kernels for that
 * scene) and by every render.  Default FRT_PRECISION_AUTO. */
int frt_set_precision(frt_ctx *ctx, int precision);

/* Copy the scene to HBM (fp32 device layout, DESIGN.md "Data layout").  The
 * view's arrays are only read during the call. */
int frt_upload_scene(frt_ctx *ctx, const frt_scene_view *scene);

/* Shard geometry: number of output slots of a shard (tiles * tile_size^2) and,
 * per slot, the linear film index y*nx+x it holds (or -1 for padding). */
int64_t frt_shard_slot_count(const frt_render_params *p);
int frt_shard_slots(const frt_render_params *p, int32_t *slot_pixel);

/* Render this shard.  `film_rgb` is the caller's full film (nx*ny*3 floats,
 * index (y*nx+x)*3, y = 0 bottom row, as viewer::fout_image); only this
 * shard's pixels are written, with the mean radiance (viewer.cpp:111).
 * PSS-MLT: every chain splats anywhere, so the shard's splat film is ADDED to
 * film_rgb (zero it first; summing all shards gives the image,
 * AccumulatePathContribution pssmlt.cpp:19-38). */
int frt_render(frt_ctx *ctx, const frt_render_params *p, float *film_rgb, frt_stats *st);

/* One process, n GPUs: ctxs[i] (each with the scene uploaded) renders shard
 * (i, n) of the whole-frame request `p` (shard_index 0, shard_count 1) on its
 * own host thread; the full film lands in film_rgb (PSS-MLT: the shard films
 * summed in order 0..n-1, added to film_rgb).  Replaces the multi-worker
 * path::Render task graph (path.cpp:118-148) across devices. */
int frt_render_multi(frt_ctx **ctxs, int n, const frt_render_params *p, float *film_rgb, frt_stats *st);

/* Device variant: writes the shard's slots (frt_shard_slot_count * 3 floats,
 * slot order) into device memory `slots_rgb` on `hip_stream` (NULL = the
 * context's stream) and returns after the work has completed.  PSS-MLT: the
 * slots are the whole film (nx*ny, natural order) holding this shard's splats;
 * shards are combined with a sum (RCCL reduce / all-reduce). */
int frt_render_device(frt_ctx *ctx, const frt_render_params *p, float *slots_rgb, void *hip_stream,
                      frt_stats *st);

/* PSS-MLT chain states of this context's last PSS-MLT render (parity tests and
 * diagnostics; pssmlt.cpp:301-365 keeps them in TMarkovChain): its local chains
 * [first, first + n), local chain j = global chain shard_index + j *
 * shard_count.  u_out (n x 92 floats, or NULL): the chain's final primary
 * samples; fp_out (n x 2, or NULL): its trajectory fingerprint = (accepted
 * proposals, sum of the accepted mutations' 1-based step indices mod 2^32).
 * FRT_E_INVALID when the last render of the context was not PSS-MLT or the
 * range is outside its chains. */
int frt_mlt_chain_state(frt_ctx *ctx, uint64_t first, uint64_t n, float *u_out, uint32_t *fp_out);

/* Ray queries on the uploaded scene: Scene::world->hit (path.cpp:10, 50;
 * parallel_bvh_node::hit parallel_bvh.h:39-64, hitable_list::hit
 * hitable_list.cpp:4-21) for a batch of rays, with the world's own t_min
 * (EPSILON * max(1, |o|) for a BVH, EPSILON for a list).  Device memory:
 * rays = n x 8 floats (origin xyz, t_max, direction xyz, flags: bit 0 = any
 * hit, the shadow query of path.cpp:50), hits = n x 4 floats (t, u, v, prim
 * as int32 bits: the scene view's triangle index or FRT_PRIM_SPHERE | k, -1 =
 * miss; a miss leaves t = t_max).  flags: FRT_FLAG_NO_LDS_SCENE / _BVH2 /
 * _NO_OCT choose the plan as for frt_render.  Returns after the work has
 * completed on `hip_stream` (NULL = the context's stream); st->kernel_ms.
 * The ray queue has its own word in the context, apart from the render's, but
 * a context is still one stream's worth of state: calls on one context are
 * issued from one host thread, one at a time (each returns when its work is
 * done).  n plus a chunk of 256 rays per resident wave must stay below 2^32.
 * Input domain: finite origins, directions and t_max, directions not zero,
 * and |origin| and the scene's coordinates below 1e8 on every axis.  (A
 * direction component below 1e-30 is nudged to +-1e-30 for the slab test;
 * with both an origin and a box plane beyond ~3.4e8 on that axis the slab
 * distances would be inf - inf = NaN, and the NaN-propagating min / max of
 * the box test would then cull the box.)  The rays a render makes stay inside
 * this domain for every scene the reference builds. */
int frt_trace_device(frt_ctx *ctx, const float *rays, int64_t n, float *hits, int flags, void *hip_stream,
                     frt_stats *st);

/* ---- host-side scene pipeline (native C++; what main.cpp + mesh_loader +
 *      parallel_bvh_node::create_bvh do in the reference) ---- */
typedef struct frt_host_scene frt_host_scene;
typedef struct frt_host_scene_info {
    int32_t n_tris, n_spheres, n_materials, n_lights, n_nodes, world_kind, n_list, bvh_depth;
    double load_ms, build_ms;
} frt_host_scene_info;
/* kind: "cornell_box_obj" (main.cpp:222-252), "veach_mis" (main.cpp:281-314),
 *       "obj_geo" / "obj_smooth" (any OBJ, cornell camera, geometric / vertex normals) */
int frt_scene_create(const char *kind, const char *obj_path, double aspect, frt_host_scene **out);
int frt_scene_view_get(const frt_host_scene *s, frt_scene_view *view);

/* Incremental construction, what main.cpp's scene functions do (e.g.
 * veach_ajar main.cpp:318-412, glass_of_water :414-480): OBJ files through
 * create_triangle_mesh(file, toWorld, bsdf, lights, use_geometry_normals)
 * (triangle.cpp:26-60), spheres, the camera, then parallel_bvh_node::create_bvh
 * or a hitable_list over the world prims in insertion order.
 *   frt_scene_new -> frt_scene_add_obj / _add_sphere ... -> frt_scene_set_camera
 *   -> frt_scene_finish -> frt_scene_view_get
 * add_obj: to_world16 = row-major Matrix4x4 or NULL (identity); bsdf = the one
 * material every mesh of the file takes, or NULL for the file's MTL materials
 * (mesh_loader.cpp:59-112); meshes whose material is a diffuse_light join
 * Scene::lights.  Returns FRT_E_IO (unreadable file) or FRT_E_INVALID (singular
 * matrix, bad material). */
enum { FRT_SPHERE_WORLD = 1, FRT_SPHERE_LIGHTS = 2, FRT_SPHERE_BOTH = 3 };
int frt_scene_new(frt_host_scene **out);
int frt_scene_add_obj(frt_host_scene *s, const char *obj_path, const double *to_world16, const frt_material *bsdf,
                      int use_geometry_normals);
/* where: FRT_SPHERE_WORLD (the world list), FRT_SPHERE_LIGHTS (a separate
 * Scene::lights object, as veach_mis main.cpp:298-302 does), or both (one object) */
int frt_scene_add_sphere(frt_host_scene *s, const double *center, double radius, const frt_material *m, int where);
/* camera.h:10-28; the reference constructs every scene's camera this way */
int frt_scene_set_camera(frt_host_scene *s, const double *lookfrom, const double *lookat, const double *vup,
                         double vfov, double aspect, double aperture, double focus_dist);
/* environment_map with a constant texture (material.h:206-232) */
int frt_scene_set_env(frt_host_scene *s, const double *rgb);
/* a decoded image (copied) for FRT_TEX_IMAGE materials; *index = its frt_material.image */
int frt_scene_add_image(frt_host_scene *s, const frt_image *img, int *index);
/* world_kind FRT_WORLD_BVH (create_bvh) or FRT_WORLD_LIST */
int frt_scene_finish(frt_host_scene *s, int world_kind);
/* GPU BVH builders: replace the finished scene's world
 * (BVH or list) with a BVH over the same world prims built on ctx's device
 * (csrc/frt_lbvh.hip), in place of parallel_bvh_node::create_bvh's SAH sweep:
 *   FRT_GPU_BVH_PLOC  Morton codes, radix sort, then PLOC clustering (mutual
 *                     nearest neighbours by union surface area within 16
 *                     clusters in Morton order);
 *   FRT_GPU_BVH_LBVH  Morton codes, radix sort, Karras hierarchy, atomic refit;
 *   FRT_GPU_BVH_SAH   top-down binned SAH, one tree level per launch, one
 *                     workgroup per node (32 centroid bins per axis in LDS,
 *                     cost N_L A_L + N_R A_R: frt_scene_build_bvh_sah's rule).
 * frt_scene_build_bvh_gpu = the binned SAH builder.  Finish with FRT_WORLD_LIST to
 * skip the host build.  The topology differs from the reference's, so exact-t
 * ties between primitives may resolve differently.  device_ms (optional) =
 * device time of the build passes. */
enum { FRT_GPU_BVH_PLOC = 0, FRT_GPU_BVH_LBVH = 1, FRT_GPU_BVH_SAH = 2 };
int frt_scene_build_bvh_gpu(frt_host_scene *s, frt_ctx *ctx, double *device_ms);
int frt_scene_build_bvh_gpu_algo(frt_host_scene *s, frt_ctx *ctx, int algo, double *device_ms);
/* Binned SAH tree (32 centroid bins per axis, host threads) over the same
 * world prims: better traversal than the reference's sweep on large meshes
 * (same tie caveat as the GPU tree). */
int frt_scene_build_bvh_sah(frt_host_scene *s);
int frt_scene_info(const frt_host_scene *s, frt_host_scene_info *info);
void frt_scene_destroy(frt_host_scene *s);

/* cornell_1m generator: every non-emissive quad of `src_obj` bilinearly
 * tessellated into k x k cells, written as OBJ + MTL. */
int frt_write_tessellated_obj(const char *src_obj, int k, const char *dst_obj);

/* image_pfm::save_image layout (image.h:89-118), path used as given. */
int frt_write_pfm(const char *path, int nx, int ny, const float *rgb);

/* ---- film / output side (viewer.cpp:109-132, image.cpp:24-58) ---- */
/* Progressive accumulation: acc = (acc * acc_spp + pass * pass_spp) / (acc_spp + pass_spp),
 * per element (n floats), so a film accumulated over passes is the mean over all of
 * their samples (viewer.cpp:111 divides by the total ns). */
int frt_film_accumulate(float *acc, int64_t acc_spp, const float *pass, int64_t pass_spp, int64_t n);
/* viewer::add_sample's display mapping (viewer.cpp:115-117): per channel
 * int(pow(1 - exp(-x), 1/2.2) * 255 + 0.5), stored as a byte, for a mean film
 * (nx*ny*3 floats, y = 0 bottom row) -> u8 rgb in the same layout. */
int frt_tonemap_u8(const float *rgb, int nx, int ny, uint8_t *out_u8);
/* image::save_image (image.cpp:24-58): u8 rgb (y = 0 bottom row) flipped to
 * top-down rows (stbi_flip_vertically_on_write) and written as PNG or BMP.  The
 * extension is appended when missing, as the reference does.  The reference's
 * switch writes BMP bytes for STBI_JPG and JPEG for STBI_BMP (image.cpp:40-52);
 * FRT_IMAGE_JPG reproduces the first, and JPEG encoding is not provided. */
enum { FRT_IMAGE_PNG = 0, FRT_IMAGE_BMP = 1, FRT_IMAGE_JPG = 2 };
int frt_write_image(const char *path, int nx, int ny, const uint8_t *rgb_u8, int format);

/* ---- self-test hook for CPU-only unit tests: runs the megakernel's per-lane
 *      path code (frt_path.hpp) on the host over the flattened fp32 scene for
 *      the listed pixels (linear y*nx+x); out_rgb = per-pixel means.  Not a
 *      render path: frt_render / frt_render_device never use it. ---- */
int frt_selftest_path_host(const frt_scene_view *scene, const frt_render_params *p, const int32_t *pixels,
                           int npix, float *out_rgb, frt_stats *st);
/* Same for PSS-MLT: n bootstrap-stream eye paths (frt_mlt.hpp) on the host;
 * out6 per path = film x, film y, r, g, b, scalar contribution. */
int frt_selftest_mlt_paths_host(const frt_scene_view *scene, int nx, int ny, uint32_t seed, int n, float *out6);

#ifdef __cplusplus
}
#endif
#endif /* FRT_H */
