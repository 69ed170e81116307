"""first_raytracer_amd -- MI355X-native path-tracing integrator (drop-in for
jammm/first_raytracer's path::Li / path::Render hot path).

The product is native: libfrt.so (HIP kernels for gfx950 + the C++ host scene
pipeline) behind the C-ABI in include/frt.h.  This module is a thin ctypes
binding used by the tests, bench.py and scripts; it never falls back to a CPU
path -- if libfrt.so is missing or no gfx950 device is present, it raises.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# FRT_LIB_PATH: an experiment build (Makefile `exp` target) for timing A/B only
LIB_PATH = os.environ.get("FRT_LIB_PATH") or os.path.join(HERE, "libfrt.so")

FRT_WORLD_BVH, FRT_WORLD_LIST = 0, 1
FRT_MAT_LAMBERTIAN, FRT_MAT_DIFFUSE_LIGHT = 0, 1
FRT_PRIM_SPHERE = 1 << 30
ABI_VERSION = 9                 # include/frt.h FRT_ABI_VERSION (frt_stats / frt_material layout)
FRT_MAT_LAMBERTIAN, FRT_MAT_DIFFUSE_LIGHT, FRT_MAT_MODIFIED_PHONG, FRT_MAT_METAL, FRT_MAT_DIELECTRIC = 0, 1, 2, 3, 4
FRT_MAT_ROUGH_CONDUCTOR = 5
FRT_DIST_GGX, FRT_DIST_BECKMANN = 0, 1
FRT_TEX_CONSTANT, FRT_TEX_CHECKER, FRT_TEX_IMAGE = 0, 1, 2
FRT_IMAGE_SRGB8, FRT_IMAGE_F32 = 0, 1
FRT_FLAG_NO_LDS_SCENE = 1
FRT_FLAG_WAVES5 = 2
FRT_FLAG_WAVES6 = 4
FRT_FLAG_WAVES4 = 8
FRT_FLAG_BVH2 = 16
FRT_FLAG_NO_OCT = 256
FRT_FLAG_FP64 = 512
FRT_FLAG_FP32 = 1024
FRT_PRECISION_AUTO, FRT_PRECISION_FP32, FRT_PRECISION_FP64 = 0, 1, 2
FRT_GPU_BVH_PLOC = 0
FRT_GPU_BVH_LBVH = 1
FRT_GPU_BVH_SAH = 2
FRT_INTEGRATOR_PATH, FRT_INTEGRATOR_PSSMLT, FRT_INTEGRATOR_AO, FRT_INTEGRATOR_NORMALS = 0, 1, 2, 3

ERRORS = {0: "ok", -1: "invalid", -2: "hip", -3: "no scene", -4: "unsupported", -5: "io", -6: "no gfx950 device"}


class FrtError(RuntimeError):
    pass


class Material(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("distribution", ctypes.c_int32),
                ("albedo", ctypes.c_double * 3), ("emit", ctypes.c_double * 3),
                ("specular", ctypes.c_double * 3), ("exponent", ctypes.c_double), ("ior", ctypes.c_double),
                ("alpha", ctypes.c_double), ("eta", ctypes.c_double * 3), ("k", ctypes.c_double * 3),
                ("texture", ctypes.c_int32), ("image", ctypes.c_int32), ("tex_odd", ctypes.c_double * 3),
                ("tex_scale", ctypes.c_double * 2)]

    @classmethod
    def from_spec(cls, m):
        """frt_material from a scene-spec material dict (see HostScene.from_spec)."""
        r = cls()
        r.type = MAT_TYPES[m["type"]]
        r.distribution = DISTRIBUTIONS[m.get("distribution", "ggx").lower()]
        for k in ("albedo", "emit", "specular", "eta", "k"):
            getattr(r, k)[:] = [float(x) for x in m.get(k, (0.0, 0.0, 0.0))]
        r.exponent = float(m.get("exponent", 0.0))
        r.ior = float(m.get("ior", 0.0))
        r.alpha = float(m.get("alpha", 0.0))
        tex = m.get("checker")               # {"odd": rgb, "scale": (u_scale, v_scale)}
        if tex is not None:
            r.texture = FRT_TEX_CHECKER
            r.tex_odd[:] = [float(x) for x in tex["odd"]]
            r.tex_scale[:] = [float(x) for x in tex["scale"]]
        if m.get("image") is not None:       # index into the spec's "images"
            r.texture = FRT_TEX_IMAGE
            r.image = int(m["image"])
        return r


class Image(ctypes.Structure):
    """frt_image: a decoded image for FRT_TEX_IMAGE (image_texture, texture.h:51-95)."""
    _fields_ = [("nx", ctypes.c_int32), ("ny", ctypes.c_int32), ("format", ctypes.c_int32),
                ("reserved", ctypes.c_int32), ("data", ctypes.c_void_p)]


def image_array(img):
    """(contiguous texel array, FRT_IMAGE_* format) of a spec image
    {"data": (ny, nx, 3) uint8 (sRGB, stb's LDR bytes) or float32 (HDR)}."""
    a = np.asarray(img["data"])
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError("image data must be (ny, nx, 3)")
    if a.dtype == np.uint8:
        return np.ascontiguousarray(a), FRT_IMAGE_SRGB8
    return np.ascontiguousarray(a, np.float32), FRT_IMAGE_F32


# cornell_box_obj's camera (main.cpp:236-242): lookfrom (0, 1, 3.9f), vfov 40, focus 10
CORNELL_CAMERA = {"lookfrom": (0.0, 1.0, float(np.float32(3.9))), "lookat": (0.0, 1.0, 0.0), "vup": (0.0, 1.0, 0.0),
                  "vfov": 40.0, "aperture": 0.0, "focus": 10.0}
MAT_TYPES = {"lambertian": 0, "diffuse_light": 1, "modified_phong": 2, "metal": 3, "dielectric": 4,
             "rough_conductor": 5}                      # FRT_MAT_*
DISTRIBUTIONS = {"ggx": 0, "beckmann": 1}               # FRT_DIST_*
SPHERE_WHERE = {"world": 1, "lights": 2, "both": 3}     # FRT_SPHERE_*


class SceneView(ctypes.Structure):
    _fields_ = [
        ("world_kind", ctypes.c_int32),
        ("n_tris", ctypes.c_int32),
        ("tri_v", ctypes.c_void_p), ("tri_n", ctypes.c_void_p), ("tri_material", ctypes.c_void_p),
        ("tri_geometry_normal", ctypes.c_void_p), ("tri_inv_area", ctypes.c_void_p),
        ("n_spheres", ctypes.c_int32), ("sphere", ctypes.c_void_p), ("sphere_material", ctypes.c_void_p),
        ("n_materials", ctypes.c_int32), ("materials", ctypes.c_void_p),
        ("n_nodes", ctypes.c_int32), ("root", ctypes.c_int32),
        ("node_box", ctypes.c_void_p), ("node_child", ctypes.c_void_p),
        ("n_list", ctypes.c_int32), ("list", ctypes.c_void_p),
        ("n_lights", ctypes.c_int32), ("lights", ctypes.c_void_p),
        ("cam_origin", ctypes.c_double * 3), ("cam_lower_left", ctypes.c_double * 3),
        ("cam_horizontal", ctypes.c_double * 3), ("cam_vertical", ctypes.c_double * 3),
        ("cam_u", ctypes.c_double * 3), ("cam_v", ctypes.c_double * 3),
        ("cam_lens_radius", ctypes.c_double),
        ("env_color", ctypes.c_double * 3),
        ("cam_w", ctypes.c_double * 3),
        ("cam_half_height", ctypes.c_double),
        ("tri_uv", ctypes.c_void_p),
        ("n_images", ctypes.c_int32), ("images", ctypes.c_void_p),
    ]


class RenderParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("nx", "ny", "spp")] + [("seed", ctypes.c_uint32)] + [
        (n, ctypes.c_int32) for n in ("max_depth", "integrator", "tile_size", "shard_index", "shard_count",
                                      "samples_per_item", "flags", "mlt_chains", "mlt_bootstrap", "sample_offset")]

    @classmethod
    def make(cls, nx, ny, spp, seed=0, max_depth=33, tile_size=32, shard_index=0, shard_count=1,
             samples_per_item=0, flags=0, integrator=0, sample_offset=0):
        """integrator: FRT_INTEGRATOR_PATH (path.cpp), _AO (ao.cpp) or _NORMALS (debug_renderer.h);
        sample_offset: first global sample index (progressive passes)."""
        return cls(nx=nx, ny=ny, spp=spp, seed=seed, max_depth=max_depth, integrator=integrator, tile_size=tile_size,
                   shard_index=shard_index, shard_count=shard_count, samples_per_item=samples_per_item, flags=flags,
                   mlt_chains=0, mlt_bootstrap=0, sample_offset=sample_offset)

    @classmethod
    def pssmlt(cls, nx, ny, mutations_per_pixel, chains, seed=0, bootstrap=10000, shard_index=0, shard_count=1,
               flags=0):
        """PSS-MLT (pssmlt.cpp): total mutations = mutations_per_pixel*nx*ny over `chains` chains."""
        return cls(nx=nx, ny=ny, spp=mutations_per_pixel, seed=seed, max_depth=10, integrator=FRT_INTEGRATOR_PSSMLT,
                   tile_size=32, shard_index=shard_index, shard_count=shard_count, samples_per_item=0, flags=flags,
                   mlt_chains=chains, mlt_bootstrap=bootstrap)


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("camera_rays", "extension_rays", "shadow_rays", "samples",
                                               "pixels", "work_items")] + [
        ("kernel_ms", ctypes.c_double), ("total_ms", ctypes.c_double)] + [
        (n, ctypes.c_uint32) for n in ("scene_in_lds", "waves_cap", "stack_entries", "bvh_depth")] + [
        ("scene_bytes", ctypes.c_uint64), ("fp64", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]

    @property
    def rays(self):
        return self.camera_rays + self.extension_rays + self.shadow_rays

    def as_dict(self):
        d = {n: getattr(self, n) for n, _ in self._fields_}
        d["rays"] = self.rays
        return d


class HostSceneInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in ("n_tris", "n_spheres", "n_materials", "n_lights", "n_nodes",
                                              "world_kind", "n_list", "bvh_depth")] + [
        ("load_ms", ctypes.c_double), ("build_ms", ctypes.c_double)]


_lib = None

# every symbol include/frt.h declares
EXPORTS = ("frt_get_abi_version", "frt_create", "frt_destroy", "frt_last_error", "frt_set_precision", "frt_upload_scene",
           "frt_shard_slot_count", "frt_shard_slots", "frt_render", "frt_render_multi", "frt_render_device", "frt_trace_device",
           "frt_mlt_chain_state",
           "frt_scene_create", "frt_scene_new", "frt_scene_add_obj", "frt_scene_add_sphere", "frt_scene_set_camera",
           "frt_scene_set_env", "frt_scene_add_image", "frt_scene_finish", "frt_scene_build_bvh_gpu",
           "frt_scene_build_bvh_sah", "frt_scene_build_bvh_gpu_algo",
           "frt_scene_view_get", "frt_scene_info", "frt_scene_destroy", "frt_write_tessellated_obj",
           "frt_write_pfm", "frt_film_accumulate", "frt_tonemap_u8", "frt_write_image", "frt_selftest_path_host",
           "frt_selftest_mlt_paths_host")


def lib():
    """Load libfrt.so (built in-tree by __graft_entry__.build()).  Raises if missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FrtError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same
    # soname as /opt/rocm's).  Load torch first so libfrt.so binds to that
    # copy; loading libfrt first would bind torch to the other runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    L.frt_get_abi_version.restype = ctypes.c_int
    if L.frt_get_abi_version() != ABI_VERSION:
        raise FrtError(f"{LIB_PATH}: ABI version {L.frt_get_abi_version()}, binding expects {ABI_VERSION}; rebuild")
    L.frt_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.frt_destroy.argtypes = [vp]
    L.frt_last_error.argtypes = [vp]
    L.frt_last_error.restype = ctypes.c_char_p
    L.frt_set_precision.argtypes = [vp, ctypes.c_int]
    L.frt_upload_scene.argtypes = [vp, ctypes.POINTER(SceneView)]
    L.frt_shard_slot_count.argtypes = [ctypes.POINTER(RenderParams)]
    L.frt_shard_slot_count.restype = ctypes.c_int64
    L.frt_shard_slots.argtypes = [ctypes.POINTER(RenderParams), vp]
    L.frt_render.argtypes = [vp, ctypes.POINTER(RenderParams), vp, ctypes.POINTER(Stats)]
    L.frt_render_device.argtypes = [vp, ctypes.POINTER(RenderParams), vp, vp, ctypes.POINTER(Stats)]
    L.frt_trace_device.argtypes = [vp, vp, ctypes.c_int64, vp, ctypes.c_int, vp, ctypes.POINTER(Stats)]
    L.frt_mlt_chain_state.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, vp, vp]
    L.frt_render_multi.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(RenderParams), vp,
                                   ctypes.POINTER(Stats)]
    L.frt_scene_create.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_double, ctypes.POINTER(vp)]
    L.frt_scene_view_get.argtypes = [vp, ctypes.POINTER(SceneView)]
    L.frt_scene_info.argtypes = [vp, ctypes.POINTER(HostSceneInfo)]
    L.frt_scene_destroy.argtypes = [vp]
    L.frt_scene_destroy.restype = None
    dp = ctypes.POINTER(ctypes.c_double)
    L.frt_scene_new.argtypes = [ctypes.POINTER(vp)]
    L.frt_scene_add_obj.argtypes = [vp, ctypes.c_char_p, dp, ctypes.POINTER(Material), ctypes.c_int]
    L.frt_scene_add_sphere.argtypes = [vp, dp, ctypes.c_double, ctypes.POINTER(Material), ctypes.c_int]
    L.frt_scene_set_camera.argtypes = [vp, dp, dp, dp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                       ctypes.c_double]
    L.frt_scene_set_env.argtypes = [vp, dp]
    L.frt_scene_add_image.argtypes = [vp, ctypes.POINTER(Image), ctypes.POINTER(ctypes.c_int)]
    L.frt_scene_finish.argtypes = [vp, ctypes.c_int]
    L.frt_scene_build_bvh_gpu.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_double)]
    L.frt_scene_build_bvh_sah.argtypes = [vp]
    L.frt_scene_build_bvh_gpu_algo.argtypes = [vp, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
    L.frt_write_tessellated_obj.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]
    L.frt_write_pfm.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, vp]
    L.frt_film_accumulate.argtypes = [vp, ctypes.c_int64, vp, ctypes.c_int64, ctypes.c_int64]
    L.frt_tonemap_u8.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    L.frt_write_image.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int]
    L.frt_selftest_path_host.argtypes = [ctypes.POINTER(SceneView), ctypes.POINTER(RenderParams), vp,
                                         ctypes.c_int, vp, ctypes.POINTER(Stats)]
    L.frt_selftest_mlt_paths_host.argtypes = [ctypes.POINTER(SceneView), ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                              ctypes.c_int, vp]
    _lib = L
    return L


def _check(rc, what, ctx=None):
    if rc != 0:
        msg = ""
        if ctx is not None:
            msg = lib().frt_last_error(ctx).decode(errors="replace")
        raise FrtError(f"{what} failed: {ERRORS.get(rc, rc)} {msg}")


class HostScene:
    """Scene built natively (main.cpp scene constructors + mesh_loader + create_bvh)."""

    def __init__(self, kind, obj_path, aspect):
        self.ptr = ctypes.c_void_p()
        _check(lib().frt_scene_create(kind.encode(), obj_path.encode(), float(aspect), ctypes.byref(self.ptr)),
               f"frt_scene_create({kind})")
        self.info = HostSceneInfo()
        lib().frt_scene_info(self.ptr, ctypes.byref(self.info))
        self.env = None

    def set_env(self, rgb):
        """Constant environment colour of the views this scene hands out
        (material.h:206-232; the reference scenes use black)."""
        self.env = tuple(float(x) for x in rgb)

    @classmethod
    def from_spec(cls, spec, aspect):
        """Build a scene the way main.cpp's scene functions do (frt_scene_new ...
        frt_scene_finish).  `spec`:
          {"objects": [{"obj": path, "to_world": 16 floats (row-major) | None,
                        "bsdf": material | None, "geo": use_geometry_normals},
                       {"sphere": (x, y, z), "radius": r, "material": material,
                        "where": "world" | "lights" | "both"}, ...],
           "camera": {"lookfrom", "lookat", "vup", "vfov", "aperture", "focus"},
           "world": "bvh" | "list", "env": (r, g, b) | None,
           "images": [{"data": (ny, nx, 3) uint8 sRGB | float32}, ...]}
        material: {"type": "lambertian" | "diffuse_light" | "modified_phong" |
                   "metal" | "dielectric" | "rough_conductor", "albedo", "emit",
                   "specular", "exponent", "ior", "alpha", "distribution":
                   "ggx" | "beckmann", "eta", "k", "checker": {"odd", "scale"},
                   "image": index into "images"}.
        oracle.OracleScene.from_spec builds the same scene in the oracle."""
        self = cls.__new__(cls)
        self.ptr = ctypes.c_void_p()
        self.env = None
        L = lib()
        _check(L.frt_scene_new(ctypes.byref(self.ptr)), "frt_scene_new")

        def dptr(x):
            a = np.ascontiguousarray(np.asarray(x, np.float64))
            return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
        for img in spec.get("images", ()):   # materials refer to them by index ({"image": i})
            a, fmt = image_array(img)
            desc = Image(a.shape[1], a.shape[0], fmt, 0, a.ctypes.data)
            idx = ctypes.c_int(-1)
            _check(L.frt_scene_add_image(self.ptr, ctypes.byref(desc), ctypes.byref(idx)), "frt_scene_add_image")
        for o in spec["objects"]:
            if "obj" in o:
                tw = dptr(o["to_world"]) if o.get("to_world") is not None else (None, None)
                bs = ctypes.byref(Material.from_spec(o["bsdf"])) if o.get("bsdf") is not None else None
                _check(L.frt_scene_add_obj(self.ptr, o["obj"].encode(), tw[1], bs, int(bool(o.get("geo", False)))),
                       f"frt_scene_add_obj({o['obj']})")
            else:
                c = dptr(o["sphere"])
                _check(L.frt_scene_add_sphere(self.ptr, c[1], float(o["radius"]),
                                              ctypes.byref(Material.from_spec(o["material"])),
                                              SPHERE_WHERE[o.get("where", "world")]), "frt_scene_add_sphere")
        cam = spec["camera"]
        f, a, u = dptr(cam["lookfrom"]), dptr(cam["lookat"]), dptr(cam.get("vup", (0, 1, 0)))
        _check(L.frt_scene_set_camera(self.ptr, f[1], a[1], u[1], float(cam["vfov"]), float(aspect),
                                      float(cam.get("aperture", 0.0)), float(cam.get("focus", 10.0))),
               "frt_scene_set_camera")
        if spec.get("env") is not None:
            e = dptr(spec["env"])
            _check(L.frt_scene_set_env(self.ptr, e[1]), "frt_scene_set_env")
        _check(L.frt_scene_finish(self.ptr, {"bvh": 0, "list": 1}[spec.get("world", "bvh")]), "frt_scene_finish")
        self.info = HostSceneInfo()
        L.frt_scene_info(self.ptr, ctypes.byref(self.info))
        return self

    def view(self):
        v = SceneView()
        _check(lib().frt_scene_view_get(self.ptr, ctypes.byref(v)), "frt_scene_view_get")
        if self.env is not None:
            v.env_color[:] = self.env
        return v

    def arrays(self):
        """numpy views of the flattened scene (copies)."""
        v = self.view()

        def arr(ptr, n, dt, w=1):
            if n == 0 or not ptr:
                return np.zeros((0, w) if w > 1 else 0, dt)
            a = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                      shape=(n * w,)).copy()
            return a.reshape(n, w) if w > 1 else a
        return {
            "tri_v": arr(v.tri_v, v.n_tris, np.float64, 9),
            "tri_material": arr(v.tri_material, v.n_tris, np.int32),
            "node_box": arr(v.node_box, v.n_nodes, np.float64, 6),
            "node_child": arr(v.node_child, v.n_nodes, np.int32, 2),
            "root": v.root,
            "lights": arr(v.lights, v.n_lights, np.int32),
            "list": arr(v.list, v.n_list, np.int32),
        }

    def build_bvh_sah(self):
        """Replace the world by a binned-SAH tree (frt_scene_build_bvh_sah); returns build ms."""
        _check(lib().frt_scene_build_bvh_sah(self.ptr), "frt_scene_build_bvh_sah")
        lib().frt_scene_info(self.ptr, ctypes.byref(self.info))
        return self.info.build_ms

    def build_bvh_gpu(self, ctx, algo="gsah"):
        """Replace the world by a GPU-built BVH (frt_scene_build_bvh_gpu_algo): "gsah"
        (top-down binned SAH, the default), "ploc" (PLOC clustering) or "lbvh" (Karras
        linear BVH); returns the device time of the build passes in ms."""
        ms = ctypes.c_double()
        a = {"ploc": FRT_GPU_BVH_PLOC, "lbvh": FRT_GPU_BVH_LBVH, "gsah": FRT_GPU_BVH_SAH}[algo]
        _check(lib().frt_scene_build_bvh_gpu_algo(self.ptr, ctx.ptr, a, ctypes.byref(ms)),
               "frt_scene_build_bvh_gpu_algo", ctx.ptr)
        lib().frt_scene_info(self.ptr, ctypes.byref(self.info))
        return ms.value

    def __del__(self):
        if getattr(self, "ptr", None):
            try:
                lib().frt_scene_destroy(self.ptr)
            except Exception:
                pass
            self.ptr = None


class Context:
    """One GPU (frt_ctx).  Raises FrtError when no gfx950 device is present."""

    def __init__(self, device=0, precision=None):
        self.ptr = ctypes.c_void_p()
        _check(lib().frt_create(int(device), ctypes.byref(self.ptr)), f"frt_create(device={device})")
        if precision is not None:
            self.set_precision(precision)

    def set_precision(self, precision):
        """FRT_PRECISION_AUTO / _FP32 / _FP64 (or "auto" / "fp32" / "fp64"); before upload()."""
        if isinstance(precision, str):
            precision = {"auto": FRT_PRECISION_AUTO, "fp32": FRT_PRECISION_FP32, "fp64": FRT_PRECISION_FP64}[precision]
        _check(lib().frt_set_precision(self.ptr, int(precision)), "frt_set_precision", self.ptr)

    def upload(self, scene):
        view = scene.view() if isinstance(scene, HostScene) else scene
        _check(lib().frt_upload_scene(self.ptr, ctypes.byref(view)), "frt_upload_scene", self.ptr)

    def render(self, params, film=None):
        """Render into a full film (nx*ny*3 float32, y=0 bottom row).  Returns (film, stats)."""
        if film is None:
            film = np.zeros((params.ny, params.nx, 3), np.float32)
        assert film.dtype == np.float32 and film.flags.c_contiguous and film.size == params.nx * params.ny * 3
        st = Stats()
        _check(lib().frt_render(self.ptr, ctypes.byref(params), film.ctypes.data, ctypes.byref(st)),
               "frt_render", self.ptr)
        return film, st

    def render_device(self, params, dev_ptr, stream_ptr=None):
        """Render this shard's slots into device memory at dev_ptr (slot_count*3 floats)."""
        st = Stats()
        _check(lib().frt_render_device(self.ptr, ctypes.byref(params), ctypes.c_void_p(dev_ptr),
                                       ctypes.c_void_p(stream_ptr) if stream_ptr else None, ctypes.byref(st)),
               "frt_render_device", self.ptr)
        return st

    def mlt_chain_state(self, first, n):
        """Local chains [first, first + n) of the last PSS-MLT render: (final
        states n x 92 float32, fingerprints n x 2 uint32 = accepted proposals,
        sum of the accepted steps' 1-based indices mod 2^32)."""
        u = np.zeros((max(n, 1), 92), np.float32)
        fp = np.zeros((max(n, 1), 2), np.uint32)
        _check(lib().frt_mlt_chain_state(self.ptr, int(first), int(n), u.ctypes.data, fp.ctypes.data),
               "frt_mlt_chain_state", self.ptr)
        return u[:n], fp[:n]

    def trace_device(self, rays_ptr, n, hits_ptr, flags=0, stream_ptr=None):
        """Batched Scene::world->hit on device buffers: rays n x 8 floats (origin, t_max,
        direction, flags bit 0 = any hit), hits n x 4 (t, u, v, prim bits).  Returns stats."""
        st = Stats()
        _check(lib().frt_trace_device(self.ptr, ctypes.c_void_p(rays_ptr), int(n), ctypes.c_void_p(hits_ptr), int(flags),
                                      ctypes.c_void_p(stream_ptr) if stream_ptr else None, ctypes.byref(st)),
               "frt_trace_device", self.ptr)
        return st

    def close(self):
        if getattr(self, "ptr", None):
            lib().frt_destroy(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_multi(contexts, params, film=None):
    """One process, several GPUs (frt_render_multi): contexts[i] renders shard
    (i, n) of the whole-frame `params` on its own host thread.  Returns (film, stats)."""
    if film is None:
        film = np.zeros((params.ny, params.nx, 3), np.float32)
    assert film.dtype == np.float32 and film.flags.c_contiguous and film.size == params.nx * params.ny * 3
    arr = (ctypes.c_void_p * len(contexts))(*[c.ptr for c in contexts])
    st = Stats()
    _check(lib().frt_render_multi(arr, len(contexts), ctypes.byref(params), film.ctypes.data, ctypes.byref(st)),
           "frt_render_multi", contexts[0].ptr)
    return film, st


def shard_slots(params):
    """Linear film index (y*nx+x) held by each output slot of a shard (-1 = padding)."""
    n = lib().frt_shard_slot_count(ctypes.byref(params))
    if n < 0:
        raise FrtError("bad render params")
    out = np.zeros(n, np.int32)
    _check(lib().frt_shard_slots(ctypes.byref(params), out.ctypes.data), "frt_shard_slots")
    return out


def selftest_path_host(scene, params, pixels):
    """Self-test hook: the megakernel's per-lane path code run on the host
    (CPU unit tests of the device logic; never a render path)."""
    pixels = np.ascontiguousarray(pixels, dtype=np.int32)
    out = np.zeros((len(pixels), 3), np.float32)
    st = Stats()
    view = scene.view()
    _check(lib().frt_selftest_path_host(ctypes.byref(view), ctypes.byref(params), pixels.ctypes.data, len(pixels),
                                        out.ctypes.data, ctypes.byref(st)), "frt_selftest_path_host")
    return out, st


def selftest_mlt_paths_host(scene, nx, ny, seed, n):
    """Self-test hook: n PSS-MLT bootstrap eye paths through the device code on the host."""
    out = np.zeros((n, 6), np.float32)
    view = scene.view()
    _check(lib().frt_selftest_mlt_paths_host(ctypes.byref(view), nx, ny, seed, n, out.ctypes.data),
           "frt_selftest_mlt_paths_host")
    return out


def write_pfm(path, film):
    film = np.ascontiguousarray(film, dtype=np.float32)
    ny, nx = film.shape[0], film.shape[1]
    _check(lib().frt_write_pfm(path.encode(), nx, ny, film.ctypes.data), "frt_write_pfm")


def film_accumulate(acc, acc_spp, film, spp):
    """Progressive accumulation (frt_film_accumulate): acc <- mean over acc_spp + spp samples."""
    acc = np.ascontiguousarray(acc, dtype=np.float32)
    film = np.ascontiguousarray(film, dtype=np.float32)
    _check(lib().frt_film_accumulate(acc.ctypes.data, int(acc_spp), film.ctypes.data, int(spp), film.size),
           "frt_film_accumulate")
    return acc


def tonemap_u8(film):
    """viewer::add_sample's display mapping (viewer.cpp:115-117) of a (ny, nx, 3) mean film."""
    film = np.ascontiguousarray(film, dtype=np.float32)
    ny, nx = film.shape[0], film.shape[1]
    out = np.zeros((ny, nx, 3), np.uint8)
    _check(lib().frt_tonemap_u8(film.ctypes.data, nx, ny, out.ctypes.data), "frt_tonemap_u8")
    return out


IMAGE_FORMATS = {"png": 0, "bmp": 1, "jpg": 2}


def write_image(path, rgb_u8, fmt="png"):
    """image::save_image (image.cpp:24-58) of a (ny, nx, 3) u8 image, y = 0 bottom."""
    rgb_u8 = np.ascontiguousarray(rgb_u8, dtype=np.uint8)
    ny, nx = rgb_u8.shape[0], rgb_u8.shape[1]
    _check(lib().frt_write_image(path.encode(), nx, ny, rgb_u8.ctypes.data, IMAGE_FORMATS[fmt]), "frt_write_image")


def work_granule(integrator, spp, n_slots, lanes, spi_req=0):
    """The render's work granule rule (frt_render.hip work_granule; an internal
    symbol of libfrt.so, for host tests): (samples per item, chunks)."""
    L = lib()
    f = L.frt_internal_work_granule
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    spi, k = ctypes.c_int(0), ctypes.c_int(0)
    _check(f(integrator, spp, n_slots, lanes, spi_req, ctypes.byref(spi), ctypes.byref(k)), "work_granule")
    return spi.value, k.value


def write_tessellated_obj(src_obj, k, dst_obj):
    _check(lib().frt_write_tessellated_obj(src_obj.encode(), int(k), dst_obj.encode()), "frt_write_tessellated_obj")
