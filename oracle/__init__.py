"""TEST INFRASTRUCTURE ONLY: ctypes bindings of the fp64 C restatement
(oracle/frt_oracle.c -> oracle/liboracle.so).

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker.  The product (first_raytracer_amd) never
imports this package.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_lib = None


class Counters(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "node_visits", "box_passes", "tri_tests", "sphere_tests",
        "camera_rays", "extension_rays", "shadow_rays", "samples")]

    @property
    def rays(self):
        return self.camera_rays + self.extension_rays + self.shadow_rays

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class SceneInfo(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n_tris", "n_spheres", "n_materials", "n_lights", "n_nodes", "world_kind", "n_list", "bvh_depth")]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle/liboracle.so missing: run `make -C oracle` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        L.ora_load_scene.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_double, ctypes.POINTER(ctypes.c_void_p)]
        L.ora_free_scene.argtypes = [ctypes.c_void_p]
        L.ora_scene_get_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(SceneInfo)]
        L.ora_scene_export_bvh.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.ora_scene_export_tris.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.ora_scene_export_camera.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.ora_scene_export_camera.restype = None
        L.ora_scene_export_lights.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.ora_scene_export_materials.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.ora_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint32,
                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(Counters)]
        L.ora_render_integrator.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.POINTER(Counters)]
        L.ora_render_depth.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.POINTER(Counters)]
        L.ora_scene_set_env.argtypes = [ctypes.c_void_p, dp]
        L.ora_scene_set_env.restype = None
        L.ora_scene_ao_tmax.argtypes = [ctypes.c_void_p]
        L.ora_scene_ao_tmax.restype = ctypes.c_double
        L.ora_world_hit.argtypes = [ctypes.c_void_p, dp, dp, ctypes.c_double, ctypes.c_double, dp,
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(Counters)]
        L.ora_rng_uniform.argtypes = [ctypes.c_uint32] * 4
        L.ora_rng_uniform.restype = ctypes.c_double
        L.ora_kat_tri_hit.argtypes = [dp, dp, ctypes.c_int, dp, dp, ctypes.c_double, ctypes.c_double, dp]
        L.ora_kat_sphere_hit.argtypes = [dp, ctypes.c_double, dp, dp, ctypes.c_double, ctypes.c_double, dp]
        L.ora_kat_texture_sphere.argtypes = [dp, ctypes.c_double, dp, dp, ctypes.c_double, ctypes.c_double, dp]
        L.ora_kat_texture_tri.argtypes = [dp, dp, dp, dp, ctypes.c_double, ctypes.c_double, dp]
        L.ora_kat_aabb_hit.argtypes = [dp, dp, dp, dp, ctypes.c_double, ctypes.c_double]
        L.ora_kat_camera.argtypes = [dp, dp, dp, ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, ctypes.c_double, dp, dp]
        L.ora_kat_cosine.argtypes = [dp, dp, dp]
        L.ora_kat_fresnel.argtypes = [dp, dp, ctypes.c_double, dp]
        L.ora_kat_phong.argtypes = [dp, dp, ctypes.c_double, ctypes.c_double, ctypes.c_double, dp, dp, dp, dp]
        L.ora_kat_dielectric.argtypes = [dp, dp, ctypes.c_double, ctypes.c_double, dp, dp, dp]
        L.ora_kat_tri_sample.argtypes = [dp, dp, ctypes.c_int, ctypes.c_int, dp, dp, dp]
        L.ora_kat_sphere_sample.argtypes = [dp, ctypes.c_double, dp, dp, dp]
        L.ora_kat_miweight.argtypes = [ctypes.c_double, ctypes.c_double]
        L.ora_kat_miweight.restype = ctypes.c_double
        L.ora_kat_fromsrgb.argtypes = [ctypes.c_double]
        L.ora_kat_fromsrgb.restype = ctypes.c_double
        L.ora_kat_atof.argtypes = [ctypes.c_char_p]
        L.ora_kat_atof.restype = ctypes.c_float
        L.ora_kat_pick.argtypes = [ctypes.c_double, ctypes.c_int]
        L.ora_kat_sort.argtypes = [dp, ctypes.c_int, ctypes.c_void_p]
        L.ora_kat_list_hit.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, dp]
        L.ora_mlt_bootstrap.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int]
        L.ora_mlt_bootstrap.restype = ctypes.c_double
        L.ora_mlt_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(Counters)]
        L.ora_mlt_render_shard.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(Counters),
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.ora_mlt_eye_path.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, dp, dp]
        L.ora_mlt_eye_path.restype = None
        L.ora_write_pfm.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, dp]
        L.ora_tonemap_u8.argtypes = [dp, ctypes.c_long, ctypes.c_void_p]
        L.ora_tonemap_u8.restype = None
        L.ora_kat_metal.argtypes = [dp, dp, dp, dp, dp]
        L.ora_kat_metal.restype = None
        L.ora_kat_conductor.argtypes = [dp, dp, ctypes.c_int, ctypes.c_double, dp, dp, dp, ctypes.c_double,
                                        ctypes.c_double, dp, dp]
        L.ora_kat_conductor.restype = None
        L.ora_scene_new.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        L.ora_scene_add_obj.argtypes = [ctypes.c_void_p, ctypes.c_char_p, dp, dp, ctypes.c_int]
        L.ora_scene_add_sphere.argtypes = [ctypes.c_void_p, dp, ctypes.c_double, dp, ctypes.c_int]
        L.ora_scene_add_image.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.POINTER(ctypes.c_int)]
        L.ora_image_lookup.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_double,
                                       ctypes.c_double, dp]
        L.ora_env_uv.argtypes = [dp, dp, dp]
        L.ora_env_uv.restype = None
        L.ora_scene_set_camera.argtypes = [ctypes.c_void_p, dp, dp, dp, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_double]
        L.ora_scene_set_camera.restype = None
        L.ora_scene_finish.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _lib = L
    return _lib


def darr(x):
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


MAT_TYPES = {"lambertian": 0, "diffuse_light": 1, "modified_phong": 2, "metal": 3, "dielectric": 4,
             "rough_conductor": 5}
DISTRIBUTIONS = {"ggx": 0, "beckmann": 1}
SPHERE_WHERE = {"world": 1, "lights": 2, "both": 3}


def material_desc(m):
    """The 26-double material description of frt_oracle.h from a scene-spec
    material dict (first_raytracer_amd.scene_spec documents the keys)."""
    d = np.zeros(27)
    d[0] = MAT_TYPES[m["type"]]
    d[1:4] = m.get("albedo", (0, 0, 0))
    d[4:7] = m.get("emit", (0, 0, 0))
    d[7:10] = m.get("specular", (0, 0, 0))
    d[10] = m.get("exponent", 0.0)
    d[11] = m.get("ior", 0.0)
    d[12] = DISTRIBUTIONS[m.get("distribution", "ggx").lower()]
    d[13] = m.get("alpha", 0.0)
    d[14:17] = m.get("eta", (0, 0, 0))
    d[17:20] = m.get("k", (0, 0, 0))
    if m.get("checker") is not None:
        d[20] = 1
        d[21:24] = m["checker"]["odd"]
        d[24:26] = m["checker"]["scale"]
    if m.get("image") is not None:               # image_texture: index into the spec's "images"
        d[20] = 2
        d[26] = m["image"]
    return d


class OracleScene:
    """Scene built by the restated reference constructors (main.cpp:222-314),
    or from a scene spec (OracleScene.from_spec)."""

    def __init__(self, kind, obj_path, aspect):
        self.ptr = ctypes.c_void_p()
        rc = lib().ora_load_scene(kind.encode(), obj_path.encode(), float(aspect), ctypes.byref(self.ptr))
        if rc != 0:
            raise RuntimeError(f"ora_load_scene({kind}, {obj_path}) failed: {rc}")
        self._refresh()

    def _refresh(self):
        self.info = SceneInfo()
        lib().ora_scene_get_info(self.ptr, ctypes.byref(self.info))

    @classmethod
    def from_spec(cls, spec, aspect):
        """Incremental construction like main.cpp's scene functions: OBJ files
        through create_triangle_mesh(file, toWorld, bsdf) (triangle.cpp:26-60),
        spheres, the camera, then create_bvh or a hitable_list."""
        self = cls.__new__(cls)
        self.ptr = ctypes.c_void_p()
        L = lib()
        if L.ora_scene_new(ctypes.byref(self.ptr)) != 0:
            raise RuntimeError("ora_scene_new failed")
        self._images = []
        for img in spec.get("images", ()):
            a = np.asarray(img["data"])
            a = np.ascontiguousarray(a) if a.dtype == np.uint8 else np.ascontiguousarray(a, np.float32)
            idx = ctypes.c_int(-1)
            if L.ora_scene_add_image(self.ptr, a.shape[1], a.shape[0], 0 if a.dtype == np.uint8 else 1,
                                     a.ctypes.data, ctypes.byref(idx)) != 0:
                raise RuntimeError("ora_scene_add_image failed")
            self._images.append(a)
        for o in spec["objects"]:
            if "obj" in o:
                tw = darr(o["to_world"]) if o.get("to_world") is not None else (None, None)
                bs = darr(material_desc(o["bsdf"])) if o.get("bsdf") is not None else (None, None)
                rc = L.ora_scene_add_obj(self.ptr, o["obj"].encode(), tw[1], bs[1], int(bool(o.get("geo", False))))
                if rc != 0:
                    raise RuntimeError(f"ora_scene_add_obj({o['obj']}) failed: {rc}")
            else:
                c = darr(o["sphere"]); m = darr(material_desc(o["material"]))
                L.ora_scene_add_sphere(self.ptr, c[1], float(o["radius"]), m[1], SPHERE_WHERE[o.get("where", "world")])
        cam = spec["camera"]
        f, a, u = darr(cam["lookfrom"]), darr(cam["lookat"]), darr(cam.get("vup", (0, 1, 0)))
        L.ora_scene_set_camera(self.ptr, f[1], a[1], u[1], float(cam["vfov"]), float(aspect),
                               float(cam.get("aperture", 0.0)), float(cam.get("focus", 10.0)))
        L.ora_scene_finish(self.ptr, {"bvh": 0, "list": 1}[spec.get("world", "bvh")])
        if spec.get("env") is not None:
            e = darr(spec["env"])
            L.ora_scene_set_env(self.ptr, e[1])
        self._refresh()
        return self

    def __del__(self):
        if getattr(self, "ptr", None) and lib is not None:
            try:
                lib().ora_free_scene(self.ptr)
            except Exception:
                pass
            self.ptr = None

    def bvh(self):
        n = self.info.n_nodes
        boxes = np.zeros((max(n, 1), 6)); left = np.zeros(max(n, 1), np.int32); right = np.zeros(max(n, 1), np.int32)
        lib().ora_scene_export_bvh(self.ptr, boxes.ctypes.data, left.ctypes.data, right.ctypes.data)
        return boxes[:n], left[:n], right[:n]

    def tris(self):
        n = self.info.n_tris
        v = np.zeros((max(n, 1), 9)); m = np.zeros(max(n, 1), np.int32)
        lib().ora_scene_export_tris(self.ptr, v.ctypes.data, m.ctypes.data)
        return v[:n], m[:n]

    def camera(self):
        out = np.zeros(19)
        lib().ora_scene_export_camera(self.ptr, out.ctypes.data)
        return out

    def lights(self):
        out = np.zeros(max(self.info.n_lights, 1), np.int32)
        lib().ora_scene_export_lights(self.ptr, out.ctypes.data)
        return out[:self.info.n_lights]

    def materials(self):
        out = np.zeros((max(self.info.n_materials, 1), 26))
        lib().ora_scene_export_materials(self.ptr, out.ctypes.data)
        return out[:self.info.n_materials]

    def set_env(self, rgb):
        """Constant environment colour (material.h:206-232)."""
        a, p = darr(rgb)
        lib().ora_scene_set_env(self.ptr, p)

    def ao_tmax(self):
        return lib().ora_scene_ao_tmax(self.ptr)

    def render(self, nx, ny, spp, seed=0, pixels=None, nthreads=None, integrator=0, max_depth=33):
        """Mean radiance per pixel (viewer::add_sample semantics) + counters.
        integrator: 0 path (path.cpp), 2 ao (ao.cpp), 3 normals (debug_renderer.h).
        max_depth: path::Li's depth cap (path.cpp:36)."""
        if pixels is None:
            pixels = np.arange(nx * ny, dtype=np.int32)
        pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        out = np.zeros((len(pixels), 3))
        cnt = Counters()
        nthreads = nthreads or min(16, os.cpu_count() or 1)
        rc = lib().ora_render_depth(self.ptr, integrator, nx, ny, spp, seed, max_depth, pixels.ctypes.data,
                                    len(pixels), nthreads, out.ctypes.data, ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError(f"ora_render failed: {rc}")
        return out, cnt

    def mlt_render(self, nx, ny, n_chains, steps, seed=0, n_init=10000, nthreads=None):
        """PSS-MLT film (pssmlt.cpp:301-365), mean-radiance scale; returns (film, b, counters)."""
        film = np.zeros((ny, nx, 3))
        b = ctypes.c_double()
        cnt = Counters()
        nthreads = nthreads or min(16, os.cpu_count() or 1)
        rc = lib().ora_mlt_render(self.ptr, nx, ny, seed, n_init, n_chains, steps, nthreads, film.ctypes.data,
                                  ctypes.byref(b), ctypes.byref(cnt))
        if rc != 0:
            raise RuntimeError(f"ora_mlt_render failed: {rc}")
        return film, b.value, cnt

    def mlt_render_shard(self, nx, ny, n_chains, steps, shard_index, shard_count, seed=0, n_init=10000,
                         nthreads=None):
        """The chains c = shard_index + j * shard_count of an n_chains PSS-MLT
        render (the GPU's shard rule): (film, b, counters, fingerprints, final
        states).  fingerprints[j] = (accepted proposals, sum of the accepted
        steps' 1-based indices mod 2^32); states[j] = the chain's final 92
        primary samples."""
        n_local = (n_chains - 1 - shard_index) // shard_count + 1 if shard_index < n_chains else 0
        film = np.zeros((ny, nx, 3))
        fp = np.zeros((max(n_local, 1), 2), np.uint32)
        u = np.zeros((max(n_local, 1), 92))
        b = ctypes.c_double()
        cnt = Counters()
        nthreads = nthreads or min(16, os.cpu_count() or 1)
        rc = lib().ora_mlt_render_shard(self.ptr, nx, ny, seed, n_init, n_chains, steps, shard_index, shard_count,
                                        nthreads, film.ctypes.data, ctypes.byref(b), ctypes.byref(cnt),
                                        fp.ctypes.data, u.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"ora_mlt_render_shard failed: {rc}")
        return film, b.value, cnt, fp[:n_local], u[:n_local]

    def mlt_bootstrap(self, nx, ny, seed=0, n_init=10000):
        return lib().ora_mlt_bootstrap(self.ptr, nx, ny, seed, n_init)

    def world_hit(self, o, d, tmin, tmax):
        oa, op = darr(o); da, dptr = darr(d)
        t = ctypes.c_double(); prim = ctypes.c_int32(); cnt = Counters()
        ok = lib().ora_world_hit(self.ptr, op, dptr, tmin, tmax, ctypes.byref(t), ctypes.byref(prim), ctypes.byref(cnt))
        return bool(ok), t.value, prim.value, cnt


def rng_uniform(seed, pixel, sample, dim):
    return lib().ora_rng_uniform(seed, pixel, sample, dim)

