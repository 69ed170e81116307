// frt_integrator.hpp -- C++ host API over the C-ABI (include/frt.h) that keeps
// the reference's integrator concept, so code written against
//   template <class I> struct renderer : I { double Render(Scene*, viewer&); }  (integrator.h:11-47)
//   struct path { void Render(Scene*, viewer*, ...); using_custom_viewer; }      (path.h:8-18)
//   struct viewer { add_sample(...); save_and_destroy(...); }                     (viewer.h:9-26)
// reads the same against frt::renderer<frt::path_gpu>.  Errors become
// exceptions (frt::error), as the reference throws std::runtime_error.
#pragma once
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "frt.h"

namespace frt {

struct error : std::runtime_error {
    int code;
    error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

inline void check(int rc, const char *what, const frt_ctx *ctx = nullptr)
{
    if (rc != FRT_OK)
        throw error(rc, std::string(what) + " failed (" + std::to_string(rc) + ")" +
                            (ctx ? std::string(": ") + frt_last_error(ctx) : std::string()));
}

// Scene (Scene.h:10-26): world + lights + camera + environment, built natively
// by the reference's scene constructors (main.cpp:222-252, 281-314).
class Scene {
public:
    Scene(const std::string &kind, const std::string &obj_path, double aspect)
    {
        frt_host_scene *s = nullptr;
        check(frt_scene_create(kind.c_str(), obj_path.c_str(), aspect, &s), "frt_scene_create");
        scene_.reset(s);
        check(frt_scene_info(s, &info_), "frt_scene_info");
    }
    static Scene cornell_box_obj(const std::string &obj, double aspect) { return Scene("cornell_box_obj", obj, aspect); }
    static Scene veach_mis(const std::string &obj, double aspect) { return Scene("veach_mis", obj, aspect); }

    frt_scene_view view() const
    {
        frt_scene_view v;
        check(frt_scene_view_get(scene_.get(), &v), "frt_scene_view_get");
        if (has_env_)
            for (int k = 0; k < 3; ++k) v.env_color[k] = env_[k];
        return v;
    }
    // Scene::env_map with another constant colour (material.h:206-232)
    void set_env(double r, double g, double b) { env_[0] = r; env_[1] = g; env_[2] = b; has_env_ = true; }
    // replace the reference-topology BVH: binned SAH on the host, or the GPU
    // linear BVH on ctx's device (frt_scene_build_bvh_sah / _gpu)
    void build_bvh_sah()
    {
        check(frt_scene_build_bvh_sah(scene_.get()), "frt_scene_build_bvh_sah");
        check(frt_scene_info(scene_.get(), &info_), "frt_scene_info");
    }
    void build_bvh_gpu(frt_ctx *ctx)
    {
        check(frt_scene_build_bvh_gpu(scene_.get(), ctx, nullptr), "frt_scene_build_bvh_gpu", ctx);
        check(frt_scene_info(scene_.get(), &info_), "frt_scene_info");
    }
    const frt_host_scene_info &info() const { return info_; }

private:
    double env_[3] = {0, 0, 0};
    bool has_env_ = false;
    struct del { void operator()(frt_host_scene *s) const { frt_scene_destroy(s); } };
    std::unique_ptr<frt_host_scene, del> scene_;
    frt_host_scene_info info_{};
};

// viewer (viewer.h:9-26, viewer.cpp:109-140) without the GL window: the linear
// film (fout_image, doubles) and the tonemapped u8 image (out_image).
struct viewer {
    viewer(int nx, int ny, uint64_t ns, int num_channels = 3)
        : nx(nx), ny(ny), ns(ns), num_channels(num_channels), out_image((size_t)nx * ny * num_channels, 0),
          fout_image((size_t)nx * ny * num_channels, 0.0)
    {
    }
    // add_sample(pixel, sum) (viewer.cpp:109-132): sum *= 1/ns, store linear + tonemapped
    void add_sample(int x, int y, double r, double g, double b)
    {
        const double k = 1.0 / double(ns);
        store_mean(x, y, r * k, g * k, b * k);
    }
    // the GPU already returns the per-pixel mean (sum * 1/ns)
    void store_mean(int x, int y, double fr, double fg, double fb)
    {
        const size_t idx = ((size_t)y * nx + x) * num_channels;
        out_image[idx] = (uint8_t)int(std::pow(1 - std::exp(-fr), 1 / 2.2) * 255 + .5);
        out_image[idx + 1] = (uint8_t)int(std::pow(1 - std::exp(-fg), 1 / 2.2) * 255 + .5);
        out_image[idx + 2] = (uint8_t)int(std::pow(1 - std::exp(-fb), 1 / 2.2) * 255 + .5);
        fout_image[idx] = fr;
        fout_image[idx + 1] = fg;
        fout_image[idx + 2] = fb;
    }
    // image_pfm::save_image layout (image.h:89-118); path used as given (no $HOME prefix)
    void save_pfm(const std::string &path) const
    {
        std::vector<float> f(fout_image.begin(), fout_image.end());
        check(frt_write_pfm(path.c_str(), nx, ny, f.data()), "frt_write_pfm");
    }
    // image::save_image of out_image (image.cpp:24-58): FRT_IMAGE_PNG / _BMP / _JPG (BMP bytes, as the
    // reference's switch writes); path used as given, extension appended when missing
    void save_image(const std::string &path, int format = FRT_IMAGE_PNG) const
    {
        check(frt_write_image(path.c_str(), nx, ny, out_image.data(), format), "frt_write_image");
    }
    // a whole mean film at once (the GPU path): linear film + display bytes (frt_tonemap_u8)
    void store_film(const float *rgb)
    {
        for (size_t i = 0; i < fout_image.size(); ++i) fout_image[i] = rgb[i];
        check(frt_tonemap_u8(rgb, nx, ny, out_image.data()), "frt_tonemap_u8");
    }
    const int nx, ny;
    const uint64_t ns;
    const int num_channels;
    bool to_exit = false;
    std::vector<uint8_t> out_image;
    std::vector<double> fout_image;
};

// One frt_ctx per listed device with the scene uploaded (uploads run in
// parallel, one host thread per device).
class device_set {
public:
    device_set(const std::vector<int> &devices, const frt_scene_view &view) : ctx_(devices.size(), nullptr)
    {
        std::vector<std::string> errs(devices.size());
        auto up = [&](size_t i) {
            try {
                check(frt_create(devices[i], &ctx_[i]), "frt_create");
                check(frt_upload_scene(ctx_[i], &view), "frt_upload_scene", ctx_[i]);
            } catch (const std::exception &e) {
                errs[i] = e.what();
            }
        };
        std::vector<std::thread> th;
        for (size_t i = 1; i < devices.size(); ++i) th.emplace_back(up, i);
        if (!devices.empty()) up(0);
        for (auto &t : th) t.join();
        for (const std::string &e : errs)
            if (!e.empty()) { release(); throw error(FRT_E_HIP, e); }
    }
    ~device_set() { release(); }
    device_set(const device_set &) = delete;
    device_set &operator=(const device_set &) = delete;
    frt_ctx **data() { return ctx_.data(); }
    int size() const { return (int)ctx_.size(); }

private:
    void release()
    {
        for (frt_ctx *&c : ctx_)
            if (c) { frt_destroy(c); c = nullptr; }
    }
    std::vector<frt_ctx *> ctx_;
};

// tile_gpu<I>: the drop-ins for the per-pixel integrators -- path_gpu for
// `path` (path.h:8-18), ao_gpu for `ao` (ao.h:8-43), normals_gpu for
// `normals_renderer` (debug_renderer.h:6-50).  Render() renders the frame on
// the listed GPUs with frt_render_multi (tile t -> device t % n) and stores
// the per-pixel means in the viewer.
template <int INTEGRATOR>
struct tile_gpu {
    std::vector<int> devices{0};
    uint32_t seed = 0;
    int max_depth = 33;     // path.cpp:36
    int tile_size = 32;
    frt_stats last_stats{};
    static constexpr bool using_custom_viewer = false;

    void Render(Scene *scene, viewer *film)
    {
        device_set gpus(devices, scene->view());
        frt_render_params p{};
        p.nx = film->nx; p.ny = film->ny; p.spp = (int)film->ns; p.seed = seed;
        p.max_depth = max_depth; p.integrator = INTEGRATOR; p.tile_size = tile_size;
        p.shard_index = 0; p.shard_count = 1;
        std::vector<float> rgb((size_t)film->nx * film->ny * 3, 0.0f);
        check(frt_render_multi(gpus.data(), gpus.size(), &p, rgb.data(), &last_stats), "frt_render_multi",
              gpus.data()[0]);
        for (int y = 0; y < film->ny; ++y)
            for (int x = 0; x < film->nx; ++x) {
                const float *px = &rgb[3 * ((size_t)y * film->nx + x)];
                film->store_mean(x, y, px[0], px[1], px[2]);
            }
    }
};

using path_gpu = tile_gpu<FRT_INTEGRATOR_PATH>;
using ao_gpu = tile_gpu<FRT_INTEGRATOR_AO>;
using normals_gpu = tile_gpu<FRT_INTEGRATOR_NORMALS>;

// pssmlt_gpu: the drop-in for `pssmlt` (pssmlt.h:20-76) -- Kelemen PSS-MLT with
// film->ns mutations per pixel over `chains` GPU chains (chain c -> device
// c % n).  The splat film is the image (AccumulatePathContribution).
struct pssmlt_gpu {
    std::vector<int> devices{0};
    uint32_t seed = 0;
    int chains = 1 << 18;
    int bootstrap = 10000;  // pssmlt.cpp:303
    frt_stats last_stats{};
    static constexpr bool using_custom_viewer = false;

    void Render(Scene *scene, viewer *film)
    {
        device_set gpus(devices, scene->view());
        frt_render_params p{};
        p.nx = film->nx; p.ny = film->ny; p.spp = (int)film->ns; p.seed = seed;
        p.max_depth = 10; p.integrator = FRT_INTEGRATOR_PSSMLT; p.tile_size = 32;
        p.shard_index = 0; p.shard_count = 1; p.mlt_chains = chains; p.mlt_bootstrap = bootstrap;
        std::vector<float> rgb((size_t)film->nx * film->ny * 3, 0.0f);
        check(frt_render_multi(gpus.data(), gpus.size(), &p, rgb.data(), &last_stats), "frt_render_multi",
              gpus.data()[0]);
        for (int y = 0; y < film->ny; ++y)
            for (int x = 0; x < film->nx; ++x) {
                const float *px = &rgb[3 * ((size_t)y * film->nx + x)];
                film->store_mean(x, y, px[0], px[1], px[2]);
            }
    }
};

// renderer<I> (integrator.h:11-47): time I::Render, print the statistics the
// reference prints -- with true 64-bit ray counts instead of node visits.
template <typename integrator>
struct renderer : public integrator {
    double Render(Scene *scene, viewer &film)
    {
        const auto t1 = std::chrono::high_resolution_clock::now();
        integrator::Render(scene, &film);
        const auto t2 = std::chrono::high_resolution_clock::now();
        const double secs = std::chrono::duration<double>(t2 - t1).count();
        const frt_stats &s = integrator::last_stats;
        const double rays = double(s.camera_rays + s.extension_rays + s.shadow_rays);
        std::printf("\nIt took me %g seconds to render.\n", secs);
        std::printf(" Camera rays: %llu\n Extension rays: %llu\n Shadow rays: %llu\n",
                    (unsigned long long)s.camera_rays, (unsigned long long)s.extension_rays,
                    (unsigned long long)s.shadow_rays);
        std::printf(" Kernel time: %.3f ms\n Rays/second: %.1fM/sec (kernel %.1fM/sec)\n", s.kernel_ms,
                    rays / secs / 1e6, rays / (s.kernel_ms * 1e-3) / 1e6);
        return secs;
    }
};

}  // namespace frt
