// frt_render -- command-line renderer: the reference's main() (main.cpp:483-525)
// with the scene, resolution, spp, seed and GPU count as flags instead of
// compile-time choices.  Writes the linear film as PFM (image.h:89-118).
//
//   frt_render --scene cornell|veach|obj --obj FILE [--res 1920x1080] [--ns 512]
//              [--seed 0] [--gpus 1] [--integrator path|pssmlt|ao|normals] [--chains 262144]
//              [--env r,g,b] [--out out.pfm] [--png out.png] [--bvh reference|sah]
//
// --integrator pssmlt: renderer<pssmlt_gpu>, --ns = mutations per pixel.
// --integrator ao / normals: renderer<ao_gpu> / renderer<normals_gpu> (ao.h, debug_renderer.h).
// --env: constant environment colour (the reference scenes' is black).
// --png: also the tonemapped display image (viewer::add_sample bytes, image::save_image).
// --bvh sah: rebuild the scene's BVH with the binned SAH builder (faster traversal;
//   exact-t ties then follow that tree's order instead of create_bvh's).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "frt_integrator.hpp"

int main(int argc, char **argv)
{
    std::string scene = "cornell", obj, out = "out.pfm", integrator = "path", png, bvh = "reference";
    int nx = 512, ny = 512, gpus = 1, chains = 1 << 18;
    long ns = 100;
    unsigned seed = 0;
    double env[3] = {0, 0, 0};
    bool has_env = false;
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--scene") scene = next();
        else if (a == "--obj") obj = next();
        else if (a == "--res") { if (std::sscanf(next(), "%dx%d", &nx, &ny) != 2) return 2; }
        else if (a == "--ns") ns = std::atol(next());
        else if (a == "--seed") seed = (unsigned)std::strtoul(next(), nullptr, 10);
        else if (a == "--gpus") gpus = std::atoi(next());
        else if (a == "--out") out = next();
        else if (a == "--png") png = next();
        else if (a == "--bvh") bvh = next();
        else if (a == "--integrator") integrator = next();
        else if (a == "--chains") chains = std::atoi(next());
        else if (a == "--env") {
            if (std::sscanf(next(), "%lf,%lf,%lf", &env[0], &env[1], &env[2]) != 3) return 2;
            has_env = true;
        }
        else { std::fprintf(stderr, "unknown flag %s\n", a.c_str()); return 2; }
    }
    if (obj.empty()) { std::fprintf(stderr, "--obj is required\n"); return 2; }
    try {
        std::printf("Resolution: %dx%d\nSetting number of samples to %ld\n", nx, ny, ns);
        const std::string kind = scene == "cornell" ? "cornell_box_obj" : scene == "veach" ? "veach_mis" : "obj_smooth";
        frt::Scene s(kind, obj, double(nx) / double(ny));
        if (has_env) s.set_env(env[0], env[1], env[2]);
        if (bvh == "sah") s.build_bvh_sah();
        else if (bvh != "reference") { std::fprintf(stderr, "unknown --bvh %s\n", bvh.c_str()); return 2; }
        std::printf("BVH construction took me %g seconds (%d triangles, depth %d).\n", s.info().build_ms * 1e-3,
                    s.info().n_tris, s.info().bvh_depth);
        frt::viewer film(nx, ny, (uint64_t)ns);
        auto run = [&](auto &render) {
            render.devices.clear();
            for (int g = 0; g < gpus; ++g) render.devices.push_back(g);
            render.seed = seed;
            render.Render(&s, film);
        };
        if (integrator == "pssmlt") {
            frt::renderer<frt::pssmlt_gpu> render;
            render.chains = chains;
            run(render);
        } else if (integrator == "path") {
            frt::renderer<frt::path_gpu> render;
            run(render);
        } else if (integrator == "ao") {
            frt::renderer<frt::ao_gpu> render;
            run(render);
        } else if (integrator == "normals") {
            frt::renderer<frt::normals_gpu> render;
            run(render);
        } else {
            std::fprintf(stderr, "unknown integrator %s\n", integrator.c_str());
            return 2;
        }
        film.save_pfm(out);
        std::printf("Saved %s\n", out.c_str());
        if (!png.empty()) {
            film.save_image(png, FRT_IMAGE_PNG);
            std::printf("Saved %s\n", png.c_str());
        }
    } catch (const std::exception &e) {
        std::fprintf(stderr, "frt_render: %s\n", e.what());
        return 1;
    }
    return 0;
}
