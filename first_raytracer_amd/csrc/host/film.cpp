// film.cpp -- the output side of the renderer (what viewer::add_sample,
// viewer::save_and_destroy and image::save_image do in the reference,
// viewer.cpp:109-132, image.cpp:24-58): progressive accumulation of passes,
// the display tonemap and the PNG / BMP writers (zlib deflate for PNG).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <zlib.h>

#include "frt.h"

namespace {

// rows [y0, y1) of a parallel loop over the host's cores (output formatting
// of a 1080p film is 6 M pow/exp: ~60 ms on one core)
template <class F>
void parallel_rows(int ny, F f)
{
    const int nt = std::max(1, std::min((int)std::thread::hardware_concurrency(), 16));
    if (nt == 1 || ny < 64) { f(0, ny); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back([&, t] { f(ny * t / nt, ny * (t + 1) / nt); });
    for (auto &x : th) x.join();
}

void put32be(std::vector<uint8_t> &v, uint32_t x)
{
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16)); v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}
void put_le(std::vector<uint8_t> &v, uint32_t x, int n)
{
    for (int i = 0; i < n; ++i) v.push_back((uint8_t)(x >> (8 * i)));
}
void chunk(std::vector<uint8_t> &out, const char *type, const std::vector<uint8_t> &data)
{
    put32be(out, (uint32_t)data.size());
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    put32be(out, (uint32_t)crc32(0L, out.data() + at, (uInt)(out.size() - at)));
}

// rows top-down (stbi_flip_vertically_on_write(true), image.cpp:30): row r of
// the file is film row ny-1-r
bool png_bytes(int nx, int ny, const uint8_t *rgb, std::vector<uint8_t> &out)
{
    std::vector<uint8_t> raw((size_t)ny * (1 + 3 * (size_t)nx));
    for (int r = 0; r < ny; ++r) {
        uint8_t *d = &raw[(size_t)r * (1 + 3 * (size_t)nx)];
        d[0] = 0;                                                          // filter: none
        memcpy(d + 1, rgb + (size_t)(ny - 1 - r) * nx * 3, 3 * (size_t)nx);
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return false;
    z.resize(zlen);
    const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    out.assign(sig, sig + 8);
    std::vector<uint8_t> ihdr;
    put32be(ihdr, (uint32_t)nx); put32be(ihdr, (uint32_t)ny);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});                              // 8-bit RGB
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    return true;
}

// 24-bit BMP: bottom-up rows (the native BMP order) of the top-down image,
// i.e. film row y at file row y; BGR, rows padded to 4 bytes
void bmp_bytes(int nx, int ny, const uint8_t *rgb, std::vector<uint8_t> &out)
{
    const uint32_t row = (3u * (uint32_t)nx + 3u) & ~3u, img = row * (uint32_t)ny;
    out.clear();
    out.push_back('B'); out.push_back('M');
    put_le(out, 54 + img, 4); put_le(out, 0, 4); put_le(out, 54, 4);
    put_le(out, 40, 4); put_le(out, (uint32_t)nx, 4); put_le(out, (uint32_t)ny, 4);
    put_le(out, 1, 2); put_le(out, 24, 2); put_le(out, 0, 4); put_le(out, img, 4);
    put_le(out, 0, 4); put_le(out, 0, 4); put_le(out, 0, 4); put_le(out, 0, 4);
    for (int y = 0; y < ny; ++y) {
        const uint8_t *s = rgb + (size_t)y * nx * 3;
        for (int x = 0; x < nx; ++x) { out.push_back(s[3 * x + 2]); out.push_back(s[3 * x + 1]); out.push_back(s[3 * x]); }
        for (uint32_t p = 3u * (uint32_t)nx; p < row; ++p) out.push_back(0);
    }
}

bool ends_with(const std::string &s, const char *suf)
{
    return s.find(suf) != std::string::npos;   // image.cpp:42: filename.find(".png") == npos -> append
}

}  // namespace

extern "C" int frt_film_accumulate(float *acc, int64_t acc_spp, const float *pass, int64_t pass_spp, int64_t n)
{
    if (!acc || !pass || n < 0 || acc_spp < 0 || pass_spp <= 0) return FRT_E_INVALID;
    const double tot = (double)acc_spp + (double)pass_spp;
    const double wa = (double)acc_spp / tot, wp = (double)pass_spp / tot;
    for (int64_t i = 0; i < n; ++i) acc[i] = (float)(wa * (double)acc[i] + wp * (double)pass[i]);
    return FRT_OK;
}

extern "C" int frt_tonemap_u8(const float *rgb, int nx, int ny, uint8_t *out)
{
    if (!rgb || !out || nx <= 0 || ny <= 0) return FRT_E_INVALID;
    parallel_rows(ny, [&](int y0, int y1) {
        for (size_t i = (size_t)y0 * nx * 3; i < (size_t)y1 * nx * 3; ++i) {
            const double f = rgb[i];                                       // viewer.cpp:115-117
            out[i] = (uint8_t)(int)(std::pow(1 - std::exp(-f), 1 / 2.2) * 255 + .5);
        }
    });
    return FRT_OK;
}

extern "C" int frt_write_image(const char *path, int nx, int ny, const uint8_t *rgb, int format)
{
    if (!path || !rgb || nx <= 0 || ny <= 0) return FRT_E_INVALID;
    std::string name = path;
    std::vector<uint8_t> bytes;
    switch (format) {
    case FRT_IMAGE_PNG:
        if (!ends_with(name, ".png")) name += ".png";
        if (!png_bytes(nx, ny, rgb, bytes)) return FRT_E_IO;
        break;
    case FRT_IMAGE_BMP:
        if (!ends_with(name, ".bmp")) name += ".bmp";
        bmp_bytes(nx, ny, rgb, bytes);
        break;
    case FRT_IMAGE_JPG:                                                    // image.cpp:40-43: BMP bytes, ".jpg"
        if (!ends_with(name, ".jpg")) name += ".jpg";
        bmp_bytes(nx, ny, rgb, bytes);
        break;
    default:
        return FRT_E_UNSUPPORTED;
    }
    FILE *f = fopen(name.c_str(), "wb");
    if (!f) return FRT_E_IO;
    const bool ok = fwrite(bytes.data(), 1, bytes.size(), f) == bytes.size();
    return (fclose(f) == 0 && ok) ? FRT_OK : FRT_E_IO;
}
