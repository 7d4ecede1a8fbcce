// orbfe_png.cpp — image ingest of the front-end: PNG decode to 8-bit grayscale, the reference's
// cv2.imread(path, cv2.IMREAD_GRAYSCALE) (stereo_kitti.py:42-43), natively (zlib inflate + PNG row
// unfiltering), one image per call or a batch of files decoded by a pool of host threads straight into one
// caller buffer (the batched-frames mode's host staging before a single host-to-device copy).
//
// Supported: bit depth 8, colour types 0 (grey), 2 (RGB), 4 (grey + alpha), 6 (RGBA), non-interlaced.  Grey
// images are returned as stored (lossless: exact).  Colour images are converted like OpenCV's PNG decoder
// asks libpng to (png_set_rgb_to_gray with 0.299 / 0.587: libpng's truncated 15-bit fixed-point weights
// 9797, 19234, 3737 and a truncating >> 15, no gamma), alpha dropped — parity of that branch is unpinned (OpenCV / libpng headers
// are absent here).  Anything else is ORBFE_EFORMAT.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "orbfe_host_util.h"

using namespace orbfe;

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

struct PngInfo {
    int w = 0, h = 0, ctype = 0, channels = 0;
    std::vector<uint8_t> idat;  // concatenated IDAT payload (zlib stream)
};

PngInfo parse(const uint8_t* d, size_t n) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (n < 8 || std::memcmp(d, sig, 8) != 0) throw Error(ORBFE_EFORMAT, "not a PNG file");
    PngInfo info;
    bool have_ihdr = false, have_iend = false;
    size_t i = 8;
    while (i + 12 <= n && !have_iend) {
        const uint32_t len = be32(d + i);
        const uint8_t* type = d + i + 4;
        if (len > n - i - 12) throw Error(ORBFE_EFORMAT, "truncated PNG chunk");
        const uint8_t* body = d + i + 8;
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len != 13) throw Error(ORBFE_EFORMAT, "bad IHDR");
            info.w = (int)be32(body);
            info.h = (int)be32(body + 4);
            const int depth = body[8];
            info.ctype = body[9];
            if (depth != 8) throw Error(ORBFE_EFORMAT, "only 8-bit PNG images are supported");
            if (body[10] != 0 || body[11] != 0) throw Error(ORBFE_EFORMAT, "unknown PNG compression / filter method");
            if (body[12] != 0) throw Error(ORBFE_EFORMAT, "interlaced PNG images are not supported");
            switch (info.ctype) {
                case 0: info.channels = 1; break;
                case 2: info.channels = 3; break;
                case 4: info.channels = 2; break;
                case 6: info.channels = 4; break;
                default: throw Error(ORBFE_EFORMAT, "unsupported PNG colour type (palette)");
            }
            if (info.w <= 0 || info.h <= 0 || info.w > (1 << 16) || info.h > (1 << 16))
                throw Error(ORBFE_EFORMAT, "PNG size out of range");
            have_ihdr = true;
        } else if (!std::memcmp(type, "IDAT", 4)) {
            info.idat.insert(info.idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            have_iend = true;
        }
        i += 12 + len;
    }
    if (!have_ihdr || info.idat.empty()) throw Error(ORBFE_EFORMAT, "PNG without IHDR / IDAT");
    return info;
}

inline uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (uint8_t)(pa <= pb && pa <= pc ? a : (pb <= pc ? b : c));
}

// Decode into out (w x h grey, row stride `stride`).
void decode(const uint8_t* data, size_t size, uint8_t* out, int64_t stride, int* w_out, int* h_out, bool size_only) {
    PngInfo info = parse(data, size);
    *w_out = info.w;
    *h_out = info.h;
    if (size_only) return;
    const int bpp = info.channels;
    const size_t row = (size_t)info.w * bpp;
    std::vector<uint8_t> raw((row + 1) * info.h);
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) throw Error(ORBFE_ENOMEM, "inflateInit failed");
    zs.next_in = info.idat.data();
    zs.avail_in = (uInt)info.idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int rc = inflate(&zs, Z_FINISH);
    const size_t got = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((rc != Z_STREAM_END && rc != Z_OK && rc != Z_BUF_ERROR) || got != raw.size())
        throw Error(ORBFE_EFORMAT, "corrupt PNG image data");
    std::vector<uint8_t> prev(row, 0), cur(row);
    for (int y = 0; y < info.h; ++y) {
        const uint8_t f = raw[(row + 1) * y];
        const uint8_t* src = &raw[(row + 1) * y + 1];
        for (size_t x = 0; x < row; ++x) {
            const int a = x >= (size_t)bpp ? cur[x - bpp] : 0, b = prev[x], c = x >= (size_t)bpp ? prev[x - bpp] : 0;
            int v = src[x];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: throw Error(ORBFE_EFORMAT, "bad PNG filter type");
            }
            cur[x] = (uint8_t)v;
        }
        uint8_t* o = out + (int64_t)y * stride;
        if (bpp == 1) {
            std::memcpy(o, cur.data(), info.w);
        } else if (bpp == 2) {
            for (int x = 0; x < info.w; ++x) o[x] = cur[2 * x];
        } else {
            // OpenCV's PNG decoder asks libpng for png_set_rgb_to_gray(png, 1, 0.299, 0.587):
            // png_set_rgb_to_gray_fixed truncates the coefficients to 15 bits (rc = 29900 * 32768 / 100000
            // = 9797, gc = 19234, bc = 32768 - rc - gc = 3737) and png_do_rgb_to_gray's 8-bit no-gamma path
            // truncates the sum ((rc R + gc G + bc B) >> 15; grey pixels pass unchanged, which the formula
            // also gives).  Parity unpinned: no colour fixture exists in the reference.
            for (int x = 0; x < info.w; ++x) {
                const uint8_t* p = &cur[(size_t)x * bpp];
                o[x] = (uint8_t)((9797u * p[0] + 19234u * p[1] + 3737u * p[2]) >> 15);
            }
        }
        std::swap(prev, cur);
    }
}

std::vector<uint8_t> read_file(const char* path) {
    FILE* f = std::fopen(path, "rb");
    if (!f) throw Error(ORBFE_EINVAL, std::string("cannot open ") + path);
    std::vector<uint8_t> d;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) d.insert(d.end(), buf, buf + k);
    std::fclose(f);
    return d;
}

}  // namespace

extern "C" {

int orbfe_png_decode(const uint8_t* data, int64_t size, uint8_t* out, int64_t stride, int32_t* width, int32_t* height) {
    return guarded([&] {
        if (!data || size <= 0 || !width || !height) throw Error(ORBFE_EINVAL, "null argument");
        int w = 0, h = 0;
        decode(data, (size_t)size, out, stride, &w, &h, true);
        *width = w;
        *height = h;
        if (!out) return;
        if (stride < w) throw Error(ORBFE_EINVAL, "stride smaller than the image width");
        decode(data, (size_t)size, out, stride, &w, &h, false);
    });
}

int orbfe_png_read_batch(const char* const* paths, int32_t n, int32_t width, int32_t height, uint8_t* out,
                         int32_t threads) {
    return guarded([&] {
        if (!paths || n < 0 || (n > 0 && !out)) throw Error(ORBFE_EINVAL, "null argument");
        const int nt = std::max(1, std::min<int>(threads, std::max(n, 1)));
        std::atomic<int> next{0};
        std::vector<std::string> err(nt);
        std::vector<int> code(nt, ORBFE_OK);
        auto work = [&](int t) {
            for (int i; (i = next.fetch_add(1)) < n;) {
                const int rc = guarded([&] {
                    const std::vector<uint8_t> d = read_file(paths[i]);
                    int w = 0, h = 0;
                    decode(d.data(), d.size(), nullptr, 0, &w, &h, true);
                    if (w != width || h != height)
                        throw Error(ORBFE_EINVAL, std::string(paths[i]) + ": size differs from the batch's");
                    decode(d.data(), d.size(), out + (int64_t)i * width * height, width, &w, &h, false);
                });
                if (rc != ORBFE_OK && code[t] == ORBFE_OK) {
                    code[t] = rc;
                    err[t] = g_err;
                }
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
        work(0);
        for (auto& th : pool) th.join();
        for (int t = 0; t < nt; ++t)
            if (code[t] != ORBFE_OK) throw Error(code[t], err[t]);
    });
}

}  // extern "C"
