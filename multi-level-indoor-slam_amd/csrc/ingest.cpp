// Keyframe ingestion: PNG keyframes -> BGR uint8, as
// process_image_sequence reads them (place_recognition.py:965-968: cv2.imread(path),
// IMREAD_COLOR) after scripts/utils/bag_utils.py:222-271 wrote them (cv2.imwrite
// '{timestamp:.6f}.png').
//
// Host code by design: DEFLATE is a serial bit stream and the PNG row filters (Sub,
// Average, Paeth) chain every byte to its left neighbour, so one image is one serial
// job; a pool of host threads decodes a batch of files straight into one caller-owned
// (pinned) [n, H, W, 3] buffer, which the Python side copies to HBM on a side stream
// while the previous batch runs through the ViT (mlgate/ingest.py).
//
// cv2.imread(IMREAD_COLOR) semantics restated (OpenCV's PNG decoder over libpng):
// palette -> RGB, gray (1/2/4/8/16 bit) -> replicated to 3 channels with 1/2/4-bit
// samples scaled to 0..255, alpha stripped, 16-bit samples reduced to their high byte,
// Adam7 interlace undone, RGB stored as BGR; a CRC or stream error fails the image
// (imread returns None).
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <exception>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/mlgate.h"

namespace {

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

struct Png {
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> plte;  // RGB triples
    std::vector<uint8_t> idat;
};

int samples_per_pixel(int ctype) {
    switch (ctype) {
        case 0: return 1;  // gray
        case 2: return 3;  // RGB
        case 3: return 1;  // palette index
        case 4: return 2;  // gray + alpha
        case 6: return 4;  // RGBA
        default: return 0;
    }
}

bool depth_ok(int ctype, int depth) {
    switch (ctype) {
        case 0: return depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16;
        case 3: return depth == 1 || depth == 2 || depth == 4 || depth == 8;
        case 2: case 4: case 6: return depth == 8 || depth == 16;
        default: return false;
    }
}

// Chunk walk with CRC checks (libpng errors on a bad critical-chunk CRC).
int parse(const uint8_t* d, size_t n, Png& p, bool header_only) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0d, 0x0a, 0x1a, 0x0a};
    if (n < 8 + 25 || std::memcmp(d, sig, 8) != 0) return MLG_EINVAL;
    size_t o = 8;
    bool have_ihdr = false, have_end = false;
    while (o + 12 <= n) {
        const uint32_t len = be32(d + o);
        if (len > n - o - 12) return MLG_EINVAL;
        const uint8_t* type = d + o + 4;
        const uint8_t* body = d + o + 8;
        const bool critical = !(type[0] & 0x20);
        if (critical || !have_ihdr) {
            const uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), type, len + 4);
            if (crc != be32(body + len)) return MLG_EINVAL;
        }
        if (!have_ihdr) {
            if (std::memcmp(type, "IHDR", 4) != 0 || len != 13) return MLG_EINVAL;
            p.w = be32(body);
            p.h = be32(body + 4);
            p.depth = body[8];
            p.ctype = body[9];
            p.interlace = body[12];
            if (p.w == 0 || p.h == 0 || p.w > (1u << 16) || p.h > (1u << 16)) return MLG_EINVAL;
            if (!depth_ok(p.ctype, p.depth) || body[10] != 0 || body[11] != 0 || p.interlace > 1) return MLG_EINVAL;
            have_ihdr = true;
            if (header_only) return MLG_OK;
        } else if (!std::memcmp(type, "PLTE", 4)) {
            if (len % 3 || len == 0 || len > 768) return MLG_EINVAL;
            p.plte.assign(body, body + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            p.idat.insert(p.idat.end(), body, body + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            have_end = true;
            break;
        } else if (critical) {
            return MLG_EINVAL;  // unknown critical chunk
        }
        o += 12 + len;
    }
    if (!have_ihdr || p.idat.empty() || !have_end) return MLG_EINVAL;
    if (p.ctype == 3 && p.plte.empty()) return MLG_EINVAL;
    return MLG_OK;
}

inline uint8_t paeth(int a, int b, int c) {
    const int pp = a + b - c;
    const int pa = std::abs(pp - a), pb = std::abs(pp - b), pc = std::abs(pp - c);
    if (pa <= pb && pa <= pc) return (uint8_t)a;
    return (uint8_t)(pb <= pc ? b : c);
}

// In-place reconstruction of one (sub)image of `rows` filtered scanlines of `rb` bytes
// (each preceded by its filter byte), bytes-per-complete-pixel `bpp` (>= 1).
bool unfilter(uint8_t* s, size_t rows, size_t rb, size_t bpp, std::vector<uint8_t>& out) {
    out.resize(rows * rb);
    const uint8_t* prev = nullptr;
    for (size_t y = 0; y < rows; ++y) {
        const uint8_t ft = s[y * (rb + 1)];
        const uint8_t* in = s + y * (rb + 1) + 1;
        uint8_t* cur = out.data() + y * rb;
        switch (ft) {
            case 0: std::memcpy(cur, in, rb); break;
            case 1:
                for (size_t i = 0; i < rb; ++i) cur[i] = (uint8_t)(in[i] + (i >= bpp ? cur[i - bpp] : 0));
                break;
            case 2:
                for (size_t i = 0; i < rb; ++i) cur[i] = (uint8_t)(in[i] + (prev ? prev[i] : 0));
                break;
            case 3:
                for (size_t i = 0; i < rb; ++i) {
                    const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0;
                    cur[i] = (uint8_t)(in[i] + ((a + b) >> 1));
                }
                break;
            case 4:
                for (size_t i = 0; i < rb; ++i) {
                    const int a = i >= bpp ? cur[i - bpp] : 0, b = prev ? prev[i] : 0;
                    const int c = (i >= bpp && prev) ? prev[i - bpp] : 0;
                    cur[i] = (uint8_t)(in[i] + paeth(a, b, c));
                }
                break;
            default: return false;
        }
        prev = cur;
    }
    return true;
}

// Sample x of a packed row at `depth` bits (1/2/4/8) or the high byte of a 16-bit sample.
inline int sample(const uint8_t* row, size_t idx, int depth) {
    switch (depth) {
        case 8: return row[idx];
        case 16: return row[2 * idx];
        case 4: return (row[idx >> 1] >> (4 - 4 * (idx & 1))) & 0xf;
        case 2: return (row[idx >> 2] >> (6 - 2 * (idx & 3))) & 0x3;
        default: return (row[idx >> 3] >> (7 - (idx & 7))) & 0x1;
    }
}

// One decoded pixel (x of `row`) as B, G, R.
inline void pixel_bgr(const Png& p, const uint8_t* row, size_t x, uint8_t* o) {
    const int spp = samples_per_pixel(p.ctype);
    if (p.ctype == 3) {
        const size_t i = (size_t)sample(row, x, p.depth);
        if (3 * i + 2 < p.plte.size()) {
            o[0] = p.plte[3 * i + 2]; o[1] = p.plte[3 * i + 1]; o[2] = p.plte[3 * i];
        } else {
            o[0] = o[1] = o[2] = 0;  // libpng leaves an out-of-palette index black
        }
        return;
    }
    if (p.ctype == 0 || p.ctype == 4) {
        int g = sample(row, x * spp, p.depth);
        if (p.depth < 8) g = g * (255 / ((1 << p.depth) - 1));  // expand_gray_1_2_4_to_8
        o[0] = o[1] = o[2] = (uint8_t)g;
        return;
    }
    o[0] = (uint8_t)sample(row, x * spp + 2, p.depth);
    o[1] = (uint8_t)sample(row, x * spp + 1, p.depth);
    o[2] = (uint8_t)sample(row, x * spp, p.depth);
}

size_t row_bytes(const Png& p, size_t w) { return (w * samples_per_pixel(p.ctype) * p.depth + 7) / 8; }

int decode_into(const uint8_t* d, size_t n, uint8_t* out, int H, int W) {
    Png p;
    int rc = parse(d, n, p, false);
    if (rc != MLG_OK) return rc;
    if ((int)p.w != W || (int)p.h != H) return MLG_ESIZE;
    const size_t bpp = std::max<size_t>(1, (size_t)samples_per_pixel(p.ctype) * p.depth / 8);
    // Adam7 passes: x0, y0, dx, dy
    static const int A7[7][4] = {{0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4},
                                 {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};
    const int npass = p.interlace ? 7 : 1;
    size_t raw_total = 0;
    size_t pw[7], ph[7];
    for (int k = 0; k < npass; ++k) {
        if (p.interlace) {
            pw[k] = p.w > (uint32_t)A7[k][0] ? (p.w - A7[k][0] + A7[k][2] - 1) / A7[k][2] : 0;
            ph[k] = p.h > (uint32_t)A7[k][1] ? (p.h - A7[k][1] + A7[k][3] - 1) / A7[k][3] : 0;
        } else {
            pw[k] = p.w;
            ph[k] = p.h;
        }
        if (pw[k] && ph[k]) raw_total += ph[k] * (row_bytes(p, pw[k]) + 1);
    }
    // one inflate call: zlib's avail_in / avail_out are uInt, so neither side may pass 4 GiB
    // (a 65536 x 65536 16-bit RGBA header would ask for 32 GiB)
    if (raw_total > UINT_MAX || p.idat.size() > UINT_MAX) return MLG_ENOMEM;
    std::vector<uint8_t> raw(raw_total);
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) return MLG_ENOMEM;
    zs.next_in = p.idat.data();
    zs.avail_in = (uInt)p.idat.size();
    zs.next_out = raw.data();
    zs.avail_out = (uInt)raw.size();
    const int zr = inflate(&zs, Z_FINISH);
    const size_t produced = raw.size() - zs.avail_out;
    inflateEnd(&zs);
    if ((zr != Z_STREAM_END && zr != Z_BUF_ERROR && zr != Z_OK) || produced != raw.size()) return MLG_EINVAL;
    std::vector<uint8_t> img;
    size_t off = 0;
    for (int k = 0; k < npass; ++k) {
        if (!pw[k] || !ph[k]) continue;
        const size_t rb = row_bytes(p, pw[k]);
        if (!unfilter(raw.data() + off, ph[k], rb, bpp, img)) return MLG_EINVAL;
        off += ph[k] * (rb + 1);
        const size_t x0 = p.interlace ? A7[k][0] : 0, y0 = p.interlace ? A7[k][1] : 0;
        const size_t dx = p.interlace ? A7[k][2] : 1, dy = p.interlace ? A7[k][3] : 1;
        for (size_t y = 0; y < ph[k]; ++y) {
            const uint8_t* row = img.data() + y * rb;
            uint8_t* orow = out + ((y0 + y * dy) * (size_t)W) * 3;
            if (p.ctype == 2 && p.depth == 8) {  // the bag_utils case: 8-bit RGB -> BGR
                for (size_t x = 0; x < pw[k]; ++x) {
                    uint8_t* o = orow + (x0 + x * dx) * 3;
                    o[0] = row[3 * x + 2]; o[1] = row[3 * x + 1]; o[2] = row[3 * x];
                }
            } else {
                for (size_t x = 0; x < pw[k]; ++x) pixel_bgr(p, row, x, orow + (x0 + x * dx) * 3);
            }
        }
    }
    return MLG_OK;
}

bool read_file(const char* path, std::vector<uint8_t>& buf) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    bool ok = std::fseek(f, 0, SEEK_END) == 0;
    const long sz = ok ? std::ftell(f) : -1;
    ok = ok && sz > 0 && std::fseek(f, 0, SEEK_SET) == 0;
    if (ok) {
        buf.resize((size_t)sz);
        ok = std::fread(buf.data(), 1, buf.size(), f) == buf.size();
    }
    std::fclose(f);
    return ok;
}

// A failed allocation (std::bad_alloc / length_error from the vectors of one file)
// becomes that file's status instead of std::terminate inside a pool thread.
template <class F>
int guarded(F&& f) {
    try {
        return f();
    } catch (const std::exception&) {
        return MLG_ENOMEM;
    }
}

template <class F>
void pool(int n, int threads, F&& job) {
    threads = std::max(1, std::min(threads, n));
    std::atomic<int> next{0};
    auto worker = [&] {
        for (int i; (i = next.fetch_add(1)) < n;) job(i);
    };
    std::vector<std::thread> ts;
    for (int t = 1; t < threads; ++t) ts.emplace_back(worker);
    worker();
    for (auto& t : ts) t.join();
}

}  // namespace

extern "C" {

int mlg_png_info(const uint8_t* data, size_t len, int32_t* width, int32_t* height, int32_t* color_type,
                 int32_t* bit_depth) {
    if (!data || !width || !height) return MLG_EINVAL;
    Png p;
    const int rc = parse(data, len, p, true);
    if (rc != MLG_OK) return rc;
    *width = (int32_t)p.w;
    *height = (int32_t)p.h;
    if (color_type) *color_type = p.ctype;
    if (bit_depth) *bit_depth = p.depth;
    return MLG_OK;
}

int mlg_png_decode_bgr(const uint8_t* const* data, const size_t* lens, int n, uint8_t* out, int H, int W,
                       int threads, int32_t* status) {
    if (n < 0 || H <= 0 || W <= 0 || (n && (!data || !lens || !out || !status))) return MLG_EINVAL;
    const size_t frame = (size_t)H * W * 3;
    pool(n, threads, [&](int i) { status[i] = guarded([&] { return decode_into(data[i], lens[i], out + frame * i, H, W); }); });
    return MLG_OK;
}

int mlg_png_load_bgr(const char* const* paths, int n, uint8_t* out, int H, int W, int threads, int32_t* status) {
    if (n < 0 || H <= 0 || W <= 0 || (n && (!paths || !out || !status))) return MLG_EINVAL;
    const size_t frame = (size_t)H * W * 3;
    pool(n, threads, [&](int i) {
        status[i] = guarded([&] {
            std::vector<uint8_t> buf;
            return read_file(paths[i], buf) ? decode_into(buf.data(), buf.size(), out + frame * i, H, W) : MLG_EINVAL;
        });
    });
    return MLG_OK;
}

}  // extern "C"
