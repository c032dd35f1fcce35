// image_io.cpp — see image_io.h.
#include "image_io.h"

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace ptio {

std::vector<unsigned char> to_rgb8(const std::vector<pt_vec3>& image, int width, int height, float samples) {
    std::vector<unsigned char> out((size_t)3 * width * height);
    for (int x = 0; x < width; x++) {
        for (int y = 0; y < height; y++) {
            const pt_vec3& pix = image[(size_t)x + (size_t)y * width];
            // main.cpp:405-407: img.setPixel(width - 1 - x, y, pix / samples)
            float c[3] = {pix.x / samples, pix.y / samples, pix.z / samples};
            size_t i = (size_t)y * width + (size_t)(width - 1 - x);
            for (int k = 0; k < 3; ++k) {
                // image.cpp:31-34: glm::clamp(pixel, 0, 1) * 255.f then (unsigned char)
                float v = c[k];
                v = v > 0.0f ? v : 0.0f;   // glm max(x, 0): NaN -> 0 (the black specks)
                v = v < 1.0f ? v : 1.0f;
                out[3 * i + k] = (unsigned char)(v * 255.f);
            }
        }
    }
    return out;
}

namespace {
// CRC-32 table built at compile time (pt_save_png may run on several threads at once)
struct CrcTable {
    uint32_t t[256];
    constexpr CrcTable() : t() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t k = i;
            for (int j = 0; j < 8; j++) k = (k & 1) ? 0xedb88320u ^ (k >> 1) : k >> 1;
            t[i] = k;
        }
    }
};
constexpr CrcTable crc_table{};
uint32_t crc32(const unsigned char* buf, size_t n, uint32_t c = 0xffffffffu) {
    for (size_t i = 0; i < n; i++) c = crc_table.t[(c ^ buf[i]) & 0xff] ^ (c >> 8);
    return c;
}
void put32(std::vector<unsigned char>& v, uint32_t x) {
    v.push_back((unsigned char)(x >> 24));
    v.push_back((unsigned char)(x >> 16));
    v.push_back((unsigned char)(x >> 8));
    v.push_back((unsigned char)x);
}
void chunk(std::vector<unsigned char>& png, const char* type, const std::vector<unsigned char>& data) {
    put32(png, (uint32_t)data.size());
    const size_t from = png.size();
    png.insert(png.end(), type, type + 4);
    png.insert(png.end(), data.begin(), data.end());
    put32(png, crc32(png.data() + from, png.size() - from) ^ 0xffffffffu);
}

// ---- the PNG stream stb_image_write 0.98 produces (image.cpp:40 -> stbi_write_png), restated so
// the saved file is byte-identical to the reference's: per-row filter choice by the smallest sum
// of |signed residual| (row 0 tries none/sub/none/avg-left/paeth-left), then one fixed-Huffman
// DEFLATE block from a hash-chained LZ77 with one-step lazy matching.

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// residuals of row y under filter byte `f` (row 0: f in 0..4 evaluates the degenerate forms with
// no row above; the byte written is still f, which decodes identically with a zero previous row)
void filter_row(const unsigned char* px, int stride, int n, int y, int f, signed char* out) {
    const unsigned char* z = px + (size_t)stride * y;
    const unsigned char* up = y ? z - stride : nullptr;
    for (int i = 0; i < stride; ++i) {
        const int left = i >= n ? z[i - n] : 0;
        const int above = up ? up[i] : 0;
        const int diag = (up && i >= n) ? up[i - n] : 0;
        int pred = 0;
        switch (f) {
            case 1: pred = left; break;
            case 2: pred = above; break;
            case 3: pred = (left + above) >> 1; break;
            case 4: pred = paeth(left, above, diag); break;
            default: pred = 0; break;
        }
        out[i] = (signed char)(unsigned char)(z[i] - pred);
    }
}

class BitSink {
  public:
    explicit BitSink(std::vector<unsigned char>& o) : out(o) {}
    void add(uint32_t code, int nbits) {
        buf |= code << count;
        count += nbits;
        while (count >= 8) {
            out.push_back((unsigned char)(buf & 0xff));
            buf >>= 8;
            count -= 8;
        }
    }
    void add_rev(uint32_t code, int nbits) {     // Huffman codes go out most-significant bit first
        uint32_t r = 0;
        for (int k = 0; k < nbits; ++k) r |= ((code >> k) & 1u) << (nbits - 1 - k);
        add(r, nbits);
    }
    void symbol(int s) {                          // fixed literal/length code (RFC 1951 3.2.6)
        if (s <= 143) add_rev(0x30 + s, 8);
        else if (s <= 255) add_rev(0x190 + s - 144, 9);
        else if (s <= 279) add_rev(s - 256, 7);
        else add_rev(0xc0 + s - 280, 8);
    }
    void pad() { while (count) add(0, 1); }

  private:
    std::vector<unsigned char>& out;
    uint32_t buf = 0;
    int count = 0;
};

uint32_t hash3(const unsigned char* d) {
    uint32_t h = d[0] + ((uint32_t)d[1] << 8) + ((uint32_t)d[2] << 16);
    h ^= h << 3;
    h += h >> 5;
    h ^= h << 4;
    h += h >> 17;
    h ^= h << 25;
    h += h >> 6;
    return h;
}

std::vector<unsigned char> zlib_fixed(const std::vector<unsigned char>& data) {
    static const int len_base[] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99,
                                   115, 131, 163, 195, 227, 258, 259};
    static const int len_extra[] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    static const int dist_base[] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025,
                                    1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577, 32768};
    static const int dist_extra[] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11,
                                     12, 12, 13, 13};
    constexpr int NBUCKET = 16384, KEEP = 8;      // stbi_zlib_compress(..., quality 8)
    const int n = (int)data.size();
    const unsigned char* d = data.data();
    std::vector<unsigned char> out = {0x78, 0x5e};
    BitSink bits(out);
    bits.add(1, 1);   // BFINAL
    bits.add(1, 2);   // fixed Huffman
    std::vector<std::vector<int>> chains(NBUCKET);   // positions per hash bucket, oldest first
    auto match_len = [&](int a, int b) {
        const int lim = std::min(n - b, 258);
        int k = 0;
        while (k < lim && d[a + k] == d[b + k]) ++k;
        return k;
    };
    int i = 0;
    while (i < n - 3) {
        std::vector<int>& chain = chains[hash3(d + i) & (NBUCKET - 1)];
        int best = 3, at = -1;
        for (int p : chain) {
            if (p > i - 32768) {
                const int m = match_len(p, i);
                if (m >= best) { best = m; at = p; }
            }
        }
        if ((int)chain.size() == 2 * KEEP) chain.erase(chain.begin(), chain.begin() + KEEP);
        chain.push_back(i);
        if (at >= 0) {   // lazy: a strictly longer match one byte later makes this byte a literal
            for (int p : chains[hash3(d + i + 1) & (NBUCKET - 1)]) {
                if (p > i - 32767 && match_len(p, i + 1) > best) { at = -1; break; }
            }
        }
        if (at >= 0) {
            const int dist = i - at;
            int j = 0;
            while (best > len_base[j + 1] - 1) ++j;
            bits.symbol(257 + j);
            if (len_extra[j]) bits.add((uint32_t)(best - len_base[j]), len_extra[j]);
            j = 0;
            while (dist > dist_base[j + 1] - 1) ++j;
            bits.add_rev((uint32_t)j, 5);
            if (dist_extra[j]) bits.add((uint32_t)(dist - dist_base[j]), dist_extra[j]);
            i += best;
        } else {
            bits.symbol(d[i]);
            ++i;
        }
    }
    for (; i < n; ++i) bits.symbol(d[i]);
    bits.symbol(256);
    bits.pad();
    uint32_t s1 = 1, s2 = 0;   // adler32
    for (int k = 0; k < n; ++k) {
        s1 = (s1 + d[k]) % 65521;
        s2 = (s2 + s1) % 65521;
    }
    put32(out, (s2 << 16) | s1);
    return out;
}
}  // namespace

std::vector<unsigned char> encode_png(const std::vector<unsigned char>& rgb, int width, int height) {
    const int n = 3, stride = 3 * width;
    std::vector<unsigned char> filt((size_t)(stride + 1) * height);
    std::vector<signed char> line((size_t)stride);
    for (int y = 0; y < height; ++y) {
        int best = 0, best_est = 0x7fffffff;
        for (int f = 0; f < 5; ++f) {
            filter_row(rgb.data(), stride, n, y, f, line.data());
            int est = 0;
            for (int k = 0; k < stride; ++k) est += std::abs((int)line[k]);
            if (est < best_est) { best_est = est; best = f; }
        }
        filter_row(rgb.data(), stride, n, y, best, line.data());
        unsigned char* row = filt.data() + (size_t)y * (stride + 1);
        row[0] = (unsigned char)best;
        std::memcpy(row + 1, line.data(), (size_t)stride);
    }
    std::vector<unsigned char> png = {137, 80, 78, 71, 13, 10, 26, 10};
    std::vector<unsigned char> ihdr;
    put32(ihdr, (uint32_t)width);
    put32(ihdr, (uint32_t)height);
    for (unsigned char b : {8, 2, 0, 0, 0}) ihdr.push_back(b);   // 8-bit RGB
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", zlib_fixed(filt));
    chunk(png, "IEND", {});
    return png;
}

bool write_png(const std::string& path, const std::vector<unsigned char>& rgb, int width, int height) {
    const std::vector<unsigned char> png = encode_png(rgb, width, height);
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(png.data(), 1, png.size(), f) == png.size();
    return (std::fclose(f) == 0) && ok;
}

bool write_pfm(const std::string& path, const std::vector<pt_vec3>& image, int width, int height) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "PF\n%d %d\n-1.0\n", width, height);
    for (int y = height - 1; y >= 0; --y) fwrite(&image[(size_t)y * width], sizeof(pt_vec3), (size_t)width, f);
    return std::fclose(f) == 0;
}

}  // namespace ptio
