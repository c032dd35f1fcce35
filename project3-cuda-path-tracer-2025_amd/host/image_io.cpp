// image_io.cpp — see image_io.h.
#include "image_io.h"

#include <cstdint>
#include <cstdio>

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
uint32_t crc_table[256];
bool crc_init = false;
uint32_t crc32(const unsigned char* buf, size_t n, uint32_t c = 0xffffffffu) {
    if (!crc_init) {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t k = i;
            for (int j = 0; j < 8; j++) k = (k & 1) ? 0xedb88320u ^ (k >> 1) : k >> 1;
            crc_table[i] = k;
        }
        crc_init = true;
    }
    for (size_t i = 0; i < n; i++) c = crc_table[(c ^ buf[i]) & 0xff] ^ (c >> 8);
    return c;
}
void put32(std::vector<unsigned char>& v, uint32_t x) {
    v.push_back((unsigned char)(x >> 24));
    v.push_back((unsigned char)(x >> 16));
    v.push_back((unsigned char)(x >> 8));
    v.push_back((unsigned char)x);
}
void chunk(FILE* f, const char* type, const std::vector<unsigned char>& data) {
    std::vector<unsigned char> buf;
    put32(buf, (uint32_t)data.size());
    buf.insert(buf.end(), type, type + 4);
    buf.insert(buf.end(), data.begin(), data.end());
    uint32_t c = crc32(buf.data() + 4, buf.size() - 4) ^ 0xffffffffu;
    put32(buf, c);
    fwrite(buf.data(), 1, buf.size(), f);
}
}  // namespace

bool write_png(const std::string& path, const std::vector<unsigned char>& rgb, int width, int height) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    fwrite(sig, 1, 8, f);
    std::vector<unsigned char> ihdr;
    put32(ihdr, (uint32_t)width);
    put32(ihdr, (uint32_t)height);
    ihdr.push_back(8);   // bit depth
    ihdr.push_back(2);   // RGB
    ihdr.push_back(0);
    ihdr.push_back(0);
    ihdr.push_back(0);
    chunk(f, "IHDR", ihdr);
    // raw scanlines with filter byte 0, zlib-wrapped in stored blocks
    std::vector<unsigned char> raw;
    raw.reserve((size_t)height * (3 * width + 1));
    for (int y = 0; y < height; y++) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb.begin() + (size_t)y * 3 * width, rgb.begin() + (size_t)(y + 1) * 3 * width);
    }
    std::vector<unsigned char> z;
    z.push_back(0x78);
    z.push_back(0x01);
    size_t pos = 0;
    do {
        size_t n = raw.size() - pos < 65535 ? raw.size() - pos : 65535;
        z.push_back(pos + n == raw.size() ? 1 : 0);
        z.push_back((unsigned char)(n & 0xff));
        z.push_back((unsigned char)(n >> 8));
        z.push_back((unsigned char)(~n & 0xff));
        z.push_back((unsigned char)((~n >> 8) & 0xff));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (unsigned char ch : raw) {
        a = (a + ch) % 65521;
        b = (b + a) % 65521;
    }
    put32(z, (b << 16) | a);
    chunk(f, "IDAT", z);
    chunk(f, "IEND", {});
    return std::fclose(f) == 0;
}

bool write_pfm(const std::string& path, const std::vector<pt_vec3>& image, int width, int height) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "PF\n%d %d\n-1.0\n", width, height);
    for (int y = height - 1; y >= 0; --y) fwrite(&image[(size_t)y * width], sizeof(pt_vec3), (size_t)width, f);
    return std::fclose(f) == 0;
}

}  // namespace ptio
