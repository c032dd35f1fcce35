// png_decode.cpp — see png_decode.h.
#include "png_decode.h"

#include <cstring>
#include <fstream>
#include <iterator>

namespace ptio {
namespace {

// ---------------------------------------------------------------------------------------------
// inflate (RFC 1951)
// ---------------------------------------------------------------------------------------------
struct BitReader {
    const uint8_t* p;
    size_t n, pos = 0;
    uint32_t bitbuf = 0;
    int bitcnt = 0;
    bool overrun = false;
    int bit() {
        if (bitcnt == 0) {
            if (pos >= n) {
                overrun = true;
                return 0;
            }
            bitbuf = p[pos++];
            bitcnt = 8;
        }
        int b = bitbuf & 1;
        bitbuf >>= 1;
        --bitcnt;
        return b;
    }
    uint32_t bits(int k) {   // LSB first
        uint32_t v = 0;
        for (int i = 0; i < k; ++i) v |= (uint32_t)bit() << i;
        return v;
    }
    void align() { bitcnt = 0; }
};

// canonical Huffman code: counts per length, symbols in code order
struct Huffman {
    uint16_t count[16] = {};
    std::vector<uint16_t> symbol;
    bool build(const uint8_t* lengths, int n) {
        memset(count, 0, sizeof count);
        for (int i = 0; i < n; ++i) count[lengths[i]]++;
        count[0] = 0;
        int left = 1;
        for (int len = 1; len < 16; ++len) {   // over-subscribed set is invalid
            left <<= 1;
            left -= count[len];
            if (left < 0) return false;
        }
        uint16_t offs[16] = {};
        for (int len = 1; len < 15; ++len) offs[len + 1] = offs[len] + count[len];
        symbol.assign(n, 0);
        for (int i = 0; i < n; ++i)
            if (lengths[i]) symbol[offs[lengths[i]]++] = (uint16_t)i;
        return true;
    }
    int decode(BitReader& br) const {
        int code = 0, first = 0, index = 0;
        for (int len = 1; len < 16; ++len) {
            code |= br.bit();
            int c = count[len];
            if (code - c < first) return symbol[index + (code - first)];
            index += c;
            first += c;
            first <<= 1;
            code <<= 1;
            if (br.overrun) return -1;
        }
        return -1;
    }
};

const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                               35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129,
                                193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6,
                                7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

bool inflate_codes(BitReader& br, const Huffman& lit, const Huffman& dist, std::vector<uint8_t>& out, size_t max_out,
                   std::string& err) {
    for (;;) {
        if (out.size() > max_out) return err = "inflate: more data than the image holds", false;
        int sym = lit.decode(br);
        if (sym < 0) return err = "inflate: bad literal/length code", false;
        if (sym < 256) {
            out.push_back((uint8_t)sym);
        } else if (sym == 256) {
            return true;
        } else {
            sym -= 257;
            if (sym >= 29) return err = "inflate: bad length symbol", false;
            size_t len = kLenBase[sym] + br.bits(kLenExtra[sym]);
            int ds = dist.decode(br);
            if (ds < 0 || ds >= 30) return err = "inflate: bad distance code", false;
            size_t d = kDistBase[ds] + br.bits(kDistExtra[ds]);
            if (d > out.size()) return err = "inflate: distance too far back", false;
            size_t from = out.size() - d;
            for (size_t i = 0; i < len; ++i) out.push_back(out[from + i]);
        }
        if (br.overrun) return err = "inflate: truncated stream", false;
    }
}

bool inflate_raw(const uint8_t* data, size_t size, std::vector<uint8_t>& out, size_t max_out, std::string& err) {
    BitReader br{data, size};
    int last = 0;
    do {
        last = br.bit();
        int type = (int)br.bits(2);
        if (type == 0) {                                   // stored
            br.align();
            if (br.pos + 4 > size) return err = "inflate: truncated stored block", false;
            uint32_t len = data[br.pos] | (data[br.pos + 1] << 8);
            uint32_t nlen = data[br.pos + 2] | (data[br.pos + 3] << 8);
            br.pos += 4;
            if ((len ^ 0xffffu) != nlen) return err = "inflate: stored length mismatch", false;
            if (br.pos + len > size) return err = "inflate: truncated stored block", false;
            if (out.size() + len > max_out) return err = "inflate: more data than the image holds", false;
            out.insert(out.end(), data + br.pos, data + br.pos + len);
            br.pos += len;
        } else if (type == 1) {                            // fixed Huffman
            uint8_t l[288], d[30];
            for (int i = 0; i < 144; ++i) l[i] = 8;
            for (int i = 144; i < 256; ++i) l[i] = 9;
            for (int i = 256; i < 280; ++i) l[i] = 7;
            for (int i = 280; i < 288; ++i) l[i] = 8;
            for (int i = 0; i < 30; ++i) d[i] = 5;
            Huffman lit, dist;
            lit.build(l, 288);
            dist.build(d, 30);
            if (!inflate_codes(br, lit, dist, out, max_out, err)) return false;
        } else if (type == 2) {                            // dynamic Huffman
            int hlit = (int)br.bits(5) + 257, hdist = (int)br.bits(5) + 1, hclen = (int)br.bits(4) + 4;
            static const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
            uint8_t cl[19] = {};
            for (int i = 0; i < hclen; ++i) cl[order[i]] = (uint8_t)br.bits(3);
            Huffman clh;
            if (!clh.build(cl, 19)) return err = "inflate: bad code-length code", false;
            uint8_t lens[320] = {};
            int k = 0;
            while (k < hlit + hdist) {
                int sym = clh.decode(br);
                if (sym < 0) return err = "inflate: bad code-length symbol", false;
                if (sym < 16) {
                    lens[k++] = (uint8_t)sym;
                } else {
                    int rep = 0;
                    uint8_t val = 0;
                    if (sym == 16) {
                        if (k == 0) return err = "inflate: repeat with no previous length", false;
                        val = lens[k - 1];
                        rep = 3 + (int)br.bits(2);
                    } else if (sym == 17) {
                        rep = 3 + (int)br.bits(3);
                    } else {
                        rep = 11 + (int)br.bits(7);
                    }
                    if (k + rep > hlit + hdist) return err = "inflate: too many code lengths", false;
                    while (rep--) lens[k++] = val;
                }
            }
            Huffman lit, dist;
            if (!lit.build(lens, hlit) || !dist.build(lens + hlit, hdist))
                return err = "inflate: bad literal/distance code", false;
            if (!inflate_codes(br, lit, dist, out, max_out, err)) return false;
        } else {
            return err = "inflate: reserved block type", false;
        }
        if (br.overrun) return err = "inflate: truncated stream", false;
    } while (!last);
    return true;
}

uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

int paeth(int a, int b, int c) {
    int p = a + b - c, pa = p > a ? p - a : a - p, pb = p > b ? p - b : b - p, pc = p > c ? p - c : c - p;
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

// reverse the scanline filters of one (sub-)image in place; returns false on a bad filter byte
bool unfilter(uint8_t* img, size_t rows, size_t stride, size_t bpp, std::vector<uint8_t>& out) {
    out.assign(rows * stride, 0);
    std::vector<uint8_t> prev(stride, 0);
    for (size_t y = 0; y < rows; ++y) {
        const uint8_t f = img[y * (stride + 1)];
        const uint8_t* src = img + y * (stride + 1) + 1;
        uint8_t* dst = out.data() + y * stride;
        for (size_t x = 0; x < stride; ++x) {
            int a = x >= bpp ? dst[x - bpp] : 0, b = prev[x], c = x >= bpp ? prev[x - bpp] : 0;
            int v = src[x];
            switch (f) {
                case 0: break;
                case 1: v += a; break;
                case 2: v += b; break;
                case 3: v += (a + b) >> 1; break;
                case 4: v += paeth(a, b, c); break;
                default: return false;
            }
            dst[x] = (uint8_t)v;
        }
        memcpy(prev.data(), dst, stride);
    }
    return true;
}

}  // namespace

bool zlib_inflate(const uint8_t* data, size_t size, std::vector<uint8_t>& out, std::string& err, size_t max_out) {
    if (size < 2) return err = "zlib: stream too short", false;
    const int cmf = data[0], flg = data[1];
    if ((cmf & 15) != 8 || ((cmf << 8) | flg) % 31 != 0) return err = "zlib: bad header", false;
    if (flg & 32) return err = "zlib: preset dictionary not supported", false;
    return inflate_raw(data + 2, size - 2, out, max_out, err);
}

bool png_decode_rgba(const uint8_t* data, size_t size, int& w, int& h, std::vector<uint8_t>& rgba, std::string& err) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (size < 8 || memcmp(data, sig, 8) != 0) return err = "png: bad signature", false;
    size_t pos = 8;
    uint32_t W = 0, H = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    bool have_ihdr = false, have_iend = false;
    while (pos + 12 <= size && !have_iend) {
        const uint32_t len = be32(data + pos);
        const uint8_t* type = data + pos + 4;
        if (pos + 12 + (size_t)len > size) return err = "png: truncated chunk", false;
        const uint8_t* body = data + pos + 8;
        if (!memcmp(type, "IHDR", 4)) {
            if (len != 13) return err = "png: bad IHDR", false;
            W = be32(body);
            H = be32(body + 4);
            depth = body[8];
            ctype = body[9];
            if (body[10] != 0 || body[11] != 0) return err = "png: unknown compression/filter method", false;
            interlace = body[12];
            have_ihdr = true;
        } else if (!memcmp(type, "PLTE", 4)) {
            plte.assign(body, body + len);
        } else if (!memcmp(type, "tRNS", 4)) {
            trns.assign(body, body + len);
        } else if (!memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), body, body + len);
        } else if (!memcmp(type, "IEND", 4)) {
            have_iend = true;
        }
        pos += 12 + len;
    }
    if (!have_ihdr) return err = "png: no IHDR", false;
    if (W == 0 || H == 0 || W > (1u << 24) || H > (1u << 24) || (uint64_t)W * H > (1ull << 28))
        return err = "png: bad dimensions", false;
    int chans;
    switch (ctype) {
        case 0: chans = 1; break;
        case 2: chans = 3; break;
        case 3: chans = 1; break;
        case 4: chans = 2; break;
        case 6: chans = 4; break;
        default: return err = "png: bad colour type", false;
    }
    const bool depth_ok = depth == 8 || depth == 16 ||
                          ((ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4));
    if (!depth_ok || (ctype == 3 && depth == 16)) return err = "png: bad bit depth", false;
    if (ctype == 3 && plte.empty()) return err = "png: palette image without PLTE", false;
    if (interlace > 1) return err = "png: bad interlace method", false;

    const size_t bits_pp = (size_t)chans * depth;
    const size_t bpp = (bits_pp + 7) / 8;                  // filter unit
    // the filtered data the header promises: checked before anything image-sized is allocated, and
    // the inflate stops there (a small file cannot make it allocate more than the image holds)
    size_t need = 0;
    if (interlace == 0) {
        need = (size_t)H * (((size_t)W * bits_pp + 7) / 8 + 1);
    } else {
        static const int xo[7] = {0, 4, 0, 2, 0, 1, 0}, yo[7] = {0, 0, 4, 0, 2, 0, 1};
        static const int xs[7] = {8, 8, 4, 4, 2, 2, 1}, ys[7] = {8, 8, 8, 4, 4, 2, 2};
        for (int p = 0; p < 7; ++p) {
            const size_t sw = W > (uint32_t)xo[p] ? (W - xo[p] + xs[p] - 1) / xs[p] : 0;
            const size_t sh = H > (uint32_t)yo[p] ? (H - yo[p] + ys[p] - 1) / ys[p] : 0;
            if (sw && sh) need += sh * ((sw * bits_pp + 7) / 8 + 1);
        }
    }
    std::vector<uint8_t> raw;
    if (!zlib_inflate(idat.data(), idat.size(), raw, err, need + 65536)) return false;
    if (raw.size() < need) return err = "png: image data shorter than the header says", false;
    // decoded samples at native depth, one row of W pixels per image row
    std::vector<uint16_t> samp((size_t)W * H * chans);
    auto read_rows = [&](const uint8_t* src, size_t sw, size_t sh, int x0, int y0, int dx, int dy,
                         size_t& consumed) -> bool {
        if (sw == 0 || sh == 0) {
            consumed = 0;
            return true;
        }
        const size_t stride = (sw * bits_pp + 7) / 8;
        consumed = sh * (stride + 1);
        if ((size_t)(src - raw.data()) + consumed > raw.size()) return false;
        std::vector<uint8_t> tmp(src, src + consumed), rows;
        if (!unfilter(tmp.data(), sh, stride, bpp, rows)) return false;
        for (size_t y = 0; y < sh; ++y) {
            const uint8_t* r = rows.data() + y * stride;
            for (size_t x = 0; x < sw; ++x)
                for (int c = 0; c < chans; ++c) {
                    uint16_t v;
                    if (depth == 16) {
                        const size_t o = (x * chans + c) * 2;
                        v = (uint16_t)(r[o] << 8 | r[o + 1]);
                    } else if (depth == 8) {
                        v = r[x * chans + c];
                    } else {
                        const size_t bit = x * depth;
                        v = (r[bit / 8] >> (8 - depth - bit % 8)) & ((1 << depth) - 1);
                    }
                    const size_t px = (size_t)(y0 + y * dy) * W + (size_t)(x0 + x * dx);
                    samp[px * chans + c] = v;
                }
        }
        return true;
    };
    if (interlace == 0) {
        size_t used;
        if (!read_rows(raw.data(), W, H, 0, 0, 1, 1, used)) return err = "png: corrupt image data", false;
    } else {                                               // Adam7
        static const int xo[7] = {0, 4, 0, 2, 0, 1, 0}, yo[7] = {0, 0, 4, 0, 2, 0, 1};
        static const int xs[7] = {8, 8, 4, 4, 2, 2, 1}, ys[7] = {8, 8, 8, 4, 4, 2, 2};
        const uint8_t* src = raw.data();
        for (int p = 0; p < 7; ++p) {
            const size_t sw = W > (uint32_t)xo[p] ? (W - xo[p] + xs[p] - 1) / xs[p] : 0;
            const size_t sh = H > (uint32_t)yo[p] ? (H - yo[p] + ys[p] - 1) / ys[p] : 0;
            size_t used;
            if (!read_rows(src, sw, sh, xo[p], yo[p], xs[p], ys[p], used))
                return err = "png: corrupt interlaced data", false;
            src += used;
        }
    }

    // -> RGBA8 with stb_image's STBI_rgb_alpha rules
    static const uint8_t depth_scale[9] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 0x01};
    auto to8 = [&](uint16_t v) -> uint8_t {
        if (depth == 16) return (uint8_t)(v >> 8);
        if (depth == 8) return (uint8_t)v;
        return (uint8_t)(v * depth_scale[depth]);
    };
    bool key = false;
    uint16_t kr = 0, kg = 0, kb = 0;
    if (!trns.empty() && ctype == 0 && trns.size() >= 2) {
        key = true;
        kr = kg = kb = (uint16_t)(trns[0] << 8 | trns[1]);
    } else if (!trns.empty() && ctype == 2 && trns.size() >= 6) {
        key = true;
        kr = (uint16_t)(trns[0] << 8 | trns[1]);
        kg = (uint16_t)(trns[2] << 8 | trns[3]);
        kb = (uint16_t)(trns[4] << 8 | trns[5]);
    }
    w = (int)W;
    h = (int)H;
    rgba.assign((size_t)W * H * 4, 0);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        const uint16_t* s = &samp[i * chans];
        uint8_t* d = &rgba[i * 4];
        switch (ctype) {
            case 0:
                d[0] = d[1] = d[2] = to8(s[0]);
                d[3] = (key && s[0] == kr) ? 0 : 255;
                break;
            case 2:
                d[0] = to8(s[0]);
                d[1] = to8(s[1]);
                d[2] = to8(s[2]);
                d[3] = (key && s[0] == kr && s[1] == kg && s[2] == kb) ? 0 : 255;
                break;
            case 3: {
                const size_t idx = s[0];
                if (idx * 3 + 2 >= plte.size()) return err = "png: palette index out of range", false;
                d[0] = plte[idx * 3];
                d[1] = plte[idx * 3 + 1];
                d[2] = plte[idx * 3 + 2];
                d[3] = idx < trns.size() ? trns[idx] : 255;
                break;
            }
            case 4:
                d[0] = d[1] = d[2] = to8(s[0]);
                d[3] = to8(s[1]);
                break;
            default:
                d[0] = to8(s[0]);
                d[1] = to8(s[1]);
                d[2] = to8(s[2]);
                d[3] = to8(s[3]);
                break;
        }
    }
    return true;
}

bool png_load_rgba(const std::string& path, int& w, int& h, std::vector<uint8_t>& rgba, std::string& err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return err = "cannot open " + path, false;
    std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    return png_decode_rgba(bytes.data(), bytes.size(), w, h, rgba, err);
}

}  // namespace ptio
