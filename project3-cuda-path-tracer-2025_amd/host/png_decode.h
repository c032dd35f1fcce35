// png_decode.h — PNG -> RGBA8 for the scene loader's textures (the reference loads them with
// stbi_load(path, &w, &h, &c, STBI_rgb_alpha), scene.cpp:366-392).  Own zlib inflate
// (RFC 1950/1951) and PNG decoding (all colour types, bit depths 1-16, Adam7, PLTE/tRNS);
// conversion to 4 channels follows stb_image's rules for STBI_rgb_alpha: grey g -> (g,g,g,255),
// low bit depths of grey are scaled to 0..255, 16-bit samples keep their high byte, a tRNS
// colour key makes matching pixels transparent.  Gamma / colour-space chunks are ignored, as
// stb_image does.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ptio {

// true on success: w, h and w*h*4 bytes of RGBA in `rgba`; false with a message in `err`
bool png_load_rgba(const std::string& path, int& w, int& h, std::vector<uint8_t>& rgba, std::string& err);
bool png_decode_rgba(const uint8_t* data, size_t size, int& w, int& h, std::vector<uint8_t>& rgba, std::string& err);

// raw zlib stream -> bytes (exposed for tests); fails once the output would exceed max_out
bool zlib_inflate(const uint8_t* data, size_t size, std::vector<uint8_t>& out, std::string& err,
                  size_t max_out = (size_t)1 << 31);

}  // namespace ptio
