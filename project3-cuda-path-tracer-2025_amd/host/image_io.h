// image_io.h — output formats of the headless driver: the reference's saveImage
// (main.cpp:395-419 + image.cpp:23-43) as an 8-bit PNG, plus the raw float accumulator.
#pragma once

#include <string>
#include <vector>

#include "pt/scene_structs.h"

namespace ptio {
// saveImage: x-flip, divide by samples, clamp to [0,1], x255 truncation -> RGB8 rows
std::vector<unsigned char> to_rgb8(const std::vector<pt_vec3>& image, int width, int height, float samples);
// the PNG bytes stbi_write_png (stb_image_write 0.98, image.cpp:40) writes for these RGB8 rows
std::vector<unsigned char> encode_png(const std::vector<unsigned char>& rgb, int width, int height);
// encode_png to a file; returns false on I/O error
bool write_png(const std::string& path, const std::vector<unsigned char>& rgb, int width, int height);
// little-endian PFM of the accumulated (not averaged) float image, rows bottom-to-top
bool write_pfm(const std::string& path, const std::vector<pt_vec3>& image, int width, int height);
}  // namespace ptio
