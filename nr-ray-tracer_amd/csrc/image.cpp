// Image texture decoding: ImageReader::open(path)?.decode()?.into_rgb32f()
// (lib/textures/image.rs:23-27).  Baseline JPEG is decoded by jpeg.cpp.
#include <cstdio>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "scene_config.hpp"

namespace nrt {

bool decode_jpeg(const std::vector<uint8_t>& data, DecodedImage& out, std::string& err);  // jpeg.cpp

DecodedImage decode_image_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("No such file or directory (os error 2): " + path);
    std::vector<uint8_t> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    data.shrink_to_fit();  // exact allocation: a decoder read past the end is a heap overflow under ASan
    DecodedImage img;
    std::string err;
    if (data.size() >= 3 && data[0] == 0xFF && data[1] == 0xD8) {
        if (!decode_jpeg(data, img, err)) throw std::runtime_error("Format error decoding Jpeg: " + err);
        return img;
    }
    throw std::runtime_error("The image format could not be determined (only baseline JPEG is supported): " + path);
}

}  // namespace nrt
