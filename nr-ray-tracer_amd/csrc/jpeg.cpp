// Placeholder until the baseline JPEG decoder lands.
#include <string>
#include <vector>

#include "scene_config.hpp"

namespace nrt {
bool decode_jpeg(const std::vector<uint8_t>&, DecodedImage&, std::string& err) {
    err = "JPEG decoding not implemented yet";
    return false;
}
}  // namespace nrt
