// SceneConfig semantics (packages/ray-tracer/src/scene_config.rs:26-497) and
// CameraConfig merge/update rules (packages/ray-tracer/src/cli.rs:157-402).
#pragma once

#include <cstdint>
#include <string>

#include "scene.hpp"
#include "value.hpp"

namespace nrt {

// cli.rs:160-270 — every field optional.
struct CameraConfig {
    bool has_width = false, has_height = false, has_aspect_ratio = false, has_background_color = false,
         has_look_at = false, has_look_from = false, has_view_up = false, has_focal_length = false,
         has_field_of_view = false, has_defocus_angle = false, has_focus_distance = false,
         has_samples_per_pixel = false, has_ray_max_bounces = false;
    uint64_t width = 0, height = 0;
    double aspect_ratio = 0;
    V3 background_color, look_at, look_from, view_up;
    double focal_length = 0, field_of_view = 0, defocus_angle = 0, focus_distance = 0;
    uint64_t samples_per_pixel = 0, ray_max_bounces = 0;

    void merge_with(const CameraConfig& other);          // cli.rs:316-355
    void try_update(CameraBuilder& builder) const;      // cli.rs:357-402 (throws on size rules)
};

struct LoadedScene {
    ObjectPtr objects;  // Scene.objects: the top-level BVH (scene_config.rs:469-472)
    Camera camera;
};

// SceneConfig::try_load_scene + merge_with(cli) + try_build  (render.rs:107-111); legacy_schema:
// also accept the index schema of scenes/triangles.toml (normalize_legacy)
LoadedScene load_scene_file(const std::string& path, const CameraConfig* cli_overrides, bool legacy_schema = false);

// Decoded Rgb32F image (u8/255 per channel), ImageReader::decode().into_rgb32f().
struct DecodedImage {
    uint32_t width = 0, height = 0;
    std::vector<float> rgb;
};
DecodedImage decode_image_file(const std::string& path);  // image.cpp

}  // namespace nrt
