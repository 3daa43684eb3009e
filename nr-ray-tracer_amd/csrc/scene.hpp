// Host-side scene graph: the reference's `Hitable` / `Material` / `Texture`
// trait objects restated as plain C++ so the BVH and every bounding box is
// built with the reference's exact f64 arithmetic before flattening.
//
//   lib/objects/object.rs:40-121   BVH (median split, un-narrowed hit, ties -> right)
//   lib/objects/sphere.rs:69-92  Sphere bbox
//   lib/objects/plane.rs:95-128   Plane precompute (normal, d, w, bbox)
//   lib/objects/translate.rs:18-30, rotate.rs:46-106, scale.rs:43-86  transform bboxes
//   lib/aabb.rs:13-132, lib/interval.rs:10-94  AABB / Interval
//   lib/camera.rs:94-159           CameraBuilder::build
//
// Every operation is written in glam 0.30.9's evaluation order (dot is
// left-to-right, normalize = v * (1/sqrt(dot)), DMat3*v = (c0*x + c1*y) + c2*z,
// DMat4::transform_point3 = w + (c2*z + (c1*y + c0*x))) and the host code is
// compiled with -ffp-contract=off, so results are bit-identical to the Rust
// reference on the same libm.
#pragma once

#include <cmath>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "noise.hpp"

namespace nrt {

struct V3 {
    double x = 0, y = 0, z = 0;
};
inline V3 v3(double x, double y, double z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 operator-(V3 a) { return {-a.x, -a.y, -a.z}; }
inline V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 operator*(double s, V3 a) { return {s * a.x, s * a.y, s * a.z}; }
inline V3 operator/(V3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3 cross(V3 a, V3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
inline V3 normalize(V3 a) { return a * (1.0 / std::sqrt(dot(a, a))); }

// glam DMat3, column major: c[0], c[1], c[2] are the columns.
struct M3 {
    V3 c[3];
};
inline V3 mul(const M3& m, V3 r) { return (m.c[0] * r.x + m.c[1] * r.y) + m.c[2] * r.z; }
M3 m3_from_axis_angle(V3 axis, double angle);  // glam DMat3::from_axis_angle

// glam DMat4, column major.
struct M4 {
    double c[4][4];  // c[col][row]
};
M4 m4_from_scale(V3 s);
M4 m4_inverse(const M4& m);  // glam DMat4::inverse (cofactor form)
V3 m4_transform_point3(const M4& m, V3 r);
V3 m4_transform_vector3(const M4& m, V3 r);

struct Interval {
    double min, max;
};
inline Interval interval_union(Interval a, Interval b) { return {std::fmin(a.min, b.min), std::fmax(a.max, b.max)}; }

struct AABB {
    Interval x, y, z;
    static AABB empty() { return {{INFINITY, -INFINITY}, {INFINITY, -INFINITY}, {INFINITY, -INFINITY}}; }
    const Interval& axis(int i) const { return i == 0 ? x : i == 1 ? y : z; }
};
AABB aabb_new(Interval x, Interval y, Interval z);  // pads thin axes (aabb.rs:14-40)
AABB aabb_union(const AABB& a, const AABB& b);
AABB aabb_from_points(V3 a, V3 b);
int aabb_longest_axis(const AABB& b);
int total_cmp(double a, double b);  // f64::total_cmp as -1/0/1

// ---------------------------------------------------------------- textures
struct Texture {
    enum Kind { Solid, Image, Checker, Noise, Marble } kind = Solid;
    V3 color{1, 1, 1};
    // Image: Rgb32F texels (decoded u8/255, no sRGB linearisation, textures/image.rs:23-27)
    uint32_t width = 0, height = 0;
    std::shared_ptr<std::vector<float>> texels;
    std::shared_ptr<Texture> even, odd;
    double scale = 0.5;
    FbmParams fbm;  // Noise / Marble (noise.hpp)
};
using TexturePtr = std::shared_ptr<Texture>;

// -------------------------------------------------------------- materials
struct Material {
    enum Kind { Lambertian, Metal, Dielectric, DiffuseLight } kind = Lambertian;
    TexturePtr texture;
    double fuzz = 0.0;
    double refraction_index = 1.5;
    double intensity = 4.0;
};
using MaterialPtr = std::shared_ptr<Material>;

// ---------------------------------------------------------------- objects
struct Object;
using ObjectPtr = std::shared_ptr<Object>;

struct Object {
    enum Kind {
        Sphere,
        Quad,
        Triangle,
        BvhEmpty,  // BVH::Leaf(None)
        BvhLeaf,   // BVH::Leaf(Some(child))
        BvhNode,   // BVH::Node{bbox, left, right}
        Translate,
        Rotate,
        Scale,
    } kind = BvhEmpty;
    AABB bbox = AABB::empty();
    MaterialPtr material;
    // Sphere
    V3 center;
    V3 speed;  // Ray::new(center, speed).at(time); zero unless a moving sphere
    double radius = 0;
    // Plane (Quad / Triangle)
    V3 p, u, v, normal, w;
    double d = 0;
    // Translate
    V3 offset;
    // Rotate: object-space ray = mat * world ray; hit point/normal back with mat_inv
    M3 rot, rot_inv;
    // Scale: ray into object space with scale_inv, hit point back with scale
    M4 scale_m, scale_inv;
    // children
    ObjectPtr child, left, right;
};

ObjectPtr make_sphere(V3 center, double radius, MaterialPtr mat, const V3* speed = nullptr);
ObjectPtr make_plane(Object::Kind shape, V3 p, V3 u, V3 v, MaterialPtr mat);
ObjectPtr make_translate(ObjectPtr child, V3 offset);
ObjectPtr make_rotate(ObjectPtr child, V3 axis, double angle);
ObjectPtr make_scale(ObjectPtr child, V3 scale);
// BVH::from — sorts `objs` in place exactly as the reference's slice sort does.
ObjectPtr make_bvh(std::vector<ObjectPtr>& objs);

// ----------------------------------------------------------------- camera
struct CameraBuilder {
    uint64_t width = 1200, height = 800;
    V3 background_color{0, 0, 0};
    V3 look_from{1, 1, 1};
    V3 look_at{0, 0, 0};
    V3 view_up{0, 1, 0};
    double defocus_angle = 0.0;
    double focus_dist = 1.0;
    double field_of_view = M_PI / 2.0;
    uint64_t ray_max_bounces = 10;
    uint64_t samples_per_pixel = 10;
};

struct Camera {
    uint64_t width, height, samples_per_pixel, ray_max_bounces;
    V3 background_color, look_from, defocus_disk_u, defocus_disk_v, pixel_delta_u, pixel_delta_v, top_left;
};
Camera camera_build(const CameraBuilder& b);

}  // namespace nrt
