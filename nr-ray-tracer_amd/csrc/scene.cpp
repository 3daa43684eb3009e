// Host scene graph construction (see scene.hpp for the reference map).
#include "scene.hpp"

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace nrt {

// glam 0.30.9 DMat3::from_axis_angle (Rodrigues), with (sin, cos) from libm.
M3 m3_from_axis_angle(V3 axis, double angle) {
    const double s = std::sin(angle), c = std::cos(angle);
    const double xsin = axis.x * s, ysin = axis.y * s, zsin = axis.z * s;
    const double x = axis.x, y = axis.y, z = axis.z;
    const double x2 = axis.x * axis.x, y2 = axis.y * axis.y, z2 = axis.z * axis.z;
    const double omc = 1.0 - c;
    const double xyomc = x * y * omc;
    const double xzomc = x * z * omc;
    const double yzomc = y * z * omc;
    M3 m;
    m.c[0] = v3(x2 * omc + c, xyomc + zsin, xzomc - ysin);
    m.c[1] = v3(xyomc - zsin, y2 * omc + c, yzomc + xsin);
    m.c[2] = v3(xzomc + ysin, yzomc - xsin, z2 * omc + c);
    return m;
}

M4 m4_from_scale(V3 s) {
    M4 m;
    std::memset(&m, 0, sizeof m);
    m.c[0][0] = s.x;
    m.c[1][1] = s.y;
    m.c[2][2] = s.z;
    m.c[3][3] = 1.0;
    return m;
}

// glam 0.30.9 DMat4::inverse, term for term.
M4 m4_inverse(const M4& M) {
    const double m00 = M.c[0][0], m01 = M.c[0][1], m02 = M.c[0][2], m03 = M.c[0][3];
    const double m10 = M.c[1][0], m11 = M.c[1][1], m12 = M.c[1][2], m13 = M.c[1][3];
    const double m20 = M.c[2][0], m21 = M.c[2][1], m22 = M.c[2][2], m23 = M.c[2][3];
    const double m30 = M.c[3][0], m31 = M.c[3][1], m32 = M.c[3][2], m33 = M.c[3][3];

    const double coef00 = m22 * m33 - m32 * m23;
    const double coef02 = m12 * m33 - m32 * m13;
    const double coef03 = m12 * m23 - m22 * m13;
    const double coef04 = m21 * m33 - m31 * m23;
    const double coef06 = m11 * m33 - m31 * m13;
    const double coef07 = m11 * m23 - m21 * m13;
    const double coef08 = m21 * m32 - m31 * m22;
    const double coef10 = m11 * m32 - m31 * m12;
    const double coef11 = m11 * m22 - m21 * m12;
    const double coef12 = m20 * m33 - m30 * m23;
    const double coef14 = m10 * m33 - m30 * m13;
    const double coef15 = m10 * m23 - m20 * m13;
    const double coef16 = m20 * m32 - m30 * m22;
    const double coef18 = m10 * m32 - m30 * m12;
    const double coef19 = m10 * m22 - m20 * m12;
    const double coef20 = m20 * m31 - m30 * m21;
    const double coef22 = m10 * m31 - m30 * m11;
    const double coef23 = m10 * m21 - m20 * m11;

    const double fac0[4] = {coef00, coef00, coef02, coef03};
    const double fac1[4] = {coef04, coef04, coef06, coef07};
    const double fac2[4] = {coef08, coef08, coef10, coef11};
    const double fac3[4] = {coef12, coef12, coef14, coef15};
    const double fac4[4] = {coef16, coef16, coef18, coef19};
    const double fac5[4] = {coef20, coef20, coef22, coef23};
    const double vec0[4] = {m10, m00, m00, m00};
    const double vec1[4] = {m11, m01, m01, m01};
    const double vec2[4] = {m12, m02, m02, m02};
    const double vec3[4] = {m13, m03, m03, m03};
    const double sign_a[4] = {1.0, -1.0, 1.0, -1.0};
    const double sign_b[4] = {-1.0, 1.0, -1.0, 1.0};

    M4 inv;
    for (int k = 0; k < 4; ++k) {
        const double i0 = (vec1[k] * fac0[k] - vec2[k] * fac1[k]) + vec3[k] * fac2[k];
        const double i1 = (vec0[k] * fac0[k] - vec2[k] * fac3[k]) + vec3[k] * fac4[k];
        const double i2 = (vec0[k] * fac1[k] - vec1[k] * fac3[k]) + vec3[k] * fac5[k];
        const double i3 = (vec0[k] * fac2[k] - vec1[k] * fac4[k]) + vec2[k] * fac5[k];
        inv.c[0][k] = i0 * sign_a[k];
        inv.c[1][k] = i1 * sign_b[k];
        inv.c[2][k] = i2 * sign_a[k];
        inv.c[3][k] = i3 * sign_b[k];
    }
    const double col0[4] = {inv.c[0][0], inv.c[1][0], inv.c[2][0], inv.c[3][0]};
    const double d0 = M.c[0][0] * col0[0], d1 = M.c[0][1] * col0[1], d2 = M.c[0][2] * col0[2],
                 d3 = M.c[0][3] * col0[3];
    const double det = ((d0 + d1) + d2) + d3;
    const double rcp = 1.0 / det;
    for (int cidx = 0; cidx < 4; ++cidx)
        for (int r = 0; r < 4; ++r) inv.c[cidx][r] = inv.c[cidx][r] * rcp;
    return inv;
}

// res = c0*x; res = c1*y + res; res = c2*z + res; res = w + res  (glam DMat4)
V3 m4_transform_point3(const M4& m, V3 r) {
    double o[3];
    for (int k = 0; k < 3; ++k) {
        double res = m.c[0][k] * r.x;
        res = m.c[1][k] * r.y + res;
        res = m.c[2][k] * r.z + res;
        res = m.c[3][k] + res;
        o[k] = res;
    }
    return v3(o[0], o[1], o[2]);
}

V3 m4_transform_vector3(const M4& m, V3 r) {
    double o[3];
    for (int k = 0; k < 3; ++k) {
        double res = m.c[0][k] * r.x;
        res = m.c[1][k] * r.y + res;
        res = m.c[2][k] * r.z + res;
        o[k] = res;
    }
    return v3(o[0], o[1], o[2]);
}

// ------------------------------------------------------------------- AABB
static Interval pad_axis(Interval a) {
    const double eps = 0.0001;  // AABB::EPSILON (aabb.rs:14)
    const double size = a.max - a.min;
    if (size < eps) {
        const double padding = (eps - size) / 2.;
        return {a.min - padding, a.max + padding};
    }
    return a;
}

AABB aabb_new(Interval x, Interval y, Interval z) { return {pad_axis(x), pad_axis(y), pad_axis(z)}; }

AABB aabb_union(const AABB& a, const AABB& b) {
    return aabb_new(interval_union(a.x, b.x), interval_union(a.y, b.y), interval_union(a.z, b.z));
}

AABB aabb_from_points(V3 a, V3 b) {
    Interval x = a.x < b.x ? Interval{a.x, b.x} : Interval{b.x, a.x};
    Interval y = a.y < b.y ? Interval{a.y, b.y} : Interval{b.y, a.y};
    Interval z = a.z < b.z ? Interval{a.z, b.z} : Interval{b.z, a.z};
    return aabb_new(x, y, z);
}

int total_cmp(double a, double b) {
    int64_t ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    ia ^= (int64_t)(((uint64_t)(ia >> 63)) >> 1);
    ib ^= (int64_t)(((uint64_t)(ib >> 63)) >> 1);
    return ia < ib ? -1 : ia > ib ? 1 : 0;
}

// [x, y, z].iter().enumerate().max_by(total_cmp): the LAST maximum wins.
int aabb_longest_axis(const AABB& b) {
    const double s[3] = {b.x.max - b.x.min, b.y.max - b.y.min, b.z.max - b.z.min};
    int best = 0;
    for (int i = 1; i < 3; ++i)
        if (total_cmp(s[best], s[i]) != 1) best = i;
    return best;
}

// ---------------------------------------------------------------- objects
ObjectPtr make_sphere(V3 center, double radius, MaterialPtr mat, const V3* speed) {
    auto o = std::make_shared<Object>();
    o->kind = Object::Sphere;
    o->center = center;
    o->radius = radius;
    o->speed = speed ? *speed : V3{0, 0, 0};
    o->material = std::move(mat);
    const V3 rvec = v3(radius, radius, radius);
    const V3 c0 = center;
    const V3 c1 = center + o->speed;
    const AABB b0 = aabb_from_points(c0 - rvec, c0 + rvec);
    const AABB b1 = aabb_from_points(c1 - rvec, c1 + rvec);
    o->bbox = aabb_union(b0, b1);
    return o;
}

ObjectPtr make_plane(Object::Kind shape, V3 p, V3 u, V3 v, MaterialPtr mat) {
    auto o = std::make_shared<Object>();
    o->kind = shape;
    o->p = p;
    o->u = u;
    o->v = v;
    o->material = std::move(mat);
    const AABB b0 = aabb_from_points(p, p + u + v);
    const AABB b1 = aabb_from_points(p + u, p + v);
    o->bbox = aabb_union(b0, b1);
    const V3 n = cross(u, v);
    o->normal = normalize(n);
    o->d = dot(o->normal, p);
    o->w = n / dot(n, n);
    return o;
}

ObjectPtr make_translate(ObjectPtr child, V3 offset) {
    auto o = std::make_shared<Object>();
    o->kind = Object::Translate;
    o->offset = offset;
    AABB b = child->bbox;  // AABB::translated: interval += offset, no re-padding
    b.x.min += offset.x; b.x.max += offset.x;
    b.y.min += offset.y; b.y.max += offset.y;
    b.z.min += offset.z; b.z.max += offset.z;
    o->bbox = b;
    o->child = std::move(child);
    return o;
}

template <class F>
static AABB transform_bbox(const AABB& bb, F&& f) {
    V3 mn = v3(INFINITY, INFINITY, INFINITY), mx = v3(-INFINITY, -INFINITY, -INFINITY);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                const double x = (double)i * bb.x.max + (1.0 - (double)i) * bb.x.min;
                const double y = (double)j * bb.y.max + (1.0 - (double)j) * bb.y.min;
                const double z = (double)k * bb.z.max + (1.0 - (double)k) * bb.z.min;
                const V3 t = f(v3(x, y, z));
                mn = v3(std::fmin(mn.x, t.x), std::fmin(mn.y, t.y), std::fmin(mn.z, t.z));
                mx = v3(std::fmax(mx.x, t.x), std::fmax(mx.y, t.y), std::fmax(mx.z, t.z));
            }
    return aabb_from_points(mn, mx);
}

ObjectPtr make_rotate(ObjectPtr child, V3 axis, double angle) {
    auto o = std::make_shared<Object>();
    o->kind = Object::Rotate;
    o->rot = m3_from_axis_angle(axis, -angle);
    o->rot_inv = m3_from_axis_angle(axis, angle);
    const M3 mi = o->rot_inv;
    o->bbox = transform_bbox(child->bbox, [&](V3 p) { return mul(mi, p); });
    o->child = std::move(child);
    return o;
}

ObjectPtr make_scale(ObjectPtr child, V3 scale) {
    auto o = std::make_shared<Object>();
    o->kind = Object::Scale;
    o->scale_m = m4_from_scale(scale);
    o->scale_inv = m4_inverse(o->scale_m);
    const M4 sm = o->scale_m;
    o->bbox = transform_bbox(child->bbox, [&](V3 p) { return m4_transform_point3(sm, p); });
    o->child = std::move(child);
    return o;
}

static ObjectPtr bvh_leaf(ObjectPtr child) {
    auto o = std::make_shared<Object>();
    o->kind = Object::BvhLeaf;
    o->bbox = child->bbox;
    o->child = std::move(child);
    return o;
}

static ObjectPtr bvh_from(std::vector<ObjectPtr>& objs, size_t lo, size_t hi) {
    const size_t n = hi - lo;
    if (n == 0) {
        auto o = std::make_shared<Object>();
        o->kind = Object::BvhEmpty;
        o->bbox = AABB::empty();
        return o;
    }
    if (n == 1) return bvh_leaf(objs[lo]);
    auto node = std::make_shared<Object>();
    node->kind = Object::BvhNode;
    if (n == 2) {
        node->left = bvh_leaf(objs[lo]);
        node->right = bvh_leaf(objs[lo + 1]);
        node->bbox = aabb_union(objs[lo]->bbox, objs[lo + 1]->bbox);
        return node;
    }
    AABB bbox = AABB::empty();
    for (size_t k = lo; k < hi; ++k) bbox = aabb_union(bbox, objs[k]->bbox);
    const int axis = aabb_longest_axis(bbox);
    std::stable_sort(objs.begin() + (long)lo, objs.begin() + (long)hi, [axis](const ObjectPtr& a, const ObjectPtr& b) {
        return total_cmp(a->bbox.axis(axis).min, b->bbox.axis(axis).min) < 0;
    });
    const size_t mid = n / 2;
    node->left = bvh_from(objs, lo, lo + mid);
    node->right = bvh_from(objs, lo + mid, hi);
    node->bbox = bbox;
    return node;
}

ObjectPtr make_bvh(std::vector<ObjectPtr>& objs) { return bvh_from(objs, 0, objs.size()); }

// ----------------------------------------------------------------- camera
Camera camera_build(const CameraBuilder& b) {
    Camera c;
    c.width = b.width;
    c.height = b.height;
    c.background_color = b.background_color;
    c.look_from = b.look_from;
    c.ray_max_bounces = b.ray_max_bounces;
    c.samples_per_pixel = std::max<uint64_t>(b.samples_per_pixel, 1);
    double defocus_angle = b.defocus_angle;
    if (defocus_angle < 0.) defocus_angle = 0.;
    if (defocus_angle > M_PI) defocus_angle = M_PI;
    const double focus_dist = b.focus_dist;
    const double h = std::tan(b.field_of_view / 2.);
    const double viewport_height = focus_dist * h * 2.0;
    const double aspect = (double)b.width / (double)b.height;
    const double viewport_width = viewport_height * aspect;
    const V3 w = normalize(b.look_from - b.look_at);
    const V3 u = normalize(cross(b.view_up, w));
    const V3 v = normalize(cross(w, u));
    const V3 viewport_u = u * viewport_width;
    const V3 viewport_v = (-v) * viewport_height;
    c.pixel_delta_u = viewport_u / (double)b.width;
    c.pixel_delta_v = viewport_v / (double)b.height;
    c.top_left = (((b.look_from - w * focus_dist) - viewport_u / 2.0) - viewport_v / 2.0) +
                 (c.pixel_delta_u + c.pixel_delta_v) / 2.0;
    const double defocus_radius = focus_dist * std::tan(defocus_angle / 2.0);
    c.defocus_disk_u = u * defocus_radius;
    c.defocus_disk_v = v * defocus_radius;
    return c;
}

}  // namespace nrt
