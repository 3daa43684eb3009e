// ORACLE — test infrastructure only.  NOT part of the product path.
//
// A CPU, f64, line-by-line restatement of nr-ray-tracer's render path, used
// solely as the parity checker by tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py.  It deliberately keeps the reference's shape:
// virtual `Hitable` objects, a recursive un-narrowed BVH::hit, recursive
// get_ray_color, and rand_chacha's BlockRng (64-word buffer, 4 blocks per
// refill) — so it is the reference's arithmetic, not the GPU kernel's.
//
// Reference (packages/ray-tracer-lib/src/, read-only at /root/reference):
//   camera.rs:94-159 (build), 236-267 (get_ray), 269-300 (get_ray_color), 302-343 (render)
//   vector.rs:27-81  objects/object.rs:40-121  objects/sphere.rs:69-163
//   objects/plane.rs:23-30, 95-174  objects/translate.rs:17-50  objects/rotate.rs:13-106
//   objects/scale.rs:10-86  aabb.rs:13-132  interval.rs:10-94  hitable.rs:37-77
//   materials/*.rs  textures/{solid_color,image,checker,noise,marble}.rs
// Third-party arithmetic restated from the pinned crates (Cargo.lock):
//   rand_core 0.9.3 seed_from_u64 (PCG32), rand_chacha 0.9.0 ChaCha8 BlockRng,
//   rand 0.9.2 UniformFloat::sample_single(_inclusive), glam 0.30.9 DVec3/DMat3/DMat4,
//   noise 0.9.0 Perlin/Fbm/Abs with rand 0.8.5 shuffle + rand_xorshift 0.3.0 (Perlin textures).
// Parity pinning: the reference publishes no tests or golden vectors;
// the ChaCha core is pinned against OpenSSL's ChaCha20 and the RFC 7539 vector
// (tests/test_oracle.py), everything else is "parity unpinned" beyond this restatement.
//
// Build: oracle/Makefile (g++ -O3 -ffp-contract=off).  Usage:
//   oracle render <tree> <out.f32> [--threads N] [--rows off stride] [--spp N] [--stats out.json]
//   oracle dump <tree>                   canonical scene-graph dump (matches nrt_scene_dump)
//   oracle rng <stream> <count>          first draws of a pixel stream (hex u64 per line)
//   oracle chacha <rounds> <key-hex64> <ctr> <nonce> <nwords>   raw keystream words
//   oracle xorshift <seed-hex32> <n> | perm <seed> | noise <seed> <oct> <freq> <lac> <pers> <x> <y> <z>
//   oracle marble <seed> <freq> <x> <y> <z>      Perlin-texture pieces (tests)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <optional>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#ifdef ORACLE_COUNTERS
#define NRT_COUNT(x) (x)
#else
#define NRT_COUNT(x) ((void)0)
#endif

namespace oracle {

// ------------------------------------------------------------- glam DVec3
struct DVec3 {
    double x, y, z;
};
static DVec3 operator+(DVec3 a, DVec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static DVec3 operator-(DVec3 a, DVec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static DVec3 operator-(DVec3 a) { return {-a.x, -a.y, -a.z}; }
static DVec3 operator*(double s, DVec3 a) { return {s * a.x, s * a.y, s * a.z}; }
static DVec3 operator*(DVec3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static DVec3 operator*(DVec3 a, DVec3 b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
static DVec3 operator/(DVec3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
static double dot(DVec3 a, DVec3 b) { return (a.x * b.x) + (a.y * b.y) + (a.z * b.z); }
static DVec3 cross(DVec3 a, DVec3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
static double length_squared(DVec3 a) { return dot(a, a); }
static DVec3 normalize(DVec3 a) { return a * (1.0 / std::sqrt(dot(a, a))); }
static DVec3 vmin(DVec3 a, DVec3 b) { return {std::fmin(a.x, b.x), std::fmin(a.y, b.y), std::fmin(a.z, b.z)}; }
static DVec3 vmax(DVec3 a, DVec3 b) { return {std::fmax(a.x, b.x), std::fmax(a.y, b.y), std::fmax(a.z, b.z)}; }
// glam reflect / refract
static DVec3 reflect(DVec3 v, DVec3 n) { return v - 2.0 * dot(v, n) * n; }
static DVec3 refract(DVec3 i, DVec3 n, double eta) {
    const double n_dot_i = dot(n, i);
    const double k = 1.0 - eta * eta * (1.0 - n_dot_i * n_dot_i);
    if (k >= 0.0) return eta * i - (eta * n_dot_i + std::sqrt(k)) * n;
    return {0, 0, 0};
}
struct DVec2 {
    double x, y;
};

struct DMat3 {  // columns
    DVec3 x_axis, y_axis, z_axis;
    DVec3 operator*(DVec3 r) const {
        DVec3 res = x_axis * r.x;
        res = res + y_axis * r.y;
        res = res + z_axis * r.z;
        return res;
    }
    static DMat3 from_axis_angle(DVec3 axis, double angle) {
        const double sin = std::sin(angle), cos = std::cos(angle);
        const DVec3 s = axis * sin;
        const DVec3 a2 = axis * axis;
        const double omc = 1.0 - cos;
        const double xyomc = axis.x * axis.y * omc;
        const double xzomc = axis.x * axis.z * omc;
        const double yzomc = axis.y * axis.z * omc;
        return {{a2.x * omc + cos, xyomc + s.z, xzomc - s.y},
                {xyomc - s.z, a2.y * omc + cos, yzomc + s.x},
                {xzomc + s.y, yzomc - s.x, a2.z * omc + cos}};
    }
};

struct DVec4 {
    double x, y, z, w;
};
static DVec4 operator*(DVec4 a, DVec4 b) { return {a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w}; }
static DVec4 operator-(DVec4 a, DVec4 b) { return {a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
static DVec4 operator+(DVec4 a, DVec4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }
static DVec4 operator*(DVec4 a, double s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }

struct DMat4 {
    DVec4 x_axis, y_axis, z_axis, w_axis;
    static DMat4 from_scale(DVec3 s) { return {{s.x, 0, 0, 0}, {0, s.y, 0, 0}, {0, 0, s.z, 0}, {0, 0, 0, 1}}; }
    DMat4 inverse() const {
        const double m00 = x_axis.x, m01 = x_axis.y, m02 = x_axis.z, m03 = x_axis.w;
        const double m10 = y_axis.x, m11 = y_axis.y, m12 = y_axis.z, m13 = y_axis.w;
        const double m20 = z_axis.x, m21 = z_axis.y, m22 = z_axis.z, m23 = z_axis.w;
        const double m30 = w_axis.x, m31 = w_axis.y, m32 = w_axis.z, m33 = w_axis.w;
        const double coef00 = m22 * m33 - m32 * m23, coef02 = m12 * m33 - m32 * m13, coef03 = m12 * m23 - m22 * m13;
        const double coef04 = m21 * m33 - m31 * m23, coef06 = m11 * m33 - m31 * m13, coef07 = m11 * m23 - m21 * m13;
        const double coef08 = m21 * m32 - m31 * m22, coef10 = m11 * m32 - m31 * m12, coef11 = m11 * m22 - m21 * m12;
        const double coef12 = m20 * m33 - m30 * m23, coef14 = m10 * m33 - m30 * m13, coef15 = m10 * m23 - m20 * m13;
        const double coef16 = m20 * m32 - m30 * m22, coef18 = m10 * m32 - m30 * m12, coef19 = m10 * m22 - m20 * m12;
        const double coef20 = m20 * m31 - m30 * m21, coef22 = m10 * m31 - m30 * m11, coef23 = m10 * m21 - m20 * m11;
        const DVec4 fac0{coef00, coef00, coef02, coef03}, fac1{coef04, coef04, coef06, coef07};
        const DVec4 fac2{coef08, coef08, coef10, coef11}, fac3{coef12, coef12, coef14, coef15};
        const DVec4 fac4{coef16, coef16, coef18, coef19}, fac5{coef20, coef20, coef22, coef23};
        const DVec4 vec0{m10, m00, m00, m00}, vec1{m11, m01, m01, m01};
        const DVec4 vec2{m12, m02, m02, m02}, vec3{m13, m03, m03, m03};
        const DVec4 inv0 = (vec1 * fac0 - vec2 * fac1) + vec3 * fac2;
        const DVec4 inv1 = (vec0 * fac0 - vec2 * fac3) + vec3 * fac4;
        const DVec4 inv2 = (vec0 * fac1 - vec1 * fac3) + vec3 * fac5;
        const DVec4 inv3 = (vec0 * fac2 - vec1 * fac4) + vec2 * fac5;
        const DVec4 sign_a{1.0, -1.0, 1.0, -1.0}, sign_b{-1.0, 1.0, -1.0, 1.0};
        DMat4 inv{inv0 * sign_a, inv1 * sign_b, inv2 * sign_a, inv3 * sign_b};
        const DVec4 col0{inv.x_axis.x, inv.y_axis.x, inv.z_axis.x, inv.w_axis.x};
        const DVec4 dot0 = x_axis * col0;
        const double dot1 = dot0.x + dot0.y + dot0.z + dot0.w;
        const double rcp_det = 1.0 / dot1;
        return {inv.x_axis * rcp_det, inv.y_axis * rcp_det, inv.z_axis * rcp_det, inv.w_axis * rcp_det};
    }
    DVec3 transform_point3(DVec3 r) const {
        DVec4 res = x_axis * r.x;
        res = y_axis * r.y + res;
        res = z_axis * r.z + res;
        res = w_axis + res;
        return {res.x, res.y, res.z};
    }
    DVec3 transform_vector3(DVec3 r) const {
        DVec4 res = x_axis * r.x;
        res = y_axis * r.y + res;
        res = z_axis * r.z + res;
        return {res.x, res.y, res.z};
    }
};

// ------------------------------------------------------------- ChaCha8Rng
static inline uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void chacha_block(int rounds, const uint32_t key[8], uint64_t ctr, uint64_t nonce, uint32_t out[16]) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                      key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), (uint32_t)nonce,
                      (uint32_t)(nonce >> 32)};
    uint32_t x[16];
    memcpy(x, s, sizeof x);
    auto qr = [&](int a, int b, int c, int d) {
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl(x[d], 16);
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl(x[b], 12);
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl(x[d], 8);
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl(x[b], 7);
    };
    for (int r = 0; r < rounds; r += 2) {
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + s[i];
}

// rand_core 0.9.3 SeedableRng::seed_from_u64 — PCG32 fills the 32-byte seed.
static void seed_from_u64(uint64_t state, uint32_t key[8]) {
    for (int i = 0; i < 8; ++i) {
        state = state * 6364136223846793005ull + 11634580027462260723ull;
        const uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
        const uint32_t rot = (uint32_t)(state >> 59);
        key[i] = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    }
}

// rand_chacha 0.9.0: BlockRng<ChaCha8Core> with a 64-word result buffer filled
// 4 blocks at a time; set_stream on a fresh rng only sets the nonce.
struct ChaCha8Rng {
    uint32_t key[8];
    uint64_t block_pos = 0, stream = 0;
    uint32_t results[64];
    size_t index = 64;
    uint64_t draws = 0;

    static ChaCha8Rng seed_from_u64(uint64_t s) {
        ChaCha8Rng r;
        oracle::seed_from_u64(s, r.key);
        return r;
    }
    void set_stream(uint64_t s) { stream = s; }  // index == 64: nothing buffered yet
    void generate() {
        for (int b = 0; b < 4; ++b) chacha_block(8, key, block_pos + (uint64_t)b, stream, results + 16 * b);
        block_pos += 4;
    }
    uint32_t next_u32() {
        if (index >= 64) { generate(); index = 0; }
        return results[index++];
    }
    uint64_t next_u64() {  // BlockRng::next_u64
        NRT_COUNT(++draws);
        const size_t len = 64;
        if (index < len - 1) {
            const uint64_t v = (uint64_t)results[index] | ((uint64_t)results[index + 1] << 32);
            index += 2;
            return v;
        } else if (index >= len) {
            generate();
            index = 2;
            return (uint64_t)results[0] | ((uint64_t)results[1] << 32);
        } else {
            const uint64_t x = results[len - 1];
            generate();
            index = 1;
            const uint64_t y = results[0];
            return (y << 32) | x;
        }
    }
};

// rand 0.9.2: Rng::random_range on f64 ranges = UniformFloat::sample_single(_inclusive):
// one draw, value1_2 = from_bits((u >> 12) | 1.0.to_bits()); (value1_2 - 1) * (high - low) + low.
static double random_range(ChaCha8Rng& rng, double low, double high) {
    const uint64_t u = rng.next_u64();
    uint64_t bits = (u >> 12) | 0x3FF0000000000000ull;
    double v12;
    memcpy(&v12, &bits, 8);
    const double value0_1 = v12 - 1.0;
    const double scale = high - low;
    return value0_1 * scale + low;
}

// ------------------------------------------------------------- vector.rs
static DVec3 random_in_unit_sphere(ChaCha8Rng& rng) {
    while (true) {
        const double x = random_range(rng, -1.0, 1.0);
        const double y = random_range(rng, -1.0, 1.0);
        const double z = random_range(rng, -1.0, 1.0);
        const DVec3 p{x, y, z};
        const double ls = length_squared(p);
        if (1e-160 < ls && ls <= 1.0) return p / ls;
    }
}
static DVec3 random_in_unit_disk(ChaCha8Rng& rng) {
    while (true) {
        const double x = random_range(rng, -1.0, 1.0);
        const double y = random_range(rng, -1.0, 1.0);
        const DVec3 p{x, y, 0.0};
        const double ls = length_squared(p);
        if (ls < 1.0) return p / ls;
    }
}
static bool almost_zero(DVec3 v, double eps) { return std::fabs(v.x) < eps && std::fabs(v.y) < eps && std::fabs(v.z) < eps; }

// ---------------------------------------------------- interval.rs / aabb.rs
struct Interval {
    double min, max;
    static Interval ensure(double a, double b) { return a < b ? Interval{a, b} : Interval{b, a}; }
    Interval unite(const Interval& o) const { return {std::fmin(min, o.min), std::fmax(max, o.max)}; }
    Interval intersection(const Interval& o) const { return {std::fmax(min, o.min), std::fmin(max, o.max)}; }
    bool is_empty() const { return min > max; }
    Interval pad(double p) const { return {min - p, max + p}; }
    double size() const { return max - min; }
    bool contains(double v) const { return min <= v && v <= max; }
    bool surrounds(double v) const { return min < v && v < max; }
};
static const double INF = INFINITY;

struct AABB {
    Interval x, y, z;
    static AABB pad_to_minimums(AABB b) {
        const double E = 0.0001;
        if (b.x.size() < E) b.x = b.x.pad((E - b.x.size()) / 2.);
        if (b.y.size() < E) b.y = b.y.pad((E - b.y.size()) / 2.);
        if (b.z.size() < E) b.z = b.z.pad((E - b.z.size()) / 2.);
        return b;
    }
    static AABB make(Interval x, Interval y, Interval z) { return pad_to_minimums({x, y, z}); }
    static AABB empty() { return {{INF, -INF}, {INF, -INF}, {INF, -INF}}; }
    AABB unite(const AABB& o) const { return make(x.unite(o.x), y.unite(o.y), z.unite(o.z)); }
    static AABB from_points(DVec3 a, DVec3 b) {
        Interval ix = a.x < b.x ? Interval{a.x, b.x} : Interval{b.x, a.x};
        Interval iy = a.y < b.y ? Interval{a.y, b.y} : Interval{b.y, a.y};
        Interval iz = a.z < b.z ? Interval{a.z, b.z} : Interval{b.z, a.z};
        return make(ix, iy, iz);
    }
    const Interval& axis_interval(int i) const { return i == 0 ? x : i == 1 ? y : z; }
};

static int total_cmp(double a, double b) {
    int64_t l, r;
    memcpy(&l, &a, 8);
    memcpy(&r, &b, 8);
    l ^= (int64_t)(((uint64_t)(l >> 63)) >> 1);
    r ^= (int64_t)(((uint64_t)(r >> 63)) >> 1);
    return (l > r) - (l < r);
}

static int longest_axis(const AABB& b) {  // max_by(total_cmp): last maximum wins
    const double s[3] = {b.x.size(), b.y.size(), b.z.size()};
    int best = 0;
    for (int i = 1; i < 3; ++i)
        if (total_cmp(s[i], s[best]) >= 0) best = i;
    return best;
}

// -------------------------------------------------------------- counters
struct Counters {
    uint64_t aabb_tests = 0, sphere_tests = 0, sphere_hits = 0, plane_tests = 0, plane_hits = 0;
    uint64_t transform_enters = 0, rays = 0, scatter_tries = 0, camera_rays = 0, draws = 0, texel_fetches = 0;
};
static thread_local Counters tl;
#ifdef ORACLE_COUNTERS
#define NRT_COUNT(x) (x)
#else
#define NRT_COUNT(x) ((void)0)
#endif

// ------------------------------------------------------------------- Ray
struct Ray {
    DVec3 origin, direction;
    uint64_t bounce = 0;
    double time = 0;
    DVec3 at(double t) const { return origin + t * direction; }
};

static bool aabb_hit(const AABB& b, const Ray& ray, Interval range) {
    NRT_COUNT(tl.aabb_tests += 1);
    Interval interval = range;
    const Interval axes[3] = {b.x, b.y, b.z};
    const double o[3] = {ray.origin.x, ray.origin.y, ray.origin.z};
    const double d[3] = {ray.direction.x, ray.direction.y, ray.direction.z};
    for (int k = 0; k < 3; ++k) {
        interval = interval.intersection(Interval::ensure((axes[k].min - o[k]) / d[k], (axes[k].max - o[k]) / d[k]));
        if (interval.is_empty()) return false;
    }
    return true;
}

// -------------------------------------------------------------- textures
struct Texture {
    virtual ~Texture() = default;
    virtual DVec3 get_color(DVec2 uv, DVec3 p) const = 0;
    virtual std::string desc() const = 0;
};
using TexP = std::shared_ptr<Texture>;

static std::string hx(double v) {
    char b[64];
    snprintf(b, sizeof b, " %a", v);
    return b;
}
static std::string hx3(DVec3 v) { return hx(v.x) + hx(v.y) + hx(v.z); }
static std::string hxbox(const AABB& b) {
    return hx(b.x.min) + hx(b.x.max) + hx(b.y.min) + hx(b.y.max) + hx(b.z.min) + hx(b.z.max);
}

struct SolidColor : Texture {
    DVec3 color;
    explicit SolidColor(DVec3 c) : color(c) {}
    DVec3 get_color(DVec2, DVec3) const override { return color; }
    std::string desc() const override { return " SOLID" + hx3(color); }
};
struct ImageTex : Texture {
    uint32_t w, h;
    std::vector<float> px;
    DVec3 get_color(DVec2 uv, DVec3) const override {
        NRT_COUNT(tl.texel_fetches += 1);
        auto clamp01 = [](double v) { return v < 0. ? 0. : (v > 1. ? 1. : v); };
        auto as_u32 = [](double v) -> uint32_t {
            if (!(v > 0)) return 0;
            if (v >= 4294967295.0) return 4294967295u;
            return (uint32_t)v;
        };
        uint32_t x = as_u32(clamp01(uv.x) * (double)w);
        uint32_t y = as_u32((1.0 - clamp01(uv.y)) * (double)h);
        // get_pixel panics for x == w / y == h; clamp like the GPU.
        if (x >= w) x = w - 1;
        if (y >= h) y = h - 1;
        const float* p = &px[3 * ((size_t)y * w + x)];
        return {(double)p[0], (double)p[1], (double)p[2]};
    }
    std::string desc() const override {
        double s = 0;
        for (float f : px) s += f;
        char b[64];
        snprintf(b, sizeof b, " IMAGE %u %u", w, h);
        return b + hx(s);
    }
};
struct Checker : Texture {
    TexP even, odd;
    double scale;
    DVec3 get_color(DVec2 uv, DVec3 p) const override {
        auto as_u64 = [](double v) -> uint64_t {
            if (!(v > 0)) return 0;
            if (v >= 18446744073709551615.0) return ~0ull;
            return (uint64_t)v;
        };
        const uint64_t v = as_u64(uv.x * scale) + as_u64(uv.y * scale);
        return v % 2 == 0 ? even->get_color(uv, p) : odd->get_color(uv, p);
    }
    std::string desc() const override { return " CHECKER" + hx(scale) + " (" + even->desc() + " ) (" + odd->desc() + " )"; }
};

// ------------------------------------------------------- Perlin textures
// textures/noise.rs:79-145 (PerlinRidgedNoise = Abs<Fbm<Perlin>>), textures/marble.rs:46-96.
// The `noise` crate is third-party (Cargo.lock: noise 0.9.0, with rand 0.8.5 and
// rand_xorshift 0.3.0) and absent from /root/reference: restated from its published
// source as remembered — PARITY UNPINNED (no reference test or vector covers it).
namespace perlin_crate {
// rand_xorshift 0.3.0: XorShiftRng::from_seed([u8; 16]) reads 4 LE u32 (x, y, z, w)
struct XorShiftRng {
    uint32_t x, y, z, w;
    explicit XorShiftRng(const uint8_t seed[16]) {
        uint32_t v[4];
        for (int i = 0; i < 4; ++i)
            v[i] = (uint32_t)seed[4 * i] | (uint32_t)seed[4 * i + 1] << 8 | (uint32_t)seed[4 * i + 2] << 16 |
                   (uint32_t)seed[4 * i + 3] << 24;
        if (!(v[0] | v[1] | v[2] | v[3])) v[0] = v[1] = v[2] = v[3] = 0x0BAD5EEDu;
        x = v[0]; y = v[1]; z = v[2]; w = v[3];
    }
    uint32_t next_u32() {
        const uint32_t t = x ^ (x << 11);
        x = y; y = z; z = w;
        w = w ^ (w >> 19) ^ (t ^ (t >> 8));
        return w;
    }
};
// rand 0.8.5: Rng::gen_range(0..ubound) for u32 = UniformInt::sample_single_inclusive(0, ubound - 1)
static uint32_t gen_range_u32(XorShiftRng& rng, uint32_t low, uint32_t high_incl) {
    const uint32_t range = high_incl - low + 1u;
    if (range == 0) return rng.next_u32();
    const uint32_t zone = (range << __builtin_clz(range)) - 1u;  // "conservative but fast approximation"
    for (;;) {
        const uint64_t m = (uint64_t)rng.next_u32() * (uint64_t)range;  // v.wmul(range)
        const uint32_t hi = (uint32_t)(m >> 32), lo = (uint32_t)m;
        if (lo <= zone) return low + hi;
    }
}
// noise 0.9.0 PermutationTable::new(seed): seed bytes [1,0,0,0, s0..s3 x3], Standard sample =
// [0..=255] shuffled by SliceRandom::shuffle (for i in (1..len).rev(): swap(i, gen_index(i + 1)))
struct PermutationTable {
    uint8_t values[256];
    explicit PermutationTable(uint32_t seed) {
        uint8_t real[16] = {0};
        real[0] = 1;
        for (int i = 1; i < 4; ++i) {
            real[i * 4] = (uint8_t)seed;
            real[i * 4 + 1] = (uint8_t)(seed >> 8);
            real[i * 4 + 2] = (uint8_t)(seed >> 16);
            real[i * 4 + 3] = (uint8_t)(seed >> 24);
        }
        XorShiftRng rng(real);
        for (int i = 0; i < 256; ++i) values[i] = (uint8_t)i;
        for (int i = 255; i >= 1; --i) {
            const uint32_t j = gen_range_u32(rng, 0, (uint32_t)i);
            std::swap(values[i], values[j]);
        }
    }
    // NoiseHasher::hash: fold (a & 0xff) with values[a] ^ b, then one more lookup
    size_t hash(const int64_t* v, int n) const {
        size_t idx = (size_t)(v[0] & 0xff);
        for (int i = 1; i < n; ++i) idx = (size_t)values[idx] ^ (size_t)(v[i] & 0xff);
        return values[idx];
    }
};
// core/perlin.rs perlin_3d
static double gradient_dot_v(size_t perm, double x, double y, double z) {
    switch (perm & 0b1111) {
        case 0: return x + y;    case 1: return -x + y;   case 2: return x - y;    case 3: return -x - y;
        case 4: return x + z;    case 5: return -x + z;   case 6: return x - z;    case 7: return -x - z;
        case 8: return y + z;    case 9: return -y + z;   case 10: return y - z;   case 11: return -y - z;
        case 12: return x + y;   case 13: return -x + y;  case 14: return -y + z;  default: return -y - z;
    }
}
static double map_quintic(double x) { return x * x * x * (x * (x * 6.0 - 15.0) + 10.0); }
static double perlin_3d(const PermutationTable& hasher, DVec3 point) {
    const double SCALE_FACTOR = 1.154'700'538'379'251'5;
    const DVec3 floored{std::floor(point.x), std::floor(point.y), std::floor(point.z)};
    const int64_t corner[3] = {(int64_t)floored.x, (int64_t)floored.y, (int64_t)floored.z};
    const DVec3 distance{point.x - floored.x, point.y - floored.y, point.z - floored.z};
    auto g = [&](int ox, int oy, int oz) {
        const int64_t c[3] = {corner[0] + ox, corner[1] + oy, corner[2] + oz};
        return gradient_dot_v(hasher.hash(c, 3), distance.x - (double)ox, distance.y - (double)oy,
                              distance.z - (double)oz);
    };
    const double g000 = g(0, 0, 0), g100 = g(1, 0, 0), g010 = g(0, 1, 0), g110 = g(1, 1, 0);
    const double g001 = g(0, 0, 1), g101 = g(1, 0, 1), g011 = g(0, 1, 1), g111 = g(1, 1, 1);
    const double a = map_quintic(distance.x), b = map_quintic(distance.y), c = map_quintic(distance.z);
    const double k0 = g000;
    const double k1 = g100 - g000;
    const double k2 = g010 - g000;
    const double k3 = g001 - g000;
    const double k4 = g000 + g110 - g100 - g010;
    const double k5 = g000 + g101 - g100 - g001;
    const double k6 = g000 + g011 - g010 - g001;
    const double k7 = g100 + g010 + g001 + g111 - g000 - g110 - g101 - g011;
    const double result = k0 + k1 * a + k2 * b + k3 * c + k4 * a * b + k5 * a * c + k6 * b * c + k7 * a * b * c;
    return std::clamp(result * SCALE_FACTOR, -1.0, 1.0);
}
// f64::powi -> llvm.powi -> compiler-rt __powidf2
static double powi(double a, int b) {
    const bool recip = b < 0;
    double r = 1;
    for (;;) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1 / r : r;
}
// source/generators/fractals/fbm.rs
struct Fbm {
    static constexpr double DEFAULT_FREQUENCY = 1.0;
    static constexpr double DEFAULT_LACUNARITY = M_PI * 2.0 / 3.0;
    static constexpr double DEFAULT_PERSISTENCE = 0.5;
    static constexpr size_t MAX_OCTAVES = 32;
    uint32_t seed;
    size_t octaves = 6;
    double frequency = DEFAULT_FREQUENCY, lacunarity = DEFAULT_LACUNARITY, persistence = DEFAULT_PERSISTENCE;
    std::vector<PermutationTable> sources;
    double scale_factor;
    static double calc_scale_factor(double persistence, size_t octaves) {
        double denom = 0.0;
        for (size_t x = 1; x <= octaves; ++x) denom = denom + powi(persistence, (int)x);
        return 1.0 / denom;
    }
    void build_sources() {
        sources.clear();
        for (size_t x = 0; x < octaves; ++x) sources.emplace_back((uint32_t)(seed + (uint32_t)x));
    }
    explicit Fbm(uint32_t s) : seed(s) {
        build_sources();
        scale_factor = calc_scale_factor(persistence, octaves);
    }
    Fbm& set_octaves(size_t o) {
        if (o == octaves) return *this;
        octaves = std::clamp<size_t>(o, 1, MAX_OCTAVES);
        build_sources();
        scale_factor = calc_scale_factor(persistence, octaves);
        return *this;
    }
    Fbm& set_frequency(double f) { frequency = f; return *this; }
    Fbm& set_lacunarity(double l) { lacunarity = l; return *this; }
    Fbm& set_persistence(double p) {
        persistence = p;
        scale_factor = calc_scale_factor(persistence, octaves);
        return *this;
    }
    double get(DVec3 point) const {
        point = point * frequency;
        double result = 0.0;
        for (size_t x = 0; x < octaves; ++x) {
            double signal = perlin_3d(sources[x], point);
            signal *= powi(persistence, (int)x);
            result += signal;
            point = point * lacunarity;
        }
        return result * scale_factor;
    }
};
}  // namespace perlin_crate

struct NoiseTex : Texture {  // PerlinRidgedNoise (noise.rs)
    perlin_crate::Fbm perlin;
    NoiseTex(uint32_t seed, size_t octaves, double frequency, double lacunarity, double persistence)
        : perlin(seed) {
        perlin.set_octaves(octaves).set_lacunarity(lacunarity).set_frequency(frequency).set_persistence(persistence);
    }
    DVec3 get_color(DVec2, DVec3 p) const override {
        const double v = std::fabs(perlin.get(p));  // Abs
        return v * DVec3{1.0, 1.0, 1.0};
    }
    std::string desc() const override {
        char b[64];
        snprintf(b, sizeof b, " NOISE %u %zu", perlin.seed, perlin.octaves);
        return b + hx(perlin.frequency) + hx(perlin.lacunarity) + hx(perlin.persistence);
    }
};
struct MarbleTex : Texture {  // Marble (marble.rs)
    perlin_crate::Fbm perlin;
    double frequency;
    MarbleTex(uint32_t seed, double f) : perlin(seed), frequency(f) { perlin.set_octaves(7).set_frequency(f); }
    DVec3 get_color(DVec2, DVec3 p) const override {
        const double n = std::fabs(perlin.get(p));
        const double v = (1. + std::sin(frequency * p.z + 10. * n)) / 2.;
        return v * DVec3{1.0, 1.0, 1.0};
    }
    std::string desc() const override {
        char b[64];
        snprintf(b, sizeof b, " MARBLE %u %zu", perlin.seed, perlin.octaves);
        return b + hx(perlin.frequency) + hx(perlin.lacunarity) + hx(perlin.persistence);
    }
};

// --------------------------------------------------------------- materials
struct HitRecord;
struct Material {
    virtual ~Material() = default;
    virtual bool scatter(const Ray&, const HitRecord&, ChaCha8Rng&, Ray&, DVec3&) const { return false; }
    virtual DVec3 emit(const Ray&, const HitRecord&) const { return {0, 0, 0}; }
    virtual std::string desc() const = 0;
};
using MatP = std::shared_ptr<Material>;

struct HitRecord {
    bool front_face;
    const Material* material;
    DVec3 normal, point;
    double t;
    DVec2 uv;
    static HitRecord make(const Ray& ray, const Material* m, DVec3 point, DVec3 outward, DVec2 uv, double t) {
        const double d = dot(ray.direction, outward);
        const double sign = std::isnan(d) ? d : std::copysign(1.0, d);  // f64::signum
        HitRecord h;
        h.front_face = sign < 0.0;
        h.normal = -sign * outward;
        h.material = m;
        h.point = point;
        h.uv = uv;
        h.t = t;
        return h;
    }
};

struct Lambertian : Material {
    TexP tex;
    bool scatter(const Ray& ray, const HitRecord& hit, ChaCha8Rng& rng, Ray& out, DVec3& att) const override {
        DVec3 dir = hit.normal + random_in_unit_sphere(rng);
        if (almost_zero(dir, 1e-8)) dir = hit.normal;
        out = Ray{hit.point, dir, 0, ray.time};
        att = tex->get_color(hit.uv, hit.point);
        return true;
    }
    std::string desc() const override { return " LAMBERTIAN" + tex->desc(); }
};
struct Metal : Material {
    double fuzz;
    TexP tex;
    bool scatter(const Ray& ray, const HitRecord& hit, ChaCha8Rng& rng, Ray& out, DVec3& att) const override {
        const DVec3 dir = normalize(reflect(ray.direction, hit.normal)) + fuzz * random_in_unit_sphere(rng);
        if (dot(dir, hit.normal) > 0.0) {
            out = Ray{hit.point, dir, 0, ray.time};
            att = tex->get_color(hit.uv, hit.point);
            return true;
        }
        return false;
    }
    std::string desc() const override { return " METAL" + hx(fuzz) + tex->desc(); }
};
static double reflectance(double cosine, double ri) {
    double r0 = (1.0 - ri) / (1.0 + ri);
    r0 = r0 * r0;
    const double x = 1.0 - cosine;
    const double x2 = x * x;
    return r0 + (1.0 - r0) * (x * (x2 * x2));  // powi(5): x * ((x*x)*(x*x))
}
struct Dielectric : Material {
    double ri;
    bool scatter(const Ray& ray, const HitRecord& hit, ChaCha8Rng& rng, Ray& out, DVec3& att) const override {
        const double r = hit.front_face ? 1.0 / ri : ri;
        const DVec3 unit = normalize(ray.direction);
        const double cos_theta = std::fmin(dot(-unit, hit.normal), 1.0);
        const double sin_theta = std::sqrt(1.0 - cos_theta * cos_theta);
        DVec3 dir;
        if (r * sin_theta > 1.0 || reflectance(cos_theta, r) > random_range(rng, 0.0, 1.0))
            dir = reflect(unit, hit.normal);
        else
            dir = refract(unit, hit.normal, r);
        out = Ray{hit.point, dir, 0, ray.time};
        att = {1, 1, 1};
        return true;
    }
    std::string desc() const override { return " DIELECTRIC" + hx(ri); }
};
struct DiffuseLight : Material {
    double intensity;
    TexP tex;
    DVec3 emit(const Ray& ray, const HitRecord& hit) const override {
        const double k = ray.bounce > 0 ? intensity : 1.0;
        return k * tex->get_color(hit.uv, hit.point);
    }
    std::string desc() const override { return " DIFFUSE_LIGHT" + hx(intensity) + tex->desc(); }
};

// ---------------------------------------------------------------- hitables
struct Hitable {
    virtual ~Hitable() = default;
    virtual AABB bbox() const = 0;
    virtual std::optional<HitRecord> hit(const Ray& ray, Interval range) const = 0;
    virtual void dump(std::string& s, int indent) const = 0;
};
using HitP = std::shared_ptr<Hitable>;

static void ind(std::string& s, int n) { s.append((size_t)n * 2, ' '); }

struct Sphere : Hitable {
    DVec3 center, speed{0, 0, 0};
    double radius;
    MatP material;
    AABB box;
    // SphereBuilder::build (sphere.rs:69-92): the box spans the centre at time 0 and 1
    Sphere(DVec3 c, double r, MatP m, DVec3 s = {0, 0, 0}) : center(c), speed(s), radius(r), material(std::move(m)) {
        const DVec3 rvec{radius, radius, radius};
        const DVec3 c1 = center + speed;
        box = AABB::from_points(center - rvec, center + rvec).unite(AABB::from_points(c1 - rvec, c1 + rvec));
    }
    AABB bbox() const override { return box; }
    std::optional<HitRecord> hit(const Ray& ray, Interval range) const override {
        NRT_COUNT(tl.sphere_tests += 1);
        const DVec3 c = center + ray.time * speed;  // Ray::new(center, speed).at(time)
        const DVec3 dir = ray.direction, eye = ray.origin;
        const DVec3 ec = c - eye;
        const double a = length_squared(dir);
        const double h = dot(ec, dir);
        const double cc = length_squared(ec) - radius * radius;
        const double disc = h * h - a * cc;
        if (disc < 0.0) return std::nullopt;
        const double sq = std::sqrt(disc);
        double t = (h - sq) / a;
        if (!range.surrounds(t)) {
            t = (h + sq) / a;
            if (!range.surrounds(t)) return std::nullopt;
        }
        NRT_COUNT(tl.sphere_hits += 1);
        const DVec3 point = ray.at(t);
        const DVec3 normal = normalize(point - c);
        const double theta = std::acos(-normal.y);
        const double phi = std::atan2(-normal.z, normal.x) + M_PI;
        return HitRecord::make(ray, material.get(), point, normal, DVec2{phi / (2.0 * M_PI), theta / M_PI}, t);
    }
    void dump(std::string& s, int n) const override {
        ind(s, n);
        s += "SPHERE" + hx3(center) + hx(radius) + hx3(speed) + hxbox(box) + material->desc() + "\n";
    }
};

struct Plane : Hitable {
    DVec3 p, u, v, normal, w;
    double d;
    bool quad;
    MatP material;
    AABB box;
    Plane(bool q, DVec3 p_, DVec3 u_, DVec3 v_, MatP m) : p(p_), u(u_), v(v_), quad(q), material(std::move(m)) {
        box = AABB::from_points(p, p + u + v).unite(AABB::from_points(p + u, p + v));
        const DVec3 n = cross(u, v);
        normal = normalize(n);
        d = dot(normal, p);
        w = n / dot(n, n);
    }
    AABB bbox() const override { return box; }
    std::optional<HitRecord> hit(const Ray& ray, Interval range) const override {
        NRT_COUNT(tl.plane_tests += 1);
        const double denom = dot(normal, ray.direction);
        if (std::fabs(denom) < 1e-8) return std::nullopt;
        const double t = (d - dot(normal, ray.origin)) / denom;
        if (!range.contains(t)) return std::nullopt;
        const DVec3 point = ray.at(t);
        const DVec3 ph = point - p;
        const double alpha = dot(w, cross(ph, v));
        const double beta = dot(w, cross(u, ph));
        const bool inside = quad ? (0.0 <= alpha && alpha <= 1.0 && 0.0 <= beta && beta <= 1.0)
                                 : (alpha > 0.0 && beta > 0.0 && (alpha + beta) < 1.0);
        if (!inside) return std::nullopt;
        NRT_COUNT(tl.plane_hits += 1);
        return HitRecord::make(ray, material.get(), point, normal, DVec2{alpha, beta}, t);
    }
    void dump(std::string& s, int n) const override {
        ind(s, n);
        s += std::string(quad ? "QUAD" : "TRIANGLE") + hx3(p) + hx3(u) + hx3(v) + hx3(normal) + hx(d) + hx3(w) +
             hxbox(box) + material->desc() + "\n";
    }
};

struct BVH : Hitable {
    enum Kind { LeafNone, LeafSome, Node } kind = LeafNone;
    HitP object;
    std::shared_ptr<BVH> left, right;
    AABB box = AABB::empty();

    static std::shared_ptr<BVH> from(std::vector<HitP>& objects, size_t lo, size_t hi) {
        auto b = std::make_shared<BVH>();
        const size_t n = hi - lo;
        if (n == 0) return b;
        if (n == 1) {
            b->kind = LeafSome;
            b->object = objects[lo];
            return b;
        }
        b->kind = Node;
        if (n == 2) {
            b->left = std::make_shared<BVH>();
            b->left->kind = LeafSome;
            b->left->object = objects[lo];
            b->right = std::make_shared<BVH>();
            b->right->kind = LeafSome;
            b->right->object = objects[lo + 1];
            b->box = objects[lo]->bbox().unite(objects[lo + 1]->bbox());
            return b;
        }
        AABB bbox = AABB::empty();
        for (size_t k = lo; k < hi; ++k) bbox = bbox.unite(objects[k]->bbox());
        const int axis = longest_axis(bbox);
        // slice::sort_by is stable: a merge sort keeps equal keys in order
        std::vector<HitP> tmp(objects.begin() + (long)lo, objects.begin() + (long)hi);
        merge_sort(tmp, axis);
        std::copy(tmp.begin(), tmp.end(), objects.begin() + (long)lo);
        const size_t mid = n / 2;
        b->left = from(objects, lo, lo + mid);
        b->right = from(objects, lo + mid, hi);
        b->box = bbox;
        return b;
    }
    static void merge_sort(std::vector<HitP>& v, int axis) {
        if (v.size() < 2) return;
        std::vector<HitP> a(v.begin(), v.begin() + (long)(v.size() / 2)), b(v.begin() + (long)(v.size() / 2), v.end());
        merge_sort(a, axis);
        merge_sort(b, axis);
        size_t i = 0, j = 0, k = 0;
        while (i < a.size() && j < b.size()) {
            // take from b only when strictly less: stability
            if (total_cmp(b[j]->bbox().axis_interval(axis).min, a[i]->bbox().axis_interval(axis).min) < 0) v[k++] = b[j++];
            else v[k++] = a[i++];
        }
        while (i < a.size()) v[k++] = a[i++];
        while (j < b.size()) v[k++] = b[j++];
    }
    AABB bbox() const override {
        if (kind == Node) return box;
        if (kind == LeafSome) return object->bbox();
        return AABB::empty();
    }
    std::optional<HitRecord> hit(const Ray& ray, Interval range) const override {
        if (kind == LeafSome) return object->hit(ray, range);
        if (kind == Node && aabb_hit(box, ray, range)) {
            auto l = left->hit(ray, range);
            auto r = right->hit(ray, range);
            if (l && !r) return l;
            if (!l && r) return r;
            if (l && r) return l->t < r->t ? l : r;
            return std::nullopt;
        }
        return std::nullopt;
    }
    void dump(std::string& s, int n) const override {
        ind(s, n);
        if (kind == LeafNone) { s += "BVH_EMPTY\n"; return; }
        if (kind == LeafSome) { s += "BVH_LEAF\n"; object->dump(s, n + 1); return; }
        s += "BVH_NODE" + hxbox(box) + "\n";
        left->dump(s, n + 1);
        right->dump(s, n + 1);
    }
};

struct Translate : Hitable {
    HitP object;
    DVec3 offset;
    AABB box;
    Translate(HitP o, DVec3 off) : object(std::move(o)), offset(off) {
        box = object->bbox();
        box.x.min += offset.x; box.x.max += offset.x;
        box.y.min += offset.y; box.y.max += offset.y;
        box.z.min += offset.z; box.z.max += offset.z;
    }
    AABB bbox() const override { return box; }
    std::optional<HitRecord> hit(const Ray& ray, Interval range) const override {
        NRT_COUNT(tl.transform_enters += 1);
        const Ray r{ray.origin - offset, ray.direction, ray.bounce, ray.time};
        auto h = object->hit(r, range);
        if (h) h->point = h->point + offset;
        return h;
    }
    void dump(std::string& s, int n) const override {
        ind(s, n);
        s += "TRANSLATE" + hx3(offset) + hxbox(box) + "\n";
        object->dump(s, n + 1);
    }
};

template <class F>
static AABB corner_box(const AABB& bb, F&& f) {
    DVec3 mn{INF, INF, INF}, mx{-INF, -INF, -INF};
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                const double x = (double)i * bb.x.max + (1.0 - (double)i) * bb.x.min;
                const double y = (double)j * bb.y.max + (1.0 - (double)j) * bb.y.min;
                const double z = (double)k * bb.z.max + (1.0 - (double)k) * bb.z.min;
                const DVec3 t = f(DVec3{x, y, z});
                mn = vmin(mn, t);
                mx = vmax(mx, t);
            }
    return AABB::from_points(mn, mx);
}

struct Rotate : Hitable {
    HitP object;
    DMat3 m, minv;
    AABB box;
    Rotate(HitP o, DVec3 axis, double angle) : object(std::move(o)) {
        m = DMat3::from_axis_angle(axis, -angle);
        minv = DMat3::from_axis_angle(axis, angle);
        box = corner_box(object->bbox(), [&](DVec3 p) { return minv * p; });
    }
    AABB bbox() const override { return box; }
    std::optional<HitRecord> hit(const Ray& ray, Interval range) const override {
        NRT_COUNT(tl.transform_enters += 1);
        const Ray r{m * ray.origin, m * ray.direction, ray.bounce, ray.time};
        auto h = object->hit(r, range);
        if (h) {
            h->point = minv * h->point;
            h->normal = minv * h->normal;
        }
        return h;
    }
    void dump(std::string& s, int n) const override {
        ind(s, n);
        s += "ROTATE" + hx3(m.x_axis) + hx3(m.y_axis) + hx3(m.z_axis) + hx3(minv.x_axis) + hx3(minv.y_axis) +
             hx3(minv.z_axis) + hxbox(box) + "\n";
        object->dump(s, n + 1);
    }
};

struct Scale : Hitable {
    HitP object;
    DMat4 m, minv;
    AABB box;
    Scale(HitP o, DVec3 s) : object(std::move(o)) {
        m = DMat4::from_scale(s);
        minv = m.inverse();
        box = corner_box(object->bbox(), [&](DVec3 p) { return m.transform_point3(p); });
    }
    AABB bbox() const override { return box; }
    std::optional<HitRecord> hit(const Ray& ray, Interval range) const override {
        NRT_COUNT(tl.transform_enters += 1);
        const Ray r{minv.transform_point3(ray.origin), minv.transform_vector3(ray.direction), ray.bounce, ray.time};
        auto h = object->hit(r, range);
        if (h) h->point = m.transform_point3(h->point);
        return h;
    }
    void dump(std::string& s, int n) const override {
        ind(s, n);
        s += "SCALE";
        const DVec4 cols[4] = {minv.x_axis, minv.y_axis, minv.z_axis, minv.w_axis};
        for (auto& c : cols) s += hx(c.x) + hx(c.y) + hx(c.z) + hx(c.w);
        s += hxbox(box) + "\n";
        object->dump(s, n + 1);
    }
};

// ------------------------------------------------------------------ camera
struct Camera {
    uint64_t width = 1200, height = 800;
    DVec3 background{0, 0, 0}, look_from{1, 1, 1};
    uint64_t ray_max_bounces = 10, samples_per_pixel = 10;
    DVec3 defocus_disk_u{}, defocus_disk_v{}, pixel_delta_u{}, pixel_delta_v{}, top_left{};

    // CameraBuilder::build
    static Camera build(uint64_t W, uint64_t H, DVec3 bg, DVec3 look_from, DVec3 look_at, DVec3 view_up,
                        double defocus_angle, double focus_dist, double fov, uint64_t bounces, uint64_t spp) {
        Camera c;
        c.width = W;
        c.height = H;
        c.background = bg;
        c.look_from = look_from;
        c.ray_max_bounces = bounces;
        c.samples_per_pixel = spp < 1 ? 1 : spp;
        if (defocus_angle < 0.) defocus_angle = 0.;
        if (defocus_angle > M_PI) defocus_angle = M_PI;
        const double h = std::tan(fov / 2.);
        const double vh = focus_dist * h * 2.0;
        const double vw = vh * ((double)W / (double)H);
        const DVec3 w = normalize(look_from - look_at);
        const DVec3 u = normalize(cross(view_up, w));
        const DVec3 v = normalize(cross(w, u));
        const DVec3 vu = u * vw;
        const DVec3 vv = -v * vh;
        c.pixel_delta_u = vu / (double)W;
        c.pixel_delta_v = vv / (double)H;
        c.top_left = look_from - w * focus_dist - vu / 2.0 - vv / 2.0 + (c.pixel_delta_u + c.pixel_delta_v) / 2.0;
        const double r = focus_dist * std::tan(defocus_angle / 2.0);
        c.defocus_disk_u = u * r;
        c.defocus_disk_v = v * r;
        return c;
    }

    Ray get_ray(uint32_t x, uint32_t y, ChaCha8Rng& rng) const {
        NRT_COUNT(tl.camera_rays += 1);
        DVec2 off{0, 0};
        if (samples_per_pixel > 1) {
            off.x = random_range(rng, -0.5, 0.5);
            off.y = random_range(rng, -0.5, 0.5);
        }
        const DVec3 point = top_left + ((double)x + off.x) * pixel_delta_u + ((double)y + off.y) * pixel_delta_v;
        const DVec3 p = random_in_unit_disk(rng);
        const DVec3 origin = look_from + p.x * defocus_disk_u + p.y * defocus_disk_v;
        const DVec3 direction = point - origin;
        const double time = random_range(rng, 0.0, 1.0);
        return Ray{origin, direction, 0, time};
    }

    DVec3 get_ray_color(const Ray& ray, uint64_t bounce, const Hitable& world, ChaCha8Rng& rng) const {
        if (bounce >= ray_max_bounces) return {0, 0, 0};
        NRT_COUNT(tl.rays += 1);
        auto hit = world.hit(ray, Interval{0.001, INF});
        if (hit) {
            const Material* m = hit->material;
            const DVec3 emitted = m->emit(ray, *hit);
            Ray scattered;
            DVec3 color;
            if (m->scatter(ray, *hit, rng, scattered, color)) {
                NRT_COUNT(tl.scatter_tries += 1);
                scattered.bounce += 1;
                return emitted + color * get_ray_color(scattered, bounce + 1, world, rng);
            }
            return emitted;
        }
        return background;
    }
};

// ---------------------------------------------------------- tree loading
struct Scene {
    Camera camera;
    HitP root;
};

static std::vector<std::string> split(const std::string& line) {
    std::istringstream is(line);
    std::vector<std::string> t;
    std::string w;
    while (is >> w) t.push_back(w);
    return t;
}
static double F(const std::string& s) { return strtod(s.c_str(), nullptr); }
static DVec3 F3(const std::vector<std::string>& t, size_t i) { return {F(t[i]), F(t[i + 1]), F(t[i + 2])}; }
static uint64_t U(const std::string& s) { return strtoull(s.c_str(), nullptr, 10); }

static Scene load_tree(const std::string& path) {
    std::ifstream f(path);
    if (!f) { fprintf(stderr, "cannot open %s\n", path.c_str()); exit(2); }
    Scene sc;
    std::vector<TexP> tex;
    std::vector<MatP> mat;
    std::vector<HitP> obj;
    std::string line;
    bool have_root = false;
    while (std::getline(f, line)) {
        auto t = split(line);
        if (t.empty() || t[0][0] == '#') continue;
        if (t[0] == "CAMERA") {
            sc.camera = Camera::build(U(t[1]), U(t[2]), F3(t, 5), F3(t, 8), F3(t, 11), F3(t, 14), F(t[17]), F(t[18]),
                                      F(t[19]), U(t[4]), U(t[3]));
        } else if (t[0] == "TEX") {
            const size_t id = U(t[1]);
            TexP p;
            if (t[2] == "SOLID") p = std::make_shared<SolidColor>(F3(t, 3));
            else if (t[2] == "IMAGE") {
                auto im = std::make_shared<ImageTex>();
                im->w = (uint32_t)U(t[3]);
                im->h = (uint32_t)U(t[4]);
                im->px.resize((size_t)im->w * im->h * 3);
                std::ifstream rf(t[5], std::ios::binary);
                rf.read((char*)im->px.data(), (long)(im->px.size() * sizeof(float)));
                if (!rf) { fprintf(stderr, "bad texel file %s\n", t[5].c_str()); exit(2); }
                p = im;
            } else if (t[2] == "CHECKER") {
                auto c = std::make_shared<Checker>();
                c->even = tex.at(U(t[3]));
                c->odd = tex.at(U(t[4]));
                c->scale = F(t[5]);
                p = c;
            } else if (t[2] == "NOISE") {  // seed octaves frequency lacunarity persistence
                p = std::make_shared<NoiseTex>((uint32_t)U(t[3]), (size_t)U(t[4]), F(t[5]), F(t[6]), F(t[7]));
            } else if (t[2] == "MARBLE") {  // seed frequency
                p = std::make_shared<MarbleTex>((uint32_t)U(t[3]), F(t[4]));
            } else { fprintf(stderr, "unsupported texture %s\n", t[2].c_str()); exit(3); }
            if (tex.size() <= id) tex.resize(id + 1);
            tex[id] = p;
        } else if (t[0] == "MAT") {
            const size_t id = U(t[1]);
            MatP p;
            if (t[2] == "LAMBERTIAN") { auto m = std::make_shared<Lambertian>(); m->tex = tex.at(U(t[3])); p = m; }
            else if (t[2] == "METAL") { auto m = std::make_shared<Metal>(); m->fuzz = F(t[3]); m->tex = tex.at(U(t[4])); p = m; }
            else if (t[2] == "DIELECTRIC") { auto m = std::make_shared<Dielectric>(); m->ri = F(t[3]); p = m; }
            else if (t[2] == "DIFFUSE_LIGHT") { auto m = std::make_shared<DiffuseLight>(); m->intensity = F(t[3]); m->tex = tex.at(U(t[4])); p = m; }
            else { fprintf(stderr, "bad material\n"); exit(2); }
            if (mat.size() <= id) mat.resize(id + 1);
            mat[id] = p;
        } else if (t[0] == "OBJ") {
            const size_t id = U(t[1]);
            HitP p;
            const std::string& k = t[2];
            if (k == "SPHERE")  // optional trailing speed (SphereBuilder::with_speed)
                p = std::make_shared<Sphere>(F3(t, 3), F(t[6]), mat.at(U(t[7])), t.size() >= 11 ? F3(t, 8) : DVec3{0, 0, 0});
            else if (k == "QUAD" || k == "TRIANGLE") p = std::make_shared<Plane>(k == "QUAD", F3(t, 3), F3(t, 6), F3(t, 9), mat.at(U(t[12])));
            else if (k == "BVH") {
                std::vector<HitP> list;
                const size_t n = U(t[3]);
                for (size_t i = 0; i < n; ++i) list.push_back(obj.at(U(t[4 + i])));
                p = BVH::from(list, 0, list.size());
            } else if (k == "TRANSLATE") p = std::make_shared<Translate>(obj.at(U(t[3])), F3(t, 4));
            else if (k == "ROTATE") {
                const DVec3 axis = t[3] == "x" ? DVec3{1, 0, 0} : t[3] == "y" ? DVec3{0, 1, 0} : DVec3{0, 0, 1};
                p = std::make_shared<Rotate>(obj.at(U(t[4])), axis, F(t[5]));
            } else if (k == "SCALE") p = std::make_shared<Scale>(obj.at(U(t[3])), F3(t, 4));
            else { fprintf(stderr, "bad object %s\n", k.c_str()); exit(2); }
            if (obj.size() <= id) obj.resize(id + 1);
            obj[id] = p;
        } else if (t[0] == "ROOT") {
            sc.root = obj.at(U(t[1]));
            have_root = true;
        }
    }
    if (!have_root) { fprintf(stderr, "tree has no ROOT\n"); exit(2); }
    return sc;
}

}  // namespace oracle

using namespace oracle;

int main(int argc, char** argv) {
    if (argc < 2) { fprintf(stderr, "usage: oracle render|dump|rng|chacha ...\n"); return 2; }
    const std::string cmd = argv[1];
    if (cmd == "chacha" && argc == 7) {
        const int rounds = atoi(argv[2]);
        uint32_t key[8];
        const std::string hexkey = argv[3];
        for (int i = 0; i < 8; ++i) {
            uint32_t w = 0;
            for (int b = 0; b < 4; ++b) w |= (uint32_t)strtoul(hexkey.substr((size_t)(8 * i + 2 * b), 2).c_str(), nullptr, 16) << (8 * b);
            key[i] = w;
        }
        const uint64_t ctr = strtoull(argv[4], nullptr, 10), nonce = strtoull(argv[5], nullptr, 10);
        const int nwords = atoi(argv[6]);
        for (int b = 0; b * 16 < nwords; ++b) {
            uint32_t out[16];
            chacha_block(rounds, key, ctr + (uint64_t)b, nonce, out);
            for (int i = 0; i < 16 && b * 16 + i < nwords; ++i) printf("%08x\n", out[i]);
        }
        return 0;
    }
    if (cmd == "xorshift" && argc == 4) {  // rand_xorshift: 16 seed bytes (hex), n x next_u32
        uint8_t seed[16];
        for (int i = 0; i < 16; ++i) seed[i] = (uint8_t)strtoul(std::string(argv[2]).substr((size_t)(2 * i), 2).c_str(), nullptr, 16);
        perlin_crate::XorShiftRng r(seed);
        for (int i = 0, n = atoi(argv[3]); i < n; ++i) printf("%u\n", r.next_u32());
        return 0;
    }
    if (cmd == "perm" && argc == 3) {  // noise PermutationTable::new(seed)
        const perlin_crate::PermutationTable t((uint32_t)strtoul(argv[2], nullptr, 10));
        for (int i = 0; i < 256; ++i) printf("%u%c", t.values[i], i == 255 ? '\n' : ' ');
        return 0;
    }
    if ((cmd == "noise" && argc == 10) || (cmd == "marble" && argc == 7)) {  // texture value at a point (%a)
        TexP t;
        int k = 2;
        if (cmd == "noise") {
            t = std::make_shared<NoiseTex>((uint32_t)strtoul(argv[2], nullptr, 10), (size_t)strtoull(argv[3], nullptr, 10),
                                           strtod(argv[4], nullptr), strtod(argv[5], nullptr), strtod(argv[6], nullptr));
            k = 7;
        } else {
            t = std::make_shared<MarbleTex>((uint32_t)strtoul(argv[2], nullptr, 10), strtod(argv[3], nullptr));
            k = 4;
        }
        const DVec3 c = t->get_color({0, 0}, {strtod(argv[k], nullptr), strtod(argv[k + 1], nullptr), strtod(argv[k + 2], nullptr)});
        printf("%a\n", c.x);
        return 0;
    }
    if (cmd == "rng" && argc == 4) {
        ChaCha8Rng r = ChaCha8Rng::seed_from_u64(0);
        r.set_stream(strtoull(argv[2], nullptr, 10));
        const int n = atoi(argv[3]);
        for (int i = 0; i < n; ++i) printf("%016llx\n", (unsigned long long)r.next_u64());
        return 0;
    }
    if (cmd == "dump" && argc == 3) {
        Scene sc = load_tree(argv[2]);
        const Camera& c = sc.camera;
        std::string s = "CAMERA " + std::to_string(c.width) + " " + std::to_string(c.height) + " " +
                        std::to_string(c.samples_per_pixel) + " " + std::to_string(c.ray_max_bounces) +
                        hx3(c.background) + hx3(c.look_from) + hx3(c.defocus_disk_u) + hx3(c.defocus_disk_v) +
                        hx3(c.pixel_delta_u) + hx3(c.pixel_delta_v) + hx3(c.top_left) + "\n";
        sc.root->dump(s, 0);
        fputs(s.c_str(), stdout);
        return 0;
    }
    if (cmd == "render" && argc >= 4) {
        Scene sc = load_tree(argv[2]);
        const std::string out = argv[3];
        unsigned threads = std::thread::hardware_concurrency();
        uint32_t row_off = 0, row_stride = 1;
        std::string stats, var_path;
        for (int i = 4; i < argc; ++i) {
            const std::string a = argv[i];
            if (a == "--threads" && i + 1 < argc) threads = (unsigned)atoi(argv[++i]);
            else if (a == "--rows" && i + 2 < argc) { row_off = (uint32_t)atoi(argv[++i]); row_stride = (uint32_t)atoi(argv[++i]); }
            else if (a == "--spp" && i + 1 < argc) sc.camera.samples_per_pixel = U(argv[++i]);
            else if (a == "--stats" && i + 1 < argc) stats = argv[++i];
            else if (a == "--var" && i + 1 < argc) var_path = argv[++i];
        }
        const bool want_var = !var_path.empty();
        if (threads < 1) threads = 1;
        const Camera& cam = sc.camera;
        const uint32_t W = (uint32_t)cam.width, H = (uint32_t)cam.height;
        std::vector<uint32_t> rows;
        for (uint32_t y = row_off; y < H; y += row_stride) rows.push_back(y);
        const size_t npix = rows.size() * W;
        std::vector<float> img(npix * 3), var(want_var ? npix * 3 : 0);
        std::atomic<size_t> next{0};
        std::vector<Counters> all(threads);
        const auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (unsigned k = 0; k < threads; ++k) {
            th.emplace_back([&, k]() {
                tl = Counters{};
                while (true) {
                    const size_t i = next.fetch_add(1);  // dynamic per-pixel scheduling (rayon analogue)
                    if (i >= npix) break;
                    const uint32_t x = (uint32_t)(i % W), y = rows[i / W];
                    const uint32_t n = y * W + x;
                    ChaCha8Rng rng = ChaCha8Rng::seed_from_u64(0);
                    rng.set_stream(n);
                    DVec3 s{0, 0, 0}, sq{0, 0, 0};
                    for (uint64_t k2 = 0; k2 < cam.samples_per_pixel; ++k2) {
                        const Ray ray = cam.get_ray(x, y, rng);
                        const DVec3 c = cam.get_ray_color(ray, 0, *sc.root, rng);
                        s = s + c;
                        if (want_var) sq = sq + c * c;
                    }
                    if (want_var) {  // unbiased per-sample variance (test statistics only)
                        const double m = (double)cam.samples_per_pixel;
                        const double dd = m > 1 ? m - 1 : 1;
                        var[3 * i + 0] = (float)((sq.x - s.x * s.x / m) / dd);
                        var[3 * i + 1] = (float)((sq.y - s.y * s.y / m) / dd);
                        var[3 * i + 2] = (float)((sq.z - s.z * s.z / m) / dd);
                    }
                    NRT_COUNT(tl.draws += rng.draws);
                    const DVec3 c = s / (double)cam.samples_per_pixel;
                    img[3 * i + 0] = (float)c.x;
                    img[3 * i + 1] = (float)c.y;
                    img[3 * i + 2] = (float)c.z;
                }
                all[k] = tl;
            });
        }
        for (auto& t : th) t.join();
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        FILE* f = fopen(out.c_str(), "wb");
        if (!f) { fprintf(stderr, "cannot write %s\n", out.c_str()); return 2; }
        fwrite(img.data(), sizeof(float), img.size(), f);
        fclose(f);
        if (want_var) {
            FILE* vf = fopen(var_path.c_str(), "wb");
            if (!vf) { fprintf(stderr, "cannot write %s\n", var_path.c_str()); return 2; }
            fwrite(var.data(), sizeof(float), var.size(), vf);
            fclose(vf);
        }
        Counters tot;
        for (auto& c : all) {
            tot.aabb_tests += c.aabb_tests; tot.sphere_tests += c.sphere_tests; tot.sphere_hits += c.sphere_hits;
            tot.plane_tests += c.plane_tests; tot.plane_hits += c.plane_hits; tot.transform_enters += c.transform_enters;
            tot.rays += c.rays; tot.scatter_tries += c.scatter_tries; tot.camera_rays += c.camera_rays;
            tot.draws += c.draws; tot.texel_fetches += c.texel_fetches;
        }
        const double samples = (double)npix * (double)cam.samples_per_pixel;
        char buf[1024];
        snprintf(buf, sizeof buf,
                 "{\"seconds\": %.6f, \"threads\": %u, \"pixels\": %zu, \"samples\": %.0f, \"msamples_per_s\": %.6f, "
                 "\"aabb_tests\": %llu, \"sphere_tests\": %llu, \"sphere_hits\": %llu, \"plane_tests\": %llu, "
                 "\"plane_hits\": %llu, \"transform_enters\": %llu, \"rays\": %llu, \"scatters\": %llu, "
                 "\"camera_rays\": %llu, \"draws\": %llu, \"texel_fetches\": %llu}\n",
                 secs, threads, npix, samples, samples / secs / 1e6, (unsigned long long)tot.aabb_tests,
                 (unsigned long long)tot.sphere_tests, (unsigned long long)tot.sphere_hits,
                 (unsigned long long)tot.plane_tests, (unsigned long long)tot.plane_hits,
                 (unsigned long long)tot.transform_enters, (unsigned long long)tot.rays,
                 (unsigned long long)tot.scatter_tries, (unsigned long long)tot.camera_rays,
                 (unsigned long long)tot.draws, (unsigned long long)tot.texel_fetches);
        if (!stats.empty()) {
            FILE* sf = fopen(stats.c_str(), "w");
            if (sf) { fputs(buf, sf); fclose(sf); }
        }
        fputs(buf, stderr);
        return 0;
    }
    fprintf(stderr, "bad arguments\n");
    return 2;
}
