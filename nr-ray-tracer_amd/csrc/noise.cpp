// Host side of the Perlin textures: permutation tables and Fbm scale (noise.hpp).
#include "noise.hpp"

namespace nrt {

double powi_rt(double a, int b) {
    const bool recip = b < 0;
    double r = 1.0;
    while (true) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1.0 / r : r;
}

double fbm_scale_factor(double persistence, uint32_t octaves) {
    double denom = 0.0;  // (1..=octaves).fold(0.0, |acc, x| acc + persistence.powi(x))
    for (uint32_t x = 1; x <= octaves; ++x) denom = denom + powi_rt(persistence, (int)x);
    return 1.0 / denom;
}

namespace {

// rand_xorshift 0.3.0 XorShiftRng
struct XorShift128 {
    uint32_t x, y, z, w;
    uint32_t next_u32() {
        const uint32_t t = x ^ (x << 11);
        x = y;
        y = z;
        z = w;
        w = w ^ (w >> 19) ^ (t ^ (t >> 8));
        return w;
    }
};

// rand 0.8.5 UniformInt<u32>::sample_single(0, range)
uint32_t gen_below(XorShift128& rng, uint32_t range) {
    const uint32_t zone = (range << __builtin_clz(range)) - 1u;
    while (true) {
        const uint64_t m = (uint64_t)rng.next_u32() * range;
        if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
    }
}

}  // namespace

void perlin_permutation(uint32_t seed, uint8_t out[256]) {
    // seed bytes [1, 0, 0, 0, s, s, s] (little-endian words): x = 1, y = z = w = seed;
    // never all zero, so the crate's 0xBAD5EED substitute never applies
    XorShift128 rng{1u, seed, seed, seed};
    for (uint32_t i = 0; i < 256; ++i) out[i] = (uint8_t)i;
    for (uint32_t i = 255; i >= 1; --i) {
        const uint32_t j = gen_below(rng, i + 1);
        const uint8_t t = out[i];
        out[i] = out[j];
        out[j] = t;
    }
}

}  // namespace nrt
