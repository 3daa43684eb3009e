// Perlin textures: `PerlinRidgedNoise` (lib/textures/noise.rs:79-145) and `Marble`
// (lib/textures/marble.rs:46-96), both `Abs<Fbm<Perlin>>` from the `noise` crate.
//
// The reference takes the arithmetic from third-party crates absent from
// /root/reference (Cargo.lock pins noise 0.9.0, its rand 0.8.5 and rand_xorshift
// 0.3.0); what follows restates their published algorithms:
//   * PermutationTable::new(seed): XorShiftRng::from_seed(16 bytes: 1, 0, 0, 0,
//     then the seed's 4 LE bytes three times), then a Fisher-Yates shuffle of
//     0..=255 (rand 0.8 SliceRandom::shuffle: for i in (1..256).rev() swap(i,
//     gen_range(0..i+1)); gen_range u32 = widening-multiply rejection with
//     zone = (range << lz(range)) - 1);
//   * Fbm::new(seed): octave k uses Perlin::new(seed + k); defaults octaves 6,
//     frequency 1, lacunarity 2π/3, persistence 0.5; set_octaves clamps to
//     [1, 32]; scale = 1 / Σ_{k=1..octaves} persistence^k (powi);
//   * Fbm::get: p *= frequency; Σ_k perlin_k(p)·persistence^k with p *= lacunarity
//     after each octave; times scale;
//   * perlin_3d: hash = P[P[P[x&255]^(y&255)]^(z&255)], the 16-case gradient
//     switch, quintic fade, the k0..k7 trilinear polynomial, × 2/√3, clamped to
//     [-1, 1].
// No reference test pins any of it: parity with the reference is unpinned; the
// oracle (oracle/oracle.cpp) restates the same algorithms independently.
#pragma once

#include <cstdint>
#include <vector>

namespace nrt {

constexpr double NOISE_DEFAULT_FREQUENCY = 1.0;
constexpr double NOISE_DEFAULT_LACUNARITY = 3.14159265358979311600 * 2.0 / 3.0;  // core::f64::consts::PI * 2 / 3
constexpr double NOISE_DEFAULT_PERSISTENCE = 0.5;
constexpr uint32_t NOISE_MAX_OCTAVES = 32;
constexpr uint32_t MARBLE_OCTAVES = 7;  // marble.rs:53

// Fbm<Perlin> parameters after the builder (noise.rs:79-101 / marble.rs:46-60).
struct FbmParams {
    uint32_t seed = 0;
    uint32_t octaves = 1;
    double frequency = NOISE_DEFAULT_FREQUENCY;
    double lacunarity = NOISE_DEFAULT_LACUNARITY;
    double persistence = NOISE_DEFAULT_PERSISTENCE;
};

// Fbm::set_octaves: clamped to [1, NOISE_MAX_OCTAVES]
inline uint32_t fbm_octaves(uint64_t octaves) {
    return (uint32_t)(octaves < 1 ? 1 : (octaves > NOISE_MAX_OCTAVES ? NOISE_MAX_OCTAVES : octaves));
}
// f64::powi as LLVM lowers it (compiler-rt __powidf2: square-and-multiply).
double powi_rt(double a, int b);
// Fbm::calc_scale_factor
double fbm_scale_factor(double persistence, uint32_t octaves);
// The 256-entry permutation table of Perlin::new(seed).
void perlin_permutation(uint32_t seed, uint8_t out[256]);

}  // namespace nrt
