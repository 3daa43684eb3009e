// MI355X (gfx950) megakernel for the reference's per-pixel path-tracing loop
// (Camera::render, packages/ray-tracer-lib/src/camera.rs:302-343).
//
// One thread per pixel; each thread runs the pixel's samples in order over the
// pixel's own RNG stream (camera.rs:318-329), an iterative bounce loop in
// place of the recursive get_ray_color (camera.rs:269-300), and a stackless
// traversal of the flattened, threaded BVH (device_scene.hpp) with t-narrowing.
//
// Template axes:
//   Real  = double : the reference-exact variant (same operation order as
//                    glam/rand, divisions kept, compiled with -ffp-contract=off)
//   Real  = float  : the fast variant (reciprocal slab test, f32 RNG floats)
//   RNG   = ChaCha8 per-pixel stream (rand_chacha 0.9, bit-exact with the
//           reference) or Philox4x32-10 keyed per (pixel, sample, draw)
//   MAXD  = 1 when instances do not nest (all BASELINE scenes), 4 otherwise;
//           0 = world-space mode (fast kernel only): instances flattened away
//           on the host, every lane tests every primitive (small scenes).
#pragma once

#ifndef __HIPCC_RTC__  // (hiprtc: the runtime and <cstdint> types are built in, jit.hip)
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#endif

#include "device_scene.hpp"
#include "render_params.hpp"

namespace nrt {
namespace dev {

#ifndef NRT_BLOCK
#define NRT_BLOCK 256  // threads per workgroup (a multiple of 64)
#endif
constexpr int BLOCK = NRT_BLOCK;
#ifndef NRT_SPECULATIVE
#define NRT_SPECULATIVE 1  // world-BVH rounds: lanes holding a leaf keep descending (Aila & Laine)
#endif
#ifndef NRT_WBVH_SORT
#define NRT_WBVH_SORT 0  // 4-wide visits: 1 = full sorting network; 0 = nearest hit child first, the rest in slot order (C4 +4 %)
#endif
#ifndef NRT_WBVH_UNIFIED
#define NRT_WBVH_UNIFIED 1  // if-if trips: a visit and a primitive test in the same trip (C4 40.2 -> 34.6 ms)
#endif
#ifndef NRT_EXACT_SETPRIO
#define NRT_EXACT_SETPRIO 3  // persistent-lane loop: wave priority of the shading step, 0 at the loop head
                             // (0: never changed): earth f64 5.94 -> 5.79 ms, C5 f64 -0.3 %, C4 f64 +-0.5 %
#endif
#ifndef NRT_SETPRIO
#define NRT_SETPRIO 3  // Philox loop: wave priority of the shading step, back to 0 at the loop head (0: never
                       // changed); a wave that has traced finishes its step first (C5 10.36 -> 10.28 ms,
                       // C4 33.50 -> 33.18, C2 0.927 -> 0.920, C3 +-0.2 %; frames identical)
#endif
#ifndef NRT_SETPRIO_TEX
#define NRT_SETPRIO_TEX 0  // ... in the textured world lists (KF_TEXPAL, the earth) at 7 waves: 0 (never
                           // changed) measured C3 5.063 -> 5.024 ms; 1: 5.061 (two alternating runs)
#endif
#ifndef NRT_WBVH_IFIF
// world BVH: one node visit or one primitive per lane and trip (wbvh_trip) in the KF_FLAT
// variant (triangles / quads only: a primitive costs a fifth of a visit; C4 6 307 -> 6 400
// Msamples/s); scenes with f64 sphere tests kept the speculative rounds (C1 -27 % if-if, round 2);
// with the f32 sphere test the sphere / texture variant takes the trips too (NRT_WBVH_IFIF_SPHERES:
// spheres 1080p 31.1 -> 30.7 ms, round 3)
#define NRT_WBVH_IFIF 1
#endif
#ifndef NRT_WBVH_IFIF_SPHERES
#define NRT_WBVH_IFIF_SPHERES 1
#endif
#ifndef NRT_SPHERE_REPROJ
#define NRT_SPHERE_REPROJ 1  // f32-tested spheres: hit points put back on the surface (make_record_world)
#endif
#ifndef NRT_WL_RELOAD
#define NRT_WL_RELOAD 0  // world list: the unit records' scalar loads per query (not hoisted out of the loop)
#endif
#ifndef NRT_CAM_RELOAD
#define NRT_CAM_RELOAD 0  // f32 camera vectors: scalar loads from the kernel arguments at the use
#endif
#ifndef XWALK_WAIT
#define XWALK_WAIT 40  // persistent exact walk: lanes done walking before a shading round (host default: launch_impl.hpp)
#endif
#ifndef NRT_REC_CARRY
#define NRT_REC_CARRY 1  // the exact hit record reuses the winner's plane-test values (HitMin::pre)
#endif
#ifndef NRT_RIUS_WAVE
#define NRT_RIUS_WAVE 1  // ChaCha8 rejection samplers as wave-converged loops (rejection_wave; see render_kernel)
#endif
#ifndef NRT_WALK_CONTRACT
#define NRT_WALK_CONTRACT 1  // FMA contraction in the exact kernel's f32 culling walk and prefilter
#endif
#ifndef NRT_PK_LIST
#define NRT_PK_LIST 0  // boxes turned about y: (d, o) pairs as packed f32 ops; 0: the same expressions per
                       // component (the same roundings, frames identical): C5 9.310 -> 9.235 ms
#endif
#ifndef NRT_PK_QUAD
#define NRT_PK_QUAD 1  // ... quads (axis and general), triangles and boxes: packed (quads.toml, five axis quads,
                       // 1024^2 spp 64: 0.760 ms packed, 0.827 unpacked)
#endif
#ifndef NRT_BOX_DEFER
// world list: 1 = a box unit's (PRIM_BOX / PRIM_BOXY) face is resolved once, for the winner of the whole
// run loop, instead of per unit and ray (the unit keeps (t, its index, entry / exit)).  Measured on C5
// (round 6, 3 alternating runs, frames identical): 9.81-9.82 ms per frame with the face per unit, 10.69-
// 10.71 ms deferred (-9 %): the winner's record comes by per-lane vector loads in a divergent branch
// after the loop, where the per-unit selects ride on scalar-loaded records; off
#define NRT_BOX_DEFER 0
#endif
#ifndef NRT_CHACHA_TOPUP
#define NRT_CHACHA_TOPUP 1  // ChaCha8 ring refilled at the persistent loop's head (ChaCha8::top_up)
#endif
constexpr int RING = 16;  // ChaCha8 ring: 2 blocks of 8 u64 draws per lane, in LDS
// ChaCha8 (persistent-lane) kernels' dynamic LDS before the stack and the staged scene: the ring,
// then each lane's f64 pixel sums (kept in LDS, not registers: the earth scene's exact kernel spilled
// them to scratch at every pixel)
constexpr uint32_t CHACHA_LDS_BYTES = RING * BLOCK * 8u + 3u * BLOCK * 8u;
// Persistent lanes with pixel claims of 2..8 (spp <= 64, render.hip): each wave stages the finished
// pixels of up to STG_SLOTS claims in LDS (3 floats per pixel, then per claim its pixels left, first
// pixel and size) and writes a claim out as one coalesced run once its last pixel is done, instead of
// 12 scattered bytes per pixel (each costing a partial-line write-back: earth f64 66 -> 59 MB).
constexpr uint32_t STG_SLOTS = 8, STG_PX = 8, NO_STG = 0xFFFFFFFFu;
constexpr uint32_t STG_WAVE_WORDS = STG_SLOTS * (STG_PX * 3u + 3u);
constexpr uint32_t STG_LDS_BYTES = (BLOCK / 64u) * STG_WAVE_WORDS * 4u;
__host__ __device__ inline uint32_t chacha_lds_bytes(uint32_t exact_stage) {
    return CHACHA_LDS_BYTES + (exact_stage ? STG_LDS_BYTES : 0u);
}

template <typename R>
struct V {
    R x, y, z;
};
template <typename R> __device__ __forceinline__ V<R> mk(R x, R y, R z) { return V<R>{x, y, z}; }
template <typename R> __device__ __forceinline__ V<R> operator+(V<R> a, V<R> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <typename R> __device__ __forceinline__ V<R> operator-(V<R> a, V<R> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <typename R> __device__ __forceinline__ V<R> operator-(V<R> a) { return {-a.x, -a.y, -a.z}; }
template <typename R> __device__ __forceinline__ V<R> operator*(R s, V<R> a) { return {s * a.x, s * a.y, s * a.z}; }
template <typename R> __device__ __forceinline__ V<R> operator*(V<R> a, V<R> b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
template <typename R> __device__ __forceinline__ V<R> operator/(V<R> a, R s) { return {a.x / s, a.y / s, a.z / s}; }
template <typename R> __device__ __forceinline__ R dot(V<R> a, V<R> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename R> __device__ __forceinline__ V<R> cross(V<R> a, V<R> b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
// Exact (f64) vs fast (f32) arithmetic helpers: the f32 kernel uses the
// hardware reciprocal / reciprocal-sqrt (1 ulp), the f64 kernel IEEE division.
template <typename R> __device__ __forceinline__ R fast_rcp(R x) { return R(1) / x; }
template <> __device__ __forceinline__ float fast_rcp<float>(float x) { return __builtin_amdgcn_rcpf(x); }
template <typename R> __device__ __forceinline__ R fast_sqrt(R x) { return sqrt(x); }
template <> __device__ __forceinline__ float fast_sqrt<float>(float x) { return __builtin_amdgcn_sqrtf(x); }
template <typename R> __device__ __forceinline__ R fast_div(R a, R b) { return a / b; }
template <> __device__ __forceinline__ float fast_div<float>(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
template <typename R> __device__ __forceinline__ V<R> vdiv(V<R> a, R s) { return a / s; }
template <> __device__ __forceinline__ V<float> vdiv<float>(V<float> a, float s) { return fast_rcp(s) * a; }
template <typename R> __device__ __forceinline__ V<R> normalize(V<R> a) {
    return (R(1) / sqrt(dot(a, a))) * a;  // glam: self * self.length().recip()
}
template <> __device__ __forceinline__ V<float> normalize<float>(V<float> a) {
    return __builtin_amdgcn_rsqf(dot(a, a)) * a;
}
// a * b + c, fused (one rounding) in f32.  The fast kernels are compiled with -ffp-contract=on
// (Makefile FAST_CONTRACT, the same for kernels_fast.o and the hiprtc build, jit.hip): only
// `a * b + c` written as one expression fuses, so the generic and the scene-specialised
// kernels round alike whatever the inliner and unroller make of the code around it (with
// -ffp-contract=fast the backend fuses across statements depending on code shape, and the two
// kernels parted on 3 of 1 048 576 C5 pixels).  The products the vector helpers below hand to
// a sum are fused here explicitly.  f64: unfused in the exact TU (-ffp-contract=off).
template <typename R> __device__ __forceinline__ R fmad(R a, R b, R c) { return a * b + c; }
template <> __device__ __forceinline__ float fmad<float>(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
template <typename R> __device__ __forceinline__ V<R> vfma(R s, V<R> a, V<R> b) {  // s * a + b
    return {fmad(s, a.x, b.x), fmad(s, a.y, b.y), fmad(s, a.z, b.z)};
}
template <typename R> __device__ __forceinline__ V<R> ld3(const R* p) { return {p[0], p[1], p[2]}; }
template <typename R> __device__ __forceinline__ V<R> ld3d(const double* p) { return {(R)p[0], (R)p[1], (R)p[2]}; }

// glam DMat3 * v = (c0*x + c1*y) + c2*z, column major m[3c+r]
template <typename R> __device__ __forceinline__ V<R> mat3(const R* m, V<R> v) {
    V<R> c0 = ld3(m), c1 = ld3(m + 3), c2 = ld3(m + 6);
    return (v.x * c0 + v.y * c1) + v.z * c2;
}
// glam DMat4::transform_point3 / transform_vector3 on a 3x4 column-major block
template <typename R> __device__ __forceinline__ V<R> xf_point(const R* m, V<R> v) {
    V<R> r;
    R* o = &r.x;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        R res = m[k] * v.x;
        res = m[3 + k] * v.y + res;
        res = m[6 + k] * v.z + res;
        res = m[9 + k] + res;
        o[k] = res;
    }
    return r;
}
template <typename R> __device__ __forceinline__ V<R> xf_vector(const R* m, V<R> v) {
    V<R> r;
    R* o = &r.x;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        R res = m[k] * v.x;
        res = m[3 + k] * v.y + res;
        res = m[6 + k] * v.z + res;
        o[k] = res;
    }
    return r;
}

// f64::signum: 1 for +0/positive, -1 for -0/negative, NaN for NaN
template <typename R> __device__ __forceinline__ R signum(R x) { return x != x ? x : copysign(R(1), x); }

// ----------------------------------------------------------------------- RNG
// rand_chacha 0.9 ChaCha8Rng::seed_from_u64(0): key = PCG32 expansion of 0.
__constant__ const uint32_t CHACHA_KEY[8] = {0xf973f2ecu, 0x45cdb581u, 0x7346f087u, 0xad6cad06u,
                                              0xe3a3d0d0u, 0x67e71733u, 0x72ea9bf2u, 0xfe7d8ad7u};

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define NRT_QR(a, b, c, d)              \
    a += b; d ^= a; d = rotl32(d, 16);  \
    c += d; b ^= c; b = rotl32(b, 12);  \
    a += b; d ^= a; d = rotl32(d, 8);   \
    c += d; b ^= c; b = rotl32(b, 7);

// One ChaCha8 block (state words 12-13 = 64-bit block counter, 14-15 = stream).
__device__ __forceinline__ void chacha8_block(uint32_t ctr_lo, uint32_t ctr_hi, uint32_t s_lo, uint32_t s_hi,
                                              uint32_t out[16]) {
    const uint32_t i0 = 0x61707865u, i1 = 0x3320646eu, i2 = 0x79622d32u, i3 = 0x6b206574u;
    uint32_t x0 = i0, x1 = i1, x2 = i2, x3 = i3;
    uint32_t x4 = CHACHA_KEY[0], x5 = CHACHA_KEY[1], x6 = CHACHA_KEY[2], x7 = CHACHA_KEY[3];
    uint32_t x8 = CHACHA_KEY[4], x9 = CHACHA_KEY[5], x10 = CHACHA_KEY[6], x11 = CHACHA_KEY[7];
    uint32_t x12 = ctr_lo, x13 = ctr_hi, x14 = s_lo, x15 = s_hi;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        NRT_QR(x0, x4, x8, x12) NRT_QR(x1, x5, x9, x13) NRT_QR(x2, x6, x10, x14) NRT_QR(x3, x7, x11, x15)
        NRT_QR(x0, x5, x10, x15) NRT_QR(x1, x6, x11, x12) NRT_QR(x2, x7, x8, x13) NRT_QR(x3, x4, x9, x14)
    }
    out[0] = x0 + i0; out[1] = x1 + i1; out[2] = x2 + i2; out[3] = x3 + i3;
    out[4] = x4 + CHACHA_KEY[0]; out[5] = x5 + CHACHA_KEY[1]; out[6] = x6 + CHACHA_KEY[2]; out[7] = x7 + CHACHA_KEY[3];
    out[8] = x8 + CHACHA_KEY[4]; out[9] = x9 + CHACHA_KEY[5]; out[10] = x10 + CHACHA_KEY[6]; out[11] = x11 + CHACHA_KEY[7];
    out[12] = x12 + ctr_lo; out[13] = x13 + ctr_hi; out[14] = x14 + s_lo; out[15] = x15 + s_hi;
}

// Per-pixel ChaCha8 stream = ChaCha8Rng::seed_from_u64(0) + set_stream(n)
// (camera.rs:318-320); every draw is a next_u64 (two consecutive keystream
// words).  Keystream words wait in an LDS ring of 16 u64 slots per lane.
// Refills are batched per wave: when any active lane is empty, every active
// lane with room for a block generates one, so a wave computes about one
// block per 8-9 draw steps even when lanes have drifted apart.
// The stream is the pixel index, below 2^32 (make_params caps images below 2^32 pixels; the probe
// checks its range), so the stream's high word is the constant 0 and two of the first column
// round's quarter rounds fold to constants (6 % of a block's operations).
struct ChaCha8 {
    static constexpr bool uses_lds = true;
    static constexpr bool exact_stream = true;  // draws must follow the reference's sequence
    uint32_t s_lo, ctr, head, count;
    uint2* ring;  // slot k of this lane at ring[k * BLOCK]

    __device__ __forceinline__ void init(uint64_t stream, uint2* base) {
        s_lo = (uint32_t)stream;
        ctr = 0;
        head = 0;
        count = 0;
        ring = base;
    }
    __device__ __forceinline__ void start_sample(uint32_t) {}
    __device__ __forceinline__ void refill() {
        uint32_t w[16];
        chacha8_block(ctr, 0u, s_lo, 0u, w);
        ++ctr;
        uint32_t slot = (head + count) & (RING - 1);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            ring[slot * BLOCK] = make_uint2(w[2 * k], w[2 * k + 1]);
            slot = (slot + 1) & (RING - 1);
        }
        count += 8;
    }
    // At least k (<= 8) words in every active lane's ring: one ballot (and at most one
    // refill site) for a sampler's k draws instead of one per draw.  Same words, same order.
    __device__ __forceinline__ void ensure(uint32_t k) {
        if (__ballot(count < k) != 0ull) {
            if (count <= RING - 8) refill();
        }
    }
    __device__ __forceinline__ uint64_t take() {  // the next word; ensure() made it present
        const uint2 v = ring[head * BLOCK];
        head = (head + 1) & (RING - 1);
        --count;
        return (uint64_t)v.x | ((uint64_t)v.y << 32);
    }
    __device__ __forceinline__ uint64_t next() {
        ensure(1);
        return take();
    }
    // At a point the whole wave reaches (the persistent loop's head): every lane with room for a
    // block generates one, together, so the samplers' own refills (inside divergent code: a
    // rejection loop runs with only its still-trying lanes) become rare.  Refill timing never
    // changes the words or their order.
    __device__ __forceinline__ void top_up() {
        if (count <= RING - 8) refill();
    }
};
// Philox and other counter-based generators: nothing to top up
template <class G>
__device__ __forceinline__ void rng_top_up(G& g) {
    if constexpr (G::uses_lds) g.top_up();
}

// Philox4x32-10 (Salmon et al. 2011), counter = (pixel, sample, pair, 0), key = (0, 0).
// Rounds 1-9 mix the round key into one word with one v_bitop3_b32 (hi ^ c ^ key):
// VOP3 takes no literal on gfx950, so the round keys live in two SGPRs stepped by
// the scalar unit (volatile: the compiler neither folds them into per-round literals,
// which would cost a second v_xor_b32 per word, nor hoists ten keys into SGPRs).
#ifndef NRT_PHILOX_SKEY
#ifdef __HIP_DEVICE_COMPILE__  // (the host pass of the TU has no SGPR / VGPR constraints)
#define NRT_PHILOX_SKEY 1
#else
#define NRT_PHILOX_SKEY 0
#endif
#endif
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t out[4]) {
#if NRT_PHILOX_SKEY
    uint32_t k0, k1;
    asm volatile("s_mov_b32 %0, 0x9e3779b9" : "=s"(k0));
    asm volatile("s_mov_b32 %0, 0xbb67ae85" : "=s"(k1));
#else
    uint32_t k0 = 0u, k1 = 0u;
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        // one widening multiply each (v_mad_u64_u32) instead of separate lo / hi multiplies
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t lo0 = (uint32_t)p0, hi0 = (uint32_t)(p0 >> 32);
        const uint32_t lo1 = (uint32_t)p1, hi1 = (uint32_t)(p1 >> 32);
        uint32_t n0, n2;
#if NRT_PHILOX_SKEY
        if (r == 0) {  // key (0, 0)
            n0 = hi1 ^ c1;
            n2 = hi0 ^ c3;
        } else {
            if (r > 1) {
                asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(k0) : : "scc");
                asm volatile("s_add_u32 %0, %0, 0xbb67ae85" : "+s"(k1) : : "scc");
            }
            // bitop3 table 0x96 = a ^ b ^ c (the compiler does not form it on its own)
            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n0) : "v"(hi1), "v"(c1), "s"(k0));
            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n2) : "v"(hi0), "v"(c3), "s"(k1));
        }
#else
        if (r > 0) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        n0 = hi1 ^ c1 ^ k0;
        n2 = hi0 ^ c3 ^ k1;
#endif
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

// Philox2x32-10 (Random123), key 0: one widening multiply and one three-way xor per
// round, half the work of 4x32.  The f32 render loop needs at most three draws per
// path segment, which 64 bits cover (Philox::block_at).
__device__ __forceinline__ uint2 philox2x32_10(uint32_t c0, uint32_t c1) {
#if NRT_PHILOX_SKEY
    uint32_t k;
    asm volatile("s_mov_b32 %0, 0x9e3779b9" : "=s"(k));
#else
    uint32_t k = 0u;
#endif
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p = (uint64_t)0xD256D193u * c0;
        const uint32_t lo = (uint32_t)p, hi = (uint32_t)(p >> 32);
        uint32_t n;
#if NRT_PHILOX_SKEY
        if (r == 0) {  // key 0
            n = hi ^ c1;
        } else {
            if (r > 1) asm volatile("s_add_u32 %0, %0, 0x9e3779b9" : "+s"(k) : : "scc");
            asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(n) : "v"(hi), "v"(c1), "s"(k));
        }
#else
        if (r > 0) k += 0x9E3779B9u;
        n = hi ^ c1 ^ k;
#endif
        c0 = n;
        c1 = lo;
    }
    return make_uint2(c0, c1);
}

struct Philox {
    static constexpr bool uses_lds = false;
    static constexpr bool exact_stream = false;  // only the distributions matter
    uint32_t pix, sample, pair;
    uint32_t w0, w1, w2, w3;  // unread words of the current block, consumed in order
    uint32_t left;
    __device__ __forceinline__ void init(uint64_t stream, uint2*) {
        pix = (uint32_t)stream;
        sample = 0;
        pair = 0;
        left = 0;
    }
    __device__ __forceinline__ void start_sample(uint32_t s) {
        sample = s;
        pair = 0;
        left = 0;
    }
    __device__ __forceinline__ uint32_t next32() {
        if (left == 0) {
            uint32_t w[4];
            philox4x32_10(pix, sample, pair, 0u, w);
            ++pair;
            w0 = w[0]; w1 = w[1]; w2 = w[2]; w3 = w[3];
            left = 4;
        }
        const uint32_t r = w0;
        w0 = w1; w1 = w2; w2 = w3;
        --left;
        return r;
    }
    __device__ __forceinline__ uint64_t next() {
        const uint32_t lo = next32();
        return (uint64_t)lo | ((uint64_t)next32() << 32);
    }
    __device__ __forceinline__ void ensure(uint32_t) {}
    __device__ __forceinline__ uint64_t take() { return next(); }
    // Render loop: one whole block per lane per iteration, keyed by (pixel, sample,
    // step): step 0 = camera ray, b + 1 = scatter at bounce b, defocus_step() = the
    // camera's second block when the defocus disk is on.  The draws are w.x, w.y, w.z.
    //   f64: Philox4x32-10, counter (pixel, sample, step, 0); 32-bit draws.
    //   f32: Philox2x32-10, counter (pixel, sample | step << 24) (host: spp <= 2^24,
    //        bounces <= 254); w.x = lo and w.y = hi (u01 reads their top 23 bits),
    //        w.z = their low 9 bits each (18-bit draw): disjoint bits of one block.
    template <typename R>
    static __device__ __forceinline__ uint4 block_at(uint32_t pixel, uint32_t smp, uint32_t step) {
        if constexpr (sizeof(R) == 4) {
            const uint2 v = philox2x32_10(pixel, smp | (step << 24));
            return make_uint4(v.x, v.y, (v.x << 23) | ((v.y & 0x1FFu) << 14), 0u);
        } else {
            uint32_t w[4];
            philox4x32_10(pixel, smp, step, 0u, w);
            return make_uint4(w[0], w[1], w[2], w[3]);
        }
    }
    template <typename R>
    static constexpr uint32_t defocus_step() { return sizeof(R) == 4 ? PHILOX2_STEPS - 1u : 0xFFFFFFFFu; }
};

// 32-bit word -> uniform [0, 1) (f32: 23 bits, f64: 32 bits)
template <typename R> __device__ __forceinline__ R u01(uint32_t w);
template <> __device__ __forceinline__ float u01<float>(uint32_t w) { return __uint_as_float(0x3F800000u | (w >> 9)) - 1.0f; }
// [1, 2) from the same 23 bits: u01<float> = u12 - 1 exactly, so an affine map of u01 folds its offset
// into one op with the same rounding (2 u01 - 1 = 2 u12 - 3, 1 - u01 = 2 - u12, u01 - 0.5 = u12 - 1.5)
__device__ __forceinline__ float u12(uint32_t w) { return __uint_as_float(0x3F800000u | (w >> 9)); }
template <> __device__ __forceinline__ double u01<double>(uint32_t w) { return (double)w * 0x1p-32; }

// rand 0.9 `random_range(low..high)` / `(low..=high)` on f64: one draw,
// value1_2 = from_bits((u >> 12) | 1.0.to_bits()), (value1_2 - 1) * scale + low.
template <typename R> struct Uniform;
template <> struct Uniform<double> {
    static __device__ __forceinline__ double range(uint64_t u, double low, double high) {
        const double v12 = __longlong_as_double((long long)((u >> 12) | 0x3FF0000000000000ull));
        const double scale = high - low;
        return (v12 - 1.0) * scale + low;
    }
};
template <> struct Uniform<float> {
    static __device__ __forceinline__ float range(uint64_t u, float low, float high) {
        const float v12 = __uint_as_float(0x3F800000u | (uint32_t)(u >> 41));
        return (v12 - 1.0f) * (high - low) + low;
    }
};

// One uniform draw in [low, high).  ChaCha8 always consumes a whole u64 (the
// reference's next_u64) so the f32 kernel keeps the reference's stream; Philox
// in the f32 kernel spends 32 bits per draw (23 are used), 4 draws per block.
template <typename R, class G>
__device__ __forceinline__ R draw(G& g, R low, R high) {
    if constexpr (sizeof(R) == 4 && !G::uses_lds) {
        const float v12 = __uint_as_float(0x3F800000u | (g.next32() >> 9));
        return (v12 - 1.0f) * (high - low) + low;
    } else {
        return Uniform<R>::range(g.next(), low, high);
    }
}
// A draw whose word g.ensure() already provided (ChaCha8: no per-draw ballot).
template <typename R, class G>
__device__ __forceinline__ R draw_taken(G& g, R low, R high) {
    if constexpr (sizeof(R) == 4 && !G::uses_lds) return draw<R>(g, low, high);
    else return Uniform<R>::range(g.take(), low, high);
}

// vector.rs:61-70 — rejection in [-1,1)^3 until 1e-160 < |p|^2 <= 1, returns p/|p|^2
template <typename R, class G> __device__ __forceinline__ V<R> random_in_unit_sphere(G& g) {
    const R tiny = sizeof(R) == 8 ? R(1e-160) : R(0);
    while (true) {
        g.ensure(3);
        const R x = draw_taken<R>(g, R(-1), R(1));
        const R y = draw_taken<R>(g, R(-1), R(1));
        const R z = draw_taken<R>(g, R(-1), R(1));
        const V<R> p = mk(x, y, z);
        const R ls = dot(p, p);
        if (tiny < ls && ls <= R(1)) return vdiv(p, ls);
    }
}
// vector.rs:72-81 — rejection in [-1,1)^2 until |p|^2 < 1, returns p/|p|^2
template <typename R, class G> __device__ __forceinline__ V<R> random_in_unit_disk(G& g) {
    while (true) {
        g.ensure(2);
        const R x = draw_taken<R>(g, R(-1), R(1));
        const R y = draw_taken<R>(g, R(-1), R(1));
        const V<R> p = mk(x, y, R(0));
        const R ls = dot(p, p);
        if (ls < R(1)) return vdiv(p, ls);
    }
}

// The two rejection samplers for the lanes with `need` set, called where the wave is converged:
// when a needing lane is short of words, every lane with room refills (not only the lanes still
// rejecting, as inside the samplers above), so the refills the wave executes serve most of its
// lanes.  Same draws, same order, same result per lane; the other lanes get a zero vector.
template <typename R, int D, class G>
__device__ __forceinline__ V<R> rejection_wave(G& g, bool need) {
    static_assert(G::uses_lds, "ChaCha8 streams only");
    V<R> out = mk(R(0), R(0), R(0));
    while (__ballot(need) != 0ull) {
        if (__ballot(need && g.count < (uint32_t)D) != 0ull) {
            if (g.count <= RING - 8) g.refill();
        }
        if (need) {
            const R x = draw_taken<R>(g, R(-1), R(1));
            const R y = draw_taken<R>(g, R(-1), R(1));
            const R z = D == 3 ? draw_taken<R>(g, R(-1), R(1)) : R(0);
            const V<R> q = mk(x, y, z);
            const R ls = dot(q, q);
            const bool ok = D == 3 ? ((sizeof(R) == 8 ? R(1e-160) : R(0)) < ls && ls <= R(1)) : ls < R(1);
            if (ok) {
                out = vdiv(q, ls);
                need = false;
            }
        }
    }
    return out;
}

// Philox mode: the same distributions as the two rejection samplers, drawn
// directly (no data-dependent loop, so no lane waits for another's retries).
// p uniform in the unit ball, p/|p|^2 = u/r with u uniform on the sphere and
// r = U^(1/3); p uniform in the unit disk, p/|p|^2 = (cos t, sin t)/sqrt(U).
template <typename R> __device__ __forceinline__ V<R> unit_ball_inverse(uint32_t w0, uint32_t w1, uint32_t w2) {
    const R z = sizeof(R) == 4 ? (R)__builtin_fmaf(2.0f, u12(w0), -3.0f) : fmad(R(2), u01<R>(w0), R(-1));
    const R turn = u01<R>(w1);
    const R w = sizeof(R) == 4 ? (R)(2.0f - u12(w2)) : R(1) - u01<R>(w2);  // (0, 1]
    const R s = fast_sqrt(fmax(R(0), R(1) - z * z));  // f32: v_sqrt_f32 (1 ulp)
    if constexpr (sizeof(R) == 4) {
        const float inv_r = __builtin_amdgcn_exp2f(-0.333333343f * __builtin_amdgcn_logf(w));
        const float c = __builtin_amdgcn_cosf(turn), sn = __builtin_amdgcn_sinf(turn);  // argument in turns
        const float k = inv_r * s;
        return mk(k * c, k * sn, inv_r * z);
    } else {
        double sn, c;
        sincospi(2.0 * turn, &sn, &c);
        const double inv_r = 1.0 / cbrt(w);
        return mk(inv_r * s * c, inv_r * s * sn, inv_r * z);
    }
}
template <typename R> __device__ __forceinline__ V<R> unit_disk_inverse(uint32_t w0, uint32_t w1) {
    const R turn = u01<R>(w0);
    const R w = sizeof(R) == 4 ? (R)(2.0f - u12(w1)) : R(1) - u01<R>(w1);  // (0, 1]
    if constexpr (sizeof(R) == 4) {
        const float inv_r = __builtin_amdgcn_rsqf(w);
        return mk(inv_r * __builtin_amdgcn_cosf(turn), inv_r * __builtin_amdgcn_sinf(turn), 0.0f);
    } else {
        double sn, c;
        sincospi(2.0 * turn, &sn, &c);
        const double inv_r = 1.0 / sqrt(w);
        return mk(inv_r * c, inv_r * sn, 0.0);
    }
}

// ----------------------------------------------------------------- geometry
template <typename R>
struct Ray {
    V<R> o, d;
    V<R> inv;  // 1/d for the slab tests
    R time;
};

// Both kernels multiply by 1/d in the slab test.  In the exact kernel 1/d is the
// IEEE quotient (3 divisions per ray instead of 6 per box): (b - o) * (1/d)
// differs from the reference's (b - o) / d by at most an ulp, while every box
// carries the reference's 1e-4 padding, so no primitive the reference would
// test is culled (or vice versa) outside measure-zero grazing cases; the
// d = +-0 cases give the same +-inf / NaN slab ends as the division.
template <typename R, bool EXACT> __device__ __forceinline__ void prep_ray(Ray<R>& r) {
    if constexpr (EXACT) r.inv = mk(R(1) / r.d.x, R(1) / r.d.y, R(1) / r.d.z);
    else r.inv = mk(fast_rcp(r.d.x), fast_rcp(r.d.y), fast_rcp(r.d.z));
}

// AABB::hit (aabb.rs:110-132) with range (0.001, t_max); t_max narrows during
// traversal.  Interval::ensure orders each slab pair by `<` (NaN-aware exactly
// like the reference); intersection uses f64::max/min (NaN-ignoring).
template <typename R, bool EXACT>
__device__ __forceinline__ bool box_hit(const R* bmin, const R* bmax, const Ray<R>& r, R t_max) {
    R lo = R(0.001), hi = t_max;
    const R* o = &r.o.x;
    const R* iv = &r.inv.x;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const R a = (bmin[k] - o[k]) * iv[k];  // reference: (bmin - o) / d (see prep_ray)
        const R b = (bmax[k] - o[k]) * iv[k];
        const bool lt = a < b;
        lo = fmax(lo, lt ? a : b);
        hi = fmin(hi, lt ? b : a);
    }
    return !(lo > hi);
}

// Sphere::hit (sphere.rs:105-163) root selection with range (0.001, inf); t or -1.
template <typename R>
__device__ __forceinline__ R sphere_t(const DPrim<R>& s, const Ray<R>& r) {
    if constexpr (sizeof(R) == 4) {
        // Fast variant: the quadratic is still evaluated in f64.  Center-relative
        // quantities of the huge ground spheres (r = 1e5 in spheres.toml, 1e3 in
        // earth.toml) keep no precision in f32; gfx950 runs f64 at
        // half the f32 rate and a sphere test is ~30 flops.
        Ray<double> rd;
        rd.o = mk((double)r.o.x, (double)r.o.y, (double)r.o.z);
        rd.d = mk((double)r.d.x, (double)r.d.y, (double)r.d.z);
        rd.time = (double)r.time;
        DPrim<double> sd;
        for (int k = 0; k < 3; ++k) { sd.a[k] = (double)s.a[k]; sd.b[k] = (double)s.b[k]; }
        sd.s = (double)s.s;
        const double t = sphere_t<double>(sd, rd);
        return t < 0.0 ? R(-1) : (R)t;
    }
    const V<R> center = ld3(s.a) + r.time * ld3(s.b);
    const V<R> ec = center - r.o;
    const R a = dot(r.d, r.d);
    const R h = dot(ec, r.d);
    const R c = dot(ec, ec) - s.s * s.s;
    const R disc = h * h - a * c;
    if (disc < R(0)) return R(-1);
    const R sq = sqrt(disc);
    R t = (h - sq) / a;
    if (R(0.001) < t && t < R(INFINITY)) return t;
    t = (h + sq) / a;
    if (R(0.001) < t && t < R(INFINITY)) return t;
    return R(-1);
}

// Plane::hit (plane.rs:141-174) with range [0.001, inf]; t or -1; alpha/beta out.
template <typename R>
__device__ __forceinline__ R plane_t(const DPrim<R>& q, const Ray<R>& r, R& alpha, R& beta, V<R>& point,
                                     R* den_out = nullptr) {
    const V<R> nrm = ld3(q.n);
    const R denom = dot(nrm, r.d);
    if (den_out) *den_out = denom;
    if (fabs(denom) < R(1e-8)) return R(-1);
    const R t = fast_div(q.s - dot(nrm, r.o), denom);
    if (!(R(0.001) <= t && t <= R(INFINITY))) return R(-1);
    point = vfma(t, r.d, r.o);
    const V<R> ph = point - ld3(q.a);
    alpha = dot(ld3(q.w), cross(ph, ld3(q.c)));
    beta = dot(ld3(q.w), cross(ld3(q.b), ph));
    bool inside;
    if (q.kind == PRIM_QUAD)
        inside = (R(0) <= alpha && alpha <= R(1)) && (R(0) <= beta && beta <= R(1));
    else
        inside = alpha > R(0) && beta > R(0) && (alpha + beta) < R(1);
    return inside ? t : R(-1);
}

// Fast kernel primitive test, branch-light (one select per condition):
// returns t in [0.001, t_max] of a hit, else -1.
template <typename R>
__device__ __forceinline__ R fast_prim_t(const DPrimFast<R>& q, const Ray<R>& r, R t_max) {
    if (q.kind == PRIM_SPHERE) {
        DPrim<R> s;
        for (int k = 0; k < 3; ++k) { s.a[k] = q.n[k]; s.b[k] = q.A[k]; }
        s.s = q.d;
        const R t = sphere_t(s, r);
        return t <= t_max ? t : R(-1);
    }
    const V<R> n = ld3(q.n);
    const R denom = dot(n, r.d);
    const R t = (q.d - dot(n, r.o)) * fast_rcp(denom);
    const V<R> p = vfma(t, r.d, r.o);
    const R alpha = dot(p, ld3(q.A)) - q.a0;
    const R beta = dot(p, ld3(q.B)) - q.b0;
    const bool quad_in = (alpha >= R(0) && alpha <= R(1)) && (beta >= R(0) && beta <= R(1));
    const bool tri_in = alpha > R(0) && beta > R(0) && (alpha + beta) < R(1);
    const bool ok = fabs(denom) >= R(1e-8) && t >= R(0.001) && t <= t_max && (q.kind == PRIM_QUAD ? quad_in : tri_in);
    return ok ? t : R(-1);
}

// Sphere::hit root selection (sphere.rs:105-163) in f32 for the world modes (the
// r = 1e5 and r = 1e3 ground spheres).  Relative to P, the sphere's point nearest the world
// origin (host, f64; moving with the centre), and V = P - center (|V| = |r|), with e = o - P:
//   c = |o - center|^2 - r^2 = |e|^2 + 2 e.V     (no |center|^2 - r^2 cancellation: a ground
//                                                 sphere's P is at the scene, e stays small)
//   h = (center - o).d = -(e.d + V.d)
// and the root nearer zero as c / q with q = h + sign(h) sqrt(h^2 - a c) (Press et al.): no
// cancellation for the self-intersection root of a ray leaving the surface.  Returns the
// smaller root in (0.001, inf), else the larger, else -1, as the reference.
template <class Q>  // Q: a DPrimWorld<float> in any address space (world list: the constant one)
__device__ __forceinline__ float sphere_t_world_f32(const Q& q, const Ray<float>& r) {
    const V<float> P = mk(q.AB[3], q.AB[4], q.AB[5]) + r.time * mk(q.AB[0], q.AB[1], q.AB[2]);
    const V<float> v = mk(q.S[0], q.S[1], q.S[2]);
    const V<float> e = r.o - P;
    const float a = dot(r.d, r.d);
    const float h = -(dot(e, r.d) + dot(v, r.d));
    const float c = dot(e, e) + 2.0f * dot(e, v);
    const float disc = h * h - a * c;
    const float qq = h + __builtin_copysignf(__builtin_amdgcn_sqrtf(fmaxf(disc, 0.0f)), h);
    const float t1 = qq * __builtin_amdgcn_rcpf(a), t2 = c * __builtin_amdgcn_rcpf(qq);
    const float tn = fminf(t1, t2), tf = fmaxf(t1, t2);
    const float t = tn > 0.001f ? tn : tf;
    return ((disc >= 0.0f) & (t > 0.001f) & (t < INFINITY)) ? t : -1.0f;
}
// The world modes' sphere tests: f32 (above) for the world list's PRIM_SPHERE32 runs, spheres whose
// anchor lies within the scene's scale (AB[6] = 0: |P| + |speed| <= SPHERE_F32_EXTENT, flatten.cpp;
// the r = 1e3 / 1e5 ground spheres included), whose hit points the record then puts back on the
// surface with an anchored Newton step (make_record_world); the quadratic in f64 (below) for spheres
// anchored far outside the scene (their e = o - P would not stay small; such a scene stays off the
// world BVH, whose leaves compile the f32 test only: world_prim_t).
template <class Q>
__device__ __forceinline__ float sphere_t_world_f64(const Q& q, const Ray<float>& r) {
    DPrim<float> sp;
    for (int c = 0; c < 3; ++c) { sp.a[c] = q.N[c]; sp.b[c] = q.AB[c]; }
    sp.s = q.D;
    return sphere_t(sp, r);  // (f32 specialisation: in f64)
}

// ray into object space through an instance's chain (outer -> inner)
template <typename R, bool EXACT, bool PREP = true>  // PREP: 1/d for slab tests (not needed by prim tests)
__device__ __forceinline__ void xform_in(const DSceneView<R>& sc, const DInstance& inst, Ray<R>& r) {
    for (uint32_t k = 0; k < inst.num_xforms; ++k) {
        const DXform<R>& x = sc.xforms[inst.first_xform + k];
        if (x.kind == XF_TRANSLATE) {
            r.o = r.o - ld3(x.m);
        } else if (x.kind == XF_ROTATE) {
            r.o = mat3(x.m, r.o);
            r.d = mat3(x.m, r.d);
        } else {
            r.o = xf_point(x.m, r.o);
            r.d = xf_vector(x.m, r.d);
        }
    }
    if constexpr (PREP) prep_ray<R, EXACT>(r);
}

template <typename R>
struct Rec {  // HitRecord (hitable.rs:14-22) of the closest hit, world space
    V<R> p, n;
    R u, v;
    bool front;
    uint32_t mat;
};
// World-mode sphere records leave u = UV_DEFERRED (no hit has it: u is in [0, 1]) and sphere_uv
// computes (u, v) when a texture needs them (HitRecord::new_with_uv's sphere uv, sphere.rs:148-161):
// the outward normal is n on the front face, -n on the back (n = -signum(d . outward) * outward).
constexpr float UV_DEFERRED = -2.0f;
// f32 acos / atan2 for the fast kernels' sphere uv: polynomials within 2.4e-7 / 1.4e-7 rad of the
// true values (the libm f32 calls: 21 / 42 VALU, these 11 / 19).  A texel index floor(u * W) then
// differs from the f64 one only within ~1e-4 texel of a texel edge (W = 2048), inside the f32
// kernels' statistical tolerance; the f64 kernels keep libm's acos / atan2.
//   acos: Abramowitz & Stegun 4.4.46, sqrt(1 - |x|) P7(|x|) (|err| <= 2e-8 in exact arithmetic),
//         acos(-x) = pi - acos(x);
//   atan2: a = min(|x|, |y|) / max(|x|, |y|), atan(a) = a P7(a^2) (least-squares fit on [0, 1]),
//         then the octant.
__device__ __forceinline__ float acos_f32(float x) {
    const float a = fabsf(x);
    float p = -0.0012624911f;
    p = __builtin_fmaf(p, a, 0.0066700901f);
    p = __builtin_fmaf(p, a, -0.0170881256f);
    p = __builtin_fmaf(p, a, 0.0308918810f);
    p = __builtin_fmaf(p, a, -0.0501743046f);
    p = __builtin_fmaf(p, a, 0.0889789874f);
    p = __builtin_fmaf(p, a, -0.2145988016f);
    p = __builtin_fmaf(p, a, 1.5707963050f);
    const float r = __builtin_amdgcn_sqrtf(1.0f - a) * p;
    return x < 0.0f ? 3.14159265f - r : r;
}
__device__ __forceinline__ float atan2_f32(float y, float x) {
    const float ax = fabsf(x), ay = fabsf(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float a = mx > 0.0f ? mn * __builtin_amdgcn_rcpf(mx) : 0.0f;
    const float s = a * a;
    float p = -0.0040731244f;
    p = __builtin_fmaf(p, s, 0.0219459739f);
    p = __builtin_fmaf(p, s, -0.0560623035f);
    p = __builtin_fmaf(p, s, 0.0965619683f);
    p = __builtin_fmaf(p, s, -0.1391578019f);
    p = __builtin_fmaf(p, s, 0.1994850487f);
    p = __builtin_fmaf(p, s, -0.3333010674f);
    p = __builtin_fmaf(p, s, 0.9999994636f);
    float r = a * p;
    r = ay > ax ? 1.57079633f - r : r;
    r = x < 0.0f ? 3.14159265f - r : r;
    return __builtin_copysignf(r, y);
}
template <typename R>
__device__ __forceinline__ void sphere_uv(const Rec<R>& h, R& u, R& v) {
    const V<R> geo = h.front ? h.n : -h.n;
    R theta, phi;
    if constexpr (sizeof(R) == 4) {
        theta = acos_f32(-geo.y);
        phi = atan2_f32(-geo.z, geo.x) + R(M_PI);
    } else {
        theta = acos(-geo.y);
        phi = atan2(-geo.z, geo.x) + R(M_PI);
    }
    u = phi * R(1.0 / (2.0 * M_PI));
    v = theta * R(1.0 / M_PI);
}

// hit point / normal back out (inner -> outer); Scale leaves the normal alone (scale.rs:82-85)
template <typename R>
__device__ __forceinline__ void xform_out(const DSceneView<R>& sc, const DInstance& inst, Rec<R>& h) {
    for (uint32_t k = inst.num_xforms; k-- > 0;) {
        const DXform<R>& x = sc.xforms[inst.first_xform + k];
        if (x.kind == XF_TRANSLATE) {
            h.p = h.p + ld3(x.m);
        } else if (x.kind == XF_ROTATE) {
            h.p = mat3(x.inv, h.p);
            h.n = mat3(x.inv, h.n);
        } else {
            h.p = xf_point(x.inv, h.p);
        }
    }
}

// Fast kernel: composed instance map (device_scene.hpp DInstFast)
template <typename R>
__device__ __forceinline__ void enter_fast(const DInstFast<R>& f, Ray<R>& r) {
    r.o = mat3(f.A, r.o) + ld3(f.b);
    r.d = mat3(f.A, r.d);
    r.inv = mk(fast_rcp(r.d.x), fast_rcp(r.d.y), fast_rcp(r.d.z));
}
template <typename R>
__device__ __forceinline__ void leave_fast(const DInstFast<R>& f, Rec<R>& h) {
    h.p = mat3(f.C, h.p) + ld3(f.c);
    h.n = mat3(f.N, h.n);
}

// Whole node in one go (16-byte loads issued together, before the kind test).
template <typename R>
__device__ __forceinline__ DNode<R> load_node(const DNode<R>* p) {
    DNode<R> n;
    const uint4* s = reinterpret_cast<const uint4*>(p);
    uint4* d = reinterpret_cast<uint4*>(&n);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(DNode<R>) / 16); ++k) d[k] = s[k];
    // keep every part live here: otherwise the box loads sink below the kind
    // test and a second dependent LDS round trip follows the first
#pragma unroll
    for (int k = 0; k < (int)(sizeof(DNode<R>) / 16); ++k)
        asm volatile("" ::"v"(d[k].x), "v"(d[k].y), "v"(d[k].z), "v"(d[k].w));
    return n;
}

template <typename R, int MAXD>
struct HitMin {
    R t;
    uint32_t prim;
    int depth;
    uint32_t inst[MAXD > 0 ? MAXD : 1];
    // the exact plane test's own object-space point, (alpha, beta) and n.d of the winner, which the
    // hit record would compute again bit for bit (xcands_finish, NRT_REC_CARRY); pre: they are set
    V<R> pp;
    R pu, pv, pden;
    bool pre = false;
};

// World-space mode (MAXD = 0, fast kernel): the wave tests every primitive,
// grouped by kind (the reference's candidate order within a kind; `t <= t_best`:
// the later candidate wins ties, as in trace).  The primitive index is wave-uniform, so
// each record is read once per wave through the scalar cache into SGPRs (the
// constant address space makes the loads s_load), and no lane diverges.
template <typename R>
using ConstPrimWorld = const __attribute__((address_space(4))) DPrimWorld<R>*;
using ConstU32 = const __attribute__((address_space(4))) uint32_t*;
typedef float f32x2 __attribute__((ext_vector_type(2)));

// Axis-aligned quad run (PRIM_QUAD_X + A; device_scene.hpp): t from the per-ray
// reciprocal, (alpha, beta) from the two in-plane coordinates only.
// Coplanar-tie key (device_scene.hpp WCLASS_*): t scaled by the unit's tie factor when TIE.
template <bool TIE>
__device__ __forceinline__ float tie_key(float t, float f) {
    if constexpr (TIE) return t * f;
    else return t;
}
__device__ __forceinline__ float tie_factor(uint32_t cls) {
    return cls == WCLASS_WIN ? 1.0f - WTIE_EPS : (cls == WCLASS_LOSE ? 1.0f + WTIE_EPS : 1.0f);
}

template <int A>
__device__ __forceinline__ void axis_quad_run(ConstPrimWorld<float> wp, uint32_t& k, uint32_t end, const Ray<float>& ray,
                                              const float inv[3], const float oinv[3], float& t_best, int32_t& best) {
    constexpr int A1 = (A + 1) % 3, A2 = (A + 2) % 3;
    const float* o = &ray.o.x;
    const float* d = &ray.d.x;
    for (; k < end; ++k) {
        const ConstPrimWorld<float> q = wp + k;
        const float t = __builtin_fmaf(q->N[A1], inv[A], -oinv[A]);  // (P - o_a) / d_a
        const float p1 = o[A1] + t * d[A1], p2 = o[A2] + t * d[A2];
#if NRT_PK_QUAD
        const f32x2 ab = f32x2{q->AB[2 * A1], q->AB[2 * A1 + 1]} * p1 + f32x2{q->AB[2 * A2], q->AB[2 * A2 + 1]} * p2 -
                         f32x2{q->AB[6], q->AB[7]};
#else  // the same expressions per component (the same contraction: the same roundings)
        const f32x2 ab = {q->AB[2 * A1] * p1 + q->AB[2 * A2] * p2 - q->AB[6],
                          q->AB[2 * A1 + 1] * p1 + q->AB[2 * A2 + 1] * p2 - q->AB[7]};
#endif
        const float lo = fminf(ab.x, ab.y);
        const bool ok = (fabsf(d[A]) >= q->N[A2]) & (t >= 0.001f) & (t <= t_best) & (lo >= 0.0f) & (ab.x <= 1.0f) &
                        (ab.y <= 1.0f);
        t_best = ok ? t : t_best;
        best = ok ? (int32_t)k : best;
    }
}

// Box units (PRIM_BOXY, PRIM_BOX): the slab planes' t along the ray per axis (a*: plane l = D,
// b*: l = D + L) and the local reciprocals that give the entry sides.  One definition serves the run
// loop and the deferred face resolution (NRT_BOX_DEFER), so both round alike (-ffp-contract=on fuses
// by expression: the same source, the same FMAs).
struct BoxPlanes {
    float ax, bx, ay, by, az, bz;
    float ix, iy, iz;  // local 1/d' (BOXY: iy unused, its y axis is the world's)
};
__device__ __forceinline__ BoxPlanes boxy_planes(ConstPrimWorld<float> q, const f32x2& dox, const f32x2& doz,
                                                 const float inv[3], const float oinv[3]) {
    BoxPlanes b;
#if NRT_PK_LIST
    const f32x2 la = dox * q->N[0] + doz * q->N[2];  // (row_A . d, row_A . o)
    const f32x2 lb = dox * q->AB[0] + doz * q->AB[2];
#else
    const f32x2 la = {dox.x * q->N[0] + doz.x * q->N[2], dox.y * q->N[0] + doz.y * q->N[2]};
    const f32x2 lb = {dox.x * q->AB[0] + doz.x * q->AB[2], dox.y * q->AB[0] + doz.y * q->AB[2]};
#endif
    b.ix = __builtin_amdgcn_rcpf(la.x);
    b.iz = __builtin_amdgcn_rcpf(lb.x);
    b.iy = 0.0f;
    b.ax = (q->D - la.y) * b.ix;
    b.az = (q->AB[3] - lb.y) * b.iz;
    b.bx = __builtin_fmaf(q->D - la.y, b.ix, b.ix);
    b.bz = __builtin_fmaf(q->AB[3] - lb.y, b.iz, b.iz);
    b.ay = __builtin_fmaf(q->AB[4], inv[1], -oinv[1]);
    b.by = __builtin_fmaf(q->AB[5], inv[1], -oinv[1]);
    return b;
}
__device__ __forceinline__ BoxPlanes box_planes(ConstPrimWorld<float> q, const f32x2& dox, const f32x2& doy,
                                                const f32x2& doz) {
    BoxPlanes b;
    // (d', E^-1 o) per local axis; x' = E^-1 x - E^-1 c
#if NRT_PK_QUAD
    const f32x2 lx = dox * q->N[0] + doy * q->N[1] + doz * q->N[2];
    const f32x2 ly = dox * q->AB[0] + doy * q->AB[1] + doz * q->AB[2];
    const f32x2 lz = dox * q->AB[4] + doy * q->AB[5] + doz * q->AB[6];
#else
    auto row = [&](float a, float b, float c) {
        return f32x2{dox.x * a + doy.x * b + doz.x * c, dox.y * a + doy.y * b + doz.y * c};
    };
    const f32x2 lx = row(q->N[0], q->N[1], q->N[2]), ly = row(q->AB[0], q->AB[1], q->AB[2]),
                lz = row(q->AB[4], q->AB[5], q->AB[6]);
#endif
    b.ix = __builtin_amdgcn_rcpf(lx.x);
    b.iy = __builtin_amdgcn_rcpf(ly.x);
    b.iz = __builtin_amdgcn_rcpf(lz.x);
    // planes l = D and l = D + L per local axis (L_a in S[a]; flatten.cpp fuse_box)
    b.ax = (q->D - lx.y) * b.ix;
    b.ay = (q->AB[3] - ly.y) * b.iy;
    b.az = (q->AB[7] - lz.y) * b.iz;
    b.bx = __builtin_fmaf(q->D - lx.y, b.ix, b.ix);
    b.by = __builtin_fmaf(q->AB[3] - ly.y, b.iy, b.iy);
    b.bz = __builtin_fmaf(q->AB[7] - lz.y, b.iz, b.iz);
    return b;
}
// The face quad (0-5, the unit's record + 1 + face) through which the ray enters (entry) or leaves
// the box: face slot 2*axis + side (side 0 = local plane x' = 0; entered there when d' > 0), the
// quad that lies there from 3 bits per slot of meta.  sy: BOXY's y slot pair from the world ray.
// 1 for a negative x, else 0: the sign bit (= x < 0 for every non-NaN x, -inf from rcp(-0) included; a
// NaN ray's tests all fail, so its slots are never read): one shift instead of a compare and a select
__device__ __forceinline__ uint32_t neg_bit(float x) { return __float_as_uint(x) >> 31; }
__device__ __forceinline__ uint32_t box_face(const BoxPlanes& b, uint32_t meta, bool entry, uint32_t sy) {
    const float nx = fminf(b.ax, b.bx), ny = fminf(b.ay, b.by), nz = fminf(b.az, b.bz);
    const float fx = fmaxf(b.ax, b.bx), fy = fmaxf(b.ay, b.by), fz = fmaxf(b.az, b.bz);
    const float tn = fmaxf(fmaxf(nx, ny), nz), tf = fminf(fminf(fx, fy), fz);
    const uint32_t sx = neg_bit(b.ix), sz = 4u | neg_bit(b.iz);
    // the plane that gave t (entry: the last near plane, x before y before z on a tie; exit: the
    // first far plane), then its side: entry slots from the signs, an exit leaves by the other side
    const float t = entry ? tn : tf, cx = entry ? nx : fx, cy = entry ? ny : fy;
    uint32_t s = sz;
    s = t == cy ? sy : s;
    s = t == cx ? sx : s;
    const uint32_t slot = entry ? s : s ^ 1u;
    return __builtin_amdgcn_ubfe(meta, WKIND_BITS + 3u * slot, 3);
}
// best of a box unit whose face is resolved after the run loop (NRT_BOX_DEFER): the unit's index |
// WBEST_BOX (| WBEST_BOXY for a box turned about y) | WBEST_ENTRY (the ray enters at t)
constexpr uint32_t WBEST_BOX = 1u << 30, WBEST_BOXY = 1u << 29, WBEST_ENTRY = 1u << 28;
template <bool BOX = true, bool BOXY = true>  // the box kinds the scene's world list holds
__device__ __forceinline__ int32_t resolve_box_face(ConstPrimWorld<float> wp, int32_t best, const f32x2& dox,
                                                    const f32x2& doy, const f32x2& doz, const float inv[3],
                                                    const float oinv[3], const uint32_t entry_slot[3]) {
    const uint32_t k = (uint32_t)best & (WBEST_ENTRY - 1u);
    const ConstPrimWorld<float> q = wp + k;
    const bool entry = ((uint32_t)best & WBEST_ENTRY) != 0u;
    uint32_t face = 0;
    if (BOXY && (!BOX || ((uint32_t)best & WBEST_BOXY))) {
        face = box_face(boxy_planes(q, dox, doz, inv, oinv), q->meta, entry, entry_slot[1]);
    } else if (BOX) {
        const BoxPlanes b = box_planes(q, dox, doy, doz);
        face = box_face(b, q->meta, entry, 2u | neg_bit(b.iy));
    }
    return (int32_t)(k + 1u + face);
}

// The units of one run (kind = the run's kind): closest hit so far in (t_best, best).
// `t <= t_best`: the later candidate wins an exact tie (the flattener orders the units
// so that this is the reference's winner of every coplanar tie, device_scene.hpp WCLASS_*).
template <bool FLAT>
__device__ __forceinline__ void world_run(ConstPrimWorld<float> wp, uint32_t kind, uint32_t& k, uint32_t count,
                                          const Ray<float>& ray, const f32x2& dox, const f32x2& doy, const f32x2& doz,
                                          const float inv[3], const float oinv[3], const uint32_t entry_slot[3],
                                          float& t_best, int32_t& best) {
    const uint32_t end = k + count;
    if (kind == PRIM_QUAD_X) { axis_quad_run<0>(wp, k, end, ray, inv, oinv, t_best, best); return; }
    if (kind == PRIM_QUAD_Y) { axis_quad_run<1>(wp, k, end, ray, inv, oinv, t_best, best); return; }
    if (kind == PRIM_QUAD_Z) { axis_quad_run<2>(wp, k, end, ray, inv, oinv, t_best, best); return; }
    if (kind == PRIM_ABOX) {  // room: axis-aligned box whose present faces are quads
        for (uint32_t b = 0; b < count; ++b, k += BOX_ENTRIES) {
            const ConstPrimWorld<float> q = wp + k;
            const uint32_t present = q->meta >> ABOX_PRESENT_SHIFT;
            const float lx = __builtin_fmaf(q->N[0], inv[0], -oinv[0]), hx = __builtin_fmaf(q->AB[0], inv[0], -oinv[0]);
            const float ly = __builtin_fmaf(q->N[1], inv[1], -oinv[1]), hy = __builtin_fmaf(q->AB[1], inv[1], -oinv[1]);
            const float lz = __builtin_fmaf(q->N[2], inv[2], -oinv[2]), hz = __builtin_fmaf(q->AB[2], inv[2], -oinv[2]);
            const float nx = fminf(lx, hx), ny = fminf(ly, hy), nz = fminf(lz, hz);
            const float fx = fmaxf(lx, hx), fy = fmaxf(ly, hy), fz = fmaxf(lz, hz);
            const float tn = fmaxf(fmaxf(nx, ny), nz), tf = fminf(fminf(fx, fy), fz);
            // face slots 2*axis + side (branch-free selects): entry slots from the ray's
            // direction signs, exit = the opposite side of the exit axis
            uint32_t e = entry_slot[2], x = entry_slot[2] ^ 1u;
            e = tn == ny ? entry_slot[1] : e;
            e = tn == nx ? entry_slot[0] : e;
            x = tf == fy ? entry_slot[1] ^ 1u : x;
            x = tf == fx ? entry_slot[0] ^ 1u : x;
            const bool use_entry = (tn >= 0.001f) & (__builtin_amdgcn_ubfe(present, e, 1) != 0u);
            const float t = use_entry ? tn : tf;
            const bool ok = (tn <= tf) & (t >= 0.001f) & (t <= t_best) &
                            (use_entry | (__builtin_amdgcn_ubfe(present, x, 1) != 0u));
            t_best = ok ? t : t_best;
            best = ok ? (int32_t)(k + 1 + (use_entry ? e : x)) : best;  // the face quad's record
        }
        return;
    }
    if (kind == PRIM_BOXY) {  // box turned about y: two local rows + the world y slab
        for (uint32_t b = 0; b < count; ++b, k += BOX_ENTRIES) {
            const ConstPrimWorld<float> q = wp + k;
            const BoxPlanes bp = boxy_planes(q, dox, doz, inv, oinv);
            const float nx = fminf(bp.ax, bp.bx), ny = fminf(bp.ay, bp.by), nz = fminf(bp.az, bp.bz);
            const float fx = fmaxf(bp.ax, bp.bx), fy = fmaxf(bp.ay, bp.by), fz = fmaxf(bp.az, bp.bz);
            const float tn = fmaxf(fmaxf(nx, ny), nz), tf = fminf(fminf(fx, fy), fz);
            const bool entry = tn >= 0.001f;
            const float t = entry ? tn : tf;
            // = (tn <= tf) & (t >= 0.001) & (t <= t_best): an entry t is >= 0.001 by choice,
            // an exit t = tf (tn < 0.001 <= tf then orders the slab)
            const bool ok = (t <= fminf(tf, t_best)) & (t >= 0.001f);
            t_best = ok ? t : t_best;
#if NRT_BOX_DEFER
            best = ok ? (int32_t)(k | WBEST_BOX | WBEST_BOXY | (entry ? WBEST_ENTRY : 0u)) : best;
#else
            best = ok ? (int32_t)(k + 1 + box_face(bp, q->meta, entry, entry_slot[1])) : best;  // the face quad's record
#endif
        }
        return;
    }
    if (kind == PRIM_BOX) {  // fused parallelepiped: one slab test in its local frame
        for (uint32_t b = 0; b < count; ++b, k += BOX_ENTRIES) {
            const ConstPrimWorld<float> q = wp + k;
            const BoxPlanes bp = box_planes(q, dox, doy, doz);
            const float tn = fmaxf(fmaxf(fminf(bp.ax, bp.bx), fminf(bp.ay, bp.by)), fminf(bp.az, bp.bz));
            const float tf = fminf(fminf(fmaxf(bp.ax, bp.bx), fmaxf(bp.ay, bp.by)), fmaxf(bp.az, bp.bz));
            // entry face unless it lies before t_min (origin on or inside the box): then the exit face
            const bool entry = tn >= 0.001f;
            const float t = entry ? tn : tf;
            const bool ok = (t <= fminf(tf, t_best)) & (t >= 0.001f);  // (as PRIM_BOXY)
            t_best = ok ? t : t_best;
#if NRT_BOX_DEFER
            best = ok ? (int32_t)(k | WBEST_BOX | (entry ? WBEST_ENTRY : 0u)) : best;
#else
            best = ok ? (int32_t)(k + 1 + box_face(bp, q->meta, entry, 2u | neg_bit(bp.iy))) : best;
#endif
        }
        return;
    }
    if (!FLAT && kind == PRIM_SPHERE32) {  // FLAT: the scene has no spheres (not compiled in)
        for (; k < end; ++k) {
            const float t = sphere_t_world_f32(wp[k], ray);
            const bool ok = (t >= 0.0f) & (t <= t_best);
            t_best = ok ? t : t_best;
            best = ok ? (int32_t)k : best;
        }
        return;
    }
    if (!FLAT && kind == PRIM_SPHERE) {  // the large spheres, in f64
        for (; k < end; ++k) {
            const float t = sphere_t_world_f64(wp[k], ray);
            const bool ok = (t >= 0.0f) & (t <= t_best);
            t_best = ok ? t : t_best;
            best = ok ? (int32_t)k : best;
        }
        return;
    }
    const bool quad = kind == PRIM_QUAD;
    for (; k < end; ++k) {
        const ConstPrimWorld<float> q = wp + k;
#if NRT_PK_QUAD
        const f32x2 dn = dox * q->N[0] + doy * q->N[1] + doz * q->N[2];  // (N.d, N.o)
#else
        const f32x2 dn = {dox.x * q->N[0] + doy.x * q->N[1] + doz.x * q->N[2],
                          dox.y * q->N[0] + doy.y * q->N[1] + doz.y * q->N[2]};  // (N.d, N.o)
#endif
        const float t = (q->D - dn.y) * __builtin_amdgcn_rcpf(dn.x);
        const float px = ray.o.x + t * ray.d.x, py = ray.o.y + t * ray.d.y, pz = ray.o.z + t * ray.d.z;
#if NRT_PK_QUAD
        const f32x2 ab = f32x2{q->AB[0], q->AB[1]} * px + f32x2{q->AB[2], q->AB[3]} * py +
                         f32x2{q->AB[4], q->AB[5]} * pz - f32x2{q->AB[6], q->AB[7]};  // (alpha, beta)
#else
        const f32x2 ab = {q->AB[0] * px + q->AB[2] * py + q->AB[4] * pz - q->AB[6],
                          q->AB[1] * px + q->AB[3] * py + q->AB[5] * pz - q->AB[7]};  // (alpha, beta)
#endif
        const float lo = fminf(ab.x, ab.y);
        // quad closed [0,1]^2 (plane.rs:121-126), triangle open (plane.rs:128-133); a NaN
        // coordinate can only come from a rejected denominator or t
        const bool inside = quad ? (lo >= 0.0f) & (ab.x <= 1.0f) & (ab.y <= 1.0f) : (lo > 0.0f) & (ab.x + ab.y < 1.0f);
        const bool ok = (fabsf(dn.x) >= 1e-8f) & (t >= 0.001f) & (t <= t_best) & inside;
        t_best = ok ? t : t_best;
        best = ok ? (int32_t)k : best;
    }
}

// World-list signature of a scene-specialised kernel (jit.hip): the run words (kind | count <<
// WRUN_KIND_BITS, FlatScene::wruns) as template arguments, so the run loop unrolls with each
// unit's test and scalar loads known at compile time.  NoSig: the generic loop over sc.wruns.
struct NoSig {
    static constexpr uint32_t n = 0;
    static constexpr int bvh = 0;  // world-BVH width known at compile time (BvhSig), 0: read sc.wbvh4
    static constexpr bool tie = false;
    static constexpr int prims = 0;  // world-BVH leaf primitive kinds (WPRIMS_*), 0: decided per primitive
    static constexpr int exact = 0;  // exact kernel: traversal fixed at compile time (ExactSig), 0: runtime
    static constexpr bool lstack = false;
    static constexpr bool persist = false;
};
template <uint32_t... RUNS>
struct WorldSig {
    static constexpr uint32_t n = sizeof...(RUNS);
    template <uint32_t KIND>
    static constexpr bool has() { return ((((RUNS & WRUN_KIND_MASK) == KIND) || ...)); }
    // the list's units use the ray's 1/d (flatten.cpp's WFLAG_AXIS_QUADS, known at compile time)
    static constexpr bool axis = ((((RUNS & WRUN_KIND_MASK) >= PRIM_QUAD_X && (RUNS & WRUN_KIND_MASK) != PRIM_SPHERE32)) || ...);
    static constexpr int bvh = 0;
    static constexpr bool tie = false;
    static constexpr int prims = 0;
    static constexpr int exact = 0;
    static constexpr bool lstack = false;
    static constexpr bool persist = false;
};
// Exact f64 kernel: the traversal nrt_exact_mode picked, as a constant, so the variant carries
// the code of that walk only (EXACT_SIG_WORLD_PF: the world-BVH walk with the f32 prefilter of
// plane-only scenes, and the unfiltered walk it falls back to).
enum : int { EXACT_SIG_WORLD_PF = 1, EXACT_SIG_SLOTS_PF = 2, EXACT_SIG_SLOTS = 3, EXACT_SIG_WORLD = 4 };
// (EXACT_SIG_WORLD: the unfiltered world walk of scenes with spheres, compact tree, LDS stack)
template <int MODE, int WIDTH, bool LSTACK = false, bool PERSIST = false>
struct ExactSig {
    static constexpr uint32_t n = 0;
    static constexpr int bvh = WIDTH;  // culling walk: 4 / 2 the stack walk of that width, XTHREAD_W the
                                       // threaded tree, WBVH_COMPACT the compact tree, 0: chosen at run time
    static constexpr bool tie = false;
    static constexpr int prims = 0;
    static constexpr int exact = MODE;
    static constexpr bool lstack = LSTACK;  // compact walk: its 16-bit stack in LDS (fewer waves), not scratch
    // the prefiltered compact walk kept across shading rounds (XWalk; render_kernel's persistent-walk loop)
    static constexpr bool persist = PERSIST;
};
// World-BVH mode (jit.hip): the tree's width (2 or 4), whether it holds coplanar-tie keys
// (WFLAG_COPLANAR) and which primitive kinds its leaves hold (WPRIMS_*) as constants, so one
// traversal and one primitive test are compiled instead of several.
template <int WIDTH, bool TIE, int PRIMS = WPRIMS_ANY>
struct BvhSig {
    static constexpr uint32_t n = 0;
    static constexpr int bvh = WIDTH;
    static constexpr bool tie = TIE;
    static constexpr int prims = PRIMS;
    static constexpr int exact = 0;
    static constexpr bool lstack = false;
    static constexpr bool persist = false;
};
template <bool FLAT, uint32_t... RUNS>
__device__ __forceinline__ void sig_runs(WorldSig<RUNS...>, ConstPrimWorld<float> wp, uint32_t& k, const Ray<float>& ray,
                                         const f32x2& dox, const f32x2& doy, const f32x2& doz, const float inv[3],
                                         const float oinv[3], const uint32_t entry_slot[3], float& t_best,
                                         int32_t& best) {
    (world_run<FLAT>(wp, RUNS & WRUN_KIND_MASK, k, RUNS >> WRUN_KIND_BITS, ray, dox, doy, doz, inv, oinv, entry_slot,
                     t_best, best),
     ...);
}

template <typename R, int MAXD, bool FLAT = false, class SIG = NoSig>
__device__ __forceinline__ bool trace_world(const DSceneView<R>& sc, const Ray<R>& ray, HitMin<R, MAXD>& hm) {
    static_assert(sizeof(R) == 4, "world-space mode is an f32-kernel mode");
#if NRT_WL_RELOAD
    // the records' scalar loads stay inside the loop (the base laundered per query): loop-invariant
    // records no longer hold ~30 SGPRs for the whole kernel (occupancy experiments)
    uint64_t wpi = (uint64_t)sc.wprims;
    asm volatile("" : "+s"(wpi));
    const ConstPrimWorld<float> wp = (ConstPrimWorld<float>)wpi;
#else
    const ConstPrimWorld<float> wp = (ConstPrimWorld<float>)sc.wprims;
#endif
    const ConstU32 runs = (ConstU32)sc.wruns;
    float t_best = INFINITY;
    int32_t best = -1;
    // (d, o) pairs: N.d and N.o come out of one packed FMA chain
    const f32x2 dox = {ray.d.x, ray.o.x}, doy = {ray.d.y, ray.o.y}, doz = {ray.d.z, ray.o.z};
    float inv[3], oinv[3];  // axis-aligned quads and rooms: 1/d and o/d
    uint32_t entry_slot[3] = {0u, 2u, 4u};  // rooms: face slot 2*axis + side entered along each axis
    bool axis;
    if constexpr (SIG::n > 0) axis = SIG::axis;  // (no uniform flag held through the loop)
    else axis = (sc.wflags & WFLAG_AXIS_QUADS) != 0u;
    if (axis) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            inv[a] = __builtin_amdgcn_rcpf((&ray.d.x)[a]);
            oinv[a] = (&ray.o.x)[a] * inv[a];
            entry_slot[a] = 2u * a + neg_bit(inv[a]);  // d > 0 enters at the low plane
        }
    }
    uint32_t k = 0;
    if constexpr (SIG::n > 0) {  // a scene-specialised kernel (jit.hip): runs known at compile time
        sig_runs<FLAT>(SIG{}, wp, k, ray, dox, doy, doz, inv, oinv, entry_slot, t_best, best);
#if NRT_BOX_DEFER
        if (best >= 0 && ((uint32_t)best & WBEST_BOX))
            best = resolve_box_face<SIG::template has<PRIM_BOX>(), SIG::template has<PRIM_BOXY>()>(wp, best, dox, doy, doz,
                                                                                               inv, oinv, entry_slot);
#endif
        hm.t = t_best;
        hm.prim = (uint32_t)best;
        hm.depth = 0;
        return best >= 0;
    }
    for (uint32_t r = 0; r < sc.n_wruns; ++r) {
        const uint32_t run = runs[r];
        const uint32_t kind = run & WRUN_KIND_MASK, count = run >> WRUN_KIND_BITS;
        world_run<FLAT>(wp, kind, k, count, ray, dox, doy, doz, inv, oinv, entry_slot, t_best, best);
    }
#if NRT_BOX_DEFER
    if (best >= 0 && ((uint32_t)best & WBEST_BOX)) best = resolve_box_face(wp, best, dox, doy, doz, inv, oinv, entry_slot);
#endif
    hm.t = t_best;
    hm.prim = (uint32_t)best;
    hm.depth = 0;
    return best >= 0;
}

// World-BVH mode (MAXD = MODE_WORLD_BVH = -1, fast kernel): per-lane traversal of
// the binned-SAH tree (device_scene.hpp DBvhNode).  Both children's boxes are
// tested per visit; the nearer hit child is taken and the farther pushed on the
// lane's stack (LDS, entry k at stack[k * BLOCK]), so t_best shrinks early and
// culls the far side.  The lanes of a wave descend until each holds a leaf (or
// is done) before leaves are tested together ("while-while").
#ifndef NRT_WBVH_SPHERE32
// world-BVH leaf spheres: 2 = the anchored f32 quadratic only (the host keeps scenes with spheres
// anchored outside the scene scale off the world BVH: flatten.cpp build_wbvh), 1 = f32 or f64 per
// record (both compiled in: 131 VGPRs, 3 waves), 0 = f64 only (118 VGPRs)
#define NRT_WBVH_SPHERE32 2
#endif
template <bool FLAT = false, bool TIE = false, int PRIMS = 0>  // PRIMS: WPRIMS_* of the scene's leaves
__device__ __forceinline__ float world_prim_t(const DPrimWorld<float>& q, const Ray<float>& ray, float t_best) {
    const uint32_t kind = q.meta & WKIND_MASK;  // BVH leaves hold spheres, quads and triangles only
    if (!FLAT && kind == PRIM_SPHERE) {  // FLAT: the scene has no spheres
        // one sphere test compiled in (both took the generic world-BVH kernel to 129 VGPRs, 3 waves
        // per SIMD: spheres.toml 1080p 34.9 -> 39.9 ms, round 3)
        float t;
        if constexpr (NRT_WBVH_SPHERE32 == 2) t = sphere_t_world_f32(q, ray);
        else if constexpr (NRT_WBVH_SPHERE32 == 1) t = q.AB[6] == 0.0f ? sphere_t_world_f32(q, ray) : sphere_t_world_f64(q, ray);
        else t = sphere_t_world_f64(q, ray);
        return (t >= 0.0f && t <= t_best) ? t : -1.0f;
    }
    const V<float> nrm = ld3(q.N);
    const float denom = dot(nrm, ray.d);
    const float t = (q.D - dot(nrm, ray.o)) * __builtin_amdgcn_rcpf(denom);
    const V<float> pt = vfma(t, ray.d, ray.o);
    const float alpha = dot(pt, mk(q.AB[0], q.AB[2], q.AB[4])) - q.AB[6];
    const float beta = dot(pt, mk(q.AB[1], q.AB[3], q.AB[5])) - q.AB[7];
    const float lo = fminf(alpha, beta);
    const bool quad = PRIMS == 1 ? false : (PRIMS == 2 ? true : kind == PRIM_QUAD);
    const bool inside = quad ? (lo >= 0.0f) & (alpha <= 1.0f) & (beta <= 1.0f) : (lo > 0.0f) & (alpha + beta < 1.0f);
    const float key = tie_key<TIE>(t, tie_factor(q.meta >> WCLASS_SHIFT));  // coplanar-tie key
    const bool ok = (fabsf(denom) >= 1e-8f) & (t >= 0.001f) & (key <= t_best) & inside;
    return ok ? key : -1.0f;
}

template <typename T>
__device__ __forceinline__ T load16(const T* p) {  // whole record, 16-byte loads issued together
    T r;
    const uint4* s = reinterpret_cast<const uint4*>(p);
    uint4* d = reinterpret_cast<uint4*>(&r);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 16); ++k) d[k] = s[k];
    return r;
}

// Traversal state of one lane's world-BVH query (kept in registers; the stack in LDS).
struct WbvhTrav {
    int32_t node;
    int32_t leaf;  // parked leaf ref (< 0), WBVH_NO_LEAF when none
    uint32_t sp;
    float t_best;
    int32_t best;
    float ix, iy, iz, ox, oy, oz;  // 1/d and o/d: slab t = bound * inv - o * inv
    __device__ __forceinline__ bool busy() const { return node != WBVH_DONE || leaf != WBVH_NO_LEAF; }
};

// 1/d clamped to +-1e20 (d = +-0 would give +-inf, and inf * 0 = NaN in the 4-wide node
// decode): a ray parallel to a slab then gets huge finite slab ends of the right signs.
__device__ __forceinline__ float wbvh_inv(float d) {
    const float r = __builtin_amdgcn_rcpf(d);
    return __builtin_copysignf(fminf(fabsf(r), 1e20f), r);
}
__device__ __forceinline__ void wbvh_begin(WbvhTrav& ts, int32_t root, const Ray<float>& ray) {
    ts.ix = wbvh_inv(ray.d.x);
    ts.iy = wbvh_inv(ray.d.y);
    ts.iz = wbvh_inv(ray.d.z);
    ts.ox = ray.o.x * ts.ix;
    ts.oy = ray.o.y * ts.iy;
    ts.oz = ray.o.z * ts.iz;
    ts.node = root;
    ts.leaf = WBVH_NO_LEAF;
    ts.sp = 0;
    ts.t_best = INFINITY;
    ts.best = -1;
}

// PROF builds (diagnostics only): traversal event counters in the wave's LDS profile row
// (slots PROF_*), added by the first active lane.
constexpr int NPROF = 16;
enum : int { PROF_VISIT_TRIPS = 8, PROF_VISIT_LANES = 9, PROF_LEAF_TRIPS = 10, PROF_LEAF_LANES = 11,
             PROF_ROUNDS = 12, PROF_ROUND_LANES = 13 };
__device__ __forceinline__ void prof_event(unsigned long long* pc, int trips, int lanes) {
    if (!pc) return;
    const uint64_t m = __ballot(true);
    if ((uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x) {
        atomicAdd(pc + trips, 1ull);
        atomicAdd(pc + lanes, (unsigned long long)__popcll(m));
    }
}

// Test the primitives of leaf `ref` (world_prim_t, closest hit so far in ts).
template <typename R, bool FLAT, bool TIE>
__device__ __forceinline__ void wbvh_leaf_t(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray, int32_t ref,
                                            unsigned long long* pc = nullptr) {
    const uint32_t v = ~(uint32_t)ref, first = v >> 3, cnt = (v & 7u) + 1u;
    for (uint32_t k = 0; k < cnt; ++k) {
        prof_event(pc, PROF_LEAF_TRIPS, PROF_LEAF_LANES);
        const DPrimWorld<float> q = load16(sc.wprims + first + k);
        const float t = world_prim_t<FLAT, TIE>(q, ray, ts.t_best);
        const bool ok = t >= 0.0f;
        ts.t_best = ok ? t : ts.t_best;
        ts.best = ok ? (int32_t)(first + k) : ts.best;
    }
}
// t_best holds the closest key; coplanar-tie keys only in scenes that have such pairs
template <typename R, bool FLAT>
__device__ __forceinline__ void wbvh_leaf(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray, int32_t ref,
                                          unsigned long long* pc = nullptr) {
    if (sc.wflags & WFLAG_COPLANAR) wbvh_leaf_t<R, FLAT, true>(ts, sc, ray, ref, pc);
    else wbvh_leaf_t<R, FLAT, false>(ts, sc, ray, ref, pc);
}

// Traversal stacks.  f32 kernels: LDS, entry k of this lane at stack[k * BLOCK].  The exact
// kernel's world-BVH mode: the compact tree's 16-bit refs in LDS as well (ExactSig LSTACK, the
// default since round 3: 3 waves per SIMD, no scratch traffic), or a private array (scratch:
// NRT_EXACT_LSTACK=0; an 8-entry LDS part paid for by not staging the scene measured slower on
// every f64 config: C5 245 -> 323 ms, C4 400 -> 473 ms, C3 5.0 -> 6.0 ms).
struct PrivStack {
    int32_t e[WBVH_STACK + 1];
};
// the compact tree's raw 16-bit refs (exact kernel, ExactSig width WBVH_COMPACT): half the
// scratch bytes per push
struct PrivStack16 {
    uint16_t e[WBVH_STACK + 1];
};
__device__ __forceinline__ void stk_write(int32_t* s, uint32_t k, int32_t v) { s[k * BLOCK] = v; }
__device__ __forceinline__ int32_t stk_read(int32_t* s, uint32_t k) { return s[k * BLOCK]; }
// compact 4-wide tree (BvhSig width WBVH_COMPACT): the raw 16-bit child refs
__device__ __forceinline__ void stk_write(uint16_t* s, uint32_t k, int32_t v) { s[k * BLOCK] = (uint16_t)v; }
__device__ __forceinline__ int32_t stk_read(uint16_t* s, uint32_t k) { return (int32_t)s[k * BLOCK]; }
__device__ __forceinline__ void stk_write(PrivStack& s, uint32_t k, int32_t v) { s.e[k] = v; }
__device__ __forceinline__ int32_t stk_read(PrivStack& s, uint32_t k) { return s.e[k]; }
__device__ __forceinline__ void stk_write(PrivStack16& s, uint32_t k, int32_t v) { s.e[k] = (uint16_t)v; }
__device__ __forceinline__ int32_t stk_read(PrivStack16& s, uint32_t k) { return (int32_t)s.e[k]; }
template <class STK>
__device__ __forceinline__ int32_t wbvh_pop(WbvhTrav& ts, STK& stack) {
    return ts.sp ? stk_read(stack, --ts.sp) : WBVH_DONE;
}

// Binary node visit: both child boxes, nearer hit child next, the other pushed.
template <typename R, class STK>
__device__ __forceinline__ void wbvh2_visit(WbvhTrav& t, const DSceneView<R>& sc, STK& stack) {
    const DBvhNode nd = load16(sc.wbvh + t.node);
    const float a0x = nd.lo0[0] * t.ix - t.ox, b0x = nd.hi0[0] * t.ix - t.ox;
    const float a0y = nd.lo0[1] * t.iy - t.oy, b0y = nd.hi0[1] * t.iy - t.oy;
    const float a0z = nd.lo0[2] * t.iz - t.oz, b0z = nd.hi0[2] * t.iz - t.oz;
    const float a1x = nd.lo1[0] * t.ix - t.ox, b1x = nd.hi1[0] * t.ix - t.ox;
    const float a1y = nd.lo1[1] * t.iy - t.oy, b1y = nd.hi1[1] * t.iy - t.oy;
    const float a1z = nd.lo1[2] * t.iz - t.oz, b1z = nd.hi1[2] * t.iz - t.oz;
    const float tn0 = fmaxf(fmaxf(fmaxf(fminf(a0x, b0x), fminf(a0y, b0y)), fminf(a0z, b0z)), 0.0f);
    const float tf0 = fminf(fminf(fminf(fmaxf(a0x, b0x), fmaxf(a0y, b0y)), fmaxf(a0z, b0z)), t.t_best);
    const float tn1 = fmaxf(fmaxf(fmaxf(fminf(a1x, b1x), fminf(a1y, b1y)), fminf(a1z, b1z)), 0.0f);
    const float tf1 = fminf(fminf(fminf(fmaxf(a1x, b1x), fmaxf(a1y, b1y)), fmaxf(a1z, b1z)), t.t_best);
    const bool h0 = tn0 <= tf0, h1 = tn1 <= tf1;
    if (h0 && h1) {
        const bool near0 = tn0 <= tn1;
        stk_write(stack, t.sp++, near0 ? nd.c1 : nd.c0);
        t.node = near0 ? nd.c0 : nd.c1;
    } else if (h0 || h1) {
        t.node = h0 ? nd.c0 : nd.c1;
    } else {
        t.node = wbvh_pop(t, stack);
    }
}

// 4-wide node visit (DBvh4Node, quantized boxes): hit children sorted by entry
// distance (5-comparator network), the nearest next, the rest pushed farthest-first.
__device__ __forceinline__ void wbvh_cswap(float& ta, int32_t& ca, float& tb, int32_t& cb) {
    const bool sw = tb < ta;
    const float t0 = ta;
    const int32_t c0 = ca;
    ta = sw ? tb : ta;
    ca = sw ? cb : ca;
    tb = sw ? t0 : tb;
    cb = sw ? c0 : cb;
}
template <typename R, class STK>
__device__ __forceinline__ void wbvh4_visit(WbvhTrav& t, const DSceneView<R>& sc, STK& stack) {
    const DBvh4Node nd = load16(sc.wbvh4 + t.node);
    // plane t = (org + q * step - o) / d = q * (step / d) + (org / d - o / d)
    const float Ax = __uint_as_float(wbvh_step_bits(nd.exps, 0)) * t.ix, Bx = nd.org[0] * t.ix - t.ox;
    const float Ay = __uint_as_float(wbvh_step_bits(nd.exps, 1)) * t.iy, By = nd.org[1] * t.iy - t.oy;
    const float Az = __uint_as_float(wbvh_step_bits(nd.exps, 2)) * t.iz, Bz = nd.org[2] * t.iz - t.oz;
    // The ray's direction signs pick each axis's near and far plane bytes for all four
    // children at once (1/d is finite, wbvh_begin), so a child's slab needs no min/max, and an
    // empty slot (qlo 255, qhi 0 on every axis) comes out with near > far: a miss.
    const bool px = t.ix >= 0.0f, py = t.iy >= 0.0f, pz = t.iz >= 0.0f;
    const uint32_t nqx = px ? nd.qlo[0] : nd.qhi[0], fqx = px ? nd.qhi[0] : nd.qlo[0];
    const uint32_t nqy = py ? nd.qlo[1] : nd.qhi[1], fqy = py ? nd.qhi[1] : nd.qlo[1];
    const uint32_t nqz = pz ? nd.qlo[2] : nd.qhi[2], fqz = pz ? nd.qhi[2] : nd.qlo[2];
    auto child_t = [&](int k) {  // entry distance of child k, +inf if missed or empty
        auto q = [&](uint32_t w) { return (float)((w >> (8 * k)) & 0xFFu); };
        const float nx = q(nqx) * Ax + Bx, fx = q(fqx) * Ax + Bx;
        const float ny = q(nqy) * Ay + By, fy = q(fqy) * Ay + By;
        const float nz = q(nqz) * Az + Bz, fz = q(fqz) * Az + Bz;
        const float n = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.0f));
        const float f = fminf(fminf(fx, fy), fminf(fz, t.t_best));
        return n <= f ? n : INFINITY;
    };
    float t0 = child_t(0), t1 = child_t(1), t2 = child_t(2), t3 = child_t(3);
    int32_t c0 = nd.child[0], c1 = nd.child[1], c2 = nd.child[2], c3 = nd.child[3];
#if NRT_WBVH_SORT
    wbvh_cswap(t0, c0, t1, c1);
    wbvh_cswap(t2, c2, t3, c3);
    wbvh_cswap(t0, c0, t2, c2);
    wbvh_cswap(t1, c1, t3, c3);
    wbvh_cswap(t1, c1, t2, c2);
#else
    // nearest hit child first; the others keep their slots (pushed 3, 2, 1: child order)
    wbvh_cswap(t0, c0, t1, c1);
    wbvh_cswap(t0, c0, t2, c2);
    wbvh_cswap(t0, c0, t3, c3);
#endif
    // branch-free pushes: every slot is written at sp, sp advances past the hit ones (the
    // stack has one spare entry above the tree's bound for the writes that do not count)
    stk_write(stack, t.sp, c3);
    t.sp += t3 != INFINITY ? 1u : 0u;
    stk_write(stack, t.sp, c2);
    t.sp += t2 != INFINITY ? 1u : 0u;
    stk_write(stack, t.sp, c1);
    t.sp += t1 != INFINITY ? 1u : 0u;
    t.node = t0 != INFINITY ? c0 : wbvh_pop(t, stack);
}

#ifndef NRT_PK_SLAB
#define NRT_PK_SLAB 0  // (near, far) pairs as v_pk_fma_f32: C4 40.2 -> 41.1 ms, off
#endif
#ifndef NRT_NODE_MIX
#define NRT_NODE_MIX 0
#endif
// Compact 4-wide visit (DBvh4cNode: the same boxes, 16-bit child refs; three loads instead of
// four).  The stack holds the raw 16-bit refs; a ref becomes the traversal's 32-bit form
// (inner index, or ~(first << 3 | count - 1) for a leaf) only when it is taken (wbvh4c_ref).
__device__ __forceinline__ int32_t wbvh4c_ref(uint32_t r) {
    return (r & WBVH4C_LEAF) ? ~(int32_t)(((r & 0x7FFCu) << 1) | (r & 3u)) : (int32_t)r;
}
template <class STK>
__device__ __forceinline__ int32_t wbvh4c_pop(WbvhTrav& ts, STK& stack) {
    return ts.sp ? wbvh4c_ref((uint32_t)stk_read(stack, --ts.sp)) : WBVH_DONE;
}
template <class STK>
__device__ __forceinline__ void wbvh4c_visit_nd(WbvhTrav& t, const DBvh4cNode& nd, STK& stack);
template <typename R, class STK>
__device__ __forceinline__ void wbvh4c_visit(WbvhTrav& t, const DSceneView<R>& sc, STK& stack) {
    // (an LDS copy of the tree's top levels, breadth-first numbered, measured C4 40.2 -> 43.8 ms)
    const DBvh4cNode nd = load16(sc.wbvh4c + t.node);
    wbvh4c_visit_nd(t, nd, stack);
}
template <class STK>
__device__ __forceinline__ void wbvh4c_visit_nd(WbvhTrav& t, const DBvh4cNode& nd, STK& stack) {
#if NRT_WALK_CONTRACT
    // FMAs in the exact kernel's culling walk too (its TU compiles without contraction): the walk
    // only culls, and the boxes' outward rounding and padding cover one rounding as well as two
    // (C4 f64 178 -> 169 ms, C5 f64 196 -> 191 ms, frames identical)
#pragma clang fp contract(on)
#endif
    const float Ax = __uint_as_float(wbvh_step_bits(nd.exps, 0)) * t.ix, Bx = nd.org[0] * t.ix - t.ox;
    const float Ay = __uint_as_float(wbvh_step_bits(nd.exps, 1)) * t.iy, By = nd.org[1] * t.iy - t.oy;
    const float Az = __uint_as_float(wbvh_step_bits(nd.exps, 2)) * t.iz, Bz = nd.org[2] * t.iz - t.oz;
    const bool px = t.ix >= 0.0f, py = t.iy >= 0.0f, pz = t.iz >= 0.0f;
    const uint32_t nqx = px ? nd.qlo[0] : nd.qhi[0], fqx = px ? nd.qhi[0] : nd.qlo[0];
    const uint32_t nqy = py ? nd.qlo[1] : nd.qhi[1], fqy = py ? nd.qhi[1] : nd.qlo[1];
    const uint32_t nqz = pz ? nd.qlo[2] : nd.qhi[2], fqz = pz ? nd.qhi[2] : nd.qlo[2];
#if NRT_NODE_MIX
    // Plane bytes without byte -> float conversions (quarter-rate v_cvt_f32_ubyte*): one v_perm_b32
    // turns two bytes q of a word into the f16 pair 1024 + q (0x64 high bytes), and v_fma_mix_f32
    // reads either half as an f16 operand: (1024 + q) * A + (B - 1024 A).  The folded offset
    // rounds B - 1024 A to f32, an error of ~2^-14 of a quantization step in t (the decode's own
    // f32 rounding is of that order).
    // (gfx9 VOP3: one SGPR or literal per instruction, so the 0x64 bytes sit in a VGPR and the
    // selector in an SGPR)
    const uint32_t k64 = 0x64646464u, sel01 = 0x04010400u, sel23 = 0x04030402u;
    const float Cx = __builtin_fmaf(-1024.0f, Ax, Bx), Cy = __builtin_fmaf(-1024.0f, Ay, By),
                Cz = __builtin_fmaf(-1024.0f, Az, Bz);
    auto pairs = [&](uint32_t w, uint32_t sel) {
        uint32_t r;
        asm("v_perm_b32 %0, %1, %2, %3" : "=v"(r) : "v"(k64), "v"(w), "s"(sel));
        return r;
    };
    auto mix_lo = [](uint32_t h, float a, float c) {
        float r;
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(a), "v"(c));
        return r;
    };
    auto mix_hi = [](uint32_t h, float a, float c) {
        float r;
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(h), "v"(a), "v"(c));
        return r;
    };
    float tc[4];
#pragma unroll
    for (int hp = 0; hp < 2; ++hp) {  // children (0, 1), then (2, 3)
        const uint32_t sel = hp ? sel23 : sel01;
        const uint32_t nx = pairs(nqx, sel), fx = pairs(fqx, sel), ny = pairs(nqy, sel), fy = pairs(fqy, sel),
                       nz = pairs(nqz, sel), fz = pairs(fqz, sel);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            auto m = [&](uint32_t h, float a, float c) { return j ? mix_hi(h, a, c) : mix_lo(h, a, c); };
            const float n = fmaxf(fmaxf(m(nx, Ax, Cx), m(ny, Ay, Cy)), fmaxf(m(nz, Az, Cz), 0.0f));
            const float f = fminf(fminf(m(fx, Ax, Cx), m(fy, Ay, Cy)), fminf(m(fz, Az, Cz), t.t_best));
            tc[2 * hp + j] = n <= f ? n : INFINITY;
        }
    }
    float t0 = tc[0], t1 = tc[1], t2 = tc[2], t3 = tc[3];
#else
    auto child_t = [&](int k) {  // entry distance of child k, +inf if missed or empty
        auto q = [&](uint32_t w) { return (float)((w >> (8 * k)) & 0xFFu); };
#if NRT_PK_SLAB
        const f32x2 x = f32x2{q(nqx), q(fqx)} * Ax + Bx;  // (near, far) plane pairs: v_pk_fma_f32
        const f32x2 y = f32x2{q(nqy), q(fqy)} * Ay + By;
        const f32x2 z = f32x2{q(nqz), q(fqz)} * Az + Bz;
        const float nx = x.x, fx = x.y, ny = y.x, fy = y.y, nz = z.x, fz = z.y;
#else
        const float nx = q(nqx) * Ax + Bx, fx = q(fqx) * Ax + Bx;
        const float ny = q(nqy) * Ay + By, fy = q(fqy) * Ay + By;
        const float nz = q(nqz) * Az + Bz, fz = q(fqz) * Az + Bz;
#endif
        const float n = fmaxf(fmaxf(nx, ny), fmaxf(nz, 0.0f));
        const float f = fminf(fminf(fx, fy), fminf(fz, t.t_best));
        return n <= f ? n : INFINITY;
    };
    float t0 = child_t(0), t1 = child_t(1), t2 = child_t(2), t3 = child_t(3);
#endif
    const uint32_t c01 = (uint32_t)nd.child[0] | ((uint32_t)nd.child[1] << 16);
    const uint32_t c23 = (uint32_t)nd.child[2] | ((uint32_t)nd.child[3] << 16);
    int32_t c0 = (int32_t)(c01 & 0xFFFFu), c1 = (int32_t)(c01 >> 16), c2 = (int32_t)(c23 & 0xFFFFu),
            c3 = (int32_t)(c23 >> 16);
    wbvh_cswap(t0, c0, t1, c1);  // nearest hit child first; the others keep their slots
    wbvh_cswap(t0, c0, t2, c2);
    wbvh_cswap(t0, c0, t3, c3);
    stk_write(stack, t.sp, c3);
    t.sp += t3 != INFINITY ? 1u : 0u;
    stk_write(stack, t.sp, c2);
    t.sp += t2 != INFINITY ? 1u : 0u;
    stk_write(stack, t.sp, c1);
    t.sp += t1 != INFINITY ? 1u : 0u;
    t.node = t0 != INFINITY ? wbvh4c_ref((uint32_t)c0) : wbvh4c_pop(t, stack);
}
// Visit / pop of a tree of width W (2 binary, 4 four-wide, WBVH_COMPACT the compact four-wide)
template <int W, typename R, class STK>
__device__ __forceinline__ void wbvh_visit_w(WbvhTrav& t, const DSceneView<R>& sc, STK& stack) {
    if constexpr (W == WBVH_COMPACT) wbvh4c_visit<R>(t, sc, stack);
    else if constexpr (W == 4) wbvh4_visit(t, sc, stack);
    else wbvh2_visit(t, sc, stack);
}
template <int W, class STK>
__device__ __forceinline__ int32_t wbvh_pop_w(WbvhTrav& ts, STK& stack) {
    if constexpr (W == WBVH_COMPACT) return wbvh4c_pop(ts, stack);
    else return wbvh_pop(ts, stack);
}

// One round: descend through inner nodes until the lane holds a leaf (or is
// done), lanes waiting for the wave's slowest; then test the leaf.  With
// NRT_SPECULATIVE (Aila & Laine) a lane that meets a leaf parks it and keeps
// descending until every lane of the wave has a leaf.
template <typename R, int W, bool FLAT, class STKP>
__device__ __forceinline__ void wbvh_round_impl(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray,
                                                STKP stack, unsigned long long* pc) {
#if NRT_SPECULATIVE
    while (true) {
        if (ts.node < 0 && ts.node != WBVH_DONE && ts.leaf == WBVH_NO_LEAF) {  // park a leaf
            ts.leaf = ts.node;
            ts.node = wbvh_pop_w<W>(ts, stack);
        }
        const bool inner = ts.node >= 0;
        if (!__any(inner)) break;                                         // nobody can descend
        if (__all(ts.leaf != WBVH_NO_LEAF || ts.node == WBVH_DONE)) break;  // every lane has a leaf (or is done)
        if (inner) {
            prof_event(pc, PROF_VISIT_TRIPS, PROF_VISIT_LANES);
            wbvh_visit_w<W>(ts, sc, stack);
        }
    }
    if (ts.leaf != WBVH_NO_LEAF) {
        wbvh_leaf<R, FLAT>(ts, sc, ray, ts.leaf, pc);
        ts.leaf = WBVH_NO_LEAF;
    }
#else
    while (ts.node >= 0) wbvh_visit_w<W>(ts, sc, stack);
    if (ts.node == WBVH_DONE) return;
    wbvh_leaf<R, FLAT>(ts, sc, ray, ts.node);
    ts.node = wbvh_pop_w<W>(ts, stack);
#endif
}

// "If-if" trip (NRT_WBVH_IFIF, KF_FLAT): every busy lane does exactly one unit of work per trip,
// one primitive of its current leaf or, without a leaf, one node visit; a leaf that a visit
// or a pop turns up becomes the lane's leaf cursor at once (the leaf ref, advanced in place:
// first + 1, count - 1).  Lanes never wait for the wave to finish a phase, so long and
// short traversals, and leaves of different sizes, interleave across trips.
template <typename R, int W, bool FLAT, bool TIE, int PRIMS = 0, class STKP>
__device__ __forceinline__ void wbvh_trip_impl(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray,
                                               STKP stack, unsigned long long* pc) {
    const bool leaf_now = ts.leaf != WBVH_NO_LEAF;
    if (leaf_now) {  // (two primitives per trip measured C4 -6 %, round 2; 41.6 ms against 40.2, round 3)
        prof_event(pc, PROF_LEAF_TRIPS, PROF_LEAF_LANES);
        const uint32_t v = ~(uint32_t)ts.leaf, first = v >> 3, more = v & 7u;
        const DPrimWorld<float> q = load16(sc.wprims + first);
        const float t = world_prim_t<FLAT, TIE, PRIMS>(q, ray, ts.t_best);
        const bool ok = t >= 0.0f;
        ts.t_best = ok ? t : ts.t_best;
        ts.best = ok ? (int32_t)first : ts.best;
        ts.leaf = more ? ts.leaf - 7 : WBVH_NO_LEAF;  // ~((first + 1) << 3 | (more - 1)) = ~v - 7
    }
    // NRT_WBVH_UNIFIED: a lane holding both a leaf cursor and a node does both in one trip (a trip
    // runs both branches whenever the wave's lanes are mixed anyway); otherwise one or the other
    if ((NRT_WBVH_UNIFIED || !leaf_now) && ts.node >= 0) {
        prof_event(pc, PROF_VISIT_TRIPS, PROF_VISIT_LANES);
        wbvh_visit_w<W>(ts, sc, stack);
    }
    if (ts.leaf == WBVH_NO_LEAF && ts.node < 0 && ts.node != WBVH_DONE) {  // a leaf turned up: its cursor
        ts.leaf = ts.node;
        ts.node = wbvh_pop_w<W>(ts, stack);
    }
}
template <typename R, int W, bool FLAT, class STKP>
__device__ __forceinline__ void wbvh_trip(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray,
                                          STKP stack, unsigned long long* pc) {
    if (sc.wflags & WFLAG_COPLANAR) wbvh_trip_impl<R, W, FLAT, true>(ts, sc, ray, stack, pc);
    else wbvh_trip_impl<R, W, FLAT, false>(ts, sc, ray, stack, pc);
}

template <typename R, bool FLAT = false, class STKP>
__device__ __forceinline__ void wbvh_round(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray,
                                           STKP stack, unsigned long long* pc) {
    wbvh_round_impl<R, 2, FLAT>(ts, sc, ray, stack, pc);
}
template <typename R, bool FLAT = false, class STKP>
__device__ __forceinline__ void wbvh4_round(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray,
                                            STKP stack, unsigned long long* pc) {
    wbvh_round_impl<R, 4, FLAT>(ts, sc, ray, stack, pc);
}

// Root and round of the tree the scene carries (4-wide when its stack bound fits).
template <typename R>
__device__ __forceinline__ int32_t wbvh_root(const DSceneView<R>& sc) {
    return sc.wbvh4 ? sc.wbvh4_root : sc.wbvh_root;
}
template <typename R, bool FLAT = false, class SIG = NoSig, class STKP>
__device__ __forceinline__ void wbvh_step(WbvhTrav& ts, const DSceneView<R>& sc, const Ray<float>& ray, STKP stack,
                                          unsigned long long* pc = nullptr) {
    if constexpr (SIG::bvh != 0) {  // a scene-specialised kernel (jit.hip)
        if constexpr ((FLAT || NRT_WBVH_IFIF_SPHERES) && NRT_WBVH_IFIF)
            wbvh_trip_impl<R, SIG::bvh, FLAT, SIG::tie, SIG::prims>(ts, sc, ray, stack, pc);
        else wbvh_round_impl<R, SIG::bvh, FLAT>(ts, sc, ray, stack, pc);
        return;
    }
    if constexpr ((FLAT || NRT_WBVH_IFIF_SPHERES) && NRT_WBVH_IFIF) {
        if (sc.wbvh4) wbvh_trip<R, 4, FLAT>(ts, sc, ray, stack, pc);
        else wbvh_trip<R, 2, FLAT>(ts, sc, ray, stack, pc);
    } else {
        if (sc.wbvh4) wbvh4_round<R, FLAT>(ts, sc, ray, stack, pc);
        else wbvh_round<R, FLAT>(ts, sc, ray, stack, pc);
    }
}

template <typename R, int MAXD, bool FLAT = false, class SIG = NoSig, class STKP>
__device__ __forceinline__ bool trace_world_bvh(const DSceneView<R>& sc, const Ray<R>& ray, HitMin<R, MAXD>& hm,
                                                STKP stack) {
    static_assert(sizeof(R) == 4, "world-BVH mode is an f32-kernel mode");
    WbvhTrav ts;
    wbvh_begin(ts, wbvh_root(sc), ray);
    while (ts.busy()) wbvh_step<R, FLAT, SIG>(ts, sc, ray, stack);
    hm.t = ts.t_best;
    hm.prim = (uint32_t)ts.best;
    hm.depth = 0;
    return ts.best >= 0;
}

// Closest hit over the flattened scene ("while-while": lanes first run through
// inner nodes until each holds a leaf, then leaves are processed together).
// Candidates arrive in the reference's depth-first, left-before-right order,
// so `t <= t_best` (the later candidate wins a tie) reproduces BVH::hit's
// `if l.t < r.t {l} else {r}` (object.rs:109-115).  Only (t, prim, instance
// path) is kept; the winner's record is rebuilt afterwards (make_record).
//
// `all` (RenderParams::exact_all, small scenes): no box is tested.  BVH::hit tests every
// primitive whose boxes the ray hits, with the same range on both sides, and keeps the
// smaller t, ties to the right (object.rs:89-121); boxes are padded (aabb.rs:14-40), so a
// primitive the ray hits lies in boxes the ray hits, and the closest hit over ALL primitives
// in depth-first order with `t <= t_best` is the reference's.  Every lane then walks the
// same node sequence: uniform control flow, broadcast reads.
template <typename R, int MAXD, bool EXACT>
__device__ __forceinline__ bool trace_bvh(const DSceneView<R>& sc, const Ray<R>& wray, HitMin<R, MAXD>& hm,
                                          bool all = false) {
    R t_best = R(INFINITY);
    bool found = false;
    int32_t node = sc.root;
    int depth = 0;
    // instance stack; MAXD == 1 keeps it in scalars (no scratch)
    int32_t ret[MAXD];
    uint32_t inst_id[MAXD];
    Ray<R> saved[MAXD];
    int32_t ret0 = NODE_END;
    uint32_t inst0 = 0;
    Ray<R> ray = wray;
    while (true) {
        uint32_t meta = 0;
        int32_t skip = NODE_END;
        while (node >= 0) {
            const DNode<R> n = load_node(sc.nodes + node);  // one fetch: box + links
            meta = n.meta;
            skip = n.skip;
            if ((meta & 3u) != NODE_INNER) break;
            node = (all || box_hit<R, EXACT>(n.bmin, n.bmax, ray, t_best)) ? node + 1 : skip;
        }
        if (node < 0) {
            if (depth == 0) break;
            --depth;
            if constexpr (MAXD == 1) {
                node = ret0;
                ray = wray;
            } else {
                node = ret[depth];
                ray = depth == 0 ? wray : saved[depth];
            }
            continue;
        }
        const uint32_t kind = meta & 3u;
        auto test_prim = [&](uint32_t pid) {
            R t;
            if constexpr (EXACT) {
                const DPrim<R>& pr = sc.prims[pid];
                if (pr.kind == PRIM_SPHERE) {
                    t = sphere_t(pr, ray);
                } else {
                    R alpha, beta;
                    V<R> point;
                    t = plane_t(pr, ray, alpha, beta, point);
                }
            } else {
                t = fast_prim_t(sc.fprims[pid], ray, t_best);
            }
            if (t >= R(0) && t <= t_best) {
                t_best = t;
                hm.prim = pid;
                hm.depth = depth;
                if constexpr (MAXD == 1) {
                    hm.inst[0] = inst0;
                } else {
#pragma unroll
                    for (int l = 0; l < MAXD; ++l) hm.inst[l] = inst_id[l];
                }
                found = true;
            }
        };
        if (kind == NODE_PRIM) {
            test_prim(meta >> 2);
            node = skip;
        } else if (!EXACT && kind == NODE_LIST) {
            // collapsed prim-only subtree: its box, then its prims in depth-first order
            const DNode<R>& n = sc.nodes[node];
            if (box_hit<R, EXACT>(n.bmin, n.bmax, ray, t_best)) {
                const uint32_t first = meta >> 8, cnt = ((meta >> 2) & 63u) + 1u;
                for (uint32_t k = 0; k < cnt; ++k) test_prim(first + k);
            }
            node = skip;
        } else {
            const uint32_t idx = meta >> 2;
            const DInstance inst = sc.instances[idx];
            if constexpr (MAXD == 1) {
                ret0 = skip;
                inst0 = idx;
            } else {
                ret[depth] = skip;
                inst_id[depth] = idx;
                saved[depth] = ray;
            }
            ++depth;
            if constexpr (EXACT) {
                xform_in<R, EXACT>(sc, inst, ray);
                node = inst.root;
            } else {
                enter_fast(sc.inst_fast[idx], ray);
                node = inst.root_fast;
            }
        }
    }
    hm.t = t_best;
    return found;
}

// Stackless culling walk of the exact world mode (DThreadNode: the binary tree threaded per ray
// octant, nearer child first): `leaf(ref)` for every reached leaf, which may lower `cut`, the
// distance beyond which boxes are skipped.  The octant comes from the signs of the clamped 1/d,
// the same ones that pick each box's near planes.
template <typename R, class LEAF>
__device__ __forceinline__ void xthread_walk(const DSceneView<R>& sc, const Ray<float>& fr, float& cut, LEAF&& leaf) {
    const float ix = wbvh_inv(fr.d.x), iy = wbvh_inv(fr.d.y), iz = wbvh_inv(fr.d.z);
    const float ox = fr.o.x * ix, oy = fr.o.y * iy, oz = fr.o.z * iz;
    const uint32_t oct = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
    const int32_t n = (int32_t)sc.n_xthread;
    const DThreadNode* base = sc.xthread + (size_t)oct * (size_t)n;
    int32_t i = 0;
    while (i < n) {
        const DThreadNode nd = load16(base + i);
        const float tn = fmaxf(fmaxf(fmaxf(nd.nearp[0] * ix - ox, nd.nearp[1] * iy - oy), nd.nearp[2] * iz - oz), 0.0f);
        const float tf = fminf(fminf(fminf(nd.farp[0] * ix - ox, nd.farp[1] * iy - oy), nd.farp[2] * iz - oz), cut);
        const bool hit = tn <= tf;
        if (hit && nd.leaf != 0) leaf(nd.leaf);
        i = (hit && nd.leaf == 0) ? i + 1 : nd.skip;
    }
}

// Exact kernel, world-BVH mode (RenderParams::exact_wbvh; large scenes whose instances do
// not nest, e.g. the teapot): the f32 world BVH (binned SAH, 4-wide) only culls, and every
// primitive in a reached leaf gets the reference's own test in f64 in its object space
// (xform_in, then Sphere::hit / Plane::hit, sphere.rs:105-163, plane.rs:141-174).  The winner
// is the smallest exact t, ties to the higher depth-first rank (object.rs:109-115), so the
// visiting order does not matter.  The culling is conservative: the f32 boxes are rounded
// outward and padded (1e-6 of the scene extent, far above the f32 slab error for origins
// inside the scene), and boxes are cut at the best exact t raised by 2^-20.  The stack: by default
// the compact tree's 16-bit refs in LDS at 3 waves per SIMD (ExactSig LSTACK, NRT_EXACT_LSTACK),
// else a private array (PrivStack / PrivStack16, scratch).
// W: the culling walk fixed at compile time (ExactSig): XTHREAD_W the threaded tree, 4 / 2 the
// stack walk of the 4-wide / binary tree; 0: chosen at run time (threaded when `thread`).
constexpr int XTHREAD_W = 1;
template <typename R, int MAXD, int W = 0, bool PLANES = false, bool LSTACK = false>  // PLANES: no spheres
__device__ __forceinline__ bool trace_exact_wbvh(const DSceneView<R>& sc, const Ray<R>& wray, HitMin<R, MAXD>& hm,
                                                 bool thread = false, uint16_t* lstk = nullptr) {
    static_assert(sizeof(R) == 8, "exact world-BVH mode is an f64-kernel mode");
    Ray<float> fr;
    fr.o = mk((float)wray.o.x, (float)wray.o.y, (float)wray.o.z);
    fr.d = mk((float)wray.d.x, (float)wray.d.y, (float)wray.d.z);
    R best_t = R(INFINITY);
    uint32_t best_rank = 0;
    int32_t best_prim = -1, best_inst = -1, cur_inst = -2;
    Ray<R> oray = wray;
    auto leaf_tests = [&](int32_t ref, float& cut) {
        const uint32_t v = ~(uint32_t)ref, first = v >> 3, cnt = (v & 7u) + 1u;
        for (uint32_t k = 0; k < cnt; ++k) {
            const DExactRef rf = sc.wexact[first + k];
            if (rf.inst != cur_inst) {  // the primitive's object-space ray (exact chain)
                oray = wray;
                if (rf.inst >= 0) xform_in<R, true, false>(sc, sc.instances[rf.inst], oray);
                cur_inst = rf.inst;
            }
            const DPrim<R>& pr = sc.prims[rf.prim];
            R t;
            if (!PLANES && pr.kind == PRIM_SPHERE) {
                t = sphere_t(pr, oray);
            } else {
                R alpha, beta;
                V<R> point;
                t = plane_t(pr, oray, alpha, beta, point);
            }
            if (t >= R(0) && (t < best_t || (t == best_t && rf.rank > best_rank))) {
                best_t = t;
                best_rank = rf.rank;
                best_prim = (int32_t)rf.prim;
                best_inst = rf.inst;
                cut = (float)best_t * (1.0f + 0x1p-20f);
            }
        }
    };
    if (W == XTHREAD_W || (W == 0 && thread)) {
        float cut = INFINITY;
        xthread_walk(sc, fr, cut, [&](int32_t ref) { leaf_tests(ref, cut); });
        hm.t = best_t;
        hm.prim = (uint32_t)best_prim;
        hm.depth = best_inst >= 0 ? 1 : 0;
        hm.inst[0] = (uint32_t)best_inst;
        return best_prim >= 0;
    }
    WbvhTrav ts;
    wbvh_begin(ts, wbvh_root(sc), fr);
    if constexpr (W == WBVH_COMPACT) {
        auto walk = [&](auto& stk) {
            while (true) {
                while (ts.node >= 0) wbvh4c_visit<R>(ts, sc, stk);
                if (ts.node == WBVH_DONE) break;
                leaf_tests(ts.node, ts.t_best);
                ts.node = wbvh4c_pop(ts, stk);
            }
        };
        if constexpr (LSTACK) {
            walk(lstk);
        } else {
            PrivStack16 stk;
            walk(stk);
        }
    } else {
        PrivStack stk;
        while (true) {
            while (ts.node >= 0) {
                if (W == 4 || (W == 0 && sc.wbvh4)) wbvh4_visit<R>(ts, sc, stk);
                else wbvh2_visit<R>(ts, sc, stk);
            }
            if (ts.node == WBVH_DONE) break;
            leaf_tests(ts.node, ts.t_best);
            ts.node = wbvh_pop(ts, stk);
        }
    }
    hm.t = best_t;
    hm.prim = (uint32_t)best_prim;
    hm.depth = best_inst >= 0 ? 1 : 0;
    hm.inst[0] = (uint32_t)best_inst;
    return best_prim >= 0;
}

// Exact world mode with an f32 prefilter (plane-only scenes, RenderParams::exact_pf).
// Phase 1 traverses the same tree in f32 and tests each reached primitive's world-space copy
// (wxprims) in f32 with a forward error bound on t, alpha and beta, relative to the magnitudes
// that enter them (absolute dot products; E = 2^-17 is 64x the f32 unit roundoff, which covers
// the f32 rounding of the flattened coefficients and of the ray, the f32 arithmetic and the
// reference's f64 rounding, for scale factors well below 2^20).  A primitive is
//   a certain miss   when the bounds put it outside Plane::hit's acceptance (|n.d| < 1e-8,
//                    t < 0.001, alpha / beta outside the quad or triangle): dropped;
//   a certain hit    when they put it inside: its upper bound t_hi bounds the winner's exact t;
//   a candidate      otherwise, kept while its lower bound t_lo <= the smallest t_hi so far.
// The winner (the reference's closest hit, plane.rs:141-174, object.rs:89-121) is accepted by
// the reference tests and its exact t is <= every certain hit's, so it is a candidate whose
// t_lo survives; phase 2 runs the reference tests in f64 on the surviving candidates only
// (smallest exact t, ties to the higher depth-first rank, as trace_exact_wbvh).  Boxes are cut
// at the bound raised by 2^-20 as there.  A lane with more than XCAND live candidates at once
// (never seen on the reference scenes) falls back to trace_exact_wbvh.
#ifndef NRT_XCAND
#define NRT_XCAND 2  // live candidates per ray (2 / 3 / 4: C5 f64 179.9 / 180.4 / 182.5 ms, C4 133.0 / 133.5 / 136.4)
#endif
constexpr int XCAND = NRT_XCAND;
#ifndef NRT_PF_RCP
#define NRT_PF_RCP 1
#endif
#ifndef NRT_EXACT_IFIF
#define NRT_EXACT_IFIF 0  // the prefiltered compact walk as if-if trips (A/B build)
#endif
__device__ __forceinline__ float absdot(V<float> a, V<float> b) {
    return fabsf(a.x * b.x) + fabsf(a.y * b.y) + fabsf(a.z * b.z);
}
// false: certain miss; otherwise [tlo, thi] bounds the reference's t and `certain` is set
// when the reference test surely accepts the primitive
__device__ __forceinline__ bool exact_prefilter(const DPrimWorld<float>& q, const Ray<float>& r, float& tlo,
                                                float& thi, bool& certain) {
#if NRT_WALK_CONTRACT
    // (FMAs: one rounding where the bound E allows for two)
#pragma clang fp contract(on)
#endif
    constexpr float E = 0x1p-17f;
    const V<float> N = ld3(q.N);
    const float den = dot(N, r.d), aden = fabsf(den), eden = E * absdot(N, r.d);
    certain = false;
    tlo = -INFINITY;
    thi = INFINITY;
    if (aden + eden < 1e-8f) return false;           // |n.d| < 1e-8: the reference rejects it
    if (!(aden - 2.0f * eden > 1e-8f)) return true;  // near-parallel (or NaN): a candidate
#if NRT_PF_RCP
    // hardware reciprocals (1 ulp) instead of IEEE divisions (the exact kernel's build has no fast
    // division): t carries ~2 ulp more, far inside E * |t|; the quotient of the bound is raised
    // by 2^-20 to stay an upper bound
    const float t = (q.D - dot(N, r.o)) * __builtin_amdgcn_rcpf(den);
    const float at = fabsf(t);
    const float et = (E * (fabsf(q.D) + absdot(N, r.o)) + at * eden) * __builtin_amdgcn_rcpf(aden - eden) *
                         (1.0f + 0x1p-20f) + E * at;
#else
    const float t = (q.D - dot(N, r.o)) / den;
    const float at = fabsf(t);
    const float et = (E * (fabsf(q.D) + absdot(N, r.o)) + at * eden) / (aden - eden) + E * at;
#endif
    if (t + et < 0.001f) return false;  // t < 0.001
    const V<float> P = mk(fabsf(r.o.x) + at * fabsf(r.d.x), fabsf(r.o.y) + at * fabsf(r.d.y),
                          fabsf(r.o.z) + at * fabsf(r.d.z));  // bounds |o + t d| per axis
    const V<float> p = r.o + t * r.d;
    const V<float> A = mk(q.AB[0], q.AB[2], q.AB[4]), B = mk(q.AB[1], q.AB[3], q.AB[5]);
    const float al = dot(p, A) - q.AB[6], be = dot(p, B) - q.AB[7];
    const float ea = E * (absdot(A, P) + fabsf(q.AB[6])) + et * absdot(A, r.d);
    const float eb = E * (absdot(B, P) + fabsf(q.AB[7])) + et * absdot(B, r.d);
    bool miss, in;
    if ((q.meta & WKIND_MASK) == PRIM_QUAD) {  // closed [0, 1]^2
        miss = (al + ea < 0.0f) | (al - ea > 1.0f) | (be + eb < 0.0f) | (be - eb > 1.0f);
        in = (al - ea >= 0.0f) & (al + ea <= 1.0f) & (be - eb >= 0.0f) & (be + eb <= 1.0f);
    } else {  // triangle, open
        miss = (al + ea <= 0.0f) | (be + eb <= 0.0f) | (al + be - (ea + eb) >= 1.0f);
        in = (al - ea > 0.0f) & (be - eb > 0.0f) & (al + be + (ea + eb) < 1.0f);
    }
    if (miss) return false;
    tlo = t - et;
    thi = t + et;
    certain = in & (tlo >= 0.001f) & (thi < INFINITY);
    if (!(tlo == tlo)) tlo = -INFINITY;  // NaN bound: keep the candidate
    if (!(thi == thi)) thi = INFINITY;
    return true;
}

// Candidate list of the prefilter: slots (-1: free) and their t_lo; a new candidate takes the
// first free slot or one whose t_lo the bound has passed, else the list overflows.
struct XCands {
    int32_t cs[XCAND];
    float cl[XCAND];
    float bound;  // smallest t_hi of a certain hit so far
    bool over;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < XCAND; ++j) {
            cs[j] = -1;
            cl[j] = INFINITY;
        }
        bound = INFINITY;
        over = false;
    }
    // prefilter slot `slot` (world primitive q); true when the bound tightened
    __device__ __forceinline__ bool offer(const DPrimWorld<float>& q, const Ray<float>& fr, uint32_t slot) {
        float tlo, thi;
        bool certain;
        if (!exact_prefilter(q, fr, tlo, thi, certain) || tlo > bound) return false;
        const bool tight = certain && thi < bound;
        bound = tight ? thi : bound;
        bool placed = false;
#pragma unroll
        for (int j = 0; j < XCAND; ++j) {
            const bool here = !placed && (cs[j] < 0 || cl[j] > bound);
            cs[j] = here ? (int32_t)slot : cs[j];
            cl[j] = here ? tlo : cl[j];
            placed |= here;
        }
        over |= !placed;
        return tight;
    }
};
// Phase 2: the reference tests on the surviving candidates (smallest exact t, ties to the
// higher depth-first rank, as trace_exact_wbvh).  (After an overflow, testing every slot of the
// tree instead of the unfiltered walk saved registers but measured C4 f64 30 -> 52 ms: teapot rays
// do overflow, and a wave then waits for 6 320 f64 tests.)
template <typename R, int MAXD>
__device__ __forceinline__ bool xcands_finish(const XCands& c, const DSceneView<R>& sc, const Ray<R>& wray,
                                              HitMin<R, MAXD>& hm) {
    R best_t = R(INFINITY);
    uint32_t best_rank = 0;
    int32_t best_prim = -1, best_inst = -1, cur_inst = -2;
    Ray<R> oray = wray;
    // one candidate per trip, shifted down the list: an unrolled loop let the scheduler hoist the
    // f64 primitive loads of all four at once (36 VGPRs of spills in the C5 / C4 f64 kernel)
    int32_t cs[XCAND];
    float cl[XCAND];
#pragma unroll
    for (int j = 0; j < XCAND; ++j) {
        cs[j] = c.cs[j];
        cl[j] = c.cl[j];
    }
#pragma unroll 1
    for (int j = 0; j < XCAND; ++j) {
        const int32_t cj = cs[0];
        const float lj = cl[0];
#pragma unroll
        for (int q = 0; q + 1 < XCAND; ++q) {
            cs[q] = cs[q + 1];
            cl[q] = cl[q + 1];
        }
        if (cj >= 0 && lj <= c.bound) {
            const DExactRef ref = sc.wexact[cj];
            if (ref.inst != cur_inst) {  // the primitive's object-space ray (exact chain)
                oray = wray;
                if (ref.inst >= 0) xform_in<R, true, false>(sc, sc.instances[ref.inst], oray);
                cur_inst = ref.inst;
            }
            R alpha, beta, den;
            V<R> point;
            const R t = plane_t(sc.prims[ref.prim], oray, alpha, beta, point, &den);
            if (t >= R(0) && (t < best_t || (t == best_t && ref.rank > best_rank))) {
                best_t = t;
                best_rank = ref.rank;
                best_prim = (int32_t)ref.prim;
                best_inst = ref.inst;
                if constexpr (NRT_REC_CARRY) {
                    hm.pp = point;
                    hm.pu = alpha;
                    hm.pv = beta;
                    hm.pden = den;
                }
            }
        }
    }
    hm.t = best_t;
    hm.prim = (uint32_t)best_prim;
    hm.depth = best_inst >= 0 ? 1 : 0;
    hm.inst[0] = (uint32_t)best_inst;
    hm.pre = NRT_REC_CARRY != 0;
    return best_prim >= 0;
}

// The prefilter over the world-BVH walk (RenderParams::exact_pf).
template <typename R, int MAXD, int W = 0, bool LSTACK = false>
__device__ __forceinline__ bool trace_exact_wbvh_pf(const DSceneView<R>& sc, const Ray<R>& wray, HitMin<R, MAXD>& hm,
                                                    bool thread = false, uint16_t* lstk = nullptr,
                                                    unsigned long long* pc = nullptr, unsigned long long* tmid = nullptr) {
    // (pc, tmid: PROF builds only -- walk events in the wave's profile row, the stamp before phase 2)
    static_assert(sizeof(R) == 8, "exact world-BVH mode is an f64-kernel mode");
    Ray<float> fr;
    fr.o = mk((float)wray.o.x, (float)wray.o.y, (float)wray.o.z);
    fr.d = mk((float)wray.d.x, (float)wray.d.y, (float)wray.d.z);
    XCands c;
    c.init();
    auto offer_leaf = [&](int32_t ref, float& cut) {
        const uint32_t v = ~(uint32_t)ref, first = v >> 3, cnt = (v & 7u) + 1u;
        for (uint32_t k = 0; k < cnt; ++k) {
            prof_event(pc, PROF_LEAF_TRIPS, PROF_LEAF_LANES);
            if (c.offer(load16(sc.wxprims + first + k), fr, first + k)) cut = c.bound * (1.0f + 0x1p-20f);
        }
    };
    if (W == XTHREAD_W || (W == 0 && thread)) {
        float cut = INFINITY;
        xthread_walk(sc, fr, cut, [&](int32_t ref) { offer_leaf(ref, cut); });
    } else if constexpr (W == WBVH_COMPACT) {
        WbvhTrav ts;
        wbvh_begin(ts, wbvh_root(sc), fr);
        auto walk = [&](auto& stk) {
#if NRT_EXACT_IFIF
            // if-if trips: one primitive offer and (2: also) one node visit per lane per trip
            int32_t leaf = WBVH_NO_LEAF;  // leaf cursor ~(first << 3 | more)
            while (true) {
                const bool leaf_now = leaf != WBVH_NO_LEAF;
                if (leaf_now) {
                    const uint32_t v = ~(uint32_t)leaf, first = v >> 3, more = v & 7u;
                    if (c.offer(load16(sc.wxprims + first), fr, first)) ts.t_best = c.bound * (1.0f + 0x1p-20f);
                    leaf = more ? leaf - 7 : WBVH_NO_LEAF;  // ~((first + 1) << 3 | (more - 1)) = ~v - 7
                }
                if ((NRT_EXACT_IFIF == 2 || !leaf_now) && ts.node >= 0) {
                    wbvh4c_visit<R>(ts, sc, stk);
                }
                if (leaf == WBVH_NO_LEAF && ts.node < 0) {
                    if (ts.node == WBVH_DONE) break;
                    leaf = ts.node;
                    ts.node = wbvh4c_pop(ts, stk);
                }
            }
#else
            while (true) {
                while (ts.node >= 0) {
                    prof_event(pc, PROF_VISIT_TRIPS, PROF_VISIT_LANES);
                    wbvh4c_visit<R>(ts, sc, stk);
                }
                if (ts.node == WBVH_DONE) break;
                offer_leaf(ts.node, ts.t_best);
                ts.node = wbvh4c_pop(ts, stk);
            }
#endif
        };
        if constexpr (LSTACK) {
            walk(lstk);
        } else {
            PrivStack16 stk;
            walk(stk);
        }
    } else {
        WbvhTrav ts;
        wbvh_begin(ts, wbvh_root(sc), fr);
        PrivStack stk;
        while (true) {
            while (ts.node >= 0) {
                if (W == 4 || (W == 0 && sc.wbvh4)) wbvh4_visit<R>(ts, sc, stk);
                else wbvh2_visit<R>(ts, sc, stk);
            }
            if (ts.node == WBVH_DONE) break;
            offer_leaf(ts.node, ts.t_best);
            ts.node = wbvh_pop(ts, stk);
        }
    }
    if (tmid) *tmid = __builtin_amdgcn_s_memtime();
    if (c.over) return trace_exact_wbvh<R, MAXD, W, true, LSTACK>(sc, wray, hm, thread, lstk);
    return xcands_finish(c, sc, wray, hm);
}

// The prefiltered compact walk as a resumable state (ExactSig PERSIST): the kernel advances the
// walks of its lanes one trip at a time and shades the lanes whose walk has ended once enough of
// them have (render_kernel), so lanes that finish early start their next segment instead of idling
// behind the wave's longest walk.  A trip offers one primitive of the parked leaf, visits one node,
// and parks the next leaf the visit or a pop reaches.  The candidates, their bounds and the winner
// are those of trace_exact_wbvh_pf: a leaf's primitives are offered in the same order, and the cut
// a certain hit sets only prunes.
struct XWalk {
    WbvhTrav ts;  // (ts.leaf: the parked leaf cursor ~(first << 3 | more))
    XCands c;
    Ray<float> fr;
    __device__ __forceinline__ bool busy() const { return ts.busy(); }
};
template <typename R>
__device__ __forceinline__ void xwalk_begin(XWalk& w, const DSceneView<R>& sc, const Ray<R>& wray, bool query) {
    w.fr.o = mk((float)wray.o.x, (float)wray.o.y, (float)wray.o.z);
    w.fr.d = mk((float)wray.d.x, (float)wray.d.y, (float)wray.d.z);
    w.c.init();
    wbvh_begin(w.ts, query ? wbvh_root(sc) : WBVH_DONE, w.fr);  // depth cap: no query (Q6)
}
template <typename R, class STK>
__device__ __forceinline__ void xwalk_trip(XWalk& w, const DSceneView<R>& sc, STK& stk) {
    WbvhTrav& ts = w.ts;
    if (ts.leaf != WBVH_NO_LEAF) {
        const uint32_t v = ~(uint32_t)ts.leaf, first = v >> 3, more = v & 7u;
        if (w.c.offer(load16(sc.wxprims + first), w.fr, first)) ts.t_best = w.c.bound * (1.0f + 0x1p-20f);
        ts.leaf = more ? ts.leaf - 7 : WBVH_NO_LEAF;  // ~((first + 1) << 3 | (more - 1)) = ~v - 7
    }
    if (ts.node >= 0) wbvh4c_visit<R>(ts, sc, stk);
    if (ts.leaf == WBVH_NO_LEAF && ts.node < 0 && ts.node != WBVH_DONE) {
        ts.leaf = ts.node;
        ts.node = wbvh4c_pop(ts, stk);
    }
}
// the walk has ended: phase 2 (or, after a candidate overflow, the unfiltered walk)
template <typename R, int MAXD, class STK>
__device__ __forceinline__ bool xwalk_finish(const XWalk& w, const DSceneView<R>& sc, const Ray<R>& wray,
                                             HitMin<R, MAXD>& hm, STK& stk) {
    if (w.c.over) return trace_exact_wbvh<R, MAXD, WBVH_COMPACT, true, true>(sc, wray, hm, false, stk);
    return xcands_finish(w.c, sc, wray, hm);
}

template <bool B, class T, class F> struct TypeIf { using type = T; };  // (hiprtc: no <type_traits>)
template <class T, class F> struct TypeIf<false, T, F> { using type = F; };
// The unfiltered world walk (EXACT_SIG_WORLD: scenes with spheres) as a resumable state, for the
// same persistent loop: a trip runs the reference test (Sphere::hit / Plane::hit in f64 in the
// primitive's object space, sphere.rs:105-163, plane.rs:141-174) on the parked leaf's next
// primitive and visits one node; the winner is trace_exact_wbvh's (smallest t, ties to the higher
// depth-first rank, object.rs:109-115), and the cut it sets only prunes.
template <typename R>
struct XWalkU {
    WbvhTrav ts;
    Ray<float> fr;
    R best_t;
    uint32_t best_rank;
    int32_t best_prim, best_inst;
    __device__ __forceinline__ bool busy() const { return ts.busy(); }
};
template <typename R>
__device__ __forceinline__ void xwalk_begin(XWalkU<R>& w, const DSceneView<R>& sc, const Ray<R>& wray, bool query) {
    w.fr.o = mk((float)wray.o.x, (float)wray.o.y, (float)wray.o.z);
    w.fr.d = mk((float)wray.d.x, (float)wray.d.y, (float)wray.d.z);
    w.best_t = R(INFINITY);
    w.best_rank = 0;
    w.best_prim = -1;
    w.best_inst = -1;
    wbvh_begin(w.ts, query ? wbvh_root(sc) : WBVH_DONE, w.fr);
}
template <typename R, class STK>
__device__ __forceinline__ void xwalk_trip(XWalkU<R>& w, const DSceneView<R>& sc, STK& stk, const Ray<R>& wray) {
    WbvhTrav& ts = w.ts;
    if (ts.leaf != WBVH_NO_LEAF) {
        const uint32_t v = ~(uint32_t)ts.leaf, first = v >> 3, more = v & 7u;
        const DExactRef rf = sc.wexact[first];
        Ray<R> oray = wray;  // the primitive's object-space ray (exact chain)
        if (rf.inst >= 0) xform_in<R, true, false>(sc, sc.instances[rf.inst], oray);
        const DPrim<R>& pr = sc.prims[rf.prim];
        R t;
        if (pr.kind == PRIM_SPHERE) {
            t = sphere_t(pr, oray);
        } else {
            R alpha, beta;
            V<R> point;
            t = plane_t(pr, oray, alpha, beta, point);
        }
        if (t >= R(0) && (t < w.best_t || (t == w.best_t && rf.rank > w.best_rank))) {
            w.best_t = t;
            w.best_rank = rf.rank;
            w.best_prim = (int32_t)rf.prim;
            w.best_inst = rf.inst;
            ts.t_best = (float)t * (1.0f + 0x1p-20f);
        }
        ts.leaf = more ? ts.leaf - 7 : WBVH_NO_LEAF;  // ~((first + 1) << 3 | (more - 1)) = ~v - 7
    }
    if (ts.node >= 0) wbvh4c_visit<R>(ts, sc, stk);
    if (ts.leaf == WBVH_NO_LEAF && ts.node < 0 && ts.node != WBVH_DONE) {
        ts.leaf = ts.node;
        ts.node = wbvh4c_pop(ts, stk);
    }
}
template <typename R, int MAXD, class STK>
__device__ __forceinline__ bool xwalk_finish(const XWalkU<R>& w, const DSceneView<R>&, const Ray<R>&,
                                             HitMin<R, MAXD>& hm, STK&) {
    hm.t = w.best_t;
    hm.prim = (uint32_t)w.best_prim;
    hm.depth = w.best_inst >= 0 ? 1 : 0;
    hm.inst[0] = (uint32_t)w.best_inst;
    return w.best_prim >= 0;
}
// (the prefiltered walk's trip takes the world ray for the same call)
template <typename R, class STK>
__device__ __forceinline__ void xwalk_trip(XWalk& w, const DSceneView<R>& sc, STK& stk, const Ray<R>&) {
    xwalk_trip<R>(w, sc, stk);
}

// Small plane-only scenes (at most EXACT_SLOTS_MAX slots, EXACT_SIG_SLOTS_PF): the prefilter over
// every slot of the culling tree in slot order instead of the walk: the slot index is wave-
// uniform, so each f32 record arrives by scalar load and no lane waits for another's walk (no
// stack, no divergence).  Slot order instead of walk order changes neither the candidate set's
// outcome nor the winner (smallest exact t, ties to the higher rank: xcands_finish).  More than
// XCAND live candidates (never seen on the reference scenes): the reference tests on every slot.
template <typename R, int MAXD>
__device__ __forceinline__ bool trace_exact_slots_pf(const DSceneView<R>& sc, const Ray<R>& wray, HitMin<R, MAXD>& hm) {
    static_assert(sizeof(R) == 8, "exact world mode is an f64-kernel mode");
    Ray<float> fr;
    fr.o = mk((float)wray.o.x, (float)wray.o.y, (float)wray.o.z);
    fr.d = mk((float)wray.d.x, (float)wray.d.y, (float)wray.d.z);
    XCands c;
    c.init();
    const ConstU32 wq = (ConstU32)sc.wxprims;
    const uint32_t n = sc.n_wexact;
    constexpr uint32_t QW = (uint32_t)(sizeof(DPrimWorld<float>) / 4);
    for (uint32_t k = 0; k < n; ++k) {
        uint32_t w[QW];
#pragma unroll
        for (uint32_t i = 0; i < QW; ++i) w[i] = wq[k * QW + i];  // (s_load: k is wave-uniform)
        DPrimWorld<float> q;
        __builtin_memcpy(&q, w, sizeof q);
        c.offer(q, fr, k);
    }
    if (!c.over) return xcands_finish(c, sc, wray, hm);
    R best_t = R(INFINITY);  // overflow: the reference tests on every slot (at most EXACT_SLOTS_MAX)
    uint32_t best_rank = 0;
    int32_t best_prim = -1, best_inst = -1, cur_inst = -2;
    Ray<R> oray = wray;
    for (uint32_t k = 0; k < n; ++k) {
        const DExactRef ref = sc.wexact[k];
        if (ref.inst != cur_inst) {
            oray = wray;
            if (ref.inst >= 0) xform_in<R, true, false>(sc, sc.instances[ref.inst], oray);
            cur_inst = ref.inst;
        }
        R alpha, beta;
        V<R> point;
        const R t = plane_t(sc.prims[ref.prim], oray, alpha, beta, point);
        if (t >= R(0) && (t < best_t || (t == best_t && ref.rank > best_rank))) {
            best_t = t;
            best_rank = ref.rank;
            best_prim = (int32_t)ref.prim;
            best_inst = ref.inst;
        }
    }
    hm.t = best_t;
    hm.prim = (uint32_t)best_prim;
    hm.depth = best_inst >= 0 ? 1 : 0;
    hm.inst[0] = (uint32_t)best_inst;
    return best_prim >= 0;
}

// Small scenes with spheres (at most EXACT_SLOTS_MAX slots of the culling tree, EXACT_SIG_SLOTS): the
// reference test (Sphere::hit / Plane::hit in f64, sphere.rs:105-163, plane.rs:141-174) on every slot
// in slot order, no walk, no boxes, no stack: the slot index is wave-uniform, so no lane waits for
// another's walk, and the kernel variant carries no traversal code (the earth scene's f64 kernel
// spilled 36 VGPRs with the walks compiled in).  The winner is the smallest t, ties to the higher
// depth-first rank (object.rs:109-115), as the walks find it: the frame is the same bit for bit.
template <typename R, int MAXD>
__device__ __forceinline__ bool trace_exact_slots(const DSceneView<R>& sc, const Ray<R>& wray, HitMin<R, MAXD>& hm) {
    static_assert(sizeof(R) == 8, "exact world mode is an f64-kernel mode");
    R best_t = R(INFINITY);
    uint32_t best_rank = 0;
    int32_t best_prim = -1, best_inst = -1, cur_inst = -2;
    Ray<R> oray = wray;
    const uint32_t n = sc.n_wexact;
    for (uint32_t k = 0; k < n; ++k) {
        const DExactRef ref = sc.wexact[k];
        if (ref.inst != cur_inst) {  // (wave-uniform: every lane switches together)
            oray = wray;
            if (ref.inst >= 0) xform_in<R, true, false>(sc, sc.instances[ref.inst], oray);
            cur_inst = ref.inst;
        }
        const DPrim<R>& pr = sc.prims[ref.prim];
        R t;
        if (pr.kind == PRIM_SPHERE) {
            t = sphere_t(pr, oray);
        } else {
            R alpha, beta;
            V<R> point;
            t = plane_t(pr, oray, alpha, beta, point);
        }
        if (t >= R(0) && (t < best_t || (t == best_t && ref.rank > best_rank))) {
            best_t = t;
            best_rank = ref.rank;
            best_prim = (int32_t)ref.prim;
            best_inst = ref.inst;
        }
    }
    hm.t = best_t;
    hm.prim = (uint32_t)best_prim;
    hm.depth = best_inst >= 0 ? 1 : 0;
    hm.inst[0] = (uint32_t)best_inst;
    return best_prim >= 0;
}

template <typename R, int MAXD, bool EXACT, bool FLAT = false, bool PF = false, class SIG = NoSig, class STKP>
__device__ __forceinline__ bool trace(const DSceneView<R>& sc, const Ray<R>& wray, HitMin<R, MAXD>& hm,
                                      STKP stack, bool all = false, bool exact_wbvh = false, uint32_t pf = 0,
                                      bool xthread = false, unsigned long long* pc = nullptr,
                                      unsigned long long* tmid = nullptr) {
    if constexpr (MAXD == 0) return trace_world<R, MAXD, FLAT, SIG>(sc, wray, hm);
    else if constexpr (MAXD < 0) return trace_world_bvh<R, MAXD, FLAT, SIG>(sc, wray, hm, stack);
    else if constexpr (EXACT && sizeof(R) == 8 && SIG::exact == EXACT_SIG_SLOTS) return trace_exact_slots<R, MAXD>(sc, wray, hm);
    else if constexpr (EXACT && sizeof(R) == 8 && SIG::exact == EXACT_SIG_SLOTS_PF) {
        static_assert(PF, "EXACT_SIG_SLOTS_PF is a KF_PLANES variant");
        return trace_exact_slots_pf<R, MAXD>(sc, wray, hm);
    } else if constexpr (EXACT && sizeof(R) == 8 && SIG::exact == EXACT_SIG_WORLD) {
        static_assert(SIG::lstack && SIG::bvh == WBVH_COMPACT, "EXACT_SIG_WORLD: the compact walk, LDS stack");
        return trace_exact_wbvh<R, MAXD, WBVH_COMPACT, PF, true>(sc, wray, hm, false, stack);
    } else if constexpr (EXACT && sizeof(R) == 8 && SIG::exact == EXACT_SIG_WORLD_PF) {
        static_assert(PF, "EXACT_SIG_WORLD_PF is a KF_PLANES variant");
        if constexpr (SIG::lstack) return trace_exact_wbvh_pf<R, MAXD, SIG::bvh, true>(sc, wray, hm, false, stack, pc, tmid);
        else return trace_exact_wbvh_pf<R, MAXD, SIG::bvh>(sc, wray, hm);
    } else if constexpr (EXACT && sizeof(R) == 8) {
        const bool thread = sc.xthread != nullptr && xthread;
        if constexpr (PF) {  // plane-only scenes (KF_PLANES)
            if (exact_wbvh && pf) return trace_exact_wbvh_pf<R, MAXD>(sc, wray, hm, thread);
        }
        if (exact_wbvh) return trace_exact_wbvh<R, MAXD, 0, PF>(sc, wray, hm, thread);
        return trace_bvh<R, MAXD, EXACT>(sc, wray, hm, all);
    } else return trace_bvh<R, MAXD, EXACT>(sc, wray, hm, EXACT && all);
}

// HitRecord of the winner (HitRecord::new_with_uv, hitable.rs:38-59).
// World-space record (MAXD <= 0; device_scene.hpp DPrimWorld): the
// reference's front-face sign signum(d'.n) = signum(d.(M^T n)), shading normal
// mapped out by the chain's rotations only.
template <typename R, int MAXD, bool FLAT = false, bool STAGED = false>  // STAGED: sc.wprims in LDS (80-B stride)
__device__ __forceinline__ Rec<R> make_record_world(const DSceneView<R>& sc, const Ray<R>& wray,
                                                     const HitMin<R, MAXD>& hm) {
    // hm.prim is always a primitive record: box and room hits name their face quad
    const DPrimWorld<R> q = load16(STAGED ? (const DPrimWorld<R>*)((const unsigned char*)sc.wprims + hm.prim * wprim_lds_stride(MAXD))
                                          : sc.wprims + hm.prim);
    R t = hm.t;  // world BVH: the closest key = t scaled by the winner's coplanar-tie factor (WCLASS_*)
    if (MAXD < 0 && (sc.wflags & WFLAG_COPLANAR)) {
        const uint32_t cls = q.meta >> WCLASS_SHIFT;
        t = cls == WCLASS_WIN ? t * R(1.0 / (1.0 - (double)WTIE_EPS)) : (cls == WCLASS_LOSE ? t * R(1.0 / (1.0 + (double)WTIE_EPS)) : t);
    }
    const V<R> pw = vfma(t, wray.d, wray.o);
    const uint32_t kind = q.meta & WKIND_MASK;
    Rec<R> h;
    h.p = pw;
    V<R> geo, shade;
    if (!FLAT && kind == PRIM_SPHERE) {
        if (NRT_SPHERE_REPROJ && sizeof(R) == 4 && q.AB[6] == R(0)) {
            // f32-tested spheres: the hit point back on the surface (its f32 t carries a few ulp,
            // which would leave the next ray's origin off the surface by more than the t_min of
            // 0.001 hides), as one Newton step on F(p) = |p - center|^2 - r^2 evaluated relative
            // to the anchor P (F = |e|^2 + 2 e.V, e = p - P, V = P - center: small terms only, so
            // the step is accurate for a ground sphere of r = 1e3 or 1e5 too, where center + r * n
            // would round to the ulp of r)
            const V<R> P = mk(q.AB[3], q.AB[4], q.AB[5]) + wray.time * ld3(q.AB);
            const V<R> Vv = mk(q.S[0], q.S[1], q.S[2]);
            const V<R> e = h.p - P;
            const V<R> g = e + Vv;  // p - center
            const R gg = dot(g, g);
            const R F = dot(e, e) + R(2) * dot(e, Vv);
            h.p = h.p - (F * fast_rcp(R(2) * gg)) * g;
            geo = normalize(g);
        } else {
            const V<R> center = ld3(q.N) + wray.time * ld3(q.AB);
            geo = normalize(h.p - center);
        }
        shade = geo;
        // uv (acos / atan2) only where a texture reads it: sphere_uv, from the record's normal
        // (the ground sphere of the earth scene is solid: 18 % of its shading was this record)
        h.u = R(UV_DEFERRED);
        h.v = R(0);
    } else {
        h.u = dot(h.p, mk(q.AB[0], q.AB[2], q.AB[4])) - q.AB[6];
        h.v = dot(h.p, mk(q.AB[1], q.AB[3], q.AB[5])) - q.AB[7];
        if (kind >= PRIM_QUAD_X) {  // axis quad: the normal is N[a] along axis a (other slots hold P, threshold)
            const uint32_t ax = kind - PRIM_QUAD_X;
            geo = mk(ax == 0 ? q.N[0] : R(0), ax == 1 ? q.N[1] : R(0), ax == 2 ? q.N[2] : R(0));
        } else {
            geo = ld3(q.N);
        }
        shade = ld3(q.S);
    }
    const R sign = signum(dot(wray.d, geo));
    h.front = sign < R(0);
    h.n = (-sign) * shade;
    h.mat = (q.meta >> WKIND_BITS) & WMAT_MASK;
    return h;
}

// Instance mode: recomputed exactly as the candidate test computed it
// (object-space point / normal / uv, then mapped out through the instances).
template <typename R, int MAXD, bool EXACT, bool PLANES = false>  // PLANES: no spheres (KF_PLANES)
__device__ __forceinline__ Rec<R> make_record_bvh(const DSceneView<R>& sc, const Ray<R>& wray, const HitMin<R, MAXD>& hm) {
    Ray<R> ray = wray;
    auto enter = [&](uint32_t iid) {
        if constexpr (EXACT) xform_in<R, true>(sc, sc.instances[iid], ray);
        else enter_fast(sc.inst_fast[iid], ray);
    };
    auto leave = [&](uint32_t iid, Rec<R>& rec) {
        if constexpr (EXACT) xform_out(sc, sc.instances[iid], rec);
        else leave_fast(sc.inst_fast[iid], rec);
    };
    const bool pre = EXACT && PLANES && NRT_REC_CARRY && hm.pre;  // (xcands_finish: object-space values carried)
    if constexpr (MAXD == 1) {
        if (hm.depth > 0 && !pre) enter(hm.inst[0]);
    } else {
        for (int l = 0; l < hm.depth; ++l) enter(hm.inst[l]);
    }
    Rec<R> h;
    V<R> outward;
    const R t = hm.t;
    if constexpr (!EXACT) {
        const DPrimFast<R>& q = sc.fprims[hm.prim];
        h.p = vfma(t, ray.d, ray.o);
        if (q.kind == PRIM_SPHERE) {
            const V<R> center = ld3(q.n) + ray.time * ld3(q.A);
            outward = normalize(h.p - center);
            h.front = true;  // (sphere_uv reads the outward normal as h.n on the front face)
            h.n = outward;
            sphere_uv(h, h.u, h.v);
        } else {
            h.u = dot(h.p, ld3(q.A)) - q.a0;
            h.v = dot(h.p, ld3(q.B)) - q.b0;
            outward = ld3(q.n);
        }
        h.mat = q.material;
    }
    const DPrim<R>& pr = sc.prims[EXACT ? hm.prim : 0];
    if (!EXACT) {
    } else if (!PLANES && pr.kind == PRIM_SPHERE) {  // sphere.rs:148-161 (f64 acos / atan2: 50 VGPRs of
                                                    // spills in the plane-only variant, were it compiled in)
        const V<R> center = ld3(pr.a) + ray.time * ld3(pr.b);
        h.p = vfma(t, ray.d, ray.o);
        outward = normalize(h.p - center);
        // (u, v) only where a texture reads them (image, checker): the f64 acos / atan2 are the
        // record's costliest part, and the earth scene's ground sphere is solid-coloured
        const DMaterial& dm = sc.materials[pr.material];  // (a dielectric has no texture)
        const uint32_t tk = dm.kind == MAT_DIELECTRIC ? (uint32_t)TEX_SOLID : sc.textures[dm.texture].kind;
        h.u = R(0);
        h.v = R(0);
        if (tk == TEX_IMAGE || tk == TEX_CHECKER) {
            const R theta = acos(-outward.y);
            const R phi = atan2(-outward.z, outward.x) + R(M_PI);
            h.u = phi / (R(2.0) * R(M_PI));
            h.v = theta / R(M_PI);
        }
    } else if (pre) {  // the same point, (alpha, beta) and n.d as plane_t computed them
        h.p = hm.pp;
        h.u = hm.pu;
        h.v = hm.pv;
        outward = ld3(pr.n);
    } else {  // plane.rs:156-159
        h.p = vfma(t, ray.d, ray.o);
        const V<R> ph = h.p - ld3(pr.a);
        h.u = dot(ld3(pr.w), cross(ph, ld3(pr.c)));
        h.v = dot(ld3(pr.w), cross(ld3(pr.b), ph));
        outward = ld3(pr.n);
    }
    // HitRecord::new_with_uv (hitable.rs:38-59) (n.d = d.n: the products commute)
    const R sign = signum(pre ? hm.pden : dot(ray.d, outward));
    h.front = sign < R(0);
    h.n = (-sign) * outward;
    if constexpr (EXACT) h.mat = pr.material;
    if constexpr (MAXD == 1) {
        if (hm.depth > 0) leave(hm.inst[0], h);
    } else {
        for (int l = hm.depth - 1; l >= 0; --l) leave(hm.inst[l], h);
    }
    return h;
}

template <typename R, int MAXD, bool EXACT, bool FLAT = false, bool STAGED = false, bool PLANES = false>
__device__ __forceinline__ Rec<R> make_record(const DSceneView<R>& sc, const Ray<R>& wray, const HitMin<R, MAXD>& hm) {
    if constexpr (MAXD <= 0) return make_record_world<R, MAXD, FLAT, STAGED>(sc, wray, hm);
    else return make_record_bvh<R, MAXD, EXACT, PLANES>(sc, wray, hm);
}

// ----------------------------------------------------------------- shading
// Perlin textures in f64 (noise 0.9.0 as restated in noise.hpp).  `perm` is the
// octave's permutation table (256 floats 0..255 in the texel array).
__device__ __forceinline__ double perlin_grad(uint32_t h, double x, double y, double z) {
    // noise 0.9 perlin_3d gradient_dot_v: every case is (±a) + (±b) with a in {x, y}, b in
    // {y, z}; the 16 cases as bit masks over h & 15
    const uint32_t bit = 1u << (h & 15u);
    const double a = (0xCF00u & bit) ? y : x, b = (0x300Fu & bit) ? y : z;
    return ((0xEAAAu & bit) ? -a : a) + ((0x8CCCu & bit) ? -b : b);
}
__device__ __forceinline__ double perlin3(const uint32_t* perm, double x, double y, double z) {
    auto P = [&](uint32_t i) { return perm[i]; };
    const double fx = floor(x), fy = floor(y), fz = floor(z);
    const uint32_t ix = (uint32_t)(long long)fx & 255u, iy = (uint32_t)(long long)fy & 255u,
                   iz = (uint32_t)(long long)fz & 255u;
    const double dx = x - fx, dy = y - fy, dz = z - fz;
    const uint32_t ix1 = (ix + 1u) & 255u, iy1 = (iy + 1u) & 255u, iz1 = (iz + 1u) & 255u;
    const uint32_t a0 = P(ix), a1 = P(ix1);
    const uint32_t b00 = P(a0 ^ iy), b10 = P(a1 ^ iy), b01 = P(a0 ^ iy1), b11 = P(a1 ^ iy1);
    const double g000 = perlin_grad(P(b00 ^ iz), dx, dy, dz);
    const double g100 = perlin_grad(P(b10 ^ iz), dx - 1.0, dy, dz);
    const double g010 = perlin_grad(P(b01 ^ iz), dx, dy - 1.0, dz);
    const double g110 = perlin_grad(P(b11 ^ iz), dx - 1.0, dy - 1.0, dz);
    const double g001 = perlin_grad(P(b00 ^ iz1), dx, dy, dz - 1.0);
    const double g101 = perlin_grad(P(b10 ^ iz1), dx - 1.0, dy, dz - 1.0);
    const double g011 = perlin_grad(P(b01 ^ iz1), dx, dy - 1.0, dz - 1.0);
    const double g111 = perlin_grad(P(b11 ^ iz1), dx - 1.0, dy - 1.0, dz - 1.0);
    auto quintic = [](double t) { return t * t * t * (t * (t * 6.0 - 15.0) + 10.0); };
    const double a = quintic(dx), b = quintic(dy), c = quintic(dz);
    const double k0 = g000, k1 = g100 - g000, k2 = g010 - g000, k3 = g001 - g000;
    const double k4 = g000 + g110 - g100 - g010, k5 = g000 + g101 - g100 - g001;
    const double k6 = g000 + g011 - g010 - g001;
    const double k7 = g100 + g010 + g001 + g111 - g000 - g110 - g101 - g011;
    const double r = k0 + k1 * a + k2 * b + k3 * c + k4 * a * b + k5 * a * c + k6 * b * c + k7 * a * b * c;
    const double s = r * 1.1547005383792515;  // 1 / (sqrt(3) / 2)
    return s < -1.0 ? -1.0 : (s > 1.0 ? 1.0 : s);
}
__device__ __forceinline__ double powi_rt(double a, uint32_t b) {  // f64::powi, b >= 0 (__powidf2)
    double r = 1.0;
    while (true) {
        if (b & 1u) r *= a;
        b /= 2u;
        if (b == 0u) break;
        a *= a;
    }
    return r;
}
// Abs<Fbm<Perlin>>::get (noise.rs:136-144, marble.rs:87-96), then the Noise / Marble
// colour (compiled into the KF_PERLIN kernel variants only).
__device__ __forceinline__ double perlin_texture(const uint32_t* texels, const DTexture& t, double x, double y, double z) {
    const uint32_t* perm = texels + t.offset;
    const double pz = z;
    x = x * t.color[0];
    y = y * t.color[0];
    z = z * t.color[0];
    double result = 0.0;
    for (uint32_t k = 0; k < t.a; ++k) {
        double signal = perlin3(perm + 256u * k, x, y, z);
        signal = signal * powi_rt(t.color[2], k);
        result = result + signal;
        x = x * t.color[1];
        y = y * t.color[1];
        z = z * t.color[1];
    }
    const double n = fabs(result * t.scale);
    return t.kind == TEX_NOISE ? n : (1.0 + sin(t.color[0] * pz + 10.0 * n)) / 2.0;
}

// k / 255.0f, correctly rounded, for a byte k (into_rgb32f, textures/image.rs:24-28): the product
// with the rounded reciprocal and one Markstein correction step, exact for all 256 values (the
// product alone is 1 ulp off for 158 of them); explicit FMAs, so the exact kernel's
// -ffp-contract=off build computes the same
#ifndef NRT_TEX_FORMATS
#define NRT_TEX_FORMATS 15  // image texel formats compiled in: 1 RGB32F, 2 RGBA8, 4 RGB8T, 8 PAL16
#endif
__device__ __forceinline__ float unorm8(uint32_t k) {
    constexpr float r = 1.0f / 255.0f;
    const float b = (float)k;
    const float q = b * r;
    return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, b), r, q);
}

// Texture::get_color (solid_color.rs:35-43, textures/image.rs:31-40, checker.rs:76-89,
// noise.rs:136-144, marble.rs:87-96); `p` = the world-space hit point
template <typename R, bool PERLIN, bool PAL_ONLY = false>  // PAL_ONLY: solid colours and PAL16 images only (KF_TEXPAL)
__device__ V<R> tex_color(const DSceneView<R>& sc, uint32_t tid, R u, R v, V<R> p) {
    for (int guard = 0; guard < (PAL_ONLY ? 1 : 64); ++guard) {
        const DTexture& t = sc.textures[tid];
        if constexpr (PAL_ONLY) {  // (the same lookup as below, without the other kinds' and formats' code)
            if (t.kind == TEX_SOLID) return ld3d<R>(t.color);
            const R cu = u < R(0) ? R(0) : (u > R(1) ? R(1) : u);
            const R cv = v < R(0) ? R(0) : (v > R(1) ? R(1) : v);
            const uint32_t th = t.b & 0xFFFFu;
            const R fx = cu * (R)t.a;
            const R fy = (R(1) - cv) * (R)th;
            const uint32_t x = !(fx > R(0)) ? 0u : (fx >= (R)t.a ? t.a - 1 : (uint32_t)fx);
            const uint32_t y = !(fy > R(0)) ? 0u : (fy >= (R)th ? th - 1 : (uint32_t)fy);
            const uint32_t* base = sc.texels + t.offset;
            const uint64_t i = tex_pal_index(x, y, (t.a + 7u) >> 3);
            const uint32_t pi = (base[i >> 1] >> ((uint32_t)(i & 1u) * 16u)) & 0xFFFFu;
            const uint32_t w = base[tex_pal_index_words(t.a, th) + tex_pal_band_word(t.b, y) + pi];
            return mk((R)unorm8(w & 0xFFu), (R)unorm8((w >> 8) & 0xFFu), (R)unorm8((w >> 16) & 0xFFu));
        }
        if (t.kind == TEX_SOLID) return ld3d<R>(t.color);
        if (t.kind == TEX_NOISE || t.kind == TEX_MARBLE) {
            // (the host launches a PERLIN variant whenever the scene holds one of these)
            if constexpr (PERLIN) {
                const double c = perlin_texture(sc.texels, t, (double)p.x, (double)p.y, (double)p.z);
                return mk((R)c, (R)c, (R)c);
            } else {
                return mk(R(0), R(0), R(0));
            }
        }
        if (t.kind == TEX_IMAGE) {
            const R cu = u < R(0) ? R(0) : (u > R(1) ? R(1) : u);  // f64::clamp keeps NaN
            const R cv = v < R(0) ? R(0) : (v > R(1) ? R(1) : v);
            const uint32_t th = t.format == TEXFMT_PAL16 ? (t.b & 0xFFFFu) : t.b;  // (PAL16: band shift above)
            const R fx = cu * (R)t.a;
            const R fy = (R(1) - cv) * (R)th;
            // `as u32` saturates (NaN -> 0); index W/H would panic in the
            // reference (Q12): clamped to the last texel here.
            uint32_t x = !(fx > R(0)) ? 0u : (fx >= (R)t.a ? t.a - 1 : (uint32_t)fx);
            uint32_t y = !(fy > R(0)) ? 0u : (fy >= (R)th ? th - 1 : (uint32_t)fy);
            if ((NRT_TEX_FORMATS & 8) && t.format == TEXFMT_PAL16) {
                // the texel's 16-bit palette index, then its band's palette word
                const uint32_t* base = sc.texels + t.offset;
                const uint64_t i = tex_pal_index(x, y, (t.a + 7u) >> 3);
                const uint32_t pi = (base[i >> 1] >> ((uint32_t)(i & 1u) * 16u)) & 0xFFFFu;
                const uint32_t w = base[tex_pal_index_words(t.a, th) + tex_pal_band_word(t.b, y) + pi];
                return mk((R)unorm8(w & 0xFFu), (R)unorm8((w >> 8) & 0xFFu), (R)unorm8((w >> 16) & 0xFFu));
            }
            if ((NRT_TEX_FORMATS & 4) && t.format == TEXFMT_RGB8T) {
                // three bytes at a byte offset: the two words that hold them, aligned (v_alignbyte)
                const uint64_t o = tex_rgb8_byte(x, y, (t.a + 7u) >> 3);
                const uint32_t* pw = sc.texels + t.offset + (o >> 2);
                const uint32_t w = __builtin_amdgcn_alignbyte(pw[1], pw[0], (uint32_t)o & 3u);
                return mk((R)unorm8(w & 0xFFu), (R)unorm8((w >> 8) & 0xFFu), (R)unorm8((w >> 16) & 0xFFu));
            }
            if ((NRT_TEX_FORMATS & 2) && (!(NRT_TEX_FORMATS & 1) || t.format == TEXFMT_RGBA8)) {
                // one word (8 x 4 tiles): the three bytes, k / 255.0f exactly
#ifdef NRT_TEX_ROWMAJOR
                const uint32_t w = sc.texels[t.offset + (uint64_t)y * t.a + x];
#else
                const uint32_t w = sc.texels[t.offset + tex_tiled_index(x, y, (t.a + 7u) >> 3)];
#endif
                return mk((R)unorm8(w & 0xFFu), (R)unorm8((w >> 8) & 0xFFu), (R)unorm8((w >> 16) & 0xFFu));
            }
            const uint32_t* px = sc.texels + t.offset + 3ull * ((uint64_t)y * t.a + x);
            return mk((R)__uint_as_float(px[0]), (R)__uint_as_float(px[1]), (R)__uint_as_float(px[2]));
        }
        // Checker: (uv * scale).as_u64vec2() summed, parity selects even/odd
        const R su = u * (R)t.scale, sv = v * (R)t.scale;
        const uint64_t iu = !(su > R(0)) ? 0ull : (su >= R(18446744073709551615.0) ? ~0ull : (uint64_t)su);
        const uint64_t iv = !(sv > R(0)) ? 0ull : (sv >= R(18446744073709551615.0) ? ~0ull : (uint64_t)sv);
        tid = ((iu + iv) % 2 == 0) ? t.a : t.b;
    }
    return mk(R(0), R(0), R(0));
}

template <typename R> __device__ __forceinline__ V<R> reflect(V<R> v, V<R> n) {
    return vfma(-(R(2.0) * dot(v, n)), n, v);
}
template <typename R> __device__ __forceinline__ V<R> refract(V<R> i, V<R> n, R eta) {
    const R ndi = dot(n, i);
    const R k = R(1.0) - eta * eta * (R(1.0) - ndi * ndi);
    if (k >= R(0)) return vfma(-(eta * ndi + fast_sqrt(k)), n, eta * i);
    return mk(R(0), R(0), R(0));
}
// dielectric.rs:13-19 (powi(5) = x * ((x*x)*(x*x)))
template <typename R> __device__ __forceinline__ R reflectance(R cosine, R ri) {
    R r0 = fast_div(R(1.0) - ri, R(1.0) + ri);
    r0 = r0 * r0;
    const R x = R(1.0) - cosine;
    const R x2 = x * x;
    return r0 + (R(1.0) - r0) * (x * (x2 * x2));
}

// Copy the LDS-stageable scene arrays into dynamic LDS at `base` (all threads).
template <typename R>
__device__ __forceinline__ DSceneView<R> stage_scene(const DSceneView<R>& g, unsigned char* base, uint32_t wstride) {
    DSceneView<R> s = g;
    uint32_t off = 0;
    auto copy = [&](const void* src, uint32_t bytes) -> const void* {
        unsigned char* dst = base + off;
        const uint4* s4 = (const uint4*)src;
        uint4* d4 = (uint4*)dst;
        for (uint32_t k = threadIdx.x; k < bytes / 16; k += BLOCK) d4[k] = s4[k];
        off += (bytes + 15) & ~15u;
        return dst;
    };
    s.nodes = (const DNode<R>*)copy(g.nodes, g.n_nodes * (uint32_t)sizeof(DNode<R>));
    s.prims = (const DPrim<R>*)copy(g.prims, g.n_prims * (uint32_t)sizeof(DPrim<R>));
    s.xforms = (const DXform<R>*)copy(g.xforms, g.n_xforms * (uint32_t)sizeof(DXform<R>));
    s.instances = (const DInstance*)copy(g.instances, g.n_instances * (uint32_t)sizeof(DInstance));
    s.materials = (const DMaterial*)copy(g.materials, g.n_materials * (uint32_t)sizeof(DMaterial));
    s.textures = (const DTexture*)copy(g.textures, g.n_textures * (uint32_t)sizeof(DTexture));
    s.fprims = (const DPrimFast<R>*)copy(g.fprims, g.n_fprims * (uint32_t)sizeof(DPrimFast<R>));
    s.inst_fast = (const DInstFast<R>*)copy(g.inst_fast, g.n_inst_fast * (uint32_t)sizeof(DInstFast<R>));
    s.mats_fast = (const DMatFast*)copy(g.mats_fast, g.n_mats_fast * (uint32_t)sizeof(DMatFast));
    {  // world primitives wstride bytes apart (device_scene.hpp wprim_lds_stride)
        unsigned char* dst = base + off;
        const uint4* s4 = (const uint4*)g.wprims;
        constexpr uint32_t Q = (uint32_t)sizeof(DPrimWorld<R>) / 16u;
        const uint32_t QS = wstride / 16u;
        for (uint32_t k = threadIdx.x; k < g.n_wprims * Q; k += BLOCK) ((uint4*)dst)[(k / Q) * QS + k % Q] = s4[k];
        off += (g.n_wprims * wstride + 15u) & ~15u;
        s.wprims = (const DPrimWorld<R>*)dst;
    }
    if constexpr (sizeof(R) == 8) {  // small culling trees of the exact world walk (DSceneView::n_xstage)
        if (g.n_xstage) {
            s.wbvh4c = (const DBvh4cNode*)copy(g.wbvh4c, g.n_xstage * (uint32_t)sizeof(DBvh4cNode));
            s.wxprims = (const DPrimWorld<float>*)copy(g.wxprims, g.n_wexact * (uint32_t)sizeof(DPrimWorld<float>));
            s.wexact = (const DExactRef*)copy(g.wexact, g.n_wexact * (uint32_t)sizeof(DExactRef));
        }
    }
    __syncthreads();
    return s;
}

// ------------------------------------------------------------------ kernel
// ChaCha8 (the reference's stream): one lane per pixel.  Path regeneration: a
// lane starts its pixel's next sample as soon as its current path terminates,
// so a wave no longer waits for its longest path every sample; each lane still
// consumes its pixel's RNG stream strictly in sample order and sums samples in
// order (camera.rs:325-331).
//
// Philox: a sample's random numbers depend only on (pixel, sample, bounce), so
// a sample need not stay on one lane.  Waves are persistent: each takes groups of
// p.wave_pixels consecutive pixels from a global queue and hands the group's
// pixels x spp samples out from a wave-uniform counter; a lane whose path ends
// claims the next unclaimed sample (ballot + mbcnt), so lanes stay busy until
// the queue is empty instead of idling behind the lane with the longest run of
// paths, and no wave idles while another still has pixels.  Sample radiance is
// rounded to a 2^-k grid (p.acc_scale) and summed in f64 into per-pixel LDS
// slots: sums of grid values below 2^53 are exact, hence independent of which
// lane finished when, and frames are bitwise identical for every row partition,
// group size and grid.
//
// PROF (diagnostic builds only, never timed): per-wave s_memtime stamps split
// each loop iteration into camera-ray / trace / shading cycles, summed into
// p.counters[0..3] = {iterations, camera, trace, shade} (+ [4] waves).
//
// Register budget: the f32 world-mode Philox kernel sits at the 80-VGPR edge of
// 6 waves per SIMD; ask for 6 (the other variants keep the compiler's choice).
//
// Kernel variant flags: KF_PROF = phase-profile stamps (diagnostics), KF_PERLIN = the
// scene has Noise / Marble textures (their f64 Fbm code is only compiled into the
// variants that need it: it would raise the register budget of every other scene),
// KF_FLAT = world-list scene without spheres whose materials all have solid colours
// (no f64 sphere test, uv mapping or texture lookup compiled in: the Cornell box).
// (KF_* values: render_params.hpp)
// KF_PLANES (f64 / ChaCha8 only): the scene has no spheres.  The f64 kernel is register-bound;
// plane-only scenes run best at 4 waves per SIMD (C5 245 ms, C4 33 ms; 3 waves: 267, 35.5),
// sphere scenes (f64 quadratic, uv, textures) at 3 (C3 earth 4.85 ms against 5.98 at 4).

// Philox sample pool: LDS slots per wave (a power of two; see the Philox branch of
// render_kernel) and the pool's LDS bytes per workgroup for P pixels per group.
#ifndef NRT_GRAB
#define NRT_GRAB 1  // Philox groups per queue atomic (render_kernel's fetch)
#endif
#ifndef NRT_GRAB_FLAT
// ... for the solid-colour (KF_FLAT) world-BVH kernels: two measured C4 29.82 -> 29.64 ms at 6 waves per
// SIMD (round 5), but at 7 one is faster again (29.69 -> 29.47 ms, three alternating runs); the world
// lists (C5) take one too (9.78-9.81 against 9.82-9.85 ms with two, and a lone launch's last groups end
// together: row shards at N = 8 unpipelined 0.838 -> 0.873 of linear), the textured earth 5.14 vs 5.27
#define NRT_GRAB_FLAT 1
#endif
#ifndef NRT_PROBE_HEAD
// 1: skip queue heads an agent-scope load shows empty before the atomic (saved C5 ~2 MB of HBM
// writes, but the extra round trip before each fetch cost C3 earth 6.67 -> 7.32 ms): off
#define NRT_PROBE_HEAD 0
#endif
#ifndef NRT_FETCH_AHEAD
#define NRT_FETCH_AHEAD 64u  // Philox: take the next group when fewer samples are left to claim
#endif
#ifndef NRT_SLOTS_LIST
#define NRT_SLOTS_LIST 2
#endif
#ifndef NRT_SLOTS_BVH
#define NRT_SLOTS_BVH 4
#endif
template <int MAXD>
constexpr uint32_t philox_slots() {
    return MAXD == 0 ? NRT_SLOTS_LIST : NRT_SLOTS_BVH;
}
template <int MAXD>
__host__ __device__ constexpr uint32_t philox_pool_bytes(uint32_t P) {
    return (BLOCK / 64) * philox_slots<MAXD>() * P * (3u * (uint32_t)sizeof(double) + 4u);
}

template <typename R, class G, int MAXD, class SIG = NoSig>
constexpr int min_waves_per_simd(int kflags = 0) {
#ifndef NRT_WORLD_LIST_WAVES
#define NRT_WORLD_LIST_WAVES 6  // the generic world-list loop (NoSig)
#endif
#ifndef NRT_JIT_LIST_WAVES
#define NRT_JIT_LIST_WAVES 7  // scene-specialised world lists with textures (the earth: 72 VGPRs; C3 5.135 -> 5.052 ms)
#endif
#ifndef NRT_FLAT_WAVES
#define NRT_FLAT_WAVES 8  // scene-specialised solid-colour world lists (C5: 61 VGPRs; 9.777 -> 9.543 ms)
#endif
#ifndef NRT_F64_WAVES
#define NRT_F64_WAVES 4  // f64 kernels, plane-only scenes (KF_PLANES): 4 waves per SIMD
#endif
#ifndef NRT_F64_SPHERE_WAVES
#define NRT_F64_SPHERE_WAVES 3
#endif
#ifndef NRT_F64_LSTACK_WAVES
#define NRT_F64_LSTACK_WAVES 3  // the LDS-stack variant: ring + stack + scene leave room for 3 workgroups
#endif
    if (sizeof(R) == 8 && SIG::lstack) return NRT_F64_LSTACK_WAVES;
    if (sizeof(R) == 8) return (kflags & KF_PLANES) ? NRT_F64_WAVES : NRT_F64_SPHERE_WAVES;
#ifndef NRT_WBVH_WAVES
#define NRT_WBVH_WAVES 6  // KF_FLAT world BVH, generic (NoSig): 80 VGPRs, no spill
#endif
#ifndef NRT_JIT_WBVH_WAVES
#define NRT_JIT_WBVH_WAVES 7  // KF_FLAT world BVH, scene-specialised (BvhSig; the teapot: C4 30.02 -> 29.74 ms)
#endif
#ifndef NRT_WBVH_SPHERE_WAVES
#define NRT_WBVH_SPHERE_WAVES 5  // world BVH with spheres / textures (not KF_FLAT): 96 VGPRs, 5 spilled (spheres 1080p 32.5 -> 31.3 ms)
#endif
    // The f32 Philox kernels at 7 or more waves per SIMD read the camera at its use (cam3 RELOAD): the
    // SGPR budget shrinks with the wave count (7 waves: 94, 8: 78 here), and the 21 camera SGPRs held
    // through the loop were spilled to VGPR lanes; the generic kernels (NoSig) keep their counts (at 7 / 8
    // they spill to scratch).  Frames identical (the waves place no work, the same loads feed the same FMAs).
    constexpr bool JIT = SIG::n > 0 || SIG::bvh != 0;
    if (sizeof(R) == 4 && MAXD < 0 && !G::uses_lds)
        return (kflags & KF_FLAT) ? (JIT ? NRT_JIT_WBVH_WAVES : NRT_WBVH_WAVES) : NRT_WBVH_SPHERE_WAVES;
    if (sizeof(R) == 4 && MAXD == 0 && !G::uses_lds && (kflags & KF_FLAT) && JIT) return NRT_FLAT_WAVES;
    if (sizeof(R) == 4 && MAXD == 0 && !G::uses_lds && !(kflags & KF_PERLIN))
        return JIT ? NRT_JIT_LIST_WAVES : NRT_WORLD_LIST_WAVES;
    return 1;
}
static_assert(BLOCK % 64 == 0, "stack / ring / accumulator layouts assume whole waves");

// Camera vector q of RenderParams: the f32 kernel takes the host-rounded copy
// (kernel arguments stay in SGPRs), the f64 kernel the double.
// RELOAD (f32): scalar loads from the kernel arguments at the use (offset laundered: not hoisted), as
// the f64 branch below: 21 SGPRs less held through the loop.  The kernels at 7+ waves per SIMD take it
// (min_waves_per_simd; C5 at 8 waves: 37 SGPRs spilled to VGPR lanes without it, 12 with it; at 6 / 7
// waves with SGPRs to spare the reloads alone cost 1-1.5 %)
template <typename R, bool RELOAD = NRT_CAM_RELOAD != 0>
__device__ __forceinline__ V<R> cam3(const RenderParams& p, int q, const double* d) {
    if constexpr (sizeof(R) == 4 && RELOAD) {
        (void)p;
        (void)d;
        uint32_t o = (uint32_t)__builtin_offsetof(RenderParams, camf) + (uint32_t)q * 12u;
        asm volatile("" : "+s"(o));
        typedef const __attribute__((address_space(4))) unsigned char* KArgF;
        const KArgF base = (KArgF)__builtin_amdgcn_kernarg_segment_ptr();
        const __attribute__((address_space(4))) float* fp = (const __attribute__((address_space(4))) float*)(base + o);
        return mk(fp[0], fp[1], fp[2]);
    } else if constexpr (sizeof(R) == 4) {
        return mk(p.camf[q][0], p.camf[q][1], p.camf[q][2]);
    } else {
        // f64: scalar loads from the kernel arguments at the use (the offset laundered, so the loads
        // are not hoisted out of the loop): seven f64 vectors held live through the loop spilled the
        // earth scene's exact kernel to scratch (42 registers' worth; the camera ray and the
        // background are the only readers).  RenderParams is the kernel's first argument (kernarg
        // offset 0; see render_kernel).
        (void)p;
        (void)d;
        constexpr uint32_t off[7] = {
            (uint32_t)__builtin_offsetof(RenderParams, top_left),       (uint32_t)__builtin_offsetof(RenderParams, pixel_delta_u),
            (uint32_t)__builtin_offsetof(RenderParams, pixel_delta_v),  (uint32_t)__builtin_offsetof(RenderParams, look_from),
            (uint32_t)__builtin_offsetof(RenderParams, defocus_disk_u), (uint32_t)__builtin_offsetof(RenderParams, defocus_disk_v),
            (uint32_t)__builtin_offsetof(RenderParams, background)};
        uint32_t o = off[q];
        asm volatile("" : "+s"(o));
        typedef const __attribute__((address_space(4))) unsigned char* KArg;
        const KArg base = (KArg)__builtin_amdgcn_kernarg_segment_ptr();
        const __attribute__((address_space(4))) double* dp = (const __attribute__((address_space(4))) double*)(base + o);
        return mk((R)dp[0], (R)dp[1], (R)dp[2]);
    }
}

// Material of a hit, as the shading step needs it.
template <typename R>
struct MatV {
    uint32_t kind = 0, tex = 0;
    R param = R(0);
    bool solid = false;  // f32 kernel: `color` is the (SolidColor) texture
    V<R> color;
};

template <bool COMPACT> struct StackEntry { using type = int32_t; };
template <> struct StackEntry<true> { using type = uint16_t; };

// RenderParams must stay the FIRST by-value parameter (kernarg offset 0): the f64 cam3 reads the camera
// vectors straight from the kernarg segment at offsetof(RenderParams, ...) (the exact earth / C5 parity
// cases, whose cameras are off the origin, catch a reordering).
template <typename R, class G, int MAXD, bool EXACT, bool LDS_SCENE, int KFLAGS = 0, class SIG = NoSig>
__global__ void __launch_bounds__(BLOCK, (min_waves_per_simd<R, G, MAXD, SIG>(KFLAGS)))
render_kernel(const RenderParams p, const DSceneView<R> gsc) {
    constexpr bool PROF = (KFLAGS & KF_PROF) != 0;
    constexpr bool PERLIN = (KFLAGS & KF_PERLIN) != 0;
    constexpr bool FLAT = (KFLAGS & KF_FLAT) != 0;
    static_assert(!FLAT || (MAXD <= 0 && !PERLIN), "KF_FLAT is a world-list / world-BVH variant");
    // ChaCha8 persistent-lane loop (MAXD >= 0): the rejection samplers run where the wave is converged
    // and refill every lane with room (rejection_wave) instead of the loop head's top-up, for the
    // plane-only exact variants and the f32 kernels: C5 f64 191.3 -> 187.5 ms, C5 f32 65.8 -> 63.6 ms;
    // the textured earth's every-slot variant measured +4 % with them and keeps the top-up
    constexpr bool RWAVE = NRT_RIUS_WAVE && G::uses_lds && MAXD >= 0 && ((KFLAGS & KF_PLANES) != 0 || sizeof(R) == 4);
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // PROF slots: 0 iterations, 1 camera, 2 trace, 3 shade (= 5 + 6 + 7), 5 record + material,
    // 6 Philox block (+ sample claim), 7 scatter / camera ray + accumulate
    __shared__ unsigned long long prof[PROF ? BLOCK / 64 : 1][NPROF];
    if constexpr (PROF) {
        if (threadIdx.x < (BLOCK / 64) * NPROF) prof[threadIdx.x / NPROF][threadIdx.x % NPROF] = 0;
        __syncthreads();
    }
    const uint32_t wave = threadIdx.x / 64;
    auto stamp = [&]() -> unsigned long long { return PROF ? __builtin_amdgcn_s_memtime() : 0ull; };
    auto leader = [&]() {  // first active lane of the wave
        return (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x) == threadIdx.x;
    };
    auto flush_prof = [&]() {
        if constexpr (PROF) {
            if (leader()) {
                for (int c = 0; c < NPROF; ++c)
                    if (c != 4) atomicAdd(&p.counters[c], prof[wave][c]);
                atomicAdd(&p.counters[4], 1ull);
            }
        }
    };
    // dynamic LDS: [ChaCha8 ring + pixel sums (+ claim staging) | Philox pool][world-BVH stack][staged scene]
    constexpr uint32_t ring_bytes = G::uses_lds ? RING * BLOCK * sizeof(uint2) : 0;
    const uint32_t acc_bytes = G::exact_stream ? chacha_lds_bytes(p.exact_stage) - ring_bytes
                                               : philox_pool_bytes<MAXD>(p.wave_pixels);
    // world-BVH stack (f32 kernels): the tree's bound + 1 entries (16-bit refs of the compact tree)
    using StackT = typename StackEntry<SIG::bvh == WBVH_COMPACT>::type;
    const uint32_t stack_bytes =
        (MAXD < 0 || SIG::lstack) ? (gsc.wbvh_stack + 1u) * BLOCK * (uint32_t)sizeof(StackT) : 0u;
    StackT* stack = stack_bytes ? (StackT*)(lds + ring_bytes + acc_bytes) + threadIdx.x : nullptr;
    DSceneView<R> sc = gsc;
    if constexpr (LDS_SCENE) sc = stage_scene(gsc, lds + ring_bytes + acc_bytes + stack_bytes, wprim_lds_stride(MAXD));

    G g;
    constexpr bool CAM_RELOAD = NRT_CAM_RELOAD || (sizeof(R) == 4 && min_waves_per_simd<R, G, MAXD, SIG>(KFLAGS) >= 7);
    // Camera vectors (camera.rs:205-227) q = 0..6: top_left, delta_u, delta_v, look_from,
    // disk_u, disk_v, background (f32: the host-rounded copies, kernel arguments in SGPRs)
    auto cam = [&](int q) -> V<R> {
        const double* d = q == 0 ? p.top_left : q == 1 ? p.pixel_delta_u : q == 2 ? p.pixel_delta_v
                        : q == 3 ? p.look_from : q == 4 ? p.defocus_disk_u : q == 5 ? p.defocus_disk_v
                        : p.background;
        return cam3<R, CAM_RELOAD>(p, q, d);
    };
    const uint32_t wv = __builtin_amdgcn_readfirstlane(wave);  // wave-uniform values live in SGPRs

    uint32_t b = 0;  // bounces of this path
    bool bounced = false;
    Ray<R> ray;
    V<R> tp = mk(R(1), R(1), R(1));
    uint4 w = make_uint4(0u, 0u, 0u, 0u);  // Philox: this segment's block

    auto albedo = [&](const MatV<R>& m, const Rec<R>& h) {
        if constexpr (FLAT) {
            return m.color;  // every texture is a SolidColor
        } else {
            if (m.solid) return m.color;
            R u = h.u, v = h.v;
            if (MAXD <= 0 && u == R(UV_DEFERRED)) sphere_uv(h, u, v);
            return tex_color<R, PERLIN, (KFLAGS & KF_TEXPAL) != 0>(sc, m.tex, u, v, h.p);
        }
    };

    auto material = [&](uint32_t mat) {  // the material table is LDS-resident: re-reading is cheap
        MatV<R> m;
        if constexpr (EXACT) {
            const DMaterial dm = sc.materials[mat];
            m.kind = dm.kind;
            m.tex = dm.texture;
            m.param = (R)dm.param;
        } else {
            const DMatFast dm = sc.mats_fast[mat];
            m.kind = dm.kind;
            m.tex = dm.texture;
            m.param = dm.param;
            m.solid = dm.solid != 0;
            m.color = mk(dm.color[0], dm.color[1], dm.color[2]);
        }
        return m;
    };

    // The part of get_ray_color (camera.rs:269-300) before the scatter, after the
    // closest-hit query of `ray` (`traced` false: the depth cap returned black, Q6):
    // the hit record and material, and the radiance `contrib` added when the path
    // ends here (background on a miss, emission on a light).  Returns true when the
    // material scatters.  L = a0*(a1*(...*T)) is accumulated as a forward product tp.
    auto surface = [&](bool traced, bool hit, const HitMin<R, MAXD>& hm, Rec<R>& h, MatV<R>& m,
                       V<R>& contrib) -> bool {
        contrib = mk(R(0), R(0), R(0));
        if (!traced) return false;
        if (!hit) {
            contrib = tp * cam(6);  // background
            return false;
        }
        h = make_record<R, MAXD, EXACT, FLAT, LDS_SCENE, (KFLAGS & KF_PLANES) != 0>(sc, ray, hm);
        m = material(h.mat);
        if (m.kind == MAT_DIFFUSE_LIGHT) {  // emit (diffuse_light.rs:62-75), no scatter
            const R k = bounced ? m.param : R(1.0);
            contrib = tp * (k * albedo(m, h));
            return false;
        }
        return true;
    };

    // Material::scatter (lambertian.rs:39-55, metal.rs:73-91, dielectric.rs:39-67)
    // into the next `ray`; false when a metal absorbs the ray (emitted = 0).  The
    // material is read again here rather than kept live across the RNG block.
    // rs_pre: the unit-sphere draw already made by rejection_wave (RWAVE)
    auto scatter_ray = [&](const Rec<R>& h, bool have_rs = false, V<R> rs_pre = V<R>{}) -> bool {
        const MatV<R> m = material(h.mat);
        V<R> dir;
        V<R> att = mk(R(1), R(1), R(1));
        bool scattered = true;
        if (m.kind == MAT_DIELECTRIC) {
            const R ri = h.front ? fast_div(R(1.0), m.param) : m.param;
            const V<R> unit = normalize(ray.d);
            const R cos_theta = fmin(dot(-unit, h.n), R(1.0));
            const R sin_theta = fast_sqrt(R(1.0) - cos_theta * cos_theta);
            bool refl = ri * sin_theta > R(1.0);
            if (!refl) {
                R r;
                if constexpr (G::exact_stream) r = draw<R>(g, R(0.0), R(1.0));
                else r = u01<R>(w.x);
                refl = reflectance(cos_theta, ri) > r;
            }
            dir = refl ? reflect(unit, h.n) : refract(unit, h.n, ri);
        } else {
            V<R> rs;
            if constexpr (G::exact_stream) rs = have_rs ? rs_pre : random_in_unit_sphere<R>(g);
            else rs = unit_ball_inverse<R>(w.x, w.y, w.z);
            if (m.kind == MAT_LAMBERTIAN) {
                dir = h.n + rs;
                if (fabs(dir.x) < R(1e-8) && fabs(dir.y) < R(1e-8) && fabs(dir.z) < R(1e-8)) dir = h.n;
            } else {  // metal: draws even when fuzz = 0 (Q5)
                dir = vfma(m.param, rs, normalize(reflect(ray.d, h.n)));
                scattered = dot(dir, h.n) > R(0.0);
            }
            if (scattered) att = albedo(m, h);
        }
        if (!scattered) return false;
        tp = tp * att;
        ray.o = h.p;
        ray.d = dir;
        if constexpr (MAXD > 0) {  // world modes need no 1/d here, nor the exact kernel's walks
            if (!EXACT || !(p.exact_all || p.exact_wbvh)) prep_ray<R, EXACT>(ray);
        }
        bounced = true;
        ++b;
        return true;
    };

    if constexpr (G::exact_stream) {
        // Persistent lanes: the grid holds as many workgroups as stay resident, each lane renders
        // pixel after pixel (its samples in order, as the reference), and a lane whose pixel is
        // done takes the next one, so no lane idles while its wave's slowest pixel finishes:
        // pixels differ widely in path work (a light's pixels end every path at once), and a
        // wave used to run to its slowest pixel (C4 f64 28.7 -> 15.6 ms at spp 16).  The pixels
        // past the grid's first round come from per-XCD counters over contiguous eighths of them
        // (as the Philox groups: an XCD's waves work on one image region, whose texels and nodes
        // its L2 then holds; one global counter cost the textured earth 4 %), one atomic per wave
        // and refill.  A pixel's result depends on its index alone (its ChaCha8 stream and
        // sample order), never on which lane ran it.
        uint32_t i = p.pixel_begin + blockIdx.x * BLOCK + threadIdx.x;
        bool have = i < p.pixel_end;
        uint32_t x = 0, y = 0;
        double* const pacc = (double*)(lds + ring_bytes) + threadIdx.x;  // this lane's pixel sums, BLOCK apart
        uint32_t s = 0;  // next sample of the pixel
        auto start_pixel = [&]() {
            x = i % p.width;
            y = p.row_offset + (i / p.width) * p.row_stride;
            g.init((uint64_t)y * p.width + x, G::uses_lds ? (uint2*)lds + threadIdx.x : nullptr);  // stream (camera.rs:320-323)
            pacc[0] = pacc[BLOCK] = pacc[2 * BLOCK] = 0.0;
            s = 0;
        };
        // claim staging (STG_SLOTS): this wave's slots, each STG_PX x 3 floats then (left, first, size)
        const bool staging = p.exact_stage != 0u;  // (host: the LDS holds the slots only then)
        uint32_t* const stg = (uint32_t*)(lds + ring_bytes + 3u * BLOCK * (uint32_t)sizeof(double)) + wv * STG_WAVE_WORDS;
        auto stg_meta = [&](uint32_t slot) { return stg + STG_SLOTS * STG_PX * 3u + slot * 3u; };
        uint32_t stg_free = (1u << STG_SLOTS) - 1u;  // uniform: free slots
        uint32_t rslot = NO_STG, rfirst = 0;        // uniform: slot and first pixel of the reservoir's claim
        uint32_t stag = NO_STG;                     // this lane's pixel: slot << 8 | its place in the claim
        uint32_t ended = NO_STG;                    // slot whose last pixel this lane just finished
        auto finish_pixel = [&]() {
            const double spp = (double)p.spp;
            const float c0 = (float)(pacc[0] / spp), c1 = (float)(pacc[BLOCK] / spp), c2 = (float)(pacc[2 * BLOCK] / spp);
            if (stag != NO_STG) {
                const uint32_t slot = stag >> 8;
                float* d = (float*)stg + slot * (STG_PX * 3u) + (stag & 0xFFu) * 3u;
                d[0] = c0;
                d[1] = c1;
                d[2] = c2;
                if (atomicSub(stg_meta(slot), 1u) == 1u) ended = slot;  // the claim's last pixel
                stag = NO_STG;
            } else {
                float* o = p.out + 3ull * i;
                o[0] = c0;
                o[1] = c1;
                o[2] = c2;
            }
        };
        const uint32_t dyn0 = p.pixel_begin + gridDim.x * BLOCK;  // first pixel handed out by the counters
        // uniform, after the lanes' finish_pixel: write out the claims whose last pixel ended
        auto flush_claims = [&]() {
            if (!staging) return;
            uint64_t fm = __ballot(ended != NO_STG);
            if (fm == 0ull) return;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const uint32_t lane = threadIdx.x & 63u;
            while (fm) {
                const uint32_t l = (uint32_t)__builtin_ctzll(fm);
                fm &= fm - 1ull;
                const uint32_t slot = __builtin_amdgcn_readlane(ended, l);
                const uint32_t first = stg_meta(slot)[1], nf = 3u * stg_meta(slot)[2];
                const float* d = (const float*)stg + slot * (STG_PX * 3u);
                float* o = p.out + 3ull * (dyn0 + first);
                for (uint32_t k = lane; k < nf; k += 64u) o[k] = d[k];
                stg_free |= 1u << slot;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            ended = NO_STG;
        };
        const uint32_t ndyn = p.pixel_end > dyn0 ? p.pixel_end - dyn0 : 0u;
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        uint32_t qk = 0;  // counters found exhausted (wave-uniform; QUEUE_HEADS: no pixel left)
        // The wave's reservoir (uniform): pixels [rb, rb + rn) claimed but not yet started.  Lanes
        // free up one at a time, so a claim of only the lanes asking cost one counter atomic per
        // pixel and a wait on its return (a device-scope atomic executes at memory: ~35 B of HBM
        // writes each, C4 f64 at spp 256: 35 of its 55 MB per launch with claims of 1); a claim takes
        // at least p.exact_claim pixels and later asks are served from the reservoir -- while the
        // head has more than one round of its lanes' pixels left (left: what the last claim saw);
        // then only what the lanes ask, so no reservoir holds pixels into the tail (guided claims)
        uint32_t rb = 0, rn = 0;
        uint32_t left = 0xFFFFFFFFu;  // uniform: pixels the head had left after this wave's last claim
        const uint32_t guide = gridDim.x * (BLOCK / QUEUE_HEADS);  // one round of a head's lanes
        auto next_pixel = [&](bool need) -> bool {  // uniform; true: this lane got a pixel
            const uint64_t m = __ballot(need);
            if (m == 0ull) return false;
            const uint32_t cnt = (uint32_t)__popcll(m);
            if (rn == 0 && qk < QUEUE_HEADS) {
                const uint32_t want = max(cnt, left > guide ? p.exact_claim : 1u);
                uint32_t base = 0, got = 0, rest = 0;
                if (leader()) {
                    for (; qk < QUEUE_HEADS; ++qk) {
                        const uint32_t xh = (xcc + qk) & (QUEUE_HEADS - 1u);
                        const uint32_t lo = (uint32_t)((uint64_t)xh * ndyn / QUEUE_HEADS);
                        const uint32_t n = (uint32_t)((uint64_t)(xh + 1u) * ndyn / QUEUE_HEADS) - lo;
                        if (n == 0) continue;
                        const uint32_t t = atomicAdd(p.queue + xh * QUEUE_STRIDE, want);
                        if (t < n) {
                            base = lo + t;
                            got = min(want, n - t);
                            rest = qk == 0 ? n - t - got : 0u;  // (a head of another XCD: its tail)
                            break;
                        }
                    }
                }
                rb = __builtin_amdgcn_readfirstlane(base);
                rn = __builtin_amdgcn_readfirstlane(got);
                left = __builtin_amdgcn_readfirstlane(rest);
                qk = __builtin_amdgcn_readfirstlane(qk);
                rslot = NO_STG;
                if (staging && rn != 0 && rn <= STG_PX && stg_free != 0u) {  // a staging slot for the claim
                    rslot = (uint32_t)__builtin_ctz(stg_free);
                    rfirst = rb;
                    stg_free &= ~(1u << rslot);
                    if ((threadIdx.x & 63u) == 0u) {
                        uint32_t* mt = stg_meta(rslot);
                        mt[0] = rn;
                        mt[1] = rb;
                        mt[2] = rn;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                }
            }
            if (rn == 0) return false;
            const uint32_t base = rb, grant = min(cnt, rn);
            rb += grant;
            rn -= grant;
            if (!need) return false;
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (rank >= grant) return false;  // (the next round asks again)
            i = dyn0 + base + rank;
            stag = rslot == NO_STG ? NO_STG : (rslot << 8) | (base + rank - rfirst);
            have = true;
            start_pixel();
            return true;
        };
        if (have) start_pixel();

        // Camera::get_ray (camera.rs:244-267) of the pixel's next sample; false when all are done.
        // (split in two around the disk draw for camera_ray_wave)
        auto camera_point = [&]() -> V<R> {
            g.start_sample(s);
            ++s;
            R ox = R(0), oy = R(0);
            if (p.spp > 1) {
                g.ensure(2);
                ox = draw_taken<R>(g, R(-0.5), R(0.5));
                oy = draw_taken<R>(g, R(-0.5), R(0.5));
            }
            return vfma((R)y + oy, cam(2), vfma((R)x + ox, cam(1), cam(0)));
        };
        auto camera_finish = [&](V<R> point, V<R> disk) {
            ray.o = vfma(disk.y, cam(5), vfma(disk.x, cam(4), cam(3)));
            ray.d = point - ray.o;
            ray.time = draw<R>(g, R(0.0), R(1.0));
            if (!EXACT || !(p.exact_all || p.exact_wbvh)) prep_ray<R, EXACT>(ray);  // 1/d: box tests only
            tp = mk(R(1), R(1), R(1));
            b = 0;
            bounced = false;  // Ray::bounce flag (Q4): 0 for camera rays
        };
        // the camera rays of the lanes with `go` set, the disk drawn where the wave is converged
        // (RWAVE: rejection_wave)
        auto camera_ray_wave = [&](bool go) {
            V<R> point = mk(R(0), R(0), R(0));
            if (go) point = camera_point();
            const V<R> disk = rejection_wave<R, 2>(g, go);
            if (go) camera_finish(point, disk);
        };
        auto camera_ray = [&]() -> bool {
            if (s >= p.spp) return false;
            const V<R> point = camera_point();
            const V<R> disk = random_in_unit_disk<R>(g);
            camera_finish(point, disk);
            return true;
        };
        // One shading step; true when the path continues with a new `ray`, otherwise
        // the sample's radiance has been added to the pixel sum.
        auto shade = [&](bool traced, bool hit, const HitMin<R, MAXD>& hm) -> bool {
            const unsigned long long s0 = stamp();
            Rec<R> h;
            MatV<R> m;
            V<R> contrib;
            const bool scatter = surface(traced, hit, hm, h, m, contrib);
            const unsigned long long s1 = stamp();
            bool cont;
            if constexpr (RWAVE) {
                // lambertian and metal draw the unit-sphere vector first thing in scatter
                // (dielectrics draw no vector): drawn here, where the wave is converged
                const V<R> rs = rejection_wave<R, 3>(g, scatter && m.kind != MAT_DIELECTRIC);
                cont = scatter && scatter_ray(h, m.kind != MAT_DIELECTRIC, rs);
            } else {
                cont = scatter && scatter_ray(h);
            }
            if (!cont) {  // metal absorption adds contrib = 0
                pacc[0] += (double)contrib.x;  // (the reference's f64 sum, in sample order)
                pacc[BLOCK] += (double)contrib.y;
                pacc[2 * BLOCK] += (double)contrib.z;
            }
            if constexpr (PROF) {
                const unsigned long long s2 = stamp();
                if (leader()) {
                    atomicAdd(&prof[wave][5], s1 - s0);
                    atomicAdd(&prof[wave][7], s2 - s1);
                }
            }
            return cont;
        };

        if constexpr (MAXD < 0) {
            // World-BVH mode: traversal lengths differ widely between lanes, so each lane
            // keeps its traversal state across rounds; the wave traverses until a ballot
            // shows at least p.wave_wait lanes finished, then only those lanes shade and
            // start their next segment (active-ray compaction within the wave).
            static_assert(sizeof(R) == 4, "world-BVH mode is an f32-kernel mode");
            WbvhTrav ts{WBVH_DONE, WBVH_NO_LEAF, 0u, INFINITY, -1, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            bool active = have && camera_ray();
            auto begin = [&]() {
                // depth cap: no query, the lane waits to be shaded as black (Q6)
                wbvh_begin(ts, b < p.max_bounces ? wbvh_root(gsc) : WBVH_DONE, ray);
            };
            if (active) begin();
            const uint32_t wait_min = p.wave_wait ? p.wave_wait : 1u;
            while (true) {
                const unsigned long long t0 = stamp();
                const uint64_t am = __ballot(active);  // (the Philox loop's one-ballot trips, below)
                while (true) {
                    const bool going = active && ts.busy();
                    const uint64_t gm = __ballot(going);
                    if (gm == 0ull || (uint32_t)__popcll(am & ~gm) >= wait_min) break;
                    if (going) wbvh_step<R, FLAT, SIG>(ts, gsc, ray, stack);
                }
                const unsigned long long t1 = stamp();
                if constexpr (NRT_CHACHA_TOPUP) {
                    if (active) rng_top_up(g);
                }
                if (active && !ts.busy()) {
                    HitMin<R, MAXD> hm;
                    hm.t = ts.t_best;
                    hm.prim = (uint32_t)ts.best;
                    hm.depth = 0;
                    if (!shade(b < p.max_bounces, ts.best >= 0, hm)) active = camera_ray();
                    if (active) begin();
                }
                if constexpr (PROF) {
                    const unsigned long long t2 = stamp();
                    if (leader()) {
                        atomicAdd(&prof[wave][0], 1ull);
                        atomicAdd(&prof[wave][2], t1 - t0);
                        atomicAdd(&prof[wave][3], t2 - t1);
                    }
                }
                if (have && !active) {  // the pixel's last sample has ended
                    finish_pixel();
                    have = false;
                }
                flush_claims();
                if (next_pixel(!have)) {
                    active = camera_ray();
                    begin();
                }
                if (__ballot(active) == 0ull) break;
            }
        } else if constexpr (SIG::persist) {
            // Exact world walk kept across shading rounds (XWalk): the wave runs walk trips until a
            // ballot shows p.wave_wait lanes (default XWALK_WAIT) done, then those lanes run the
            // candidate tests, shade and begin their next segment, as the f32 world-BVH loop above.
            static_assert(EXACT && sizeof(R) == 8 && SIG::lstack, "persistent exact walk: f64, LDS stack");
            // the prefiltered walk (plane-only scenes) or the unfiltered one (EXACT_SIG_WORLD: spheres)
            using XW = typename TypeIf<SIG::exact == EXACT_SIG_WORLD, XWalkU<R>, XWalk>::type;
            XW xw;
            xw.ts.node = WBVH_DONE;
            xw.ts.leaf = WBVH_NO_LEAF;
            bool active = false;
            bool want = have;  // the lane starts its pixel's next sample (one camera_ray call site)
            auto begin = [&]() { xwalk_begin(xw, sc, ray, b < p.max_bounces); };
            const uint32_t wait_min = p.wave_wait ? p.wave_wait : (uint32_t)XWALK_WAIT;
            while (true) {
                if (want) {
                    active = camera_ray();  // (s < spp)
                    begin();
                    want = false;
                }
                const unsigned long long t0 = stamp();
                const uint64_t am = __ballot(active);
                while (true) {
                    const bool going = active && xw.busy();
                    const uint64_t gm = __ballot(going);
                    if (gm == 0ull || (uint32_t)__popcll(am & ~gm) >= wait_min) break;
                    if (going) xwalk_trip<R>(xw, sc, stack, ray);
                }
                const unsigned long long t1 = stamp();
                if (active && !xw.busy()) {
                    HitMin<R, MAXD> hm;
                    const bool traced = b < p.max_bounces;  // depth cap returns black (Q6)
                    const bool hit = traced && xwalk_finish<R, MAXD>(xw, sc, ray, hm, stack);
                    if (shade(traced, hit, hm)) {
                        begin();
                    } else {
                        active = false;
                        want = s < p.spp;
                    }
                }
                if constexpr (PROF) {
                    const unsigned long long t2 = stamp();
                    if (leader()) {
                        atomicAdd(&prof[wave][0], 1ull);
                        atomicAdd(&prof[wave][2], t1 - t0);
                        atomicAdd(&prof[wave][3], t2 - t1);
                    }
                }
                if (have && !active && !want) {  // the pixel's last sample has ended
                    finish_pixel();
                    have = false;
                }
                flush_claims();
                if (next_pixel(!have)) want = true;
                if (__ballot(active || want) == 0ull) break;
            }
        } else {
            bool fresh = true;
            while (true) {
                if constexpr (NRT_EXACT_SETPRIO > 0) __builtin_amdgcn_s_setprio(0);
                if (have && fresh && s >= p.spp) {  // the pixel's last sample has ended
                    finish_pixel();
                    have = false;
                }
                flush_claims();
                next_pixel(!have);
                if (__ballot(have) == 0ull) break;  // (no lane holds a pixel: the counters are exhausted)
                if (!have) continue;
                const unsigned long long t0 = stamp();
                if constexpr (NRT_CHACHA_TOPUP && !RWAVE) rng_top_up(g);
                if constexpr (RWAVE) {
                    camera_ray_wave(fresh);  // (s < spp: a sample is left)
                    fresh = false;
                } else if (fresh) {
                    camera_ray();  // (s < spp: a sample is left)
                    fresh = false;
                }
                const unsigned long long t1 = stamp();
                unsigned long long t2 = t1, tmid = 0;
                HitMin<R, MAXD> hm;
                bool hit = false;
                const bool traced = b < p.max_bounces;  // depth cap returns black (Q6)
                if (traced) {
                    // world list: the global tables through the scalar cache; records read LDS
                    hit = trace<R, MAXD, EXACT, FLAT, (KFLAGS & KF_PLANES) != 0, SIG>(
                        MAXD == 0 ? gsc : sc, ray, hm, stack, p.exact_all != 0, p.exact_wbvh != 0, p.exact_pf,
                        p.exact_thread != 0, PROF ? prof[wave] : nullptr, PROF ? &tmid : nullptr);
                    t2 = stamp();
                    if constexpr (PROF) {
                        if (leader() && tmid) atomicAdd(&prof[wave][6], t2 - tmid);  // phase 2 (f64 candidate tests)
                    }
                }
                if constexpr (NRT_EXACT_SETPRIO > 0) __builtin_amdgcn_s_setprio(NRT_EXACT_SETPRIO);
                fresh = !shade(traced, hit, hm);
                if constexpr (PROF) {
                    const unsigned long long t3 = stamp();
                    if (leader()) {
                        atomicAdd(&prof[wave][0], 1ull);
                        atomicAdd(&prof[wave][1], t1 - t0);
                        atomicAdd(&prof[wave][2], t2 - t1);
                        atomicAdd(&prof[wave][3], t3 - t2);
                    }
                }
            }
        }
        flush_prof();
    } else {
        // ------------------------------------------------ Philox: per-wave sample pool
        // Persistent waves.  A wave takes groups of P consecutive pixels from a global
        // queue (one atomic per group) into a ring of NS LDS slots and hands the
        // P x spp samples of a group (index s * P + j; pixels past the end of the launch
        // are padding samples that end at once) to whichever lane is free.  A group's
        // pixel sums are written out when its last sample finishes; the next group goes
        // into the slot after the one being claimed from, which must have been flushed:
        // with two slots one long path of the previous group starves the wave's lanes
        // (world BVH: long and short paths mix), so the BVH modes keep four.
        constexpr uint32_t NS = philox_slots<MAXD>();
        constexpr int SETPRIO = (KFLAGS & KF_TEXPAL) ? NRT_SETPRIO_TEX : NRT_SETPRIO;
        constexpr uint32_t GRAB = FLAT && MAXD < 0 ? (uint32_t)NRT_GRAB_FLAT : (uint32_t)NRT_GRAB;  // groups per queue atomic
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t P = p.wave_pixels, logP = p.wave_pixels_log2;
        const uint32_t GS = P * p.spp;  // samples per group (host: < 2^32)
        // LDS per wave: NS slots x P pixel sums (3 x f64) and NS x P packed coordinates x | y << 16
        double* acc = (double*)(lds + ring_bytes) + wv * NS * P * 3u;
        uint32_t* slot_xy = (uint32_t*)(lds + ring_bytes + (BLOCK / 64) * NS * P * 3u * sizeof(double)) + wv * NS * P;
        constexpr uint32_t NO_GROUP = 0xFFFFFFFFu, PAD_XY = 0xFFFFFFFFu;
        uint32_t gids[NS], dones[NS];  // group held by each slot and its finished samples (wave-uniform)
#pragma unroll
        for (uint32_t k = 0; k < NS; ++k) {
            gids[k] = NO_GROUP;
            dones[k] = 0;
        }
        uint32_t cs = 0, next = GS;                 // claiming from slot cs at index next
        bool ready = false;                         // slot (cs + 1) % NS holds a group not yet claimed from
        bool exhausted = false;                     // the queue is empty
        // Group distribution: per-XCD queue heads.  Head x hands out the x-th contiguous eighth
        // of the groups, and a wave pulls from its own XCD's head first (then the next heads in
        // turn), so the XCD's waves work on neighbouring groups at any moment (the rays of a small
        // image region: node, texel and framebuffer lines shared in the XCD's L1s and L2), and no
        // head is contended by more than one XCD's waves until the tail.  A device-scope atomic
        // executes at the memory side (one ~32-B HBM write each; with one per group they were
        // 45 % of the C5 launch's HBM writes): a wave takes GRAB consecutive groups per atomic
        // (more per grab spreads the XCD's waves over a larger image region: guided runs of up
        // to 25 groups cost C4 +50 %, C5 +12 %), and skips heads an agent-scope load already
        // shows empty (a stale value only lags).  The XCD id only places work: never correctness.
        uint32_t xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
        uint32_t qk = 0;              // heads found empty so far (wave-uniform)
        uint32_t lcur = 0, lend = 0;  // groups of the last grab not yet taken (wave-uniform)
        auto fetch = [&](uint32_t r) {              // uniform: take the next group into (free) slot r
            uint32_t gid = 0xFFFFFFFFu;
            if (GRAB > 1 && lcur < lend) {
                gid = lcur++;
            } else {
                if (lane == 0) {
                    for (; qk < QUEUE_HEADS; ++qk) {
                        const uint32_t x = (xcc + qk) & (QUEUE_HEADS - 1u);
                        const uint32_t lo = (uint32_t)((uint64_t)x * p.groups / QUEUE_HEADS);
                        const uint32_t n = (uint32_t)((uint64_t)(x + 1u) * p.groups / QUEUE_HEADS) - lo;
                        unsigned int* head = p.queue + x * QUEUE_STRIDE;
                        if (n == 0 || (NRT_PROBE_HEAD && __hip_atomic_load(head, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT) >= n))
                            continue;
                        const uint32_t k = qk ? 1u : GRAB;  // a steal takes one group
                        const uint32_t t = atomicAdd(head, k);
                        if (t < n) {
                            gid = lo + t;
                            lcur = gid + 1u;
                            lend = lo + min(t + k, n);
                            break;
                        }
                    }
                }
                gid = __builtin_amdgcn_readlane(gid, 0);
                qk = __builtin_amdgcn_readlane(qk, 0);
                if (GRAB > 1) {
                    lcur = __builtin_amdgcn_readlane(lcur, 0);
                    lend = __builtin_amdgcn_readlane(lend, 0);
                }
            }
            exhausted = gid == 0xFFFFFFFFu;  // (plain stores and selects: the flags stay in registers)
            if (exhausted) return;
            const uint32_t base = p.pixel_begin + gid * P;
            double* a = acc + r * P * 3u;
            uint32_t* xy = slot_xy + r * P;
            for (uint32_t k = lane; k < P; k += 64u) {
                a[3 * k] = a[3 * k + 1] = a[3 * k + 2] = 0.0;
                const uint32_t il = base + k;
                xy[k] = il >= p.pixel_end ? PAD_XY
                                          : (il % p.width) | ((p.row_offset + (il / p.width) * p.row_stride) << 16);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (uint32_t k = 0; k < NS; ++k) {
                gids[k] = k == r ? gid : gids[k];
                dones[k] = k == r ? 0u : dones[k];
            }
            ready = true;
        };
        auto flush = [&](uint32_t gid, uint32_t r) {  // uniform: the group's last sample has finished
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            const double* a = acc + r * P * 3u;
            const double spp = (double)p.spp;
            const uint32_t base = p.pixel_begin + gid * P;
            // the group's pixels are 3 x P contiguous floats in LDS and in the framebuffer:
            // one coalesced dword per lane (16-B stores cost the shading loop a spill)
            const uint32_t nf = 3u * min(P, p.pixel_end - base);
            float* o = p.out + 3ull * base;
            for (uint32_t l = lane; l < nf; l += 64u) o[l] = (float)((a[l] * p.acc_unscale) / spp);
        };

        uint32_t slot = 0, j = 0, cur = 0;  // ring slot, pixel in the group, sample index of this lane's path
        uint32_t pxy = 0;                   // this path's pixel, x | y << 16
        bool alive = false;                 // the lane holds a path
        bool killed = false;                // absorbed by a metal (or padding): black, ends at the next shading step
        auto pixel_index = [&]() { return (pxy >> 16) * p.width + (pxy & 0xFFFFu); };  // RNG stream (camera.rs:320-323)

        // Camera::get_ray (camera.rs:244-267) for sample `cur` of pixel pxy; w holds its
        // block (pixel, sample, 0).
        auto camera = [&]() {
            const uint32_t px = pxy & 0xFFFFu, py = pxy >> 16;
            R ox = R(0), oy = R(0);
            if (p.spp > 1) {
                if constexpr (sizeof(R) == 4) {
                    ox = u12(w.x) - 1.5f;
                    oy = u12(w.y) - 1.5f;
                } else {
                    ox = u01<R>(w.x) - R(0.5);
                    oy = u01<R>(w.y) - R(0.5);
                }
            }
            const V<R> point = vfma((R)py + oy, cam(2), vfma((R)px + ox, cam(1), cam(0)));
            if (p.defocus) {
                const uint4 wd = G::template block_at<R>(pixel_index(), cur, G::template defocus_step<R>());
                const V<R> disk = unit_disk_inverse<R>(wd.x, wd.y);
                ray.o = vfma(disk.y, cam(5), vfma(disk.x, cam(4), cam(3)));
            } else {
                ray.o = cam(3);  // zero disk: the draws would only scale zero vectors
            }
            ray.d = point - ray.o;
            ray.time = u01<R>(w.z);
            prep_ray<R, EXACT>(ray);
            tp = mk(R(1), R(1), R(1));
            b = 0;
            bounced = false;  // Ray::bounce flag (Q4): 0 for camera rays
            killed = false;
        };

        WbvhTrav ts{WBVH_DONE, WBVH_NO_LEAF, 0u, INFINITY, -1, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        auto begin = [&]() {  // world-BVH mode; depth cap / absorbed: no query (Q6)
            if constexpr (MAXD < 0) wbvh_begin(ts, (!killed && b < p.max_bounces) ? wbvh_root(gsc) : WBVH_DONE, ray);
        };
        const uint32_t wait_min = p.wave_wait ? p.wave_wait : 1u;

        while (true) {
            // Group bookkeeping at the loop head, where little state is live: write out
            // finished groups, and take the next group into the free slot as soon as
            // fewer than a wave's worth of samples are left to claim.
#pragma unroll
            for (uint32_t k = 0; k < NS; ++k) {
                if (gids[k] != NO_GROUP && dones[k] == GS) {
                    flush(gids[k], k);
                    gids[k] = NO_GROUP;
                }
            }
            if constexpr (NS == 2) {
                if (!exhausted && !ready && GS - next < NRT_FETCH_AHEAD && (cs ? gids[0] : gids[1]) == NO_GROUP) fetch(cs ^ 1u);
            } else if (!exhausted && !ready && GS - next < NRT_FETCH_AHEAD) {
                const uint32_t r = (cs + 1u) & (NS - 1u);
                bool free = false;
#pragma unroll
                for (uint32_t k = 0; k < NS; ++k) free |= k == r && gids[k] == NO_GROUP;
                if (free) fetch(r);
            }
            if (exhausted && !ready && GS - next == 0u && __ballot(alive) == 0ull) break;
            if constexpr (SETPRIO > 0) __builtin_amdgcn_s_setprio(0);
            const unsigned long long t0 = stamp();
            HitMin<R, MAXD> hm;
            bool hit = false, sh, traced;
            if constexpr (MAXD < 0) {
                // World-BVH mode: lanes keep their traversal state across rounds; the wave
                // traverses until a ballot shows >= p.wave_wait lanes finished, then only
                // those lanes shade (active-ray compaction within the wave).
                static_assert(sizeof(R) == 4, "world-BVH mode is an f32-kernel mode");
                // the finished lanes as scalar mask arithmetic: alive does not change inside the loop,
                // so one ballot per trip (the busy lanes) instead of two (C4 34.3 -> 33.9 ms)
                const uint64_t am = __ballot(alive);
                while (true) {
                    const bool going = alive && ts.busy();
                    const uint64_t gm = __ballot(going);
                    if (gm == 0ull || (uint32_t)__popcll(am & ~gm) >= wait_min) break;
                    if (going) wbvh_step<R, FLAT, SIG>(ts, gsc, ray, stack, PROF ? prof[wave] : nullptr);
                }
                sh = alive && !ts.busy();
                if constexpr (PROF) {
                    if (sh) prof_event(prof[wave], PROF_ROUNDS, PROF_ROUND_LANES);
                }
                traced = sh && !killed && b < p.max_bounces;
                hm.t = ts.t_best;
                hm.prim = (uint32_t)ts.best;
                hm.depth = 0;
                hit = ts.best >= 0;
            } else {
                sh = alive;
                traced = alive && !killed && b < p.max_bounces;  // depth cap returns black (Q6)
                // world list: the global tables through the scalar cache; records read LDS
                if (traced)
                    hit = trace<R, MAXD, EXACT, FLAT, false, SIG>(MAXD == 0 ? gsc : sc, ray, hm, stack,
                                                                   p.exact_all != 0, p.exact_wbvh != 0, 0u,
                                                                   p.exact_thread != 0);
            }
            const unsigned long long t1 = stamp();
            if constexpr (SETPRIO > 0) __builtin_amdgcn_s_setprio(SETPRIO);  // shading at raised priority
            Rec<R> h;
            MatV<R> m;
            V<R> contrib;  // (set by surface() wherever it is read: ends implies sh)
            bool scatter = false;
            if (sh) scatter = surface(traced, hit, hm, h, m, contrib);
            const unsigned long long t2 = stamp();

            // finished samples: radiance into the pixel's LDS sum, completion counts per slot
            const bool ends = sh && !scatter;
            if (ends && (contrib.x != R(0) || contrib.y != R(0) || contrib.z != R(0))) {
                double* a = acc + (slot * P + j) * 3u;
                if constexpr (sizeof(R) == 4) {  // 2^k scaling and rint exact in f32 (host: k in range)
                    atomicAdd(a, (double)__builtin_rintf(contrib.x * p.acc_scale_f));
                    atomicAdd(a + 1, (double)__builtin_rintf(contrib.y * p.acc_scale_f));
                    atomicAdd(a + 2, (double)__builtin_rintf(contrib.z * p.acc_scale_f));
                } else {
                    atomicAdd(a, rint((double)contrib.x * p.acc_scale));
                    atomicAdd(a + 1, rint((double)contrib.y * p.acc_scale));
                    atomicAdd(a + 2, rint((double)contrib.z * p.acc_scale));
                }
            }
#pragma unroll
            for (uint32_t k = 0; k < NS; ++k) dones[k] += (uint32_t)__popcll(__ballot(ends && slot == k));

            // lanes without a path claim the next samples, in lane order: slot cs from
            // `next`, then the group waiting in slot (cs + 1) % NS
            const bool want = ends || !alive;
            const uint64_t em = __ballot(want);
            const uint32_t nwant = (uint32_t)__popcll(em);
            const uint32_t granted = min(nwant, (GS - next) + (ready ? GS : 0u));
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(em >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)em, 0u));
            const uint32_t claim = next + rank;
            const uint32_t cs0 = cs;
            next += granted;
            if (next >= GS && ready) {
                cs = NS == 2 ? cs ^ 1u : (cs + 1u) & (NS - 1u);
                next -= GS;
                ready = false;
            }
            if (want) {
                alive = rank < granted;
                if (alive) {
                    const bool second = claim >= GS;
                    slot = second ? (NS == 2 ? cs0 ^ 1u : (cs0 + 1u) & (NS - 1u)) : cs0;
                    const uint32_t idx = second ? claim - GS : claim;
                    j = idx & (P - 1u);
                    cur = idx >> logP;
                    pxy = slot_xy[slot * P + j];
                }
            }
            // this segment's block: the scatter's (pixel, sample, bounce + 1) or the
            // claimed sample's camera block (pixel', sample', 0)
            w = G::template block_at<R>(pixel_index(), cur, scatter ? b + 1u : 0u);
            const unsigned long long t3 = stamp();
            if (scatter && !scatter_ray(h)) killed = true;
            if (want && alive) {
                camera();
                killed = pxy == PAD_XY;  // padding sample: no pixel, ends at once
            }
            if ((sh || want) && alive) begin();
            if constexpr (PROF) {
                const unsigned long long t4 = stamp();
                const uint32_t busy = (uint32_t)__popcll(__ballot(sh));
                if (leader()) {
                    atomicAdd(&prof[wave][0], 1ull);
                    atomicAdd(&prof[wave][1], (unsigned long long)busy);  // lane-iterations shading a path
                    atomicAdd(&prof[wave][2], t1 - t0);
                    atomicAdd(&prof[wave][3], t4 - t1);
                    atomicAdd(&prof[wave][5], t2 - t1);
                    atomicAdd(&prof[wave][6], t3 - t2);
                    atomicAdd(&prof[wave][7], t4 - t3);
                }
            }
        }
        flush_prof();
    }
}

// First `count` next_u64 draws of a ChaCha8 / Philox stream (tests only).
template <class G>
__global__ void __launch_bounds__(BLOCK) rng_probe_kernel(uint64_t stream0, uint32_t count, uint32_t sample,
                                                          unsigned long long* out) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const uint64_t stream = stream0 + threadIdx.x;
    G g;
    g.init(stream, G::uses_lds ? (uint2*)lds + threadIdx.x : nullptr);
    g.start_sample(sample);
    for (uint32_t k = 0; k < count; ++k) out[(uint64_t)threadIdx.x * count + k] = g.next();
}

// The f32 render loop's Philox2x32-10 blocks (tests only): lane l, word k = block
// (pixel0 + l, sample, step k) as lo | hi << 32.
template <typename R = float>  // (a template: the header is in two translation units)
__global__ void __launch_bounds__(BLOCK) philox_block_probe_kernel(uint32_t pixel0, uint32_t count, uint32_t sample,
                                                                   unsigned long long* out) {
    for (uint32_t k = 0; k < count; ++k) {
        const uint4 w = Philox::block_at<R>(pixel0 + threadIdx.x, sample, k);
        out[(uint64_t)threadIdx.x * count + k] = (unsigned long long)w.x | ((unsigned long long)w.y << 32);
    }
}

}  // namespace dev
}  // namespace nrt
