// Flattened scene as it lives in HBM (one copy per GPU, uploaded once).
//
// The reference's `Arc<dyn Hitable>` tree (scene_config.rs:277-381 ->
// object.rs BVH + transforms) becomes:
//   * one node array holding every threaded BVH (the top level and one per
//     distinct instanced sub-scene, a "BLAS"), laid out depth-first so the
//     left child of an inner node is the next node and each node carries a
//     `skip` link to the first node after its subtree (END = -1 terminates
//     the tree).  Depth-first, left-before-right order is exactly the
//     reference's candidate order, so "the later candidate wins ties"
//     reproduces `if hit_l.t < hit_r.t {l} else {r}` (object.rs:109-115).
//   * primitives (sphere / quad / triangle) with the PlaneBuilder
//     precomputation (plane.rs:95-128),
//   * instances = a chain of Translate/Rotate/Scale applied outer -> inner to
//     the ray, inner -> outer to the hit point/normal (translate.rs:37-49,
//     rotate.rs:91-106, scale.rs:73-86), plus the BLAS root,
//   * materials and textures (image texels as f32 RGB, row-major).
// Layout is precision-templated: Real = double for the reference-exact
// kernel, float for the fast kernel.  Nothing here is torch-aware.
#pragma once

#ifndef __HIPCC_RTC__
#include <cstdint>
#endif

namespace nrt {

enum : uint32_t { NODE_INNER = 0, NODE_PRIM = 1, NODE_INSTANCE = 2, NODE_LIST = 3 };
// NODE_LIST (fast kernel only): a BVH subtree holding only primitives, at most
// LIST_MAX of them, collapsed into one node: its box is tested, then every
// primitive in the subtree's depth-first order, stored contiguously in the fast
// primitive array.  meta = 3 | (count-1) << 2 | first << 8.
constexpr uint32_t LIST_MAX = 8;
enum : uint32_t { PRIM_SPHERE = 0, PRIM_QUAD = 1, PRIM_TRIANGLE = 2, PRIM_BOX = 3 /* world mode only */ };
// World primitives (DPrimWorld, wruns) carry a 3-bit kind: meta = kind | material << 3
// (box headers: kind | face map << 3), runs = kind | count << 3.  World-list
// only: quads whose plane normal is a coordinate axis (PRIM_QUAD_X + axis).
constexpr uint32_t WKIND_BITS = 3, WKIND_MASK = 7;
enum : uint32_t { PRIM_QUAD_X = 4, PRIM_QUAD_Y = 5, PRIM_QUAD_Z = 6, PRIM_ABOX = 7 };
enum : uint32_t { XF_TRANSLATE = 0, XF_ROTATE = 1, XF_SCALE = 2 };
enum : uint32_t { MAT_LAMBERTIAN = 0, MAT_METAL = 1, MAT_DIELECTRIC = 2, MAT_DIFFUSE_LIGHT = 3 };
enum : uint32_t { TEX_SOLID = 0, TEX_IMAGE = 1, TEX_CHECKER = 2, TEX_NOISE = 3, TEX_MARBLE = 4 };

constexpr int32_t NODE_END = -1;
constexpr int MAX_INSTANCE_DEPTH = 4;

template <typename Real>
struct alignas(16) DNode {
    Real bmin[3];   // AABB x/y/z .min (inner nodes only)
    Real bmax[3];   // AABB x/y/z .max
    uint32_t meta;  // kind | payload << 2 (payload = prim or instance index)
    int32_t skip;   // next node after this subtree, or NODE_END
};

template <typename Real>
struct alignas(16) DPrim {
    Real a[3];  // sphere: center           plane: p
    Real b[3];  // sphere: speed            plane: u
    Real c[3];  //                          plane: v
    Real n[3];  //                          plane: normal (unit)
    Real w[3];  //                          plane: w = n / (n.n)
    Real s;     // sphere: radius           plane: d = normal.p
    uint32_t kind;
    uint32_t material;
};

// Fast kernel primitive (64 B in f32).  Plane: alpha = (point-p).(v x w),
// beta = (point-p).(w x u) (scalar triple products of plane.rs:156-157), so
// A = v x w, a0 = p.A, B = w x u, b0 = p.B are precomputed on the host in f64.
template <typename Real>
struct alignas(16) DPrimFast {
    Real n[3];  // plane: unit normal        sphere: center
    Real d;     // plane: d = normal.p       sphere: radius
    Real A[3];  // plane: v x w              sphere: speed
    Real a0;    // plane: p.A
    Real B[3];  // plane: w x u
    Real b0;    // plane: p.B
    uint32_t kind;
    uint32_t material;
    uint32_t pad[2];
};

// Fast kernel, world-space mode (instances flattened away; MAXD = 0 kernels).
// A quad/triangle reached through a Translate/Rotate/Scale chain whose
// world->object map is o' = M o + b keeps the reference's object-space
// arithmetic when its planes are pulled back to world space: n.o' = d becomes
// (M^T n).o = d - n.b, alpha = A.o' - a0 becomes (M^T A).o - (a0 - A.b), and
// t is the same in both spaces (directions are transformed, not normalised).
// The front-face sign of the reference, signum(d'.n), is signum(d.(M^T n)); the
// shading normal is the object normal mapped out by the chain's rotations only
// (Q11: Scale leaves normals alone).  Spheres qualify under translations only.
template <typename Real>
struct alignas(16) DPrimWorld {
    Real N[3];      // plane: M^T n (unnormalised)   sphere: world center at time 0
    Real D;         // plane: d - n.b                sphere: radius
    // plane: (A.x, B.x, A.y, B.y, A.z, B.z, a0', b0') with A = M^T (v x w),
    // B = M^T (w x u), a0' = a0 - (v x w).b, b0' = b0 - (w x u).b: pairs, so the
    // kernel gets (alpha, beta) from packed FMAs;   sphere: speed in [0..2], P in [3..5] = the
    // point of the sphere (at time 0) nearest the world origin, [6] = 1 when tested in f64
    Real AB[8];
    Real S[3];      // plane: shading normal (rotations of the chain applied to n)   sphere: V = P - center
    uint32_t meta;  // kind | material << 2
};
// PRIM_QUAD_X/Y/Z (world list): the plane is x_a = P with a = kind - PRIM_QUAD_X;
// N[a] = M^T n along the axis, N[(a+1)%3] = P = D / N[a], N[(a+2)%3] = 1e-8 / |N[a]|
// (the reference's |n.d| >= 1e-8 test as |d_a| >= that), A_a = B_a = 0 with the
// plane coordinate folded into a0' = a0 - A_a P, b0' = b0 - B_a P.
// PRIM_BOX (world mode): six consecutive quads that close a parallelepiped
// {c + a e1 + b e2 + g e3 : a, b, g in [0, 1]} are tested as one slab test in
// a local frame: per axis k, l_k(x) = row_k . x with faces on l_k = D_k and
// l_k = D_k + L_k (row_k = s_k (E^-1)_k, D_k = s_k (E^-1 c)_k, L_k = |s_k|; the
// scale makes a row's largest entry a power of two, flatten.cpp fuse_box).  The
// header holds (row_0, D_0) in (N, D), (row_1, D_1) in (AB[0..2], AB[3]),
// (row_2, D_2) in (AB[4..6], AB[7]), L in S; meta = PRIM_BOX | face << 3 with
// 3 bits per (axis, side) naming which of the six quads that follow the header
// lies on plane l_axis = D + side * L.  The quads keep their own records (uv,
// normals, material) for the hit record.
constexpr uint32_t BOX_ENTRIES = 7;
// f32 kernels test a sphere in f32 when its anchor P (the point nearest the world origin) plus
// |speed| stays within this (kernel.hpp sphere_t_world_f32: any radius), else in f64
constexpr double SPHERE_F32_EXTENT = 100.0;
// PRIM_BOXY (world-list run kind only; header meta kind stays PRIM_BOX): a box turned
// about the world y axis only.  Local axes (A, y, B): (N[0], N[2], D) = x, z entries
// of row A and its offset, (AB[0], AB[2], AB[3]) the same for row B (their y entries
// are 0), AB[4] <= AB[5] = the world y of the bottom and top faces, whose slab is the
// world y slab of axis quads and rooms (t = fma(Y, 1/d_y, -o_y/d_y)); face slots as
// PRIM_BOX with axis 1 = y (side 0 = bottom).
constexpr uint32_t PRIM_BOXY = 8;
// PRIM_SPHERE32 (world-list run kind only; the unit's meta kind stays PRIM_SPHERE): spheres the
// f32 test takes (AB[6] = 0).  A PRIM_SPHERE run is tested in f64 only, so a scene-specialised
// kernel compiles one sphere test per unit instead of both (C3 earth: 2350 -> 2063 instructions).
constexpr uint32_t PRIM_SPHERE32 = 9;
// PRIM_ABOX (world list): axis quads that each cover a whole face of one axis-
// aligned box (a "room": the Cornell walls) as one slab test; header N = lo,
// AB[0..2] = hi, meta = PRIM_ABOX | face slots << 3 (3 bits per (axis, side),
// 7 = no quad) | present-face mask << ABOX_PRESENT_SHIFT; then six slots
// (present faces' quad records).  A ray hits the entry face if it is present
// and t >= t_min, otherwise the exit face if present (the box is convex).
constexpr uint32_t ABOX_PRESENT_SHIFT = 21;
constexpr uint32_t WFLAG_AXIS_QUADS = 1;
// Coplanar overlapping surfaces (e.g. a cube standing on the Cornell floor: its
// bottom face and the floor quad share the plane y = 0).  The reference resolves
// their hits as an exact tie -- its t is bit-identical on both -- in favour of the
// later candidate of its depth-first order (BVH::hit, object.rs:109-115).  The host
// marks the pair's later surface WCLASS_WIN and the earlier WCLASS_LOSE (top bits of
// meta; box / room headers: the class of their faces).
//  * World list: units are ordered losers first, winners last, and `t <= t_best` lets
//    the later of two equal t win; the flattener keeps the list only when each pair's
//    two f32 t formulas are provably bit-identical (flatten.cpp tie forms), so the
//    hot loop pays nothing.
//  * World BVH (any visiting order, any formulas): with WFLAG_COPLANAR the leaf test
//    compares keys, t * (1 - WTIE_EPS) for winners and t * (1 + WTIE_EPS) for losers,
//    so near-ties go the reference's way; the hit record divides the factor out.
constexpr uint32_t WCLASS_SHIFT = 30, WCLASS_WIN = 1, WCLASS_LOSE = 2;
constexpr uint32_t WMAT_MASK = (1u << (WCLASS_SHIFT - WKIND_BITS)) - 1u;  // material index bits of meta
constexpr uint32_t WFLAG_COPLANAR = 2;
constexpr float WTIE_EPS = 1.0f / 1048576.0f;  // 2^-20: 16 ulps of f32
// Consecutive units of one kind form a run (kind | count << WRUN_KIND_BITS; a box
// unit is BOX_ENTRIES entries), so the kernel's inner loops are kind-specialised
// without reordering candidates.
constexpr uint32_t WRUN_KIND_BITS = 4, WRUN_KIND_MASK = 15;

// Fast kernel, world-BVH mode (large flattenable scenes): a binary BVH over the
// world-space primitives built with binned SAH on the host.  Each node holds
// both children's boxes so one visit tests two boxes and descends into the
// nearer hit child first (the farther one goes on a per-lane LDS stack).
// Child refs: >= 0 inner node index; < 0 leaf, ~ref = first << 3 | (count - 1)
// over the BVH-ordered primitive array (count 1..8).
struct alignas(16) DBvhNode {
    float lo0[3], hi0[3];
    float lo1[3], hi1[3];
    int32_t c0, c1;
    uint32_t pad[2];
};
// 4-wide form of the same tree (collapsed on the host), 64 bytes per node:
// child boxes quantized to 8 bits per plane relative to the node's box,
// lo_k = org + qlo_k * 2^(e - 127) per axis, rounded outward on the host (the
// decoded box always contains the f32 child box).  Traversal is gather-bound
// (each lane loads a different node), so bytes per visit set the speed: a 128-byte
// node with the child planes in f32 (no decode, 40 % fewer VALU instructions per visit)
// measured 20 % slower on the teapot (C4 40.3 -> 48.5 ms, round 3).
struct alignas(16) DBvh4Node {
    float org[3];      // lower corner of the node's box
    uint32_t exps;     // quantization step per axis, 10 bits each (x bits 0-9, y 10-19, z 20-29): wbvh_step
    uint32_t qlo[3];   // per axis, byte k = child k's low plane
    uint32_t qhi[3];   // per axis, byte k = child k's high plane
    int32_t child[4];  // refs as in DBvhNode (inner = DBvh4Node index), WBVH_DONE = empty slot
    uint32_t pad[2];
};
static_assert(sizeof(DBvh4Node) == 64, "one half cache line per 4-wide node");
// Compact 4-wide node, 48 bytes (three 16-byte loads per visit instead of four): the 64-byte
// node's quantized boxes with 16-bit child refs.  The teapot's traversal is bound by the
// vector memory path (L1 accesses: one per lane and load instruction), so a load less per
// visit is a quarter of the node traffic.  Built when every leaf holds at most 4 primitives,
// the tree has < 32768 nodes and < 8192 primitive slots (wbvh.cpp); the scene-specialised
// world-BVH kernel reads it (BvhSig width WBVH_COMPACT), with a 16-bit LDS stack.
struct alignas(16) DBvh4cNode {
    float org[3];
    uint32_t exps;
    uint32_t qlo[3];
    uint32_t qhi[3];
    uint16_t child[4];  // leaf: WBVH4C_LEAF | first << 2 | (count - 1); inner: node index
};
static_assert(sizeof(DBvh4cNode) == 48, "three 16-byte loads per compact 4-wide node");
constexpr uint32_t WBVH4C_LEAF = 0x8000u, WBVH4C_LEAF_MAX = 4, WBVH4C_MAX_PRIMS = 8192, WBVH4C_MAX_NODES = 32768;
constexpr int WBVH_COMPACT = 5;  // BvhSig width code of the compact 4-wide tree
// primitive kinds of a world BVH's leaves (the scene-specialised kernel's BvhSig)
enum : int { WPRIMS_ANY = 0, WPRIMS_TRIANGLES = 1, WPRIMS_QUADS = 2 };
constexpr int32_t WBVH_DONE = INT32_MIN;  // "stack empty" marker (never a valid leaf ref)
constexpr int32_t WBVH_NO_LEAF = 0;       // "no parked leaf" (leaf refs are negative)
constexpr uint32_t WBVH_STACK = 32;       // per-lane stack entries at most (host checks the tree's bound)
constexpr uint32_t WBVH_LEAF_MAX = 8;

// Exact kernel's culling walk without a stack: the binary world BVH threaded in depth-first
// order, one copy per ray-direction octant (bit 0: d.x < 0, bit 1: d.y < 0, bit 2: d.z < 0) in
// which every node's nearer child (box centres along the octant's diagonal) comes first and the
// box planes are stored as (near, far) for that octant's signs.  A hit node continues at the
// next record (its first child, or past a leaf's primitives at skip), a missed one at skip,
// the subtree's end: no stack, so no scratch traffic (round 2's private-array stack and the
// spills around it wrote 8.7 GB per C5 launch), and the walk keeps near-first order.
struct alignas(16) DThreadNode {
    float nearp[3];  // the box planes the octant's rays enter through (lo for d >= 0, else hi)
    int32_t skip;    // index (within the octant's copy) of the record after this subtree
    float farp[3];
    int32_t leaf;    // leaf ref ~(first << 3 | count - 1), 0 for an inner node
};
static_assert(sizeof(DThreadNode) == 32, "two 16-byte loads per threaded node");

// Exact kernel over the world BVH (RenderParams::exact_wbvh): for each BVH primitive slot,
// the reference primitive it is (DPrim index), the instance whose Translate/Rotate/Scale
// chain maps the world ray into that primitive's object space (-1: none), and its rank in the
// reference's depth-first candidate order (ties go to the higher rank, object.rs:109-115).
struct alignas(16) DExactRef {
    uint32_t prim;
    int32_t inst;
    uint32_t rank;
    uint32_t pad;
};

template <typename Real>
struct alignas(16) DXform {
    // TRANSLATE: m[0..2] = offset
    // ROTATE:    m[0..8] = rotation (world->object), column major; inv[0..8] = inverse
    // SCALE:     m = inverse scale matrix (world->object), inv = forward scale matrix,
    //            both as 3x4 column major (cols 0..3, rows 0..2) of glam DMat4
    Real m[12];
    Real inv[12];
    uint32_t kind;
    uint32_t pad[3];
};

struct alignas(16) DInstance {
    uint32_t first_xform;
    uint32_t num_xforms;
    int32_t root;       // BLAS root in the exact node array (NODE_END = empty)
    int32_t root_fast;  // BLAS root in the fast (list-collapsed) node array
};

// Fast kernel: an instance's Translate/Rotate/Scale chain composed into one
// affine map (host, f64, then rounded): object ray o' = A o + b, d' = A d;
// hit point back p = C p' + c; normal back n = N n' (rotations only, Q11).
template <typename Real>
struct alignas(16) DInstFast {
    Real A[9], b[3], C[9], c[3], N[9];  // 3x3 column major
    Real pad[3];
};

struct alignas(16) DMaterial {
    uint32_t kind;
    uint32_t texture;
    double param;  // Metal fuzz / Dielectric refraction index / DiffuseLight intensity
};

// Fast kernel material: parameter in f32 and a solid texture's colour inline
// (the common case needs one 32-B LDS read per bounce).
struct alignas(16) DMatFast {
    uint32_t kind;
    uint32_t texture;
    float param;
    uint32_t solid;  // 1: `color` is the (SolidColor) texture
    float color[3];
    float pad;
};

// Image texel formats in the texel array (32-bit words): RGBA8 = one word per texel, bytes
// r | g << 8 | b << 16, for images whose every value is k / 255 (every image a file gives:
// into_rgb32f, textures/image.rs:24-28; the kernel rebuilds k / 255.0f exactly); RGB32F =
// three f32 words per texel (images from the constructor API with other values).
// RGBA8 images are stored in tiles of 8 x 4 texels (128 bytes, one cache line), tiles in rows
// of ceil(W / 8): rays that hit nearby points of a sphere read nearby texels in both directions,
// so a line fetched for one serves its neighbours above and below as well (earth.toml: 4.96 GB
// of HBM/MALL fetches per C3 launch with f32 row-major texels).
// RGB8T (default; NRT_TEX_RGB8=0 keeps RGBA8): the same bytes packed three per texel, tiles of 8 x 5 texels (120
// bytes + 8 of padding, one 128-byte line): a line covers 40 texels instead of 32, at the cost of two
// word loads and a byte align per lookup (tex_rgb8_byte; heights below 65536).
// PAL16 (default where it applies; NRT_TEX_PAL=0 keeps RGB8T): a 16-bit palette index per texel in
// 8 x 8 tiles (one 128-byte line), then per horizontal band of 2^s rows a palette of at most 65536
// RGBA8 words, 2^p words apart (2^p = the largest band's colour count rounded up to a power of two):
// images with few distinct colours per band (earth.jpg: 99 388 in all, at most 62 033 per band of
// 256 rows; moon.jpg: 10 532) cost 2 bytes per texel instead of 3.2, for a second, dependent load that
// mostly hits the L2 (the palettes are small).  Taken only where index + palettes are smaller than
// the RGB8T layout.  The texture's `b` holds the height | s << 16 | p << 24 (heights below 65536).
enum : uint32_t { TEXFMT_RGB32F = 0, TEXFMT_RGBA8 = 1, TEXFMT_RGB8T = 2, TEXFMT_PAL16 = 3 };
#if defined(__HIPCC_RTC__)
#define NRT_HD __device__
#elif defined(__HIPCC__)
#define NRT_HD __host__ __device__
#else
#define NRT_HD
#endif
NRT_HD inline uint64_t tex_tiled_index(uint32_t x, uint32_t y, uint32_t tiles_per_row) {
    return ((uint64_t)(y >> 2) * tiles_per_row + (x >> 3)) * 32u + (y & 3u) * 8u + (x & 7u);
}
// RGB8T: byte offset of texel (x, y) (y < 65536: y / 5 as (y * 52429) >> 18, exact there)
NRT_HD inline uint64_t tex_rgb8_byte(uint32_t x, uint32_t y, uint32_t tiles_per_row) {
    const uint32_t ty = (y * 52429u) >> 18, ly = y - 5u * ty;
    return ((uint64_t)ty * tiles_per_row + (x >> 3)) * 128u + (ly * 8u + (x & 7u)) * 3u;
}
// World BVH 4-wide nodes: the quantization step of axis a, 2^e (1 + m / 4) from its 10-bit field
// (e + 127) << 2 | m: the field shifted into an f32's exponent and top two mantissa bits, exactly
#ifndef NRT_WBVH_STEP_MANTISSA
#define NRT_WBVH_STEP_MANTISSA 1  // 0: powers of two only (the round-4 steps)
#endif
NRT_HD inline uint32_t wbvh_step_bits(uint32_t exps, int a) { return ((exps >> (10 * a)) & 0x3FFu) << 21; }
// PAL16: 16-bit word index of texel (x, y) in the index array (two texels per 32-bit word), and
// the words the index array takes
NRT_HD inline uint64_t tex_pal_index(uint32_t x, uint32_t y, uint32_t tiles_per_row) {
    return ((uint64_t)(y >> 3) * tiles_per_row + (x >> 3)) * 64u + (y & 7u) * 8u + (x & 7u);
}
NRT_HD inline uint64_t tex_pal_index_words(uint32_t w, uint32_t h) {
    return (uint64_t)((w + 7u) >> 3) * ((h + 7u) >> 3) * 32u;
}
// PAL16: first word of row y's band palette after the index array (b = height | s << 16 | p << 24)
NRT_HD inline uint64_t tex_pal_band_word(uint32_t b, uint32_t y) {
    return (uint64_t)(y >> ((b >> 16) & 31u)) << ((b >> 24) & 31u);
}
struct alignas(16) DTexture {
    uint32_t kind;
    uint32_t a, b;     // image: width, height; checker: even, odd texture ids; noise/marble: octaves, seed
    uint32_t format;   // image: TEXFMT_*
    uint64_t offset;   // image: first word of its texels in the texel array; noise/marble: first word of
                       // its permutation tables (octaves x 256 words, values 0..255)
    double color[3];   // solid colour; noise/marble: frequency, lacunarity, persistence
    double scale;      // checker scale; noise/marble: Fbm scale factor
};

// What the kernel gets: device pointers + sizes (per precision).
template <typename Real>
struct DSceneView {
    const DNode<Real>* nodes;
    const DPrim<Real>* prims;
    const DXform<Real>* xforms;
    const DInstance* instances;
    const DMaterial* materials;
    const DTexture* textures;
    const uint32_t* texels;  // image texels (TEXFMT_*) and Perlin permutation tables, 32-bit words
    int32_t root;
    int32_t max_depth;  // deepest instance nesting (0 = no instances)
    uint32_t n_nodes, n_prims, n_xforms, n_instances, n_materials, n_textures;
    const DPrimFast<Real>* fprims;     // fast kernel: primitives in list order
    const DInstFast<Real>* inst_fast;  // fast kernel: composed instance transforms
    const DMatFast* mats_fast;         // fast kernel: materials with inline solid colour
    uint32_t n_fprims, n_inst_fast, n_mats_fast;
    const DPrimWorld<Real>* wprims;  // fast kernel, world-space mode (MAXD = 0)
    uint32_t n_wprims;
    const uint32_t* wruns;           // runs of same-kind world primitives
    uint32_t n_wruns;
    uint32_t wflags;                 // WFLAG_*: what the world list holds
    const DBvhNode* wbvh;            // world-BVH mode: nodes (wprims then holds the BVH-ordered prims)
    const DBvh4Node* wbvh4;          // the same tree collapsed to 4-wide nodes (root = wbvh4_root)
    const DBvh4cNode* wbvh4c;        // ... in the compact 48-byte form (same indices and root), or null
    int32_t wbvh4_root;
    int32_t wbvh_root;               // child ref of the root
    uint32_t n_wbvh;
    // per-lane stack entries the tree in use can need (<= WBVH_STACK): the world-BVH kernels
    // allocate that many + 1 (branch-free pushes) in LDS, so shallow trees leave room for
    // more workgroups per CU
    uint32_t wbvh_stack;
    const DThreadNode* xthread;  // f64 view: the culling tree threaded per octant (8 copies of n_xthread)
    uint32_t n_xthread;
    const DExactRef* wexact;  // f64 view: exact reference of each world-BVH slot (exact_wbvh mode)
    const DPrimWorld<float>* wxprims;  // f64 view: f32 world primitive of each of those slots (prefilter)
    uint32_t n_wexact;                 // slots of that tree
    // f64 view: 4-wide nodes of that tree when the tree, wxprims and wexact are small enough to be
    // staged in LDS with the scene (XSTAGE_MAX_BYTES; the Cornell box: 2 KB), else 0
    uint32_t n_xstage;
};
constexpr uint32_t XSTAGE_MAX_BYTES = 8192;

// World primitives staged in LDS sit 80 bytes apart (64-byte records + 16 bytes of padding): the
// lanes of a ds_read_b128 group that read different records then start on different banks of
// the 64 (a 64-byte stride puts every fourth record on the same banks: the hit-record reads
// made 46 % of the headline kernel's LDS cycles conflict cycles).
// World-list mode only (MAXD 0): the world-BVH modes read staged records for the hit record
// alone, and the padding would cost them LDS occupancy (spheres.toml: 490 records).
constexpr uint32_t WPRIM_LDS_STRIDE = 80;
constexpr uint32_t wprim_lds_stride(int maxd) { return maxd == 0 ? WPRIM_LDS_STRIDE : 64u; }

// Bytes of the LDS-stageable part of a scene (everything but texels), each
// array starting on a 16-byte boundary, in the order nodes, prims, xforms,
// instances, materials, textures.
template <typename Real>
inline uint32_t lds_scene_bytes(const DSceneView<Real>& v, int maxd) {
    auto r16 = [](uint64_t b) { return (uint32_t)((b + 15) & ~uint64_t(15)); };
    return r16(v.n_nodes * sizeof(DNode<Real>)) + r16(v.n_prims * sizeof(DPrim<Real>)) +
           r16(v.n_xforms * sizeof(DXform<Real>)) + r16(v.n_instances * sizeof(DInstance)) +
           r16(v.n_materials * sizeof(DMaterial)) + r16(v.n_textures * sizeof(DTexture)) +
           r16(v.n_fprims * sizeof(DPrimFast<Real>)) + r16(v.n_inst_fast * sizeof(DInstFast<Real>)) +
           r16(v.n_mats_fast * sizeof(DMatFast)) + r16(v.n_wprims * wprim_lds_stride(maxd)) +
           (v.n_xstage ? r16(v.n_xstage * sizeof(DBvh4cNode)) + r16(v.n_wexact * sizeof(DPrimWorld<float>)) +
                             r16(v.n_wexact * sizeof(DExactRef))
                       : 0u);
}

}  // namespace nrt
