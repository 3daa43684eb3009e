// Scene graph -> threaded BVH arrays (device_scene.hpp).
#include "flatten.hpp"

#include <climits>
#include <cmath>
#include <cstring>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <array>
#include <deque>
#include <map>
#include <unordered_map>
#include <stdexcept>

#ifndef NRT_SPHERE_COST
#define NRT_SPHERE_COST 4.0f  // SAH weight of an (f64) sphere test relative to a plane test
#endif

namespace nrt {

namespace {

bool is_transform(const Object* o) {
    return o->kind == Object::Translate || o->kind == Object::Rotate || o->kind == Object::Scale;
}

struct Flattener {
    FlatScene out;
    std::map<const Object*, uint32_t> prim_ids;
    std::map<const Material*, uint32_t> mat_ids;
    std::map<const Texture*, uint32_t> tex_ids;
    std::map<const Object*, int32_t> blas_roots;          // target object -> tree root
    std::map<const Object*, uint32_t> inst_ids;           // transform-chain head -> instance
    std::vector<const Object*> inst_targets;              // instance -> BLAS object
    std::deque<std::pair<uint32_t, const Object*>> pending;  // (instance id, target) to emit
    std::vector<std::pair<uint32_t, uint32_t>> tree_ranges;   // [begin, end) node index per tree

    uint32_t texture(const TexturePtr& t) {
        auto it = tex_ids.find(t.get());
        if (it != tex_ids.end()) return it->second;
        DTexture d{};
        switch (t->kind) {
            case Texture::Solid:
                d.kind = TEX_SOLID;
                d.color[0] = t->color.x; d.color[1] = t->color.y; d.color[2] = t->color.z;
                break;
            case Texture::Image: {
                d.kind = TEX_IMAGE;
                d.a = t->width;
                d.b = t->height;
                d.offset = out.texels.size();
                out.texel_count += (uint64_t)t->width * t->height;
                // RGBA8 when every value is k / 255 in f32 (files always are: into_rgb32f), else RGB32F
                const std::vector<float>& px = *t->texels;
                bool unorm8 = true;
                for (size_t i = 0; i < px.size() && unorm8; ++i) {
                    const float v = px[i];
                    const float k = std::nearbyint(v * 255.0f);
                    unorm8 = k >= 0.0f && k <= 255.0f && (float)k / 255.0f == v && !std::signbit(v);
                }
                static const bool rgba8_ok = [] {  // knob NRT_TEX_RGBA8=0 (A/B runs): keep RGB32F texels
                    const char* e = std::getenv("NRT_TEX_RGBA8");
                    return !(e && e[0] == '0');
                }();
                unorm8 &= rgba8_ok;
                // 3-byte texels (RGB8T) by default: C3 HBM fetch 2.35 -> 1.74 GB per launch, time within
                // 1 % (the decode's extra word load and byte align on a VALU-bound kernel); knob
                // NRT_TEX_RGB8=0 keeps the one-word RGBA8 tiles
                static const bool rgb8_on = [] {
                    const char* e = std::getenv("NRT_TEX_RGB8");
                    return !(e && e[0] == '0');
                }();
                d.format = unorm8 ? TEXFMT_RGBA8 : TEXFMT_RGB32F;
                const char* pe = std::getenv("NRT_TEX_PAL");  // knob NRT_TEX_PAL=0 (A/B runs, tests): no palettes
                const bool pal_on = !(pe && pe[0] == '0');
                if (unorm8 && pal_on && t->height < 65536u && pal16_texture(*t, d)) break;
                if (unorm8 && rgb8_on && t->height < 65536u) {  // 8 x 5 tiles of 3-byte texels (tex_rgb8_byte)
                    d.format = TEXFMT_RGB8T;
                    const uint32_t tw = (t->width + 7u) / 8u, th = (t->height + 4u) / 5u;
                    const size_t base = out.texels.size();
                    out.texels.resize(base + (size_t)tw * th * 32u, 0u);
                    unsigned char* bytes = reinterpret_cast<unsigned char*>(out.texels.data() + base);
                    for (uint32_t y = 0; y < t->height; ++y)
                        for (uint32_t x = 0; x < t->width; ++x) {
                            const float* v = px.data() + 3ull * ((size_t)y * t->width + x);
                            const uint64_t o = tex_rgb8_byte(x, y, tw);
                            for (int c = 0; c < 3; ++c) bytes[o + c] = (unsigned char)std::nearbyint(v[c] * 255.0f);
                        }
                } else if (unorm8) {  // 8 x 4 texel tiles of one 128-byte line each, rows of tiles (tex_texel_index)
                    const uint32_t tw = (t->width + 7u) / 8u, th = (t->height + 3u) / 4u;
                    const size_t base = out.texels.size();
                    out.texels.resize(base + (size_t)tw * th * 32u, 0u);
                    for (uint32_t y = 0; y < t->height; ++y)
                        for (uint32_t x = 0; x < t->width; ++x) {
                            const float* v = px.data() + 3ull * ((size_t)y * t->width + x);
                            uint32_t w = 0;
                            for (int c = 0; c < 3; ++c) w |= (uint32_t)std::nearbyint(v[c] * 255.0f) << (8 * c);
#ifdef NRT_TEX_ROWMAJOR  // (A/B build: row-major RGBA8)
                            out.texels[base + (size_t)y * t->width + x] = w;
#else
                            out.texels[base + tex_tiled_index(x, y, tw)] = w;
#endif
                        }
                } else {
                    for (float v : px) {
                        uint32_t w;
                        std::memcpy(&w, &v, 4);
                        out.texels.push_back(w);
                    }
                }
                break;
            }
            case Texture::Checker: {
                d.kind = TEX_CHECKER;
                d.scale = t->scale;
                const uint32_t e = texture(t->even), o = texture(t->odd);
                d.a = e;
                d.b = o;
                break;
            }
            case Texture::Noise:
            case Texture::Marble: {
                // Abs<Fbm<Perlin>>: one permutation table per octave (seed + k), stored
                // in the texel array, one word per entry
                d.kind = t->kind == Texture::Noise ? TEX_NOISE : TEX_MARBLE;
                const FbmParams& f = t->fbm;
                d.a = f.octaves;
                d.b = f.seed;
                d.color[0] = f.frequency;
                d.color[1] = f.lacunarity;
                d.color[2] = f.persistence;
                d.scale = fbm_scale_factor(f.persistence, f.octaves);
                d.offset = out.texels.size();
                uint8_t perm[256];
                for (uint32_t k = 0; k < f.octaves; ++k) {
                    perlin_permutation(f.seed + k, perm);  // Fbm build_sources: seed + k (u32 wrap)
                    for (int i = 0; i < 256; ++i) out.texels.push_back(perm[i]);
                }
                break;
            }
        }
        const uint32_t id = (uint32_t)out.textures.size();
        out.textures.push_back(d);
        tex_ids[t.get()] = id;
        return id;
    }

    // PAL16 layout (device_scene.hpp) of a k / 255 image, if every band of 2^s rows (s as large as
    // possible, at least 0) holds at most 65536 colours: index array, then the bands' palettes.
    bool pal16_texture(const Texture& t, DTexture& d) {
        const uint32_t W = t.width, H = t.height;
        const std::vector<float>& px = *t.texels;
        std::vector<uint32_t> rgb((size_t)W * H);
        for (size_t i = 0; i < rgb.size(); ++i) {
            uint32_t w = 0;
            for (int c = 0; c < 3; ++c) w |= (uint32_t)std::nearbyint(px[3 * i + c] * 255.0f) << (8 * c);
            rgb[i] = w;
        }
        uint32_t shift = 0;
        while ((1u << shift) < H) ++shift;  // one band first
        std::vector<std::vector<uint32_t>> pals;
        std::vector<std::unordered_map<uint32_t, uint32_t>> maps;
        for (;; --shift) {
            const uint32_t bands = ((H - 1u) >> shift) + 1u;
            pals.assign(bands, {});
            maps.assign(bands, {});
            bool ok = true;
            for (uint32_t y = 0; y < H && ok; ++y) {
                auto& m = maps[y >> shift];
                auto& pal = pals[y >> shift];
                for (uint32_t x = 0; x < W; ++x) {
                    const uint32_t c = rgb[(size_t)y * W + x];
                    if (m.emplace(c, (uint32_t)pal.size()).second) pal.push_back(c);
                }
                ok = pal.size() <= 65536u;
            }
            if (ok) break;
            if (shift == 0 || bands >= 256u) return false;  // (too many colours per row band: RGB8T)
        }
        // palettes 2^p words apart (p: the largest band's colour count, rounded up to a power of two),
        // and only where index + palettes take fewer bytes than RGB8T (a small or many-coloured image
        // would otherwise grow: a 64 x 64 image with 65536-word palettes took 264 KB against 13 KB)
        size_t most = 1;
        for (const auto& pal : pals) most = std::max(most, pal.size());
        uint32_t p = 0;
        while (((size_t)1 << p) < most) ++p;
        const uint64_t iw = tex_pal_index_words(W, H);
        const uint64_t pal_words = iw + ((uint64_t)pals.size() << p);
        const uint64_t rgb8t_words = (uint64_t)((W + 7u) / 8u) * ((H + 4u) / 5u) * 32u;
        if (pal_words >= rgb8t_words) return false;
        d.format = TEXFMT_PAL16;
        d.b = H | (shift << 16) | (p << 24);
        const size_t base = out.texels.size();
        out.texels.resize(base + pal_words, 0u);
        uint16_t* idx = reinterpret_cast<uint16_t*>(out.texels.data() + base);
        const uint32_t tw = (W + 7u) >> 3;
        for (uint32_t y = 0; y < H; ++y)
            for (uint32_t x = 0; x < W; ++x)
                idx[tex_pal_index(x, y, tw)] = (uint16_t)maps[y >> shift].at(rgb[(size_t)y * W + x]);
        for (size_t k = 0; k < pals.size(); ++k)
            std::copy(pals[k].begin(), pals[k].end(), out.texels.begin() + (std::ptrdiff_t)(base + iw + (k << p)));
        // (the palettes' unused tail slots are never read)
        return true;
    }

    uint32_t material(const MaterialPtr& m) {
        auto it = mat_ids.find(m.get());
        if (it != mat_ids.end()) return it->second;
        DMaterial d{};
        switch (m->kind) {
            case Material::Lambertian: d.kind = MAT_LAMBERTIAN; d.texture = texture(m->texture); break;
            case Material::Metal: d.kind = MAT_METAL; d.texture = texture(m->texture); d.param = m->fuzz; break;
            case Material::Dielectric: d.kind = MAT_DIELECTRIC; d.param = m->refraction_index; break;
            case Material::DiffuseLight:
                d.kind = MAT_DIFFUSE_LIGHT; d.texture = texture(m->texture); d.param = m->intensity;
                break;
        }
        const uint32_t id = (uint32_t)out.materials.size();
        out.materials.push_back(d);
        mat_ids[m.get()] = id;
        return id;
    }

    static void set3(double* dst, V3 v) { dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; }

    uint32_t prim(const Object* o, const MaterialPtr& mat) {
        auto it = prim_ids.find(o);
        if (it != prim_ids.end()) return it->second;
        DPrim<double> p{};
        if (o->kind == Object::Sphere) {
            p.kind = PRIM_SPHERE;
            set3(p.a, o->center);
            set3(p.b, o->speed);
            p.s = o->radius;
        } else {
            p.kind = o->kind == Object::Quad ? PRIM_QUAD : PRIM_TRIANGLE;
            set3(p.a, o->p);
            set3(p.b, o->u);
            set3(p.c, o->v);
            set3(p.n, o->normal);
            set3(p.w, o->w);
            p.s = o->d;
        }
        p.material = material(mat);
        const uint32_t id = (uint32_t)out.prims.size();
        out.prims.push_back(p);
        prim_ids[o] = id;
        return id;
    }

    uint32_t push(uint32_t kind, uint32_t payload) {
        DNode<double> n{};
        n.meta = kind | (payload << 2);
        n.skip = NODE_END;
        out.nodes.push_back(n);
        return (uint32_t)out.nodes.size() - 1;
    }

    uint32_t xform(const Object* t) {
        DXform<double> x{};
        if (t->kind == Object::Translate) {
            x.kind = XF_TRANSLATE;
            x.m[0] = t->offset.x; x.m[1] = t->offset.y; x.m[2] = t->offset.z;
        } else if (t->kind == Object::Rotate) {
            x.kind = XF_ROTATE;
            for (int c = 0; c < 3; ++c) {
                x.m[3 * c + 0] = t->rot.c[c].x; x.m[3 * c + 1] = t->rot.c[c].y; x.m[3 * c + 2] = t->rot.c[c].z;
                x.inv[3 * c + 0] = t->rot_inv.c[c].x; x.inv[3 * c + 1] = t->rot_inv.c[c].y;
                x.inv[3 * c + 2] = t->rot_inv.c[c].z;
            }
        } else {
            x.kind = XF_SCALE;
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 3; ++r) {
                    x.m[3 * c + r] = t->scale_inv.c[c][r];
                    x.inv[3 * c + r] = t->scale_m.c[c][r];
                }
        }
        out.xforms.push_back(x);
        return (uint32_t)out.xforms.size() - 1;
    }

    void emit(const Object* o) {
        switch (o->kind) {
            case Object::BvhEmpty:
                return;  // BVH::Leaf(None).hit is None: no node needed
            case Object::BvhLeaf:
                emit(o->child.get());  // Leaf(Some(o)).hit = o.hit, no bbox test
                return;
            case Object::BvhNode: {
                const uint32_t idx = push(NODE_INNER, 0);
                DNode<double>& n = out.nodes[idx];
                n.bmin[0] = o->bbox.x.min; n.bmax[0] = o->bbox.x.max;
                n.bmin[1] = o->bbox.y.min; n.bmax[1] = o->bbox.y.max;
                n.bmin[2] = o->bbox.z.min; n.bmax[2] = o->bbox.z.max;
                emit(o->left.get());
                emit(o->right.get());
                out.nodes[idx].skip = (int32_t)out.nodes.size();
                return;
            }
            case Object::Sphere:
            case Object::Quad:
            case Object::Triangle: {
                const uint32_t pid = prim(o, o->material);
                const uint32_t idx = push(NODE_PRIM, pid);
                out.nodes[idx].skip = (int32_t)idx + 1;
                return;
            }
            case Object::Translate:
            case Object::Rotate:
            case Object::Scale: {
                const uint32_t iid = instance(o);
                const uint32_t idx = push(NODE_INSTANCE, iid);
                out.nodes[idx].skip = (int32_t)idx + 1;
                return;
            }
        }
    }

    // One instance per distinct transform-chain head (a Ref'd chain is shared).
    uint32_t instance(const Object* o) {
        auto it = inst_ids.find(o);
        if (it != inst_ids.end()) return it->second;
        DInstance inst{};
        inst.first_xform = (uint32_t)out.xforms.size();
        const Object* t = o;
        while (is_transform(t)) {
            xform_of[t] = xform(t);
            t = t->child.get();
        }
        inst.num_xforms = (uint32_t)out.xforms.size() - inst.first_xform;
        inst.root = NODE_END;
        inst.root_fast = NODE_END;
        const uint32_t iid = (uint32_t)out.instances.size();
        out.instances.push_back(inst);
        out.inst_fast.push_back(compose(inst));
        inst_targets.push_back(t);
        pending.emplace_back(iid, t);
        inst_ids[o] = iid;
        return iid;
    }

    // Compose the chain into one affine map each way (f64), for the fast kernel.
    DInstFast<double> compose(const DInstance& inst) {
        using Mat = std::array<double, 9>;  // column major
        auto I = []() { Mat m{}; m[0] = m[4] = m[8] = 1.0; return m; };
        auto mm = [](const Mat& a, const Mat& b) {  // a * b
            Mat r{};
            for (int c = 0; c < 3; ++c)
                for (int rr = 0; rr < 3; ++rr)
                    r[3 * c + rr] = a[rr] * b[3 * c] + a[3 + rr] * b[3 * c + 1] + a[6 + rr] * b[3 * c + 2];
            return r;
        };
        auto mv = [](const Mat& a, const std::array<double, 3>& v) {
            return std::array<double, 3>{a[0] * v[0] + a[3] * v[1] + a[6] * v[2], a[1] * v[0] + a[4] * v[1] + a[7] * v[2],
                                         a[2] * v[0] + a[5] * v[1] + a[8] * v[2]};
        };
        Mat A = I(), C = I(), N = I();
        std::array<double, 3> b{0, 0, 0}, c{0, 0, 0};
        for (uint32_t k = 0; k < inst.num_xforms; ++k) {  // world -> object, outer first
            const DXform<double>& x = out.xforms[inst.first_xform + k];
            if (x.kind == XF_TRANSLATE) {
                for (int r = 0; r < 3; ++r) b[r] -= x.m[r];
            } else {
                Mat L;
                for (int q = 0; q < 9; ++q) L[q] = x.m[q];
                A = mm(L, A);
                b = mv(L, b);
                if (x.kind == XF_SCALE)
                    for (int r = 0; r < 3; ++r) b[r] += x.m[9 + r];
            }
        }
        for (uint32_t k = inst.num_xforms; k-- > 0;) {  // object -> world, inner first
            const DXform<double>& x = out.xforms[inst.first_xform + k];
            if (x.kind == XF_TRANSLATE) {
                for (int r = 0; r < 3; ++r) c[r] += x.m[r];
            } else {
                Mat L;
                for (int q = 0; q < 9; ++q) L[q] = x.inv[q];
                C = mm(L, C);
                c = mv(L, c);
                if (x.kind == XF_SCALE)
                    for (int r = 0; r < 3; ++r) c[r] += x.inv[9 + r];
                else
                    N = mm(L, N);  // only rotations turn the normal (Q11)
            }
        }
        DInstFast<double> f{};
        for (int q = 0; q < 9; ++q) { f.A[q] = A[q]; f.C[q] = C[q]; f.N[q] = N[q]; }
        for (int r = 0; r < 3; ++r) { f.b[r] = b[r]; f.c[r] = c[r]; }
        return f;
    }

    // ---- fast node array: prim-only subtrees with <= LIST_MAX leaves become NODE_LIST
    static bool prims_only(const Object* o, uint32_t& n) {
        switch (o->kind) {
            case Object::BvhEmpty: return true;
            case Object::BvhLeaf: return prims_only(o->child.get(), n);
            case Object::BvhNode: return prims_only(o->left.get(), n) && prims_only(o->right.get(), n);
            case Object::Sphere:
            case Object::Quad:
            case Object::Triangle: ++n; return true;
            default: return false;
        }
    }
    uint32_t fast_prim(const Object* o) {
        DPrimFast<double> f{};
        f.material = material(o->material);
        if (o->kind == Object::Sphere) {
            f.kind = PRIM_SPHERE;
            set3(f.n, o->center);
            f.d = o->radius;
            set3(f.A, o->speed);
        } else {
            f.kind = o->kind == Object::Quad ? PRIM_QUAD : PRIM_TRIANGLE;
            set3(f.n, o->normal);
            f.d = o->d;
            const V3 A = cross(o->v, o->w), B = cross(o->w, o->u);
            set3(f.A, A);
            set3(f.B, B);
            f.a0 = dot(o->p, A);
            f.b0 = dot(o->p, B);
        }
        out.fprims.push_back(f);
        return (uint32_t)out.fprims.size() - 1;
    }
    void collect_prims(const Object* o) {
        switch (o->kind) {
            case Object::BvhLeaf: collect_prims(o->child.get()); return;
            case Object::BvhNode: collect_prims(o->left.get()); collect_prims(o->right.get()); return;
            case Object::Sphere:
            case Object::Quad:
            case Object::Triangle: fast_prim(o); return;
            default: return;
        }
    }
    uint32_t push_fast(uint32_t meta) {
        DNode<double> n{};
        n.meta = meta;
        n.skip = NODE_END;
        out.nodes_fast.push_back(n);
        return (uint32_t)out.nodes_fast.size() - 1;
    }
    void emit_fast(const Object* o) {
        switch (o->kind) {
            case Object::BvhEmpty: return;
            case Object::BvhLeaf: emit_fast(o->child.get()); return;
            case Object::BvhNode: {
                uint32_t count = 0;
                const bool list = prims_only(o, count) && count >= 2 && count <= LIST_MAX;
                const uint32_t first = (uint32_t)out.fprims.size();
                const uint32_t idx = push_fast(list ? (NODE_LIST | ((count - 1) << 2) | (first << 8)) : NODE_INNER);
                DNode<double>& n = out.nodes_fast[idx];
                n.bmin[0] = o->bbox.x.min; n.bmax[0] = o->bbox.x.max;
                n.bmin[1] = o->bbox.y.min; n.bmax[1] = o->bbox.y.max;
                n.bmin[2] = o->bbox.z.min; n.bmax[2] = o->bbox.z.max;
                if (list) {
                    if (first >= (1u << 24)) throw std::runtime_error("too many primitives for the fast layout");
                    collect_prims(o);
                } else {
                    emit_fast(o->left.get());
                    emit_fast(o->right.get());
                }
                out.nodes_fast[idx].skip = (int32_t)out.nodes_fast.size();
                return;
            }
            case Object::Sphere:
            case Object::Quad:
            case Object::Triangle: {
                const uint32_t idx = push_fast(NODE_PRIM | (fast_prim(o) << 2));
                out.nodes_fast[idx].skip = (int32_t)idx + 1;
                return;
            }
            default: {
                const uint32_t idx = push_fast(NODE_INSTANCE | (instance(o) << 2));
                out.nodes_fast[idx].skip = (int32_t)idx + 1;
                return;
            }
        }
    }
    int32_t tree_fast(const Object* o) {
        const uint32_t begin = (uint32_t)out.nodes_fast.size();
        emit_fast(o);
        const uint32_t end = (uint32_t)out.nodes_fast.size();
        for (uint32_t k = begin; k < end; ++k)
            if (out.nodes_fast[k].skip == (int32_t)end) out.nodes_fast[k].skip = NODE_END;
        return end > begin ? (int32_t)begin : NODE_END;
    }

    // ---- world-space primitives (fast kernel, MAXD = 0 mode; device_scene.hpp DPrimWorld)
    static constexpr size_t WORLD_PRIM_CAP = size_t(1) << 22;
    using M3a = std::array<double, 9>;  // column major
    using V3a = std::array<double, 3>;
    struct Affine {
        M3a M{1, 0, 0, 0, 1, 0, 0, 0, 1};  // world -> object: o' = M o + b
        V3a b{0, 0, 0};
        M3a R{1, 0, 0, 0, 1, 0, 0, 0, 1};  // object normal -> world (rotations only)
        bool translate_only = true;
    };
    static M3a mmul(const M3a& a, const M3a& c) {
        M3a r{};
        for (int col = 0; col < 3; ++col)
            for (int row = 0; row < 3; ++row)
                r[3 * col + row] = a[row] * c[3 * col] + a[3 + row] * c[3 * col + 1] + a[6 + row] * c[3 * col + 2];
        return r;
    }
    static V3a mvec(const M3a& a, const V3a& v) {
        return {a[0] * v[0] + a[3] * v[1] + a[6] * v[2], a[1] * v[0] + a[4] * v[1] + a[7] * v[2],
                a[2] * v[0] + a[5] * v[1] + a[8] * v[2]};
    }
    static V3a mtvec(const M3a& a, const V3a& v) {  // a^T v
        return {a[0] * v[0] + a[1] * v[1] + a[2] * v[2], a[3] * v[0] + a[4] * v[1] + a[5] * v[2],
                a[6] * v[0] + a[7] * v[1] + a[8] * v[2]};
    }
    static V3a va(V3 v) { return {v.x, v.y, v.z}; }
    static M3a inverse3(const M3a& m) {  // column major; adjugate / determinant
        const double a = m[0], b = m[3], c = m[6], d = m[1], e = m[4], f = m[7], g = m[2], h = m[5], i = m[8];
        const double A = e * i - f * h, B = -(d * i - f * g), C = d * h - e * g;
        const double det = a * A + b * B + c * C;
        const double r = 1.0 / det;
        M3a o;  // o[3*col + row]
        o[0] = A * r; o[3] = -(b * i - c * h) * r; o[6] = (b * f - c * e) * r;
        o[1] = B * r; o[4] = (a * i - c * g) * r; o[7] = -(a * f - c * d) * r;
        o[2] = C * r; o[5] = -(a * h - b * g) * r; o[8] = (a * e - b * d) * r;
        return o;
    }
    std::vector<std::array<V3a, 3>> wgeom;  // world (p, u, v) of each world prim (quads; zero otherwise)

    // A world quad whose plane normal lies on a coordinate axis -> PRIM_QUAD_X + axis
    // (device_scene.hpp): plane coordinate, threshold and folded offsets.
    static void axis_quad(DPrimWorld<double>& w) {
        int a = -1, zeros = 0;
        for (int k = 0; k < 3; ++k) {
            if (w.N[k] == 0.0) ++zeros;
            else a = k;
        }
        if (zeros != 2 || !std::isfinite(w.N[a]) || !std::isfinite(w.D)) return;
        const double Na = w.N[a], P = w.D / Na;
        w.AB[6] -= w.AB[2 * a] * P;
        w.AB[7] -= w.AB[2 * a + 1] * P;
        w.AB[2 * a] = 0.0;
        w.AB[2 * a + 1] = 0.0;
        w.N[(a + 1) % 3] = P;
        w.N[(a + 2) % 3] = 1e-8 / std::fabs(Na);
        w.meta = (PRIM_QUAD_X + (uint32_t)a) | (w.meta & ~WKIND_MASK);
    }

    // Axis quads that each cover a whole face of the bounding box of all axis
    // quads (e.g. the Cornell room's walls) -> one PRIM_ABOX unit (device_scene.hpp).
    void fuse_room(std::vector<std::vector<DPrimWorld<double>>>& units, std::vector<uint32_t>& kind,
                   std::vector<size_t>& src) {
        std::vector<size_t> aq;
        for (size_t u = 0; u < units.size(); ++u)
            if (kind[u] >= PRIM_QUAD_X && kind[u] <= PRIM_QUAD_Z) aq.push_back(u);
        if (aq.size() < 2) return;
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, scale = 0;
        auto corners = [&](size_t u, V3a c[4]) {
            const auto& g = wgeom[src[u]];
            for (int k = 0; k < 4; ++k)
                for (int r = 0; r < 3; ++r) c[k][r] = g[0][r] + ((k & 1) ? g[1][r] : 0.0) + ((k & 2) ? g[2][r] : 0.0);
        };
        for (size_t u : aq) {
            V3a c[4];
            corners(u, c);
            for (auto& x : c)
                for (int r = 0; r < 3; ++r) {
                    lo[r] = std::min(lo[r], x[r]);
                    hi[r] = std::max(hi[r], x[r]);
                    scale = std::max(scale, std::fabs(x[r]));
                }
        }
        const double tol = 1e-9 * std::max(scale, 1e-300);
        long face[3][2] = {{-1, -1}, {-1, -1}, {-1, -1}};
        int nfaces = 0;
        for (size_t u : aq) {
            const int a = (int)(kind[u] - PRIM_QUAD_X), a1 = (a + 1) % 3, a2 = (a + 2) % 3;
            V3a c[4];
            corners(u, c);
            const double plane = c[0][a];
            const int side = std::fabs(plane - lo[a]) <= tol ? 0 : (std::fabs(plane - hi[a]) <= tol ? 1 : -1);
            if (side < 0 || face[a][side] >= 0 || !(hi[a1] > lo[a1]) || !(hi[a2] > lo[a2])) continue;
            int seen = 0;  // the four corners must be the face's four corners
            for (auto& x : c) {
                const int b1 = std::fabs(x[a1] - lo[a1]) <= tol ? 0 : (std::fabs(x[a1] - hi[a1]) <= tol ? 1 : -1);
                const int b2 = std::fabs(x[a2] - lo[a2]) <= tol ? 0 : (std::fabs(x[a2] - hi[a2]) <= tol ? 1 : -1);
                if (b1 < 0 || b2 < 0 || std::fabs(x[a] - plane) > tol) { seen = -1; break; }
                seen |= 1 << (b1 + 2 * b2);
            }
            if (seen != 15) continue;
            face[a][side] = (long)u;
            ++nfaces;
        }
        if (nfaces < 2) return;
        uint32_t cls = 0;  // the faces' coplanar-tie class (device_scene.hpp WCLASS_*), one per unit
        for (int a = 0; a < 3; ++a)
            for (int sd = 0; sd < 2; ++sd)
                if (face[a][sd] >= 0) cls |= units[face[a][sd]][0].meta >> WCLASS_SHIFT;
        if (cls == (WCLASS_WIN | WCLASS_LOSE)) return;
        std::vector<DPrimWorld<double>> unit(1 + 6);
        DPrimWorld<double>& h = unit[0];
        h = DPrimWorld<double>{};
        for (int r = 0; r < 3; ++r) { h.N[r] = lo[r]; h.AB[r] = hi[r]; }
        uint32_t map = 0, present = 0;
        std::vector<bool> dead(units.size(), false);
        for (int a = 0; a < 3; ++a)
            for (int sd = 0; sd < 2; ++sd) {
                const int slot = 2 * a + sd;
                if (face[a][sd] >= 0) {
                    if (src[face[a][sd]] != SIZE_MAX) tie_form[src[face[a][sd]]] = axis_form(a, sd ? hi[a] : lo[a]);
                    unit[1 + slot] = units[face[a][sd]][0];
                    map |= (uint32_t)slot << (3 * slot);
                    present |= 1u << slot;
                    dead[face[a][sd]] = true;
                } else {
                    unit[1 + slot] = DPrimWorld<double>{};  // absent face: never referenced
                    map |= 7u << (3 * slot);
                }
            }
        h.meta = PRIM_ABOX | (map << WKIND_BITS) | (present << ABOX_PRESENT_SHIFT) | (cls << WCLASS_SHIFT);
        std::vector<std::vector<DPrimWorld<double>>> nu;
        std::vector<uint32_t> nk;
        std::vector<size_t> ns;
        for (size_t u = 0; u < units.size(); ++u)
            if (!dead[u]) { nu.push_back(std::move(units[u])); nk.push_back(kind[u]); ns.push_back(src[u]); }
        nu.push_back(std::move(unit));
        nk.push_back(PRIM_ABOX);
        ns.push_back(SIZE_MAX);
        units.swap(nu);
        kind.swap(nk);
        src.swap(ns);
    }

    // Six consecutive quads closing a parallelepiped -> PRIM_BOX header (device_scene.hpp).
    bool fuse_box(size_t i, DPrimWorld<double>& hdr) {
        std::vector<V3a> pts;
        double scale = 0;
        for (size_t q = i; q < i + 6; ++q) {
            if ((out.wprims[q].meta & WKIND_MASK) != PRIM_QUAD) return false;
            const auto& g = wgeom[q];
            const V3a c[4] = {g[0], {g[0][0] + g[1][0], g[0][1] + g[1][1], g[0][2] + g[1][2]},
                              {g[0][0] + g[2][0], g[0][1] + g[2][1], g[0][2] + g[2][2]},
                              {g[0][0] + g[1][0] + g[2][0], g[0][1] + g[1][1] + g[2][1], g[0][2] + g[1][2] + g[2][2]}};
            for (const V3a& x : c) {
                pts.push_back(x);
                for (int k = 0; k < 3; ++k) scale = std::max(scale, std::fabs(x[k]));
            }
        }
        const double tol = 1e-9 * std::max(scale, 1e-300);
        auto same = [&](const V3a& a, const V3a& b) {
            return std::fabs(a[0] - b[0]) <= tol && std::fabs(a[1] - b[1]) <= tol && std::fabs(a[2] - b[2]) <= tol;
        };
        std::vector<V3a> uniq;
        std::vector<int> mult;
        for (const V3a& x : pts) {
            size_t k = 0;
            while (k < uniq.size() && !same(uniq[k], x)) ++k;
            if (k == uniq.size()) { uniq.push_back(x); mult.push_back(0); }
            ++mult[k];
        }
        if (uniq.size() != 8) return false;
        for (int m : mult) if (m != 3) return false;
        auto has = [&](const V3a& x) {
            for (const V3a& u : uniq) if (same(u, x)) return true;
            return false;
        };
        const auto& g0 = wgeom[i];
        const V3a c = g0[0], e1 = g0[1], e2 = g0[2];
        V3a e3{};
        bool found = false;
        for (const V3a& r : uniq) {
            const V3a w{r[0] - c[0], r[1] - c[1], r[2] - c[2]};
            if (std::fabs(w[0]) <= tol && std::fabs(w[1]) <= tol && std::fabs(w[2]) <= tol) continue;
            auto plus = [&](const V3a& a, const V3a& b) { return V3a{a[0] + b[0], a[1] + b[1], a[2] + b[2]}; };
            if (has(plus(c, w)) && has(plus(plus(c, e1), w)) && has(plus(plus(c, e2), w)) &&
                has(plus(plus(plus(c, e1), e2), w)) && !same(plus(c, w), plus(c, e1)) && !same(plus(c, w), plus(c, e2)) &&
                !same(plus(c, w), plus(plus(c, e1), e2))) {
                e3 = w;
                found = true;
                break;
            }
        }
        if (!found) return false;
        const M3a E{e1[0], e1[1], e1[2], e2[0], e2[1], e2[2], e3[0], e3[1], e3[2]};
        const double det = E[0] * (E[4] * E[8] - E[7] * E[5]) - E[3] * (E[1] * E[8] - E[7] * E[2]) +
                           E[6] * (E[1] * E[5] - E[4] * E[2]);
        const double vol = std::sqrt(vdot(e1, e1) * vdot(e2, e2) * vdot(e3, e3));
        if (!(std::fabs(det) > 1e-9 * vol)) return false;
        const M3a Ei = inverse3(E);
        const V3a cl = mvec(Ei, c);
        int face[3][2] = {{-1, -1}, {-1, -1}, {-1, -1}};
        for (size_t q = 0; q < 6; ++q) {
            const auto& g = wgeom[i + q];
            int onaxis = -1, side = -1, combos = 0;
            for (int a = 0; a < 3; ++a) {
                int vals = 0;  // bit0: some corner at 0, bit1: some corner at 1
                for (int k = 0; k < 4; ++k) {
                    V3a x = g[0];
                    for (int r = 0; r < 3; ++r) x[r] += ((k & 1) ? g[1][r] : 0.0) + ((k & 2) ? g[2][r] : 0.0);
                    const V3a l = mvec(Ei, x);
                    const double la = l[a] - cl[a];
                    if (std::fabs(la) <= 1e-6) vals |= 1;
                    else if (std::fabs(la - 1.0) <= 1e-6) vals |= 2;
                    else return false;
                }
                if (vals == 3) ++combos;
                else { onaxis = a; side = vals == 1 ? 0 : 1; }
            }
            if (onaxis < 0 || combos != 2 || face[onaxis][side] >= 0) return false;
            face[onaxis][side] = (int)q;
        }
        uint32_t cls = 0;  // the faces' coplanar-tie class (device_scene.hpp WCLASS_*), one per unit
        for (size_t q = 0; q < 6; ++q) cls |= out.wprims[i + q].meta >> WCLASS_SHIFT;
        if (cls == (WCLASS_WIN | WCLASS_LOSE)) return false;
        hdr = DPrimWorld<double>{};
        // A box turned about the world y axis only (one edge exactly along y, the others with
        // y = 0: the common "object standing on a floor") -> PRIM_BOXY: its y slab is the
        // world y slab the axis quads and rooms use (t = fma(Y, 1/d_y, -o_y/d_y)), so a face
        // on a floor plane ties bit for bit with the floor, and it costs two rows, not three.
        int ya = -1;
        const V3a ed[3] = {e1, e2, e3};
        for (int a = 0; a < 3; ++a)
            if (ed[a][0] == 0.0 && ed[a][2] == 0.0 && ed[a][1] != 0.0 && ed[(a + 1) % 3][1] == 0.0 &&
                ed[(a + 2) % 3][1] == 0.0)
                ya = a;
        auto row = [&](int a) { return V3a{Ei[0 + a], Ei[3 + a], Ei[6 + a]}; };  // column-major Ei[3*col + row]
        if (ya >= 0) {
            const int A = ya == 0 ? 1 : 0, B = ya == 2 ? 1 : 2;
            double y0 = c[1], y1 = c[1] + ed[ya][1];
            int f0 = face[ya][0], f1 = face[ya][1];
            if (y1 < y0) { std::swap(y0, y1); std::swap(f0, f1); }
            const V3a ra = row(A), rb = row(B);
            hdr.N[0] = ra[0]; hdr.N[2] = ra[2]; hdr.D = cl[A];
            hdr.AB[0] = rb[0]; hdr.AB[2] = rb[2]; hdr.AB[3] = cl[B];
            hdr.AB[4] = y0; hdr.AB[5] = y1;
            const int slots[3][2] = {{face[A][0], face[A][1]}, {f0, f1}, {face[B][0], face[B][1]}};
            uint32_t map = 0;
            for (int a = 0; a < 3; ++a)
                for (int sd = 0; sd < 2; ++sd) map |= (uint32_t)slots[a][sd] << (3 * (2 * a + sd));
            hdr.meta = PRIM_BOX | (map << WKIND_BITS) | (cls << WCLASS_SHIFT);
            tie_form[i + f0] = axis_form(1, y0);
            tie_form[i + f1] = axis_form(1, y1);
            for (int a : {A, B})
                for (int sd = 0; sd < 2; ++sd)
                    tie_form[i + face[a][sd]] = {5.0f, (float)row(a)[0], (float)row(a)[2], (float)cl[a], (float)sd};
            box_y = true;
            return true;
        }
        box_y = false;
        for (int k = 0; k < 3; ++k) {  // rows of E^-1 (column-major Ei[3*col + row])
            hdr.N[k] = Ei[3 * k + 0];
            hdr.AB[k] = Ei[3 * k + 1];
            hdr.AB[4 + k] = Ei[3 * k + 2];
        }
        hdr.D = cl[0];
        hdr.AB[3] = cl[1];
        hdr.AB[7] = cl[2];
        uint32_t map = 0;
        for (int a = 0; a < 3; ++a)
            for (int sd = 0; sd < 2; ++sd) map |= (uint32_t)face[a][sd] << (3 * (2 * a + sd));
        hdr.meta = PRIM_BOX | (map << WKIND_BITS) | (cls << WCLASS_SHIFT);
        for (int a = 0; a < 3; ++a) {  // tie forms of the six faces (local axis a, side sd), in f32
            const V3a r = row(a);
            const float rf[3] = {(float)r[0], (float)r[1], (float)r[2]};
            const float off = (float)cl[a];
            int nz = -1, count = 0;
            for (int k = 0; k < 3; ++k)
                if (rf[k] != 0.0f) { nz = k; ++count; }
            int e = 0;
            const bool pow2 = count == 1 && std::fabs(std::frexp(rf[nz], &e)) == 0.5f;
            for (int sd = 0; sd < 2; ++sd) {
                if (sd == 0 && off == 0.0f && pow2) tie_form[i + face[a][sd]] = {1.0f, (float)nz};
                else tie_form[i + face[a][sd]] = {3.0f, rf[0], rf[1], rf[2], off, (float)sd};
            }
        }
        return true;
    }
    static double vdot(const V3a& a, const V3a& c) { return a[0] * c[0] + a[1] * c[1] + a[2] * c[2]; }

    // Coplanar overlapping planar primitives (device_scene.hpp WCLASS_*): the later one
    // of each pair in the reference's depth-first candidate order (= wprims order, which
    // world_walk emits left before right) wins the reference's exact tie; mark it
    // WCLASS_WIN and the earlier WCLASS_LOSE.  A primitive that would be both leaves the
    // world modes off (the instance BVH keeps the reference's order exactly).
    // f32 t formula of each world-list face (wprims index before fusion).  Two faces with
    // equal forms compute bit-identical t in the kernel's world list:
    //   {1, a}           t = -(o_a * 1/d_a): an axis plane at 0 -- axis quads and room faces
    //                    (fma(0, 1/d, -o/d)) and box faces on local plane 0 whose E^-1 row is
    //                    one power of two c on world axis a with offset 0 (c cancels exactly);
    //   {2, a, P}        t = fma(P, 1/d_a, -o_a/d_a): axis quads and room faces;
    //   {3, row, off, s} a box face (local slab formula);
    //   {4, N, D}        t = (D - N.o) / (N.d): quads and triangles.
    std::map<size_t, std::vector<float>> tie_form;
    bool box_y = false;  // the last fused box is a PRIM_BOXY unit
    std::vector<std::pair<size_t, size_t>> tie_pairs;  // (loser, winner) wprims indices
    static std::vector<float> axis_form(int a, double P) {
        const float p32 = (float)P;
        return p32 == 0.0f ? std::vector<float>{1.0f, (float)a} : std::vector<float>{2.0f, (float)a, p32};
    }

    bool mark_coplanar() {
        struct Pl { size_t i; V3a n; double d; };
        std::vector<Pl> pl;
        double scale = 0;
        for (size_t i = 0; i < out.wprims.size(); ++i) {
            const uint32_t kind = out.wprims[i].meta & WKIND_MASK;
            if (kind != PRIM_QUAD && kind != PRIM_TRIANGLE) continue;
            const auto& g = wgeom[i];
            V3a n = {g[1][1] * g[2][2] - g[1][2] * g[2][1], g[1][2] * g[2][0] - g[1][0] * g[2][2],
                     g[1][0] * g[2][1] - g[1][1] * g[2][0]};
            const double len = std::sqrt(vdot(n, n));
            if (!(len > 0) || !std::isfinite(len)) continue;
            for (double& c : n) c /= len;
            for (int k = 0; k < 3; ++k)  // canonical orientation: first clearly non-zero component positive
                if (std::fabs(n[k]) > 1e-12) {
                    if (n[k] < 0) for (double& c : n) c = -c;
                    break;
                }
            for (int k = 0; k < 3; ++k) scale = std::max({scale, std::fabs(g[0][k]), std::fabs(g[0][k] + g[1][k] + g[2][k])});
            pl.push_back({i, n, vdot(n, g[0])});
        }
        const double tol = 1e-9 * std::max(scale, 1e-300);
        std::sort(pl.begin(), pl.end(), [](const Pl& a, const Pl& b) { return a.d < b.d; });
        auto corners = [&](size_t i, std::vector<V3a>& c) {
            const auto& g = wgeom[i];
            const bool quad = (out.wprims[i].meta & WKIND_MASK) == PRIM_QUAD;
            c = {g[0], {g[0][0] + g[1][0], g[0][1] + g[1][1], g[0][2] + g[1][2]}};
            if (quad) c.push_back({g[0][0] + g[1][0] + g[2][0], g[0][1] + g[1][1] + g[2][1], g[0][2] + g[1][2] + g[2][2]});
            c.push_back({g[0][0] + g[2][0], g[0][1] + g[2][1], g[0][2] + g[2][2]});
        };
        // positive-area overlap of two convex polygons in one plane (separating axis test;
        // polygons that only touch along an edge or at a corner do not overlap)
        auto overlap = [&](const Pl& a, size_t j) {
            std::vector<V3a> pa, pb;
            corners(a.i, pa);
            corners(j, pb);
            V3a e1 = {pa[1][0] - pa[0][0], pa[1][1] - pa[0][1], pa[1][2] - pa[0][2]};
            const double l1 = std::sqrt(vdot(e1, e1));
            for (double& c : e1) c /= l1;
            const V3a e2 = {a.n[1] * e1[2] - a.n[2] * e1[1], a.n[2] * e1[0] - a.n[0] * e1[2], a.n[0] * e1[1] - a.n[1] * e1[0]};
            auto flat = [&](const std::vector<V3a>& p) {
                std::vector<std::array<double, 2>> q;
                for (const V3a& x : p) q.push_back({vdot(x, e1), vdot(x, e2)});
                return q;
            };
            const auto qa = flat(pa), qb = flat(pb);
            for (const auto* poly : {&qa, &qb})
                for (size_t k = 0; k < poly->size(); ++k) {
                    const auto& u = (*poly)[k];
                    const auto& v = (*poly)[(k + 1) % poly->size()];
                    const double ax = -(v[1] - u[1]), ay = v[0] - u[0];
                    double amin = INFINITY, amax = -INFINITY, bmin = INFINITY, bmax = -INFINITY;
                    for (const auto& x : qa) { const double t = ax * x[0] + ay * x[1]; amin = std::min(amin, t); amax = std::max(amax, t); }
                    for (const auto& x : qb) { const double t = ax * x[0] + ay * x[1]; bmin = std::min(bmin, t); bmax = std::max(bmax, t); }
                    const double slack = tol * std::sqrt(ax * ax + ay * ay);
                    if (amax <= bmin + slack || bmax <= amin + slack) return false;
                }
            return true;
        };
        std::vector<uint32_t> cls(out.wprims.size(), 0);
        bool any = false;
        for (size_t a = 0; a < pl.size(); ++a)
            for (size_t b = a + 1; b < pl.size() && pl[b].d - pl[a].d <= tol; ++b) {
                const V3a& na = pl[a].n;
                const V3a& nb = pl[b].n;
                if (std::fabs(na[0] - nb[0]) > 1e-9 || std::fabs(na[1] - nb[1]) > 1e-9 || std::fabs(na[2] - nb[2]) > 1e-9) continue;
                if (!overlap(pl[a], pl[b].i)) continue;
                const size_t lo = std::min(pl[a].i, pl[b].i), hi = std::max(pl[a].i, pl[b].i);
                cls[lo] |= WCLASS_LOSE;
                cls[hi] |= WCLASS_WIN;
                tie_pairs.emplace_back(lo, hi);
                any = true;
            }
        for (size_t i = 0; i < cls.size(); ++i) {
            if (cls[i] == (WCLASS_WIN | WCLASS_LOSE)) return false;
            out.wprims[i].meta |= cls[i] << WCLASS_SHIFT;
        }
        if (any) out.wflags |= WFLAG_COPLANAR;
        out.coplanar_pairs = (uint32_t)tie_pairs.size();
        return true;
    }

    void world_walk(const Object* o, const Affine& f) {
        if (!out.world_ok) return;
        switch (o->kind) {
            case Object::BvhEmpty: return;
            case Object::BvhLeaf: world_walk(o->child.get(), f); return;
            case Object::BvhNode: world_walk(o->left.get(), f); world_walk(o->right.get(), f); return;
            case Object::Sphere: {
                if (!f.translate_only) { out.world_ok = false; return; }  // uv needs the object frame
                DPrimWorld<double> w{};
                const V3a c = va(o->center);
                for (int k = 0; k < 3; ++k) { w.N[k] = c[k] - f.b[k]; w.AB[k] = va(o->speed)[k]; }
                w.D = o->radius;
                // f32 kernels (kernel.hpp sphere_t_world): the point P of the sphere (at time 0)
                // nearest the world origin in AB[3..5] and V = P - center in S, in f64 here
                const double cl = std::sqrt(w.N[0] * w.N[0] + w.N[1] * w.N[1] + w.N[2] * w.N[2]);
                const double ar = std::fabs(o->radius);
                for (int k = 0; k < 3; ++k) {
                    const double u = cl > 0.0 ? -w.N[k] / cl : (k == 1 ? -1.0 : 0.0);  // toward the origin
                    w.S[k] = ar * u;
                    w.AB[3 + k] = w.N[k] + ar * u;
                }
                // AB[6] = 1: tested in f64 (spheres larger than the scene scale)
                const double sl = std::sqrt(w.AB[0] * w.AB[0] + w.AB[1] * w.AB[1] + w.AB[2] * w.AB[2]);
                // knob NRT_SPHERE_F32 (A/B runs): 0 every sphere in f64, 2 every sphere in f32,
                // 1 spheres within the scene scale (|center| + |speed| + r; round 3 draft), 3 (default)
                // spheres whose anchor P lies within it (|P| + |speed|, any radius: the anchored
                // quadratic and the record's anchored surface step keep a ground sphere's f32 hits on
                // the surface; earth C3 6.48 -> 5.83 ms, earth_48 statistics green)
                static const int f32_mode = [] {
                    const char* e = std::getenv("NRT_SPHERE_F32");
                    return e ? (int)std::strtol(e, nullptr, 10) : 3;
                }();
                const double pl = std::sqrt(w.AB[3] * w.AB[3] + w.AB[4] * w.AB[4] + w.AB[5] * w.AB[5]);
                w.AB[6] = f32_mode == 2 || (f32_mode == 1 && cl + sl + ar <= SPHERE_F32_EXTENT) ||
                                  (f32_mode == 3 && pl + sl <= SPHERE_F32_EXTENT)
                              ? 0.0
                              : 1.0;
                const uint32_t mat = material(o->material);
                if (mat > WMAT_MASK) { out.world_ok = false; return; }
                w.meta = PRIM_SPHERE | (mat << WKIND_BITS);
                out.wprims.push_back(w);
                wgeom.push_back({});
                break;
            }
            case Object::Quad:
            case Object::Triangle: {
                const V3a n = va(o->normal), Aq = va(cross(o->v, o->w)), Bq = va(cross(o->w, o->u));
                const double a0 = dot(o->p, cross(o->v, o->w)), b0 = dot(o->p, cross(o->w, o->u));
                const V3a N = mtvec(f.M, n), A = mtvec(f.M, Aq), B = mtvec(f.M, Bq), S = mvec(f.R, n);
                {  // world-space parallelogram (for box fusion): x = M^-1 (x' - b)
                    const M3a Mi = inverse3(f.M);
                    const V3a p0 = va(o->p);
                    wgeom.push_back({mvec(Mi, {p0[0] - f.b[0], p0[1] - f.b[1], p0[2] - f.b[2]}), mvec(Mi, va(o->u)),
                                     mvec(Mi, va(o->v))});
                }
                DPrimWorld<double> w{};
                for (int k = 0; k < 3; ++k) { w.N[k] = N[k]; w.AB[2 * k] = A[k]; w.AB[2 * k + 1] = B[k]; w.S[k] = S[k]; }
                w.D = o->d - vdot(n, f.b);
                w.AB[6] = a0 - vdot(Aq, f.b);
                w.AB[7] = b0 - vdot(Bq, f.b);
                const uint32_t mat = material(o->material);
                if (mat > WMAT_MASK) { out.world_ok = false; return; }
                w.meta = (o->kind == Object::Quad ? PRIM_QUAD : PRIM_TRIANGLE) | (mat << WKIND_BITS);
                out.wprims.push_back(w);
                break;
            }
            case Object::Translate: {
                Affine g = f;
                for (int k = 0; k < 3; ++k) g.b[k] -= va(o->offset)[k];
                world_walk(o->child.get(), g);
                return;
            }
            case Object::Rotate:
            case Object::Scale: {
                const DXform<double>& x = out.xforms[xform_index(o)];
                M3a L, Linv;
                for (int q = 0; q < 9; ++q) { L[q] = x.m[q]; Linv[q] = x.inv[q]; }
                Affine g;
                g.M = mmul(L, f.M);
                g.b = mvec(L, f.b);
                g.R = f.R;
                g.translate_only = false;
                if (o->kind == Object::Scale) {
                    for (int k = 0; k < 3; ++k) g.b[k] += x.m[9 + k];
                } else {
                    g.R = mmul(f.R, Linv);
                }
                world_walk(o->child.get(), g);
                return;
            }
        }
        if (out.wprims.size() > WORLD_PRIM_CAP) out.world_ok = false;
    }
    // World BVH over the world primitives (wbvh.hpp); unusable trees (too deep for
    // the kernel's stack) leave wbvh_ok false and the instance BVH in charge.
    std::vector<std::array<double, 6>> wbounds;  // the world BVH's inputs (exact tree rebuild)
    std::vector<float> wcost;
    void build_wbvh() {
        std::vector<std::array<double, 6>> bounds(out.wprims.size());
        // SAH weights relative to a (binary) node visit: a plane test; f64 sphere tests cost ~4 of
        // them.  Tuning knob NRT_SAH_PRIM_COST scales the plane-test weight (host build only).
        float prim_cost = 1.0f;
        if (const char* e = std::getenv("NRT_SAH_PRIM_COST")) {
            const float v = std::strtof(e, nullptr);
            if (v > 0.0f && v < 100.0f) prim_cost = v;
        }
        float sphere_cost = NRT_SPHERE_COST;  // knob NRT_SPHERE_COST (A/B runs)
        if (const char* e = std::getenv("NRT_SPHERE_COST")) {
            const float v = std::strtof(e, nullptr);
            if (v > 0.0f && v < 100.0f) sphere_cost = v;
        }
        std::vector<float> cost(out.wprims.size(), prim_cost);
        bool far_sphere = false;
        for (size_t i = 0; i < out.wprims.size(); ++i) {
            const DPrimWorld<double>& w = out.wprims[i];
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            auto grow = [&](const double* p) {
                for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
            };
            const uint32_t kind = w.meta & WKIND_MASK;
            if (kind == PRIM_SPHERE) {  // center(t) = N + t * speed, t in [0, 1]
                // the f32 kernels' world-BVH leaves test spheres in f32 only (kernel.hpp world_prim_t,
                // the anchored quadratic): a sphere anchored outside the scene scale leaves the
                // scene's f32 renders to the instance BVH (wbvh_f32_ok); the tree is still built, for
                // the exact kernel's culling walk, which tests every primitive in f64
                if (w.AB[6] != 0.0) far_sphere = true;
                cost[i] = sphere_cost * prim_cost;
                for (int end = 0; end < 2; ++end)
                    for (int sg = -1; sg <= 1; sg += 2) {
                        double p[3];
                        for (int k = 0; k < 3; ++k) p[k] = w.N[k] + end * w.AB[k] + sg * std::fabs(w.D);
                        grow(p);
                    }
            } else {
                const auto& g = wgeom[i];
                for (int c = 0; c < (kind == PRIM_QUAD ? 4 : 3); ++c) {
                    double p[3];
                    for (int k = 0; k < 3; ++k) p[k] = g[0][k] + ((c & 1) ? g[1][k] : 0.0) + ((c & 2) ? g[2][k] : 0.0);
                    grow(p);
                }
            }
            for (int k = 0; k < 3; ++k) { bounds[i][k] = lo[k]; bounds[i][3 + k] = hi[k]; }
        }
        try {
            // leaves of at most WBVH4C_LEAF_MAX primitives where the compact 4-wide form can hold the
            // tree (DBvh4cNode; knob NRT_WBVH_LEAF = 1..8 for A/B runs)
            uint32_t leaf_max = out.wprims.size() < WBVH4C_MAX_PRIMS ? WBVH4C_LEAF_MAX : WBVH_LEAF_MAX;
            if (const char* e = std::getenv("NRT_WBVH_LEAF")) {
                const long v = std::strtol(e, nullptr, 10);
                if (v >= 1 && v <= (long)WBVH_LEAF_MAX) leaf_max = (uint32_t)v;
            }
            out.wbvh = build_world_bvh(bounds, cost, leaf_max);
        } catch (const std::runtime_error&) {
            out.wbvh_ok = false;
            return;
        }
        wbounds = bounds;
        wcost = cost;
        out.wprims_kind.resize(out.wprims.size());
        for (size_t i = 0; i < out.wprims.size(); ++i) out.wprims_kind[i] = out.wprims[i].meta & WKIND_MASK;
        out.wbvh_prims.reserve(out.wbvh.order.size());
        for (uint32_t idx : out.wbvh.order) out.wbvh_prims.push_back(out.wprims[idx]);
        out.wbvh_ok = true;
        out.wbvh_f32_ok = !far_sphere;
    }

    // DXform of a transform node (every chain was emitted by instance()).
    std::map<const Object*, uint32_t> xform_of;
    uint32_t xform_index(const Object* t) {
        auto it = xform_of.find(t);
        if (it == xform_of.end()) throw std::runtime_error("internal: transform without an instance");
        return it->second;
    }

    int32_t tree(const Object* o) {
        const uint32_t begin = (uint32_t)out.nodes.size();
        emit(o);
        const uint32_t end = (uint32_t)out.nodes.size();
        for (uint32_t k = begin; k < end; ++k)
            if (out.nodes[k].skip == (int32_t)end) out.nodes[k].skip = NODE_END;
        tree_ranges.emplace_back(begin, end);
        return end > begin ? (int32_t)begin : NODE_END;
    }

    int depth_of(int32_t root, std::map<int32_t, int>& memo, int guard) {
        if (root == NODE_END) return 0;
        if (guard > 64) throw std::runtime_error("instance nesting too deep");
        auto it = memo.find(root);
        if (it != memo.end()) return it->second;
        uint32_t end = root;
        for (auto& r : tree_ranges)
            if (r.first == (uint32_t)root) end = r.second;
        int d = 0;
        for (uint32_t k = (uint32_t)root; k < end; ++k) {
            const uint32_t meta = out.nodes[k].meta;
            if ((meta & 3) == NODE_INSTANCE) {
                const DInstance& inst = out.instances[meta >> 2];
                d = std::max(d, 1 + depth_of(inst.root, memo, guard + 1));
            }
        }
        memo[root] = d;
        return d;
    }

    void run(const Object* top) {
        out.root = tree(top);
        while (!pending.empty()) {
            auto [iid, target] = pending.front();
            pending.pop_front();
            auto it = blas_roots.find(target);
            if (it == blas_roots.end()) it = blas_roots.emplace(target, tree(target)).first;
            out.instances[iid].root = it->second;
        }
        // fast node array over the same instances
        out.root_fast = tree_fast(top);
        std::map<const Object*, int32_t> fast_roots;
        for (size_t iid = 0; iid < out.instances.size(); ++iid) {
            const Object* target = inst_targets[iid];
            auto it = fast_roots.find(target);
            if (it == fast_roots.end()) it = fast_roots.emplace(target, tree_fast(target)).first;
            out.instances[iid].root_fast = it->second;
        }
        if (!pending.empty()) throw std::runtime_error("internal: instance discovered only by the fast pass");
        for (const DMaterial& m : out.materials) {
            DMatFast f{};
            f.kind = m.kind;
            f.texture = m.texture;
            f.param = (float)m.param;
            if (m.kind != MAT_DIELECTRIC && out.textures[m.texture].kind == TEX_SOLID) {
                f.solid = 1;
                for (int k = 0; k < 3; ++k) f.color[k] = (float)out.textures[m.texture].color[k];
            }
            out.mats_fast.push_back(f);
        }
        std::map<int32_t, int> memo;
        out.max_depth = depth_of(out.root, memo, 0);
        if (out.max_depth > MAX_INSTANCE_DEPTH)
            throw std::runtime_error("instance nesting depth " + std::to_string(out.max_depth) + " exceeds " +
                                     std::to_string(MAX_INSTANCE_DEPTH));
        out.num_trees = (uint32_t)tree_ranges.size();
        out.world_ok = true;
        world_walk(top, Affine{});
        if (out.world_ok) out.world_ok = mark_coplanar();
        if (!out.world_ok) out.wprims.clear();
        if (out.world_ok && !out.wprims.empty()) build_wbvh();
        // fuse closed boxes, then group units by kind: one run per kind.  The f32
        // kernel's closest hit does not depend on the order except for exact ties
        // between coincident surfaces (the reference's order is kept within a kind).
        std::vector<std::vector<DPrimWorld<double>>> units;
        std::vector<uint32_t> unit_kind;
        std::vector<size_t> unit_src;  // wprims index of a single-primitive unit
        for (size_t i = 0; i < out.wprims.size();) {
            DPrimWorld<double> hdr;
            if (i + 6 <= out.wprims.size() && fuse_box(i, hdr)) {
                std::vector<DPrimWorld<double>> u{hdr};
                u.insert(u.end(), out.wprims.begin() + i, out.wprims.begin() + i + 6);
                units.push_back(std::move(u));
                unit_kind.push_back(box_y ? PRIM_BOXY : PRIM_BOX);
                unit_src.push_back(SIZE_MAX);
                i += 6;
            } else {
                DPrimWorld<double> w = out.wprims[i];
                if ((w.meta & WKIND_MASK) == PRIM_QUAD) axis_quad(w);
                const uint32_t wk = w.meta & WKIND_MASK;
                if (wk >= PRIM_QUAD_X && wk <= PRIM_QUAD_Z) {
                    const int a = (int)(wk - PRIM_QUAD_X);
                    tie_form[i] = axis_form(a, w.N[(a + 1) % 3]);
                } else if (wk == PRIM_QUAD || wk == PRIM_TRIANGLE) {
                    tie_form[i] = {4.0f, (float)w.N[0], (float)w.N[1], (float)w.N[2], (float)w.D};
                }
                units.push_back({w});
                unit_kind.push_back(w.meta & WKIND_MASK);
                unit_src.push_back(i);
                ++i;
            }
        }
        fuse_room(units, unit_kind, unit_src);
        // the world list resolves a coplanar tie by order alone: only when both faces compute
        // bit-identical t (equal tie forms); otherwise the scene uses the world BVH's keys
        for (const auto& [lo, hi] : tie_pairs) {
            auto a = tie_form.find(lo), b = tie_form.find(hi);
            if (a == tie_form.end() || b == tie_form.end() || a->second != b->second) out.list_ok = false;
            if (std::getenv("NRT_DEBUG_TIES")) {
                auto pr = [&](size_t i, decltype(a) it) {
                    fprintf(stderr, "  prim %zu:", i);
                    if (it != tie_form.end()) for (float v : it->second) fprintf(stderr, " %.9g", v);
                    fprintf(stderr, "\n");
                };
                fprintf(stderr, "tie pair\n");
                pr(lo, a);
                pr(hi, b);
            }
        }
        // Order: coplanar-tie losers, then the rest, then winners, by kind within each: the
        // later of two equal t wins in the kernel (device_scene.hpp WCLASS_*).
        // X, Y, Z quads, quads, triangles, spheres, y boxes, boxes, rooms
        static const int rank[9] = {5, 3, 4, 7, 0, 1, 2, 8, 6};
        auto cls_of = [&](size_t u) { return units[u][0].meta >> WCLASS_SHIFT; };
        auto phase = [&](size_t u) { return cls_of(u) == WCLASS_LOSE ? 0 : (cls_of(u) == WCLASS_WIN ? 2 : 1); };
        std::vector<size_t> order(units.size());
        for (size_t k = 0; k < order.size(); ++k) order[k] = k;
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
            if (phase(a) != phase(b)) return phase(a) < phase(b);
            return rank[unit_kind[a]] < rank[unit_kind[b]];
        });
        std::vector<DPrimWorld<double>> fused;
        std::vector<uint32_t> kinds;
        for (size_t k : order) {
            fused.insert(fused.end(), units[k].begin(), units[k].end());
            kinds.push_back(unit_kind[k]);
        }
        out.wprims.swap(fused);
        out.world_units = kinds.size();
        const uint32_t one = 1u << WRUN_KIND_BITS;
        size_t at = 0;  // first entry of the unit
        for (size_t u = 0; u < kinds.size(); ++u) {
            uint32_t kind = kinds[u];
            const size_t first = at;
            at += units[order[u]].size();
            if (kind == PRIM_SPHERE && out.wprims[first].AB[6] == 0.0) kind = PRIM_SPHERE32;
            if (kind >= PRIM_QUAD_X && kind != PRIM_SPHERE32)
                out.wflags |= WFLAG_AXIS_QUADS;  // axis quads, rooms and y boxes use 1/d
            if (!out.wruns.empty() && (out.wruns.back() & WRUN_KIND_MASK) == kind &&
                (out.wruns.back() >> WRUN_KIND_BITS) < (1u << 27))
                out.wruns.back() += one;
            else
                out.wruns.push_back(kind | one);
        }
    }
};

float round_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = std::nextafter(f, -INFINITY);
    return f;
}
float round_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = std::nextafter(f, INFINITY);
    return f;
}

}  // namespace

// World primitive k (the reference's depth-first candidate order, world_walk) is the k-th
// primitive of a full depth-first walk of the exact tree (every box taken); record the DPrim
// and instance of each BVH slot for the exact kernel's world-BVH mode.  Nested instances, or
// any disagreement in count or kind, leave the mapping empty (mode unavailable).
static void map_exact_refs(FlatScene& s) {
    s.wexact.clear();
    s.wexact_prims.clear();
    const WorldBvh& tree = s.exact_tree();
    if (!s.wbvh_ok || tree.order.empty()) return;
    std::vector<std::pair<uint32_t, int32_t>> seq;
    bool ok = true;
    auto walk = [&](int32_t node, int32_t inst, auto&& self) -> void {
        while (ok && node >= 0 && node < (int32_t)s.nodes.size()) {
            const DNode<double>& d = s.nodes[node];
            const uint32_t kind = d.meta & 3u;
            if (kind == NODE_INNER) {
                ++node;
                continue;
            }
            if (kind == NODE_PRIM) {
                seq.emplace_back(d.meta >> 2, inst);
            } else if (kind == NODE_INSTANCE) {
                const uint32_t idx = d.meta >> 2;
                if (inst >= 0 || idx >= s.instances.size()) {
                    ok = false;
                    return;
                }
                self(s.instances[idx].root, (int32_t)idx, self);
            } else {
                ok = false;
                return;
            }
            node = d.skip;
        }
    };
    walk(s.root, -1, walk);
    if (!ok || seq.size() != tree.order.size() || seq.size() != s.wbvh.order.size()) return;
    std::vector<DExactRef> refs(tree.order.size());
    for (size_t slot = 0; slot < refs.size(); ++slot) {
        const uint32_t rank = tree.order[slot];
        if (rank >= seq.size() || rank >= s.wbvh.order.size()) return;
        const auto& e = seq[rank];
        // kind of world primitive `rank` (the shared tree's slot order is a permutation of it)
        const uint32_t wkind = rank < s.wprims_kind.size() ? s.wprims_kind[rank] : 0xFFFFFFFFu;
        if (e.first >= s.prims.size() || s.prims[e.first].kind != wkind) return;
        refs[slot] = DExactRef{e.first, e.second, rank, 0u};
    }
    // the same slots' world primitives (the shared tree's slot order is wbvh.order)
    std::vector<uint32_t> shared_slot(s.wbvh.order.size());
    for (size_t k = 0; k < s.wbvh.order.size(); ++k) shared_slot[s.wbvh.order[k]] = (uint32_t)k;
    std::vector<DPrimWorld<double>> prims(tree.order.size());
    for (size_t slot = 0; slot < prims.size(); ++slot) prims[slot] = s.wbvh_prims[shared_slot[tree.order[slot]]];
    s.wexact = std::move(refs);
    s.wexact_prims = std::move(prims);
}

constexpr float EXACT_SAH_PRIM_COST = 3.0f;

FlatScene flatten_scene(const ObjectPtr& top) {
    Flattener f;
    f.run(top.get());
    map_exact_refs(f.out);
    if (!f.out.wexact.empty()) {
        // several instance chains (or the top level and a chain): a tree of its own for the
        // exact kernel, with heavier primitives (smaller leaves)
        int32_t first = f.out.wexact[0].inst;
        bool several = false;
        for (const DExactRef& r : f.out.wexact) several |= r.inst != first;
        if (several) {
            std::vector<float> cost = f.wcost;
            for (float& c : cost) c *= EXACT_SAH_PRIM_COST;
            try {
                f.out.wbvh_x = build_world_bvh(f.wbounds, cost);
                map_exact_refs(f.out);
            } catch (const std::runtime_error&) {
                f.out.wbvh_x = WorldBvh();
                map_exact_refs(f.out);
            }
        }
    }
    return std::move(f.out);
}

FlatScene32 to_f32(const FlatScene& s) {
    FlatScene32 o;
    o.nodes.resize(s.nodes_fast.size());
    for (size_t i = 0; i < s.nodes_fast.size(); ++i) {
        for (int k = 0; k < 3; ++k) {
            o.nodes[i].bmin[k] = round_down(s.nodes_fast[i].bmin[k]);
            o.nodes[i].bmax[k] = round_up(s.nodes_fast[i].bmax[k]);
        }
        o.nodes[i].meta = s.nodes_fast[i].meta;
        o.nodes[i].skip = s.nodes_fast[i].skip;
    }
    o.fprims.resize(s.fprims.size());
    for (size_t i = 0; i < s.fprims.size(); ++i) {
        const auto& a = s.fprims[i];
        auto& b = o.fprims[i];
        for (int k = 0; k < 3; ++k) { b.n[k] = (float)a.n[k]; b.A[k] = (float)a.A[k]; b.B[k] = (float)a.B[k]; }
        b.d = (float)a.d; b.a0 = (float)a.a0; b.b0 = (float)a.b0;
        b.kind = a.kind; b.material = a.material; b.pad[0] = b.pad[1] = 0;
    }
    auto world32 = [](const std::vector<DPrimWorld<double>>& src, std::vector<DPrimWorld<float>>& dst) {
        dst.resize(src.size());
        for (size_t i = 0; i < src.size(); ++i) {
            const auto& a = src[i];
            auto& b = dst[i];
            for (int k = 0; k < 3; ++k) { b.N[k] = (float)a.N[k]; b.S[k] = (float)a.S[k]; }
            for (int k = 0; k < 8; ++k) b.AB[k] = (float)a.AB[k];
            b.D = (float)a.D;
            b.meta = a.meta;
        }
    };
    world32(s.wprims, o.wprims);
    world32(s.wbvh_prims, o.wbvh_prims);
    world32(s.wexact_prims, o.wexact_prims);
    o.inst_fast.resize(s.inst_fast.size());
    for (size_t i = 0; i < s.inst_fast.size(); ++i) {
        const auto& a = s.inst_fast[i];
        auto& b = o.inst_fast[i];
        for (int q = 0; q < 9; ++q) { b.A[q] = (float)a.A[q]; b.C[q] = (float)a.C[q]; b.N[q] = (float)a.N[q]; }
        for (int r = 0; r < 3; ++r) { b.b[r] = (float)a.b[r]; b.c[r] = (float)a.c[r]; b.pad[r] = 0.f; }
    }
    o.prims.resize(s.prims.size());
    for (size_t i = 0; i < s.prims.size(); ++i) {
        const auto& a = s.prims[i];
        auto& b = o.prims[i];
        for (int k = 0; k < 3; ++k) {
            b.a[k] = (float)a.a[k]; b.b[k] = (float)a.b[k]; b.c[k] = (float)a.c[k];
            b.n[k] = (float)a.n[k]; b.w[k] = (float)a.w[k];
        }
        b.s = (float)a.s;
        b.kind = a.kind;
        b.material = a.material;
    }
    o.xforms.resize(s.xforms.size());
    for (size_t i = 0; i < s.xforms.size(); ++i) {
        for (int k = 0; k < 12; ++k) {
            o.xforms[i].m[k] = (float)s.xforms[i].m[k];
            o.xforms[i].inv[k] = (float)s.xforms[i].inv[k];
        }
        o.xforms[i].kind = s.xforms[i].kind;
    }
    return o;
}

// ------------------------------------------------------------------- dump
namespace {

void hex(std::string& s, double v) {
    char buf[64];
    snprintf(buf, sizeof buf, " %a", v);
    s += buf;
}
void hex3(std::string& s, V3 v) { hex(s, v.x); hex(s, v.y); hex(s, v.z); }
void hexbox(std::string& s, const AABB& b) {
    hex(s, b.x.min); hex(s, b.x.max); hex(s, b.y.min); hex(s, b.y.max); hex(s, b.z.min); hex(s, b.z.max);
}

void dump_tex(std::string& s, const Texture* t) {
    switch (t->kind) {
        case Texture::Solid: s += " SOLID"; hex3(s, t->color); break;
        case Texture::Image: {
            char buf[64];
            double sum = 0;
            for (float f : *t->texels) sum += f;
            snprintf(buf, sizeof buf, " IMAGE %u %u", t->width, t->height);
            s += buf;
            hex(s, sum);
            break;
        }
        case Texture::Checker:
            s += " CHECKER";
            hex(s, t->scale);
            s += " (";
            dump_tex(s, t->even.get());
            s += " ) (";
            dump_tex(s, t->odd.get());
            s += " )";
            break;
        case Texture::Noise:
        case Texture::Marble: {
            char buf[64];
            const FbmParams& f = t->fbm;
            snprintf(buf, sizeof buf, t->kind == Texture::Noise ? " NOISE %u %u" : " MARBLE %u %u", f.seed, f.octaves);
            s += buf;
            hex(s, f.frequency);
            hex(s, f.lacunarity);
            hex(s, f.persistence);
            break;
        }
    }
}

void dump_mat(std::string& s, const Material* m) {
    switch (m->kind) {
        case Material::Lambertian: s += " LAMBERTIAN"; dump_tex(s, m->texture.get()); break;
        case Material::Metal: s += " METAL"; hex(s, m->fuzz); dump_tex(s, m->texture.get()); break;
        case Material::Dielectric: s += " DIELECTRIC"; hex(s, m->refraction_index); break;
        case Material::DiffuseLight: s += " DIFFUSE_LIGHT"; hex(s, m->intensity); dump_tex(s, m->texture.get()); break;
    }
}

void dump_obj(std::string& s, const Object* o, int indent) {
    s.append((size_t)indent * 2, ' ');
    switch (o->kind) {
        case Object::BvhEmpty: s += "BVH_EMPTY\n"; return;
        case Object::BvhLeaf: s += "BVH_LEAF\n"; dump_obj(s, o->child.get(), indent + 1); return;
        case Object::BvhNode:
            s += "BVH_NODE";
            hexbox(s, o->bbox);
            s += "\n";
            dump_obj(s, o->left.get(), indent + 1);
            dump_obj(s, o->right.get(), indent + 1);
            return;
        case Object::Sphere:
            s += "SPHERE";
            hex3(s, o->center); hex(s, o->radius); hex3(s, o->speed); hexbox(s, o->bbox);
            dump_mat(s, o->material.get());
            s += "\n";
            return;
        case Object::Quad:
        case Object::Triangle:
            s += o->kind == Object::Quad ? "QUAD" : "TRIANGLE";
            hex3(s, o->p); hex3(s, o->u); hex3(s, o->v); hex3(s, o->normal); hex(s, o->d); hex3(s, o->w);
            hexbox(s, o->bbox);
            dump_mat(s, o->material.get());
            s += "\n";
            return;
        case Object::Translate:
            s += "TRANSLATE"; hex3(s, o->offset); hexbox(s, o->bbox); s += "\n";
            dump_obj(s, o->child.get(), indent + 1);
            return;
        case Object::Rotate:
            s += "ROTATE";
            for (int c = 0; c < 3; ++c) hex3(s, o->rot.c[c]);
            for (int c = 0; c < 3; ++c) hex3(s, o->rot_inv.c[c]);
            hexbox(s, o->bbox);
            s += "\n";
            dump_obj(s, o->child.get(), indent + 1);
            return;
        case Object::Scale:
            s += "SCALE";
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < 4; ++r) hex(s, o->scale_inv.c[c][r]);
            hexbox(s, o->bbox);
            s += "\n";
            dump_obj(s, o->child.get(), indent + 1);
            return;
    }
}

}  // namespace

std::string dump_graph(const ObjectPtr& root) {
    std::string s;
    dump_obj(s, root.get(), 0);
    return s;
}

}  // namespace nrt
