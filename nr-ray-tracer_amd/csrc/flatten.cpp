// Scene graph -> threaded BVH arrays (device_scene.hpp).
#include "flatten.hpp"

#include <cmath>
#include <cstdio>
#include <deque>
#include <map>
#include <stdexcept>

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
            case Texture::Image:
                d.kind = TEX_IMAGE;
                d.a = t->width;
                d.b = t->height;
                d.offset = out.texels.size() / 3;
                out.texels.insert(out.texels.end(), t->texels->begin(), t->texels->end());
                break;
            case Texture::Checker: {
                d.kind = TEX_CHECKER;
                d.scale = t->scale;
                const uint32_t e = texture(t->even), o = texture(t->odd);
                d.a = e;
                d.b = o;
                break;
            }
            case Texture::Unsupported:
                throw std::runtime_error("texture kind '" + t->note +
                                         "' (Perlin noise) is outside the accelerated path (SURVEY.md §8f rank 4)");
        }
        const uint32_t id = (uint32_t)out.textures.size();
        out.textures.push_back(d);
        tex_ids[t.get()] = id;
        return id;
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
                DInstance inst{};
                inst.first_xform = (uint32_t)out.xforms.size();
                const Object* t = o;
                while (is_transform(t)) {
                    xform(t);
                    t = t->child.get();
                }
                inst.num_xforms = (uint32_t)out.xforms.size() - inst.first_xform;
                inst.root = NODE_END;
                const uint32_t iid = (uint32_t)out.instances.size();
                out.instances.push_back(inst);
                pending.emplace_back(iid, t);
                const uint32_t idx = push(NODE_INSTANCE, iid);
                out.nodes[idx].skip = (int32_t)idx + 1;
                return;
            }
        }
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
        std::map<int32_t, int> memo;
        out.max_depth = depth_of(out.root, memo, 0);
        if (out.max_depth > MAX_INSTANCE_DEPTH)
            throw std::runtime_error("instance nesting depth " + std::to_string(out.max_depth) + " exceeds " +
                                     std::to_string(MAX_INSTANCE_DEPTH));
        out.num_trees = (uint32_t)tree_ranges.size();
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

FlatScene flatten_scene(const ObjectPtr& top) {
    Flattener f;
    f.run(top.get());
    return std::move(f.out);
}

FlatScene32 to_f32(const FlatScene& s) {
    FlatScene32 o;
    o.nodes.resize(s.nodes.size());
    for (size_t i = 0; i < s.nodes.size(); ++i) {
        for (int k = 0; k < 3; ++k) {
            o.nodes[i].bmin[k] = round_down(s.nodes[i].bmin[k]);
            o.nodes[i].bmax[k] = round_up(s.nodes[i].bmax[k]);
        }
        o.nodes[i].meta = s.nodes[i].meta;
        o.nodes[i].skip = s.nodes[i].skip;
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
        case Texture::Unsupported: s += " UNSUPPORTED " + t->note; break;
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
