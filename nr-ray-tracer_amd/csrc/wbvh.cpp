// Binned-SAH build of the f32 kernel's world BVH (wbvh.hpp).
//
// Standard top-down binned SAH (16 bins per axis, all three axes), traversal
// cost 1, per-primitive intersection costs from the caller, leaves of at most
// WBVH_LEAF_MAX primitives.  The
// tree is only an acceleration structure of the fast kernel: which primitive
// is hit does not depend on it (closest hit, f32 statistical parity).
#include "wbvh.hpp"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <stdexcept>

namespace nrt {

namespace {

struct Box {
    double lo[3] = {INFINITY, INFINITY, INFINITY};
    double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], b.lo[k]); hi[k] = std::max(hi[k], b.hi[k]); }
    }
    void grow(const double* p) {
        for (int k = 0; k < 3; ++k) { lo[k] = std::min(lo[k], p[k]); hi[k] = std::max(hi[k], p[k]); }
    }
    double area() const {
        if (!(hi[0] >= lo[0])) return 0.0;
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }
};

struct Item {
    Box box;
    double c[3];
    uint32_t index;
    float cost;
};

struct Builder {
    std::vector<Item> items;
    WorldBvh out;
    double pad = 0.0;
    uint32_t leaf_max = WBVH_LEAF_MAX;

    int BINS = 16;  // SAH bins per axis (NRT_WBVH_BINS, 2..256)

    float down(double x) const {
        float f = (float)(x - pad);
        if ((double)f > x - pad) f = std::nextafter(f, -INFINITY);
        return f;
    }
    float up(double x) const {
        float f = (float)(x + pad);
        if ((double)f < x + pad) f = std::nextafter(f, INFINITY);
        return f;
    }

    Box bounds(size_t b, size_t e) const {
        Box r;
        for (size_t i = b; i < e; ++i) r.grow(items[i].box);
        return r;
    }

    int32_t leaf(size_t b, size_t e) {
        const uint32_t first = (uint32_t)out.order.size();
        if (first >= (1u << 27)) throw std::runtime_error("world BVH: too many primitives");
        for (size_t i = b; i < e; ++i) out.order.push_back(items[i].index);
        return ~(int32_t)((first << 3) | (uint32_t)(e - b - 1));
    }

    // Returns the child ref of items[b, e).
    int32_t build(size_t b, size_t e, uint32_t depth) {
        const size_t n = e - b;
        if (n <= 1) return leaf(b, e);
        Box cb;  // centroid bounds
        for (size_t i = b; i < e; ++i) cb.grow(items[i].c);
        const Box all = bounds(b, e);
        double best_cost = INFINITY;
        int best_axis = -1, best_split = 0;
        for (int a = 0; a < 3; ++a) {
            const double ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0.0)) continue;
            std::vector<Box> bin_box((size_t)BINS);
            std::vector<size_t> bin_n((size_t)BINS, 0);
            std::vector<double> bin_c((size_t)BINS, 0.0);
            const double scale = BINS / ext;
            for (size_t i = b; i < e; ++i) {
                int k = (int)((items[i].c[a] - cb.lo[a]) * scale);
                k = std::min(std::max(k, 0), BINS - 1);
                bin_box[k].grow(items[i].box);
                ++bin_n[k];
                bin_c[k] += items[i].cost;
            }
            std::vector<double> right_area((size_t)BINS), right_c((size_t)BINS);
            std::vector<size_t> right_n((size_t)BINS);
            Box acc;
            size_t cnt = 0;
            double csum = 0;
            for (int k = BINS - 1; k > 0; --k) {
                acc.grow(bin_box[k]);
                cnt += bin_n[k];
                csum += bin_c[k];
                right_area[k] = acc.area();
                right_n[k] = cnt;
                right_c[k] = csum;
            }
            acc = Box();
            cnt = 0;
            csum = 0;
            for (int k = 0; k < BINS - 1; ++k) {  // split between bin k and k + 1
                acc.grow(bin_box[k]);
                cnt += bin_n[k];
                csum += bin_c[k];
                if (cnt == 0 || right_n[k + 1] == 0) continue;
                const double cost = acc.area() * csum + right_area[k + 1] * right_c[k + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_split = k;
                }
            }
        }
        double leaf_cost = 0;
        for (size_t i = b; i < e; ++i) leaf_cost += items[i].cost;
        const double split_cost = 1.0 + best_cost / std::max(all.area(), 1e-300);
        size_t mid;
        if (best_axis < 0) {  // all centroids coincide: split by count
            if (n <= leaf_max) return leaf(b, e);
            mid = b + n / 2;
        } else {
            if (n <= leaf_max && leaf_cost <= split_cost) return leaf(b, e);
            const double ext = cb.hi[best_axis] - cb.lo[best_axis], scale = BINS / ext;
            auto it = std::partition(items.begin() + b, items.begin() + e, [&](const Item& x) {
                int k = (int)((x.c[best_axis] - cb.lo[best_axis]) * scale);
                k = std::min(std::max(k, 0), BINS - 1);
                return k <= best_split;
            });
            mid = (size_t)(it - items.begin());
            if (mid == b || mid == e) mid = b + n / 2;
        }
        if (depth + 1 > out.depth) out.depth = depth + 1;
        const int32_t idx = (int32_t)out.nodes.size();
        out.nodes.emplace_back();
        const int32_t c0 = build(b, mid, depth + 1);
        const int32_t c1 = build(mid, e, depth + 1);
        const Box b0 = bounds(b, mid), b1 = bounds(mid, e);
        DBvhNode& nd = out.nodes[idx];
        for (int k = 0; k < 3; ++k) {
            nd.lo0[k] = down(b0.lo[k]); nd.hi0[k] = up(b0.hi[k]);
            nd.lo1[k] = down(b1.lo[k]); nd.hi1[k] = up(b1.hi[k]);
        }
        nd.c0 = c0;
        nd.c1 = c1;
        return idx;
    }
};

// Collapse the binary tree into 4-wide nodes.  Greedy (the round-2 default): a 4-node's children are
// the binary node's children with inner ones opened (largest box first) until four.  SAH (NRT_WBVH_COLLAPSE
// = 1): the cover of every 4-node is chosen by dynamic programming over the binary tree to minimise the
// expected cost (surface area heuristic: a node visit costs `visit` per unit of its box's area, a leaf its
// primitives' costs), and a subtree of at most `leaf_max` primitives may become one leaf (its primitives
// are contiguous in the binary tree's order) -- Ylitie, Karras & Laine, "Efficient incoherent ray
// traversal on GPUs through compressed wide BVHs", HPG 2017, section 4.1, for a 4-wide tree.
struct Collapse {
    const std::vector<DBvhNode>& n2;
    std::vector<DBvh4Node>& n4;
    struct Slot {
        int32_t ref;
        float lo[3], hi[3];
    };
    static float area(const Slot& c) {
        const float x = c.hi[0] - c.lo[0], y = c.hi[1] - c.lo[1], z = c.hi[2] - c.lo[2];
        return x * y + y * z + z * x;
    }
    int32_t build(int32_t ref) {  // ref: an inner binary node
        std::vector<Slot> kids;
        auto open = [&](int32_t r) {
            const DBvhNode& b = n2[r];
            Slot a{b.c0, {b.lo0[0], b.lo0[1], b.lo0[2]}, {b.hi0[0], b.hi0[1], b.hi0[2]}};
            Slot c{b.c1, {b.lo1[0], b.lo1[1], b.lo1[2]}, {b.hi1[0], b.hi1[1], b.hi1[2]}};
            kids.push_back(a);
            kids.push_back(c);
        };
        open(ref);
        while (kids.size() < 4) {
            int best = -1;
            for (int k = 0; k < (int)kids.size(); ++k)
                if (kids[k].ref >= 0 && (best < 0 || area(kids[k]) > area(kids[best]))) best = k;
            if (best < 0) break;
            const int32_t r = kids[best].ref;
            kids.erase(kids.begin() + best);
            open(r);
        }
        const int32_t idx = (int32_t)n4.size();
        n4.emplace_back();
        int32_t child[4];
        for (int k = 0; k < 4; ++k)
            child[k] = k < (int)kids.size() ? (kids[k].ref >= 0 ? build(kids[k].ref) : kids[k].ref) : WBVH_DONE;
        quantize(idx, kids, child);
        return idx;
    }

    // ---- SAH collapse (dynamic programming)
    double visit = 1.0;        // cost of a 4-node visit per unit area
    uint32_t leaf_max = 4;     // a subtree of at most this many primitives may become a leaf
    const std::vector<float>* prim_cost = nullptr;  // per BVH slot (binary order)
    struct Info {
        Slot box;
        uint32_t first = 0, count = 0;  // the subtree's primitive slots in the binary order
        double cost_sum = 0;            // its primitives' costs
        double F[5] = {0, 0, 0, 0, 0};  // F[k]: best cover of the subtree with at most k slots
        int8_t split[5] = {0, 0, 0, 0, 0};  // k >= 2: slots given to the left child (0: one slot)
        bool as_leaf = false;           // F[1] is a leaf (else a 4-node / the binary leaf)
        int8_t root_split = 0;          // the 4-node's slots to the left child
    };
    std::vector<Info> inner;               // per inner binary node
    std::vector<Info> leaves;              // per binary leaf (index by order)
    std::vector<int32_t> leaf_of_ref;      // (unused by value; leaves are keyed by their first slot)

    Info& info(int32_t ref) {
        if (ref >= 0) return inner[(size_t)ref];
        const uint32_t v = ~(uint32_t)ref;
        return leaves[v >> 3];
    }
    void prepare(int32_t ref, const Slot& box) {
        Info& in = info(ref);
        in.box = box;
        if (ref < 0) {
            const uint32_t v = ~(uint32_t)ref;
            in.first = v >> 3;
            in.count = (v & 7u) + 1u;
            in.cost_sum = 0;
            for (uint32_t k = 0; k < in.count; ++k) in.cost_sum += (*prim_cost)[in.first + k];
            const double c = area(box) * in.cost_sum;
            for (int k = 0; k <= 4; ++k) in.F[k] = c;
            in.as_leaf = true;
            return;
        }
        const DBvhNode& b = n2[(size_t)ref];
        const Slot l{b.c0, {b.lo0[0], b.lo0[1], b.lo0[2]}, {b.hi0[0], b.hi0[1], b.hi0[2]}};
        const Slot r{b.c1, {b.lo1[0], b.lo1[1], b.lo1[2]}, {b.hi1[0], b.hi1[1], b.hi1[2]}};
        prepare(b.c0, l);
        prepare(b.c1, r);
        const Info &L = info(b.c0), &R = info(b.c1);
        in.first = L.first;
        in.count = L.count + R.count;
        in.cost_sum = L.cost_sum + R.cost_sum;
        // as a 4-node: its own visit plus the best 4-slot cover of its two children
        double g = INFINITY;
        for (int j = 1; j <= 3; ++j) {
            const double c = L.F[j] + R.F[4 - j];
            if (c < g) {
                g = c;
                in.root_split = (int8_t)j;
            }
        }
        g += visit * area(box);
        const bool can_leaf = in.count <= leaf_max && L.first + L.count == R.first;
        const double lf = can_leaf ? area(box) * in.cost_sum : INFINITY;
        in.as_leaf = lf < g;
        in.F[1] = std::min(g, lf);
        in.split[1] = 0;
        for (int k = 2; k <= 4; ++k) {
            in.F[k] = in.F[1];
            in.split[k] = 0;
            for (int j = 1; j < k; ++j) {
                const double c = L.F[j] + R.F[k - j];
                if (c < in.F[k]) {
                    in.F[k] = c;
                    in.split[k] = (int8_t)j;
                }
            }
        }
    }
    // the cover items of `ref` with at most k slots
    void cover(int32_t ref, int k, std::vector<Slot>& out) {
        Info& in = info(ref);
        if (ref < 0 || k == 1 || in.split[k] == 0) {
            Slot s = in.box;
            if (ref >= 0 && in.as_leaf) s.ref = ~(int32_t)((in.first << 3) | (in.count - 1u));
            else s.ref = ref;
            out.push_back(s);
            return;
        }
        const DBvhNode& b = n2[(size_t)ref];
        cover(b.c0, in.split[k], out);
        cover(b.c1, k - in.split[k], out);
    }
    int32_t build_sah(int32_t ref) {  // ref: an inner binary node that is a 4-node
        Info& in = info(ref);
        const DBvhNode& b = n2[(size_t)ref];
        std::vector<Slot> kids;
        cover(b.c0, in.root_split, kids);
        cover(b.c1, 4 - in.root_split, kids);
        const int32_t idx = (int32_t)n4.size();
        n4.emplace_back();
        int32_t child[4];
        for (int k = 0; k < 4; ++k)
            child[k] = k < (int)kids.size() ? (kids[k].ref >= 0 ? build_sah(kids[k].ref) : kids[k].ref) : WBVH_DONE;
        quantize(idx, kids, child);
        return idx;
    }

    // node idx: quantized boxes of `kids`, child refs
    void quantize(int32_t idx, const std::vector<Slot>& kids, const int32_t child[4]) {
        DBvh4Node& nd = n4[(size_t)idx];
        std::memset(&nd, 0, sizeof nd);
        for (int a = 0; a < 3; ++a) {
            float lo = INFINITY, hi = -INFINITY;
            for (const Slot& k : kids) { lo = std::min(lo, k.lo[a]); hi = std::max(hi, k.hi[a]); }
            nd.org[a] = lo;
            // smallest step 2^e (1 + m / 4) (m = 0..3: a power of two with two mantissa bits, so the
            // quantized boxes are up to 1.6x tighter than with powers of two alone) with 255 steps
            // covering the extent, then outward rounding; steps tried in increasing order
            int e = hi > lo ? (int)std::floor(std::log2(((double)hi - (double)lo) / 255.0)) : -126;
            e = std::max(-126, std::min(127, e));
            for (int mi = 0;; ++mi) {
                int m = NRT_WBVH_STEP_MANTISSA ? (mi & 3) : 0;
                if (NRT_WBVH_STEP_MANTISSA ? (mi > 0 && m == 0) : mi > 0) ++e;
                e = std::max(-126, std::min(127, e));
                const float step = std::ldexp(1.0f + 0.25f * (float)m, e);
                bool ok = true;
                uint32_t qlo = 0, qhi = 0;
                for (size_t k = 0; k < kids.size() && ok; ++k) {
                    double ql = std::floor(((double)kids[k].lo[a] - lo) / step), qh = std::ceil(((double)kids[k].hi[a] - lo) / step);
                    ql = std::max(0.0, ql);
                    while (ql > 0 && std::fma((float)ql, step, lo) > kids[k].lo[a]) ql -= 1;
                    while (qh <= 255 && std::fma((float)qh, step, lo) < kids[k].hi[a]) qh += 1;
                    if (qh > 255) { ok = false; break; }
                    qlo |= (uint32_t)ql << (8 * k);
                    qhi |= (uint32_t)qh << (8 * k);
                }
                if (!ok && (e < 127 || m < 3)) continue;
                for (size_t k = kids.size(); k < 4; ++k) qlo |= 255u << (8 * k);  // empty slots (also ref-checked)
                nd.qlo[a] = qlo;
                nd.qhi[a] = qhi;
                nd.exps |= ((uint32_t)(e + 127) << 2 | (uint32_t)m) << (10 * a);  // (device_scene.hpp wbvh_step)
                break;
            }
        }
        for (int k = 0; k < 4; ++k) nd.child[k] = child[k];
    }
};

}  // namespace

// The compact form of nodes4 (device_scene.hpp DBvh4cNode), or empty when a ref does not fit.
static std::vector<DBvh4cNode> compact_nodes(const std::vector<DBvh4Node>& n4, size_t slots) {
    std::vector<DBvh4cNode> out;
    if (n4.size() >= WBVH4C_MAX_NODES || slots >= WBVH4C_MAX_PRIMS) return out;
    out.resize(n4.size());
    for (size_t i = 0; i < n4.size(); ++i) {
        const DBvh4Node& a = n4[i];
        DBvh4cNode& c = out[i];
        std::memset(&c, 0, sizeof c);
        for (int k = 0; k < 3; ++k) {
            c.org[k] = a.org[k];
            c.qlo[k] = a.qlo[k];
            c.qhi[k] = a.qhi[k];
        }
        c.exps = a.exps;
        for (int k = 0; k < 4; ++k) {
            const int32_t r = a.child[k];
            if (r == WBVH_DONE) {
                c.child[k] = 0;  // empty slot: its box is never hit
            } else if (r >= 0) {
                c.child[k] = (uint16_t)r;
            } else {
                const uint32_t v = ~(uint32_t)r, first = v >> 3, cnt = (v & 7u) + 1u;
                if (cnt > WBVH4C_LEAF_MAX) return {};
                c.child[k] = (uint16_t)(WBVH4C_LEAF | first << 2 | (cnt - 1u));
            }
        }
    }
    return out;
}

// The binary tree threaded in depth-first order for octant `oct` (device_scene.hpp DThreadNode):
// nearer child first along the octant's diagonal, planes as (near, far).
static void thread_tree(const std::vector<DBvhNode>& nodes, int32_t root, int oct, std::vector<DThreadNode>& out) {
    const float sg[3] = {(oct & 1) ? -1.0f : 1.0f, (oct & 2) ? -1.0f : 1.0f, (oct & 4) ? -1.0f : 1.0f};
    const size_t base = out.size();
    auto emit = [&](auto&& self, int32_t ref, const float* lo, const float* hi) -> void {
        const size_t idx = out.size();
        DThreadNode t{};
        for (int k = 0; k < 3; ++k) {
            t.nearp[k] = sg[k] > 0 ? lo[k] : hi[k];
            t.farp[k] = sg[k] > 0 ? hi[k] : lo[k];
        }
        t.leaf = ref < 0 ? ref : 0;
        out.push_back(t);
        if (ref >= 0) {
            const DBvhNode& b = nodes[(size_t)ref];
            float d0 = 0, d1 = 0;
            for (int k = 0; k < 3; ++k) {
                d0 += sg[k] * (b.lo0[k] + b.hi0[k]);
                d1 += sg[k] * (b.lo1[k] + b.hi1[k]);
            }
            if (d0 <= d1) {
                self(self, b.c0, b.lo0, b.hi0);
                self(self, b.c1, b.lo1, b.hi1);
            } else {
                self(self, b.c1, b.lo1, b.hi1);
                self(self, b.c0, b.lo0, b.hi0);
            }
        }
        out[idx].skip = (int32_t)(out.size() - base);
    };
    // the root's box: the union of its children's, or everything for a single leaf
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = -3e38f;
        hi[k] = 3e38f;
    }
    if (root >= 0) {
        const DBvhNode& b = nodes[(size_t)root];
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(b.lo0[k], b.lo1[k]);
            hi[k] = std::max(b.hi0[k], b.hi1[k]);
        }
    }
    if (root != WBVH_DONE) emit(emit, root, lo, hi);
}

WorldBvh build_world_bvh(const std::vector<std::array<double, 6>>& bounds, const std::vector<float>& cost,
                         uint32_t leaf_max) {
    Builder bld;
    bld.leaf_max = std::max<uint32_t>(1u, std::min(leaf_max, WBVH_LEAF_MAX));
    if (const char* e = std::getenv("NRT_WBVH_BINS")) {  // (A/B knob)
        const long v = std::strtol(e, nullptr, 10);
        if (v >= 2 && v <= 256) bld.BINS = (int)v;
    }
    bld.items.resize(bounds.size());
    double scale = 0.0;
    for (size_t i = 0; i < bounds.size(); ++i) {
        Item& it = bld.items[i];
        for (int k = 0; k < 3; ++k) {
            it.box.lo[k] = bounds[i][k];
            it.box.hi[k] = bounds[i][3 + k];
            it.c[k] = 0.5 * (it.box.lo[k] + it.box.hi[k]);
            if (std::isfinite(it.box.lo[k])) scale = std::max(scale, std::fabs(it.box.lo[k]));
            if (std::isfinite(it.box.hi[k])) scale = std::max(scale, std::fabs(it.box.hi[k]));
        }
        it.index = (uint32_t)i;
        it.cost = i < cost.size() ? cost[i] : 1.0f;
    }
    bld.pad = 1e-6 * std::max(scale, 1e-30);  // flat (axis-plane) primitives keep a volume
    bld.out.scale = scale;
    if (!bounds.empty()) bld.out.root = bld.build(0, bld.items.size(), 0);
    if (bld.out.depth > WBVH_STACK) throw std::runtime_error("world BVH deeper than the kernel's stack");
    if (bld.out.root >= 0) {
        Collapse c{bld.out.nodes, bld.out.nodes4};
        const char* ce = std::getenv("NRT_WBVH_COLLAPSE");
        if (ce && std::strtol(ce, nullptr, 10) == 1) {  // SAH collapse (A/B knob)
            std::vector<float> slot_cost(bld.out.order.size());
            for (size_t i = 0; i < slot_cost.size(); ++i) slot_cost[i] = bld.items.size() ? 1.0f : 1.0f;
            for (size_t i = 0; i < slot_cost.size(); ++i)
                slot_cost[i] = bld.out.order[i] < cost.size() ? cost[bld.out.order[i]] : 1.0f;
            c.prim_cost = &slot_cost;
            c.leaf_max = bld.leaf_max;
            if (const char* v = std::getenv("NRT_WBVH_VISIT")) c.visit = std::strtod(v, nullptr);
            c.inner.resize(bld.out.nodes.size());
            c.leaves.resize(bld.out.order.size());
            const DBvhNode& rb = bld.out.nodes[(size_t)bld.out.root];
            Collapse::Slot root{bld.out.root, {}, {}};
            for (int k = 0; k < 3; ++k) {
                root.lo[k] = std::min(rb.lo0[k], rb.lo1[k]);
                root.hi[k] = std::max(rb.hi0[k], rb.hi1[k]);
            }
            c.prepare(bld.out.root, root);
            if (std::getenv("NRT_DEBUG_WBVH")) {
                const Collapse::Info& ri = c.inner[(size_t)bld.out.root];
                const Collapse::Info &L = c.info(rb.c0), &R = c.info(rb.c1);
                std::fprintf(stderr, "nrt: SAH collapse objective %.3f (root split %d: %.3f + %.3f), root area %.4g\n",
                             (L.F[ri.root_split] + R.F[4 - ri.root_split]) / Collapse::area(root) + c.visit,
                             (int)ri.root_split, L.F[ri.root_split] / Collapse::area(root),
                             R.F[4 - ri.root_split] / Collapse::area(root), (double)Collapse::area(root));
            }
            bld.out.root4 = c.build_sah(bld.out.root);
        } else {
            bld.out.root4 = c.build(bld.out.root);
        }
        // nearest-first pushes all but one hit child: bound the stack along every path
        std::vector<uint32_t> need(bld.out.nodes4.size(), 0);
        for (size_t i = bld.out.nodes4.size(); i-- > 0;) {  // children have larger indices
            const DBvh4Node& nd = bld.out.nodes4[i];
            uint32_t kids = 0, deepest = 0;
            for (int k = 0; k < 4; ++k) {
                if (nd.child[k] == WBVH_DONE) continue;
                ++kids;
                if (nd.child[k] >= 0) deepest = std::max(deepest, need[nd.child[k]]);
            }
            need[i] = (kids ? kids - 1 : 0) + deepest;
        }
        bld.out.stack4 = need[bld.out.root4];
        if (std::getenv("NRT_DEBUG_WBVH")) {  // (diagnostics: the 4-wide tree's SAH cost, unit visit cost)
            auto dec = [](const DBvh4Node& nd, int k, int a, float* lo, float* hi) {
                const uint32_t ex = (nd.exps >> (10 * a)) & 1023u;
                const float step = std::ldexp(1.0f + 0.25f * (float)(ex & 3u), (int)(ex >> 2) - 127);
                *lo = nd.org[a] + (float)((nd.qlo[a] >> (8 * k)) & 255u) * step;
                *hi = nd.org[a] + (float)((nd.qhi[a] >> (8 * k)) & 255u) * step;
            };
            double visits = 0, tests = 0, root_area = 0;
            float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            size_t leaves = 0, leaf_prims = 0;
            std::vector<double> node_area(bld.out.nodes4.size(), 0.0);
            for (size_t i = 0; i < bld.out.nodes4.size(); ++i) {
                const DBvh4Node& nd = bld.out.nodes4[i];
                for (int k = 0; k < 4; ++k) {
                    if (nd.child[k] == WBVH_DONE) continue;
                    float lo[3], hi[3];
                    for (int a = 0; a < 3; ++a) dec(nd, k, a, &lo[a], &hi[a]);
                    const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2], ar = x * y + y * z + z * x;
                    if (i == (size_t)bld.out.root4)
                        for (int a = 0; a < 3; ++a) { rlo[a] = std::min(rlo[a], lo[a]); rhi[a] = std::max(rhi[a], hi[a]); }
                    if (nd.child[k] >= 0) {
                        node_area[(size_t)nd.child[k]] = ar;
                    } else {
                        const uint32_t v = ~(uint32_t)nd.child[k], cnt = (v & 7u) + 1u;
                        ++leaves;
                        leaf_prims += cnt;
                        tests += ar * cnt;
                    }
                }
            }
            {
                const double x = rhi[0] - rlo[0], y = rhi[1] - rlo[1], z = rhi[2] - rlo[2];
                root_area = x * y + y * z + z * x;
            }
            for (size_t i = 0; i < node_area.size(); ++i) visits += i == (size_t)bld.out.root4 ? root_area : node_area[i];
            std::fprintf(stderr, "nrt: world BVH %zu prims: %zu 4-nodes, %zu leaves (%zu prim slots), per ray ~%.2f visits "
                                 "+ %.2f prim tests (SAH, root area = 1), stack %u\n",
                         bld.out.order.size(), bld.out.nodes4.size(), leaves, leaf_prims, visits / root_area,
                         tests / root_area, bld.out.stack4);
        }
        if (need[bld.out.root4] > WBVH_STACK) {  // too deep for 4-wide traversal: binary only
            bld.out.nodes4.clear();
            bld.out.root4 = WBVH_DONE;
        }
        bld.out.nodes4c = compact_nodes(bld.out.nodes4, bld.out.order.size());
    } else {
        bld.out.root4 = bld.out.root;  // a single leaf (or empty)
    }
    for (int oct = 0; oct < 8; ++oct) thread_tree(bld.out.nodes, bld.out.root, oct, bld.out.threaded);
    bld.out.threaded_n = (uint32_t)(bld.out.threaded.size() / 8);
    return std::move(bld.out);
}

}  // namespace nrt
