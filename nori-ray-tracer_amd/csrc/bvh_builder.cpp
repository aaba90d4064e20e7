// bvh_builder.cpp -- host BVH construction for the device traversal kernels.
//
// Split selection restates BVH::build / BVHBuildTask (bvh.cpp:100-382):
// 16-bin SAH along the node's largest axis above 32 primitives, a full
// three-axis sweep below, T = I = 1 costs.  It runs serially and is
// deterministic (centroid ties broken by primitive id, order-preserving
// partition) -- the reference's TBB partition order is scheduling dependent.
// The finished tree is re-emitted in the device layout of host_scene.h:
// child boxes stored in the parent so one 64-byte fetch tests both children,
// leaves inlined into the child reference.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "host_scene.h"

namespace nori {
namespace {


struct Box {
    float mn[3], mx[3];
    Box() {
        for (int i = 0; i < 3; ++i) mn[i] = __builtin_inff(), mx[i] = -__builtin_inff();
    }
    void expand(const Box &b) {
        for (int i = 0; i < 3; ++i) {
            mn[i] = std::fmin(mn[i], b.mn[i]);
            mx[i] = std::fmax(mx[i], b.mx[i]);
        }
    }
    void expand(const float *p) {
        for (int i = 0; i < 3; ++i) {
            mn[i] = std::fmin(mn[i], p[i]);
            mx[i] = std::fmax(mx[i], p[i]);
        }
    }
    float area() const {  // bbox.h:87-100
        float d[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        float r = 0.0f;
        for (int i = 0; i < 3; ++i) {
            float t = 1.0f;
            for (int j = 0; j < 3; ++j)
                if (i != j) t *= d[j];
            r += t;
        }
        return 2.0f * r;
    }
    int largest_axis() const {  // bbox.h:308-317
        float e[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        if (e[0] >= e[1] && e[0] >= e[2]) return 0;
        if (e[1] >= e[0] && e[1] >= e[2]) return 1;
        return 2;
    }
};

struct RefNode {  // bvh.h:127-164 semantics
    bool leaf = false, used = false;
    uint32_t a = 0;  // leaf: size | inner: axis
    uint32_t b = 0;  // leaf: start | inner: right child
    Box box;
};

constexpr int kParDepth = 5;          // up to 2^5 concurrent subtree builds
constexpr uint32_t kParMin = 16384;   // smallest subtree given its own thread
constexpr uint32_t kPresortMin = 256; // serial sweeps at least this large keep presorted axis orders

struct Builder {
    std::vector<RefNode> nodes;
    std::vector<uint32_t> idx, temp;
    std::vector<uint8_t> side;  // per primitive: left/right of the split being partitioned
    std::vector<float> cent;  // 3 per prim
    std::vector<Box> pbox;

    void sort_axis(uint32_t *s, uint32_t n, int axis) {
        std::sort(s, s + n, [&](uint32_t a, uint32_t b) {
            float ca = cent[3 * a + axis], cb = cent[3 * b + axis];
            if (ca < cb) return true;
            if (cb < ca) return false;
            return a < b;
        });
    }
    // bvh.cpp:236-305: full-sweep SAH over the three axis orders of the node.
    // Small nodes re-sort their range per axis like the reference; large ones
    // (the reference falls back here when binning finds no split, e.g. a
    // 250k-triangle node next to the Cornell-box walls, and then peels a few
    // primitives off per level) keep all three orders sorted from the top and
    // stably partition them at each split: a stable partition of a sorted list
    // is the sorted list of the part, so the tree is identical without the
    // O(n log n) re-sort per level.
    void serial(uint32_t ni, uint32_t *start, uint32_t *end, uint32_t *tmp, int depth = 0) {
        const uint32_t size = (uint32_t)(end - start);
        if (size < kPresortMin) {
            serial_small(ni, start, end, tmp);
            return;
        }
        std::vector<uint32_t> ord(3 * (size_t)size), scratch(size);
        uint32_t *o[3] = {ord.data(), ord.data() + size, ord.data() + 2 * (size_t)size};
        for (int a = 0; a < 3; ++a) {
            std::memcpy(o[a], start, size * sizeof(uint32_t));
            sort_axis(o[a], size, a);
        }
        sweep(ni, start, o, size, scratch.data(), depth);
    }
    void serial_small(uint32_t ni, uint32_t *start, uint32_t *end, uint32_t *tmp) {
        RefNode &node = nodes[ni];
        node.used = true;
        uint32_t size = (uint32_t)(end - start);
        float best_cost = (float)1 * size;
        int64_t best_index = -1, best_axis = -1;
        float *left_areas = reinterpret_cast<float *>(tmp);
        for (int axis = 0; axis < 3; ++axis) {
            sort_axis(start, size, axis);
            Box bb;
            for (uint32_t i = 0; i < size; ++i) {
                bb.expand(pbox[start[i]]);
                left_areas[i] = bb.area();
            }
            if (axis == 0) node.box = bb;
            bb = Box();
            float tri_factor = 1 / node.box.area();
            for (uint32_t i = size - 1; i >= 1; --i) {
                bb.expand(pbox[start[i]]);
                float sah = 2.0f * 1 + tri_factor * ((float)i * left_areas[i - 1] + (float)(size - i) * bb.area());
                if (sah < best_cost) {
                    best_cost = sah;
                    best_index = i;
                    best_axis = axis;
                }
            }
        }
        if (best_index == -1) {
            node.leaf = true;
            node.a = size;
            node.b = (uint32_t)(start - idx.data());
            return;
        }
        sort_axis(start, size, (int)best_axis);
        uint32_t lc = (uint32_t)best_index, l = ni + 1, r = ni + 2 * lc;
        node.leaf = false;
        node.a = (uint32_t)best_axis;
        node.b = r;
        serial_small(l, start, start + lc, tmp);
        serial_small(r, start + lc, end, tmp + lc);
    }
    // o[a]: the node's primitives sorted along axis a (ties by id); out: the
    // node's range of the final index array; la: `size` words of scratch.
    void sweep(uint32_t ni, uint32_t *out, uint32_t *const o[3], uint32_t size, uint32_t *la, int depth) {
        if (size < kPresortMin) {  // small enough: back to the plain form on the z-sorted range
            std::memcpy(out, o[2], size * sizeof(uint32_t));
            serial_small(ni, out, out + size, la);
            return;
        }
        RefNode &node = nodes[ni];
        node.used = true;
        float best_cost = (float)1 * size;
        int64_t best_index = -1, best_axis = -1;
        float *left_areas = reinterpret_cast<float *>(la);
        for (int axis = 0; axis < 3; ++axis) {
            const uint32_t *s = o[axis];
            Box bb;
            for (uint32_t i = 0; i < size; ++i) {
                bb.expand(pbox[s[i]]);
                left_areas[i] = bb.area();
            }
            if (axis == 0) node.box = bb;
            bb = Box();
            float tri_factor = 1 / node.box.area();
            for (uint32_t i = size - 1; i >= 1; --i) {
                bb.expand(pbox[s[i]]);
                float sah = 2.0f * 1 + tri_factor * ((float)i * left_areas[i - 1] + (float)(size - i) * bb.area());
                if (sah < best_cost) {
                    best_cost = sah;
                    best_index = i;
                    best_axis = axis;
                }
            }
        }
        if (best_index == -1) {  // leaf: the reference leaves its range sorted along z
            std::memcpy(out, o[2], size * sizeof(uint32_t));
            node.leaf = true;
            node.a = size;
            node.b = (uint32_t)(out - idx.data());
            return;
        }
        const uint32_t lc = (uint32_t)best_index, l = ni + 1, r = ni + 2 * lc;
        node.leaf = false;
        node.a = (uint32_t)best_axis;
        node.b = r;
        const uint32_t *sb = o[best_axis];
        for (uint32_t i = 0; i < size; ++i) side[sb[i]] = i < lc ? 0 : 1;
        for (int a = 0; a < 3; ++a) {
            if (a == best_axis) continue;
            uint32_t il = 0, ir = lc;
            for (uint32_t i = 0; i < size; ++i) {
                const uint32_t f = o[a][i];
                if (side[f] == 0) la[il++] = f;
                else la[ir++] = f;
            }
            std::memcpy(o[a], la, size * sizeof(uint32_t));
        }
        uint32_t *ol[3] = {o[0], o[1], o[2]}, *orr[3] = {o[0] + lc, o[1] + lc, o[2] + lc};
        if (depth < kParDepth && size - lc >= kParMin && lc >= kParMin) {
            std::thread t([this, r, out, lc, orr, size, la, depth] { sweep(r, out + lc, orr, size - lc, la + lc, depth + 1); });
            sweep(l, out, ol, lc, la, depth + 1);
            t.join();
        } else {
            sweep(l, out, ol, lc, la, depth + 1);
            sweep(r, out + lc, orr, size - lc, la + lc, depth + 1);
        }
    }
    // bvh.cpp:100-233.  Subtrees own disjoint index, scratch and node ranges
    // (the left subtree of a node with lc primitives gets nodes ni+1 ..
    // ni+2lc-1), so large right subtrees are built on their own threads --
    // the reference's tbb::task tree -- with a result independent of scheduling.
    void task(uint32_t ni, uint32_t *start, uint32_t *end, uint32_t *tmp, int depth = 0) {
        std::vector<std::thread> kids;
        struct Join {
            std::vector<std::thread> &k;
            ~Join() {
                for (auto &t : k) t.join();
            }
        } join{kids};
        for (;;) {
            uint32_t size = (uint32_t)(end - start);
            RefNode &node = nodes[ni];
            node.used = true;
            if (size < 32) {
                serial(ni, start, end, tmp, depth);
                return;
            }
            int axis = node.box.largest_axis();
            float mn = node.box.mn[axis], mx = node.box.mx[axis], inv_bin = 16 / (mx - mn);
            uint32_t counts[16] = {0};
            Box bins[16];
            for (uint32_t i = 0; i < size; ++i) {
                uint32_t f = start[i];
                int index = (int)((cent[3 * f + axis] - mn) * inv_bin);
                index = std::min(std::max(index, 0), 15);
                counts[index]++;
                bins[index].expand(pbox[f]);
            }
            Box left[16];
            left[0] = bins[0];
            for (int i = 1; i < 16; ++i) {
                counts[i] += counts[i - 1];
                left[i] = left[i - 1];
                left[i].expand(bins[i]);
            }
            Box right = bins[15], best_right;
            int64_t best_index = -1;
            float best_cost = (float)1 * size, tri_factor = (float)1 / node.box.area();
            for (int i = 14; i >= 0; --i) {
                uint32_t pl = counts[i], pr = size - counts[i];
                float sah = 2.0f * 1 + tri_factor * ((float)pl * left[i].area() + (float)pr * right.area());
                if (sah < best_cost) {
                    best_cost = sah;
                    best_index = i;
                    best_right = right;
                }
                right.expand(bins[i]);
            }
            if (best_index == -1) {
                serial(ni, start, end, tmp, depth);
                return;
            }
            uint32_t lc = counts[best_index], l = ni + 1, r = ni + 2 * lc;
            nodes[l].box = left[best_index];
            nodes[r].box = best_right;
            node.leaf = false;
            node.a = (uint32_t)axis;
            node.b = r;
            uint32_t il = 0, ir = lc;
            for (uint32_t i = 0; i < size; ++i) {
                uint32_t f = start[i];
                int index = (int)((cent[3 * f + axis] - mn) * inv_bin);
                if (index <= best_index) tmp[il++] = f;
                else tmp[ir++] = f;
            }
            std::memcpy(start, tmp, size * sizeof(uint32_t));
            if (depth < kParDepth && size - lc >= kParMin) {
                uint32_t *s2 = start + lc, *e2 = end, *t2 = tmp + lc;
                const int d2 = depth + 1;
                kids.emplace_back([this, r, s2, e2, t2, d2] { task(r, s2, e2, t2, d2); });
            } else {
                task(r, start + lc, end, tmp + lc, depth + 1);
            }
            ni = l;
            end = start + lc;
            ++depth;
        }
    }
    float statistics(uint32_t ni, uint32_t &count) const {  // bvh.cpp:384-402
        const RefNode &n = nodes[ni];
        if (n.leaf) {
            count = 1;
            return (float)n.a;
        }
        uint32_t cl, cr;
        float sl = statistics(ni + 1, cl), sr = statistics(n.b, cr);
        count = cl + cr + 1;
        return 2 + (nodes[ni + 1].box.area() * sl + nodes[n.b].box.area() * sr) / n.box.area();
    }
};

}  // namespace

void build_device_bvh(const nori_scene_desc &d, const float root_min[3], const float root_max[3], DeviceBvh &out) {
    // primitive table in shape order (BVH::addShape, bvh.cpp:307-311)
    std::vector<uint32_t> prim_shape;
    std::vector<uint32_t> prim_local;
    for (uint32_t s = 0; s < d.num_shapes; ++s) {
        uint32_t n = d.shapes[s].type == NORI_SHAPE_SPHERE ? 1 : d.shapes[s].tri_count;
        for (uint32_t i = 0; i < n; ++i) {
            prim_shape.push_back(s);
            prim_local.push_back(i);
        }
    }
    uint32_t n = (uint32_t)prim_shape.size();
    out = DeviceBvh();
    if (n == 0) throw NoriException(NORI_ERR_INVALID, "scene has no primitives");
    if (n >= (1u << 25)) throw NoriException(NORI_ERR_UNSUPPORTED, "more than 2^25 primitives");
    auto T0 = std::chrono::steady_clock::now();
    auto lap = [&](const char *what) {
        if (!std::getenv("NORI_DEBUG")) return;
        auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[nori] bvh %s %.1f ms\n", what, std::chrono::duration<double, std::milli>(t - T0).count());
        T0 = t;
    };
    Builder b;
    b.cent.resize(3 * (size_t)n);
    b.pbox.resize(n);
    auto vtx = [&](uint32_t i) { return d.positions + 3 * (size_t)i; };
    for (uint32_t p = 0; p < n; ++p) {
        const nori_shape_desc &sh = d.shapes[prim_shape[p]];
        if (sh.type == NORI_SHAPE_SPHERE) {  // sphere.cpp:32-41
            float lo[3], hi[3];
            for (int k = 0; k < 3; ++k) lo[k] = sh.center[k] - sh.radius, hi[k] = sh.center[k] + sh.radius;
            b.pbox[p].expand(lo);
            b.pbox[p].expand(hi);
            for (int k = 0; k < 3; ++k) b.cent[3 * p + k] = sh.center[k];
        } else {  // mesh.cpp:172-184
            const uint32_t *f = d.indices + 3 * (size_t)(sh.tri_offset + prim_local[p]);
            const float *p0 = vtx(f[0]), *p1 = vtx(f[1]), *p2 = vtx(f[2]);
            b.pbox[p].expand(p0);
            b.pbox[p].expand(p1);
            b.pbox[p].expand(p2);
            for (int k = 0; k < 3; ++k) b.cent[3 * p + k] = (1.0f / 3.0f) * ((p0[k] + p1[k]) + p2[k]);
        }
    }
    b.nodes.assign(2 * (size_t)n, RefNode());
    b.idx.resize(n);
    b.temp.resize(n);
    b.side.assign(n, 0);
    for (uint32_t i = 0; i < n; ++i) b.idx[i] = i;
    for (int k = 0; k < 3; ++k) b.nodes[0].box.mn[k] = root_min[k], b.nodes[0].box.mx[k] = root_max[k];
    lap("setup");
    b.task(0, b.idx.data(), b.idx.data() + n, b.temp.data());
    lap("build");
    uint32_t cnt = 0;
    out.sah_cost = b.statistics(0, cnt);
    out.ref_nodes = cnt;
    lap("statistics");

    // ---- primitive records in leaf order
    out.prims.assign(12 * (size_t)n, 0.0f);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t p = b.idx[i];
        float *r = &out.prims[12 * (size_t)i];
        const nori_shape_desc &sh = d.shapes[prim_shape[p]];
        uint32_t pid = p;
        if (sh.type == NORI_SHAPE_SPHERE) {
            r[0] = sh.center[0]; r[1] = sh.center[1]; r[2] = sh.center[2];
            r[4] = sh.radius;
            uint32_t one = 1;
            std::memcpy(&r[7], &one, 4);
        } else {
            const uint32_t *f = d.indices + 3 * (size_t)(sh.tri_offset + prim_local[p]);
            const float *p0 = vtx(f[0]), *p1 = vtx(f[1]), *p2 = vtx(f[2]);
            for (int k = 0; k < 3; ++k) {
                r[k] = p0[k];
                r[4 + k] = p1[k] - p0[k];  // edge1 (mesh.cpp:88)
                r[8 + k] = p2[k] - p0[k];  // edge2
            }
        }
        std::memcpy(&r[3], &pid, 4);
    }

    // ---- device nodes: DFS over the reference tree
    struct Child {
        uint32_t ref;
        Box box;
    };
    std::vector<float> &nodes = out.nodes;
    uint32_t max_depth = 0;
    // returns the child ref for reference node `ri`; leaves larger than
    // kLeafMaxPrims are split into a chain of inner nodes (same primitive set).
    std::function<Child(uint32_t, uint32_t, uint32_t, uint32_t)> leaf_ref = [&](uint32_t start, uint32_t count,
                                                                              uint32_t depth, uint32_t) -> Child {
        Child c;
        for (uint32_t i = start; i < start + count; ++i) c.box.expand(b.pbox[b.idx[i]]);
        if (count <= kLeafMaxPrims) {
            c.ref = kLeafBit | ((count - 1) << 25) | start;
            return c;
        }
        uint32_t me = (uint32_t)(nodes.size() / 16);
        nodes.resize(nodes.size() + 16, 0.0f);
        max_depth = std::max(max_depth, depth + 1);
        uint32_t half = count / 2;
        Child l = leaf_ref(start, half, depth + 1, 0), r = leaf_ref(start + half, count - half, depth + 1, 0);
        float *nd = &nodes[16 * (size_t)me];
        for (int k = 0; k < 3; ++k) {
            nd[k] = l.box.mn[k]; nd[4 + k] = l.box.mx[k];
            nd[8 + k] = r.box.mn[k]; nd[12 + k] = r.box.mx[k];
        }
        std::memcpy(&nd[3], &l.ref, 4);
        std::memcpy(&nd[7], &r.ref, 4);
        c.ref = me;
        return c;
    };
    std::function<Child(uint32_t, uint32_t)> emit = [&](uint32_t ri, uint32_t depth) -> Child {
        const RefNode &rn = b.nodes[ri];
        if (rn.leaf) {
            Child c = leaf_ref(rn.b, rn.a, depth, 0);
            c.box = rn.box;
            return c;
        }
        uint32_t me = (uint32_t)(nodes.size() / 16);
        nodes.resize(nodes.size() + 16, 0.0f);
        max_depth = std::max(max_depth, depth + 1);
        Child l = emit(ri + 1, depth + 1), r = emit(rn.b, depth + 1);
        float *nd = &nodes[16 * (size_t)me];
        for (int k = 0; k < 3; ++k) {
            nd[k] = b.nodes[ri + 1].box.mn[k]; nd[4 + k] = b.nodes[ri + 1].box.mx[k];
            nd[8 + k] = b.nodes[rn.b].box.mn[k]; nd[12 + k] = b.nodes[rn.b].box.mx[k];
        }
        std::memcpy(&nd[3], &l.ref, 4);
        std::memcpy(&nd[7], &r.ref, 4);
        Child c;
        c.ref = me;
        c.box = rn.box;
        return c;
    };
    if (b.nodes[0].leaf) {
        // root leaf: one inner node whose right child box is empty
        nodes.resize(16, 0.0f);
        Child l = leaf_ref(b.nodes[0].b, b.nodes[0].a, 1, 0);
        float *nd = &nodes[0];
        for (int k = 0; k < 3; ++k) {
            nd[k] = b.nodes[0].box.mn[k]; nd[4 + k] = b.nodes[0].box.mx[k];
            nd[8 + k] = __builtin_inff(); nd[12 + k] = -__builtin_inff();
        }
        std::memcpy(&nd[3], &l.ref, 4);
        uint32_t empty = kLeafBit;  // never visited: its box is empty
        std::memcpy(&nd[7], &empty, 4);
        max_depth = std::max<uint32_t>(max_depth, 1);
    } else {
        emit(0, 0);
    }
    // ---- collapse the binary device tree into the 4-wide layout
    std::vector<float> bin;
    bin.swap(nodes);
    struct C4 {
        uint32_t ref;
        float mn[3], mx[3];
    };
    auto kids = [&](uint32_t n, C4 c[2]) {
        const float *nd = &bin[16 * (size_t)n];
        for (int k = 0; k < 3; ++k) {
            c[0].mn[k] = nd[k];
            c[0].mx[k] = nd[4 + k];
            c[1].mn[k] = nd[8 + k];
            c[1].mx[k] = nd[12 + k];
        }
        std::memcpy(&c[0].ref, &nd[3], 4);
        std::memcpy(&c[1].ref, &nd[7], 4);
    };
    auto area = [](const C4 &c) {
        float d[3] = {c.mx[0] - c.mn[0], c.mx[1] - c.mn[1], c.mx[2] - c.mn[2]};
        return 2.0f * ((d[0] * d[1] + d[1] * d[2]) + d[2] * d[0]);
    };
    auto empty = [](const C4 &c) { return c.mn[0] > c.mx[0] || c.mn[1] > c.mx[1] || c.mn[2] > c.mx[2]; };
    uint32_t depth4 = 0;
    std::function<uint32_t(uint32_t, uint32_t)> collapse = [&](uint32_t n, uint32_t depth) -> uint32_t {
        C4 two[2];
        kids(n, two);
        std::vector<C4> ch(two, two + 2);
        while (ch.size() < 4) {  // open the inner child of largest area (DFS order kept)
            int best = -1;
            float ba = -1.0f;
            for (size_t i = 0; i < ch.size(); ++i)
                if (!(ch[i].ref & kLeafBit) && !empty(ch[i]) && area(ch[i]) > ba) {
                    ba = area(ch[i]);
                    best = (int)i;
                }
            if (best < 0) break;
            kids(ch[(size_t)best].ref, two);
            ch[(size_t)best] = two[0];
            ch.insert(ch.begin() + best + 1, two[1]);
        }
        const uint32_t me = (uint32_t)(nodes.size() / 32);
        nodes.resize(nodes.size() + 32, 0.0f);
        depth4 = std::max(depth4, depth + 1);
        uint32_t refs[4];
        for (int i = 0; i < 4; ++i) {
            const bool use = (size_t)i < ch.size() && !empty(ch[(size_t)i]);
            refs[i] = use ? ch[(size_t)i].ref : kLeafBit;  // unused: NaN box, never entered
            if (use && !(refs[i] & kLeafBit)) refs[i] = collapse(refs[i], depth + 1);
            float *nd = &nodes[32 * (size_t)me];
            for (int k = 0; k < 3; ++k) {
                nd[4 * k + i] = use ? ch[(size_t)i].mn[k] : __builtin_nanf("");
                nd[4 * (3 + k) + i] = use ? ch[(size_t)i].mx[k] : __builtin_nanf("");
            }
        }
        std::memcpy(&nodes[32 * (size_t)me + 24], refs, 16);
        return me;
    };
    collapse(0, 0);
    out.num_nodes = (uint32_t)(nodes.size() / 32);
    out.depth = depth4;
    (void)max_depth;
    lap("device layout");
}

}  // namespace nori
