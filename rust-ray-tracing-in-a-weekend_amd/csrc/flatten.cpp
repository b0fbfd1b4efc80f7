// flatten.cpp — lowers the World's Hittable tree into the SoA tables of
// rt_scene.h and builds the SAH BVHs the megakernel traverses.
//
// Lowering rules (hittable.rs:30-41):
//   Sphere / MovingSphere / XY,XZ,YZ rects / Box   -> one rt_prim each
//   BvhNode (reference median BVH, :77-130)        -> dissolved; its leaves join the
//                                                     enclosing SAH BVH (closest-hit is
//                                                     independent of the hierarchy)
//   Translate / RotateY chains (:232-244, :386-415) -> rt_instance (<= 4 ops) whose child
//                                                     is a single prim or its own BLAS
//   ConstantMedium (:417-473)                       -> RT_PRIM_MEDIUM whose boundary is a
//                                                     hidden prim (sphere / box / instance)
// The top-level list becomes the TLAS. Nested instances, BVHs and media are lowered by
// pushing Translate/RotateY chains down (lower_instance); a medium boundary that holds
// instances or media, and chains longer than 4 ops, are not (RT_ERR_UNSUPPORTED).
//
// accel (rt_scene.h) picks the hierarchy: SAH (above), LINEAR (every list a chain of
// unbounded nodes over <=31-prim leaves, in list order: hit_hittables' linear scan), or
// MEDIAN (the reference's BvhNodes kept node for node, the top-level list a chain).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>

#include "rt/rt_abi.h"
#include "scene_model.hpp"

namespace rtw {

namespace {

struct Item {
    int prim;   // >= 0: a primitive; -1: a prebuilt subtree (MEDIAN mode), see ref
    int ref;
    double lo[3], hi[3];
    double c[3];
};

struct Builder {
    World& w;
    FlatScene& f;
    std::string& err;
    int accel = RT_ACCEL_SAH;

    int add_prim(const rt_prim& p)
    {
        f.prims.push_back(p);
        return (int)f.prims.size() - 1;
    }

    static rt_prim blank(int kind, int mat)
    {
        rt_prim p;
        std::memset(&p, 0, sizeof p);
        p.kind = kind;
        p.mat = mat;
        return p;
    }

    bool is_simple(HKind k) const
    {
        return k == HKind::Sphere || k == HKind::MovingSphere || k == HKind::XYRect || k == HKind::XZRect ||
               k == HKind::YZRect || k == HKind::Box;
    }

    int lower_simple(int id)
    {
        const HNode& h = w.nodes[id];
        rt_prim p = blank(0, h.mat - 1);
        switch (h.kind) {
        case HKind::Sphere:
            p.kind = RT_PRIM_SPHERE;
            p.p[0] = h.c0.x; p.p[1] = h.c0.y; p.p[2] = h.c0.z;
            p.p[3] = h.radius;
            p.p[4] = 1.0 / h.radius;  // the reference's Div: (1/r) * v (math.rs:260-266)
            break;
        case HKind::MovingSphere:
            p.kind = RT_PRIM_MOVING_SPHERE;
            p.p[0] = h.c0.x; p.p[1] = h.c0.y; p.p[2] = h.c0.z;
            p.p[3] = h.radius;
            p.p[4] = 1.0 / h.radius;
            p.p[5] = h.c1.x - h.c0.x; p.p[6] = h.c1.y - h.c0.y; p.p[7] = h.c1.z - h.c0.z;  // hittable.rs:557
            p.p[8] = h.t0; p.p[9] = h.t1;
            p.a = (h.t0 == 0.0 && h.t1 == 1.0) ? 1 : 0;  // (time - 0) / (1 - 0) == time exactly
            break;
        case HKind::XYRect: case HKind::XZRect: case HKind::YZRect:
            p.kind = h.kind == HKind::XYRect ? RT_PRIM_XY_RECT : h.kind == HKind::XZRect ? RT_PRIM_XZ_RECT
                                                                                         : RT_PRIM_YZ_RECT;
            p.p[0] = h.a0; p.p[1] = h.a1; p.p[2] = h.b0; p.p[3] = h.b1; p.p[4] = h.k;
            break;
        case HKind::Box: {
            p.kind = RT_PRIM_BOX;
            p.p[0] = h.bmin.x; p.p[1] = h.bmin.y; p.p[2] = h.bmin.z;
            p.p[3] = h.bmax.x; p.p[4] = h.bmax.y; p.p[5] = h.bmax.z;
            // the box's own bounds in f32, padded and rounded outward like a BVH node's
            // (rt_scene.h; the kernel's per-box pre-test measured slower and is not built)
            const double lo[3] = {h.bmin.x, h.bmin.y, h.bmin.z}, hi[3] = {h.bmax.x, h.bmax.y, h.bmax.z};
            float fb[6];
            to_f32_box(lo, hi, fb, fb + 3);
            std::memcpy(&p.p[6], fb, sizeof fb);
            p.b = 1;
            break;
        }
        default: break;
        }
        return add_prim(p);
    }

    Item item_of(int prim, int hid)
    {
        Item it;
        it.prim = prim;
        it.ref = 0;
        AABB b;
        w.bounding_box(hid, 0.0, 1.0, b);
        it.lo[0] = b.minimum.x; it.lo[1] = b.minimum.y; it.lo[2] = b.minimum.z;
        it.hi[0] = b.maximum.x; it.hi[1] = b.maximum.y; it.hi[2] = b.maximum.z;
        for (int a = 0; a < 3; ++a) it.c[a] = 0.5 * (it.lo[a] + it.hi[a]);
        return it;
    }

    // ---- Translate / RotateY (hittable.rs:232-244, 386-415) and general nesting --------
    // A chain of ops (outermost first) is pushed down through everything under it: for the
    // closest hit, Outer(BVH[a, b]) = BVH[Outer(a), Outer(b)] (the ray is transformed the
    // same way for each child, the hit parameter t is the ray's, and the record is mapped
    // back op by op — with each op's set_face_normal quirk — for the winning child only),
    // and Outer(Inner(x)) is one chain of Outer's ops followed by Inner's. So any nesting of
    // instances, BVHs and media lowers to instances whose child is one primitive, one medium
    // or a BLAS of primitives, each with a chain of <= 4 ops.
    struct Ops {
        int n = 0;
        int32_t kind[4] = {0, 0, 0, 0};
        double op[4][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    };

    // Appends the Translate / RotateY chain starting at id to ops; returns the node it ends on.
    int chain(int id, Ops& ops, int& rc)
    {
        int cur = id;
        while (w.nodes[cur].kind == HKind::Translate || w.nodes[cur].kind == HKind::RotateY) {
            if (ops.n == 4) {
                err = "instance chain longer than 4 Translate/RotateY ops";
                rc = RT_ERR_UNSUPPORTED;
                return -1;
            }
            const HNode& h = w.nodes[cur];
            if (h.kind == HKind::Translate) {
                ops.kind[ops.n] = RT_OP_TRANSLATE;
                ops.op[ops.n][0] = h.offset.x; ops.op[ops.n][1] = h.offset.y; ops.op[ops.n][2] = h.offset.z;
            } else {
                ops.kind[ops.n] = RT_OP_ROTATE_Y;
                ops.op[ops.n][0] = h.sin_theta; ops.op[ops.n][1] = h.cos_theta; ops.op[ops.n][2] = 0.0;
            }
            ops.n++;
            cur = h.ptr;
        }
        return cur;
    }

    // The world box of an object-space box seen through ops (corners mapped back op by op,
    // innermost first: rotate back x' = c x + s z, z' = -s x + c z; translate back + offset).
    static AABB box_through(const Ops& ops, AABB b)
    {
        for (int i = ops.n - 1; i >= 0; --i) {
            if (ops.kind[i] == RT_OP_TRANSLATE) {
                const V3 off = v3(ops.op[i][0], ops.op[i][1], ops.op[i][2]);
                b.minimum = b.minimum + off;
                b.maximum = b.maximum + off;
                continue;
            }
            const double sn = ops.op[i][0], cs = ops.op[i][1];
            AABB r{v3(INFINITY, b.minimum.y, INFINITY), v3(-INFINITY, b.maximum.y, -INFINITY)};
            for (int k = 0; k < 4; ++k) {
                const double x = (k & 1) ? b.maximum.x : b.minimum.x, z = (k & 2) ? b.maximum.z : b.minimum.z;
                const double nx = cs * x + sn * z, nz = -sn * x + cs * z;
                r.minimum.x = std::min(r.minimum.x, nx); r.maximum.x = std::max(r.maximum.x, nx);
                r.minimum.z = std::min(r.minimum.z, nz); r.maximum.z = std::max(r.maximum.z, nz);
            }
            b = r;
        }
        return b;
    }

    Item item_box(int prim, const AABB& b)
    {
        Item it;
        it.prim = prim;
        it.ref = 0;
        it.lo[0] = b.minimum.x; it.lo[1] = b.minimum.y; it.lo[2] = b.minimum.z;
        it.hi[0] = b.maximum.x; it.hi[1] = b.maximum.y; it.hi[2] = b.maximum.z;
        for (int a = 0; a < 3; ++a) it.c[a] = 0.5 * (it.lo[a] + it.hi[a]);
        return it;
    }

    AABB box_of(int hid) const
    {
        AABB b;
        w.bounding_box(hid, 0.0, 1.0, b);
        return b;
    }

    int make_instance(const Ops& ops, int child_kind, int child)
    {
        rt_instance in;
        std::memset(&in, 0, sizeof in);
        in.n_ops = ops.n;
        in.child_kind = child_kind;
        in.child = child;
        for (int i = 0; i < ops.n; ++i) {
            in.op_kind[i] = ops.kind[i];
            for (int a = 0; a < 3; ++a) in.op[i][a] = ops.op[i][a];
        }
        f.instances.push_back(in);
        rt_prim p = blank(RT_PRIM_INSTANCE, -1);
        p.a = (int)f.instances.size() - 1;
        return add_prim(p);
    }

    // Box padding for object space seen through ops: object-space origins have |o_obj| <=
    // |o_world| + sum |offsets|, which the padding must cover.
    double pad_through(const Ops& ops) const
    {
        double off = 0.0;
        for (int i = 0; i < ops.n; ++i)
            if (ops.kind[i] == RT_OP_TRANSLATE)
                off += std::sqrt(ops.op[i][0] * ops.op[i][0] + ops.op[i][1] * ops.op[i][1] + ops.op[i][2] * ops.op[i][2]);
        return 0x1.0p-18 * (world_extent + off);
    }

    int lower_simple_in(const Ops& ops, int hid)
    {
        const double saved = pad_abs;
        pad_abs = pad_through(ops);
        const int prim = lower_simple(hid);
        pad_abs = saved;
        return prim;
    }

    // A BLAS over simple leaves seen through ops.
    int make_blas(const Ops& ops, const std::vector<int>& leaves, int bvh_node, int& rc)
    {
        const double saved = pad_abs;
        pad_abs = pad_through(ops);
        int root;
        if (accel == RT_ACCEL_MEDIAN && bvh_node >= 0) {
            root = lower_ref_bvh(bvh_node, /*in_instance=*/true, rc);
        } else {
            std::vector<Item> items;
            for (int hid : leaves) items.push_back(item_of(lower_simple(hid), hid));
            in_blas = true;
            root = build_bvh(items);
            in_blas = false;
        }
        pad_abs = saved;
        if (rc) return 0;
        blas_depth = std::max(blas_depth, stack_need(root) + 1);
        return root;
    }

    // The leaves under a BVH node (through nested BvhNodes): simple ones and the rest.
    void collect_split(int id, std::vector<int>& simple, std::vector<int>& complex)
    {
        const HNode& h = w.nodes[id];
        if (h.kind == HKind::BvhNode) {
            collect_split(h.left, simple, complex);
            if (h.right != h.left) collect_split(h.right, simple, complex);  // span-1 duplicate
            return;
        }
        (is_simple(h.kind) ? simple : complex).push_back(id);
    }

    // Lowers the object `id` seen through the ops `prefix` into instance items.
    int lower_instance(int id, const Ops& prefix, std::vector<Item>& items)
    {
        Ops ops = prefix;
        int rc = RT_OK;
        const int child = chain(id, ops, rc);
        if (rc) return rc;
        const HNode& c = w.nodes[child];
        if (is_simple(c.kind)) {
            items.push_back(item_box(make_instance(ops, RT_CHILD_PRIM, lower_simple_in(ops, child)),
                                     box_through(ops, box_of(child))));
            return RT_OK;
        }
        if (c.kind == HKind::ConstantMedium) return lower_medium(child, ops, items);
        if (c.kind != HKind::BvhNode) {
            err = "unsupported hittable under an instance";
            return RT_ERR_UNSUPPORTED;
        }
        std::vector<int> simple, complex;
        collect_split(child, simple, complex);
        if (!simple.empty()) {
            AABB b = box_of(simple[0]);
            for (int hid : simple) {
                const AABB bi = box_of(hid);
                b.minimum = v3(std::min(b.minimum.x, bi.minimum.x), std::min(b.minimum.y, bi.minimum.y),
                               std::min(b.minimum.z, bi.minimum.z));
                b.maximum = v3(std::max(b.maximum.x, bi.maximum.x), std::max(b.maximum.y, bi.maximum.y),
                               std::max(b.maximum.z, bi.maximum.z));
            }
            const int root = make_blas(ops, simple, complex.empty() ? child : -1, rc);
            if (rc) return rc;
            items.push_back(item_box(make_instance(ops, RT_CHILD_BVH, root), box_through(ops, b)));
        }
        for (int k : complex) {
            const HKind kk = w.nodes[k].kind;
            if (kk == HKind::Translate || kk == HKind::RotateY) rc = lower_instance(k, ops, items);
            else if (kk == HKind::ConstantMedium) rc = lower_medium(k, ops, items);
            else { err = "unsupported hittable under an instance"; rc = RT_ERR_UNSUPPORTED; }
            if (rc) return rc;
        }
        return RT_OK;
    }

    // ConstantMedium (hittable.rs:417-473) seen through ops: a medium primitive (boundary: a
    // primitive, or an instance over a primitive or a BLAS), itself the child of an instance
    // when ops is not empty.
    int lower_medium(int id, const Ops& ops, std::vector<Item>& items)
    {
        const HNode& h = w.nodes[id];
        int bprim;
        int rc = lower_boundary(h.ptr, bprim);
        if (rc) return rc;
        rt_prim p = blank(RT_PRIM_MEDIUM, h.mat - 1);
        p.a = bprim;
        p.b = h.medium_id;
        p.p[0] = h.neg_inv_density;
        const int mprim = add_prim(p);
        if (ops.n == 0) items.push_back(item_of(mprim, id));
        else items.push_back(item_box(make_instance(ops, RT_CHILD_PRIM, mprim), box_through(ops, box_of(id))));
        return RT_OK;
    }

    // One primitive standing for a medium's boundary: a simple primitive, or an instance (a
    // Translate/RotateY chain, or none for a bare BvhNode) over a primitive or a BLAS. A
    // boundary holding instances or media below its chain is not lowered.
    int lower_boundary(int id, int& prim_out)
    {
        if (is_simple(w.nodes[id].kind)) {
            prim_out = lower_simple(id);
            return RT_OK;
        }
        Ops ops;
        int rc = RT_OK;
        const int child = chain(id, ops, rc);
        if (rc) return rc;
        if (is_simple(w.nodes[child].kind)) {
            prim_out = make_instance(ops, RT_CHILD_PRIM, lower_simple_in(ops, child));
            return RT_OK;
        }
        if (w.nodes[child].kind == HKind::BvhNode) {
            std::vector<int> simple, complex;
            collect_split(child, simple, complex);
            if (complex.empty() && !simple.empty()) {
                const int root = make_blas(ops, simple, child, rc);
                if (rc) return rc;
                prim_out = make_instance(ops, RT_CHILD_BVH, root);
                return RT_OK;
            }
        }
        err = "a medium boundary holding instances or media is not lowered";
        return RT_ERR_UNSUPPORTED;
    }

    // MEDIAN mode: a reference BvhNode subtree lowered node for node (both child boxes from
    // bounding_box, hittable.rs:118-130); a non-BVH child becomes a one-primitive leaf.
    // A span-1 node (left == right, :100-102) tests the same leaf twice, as the reference does.
    int lower_ref_bvh(int id, bool in_instance, int& rc)
    {
        const HNode& h = w.nodes[id];
        if (h.kind != HKind::BvhNode) {
            int prim = -1;
            if (is_simple(h.kind)) {
                prim = lower_simple(id);
            } else if (in_instance) {
                err = "instance over a BVH that contains an instance or a medium";
                rc = RT_ERR_UNSUPPORTED;
                return 0;
            } else {
                std::vector<Item> one;
                rc = lower_top(id, one);
                if (rc) return 0;
                prim = one[0].prim;
            }
            const int first = (int)f.prim_refs.size();
            f.prim_refs.push_back(prim);
            return RT_LEAF_CODE(first, 1);
        }
        const int node = (int)f.nodes.size();
        f.nodes.emplace_back();
        const int lc = lower_ref_bvh(h.left, in_instance, rc);
        if (rc) return 0;
        const int rc_ref = h.right == h.left ? lc : lower_ref_bvh(h.right, in_instance, rc);
        if (rc) return 0;
        const Item li = item_of(-1, h.left), ri = item_of(-1, h.right);
        rt_bvh_node& nd = f.nodes[node];
        std::memset(&nd, 0, sizeof nd);
        to_f32_box(li.lo, li.hi, nd.lo0, nd.hi0);
        to_f32_box(ri.lo, ri.hi, nd.lo1, nd.hi1);
        nd.child[0] = lc;
        nd.child[1] = rc_ref;
        return node;
    }

    int lower_top(int id, std::vector<Item>& items)
    {
        const HNode& h = w.nodes[id];
        switch (h.kind) {
        case HKind::BvhNode: {
            if (accel == RT_ACCEL_MEDIAN) {
                int rc = RT_OK;
                Item it = item_of(-1, id);
                it.ref = lower_ref_bvh(id, false, rc);
                if (rc) return rc;
                items.push_back(it);
                return RT_OK;
            }
            int rc = lower_top(h.left, items);
            if (rc) return rc;
            if (h.right != h.left) return lower_top(h.right, items);
            return RT_OK;
        }
        case HKind::Translate: case HKind::RotateY: return lower_instance(id, Ops(), items);
        case HKind::ConstantMedium: return lower_medium(id, Ops(), items);
        default:
            items.push_back(item_of(lower_simple(id), id));
            return RT_OK;
        }
    }

    // ---- SAH BVH ---------------------------------------------------------------
    static double area(const double lo[3], const double hi[3])
    {
        double dx = std::max(0.0, hi[0] - lo[0]), dy = std::max(0.0, hi[1] - lo[1]), dz = std::max(0.0, hi[2] - lo[2]);
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }

    static void bounds(const std::vector<Item>& items, int b, int e, double lo[3], double hi[3])
    {
        for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
        for (int i = b; i < e; ++i)
            for (int a = 0; a < 3; ++a) {
                lo[a] = std::min(lo[a], items[i].lo[a]);
                hi[a] = std::max(hi[a], items[i].hi[a]);
            }
    }

    // Pads and rounds a box outward to f32 so that neither the f64 slab test nor the
    // conservative f32 one ever culls a primitive the exact test would hit (the box only
    // gates traversal). pad_abs = 2^-18 * M covers the f32 rounding of ray origins with
    // |o| <= 2M and of the slab products (DESIGN.md §Traversal precision).
    double pad_abs = 0.0;

    void to_f32_box(const double lo[3], const double hi[3], float flo[3], float fhi[3]) const
    {
        for (int a = 0; a < 3; ++a) {
            double mag = std::max(std::fabs(lo[a]), std::fabs(hi[a]));
            double pad = 1e-6 * (1.0 + mag) + pad_abs;
            double l = lo[a] - pad, h = hi[a] + pad;
            float fl = (float)l, fh = (float)h;
            if ((double)fl > l) fl = std::nextafter(fl, -INFINITY);
            if ((double)fh < h) fh = std::nextafter(fh, INFINITY);
            flo[a] = fl;
            fhi[a] = fh;
        }
    }

    int make_leaf(std::vector<Item>& items, int b, int e)
    {
        int first = (int)f.prim_refs.size();
        for (int i = b; i < e; ++i) f.prim_refs.push_back(items[i].prim);
        return RT_LEAF_CODE(first, e - b);
    }

    double world_extent = 0.0;  // M: max |coordinate| over the top-level items' boxes

    // SAH costs (traversal step vs primitive test) and the largest leaf; RT_BVH_CI /
    // RT_BVH_MAXLEAF override them for tuning experiments (the image does not change).
    // Measured on MI355X (DESIGN.md §BVH build): c_isect 1.0 / max_leaf 8 keeps the sphere
    // scenes' trees and lets a Cornell box's top level (8 wall / box items that every bounce
    // from inside hits anyway) collapse: 177 -> 118 ms on C3's geometry.
    double c_isect = 1.0;
    int max_leaf = 8;
    int force_leaf = 2;   // RT_BVH_LEAFN: a set this small is always one leaf
    // ... unless it holds a Box (RT_BVH_BOXPAIRS=0: no exception): two Boxes' twelve rect tests in
    // one leaf cost more than a node visit that separates them (C4 1920x1080x100: 108.51 -> 103.52
    // ms with sets of two split by the SAH, profiles/r04v_ab_c4.log; the random scene's sphere
    // pairs stay leaves, whose split would push its TLAS past the LDS node budget)
    bool split_box_pairs = true;
    // ... and inside an instance's BLAS any set of two (RT_BVH_BLASPAIRS=0: no): the final scene's
    // 1000-sphere cluster, walked by the lanes that reach it together after the top-level walk
    // (C4 1920x1080x100 with every pair split, the top level's too: 105.84 -> 103.40 ms,
    // profiles/r04w_ab_c4.log; the random scene's top level keeps its pairs, see above)
    bool split_blas_pairs = true;
    bool in_blas = false;   // make_blas is building
    int root_leaf = 8;    // a whole BVH of at most this many items is one leaf

    int build_rec(std::vector<Item>& items, int b, int e, int depth)
    {
        const int n = e - b;
        const double c_trav = 1.0;
        double plo[3], phi[3];
        bounds(items, b, e, plo, phi);
        double parea = area(plo, phi);
        bool has_box = false;   // a Box, a medium or an instance over a BVH: a costly test
        if (split_box_pairs)
            for (int i = b; i < e && !has_box; ++i) {
                if (items[i].prim < 0) continue;
                const rt_prim& q = f.prims[(size_t)items[i].prim];
                has_box = q.kind == RT_PRIM_BOX || q.kind == RT_PRIM_MEDIUM ||
                          (q.kind == RT_PRIM_INSTANCE && f.instances[(size_t)q.a].child_kind == RT_CHILD_BVH);
            }
        const bool split_pair = has_box || (split_blas_pairs && in_blas);
        if (n <= 1 || (n <= force_leaf && !split_pair) || (depth == 0 && n <= root_leaf)) return make_leaf(items, b, e);
        if (depth >= 20) {  // bound the traversal stack: median split on the widest centroid axis
            double clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = b; i < e; ++i)
                for (int a = 0; a < 3; ++a) { clo[a] = std::min(clo[a], items[i].c[a]); chi[a] = std::max(chi[a], items[i].c[a]); }
            int ax = 0;
            for (int a = 1; a < 3; ++a) if (chi[a] - clo[a] > chi[ax] - clo[ax]) ax = a;
            return split_at(items, b, e, ax, n / 2, depth);
        }
        // full-sweep SAH over the three axes (centroid order; ties by prim index)
        double best_cost = INFINITY;
        int best_axis = -1, best_split = -1;
        std::vector<double> right_area(n);
        for (int axis = 0; axis < 3; ++axis) {
            std::sort(items.begin() + b, items.begin() + e, [axis](const Item& x, const Item& y) {
                return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.prim < y.prim);
            });
            double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = n - 1; i >= 1; --i) {
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::min(lo[a], items[b + i].lo[a]);
                    hi[a] = std::max(hi[a], items[b + i].hi[a]);
                }
                right_area[i] = area(lo, hi);
            }
            for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
            for (int i = 1; i < n; ++i) {
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::min(lo[a], items[b + i - 1].lo[a]);
                    hi[a] = std::max(hi[a], items[b + i - 1].hi[a]);
                }
                double cost = c_trav + c_isect * (area(lo, hi) * i + right_area[i] * (n - i)) / std::max(parea, 1e-300);
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_split = i;
                }
            }
        }
        double leaf_cost = c_isect * n;
        if (n <= max_leaf && leaf_cost <= best_cost) return make_leaf(items, b, e);
        if (best_axis < 0) best_axis = 0, best_split = n / 2;
        return split_at(items, b, e, best_axis, best_split, depth);
    }

    int split_at(std::vector<Item>& items, int b, int e, int axis, int split, int depth)
    {
        std::sort(items.begin() + b, items.begin() + e, [axis](const Item& x, const Item& y) {
            return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.prim < y.prim);
        });
        int mid = b + split;
        int node = (int)f.nodes.size();
        f.nodes.emplace_back();
        double llo[3], lhi[3], rlo[3], rhi[3];
        bounds(items, b, mid, llo, lhi);
        bounds(items, mid, e, rlo, rhi);
        int lc = build_rec(items, b, mid, depth + 1);
        int rc = build_rec(items, mid, e, depth + 1);
        rt_bvh_node& nd = f.nodes[node];
        std::memset(&nd, 0, sizeof nd);
        to_f32_box(llo, lhi, nd.lo0, nd.hi0);
        to_f32_box(rlo, rhi, nd.lo1, nd.hi1);
        nd.child[0] = lc;
        nd.child[1] = rc;
        return node;
    }

    int blas_depth = 0;   // max over instance BLASes

    // LINEAR / MEDIAN: the list in order. Runs of primitives become <=31-prim leaves, a
    // subtree stays a child; node k = (segment k, node k+1), both boxes unbounded, so the
    // slab tests return t_near = t_min for both and the walk always takes segment k first
    // (list order) with the rest of the chain as its one stack entry.
    int build_chain(std::vector<Item>& items)
    {
        std::vector<int> segs;
        for (size_t i = 0; i < items.size();) {
            if (items[i].prim < 0) {
                segs.push_back(items[i].ref);
                ++i;
                continue;
            }
            size_t j = i;
            while (j < items.size() && items[j].prim >= 0 && j - i < 31) ++j;
            segs.push_back(make_leaf(items, (int)i, (int)j));
            i = j;
        }
        if (segs.empty()) return RT_LEAF_CODE((int)f.prim_refs.size(), 0);
        if (segs.size() == 1) return segs[0];
        const int base = (int)f.nodes.size(), n = (int)segs.size() - 1;
        f.nodes.resize(base + n);
        for (int k = 0; k < n; ++k) {
            rt_bvh_node& nd = f.nodes[base + k];
            std::memset(&nd, 0, sizeof nd);
            for (int a = 0; a < 3; ++a) {
                nd.lo0[a] = nd.lo1[a] = -INFINITY;
                nd.hi0[a] = nd.hi1[a] = INFINITY;
            }
            nd.child[0] = segs[k];
            nd.child[1] = k + 1 < n ? base + k + 1 : segs[n];
        }
        return base;
    }

    // Stack entries a walk from ref can need (the kernel's visit pushes the farther child
    // when both are hit). With two identical child boxes both t_near are equal and child 0
    // is always taken first, so only it stacks on top of the pushed child 1.
    int stack_need(int ref) const
    {
        if (ref < 0) return 0;
        std::vector<int> need(f.nodes.size(), -1);
        std::vector<int> todo{ref};  // iterative post-order (a LINEAR chain can be long)
        while (!todo.empty()) {
            const int i = todo.back();
            const rt_bvh_node& nd = f.nodes[i];
            bool ready = true;
            for (int c : nd.child)
                if (c >= 0 && need[c] < 0) {
                    todo.push_back(c);
                    ready = false;
                }
            if (!ready) continue;
            todo.pop_back();
            auto nc = [&](int c) { return c < 0 ? 0 : need[c]; };
            const bool same = std::memcmp(nd.lo0, nd.lo1, 12) == 0 && std::memcmp(nd.hi0, nd.hi1, 12) == 0;
            need[i] = same ? std::max(1 + nc(nd.child[0]), nc(nd.child[1]))
                           : 1 + std::max(nc(nd.child[0]), nc(nd.child[1]));
        }
        return need[ref];
    }

    int build_bvh(std::vector<Item>& items)
    {
        if (accel != RT_ACCEL_SAH) return build_chain(items);
        if (items.empty()) return RT_LEAF_CODE((int)f.prim_refs.size(), 0);
        return build_rec(items, 0, (int)items.size(), 0);
    }
};

}  // namespace

int flatten(World& w, int accel, std::string& err)
{
    if (accel != RT_ACCEL_SAH && accel != RT_ACCEL_LINEAR && accel != RT_ACCEL_MEDIAN) {
        err = "unknown accel mode";
        return RT_ERR_INVALID;
    }
    FlatScene f;
    Builder bld{w, f, err};
    bld.accel = accel;
    // SAH build options (rt_world_set_build_option; defaults DESIGN.md §2 / §5.2)
    const BuildOptions& bo = w.build;
    if (bo.c_isect > 0.0) bld.c_isect = std::max(0.01, bo.c_isect);
    if (bo.max_leaf > 0) bld.max_leaf = std::min(31, std::max(2, bo.max_leaf));
    if (bo.force_leaf > 0) bld.force_leaf = std::min(31, std::max(1, bo.force_leaf));
    if (bo.root_leaf >= 0) bld.root_leaf = std::min(31, bo.root_leaf);
    if (bo.split_box_pairs >= 0) bld.split_box_pairs = bo.split_box_pairs != 0;
    if (bo.split_blas_pairs >= 0) bld.split_blas_pairs = bo.split_blas_pairs != 0;
    std::vector<Item> top;
    for (int id : w.hittables) {  // M for the f32-slab padding (see to_f32_box)
        AABB b;
        if (w.valid_hittable(id) && w.bounding_box(id, 0.0, 1.0, b)) {
            const double c[6] = {b.minimum.x, b.minimum.y, b.minimum.z, b.maximum.x, b.maximum.y, b.maximum.z};
            for (double v : c)
                if (std::isfinite(v)) bld.world_extent = std::max(bld.world_extent, std::fabs(v));
        }
    }
    bld.pad_abs = 0x1.0p-18 * bld.world_extent;
    for (int id : w.hittables) {
        if (!w.valid_hittable(id)) {
            err = "invalid hittable id in world list";
            return RT_ERR_INVALID;
        }
        int rc = bld.lower_top(id, top);
        if (rc) return rc;
    }
    // instances build their BLAS while being lowered, so take M from the world's boxes first
    f.tlas_root = bld.build_bvh(top);
    const int tlas_depth = bld.stack_need(f.tlas_root) + 1;
    // the kernel's traversal stack: a TLAS walk, and a nested BLAS walk above it (<= 32 each)
    if (tlas_depth > 32 || bld.blas_depth > 32) {
        err = "BVH too deep for the kernel's traversal stack";
        return RT_ERR_UNSUPPORTED;
    }
    // Renumber: the TLAS's nodes first, in BFS order (the kernel copies that prefix into
    // LDS), then every BLAS node in build order.
    int n_tlas_nodes = 0;
    if (f.tlas_root >= 0) {
        std::vector<int> order, remap(f.nodes.size(), -1);
        order.push_back(f.tlas_root);
        for (size_t i = 0; i < order.size(); ++i)
            for (int c : f.nodes[order[i]].child)
                if (c >= 0) order.push_back(c);
        n_tlas_nodes = (int)order.size();
        for (int i = 0; i < (int)order.size(); ++i) remap[order[i]] = i;
        int next = n_tlas_nodes;
        for (size_t i = 0; i < f.nodes.size(); ++i)
            if (remap[i] < 0) remap[i] = next++;
        std::vector<rt_bvh_node> nodes(f.nodes.size());
        for (size_t i = 0; i < f.nodes.size(); ++i) {
            rt_bvh_node nd = f.nodes[i];
            for (int& c : nd.child)
                if (c >= 0) c = remap[c];
            nodes[remap[i]] = nd;
        }
        f.nodes.swap(nodes);
        f.tlas_root = remap[f.tlas_root];
        for (rt_instance& in : f.instances)
            if (in.child_kind == RT_CHILD_BVH && in.child >= 0) in.child = remap[in.child];
    }
    f.media = w.n_media;

    for (const Material& m : w.materials) {
        rt_material rm;
        std::memset(&rm, 0, sizeof rm);
        rm.kind = m.kind;
        rm.tex = m.tex;
        rm.albedo[0] = m.albedo.x; rm.albedo[1] = m.albedo.y; rm.albedo[2] = m.albedo.z;
        rm.fuzz = m.fuzz;
        rm.ir = m.ir;
        f.materials.push_back(rm);
    }
    for (const PerlinTables& p : w.perlins) {
        for (int i = 0; i < 256; ++i)
            for (int a = 0; a < 3; ++a) f.perlin_ranvec.push_back(p.ranvec[i][a]);
        for (int a = 0; a < 3; ++a)
            for (int i = 0; i < 256; ++i) f.perlin_perm.push_back(p.perm[a][i]);
    }
    std::vector<int64_t> img_off;
    for (const Image& im : w.images) {
        img_off.push_back((int64_t)f.image.size());
        f.image.insert(f.image.end(), im.rgb.begin(), im.rgb.end());
    }
    for (const Texture& t : w.textures) {
        rt_texture rt;
        std::memset(&rt, 0, sizeof rt);
        rt.kind = t.kind;
        rt.perlin = t.perlin;
        rt.c0[0] = t.c0.x; rt.c0[1] = t.c0.y; rt.c0[2] = t.c0.z;
        rt.c1[0] = t.c1.x; rt.c1[1] = t.c1.y; rt.c1[2] = t.c1.z;
        rt.scale = t.scale;
        if (t.kind == RT_TEX_IMAGE) {
            const Image& im = w.images[t.image];
            rt.img_w = im.rgb.empty() ? 0 : im.w;
            rt.img_h = im.rgb.empty() ? 0 : im.h;
            rt.img_offset = img_off[t.image];
            rt.img_bps = 3 * (int64_t)im.w;
        }
        f.textures.push_back(rt);
    }

    rt_scene_soa& s = f.soa;
    std::memset(&s, 0, sizeof s);
    s.n_prims = (int32_t)f.prims.size();
    s.n_prim_refs = (int32_t)f.prim_refs.size();
    s.n_nodes = (int32_t)f.nodes.size();
    s.n_instances = (int32_t)f.instances.size();
    s.n_materials = (int32_t)f.materials.size();
    s.n_textures = (int32_t)f.textures.size();
    s.n_perlin = (int32_t)w.perlins.size();
    s.n_media = f.media;
    s.tlas_root = f.tlas_root;
    s.accel = accel;
    s.image_bytes = (int64_t)f.image.size();
    s.pad_extent = bld.world_extent;
    s.tlas_depth = tlas_depth;
    s.n_tlas_nodes = n_tlas_nodes;
    s.blas_depth = bld.blas_depth;
    w.flat = std::move(f);
    FlatScene& g = w.flat;
    rt_scene_soa& t = g.soa;
    t.prims = g.prims.data();
    t.prim_refs = g.prim_refs.data();
    t.nodes = g.nodes.data();
    t.instances = g.instances.data();
    t.materials = g.materials.data();
    t.textures = g.textures.data();
    t.perlin_ranvec = g.perlin_ranvec.data();
    t.perlin_perm = g.perlin_perm.data();
    t.image_data = g.image.data();
    return RT_OK;
}

}  // namespace rtw
