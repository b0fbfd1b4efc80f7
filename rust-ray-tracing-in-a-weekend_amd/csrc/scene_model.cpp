// scene_model.cpp — World construction with the reference's semantics and draw
// order. Citations: /root/reference/src/<file>:<line>.
#include "scene_model.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "rt/rt_abi.h"

namespace rtw {

static inline double degrees_to_radians(double d) { return d * RT_PI / 180.0; }  // math.rs:8-10
static inline V3 normalize(V3 v) { return v / std::sqrt(length_squared(v)); }    // math.rs:102-104

World::World(uint64_t scene_seed) { rt_stream_init(&rng, scene_seed, 0, 0, RT_STREAM_SCENE); }

// math.rs:268-280 restated over the seeded stream (rt_numerics.h).
double World::random_double() { return rt_unit53(rt_stream_next_u64(&rng)); }
double World::random_double_range(double a, double b)
{
    return rt_uniform_sample(rt_stream_next_u64(&rng), a, rt_uniform_incl_scale(a, b));
}
int World::random_int_range(int a, int b) { return rt_sat_i32(random_double_range((double)a, (double)(b + 1))); }
V3 World::random_v3()  // math.rs:35-41 (fields drawn x, y, z)
{
    double x = random_double();
    double y = random_double();
    double z = random_double();
    return v3(x, y, z);
}
V3 World::random_v3_range(double a, double b)  // math.rs:43-49
{
    double x = random_double_range(a, b);
    double y = random_double_range(a, b);
    double z = random_double_range(a, b);
    return v3(x, y, z);
}

int World::texture_solid(V3 c)
{
    Texture t;
    t.kind = RT_TEX_SOLID;
    t.c0 = c;
    textures.push_back(t);
    return (int)textures.size() - 1;
}
int World::texture_checker(V3 even, V3 odd)
{
    Texture t;
    t.kind = RT_TEX_CHECKER;
    t.c0 = even;
    t.c1 = odd;
    textures.push_back(t);
    return (int)textures.size() - 1;
}
// Perlin::new (perlin.rs:13-30) with perlin_generate_perm / permute (:110-129).
int World::texture_noise(double scale)
{
    PerlinTables pt;
    for (int i = 0; i < 256; ++i) {
        V3 r = normalize(random_v3_range(-1.0, 1.0));
        pt.ranvec[i][0] = r.x;
        pt.ranvec[i][1] = r.y;
        pt.ranvec[i][2] = r.z;
    }
    for (int axis = 0; axis < 3; ++axis) {
        int32_t* p = pt.perm[axis];
        for (int i = 0; i < 256; ++i) p[i] = i;
        for (int i = 255; i >= 0; --i) {
            int target = random_int_range(0, i);
            target = std::min(std::max(target, 0), 255);
            int32_t tmp = p[i];
            p[i] = target;  // the index, not p[target]
            p[target] = tmp;
        }
    }
    perlins.push_back(pt);
    Texture t;
    t.kind = RT_TEX_NOISE;
    t.perlin = (int)perlins.size() - 1;
    t.scale = scale;
    textures.push_back(t);
    return (int)textures.size() - 1;
}
int World::texture_image(const uint8_t* rgb, int w, int h)  // texture.rs:12-22
{
    Image im;
    im.w = w;
    im.h = h;
    if (rgb && w > 0 && h > 0) im.rgb.assign(rgb, rgb + (size_t)w * h * 3);
    images.push_back(std::move(im));
    Texture t;
    t.kind = RT_TEX_IMAGE;
    t.image = (int)images.size() - 1;
    textures.push_back(t);
    return (int)textures.size() - 1;
}

int World::register_material(const Material& m)  // main.rs:46-49
{
    materials.push_back(m);
    return (int)materials.size();
}
int World::lambertian(int tex) { Material m; m.kind = RT_MAT_LAMBERTIAN; m.tex = tex; return register_material(m); }
int World::metal(V3 albedo, double fuzz)
{
    Material m;
    m.kind = RT_MAT_METAL;
    m.albedo = albedo;
    m.fuzz = fuzz;
    return register_material(m);
}
int World::dielectric(double ir) { Material m; m.kind = RT_MAT_DIELECTRIC; m.ir = ir; return register_material(m); }
int World::diffuse_light(int tex) { Material m; m.kind = RT_MAT_DIFFUSE_LIGHT; m.tex = tex; return register_material(m); }
int World::isotropic(int tex) { Material m; m.kind = RT_MAT_ISOTROPIC; m.tex = tex; return register_material(m); }

int World::sphere(int mat, V3 c, double r)
{
    HNode n;
    n.kind = HKind::Sphere;
    n.mat = mat;
    n.c0 = c;
    n.radius = r;
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}
int World::moving_sphere(int mat, V3 c0, V3 c1, double t0, double t1, double r)
{
    HNode n;
    n.kind = HKind::MovingSphere;
    n.mat = mat;
    n.c0 = c0;
    n.c1 = c1;
    n.t0 = t0;
    n.t1 = t1;
    n.radius = r;
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}
int World::rect(HKind kind, int mat, double a0, double a1, double b0, double b1, double k)
{
    HNode n;
    n.kind = kind;
    n.mat = mat;
    n.a0 = a0;
    n.a1 = a1;
    n.b0 = b0;
    n.b1 = b1;
    n.k = k;
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}
int World::box(V3 mn, V3 mx, int mat)  // hittable.rs:132-145 (the 6 sides are implied by min/max)
{
    HNode n;
    n.kind = HKind::Box;
    n.mat = mat;
    n.bmin = mn;
    n.bmax = mx;
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}
int World::translate(int child, V3 offset)
{
    HNode n;
    n.kind = HKind::Translate;
    n.ptr = child;
    n.offset = offset;
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}
int World::rotate_y(int child, double angle)  // hittable.rs:147-199
{
    HNode n;
    n.kind = HKind::RotateY;
    n.ptr = child;
    double radians = degrees_to_radians(angle);
    n.sin_theta = std::sin(radians);
    n.cos_theta = std::cos(radians);
    AABB bbox;
    if (bounding_box(child, 0.0, 1.0, bbox)) {
        n.has_box = true;
    } else {
        n.has_box = false;
        bbox = AABB{v3(0, 0, 0), v3(0, 0, 0)};
    }
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int k = 0; k < 2; ++k) {
                double fi = i, fj = j, fk = k;
                double x = fi * bbox.maximum.x + (1.0 - fi) * bbox.minimum.x;
                double y = fj * bbox.maximum.y + (1.0 - fj) * bbox.minimum.y;
                double z = fk * bbox.maximum.z + (1.0 - fk) * bbox.minimum.z;
                double newx = n.cos_theta * x + n.sin_theta * z;
                double newz = -n.sin_theta * x + n.cos_theta * z;
                double tester[3] = {newx, y, newz};
                for (int c = 0; c < 3; ++c) {
                    mn[c] = std::fmin(mn[c], tester[c]);
                    mx[c] = std::fmax(mx[c], tester[c]);
                }
            }
    n.box = AABB{v3(mn[0], mn[1], mn[2]), v3(mx[0], mx[1], mx[2])};
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}
int World::constant_medium(int boundary, double density, int phase)  // hittable.rs:201-207
{
    HNode n;
    n.kind = HKind::ConstantMedium;
    n.ptr = boundary;
    n.mat = phase;
    n.neg_inv_density = -1.0 / density;
    n.medium_id = n_media++;
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}

static V3 center_at_time(V3 c0, V3 c1, double t0, double t1, double time)  // hittable.rs:556-558
{
    return c0 + (c1 - c0) * ((time - t0) / (t1 - t0));
}
static AABB surrounding(AABB a, AABB b)  // aabb.rs:19-33
{
    return AABB{v3(std::fmin(a.minimum.x, b.minimum.x), std::fmin(a.minimum.y, b.minimum.y),
                   std::fmin(a.minimum.z, b.minimum.z)),
                v3(std::fmax(a.maximum.x, b.maximum.x), std::fmax(a.maximum.y, b.maximum.y),
                   std::fmax(a.maximum.z, b.maximum.z))};
}

bool World::bounding_box(int id, double time0, double time1, AABB& out) const  // hittable.rs:475-554
{
    const HNode& h = nodes[id];
    switch (h.kind) {
    case HKind::Sphere: {
        V3 r = v3(h.radius, h.radius, h.radius);
        out = AABB{h.c0 - r, h.c0 + r};
        return true;
    }
    case HKind::MovingSphere: {
        V3 c0 = center_at_time(h.c0, h.c1, h.t0, h.t1, h.t0);
        V3 c1 = center_at_time(h.c0, h.c1, h.t0, h.t1, h.t1);
        V3 r = v3(h.radius, h.radius, h.radius);
        out = surrounding(AABB{c0 - r, c0 + r}, AABB{c1 - r, c1 + r});
        return true;
    }
    case HKind::BvhNode: out = h.box; return true;
    case HKind::XYRect: out = AABB{v3(h.a0, h.b0, h.k - 0.0001), v3(h.a1, h.b1, h.k + 0.0001)}; return true;
    case HKind::XZRect: out = AABB{v3(h.a0, h.k - 0.0001, h.b0), v3(h.a1, h.k + 0.0001, h.b1)}; return true;
    case HKind::YZRect: out = AABB{v3(h.k - 0.0001, h.a0, h.b0), v3(h.k + 0.0001, h.a1, h.b1)}; return true;
    case HKind::Box: out = AABB{h.bmin, h.bmax}; return true;
    case HKind::Translate: {
        AABB b;
        if (!bounding_box(h.ptr, time0, time1, b)) return false;
        out = AABB{b.minimum + h.offset, b.maximum + h.offset};
        return true;
    }
    case HKind::RotateY:
        if (!h.has_box) return false;
        out = h.box;
        return true;
    case HKind::ConstantMedium: return bounding_box(h.ptr, time0, time1, out);
    }
    return false;
}

// new_bvh_node (hittable.rs:77-130): axis drawn at every node, span 1 duplicates,
// span 2 ordered by the comparator, otherwise a stable sort by the box minimum
// (aabb.rs:35-60) and a median split.
int World::bvh(const std::vector<int>& list, int start, int end, double t0, double t1)
{
    std::vector<int> cpy = list;
    int axis = random_int_range(0, 2);
    if (axis != 0 && axis != 1) axis = 2;
    auto key = [&](int id, double& v) {
        AABB b;
        if (!bounding_box(id, 0.0, 0.0, b)) return false;
        v = axis == 0 ? b.minimum.x : axis == 1 ? b.minimum.y : b.minimum.z;
        return true;
    };
    auto is_less = [&](int a, int b) {
        double ka, kb;
        if (!key(a, ka) || !key(b, kb)) return false;
        return ka < kb;
    };
    HNode n;
    n.kind = HKind::BvhNode;
    int span = end - start;
    if (span == 1) {
        n.left = n.right = cpy[start];
    } else if (span == 2) {
        if (is_less(cpy[start], cpy[start + 1])) {
            n.left = cpy[start];
            n.right = cpy[start + 1];
        } else {
            n.left = cpy[start + 1];
            n.right = cpy[start];
        }
    } else {
        std::stable_sort(cpy.begin() + start, cpy.begin() + end, is_less);
        int mid = start + span / 2;
        n.left = bvh(cpy, start, mid, t0, t1);
        n.right = bvh(cpy, mid, end, t0, t1);
    }
    AABB bl, br;
    if (bounding_box(n.left, t0, t1, bl) && bounding_box(n.right, t0, t1, br))
        n.box = surrounding(bl, br);
    else
        n.box = AABB{v3(0, 0, 0), v3(0, 0, 0)};
    nodes.push_back(n);
    return (int)nodes.size() - 1;
}

// ---------------------------------------------------------------------------
// Scene builders (main.rs:52-289), same draw order as the reference.
// ---------------------------------------------------------------------------
static void two_spheres(World& w)  // main.rs:52-63
{
    int ground = w.lambertian(w.texture_checker(v3(0.2, 0.3, 0.1), v3(0.9, 0.9, 0.9)));
    w.push(w.sphere(ground, v3(0.0, -10.0, 0.0), 10.0));
    w.push(w.sphere(ground, v3(0.0, 10.0, 0.0), 10.0));
}
static void two_perlin_spheres(World& w)  // main.rs:65-76
{
    int ground = w.lambertian(w.texture_noise(4.0));
    w.push(w.sphere(ground, v3(0.0, -1000.0, 0.0), 1000.0));
    w.push(w.sphere(ground, v3(0.0, 2.0, 0.0), 2.0));
}
static void earth(World& w, const uint8_t* img, int iw, int ih)  // main.rs:78-89
{
    int m = w.lambertian(w.texture_image(img, iw, ih));
    w.push(w.sphere(m, v3(0.0, 0.0, 0.0), 2.0));
}
static void simple_light(World& w)  // main.rs:91-105
{
    int ground = w.lambertian(w.texture_noise(4.0));
    w.push(w.sphere(ground, v3(0.0, -1000.0, 0.0), 1000.0));
    w.push(w.sphere(ground, v3(0.0, 2.0, 0.0), 2.0));
    int light = w.diffuse_light(w.texture_solid(v3(4.0, 4.0, 4.0)));
    w.push(w.rect(HKind::XYRect, light, 3.0, 5.0, 1.0, 3.0, -2.0));
}
static void cornell_walls(World& w, int red, int white, int green, int light, double lx0, double lx1, double lz0,
                          double lz1)  // main.rs:118-123
{
    w.push(w.rect(HKind::YZRect, green, 0.0, 555.0, 0.0, 555.0, 555.0));
    w.push(w.rect(HKind::YZRect, red, 0.0, 555.0, 0.0, 555.0, 0.0));
    w.push(w.rect(HKind::XZRect, light, lx0, lx1, lz0, lz1, 554.0));
    w.push(w.rect(HKind::XZRect, white, 0.0, 555.0, 0.0, 555.0, 0.0));
    w.push(w.rect(HKind::XZRect, white, 0.0, 555.0, 0.0, 555.0, 555.0));
    w.push(w.rect(HKind::XYRect, white, 0.0, 555.0, 0.0, 555.0, 555.0));
}
static void cornell_box(World& w)  // main.rs:107-136
{
    int red = w.lambertian(w.texture_solid(v3(0.65, 0.05, 0.05)));
    int white = w.lambertian(w.texture_solid(v3(0.73, 0.73, 0.73)));
    int green = w.lambertian(w.texture_solid(v3(0.12, 0.45, 0.15)));
    int light = w.diffuse_light(w.texture_solid(v3(15.0, 15.0, 15.0)));
    cornell_walls(w, red, white, green, light, 213.0, 343.0, 227.0, 332.0);
    int box1 = w.box(v3(0, 0, 0), v3(165.0, 330.0, 165.0), white);
    box1 = w.rotate_y(box1, 15.0);
    box1 = w.translate(box1, v3(265.0, 0.0, 295.0));
    w.push(box1);
    int box2 = w.box(v3(0, 0, 0), v3(165.0, 165.0, 165.0), white);
    box2 = w.rotate_y(box2, -18.0);
    box2 = w.translate(box2, v3(130.0, 0.0, 65.0));
    w.push(box2);
}
static void cornell_smoke(World& w)  // main.rs:138-171
{
    int red = w.lambertian(w.texture_solid(v3(0.65, 0.05, 0.05)));
    int white = w.lambertian(w.texture_solid(v3(0.73, 0.73, 0.73)));
    int green = w.lambertian(w.texture_solid(v3(0.12, 0.45, 0.15)));
    int light = w.diffuse_light(w.texture_solid(v3(7.0, 7.0, 7.0)));
    cornell_walls(w, red, white, green, light, 113.0, 443.0, 127.0, 432.0);
    int box1_phase = w.isotropic(w.texture_solid(v3(0.0, 0.0, 0.0)));
    int box1 = w.box(v3(0, 0, 0), v3(165.0, 330.0, 165.0), white);
    box1 = w.rotate_y(box1, 15.0);
    box1 = w.translate(box1, v3(265.0, 0.0, 295.0));
    box1 = w.constant_medium(box1, 0.01, box1_phase);
    w.push(box1);
    int box2_phase = w.isotropic(w.texture_solid(v3(1.0, 1.0, 1.0)));
    int box2 = w.box(v3(0, 0, 0), v3(165.0, 165.0, 165.0), white);
    box2 = w.rotate_y(box2, -18.0);
    box2 = w.translate(box2, v3(130.0, 0.0, 65.0));
    box2 = w.constant_medium(box2, 0.01, box2_phase);
    w.push(box2);
}
static void final_scene(World& w, const uint8_t* img, int iw, int ih)  // main.rs:173-243
{
    std::vector<int> boxes1;
    int ground = w.lambertian(w.texture_solid(v3(0.48, 0.83, 0.53)));
    const int boxes_per_side = 20;
    for (int i = 0; i < boxes_per_side; ++i)
        for (int j = 0; j < boxes_per_side; ++j) {
            double wd = 100.0;
            double x0 = -1000.0 + (double)i * wd;
            double z0 = -1000.0 + (double)j * wd;
            double y0 = 0.0;
            double x1 = x0 + wd;
            double y1 = w.random_double_range(1.0, 101.0);
            double z1 = z0 + wd;
            boxes1.push_back(w.box(v3(x0, y0, z0), v3(x1, y1, z1), ground));
        }
    w.push(w.bvh(boxes1, 0, (int)boxes1.size(), 0.0, 1.0));
    int light = w.diffuse_light(w.texture_solid(v3(7.0, 7.0, 7.0)));
    w.push(w.rect(HKind::XZRect, light, 123.0, 423.0, 147.0, 412.0, 554.0));
    V3 center_1 = v3(400.0, 400.0, 200.0);
    V3 center_2 = center_1 + v3(30.0, 0.0, 0.0);
    int msm = w.lambertian(w.texture_solid(v3(0.7, 0.3, 0.1)));
    w.push(w.moving_sphere(msm, center_1, center_2, 0.0, 1.0, 50.0));
    int dielectric = w.dielectric(1.5);
    w.push(w.sphere(dielectric, v3(260.0, 150.0, 45.0), 50.0));
    int metal = w.metal(v3(0.8, 0.8, 0.9), 1.0);
    w.push(w.sphere(metal, v3(0.0, 150.0, 145.0), 50.0));
    int boundary = w.sphere(dielectric, v3(360.0, 150.0, 145.0), 70.0);
    w.push(boundary);
    int phase = w.isotropic(w.texture_solid(v3(0.2, 0.4, 0.9)));
    w.push(w.constant_medium(boundary, 0.2, phase));
    boundary = w.sphere(dielectric, v3(0.0, 0.0, 0.0), 5000.0);
    phase = w.isotropic(w.texture_solid(v3(1.0, 1.0, 1.0)));
    w.push(w.constant_medium(boundary, 0.0001, phase));
    int emat = w.lambertian(w.texture_image(img, iw, ih));
    w.push(w.sphere(emat, v3(400.0, 200.0, 400.0), 100.0));
    int pertext = w.lambertian(w.texture_noise(0.1));
    w.push(w.sphere(pertext, v3(220.0, 280.0, 300.0), 80.0));
    std::vector<int> boxes2;
    int white = w.lambertian(w.texture_solid(v3(0.73, 0.73, 0.73)));
    for (int j = 0; j < 1000; ++j) boxes2.push_back(w.sphere(white, w.random_v3_range(0.0, 165.0), 10.0));
    int bvh2 = w.bvh(boxes2, 0, (int)boxes2.size(), 0.0, 1.0);
    w.push(w.translate(w.rotate_y(bvh2, 15.0), v3(-100.0, 270.0, 395.0)));
}
static void random_scene(World& w)  // main.rs:245-289
{
    int ground = w.lambertian(w.texture_checker(v3(0.2, 0.5, 0.5), v3(0.9, 0.9, 0.9)));
    w.push(w.sphere(ground, v3(0.0, -1000.0, 0.0), 1000.0));
    for (int a = -11; a < 11; ++a)
        for (int b = -11; b < 11; ++b) {
            double choose_mat = w.random_double();
            double cx = (double)a + 0.9 * w.random_double();
            double cz = (double)b + 0.9 * w.random_double();
            V3 center = v3(cx, 0.2, cz);
            if (std::sqrt(length_squared(center - v3(4.0, 0.2, 0.0))) > 0.9) {
                if (choose_mat < 0.8) {
                    V3 albedo = w.random_v3();
                    int m = w.lambertian(w.texture_solid(albedo));
                    V3 center2 = center + v3(0.0, w.random_double_range(0.0, 0.5), 0.0);
                    w.push(w.moving_sphere(m, center, center2, 0.0, 1.0, 0.2));
                } else if (choose_mat < 0.95) {
                    V3 albedo = w.random_v3_range(0.5, 1.0);
                    double fuzz = w.random_double_range(0.0, 0.5);
                    int m = w.metal(albedo, fuzz);
                    w.push(w.sphere(m, center, 0.2));
                } else {
                    int m = w.dielectric(1.5);
                    w.push(w.sphere(m, center, 0.2));
                }
            }
        }
    int m1 = w.dielectric(1.5);
    w.push(w.sphere(m1, v3(0.0, 1.0, 0.0), 1.0));
    int m2 = w.lambertian(w.texture_solid(v3(0.4, 0.2, 0.1)));
    w.push(w.sphere(m2, v3(-4.0, 1.0, 0.0), 1.0));
    int m3 = w.metal(v3(0.7, 0.6, 0.5), 0.0);
    w.push(w.sphere(m3, v3(4.0, 1.0, 0.0), 1.0));
}

int build_scene(World& w, int scene_id, const uint8_t* img, int iw, int ih)
{
    if ((scene_id == 3 || scene_id == 7) && (!img || iw <= 0 || ih <= 0)) return RT_ERR_INVALID;
    switch (scene_id) {
    case 0: random_scene(w); return RT_OK;
    case 1: two_spheres(w); return RT_OK;
    case 2: two_perlin_spheres(w); return RT_OK;
    case 3: earth(w, img, iw, ih); return RT_OK;
    case 4: simple_light(w); return RT_OK;
    case 5: cornell_box(w); return RT_OK;
    case 6: cornell_smoke(w); return RT_OK;
    case 7: final_scene(w, img, iw, ih); return RT_OK;
    default: return RT_ERR_INVALID;  // main.rs:461-463 panics
    }
}

bool scene_preset(int id, Preset& p)  // main.rs:314-464
{
    switch (id) {
    case 0: case 1: case 2: case 3:
        p = Preset{v3(13.0, 2.0, 3.0), v3(0.0, 0.0, 0.0), v3(0.7, 0.8, 1.0), 20.0, 400, 100, 16.0 / 9.0};
        return true;
    case 4:
        p = Preset{v3(26.0, 3.0, 6.0), v3(0.0, 2.0, 0.0), v3(0.0, 0.0, 0.0), 20.0, 400, 100, 16.0 / 9.0};
        return true;
    case 5:
        p = Preset{v3(278.0, 278.0, -800.0), v3(278.0, 278.0, 0.0), v3(0.0, 0.0, 0.0), 40.0, 600, 200, 1.0};
        return true;
    case 6:
        p = Preset{v3(278.0, 278.0, -800.0), v3(278.0, 278.0, 0.0), v3(0.0, 0.0, 0.0), 40.0, 600, 40, 1.0};
        return true;
    case 7:
        p = Preset{v3(478.0, 278.0, -600.0), v3(278.0, 278.0, 0.0), v3(0.0, 0.0, 0.0), 40.0, 800, 2000, 1.0};
        return true;
    default: return false;
    }
}

rt_camera camera_new(V3 look_from, V3 look_at, V3 vup, double vfov, double aspect_ratio, double aperture,
                     double focus_dist, double time0, double time1)  // camera.rs:18-56
{
    double theta = degrees_to_radians(vfov);
    double h = std::tan(theta / 2.0);
    double viewport_height = 2.0 * h;
    double viewport_width = aspect_ratio * viewport_height;
    V3 w = normalize(look_from - look_at);
    V3 u = normalize(cross(vup, w));
    V3 v = cross(w, u);
    V3 origin = look_from;
    V3 horizontal = u * (focus_dist * viewport_width);
    V3 vertical = v * (focus_dist * viewport_height);
    V3 llc = origin - horizontal * 0.5 - vertical * 0.5 - w * focus_dist;
    rt_camera c;
    auto put = [](double* d, V3 a) { d[0] = a.x; d[1] = a.y; d[2] = a.z; };
    put(c.origin, origin);
    put(c.lower_left_corner, llc);
    put(c.horizontal, horizontal);
    put(c.vertical, vertical);
    put(c.u, u);
    put(c.v, v);
    put(c.w, w);
    c.lens_radius = aperture * 0.5;
    c.time0 = time0;
    c.time1 = time1;
    return c;
}

}  // namespace rtw
