// scene_model.hpp — host-side scene model: the reference's World / Hittable /
// Material / Texture / Perlin surface (main.rs:40-50, hittable.rs:29-41,
// material.rs:6-12, texture.rs:4-9, perlin.rs:5-11) as an index-linked arena,
// plus the lowering of that tree into the SoA tables of rt_scene.h.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "rt/rt_numerics.h"
#include "rt/rt_scene.h"

namespace rtw {

struct V3 {
    double x, y, z;
};
inline V3 v3(double x, double y, double z) { return V3{x, y, z}; }
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
inline V3 operator*(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }    // math.rs:223-257
inline V3 operator/(V3 a, double s) { return a * (1.0 / s); }                     // math.rs:260-266
inline double dot(V3 u, V3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }
inline double length_squared(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }
inline V3 cross(V3 u, V3 v) { return v3(u.y * v.z - u.z * v.y, u.z * v.x - u.x * v.z, u.x * v.y - u.y * v.x); }

struct AABB {
    V3 minimum, maximum;
};

enum class HKind { Sphere, MovingSphere, BvhNode, XYRect, XZRect, YZRect, Box, Translate, RotateY, ConstantMedium };

// One Hittable (hittable.rs:30-41). Children are arena indices.
struct HNode {
    HKind kind = HKind::Sphere;
    int mat = 0;                       // 1-based MaterialHandle (medium: phase function)
    V3 c0{}, c1{};                     // spheres
    double t0 = 0, t1 = 0, radius = 0;
    int left = -1, right = -1;         // BvhNode
    AABB box{};                        // BvhNode aabb_box / RotateY bbox
    double a0 = 0, a1 = 0, b0 = 0, b1 = 0, k = 0;  // rects
    V3 bmin{}, bmax{};                 // Box
    V3 offset{};                       // Translate
    int ptr = -1;                      // Translate / RotateY / ConstantMedium boundary
    double sin_theta = 0, cos_theta = 1;
    bool has_box = false;
    double neg_inv_density = 0;
    int medium_id = -1;
};

struct Texture {
    int kind = RT_TEX_SOLID;
    V3 c0{}, c1{};
    int perlin = -1;
    double scale = 0;
    int image = -1;
};

struct Material {
    int kind = RT_MAT_LAMBERTIAN;
    int tex = -1;
    V3 albedo{};
    double fuzz = 0, ir = 0;
};

struct PerlinTables {
    double ranvec[256][3];
    int32_t perm[3][256];
};

struct Image {
    int w = 0, h = 0;
    std::vector<uint8_t> rgb;
};

// The lowered scene (rt_scene.h tables), owned by the world.
struct FlatScene {
    std::vector<rt_prim> prims;
    std::vector<int32_t> prim_refs;
    std::vector<rt_bvh_node> nodes;
    std::vector<rt_instance> instances;
    std::vector<rt_material> materials;
    std::vector<rt_texture> textures;
    std::vector<double> perlin_ranvec;
    std::vector<int32_t> perlin_perm;
    std::vector<uint8_t> image;
    int media = 0;
    int tlas_root = 0;
    rt_scene_soa soa{};
};

// SAH builder options of a world's flatten (rt_world_set_build_option; a value < 0, or 0 for the
// sizes and the cost, keeps the builder's default)
struct BuildOptions {
    double c_isect = 0.0;       // RT_BUILD_C_ISECT: primitive-test cost relative to a node visit
    int max_leaf = 0;           // RT_BUILD_MAX_LEAF: the largest leaf the cost model may pick
    int force_leaf = 0;         // RT_BUILD_FORCE_LEAF: a set this small is always one leaf
    int root_leaf = -1;         // RT_BUILD_ROOT_LEAF: a whole BVH of at most this many items is one leaf
    int split_box_pairs = -1;   // RT_BUILD_SPLIT_BOX_PAIRS: pairs holding a Box / medium / BLAS instance split by cost
    int split_blas_pairs = -1;  // RT_BUILD_SPLIT_BLAS_PAIRS: pairs inside instance BLASes split by cost
};

class World {
public:
    explicit World(uint64_t scene_seed);

    // thread_rng() replacement during construction (math.rs:268-280).
    double random_double();
    double random_double_range(double a, double b);
    int random_int_range(int a, int b);
    V3 random_v3();
    V3 random_v3_range(double a, double b);

    int texture_solid(V3 c);
    int texture_checker(V3 even, V3 odd);
    int texture_noise(double scale);                 // Perlin::new() + Texture::Noise
    int texture_image(const uint8_t* rgb, int w, int h);

    int register_material(const Material& m);        // returns the 1-based handle
    int lambertian(int tex);
    int metal(V3 albedo, double fuzz);
    int dielectric(double ir);
    int diffuse_light(int tex);
    int isotropic(int tex);

    int sphere(int mat, V3 c, double r);
    int moving_sphere(int mat, V3 c0, V3 c1, double t0, double t1, double r);
    int rect(HKind kind, int mat, double a0, double a1, double b0, double b1, double k);
    int box(V3 mn, V3 mx, int mat);
    int translate(int child, V3 offset);
    int rotate_y(int child, double angle);
    int constant_medium(int boundary, double density, int phase);
    int bvh(const std::vector<int>& list, int start, int end, double t0, double t1);
    void push(int id) { hittables.push_back(id); }

    bool bounding_box(int id, double time0, double time1, AABB& out) const;
    bool valid_hittable(int id) const { return id >= 0 && id < (int)nodes.size(); }
    bool valid_material(int h) const { return h >= 1 && h <= (int)materials.size(); }
    bool valid_texture(int t) const { return t >= 0 && t < (int)textures.size(); }

    rt_stream rng;
    std::vector<Texture> textures;
    std::vector<Material> materials;
    std::vector<PerlinTables> perlins;
    std::vector<Image> images;
    std::vector<HNode> nodes;
    std::vector<int> hittables;
    int n_media = 0;
    BuildOptions build;
    FlatScene flat;
};

// main.rs:52-289. Returns 0 or an RT_ERR_* code.
int build_scene(World& w, int scene_id, const uint8_t* image_rgb, int image_w, int image_h);

// Scene presets (main.rs:314-464) and Camera::new (camera.rs:18-56).
struct Preset {
    V3 look_from, look_at, background;
    double vfov;
    int width, spp;
    double aspect;
};
bool scene_preset(int scene_id, Preset& out);
rt_camera camera_new(V3 look_from, V3 look_at, V3 vup, double vfov, double aspect, double aperture,
                     double focus_dist, double time0, double time1);

// Lowering to rt_scene.h tables (flatten.cpp). Returns 0 or an RT_ERR_* code and
// sets err to a message.
int flatten(World& w, int accel, std::string& err);

}  // namespace rtw
