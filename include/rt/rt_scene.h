/*
 * rt_scene.h — the flattened scene as plain-old-data device buffers (SoA tables).
 *
 * This is what the host's Hittable/Material/Texture tree (reference:
 * hittable.rs:29-41, material.rs:6-12, texture.rs:4-9, perlin.rs:5-11) lowers to
 * before upload. Everything is C, fixed-size, pointer-free inside records (records
 * refer to each other by index), so a foreign host (e.g. the reference's Rust
 * crate over FFI) can fill these tables itself and call rt_ctx_upload_soa().
 *
 * HBM layout (one contiguous device allocation, 256-B aligned tables):
 *   nodes      rt_bvh_node[n_nodes]        64 B  two child boxes (f32, rounded outward)
 *   prim_refs  int32[n_prim_refs]           4 B  leaf ranges index this
 *   prims      rt_prim[n_prims]            96 B  geometry, material, kind
 *   instances  rt_instance[n_instances]   128 B  Translate/RotateY chains
 *   materials  rt_material[n_materials]    64 B
 *   textures   rt_texture[n_textures]      96 B
 *   perlin     f64 ranvec[n][256][3] + i32 perm[n][3][256]
 *   image      uint8 texels (RGB8 rows, texture.rs:46-73)
 */
#ifndef RT_SCENE_H
#define RT_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Primitive kinds (hittable.rs:30-41 minus BvhNode, which becomes nodes). */
enum {
    RT_PRIM_SPHERE = 0,        /* p: cx cy cz r 1/r */
    RT_PRIM_MOVING_SPHERE = 1, /* p: c0x c0y c0z r 1/r (c1-c0)xyz t0 t1; a = 1 if t0 == 0 && t1 == 1 */
    RT_PRIM_XY_RECT = 2,       /* p: x0 x1 y0 y1 k */
    RT_PRIM_XZ_RECT = 3,       /* p: x0 x1 z0 z1 k */
    RT_PRIM_YZ_RECT = 4,       /* p: y0 y1 z0 z1 k */
    RT_PRIM_BOX = 5,           /* p: minxyz maxxyz (6 rects, hittable.rs:132-145); b = 1: p[6..8] hold
                                  the box's f32 bounds (lo xyz, hi xyz), padded and rounded outward
                                  like a node's, for the kernel's conservative candidate-side test
                                  (b = 0: none, all six sides tested). The upload derives the face
                                  slabs' width from that padding (device copy: b = 2, p[9]). */
    RT_PRIM_INSTANCE = 6,      /* a: instance index */
    RT_PRIM_MEDIUM = 7         /* a: boundary prim index (SPHERE/BOX/INSTANCE), b: medium id, p[0]: -1/density */
};

typedef struct rt_prim {
    int32_t kind;
    int32_t mat;   /* 0-based material index (= reference MaterialHandle - 1); medium: phase function */
    int32_t a, b;
    double p[10];
} rt_prim; /* 96 B */

enum { RT_OP_TRANSLATE = 0, RT_OP_ROTATE_Y = 1 };
enum { RT_CHILD_PRIM = 0, RT_CHILD_BVH = 1 };

/* A chain of Translate / RotateY (hittable.rs:232-244, 386-415), outermost first. */
typedef struct rt_instance {
    int32_t n_ops;
    int32_t child_kind;      /* RT_CHILD_* */
    int32_t child;           /* prim index, or BVH root reference */
    int32_t pad;             /* reserved (0); the device copy keeps a BLAS's first leaf slot here */
    int32_t op_kind[4];
    double op[4][3];         /* translate: offset xyz; rotate_y: sin cos 0 */
} rt_instance; /* 128 B */

/* BVH node: both children's boxes (so one fetch decides both), f32 rounded outward.
 * child >= 0: node index; child < 0: leaf, code = ~child, first = code >> 5,
 * count = code & 31 (range in prim_refs). A BVH "root reference" uses the same code. */
typedef struct rt_bvh_node {
    float lo0[3], hi0[3];
    float lo1[3], hi1[3];
    int32_t child[2];
    int32_t pad[2];
} rt_bvh_node; /* 64 B */

#define RT_LEAF_CODE(first, count) (~(((int32_t)(first) << 5) | (int32_t)(count)))

enum { RT_MAT_LAMBERTIAN = 0, RT_MAT_METAL = 1, RT_MAT_DIELECTRIC = 2, RT_MAT_DIFFUSE_LIGHT = 3, RT_MAT_ISOTROPIC = 4 };

typedef struct rt_material {
    int32_t kind;
    int32_t tex;             /* texture index (lambertian / light / isotropic) */
    int32_t pad[2];
    double albedo[3];        /* metal */
    double fuzz;             /* metal */
    double ir;               /* dielectric */
    double pad2;
} rt_material; /* 64 B */

enum { RT_TEX_SOLID = 0, RT_TEX_CHECKER = 1, RT_TEX_NOISE = 2, RT_TEX_IMAGE = 3 };

typedef struct rt_texture {
    int32_t kind;
    int32_t perlin;          /* noise: perlin table index */
    int32_t img_w, img_h;    /* image */
    int64_t img_offset;      /* byte offset of the texels in the image blob */
    int64_t img_bps;         /* bytes per scanline */
    double c0[3];            /* solid color / checker even */
    double c1[3];            /* checker odd */
    double scale;            /* noise */
    double pad;
} rt_texture; /* 96 B */

typedef struct rt_scene_soa {
    int32_t n_prims, n_prim_refs, n_nodes, n_instances;
    int32_t n_materials, n_textures, n_perlin, n_media;
    int32_t tlas_root;       /* BVH root reference of the top level */
    int32_t accel;           /* RT_ACCEL_* the tables were built with */
    int64_t image_bytes;
    /* M such that every node box is padded by >= 2^-18 * M (plus BLAS offsets); the
     * kernel uses its conservative f32 slab test only when ray origins stay within 2M.
     * 0: boxes not padded, f64 slab tests only. */
    double pad_extent;
    /* stack entries a walk of the TLAS / of the deepest instance BLAS needs (<= 32 each);
     * 0: unknown (the kernel then uses a 64-entry scratch stack) */
    int32_t tlas_depth, blas_depth;
    /* the TLAS occupies nodes[0, n_tlas_nodes) in BFS order (root = 0), so the kernel can
     * keep it in LDS; 0: not arranged that way */
    int32_t n_tlas_nodes, pad0;
    const rt_prim* prims;
    const int32_t* prim_refs;
    const rt_bvh_node* nodes;
    const rt_instance* instances;
    const rt_material* materials;
    const rt_texture* textures;
    const double* perlin_ranvec;   /* [n_perlin][256][3] */
    const int32_t* perlin_perm;    /* [n_perlin][3][256] (x, y, z) */
    const uint8_t* image_data;
} rt_scene_soa;

/* Acceleration structure the flattener builds. The image does not depend
 * on it (closest hit is independent of the hierarchy); only the traversal cost does.
 *   SAH    : full-sweep SAH BVHs over the dissolved reference BvhNodes (default, fastest)
 *   LINEAR : every list scanned in order, as hit_hittables (hittable.rs:31-41) does:
 *            a chain of unbounded nodes over <=31-primitive leaves
 *   MEDIAN : the reference's own hierarchy: each BvhNode (hittable.rs:77-130, random
 *            axis + median split as drawn by the scene builder) kept as a node, the
 *            top-level list scanned in order */
enum { RT_ACCEL_SAH = 0, RT_ACCEL_LINEAR = 1, RT_ACCEL_MEDIAN = 2 };

/* Camera::new output (camera.rs:4-15). */
typedef struct rt_camera {
    double origin[3], lower_left_corner[3], horizontal[3], vertical[3];
    double u[3], v[3], w[3];
    double lens_radius, time0, time1;
} rt_camera;

#ifdef __cplusplus
}
#endif
#endif
