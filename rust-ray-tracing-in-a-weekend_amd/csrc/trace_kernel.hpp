// trace_kernel.hpp — launch interface of the megakernel (trace_kernel.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "rt/rt_scene.h"

namespace rtk {

// Device view of the uploaded rt_scene_soa tables.
struct SceneDev {
    const rt_prim* prims;
    const int32_t* prim_refs;
    const rt_bvh_node* nodes;
    const rt_instance* instances;
    const rt_material* materials;
    const rt_texture* textures;
    const double* perlin_ranvec;
    const int32_t* perlin_perm;
    const uint8_t* image;
    int32_t tlas_root;
    int32_t pad;
};

struct KParams {
    rt_camera cam;
    double bg[3];
    double scale_m11;   // rand UniformFloat::new_inclusive(-1, 1) scale
    double scale_time;  // rand UniformFloat::new_inclusive(time0, time1) scale
    uint64_t seed;
    int32_t width, height, spp, max_depth;
    int32_t spp_chunk, n_chunks;
    int32_t row_begin, row_stride, n_rows;
    int32_t tiles_x, tiles_y;   // 8x8 pixel tiles over (width, n_rows)
    int32_t pad;
};

hipError_t launch_trace(const SceneDev& S, const KParams& P, double* partial, unsigned long long* counters,
                        bool count, hipStream_t stream);
hipError_t launch_reduce(const double* partial, void* out, bool f64, long long n_px, int n_chunks, double scale,
                         hipStream_t stream);
hipError_t launch_eval(int fn, const double* x, const double* y, const double* z, double* out, int n,
                       hipStream_t stream);

}  // namespace rtk
