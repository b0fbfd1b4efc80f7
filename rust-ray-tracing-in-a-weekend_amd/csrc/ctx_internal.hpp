// ctx_internal.hpp — what comm.cpp (the multi-GPU entry points) reads of a context that the
// C ABI does not show: its device, its stream, its tile order and tile costs on the device,
// and the last-error slot of the calling thread. Implemented in abi.cpp; not exported in
// include/rt/rt_abi.h.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "rt/rt_abi.h"

namespace rtx {

// rt_last_error's text for this thread; returns code
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

int ctx_device(const rt_ctx* c);
// the context's own stream (a render with a null rt_render_params.stream runs on it)
hipStream_t ctx_stream(const rt_ctx* c);
// rt_ctx_set_tile_order's order on the device (n = 0: raster order, null)
const uint32_t* ctx_tile_order(const rt_ctx* c, int64_t* n);
// rt_ctx_set_schedule / rt_ctx_set_precision as set (RT_SCHED_*, RT_PREC_*)
int ctx_schedule(const rt_ctx* c);
int ctx_precision(const rt_ctx* c);
// RT_OPT_COMM_DIRECT as set
bool ctx_comm_direct(const rt_ctx* c);

}  // namespace rtx
