// trace_f32_final_count.hip — the f32 fast mode's count_work variant (trace_device.hpp) for one
// feature set (FEAT_SET_FINAL): path lengths and phase times of the f32 paths against the f64 ones.
#include "trace_device.hpp"

namespace rtk {
template hipError_t launch_variant_f32_count<FEAT_SET_FINAL>(const Launch&, const LaunchOpts&, hipStream_t);
}  // namespace rtk
