// trace_f32_rectinst.hip — instantiates the f32 fast mode of the megakernel (trace_device.hpp,
// Cfg::F32) for one feature set (FEAT_SET_RECTINST); one translation unit per variant
// so the build compiles them in parallel.
#include "trace_device.hpp"

namespace rtk {
template hipError_t launch_variant_f32<FEAT_SET_RECTINST>(const Launch&, const LaunchOpts&, hipStream_t);
}  // namespace rtk
