// trace_v_final.hip — instantiates the megakernel (trace_device.hpp) for one feature set
// (FEAT_SET_FINAL, count_work false); each variant is its own translation unit so the build
// compiles them in parallel.
#include "trace_device.hpp"

namespace rtk {
template hipError_t launch_variant<FEAT_SET_FINAL, false>(const Launch&, const LaunchOpts&, hipStream_t);
}  // namespace rtk
