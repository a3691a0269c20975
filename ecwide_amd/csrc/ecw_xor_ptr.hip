// Exported XOR launchers over explicit pointers and device pointer tables
// (ecw_xor.hpp): ecw_xor_reduce_dev / ecw_decode_dev / the host pipeline, and
// ecw_xor_reduce_ptrs_dev over separately allocated blocks.
#include "ecw_xor.hpp"

namespace ecw {

hipError_t launch_xor_ptr(const XorPtr& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }
hipError_t launch_xor_tab(const XorTab& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }

}  // namespace ecw
