// Exported XOR launchers over the slab layouts (ecw_xor.hpp): the block slab
// (ecw_repair_batch_dev) and the split / tiled slabs (ecw_repair_batch_split_dev).
#include "ecw_xor.hpp"

namespace ecw {

hipError_t launch_xor_slab(const XorSlab& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }
hipError_t launch_xor_split(const XorSplit& p, const XorGeom& g, hipStream_t s) { return launch_xor(p, g, s); }

}  // namespace ecw
