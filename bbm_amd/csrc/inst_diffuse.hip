// bbm_amd/csrc/inst_diffuse.hip -- kernel instantiations for the diffuse models
// (separate unit so the library builds in parallel).
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {
BBM_HIP_DIFFUSE_MODELS(BBM_HIP_INSTANTIATE)
}  // namespace bbmhip
