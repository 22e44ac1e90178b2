// bbm_amd/csrc/inst_microfacet.hip -- kernel instantiations for the microfacet compositions
// (separate unit so the library builds in parallel).
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {
BBM_HIP_MICROFACET_MODELS(BBM_HIP_INSTANTIATE)
}  // namespace bbmhip
