// bbm_amd/csrc/inst_he.hip -- kernel instantiations for the He family (he.hpp): He, HeWestin,
// HeHolzschuch, NganHe (separate unit: their Taylor-series eval is the largest code in the library).
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {
BBM_HIP_HE_MODELS(BBM_HIP_INSTANTIATE)
}  // namespace bbmhip
