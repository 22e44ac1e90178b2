// bbm_amd/csrc/inst_spectral.hip -- kernel instantiations for the Spectrum-valued microfacet
// models (Bagher); separate unit so the library builds in parallel.
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {
BBM_HIP_SPECTRAL_MODELS(BBM_HIP_INSTANTIATE)
}  // namespace bbmhip
