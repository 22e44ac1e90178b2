// bbm_amd/csrc/inst_lobes.hip -- kernel instantiations for the Ward / Phong / Lafortune / Ashikhmin-Shirley / Low smooth
// (separate unit so the library builds in parallel).
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {
BBM_HIP_LOBE_MODELS(BBM_HIP_INSTANTIATE)
}  // namespace bbmhip
