// bbm_amd/csrc/inst_aggregate.hip -- kernel instantiations for the Aggregate(Lambertian, X)
// compositions (the published fits' form); separate unit so the library builds in parallel.
#include "kernels.hpp"
#include "models.hpp"

namespace bbmhip {
BBM_HIP_AGGREGATE_MODELS(BBM_HIP_INSTANTIATE)
}  // namespace bbmhip
