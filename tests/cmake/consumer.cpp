// tests/cmake/consumer.cpp -- one translation unit of a BBM user, compiled against the ${BBM_NAME} target that the
// reference's CMake set up with BBM_BACKBONE=hip (tests/cmake/CMakeLists.txt): the reference's own headers, the
// HIP backbone's backbone.h in front of them, and libbbm_hip linked through backbone/hip/backbone.cmake.  CPU only:
// resolves models to libbbm_hip registry entries (by type and by string), no kernel runs.
#include "bbm/bbm_core.h"
#include "bsdfmodel/aggregatemodel.h"
#include "bsdfmodel/cooktorrance.h"
#include "bsdfmodel/ggx.h"
#include "bsdfmodel/lambertian.h"
#include "bsdfmodel/ward.h"
#include "bbm_hip/batch.h"
#include "bbm_hip/fit.h"
#include "bbm_hip/check.h"
#include "linearizer/spherical_linearizer.h"

#include <cstdio>
#include <string>

// the fitting and checkBsdf API compile in a consumer of the reference's CMake target: the GPU sampled loss and its
// batch satisfy the reference's loss concepts (compass takes either)
using consumer_model = bbm::aggregatemodel<bbm::lambertian<bbm::floatRGB>, bbm::cooktorrance<bbm::floatRGB>>;
static_assert(bbm::concepts::sampledlossfunction<bbm::hip::sampledlossfunction<consumer_model>>);
static_assert(bbm::concepts::sampledlossfunction<bbm::hip::batch<bbm::hip::sampledlossfunction<consumer_model>>>);

#ifndef BBM_BACKBONE_HIP
#error "the HIP backbone's backbone.h was not the one included"
#endif

int main()
{
  using C = bbm::floatRGB;
  int failures = 0;
  const auto ct = bbm::hip::describe(bbm::cooktorrance<C>());
  if(ct.composed() || std::string(bbm_hip_model_name(ct.id)) != "CookTorrance") ++failures;
  const auto nested = bbm::hip::describe(bbm::aggregatemodel<bbm::aggregatemodel<bbm::lambertian<C>, bbm::ward<C>>, bbm::ggx<C>>());
  if(!nested.composed() || nested.kids.size() != 2 || !nested.kids[0].composed()) ++failures;
  const auto s = bbm::hip::from_string(bbm::toString(bbm::aggregatemodel<bbm::lambertian<C>, bbm::cooktorrance<C>>()));
  if(s.composed() || std::string(bbm_hip_model_name(s.id)) != "Aggregate<Lambertian,CookTorrance>") ++failures;
  const auto d = bbm::hip::describe_as<double>(bbm::cooktorrance<bbm::doubleRGB>());
  if(bbm_hip_model_has_f64(d.id) != 1) ++failures;
  std::printf("{\"abi\": %d, \"cooktorrance\": \"%s\", \"nested_children\": %zu, \"failures\": %d}\n",
              bbm_hip_abi_version(), bbm_hip_model_name(ct.id), nested.kids.size(), failures);
  return failures ? 1 : 0;
}
