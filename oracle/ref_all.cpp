/* oracle/ref_all.cpp -- TEST INFRASTRUCTURE ONLY: unity build of the reference shim.  Some reference
 * headers define non-inline functions (e.g. bbm::string::get_keyword in include/core/stringconvert.h),
 * so the shim's parts must share one translation unit. */
#include "ref_harness.cpp"
#include "ref_fit.cpp"
#include "ref_check.cpp"
#include "ref_merl.cpp"
#include "ref_runtime.cpp"
#include "ref_cli.cpp"
