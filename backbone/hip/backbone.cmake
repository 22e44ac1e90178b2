#########################################################################
# BBM HIP backbone (BBM_BACKBONE=hip): batched bsdfmodel evaluation on
# MI355X (gfx950) through libbbm_hip.
#
# Drop this directory in as <bbm>/backbone/hip; cmake/bbm_helpers.cmake
# includes this file when BBM_BACKBONE=hip.  Host lanes are the native
# backbone's scalar types (backbone/hip/include/backbone.h); batched work
# goes to libbbm_hip (include/bbm_hip.h) via bbm_hip/batch.h.
#
# BBM_HIP_ROOT: root of the bbm_amd tree (holds include/bbm_hip.h and
# bbm_amd/lib/libbbm_hip.so, built by `python -c "import __graft_entry__ as
# g; g.build()"`).
#########################################################################

#########################################################################
# Available configurations (device kernels: floatRGB)
#########################################################################
set(BBM_BACKBONE_CONFIGURATIONS "floatRGB" "doubleRGB")

#########################################################################
# libbbm_hip and the HIP runtime
#########################################################################
if(NOT BBM_HIP_ROOT)
  set(BBM_HIP_ROOT "$ENV{BBM_HIP_ROOT}")
endif()
if(NOT BBM_HIP_ROOT OR NOT EXISTS "${BBM_HIP_ROOT}/include/bbm_hip.h")
  message(FATAL_ERROR "BBM_BACKBONE=hip needs BBM_HIP_ROOT (the bbm_amd tree with include/bbm_hip.h).")
endif()
find_library(BBM_HIP_LIBRARY NAMES bbm_hip PATHS "${BBM_HIP_ROOT}/bbm_amd/lib" NO_DEFAULT_PATH)
if(NOT BBM_HIP_LIBRARY)
  message(FATAL_ERROR "libbbm_hip.so not found under ${BBM_HIP_ROOT}/bbm_amd/lib; build it first.")
endif()
if(NOT ROCM_PATH)
  set(ROCM_PATH "/opt/rocm")
endif()
find_library(BBM_HIP_RUNTIME NAMES amdhip64 PATHS "${ROCM_PATH}/lib" NO_DEFAULT_PATH)

#########################################################################
# Include dirs: the HIP backbone first (backbone.h, bbm_hip/batch.h), then
# the native backbone's scalar lane headers, then the C-ABI and HIP headers
#########################################################################
target_include_directories(${BBM_NAME} INTERFACE
  ${BBM_SOURCE_DIR}/backbone/hip/include
  ${BBM_SOURCE_DIR}/backbone/native/include
  ${BBM_HIP_ROOT}/include
  ${ROCM_PATH}/include)
target_compile_definitions(${BBM_NAME} INTERFACE __HIP_PLATFORM_AMD__)
target_link_libraries(${BBM_NAME} INTERFACE ${BBM_HIP_LIBRARY} ${BBM_HIP_RUNTIME})
