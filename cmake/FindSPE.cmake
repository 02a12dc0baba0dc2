# Find the MI355X path engine (libspe + the topology shim libshdtopo), the way
# Shadow's cmake/FindIGRAPH.cmake finds igraph.  Hint: SPE_ROOT (an install
# prefix, or this repository after an in-tree build).
#
#   find_package(SPE REQUIRED)
#   include_directories(${SPE_INCLUDES})
#   target_link_libraries(shadow ... ${SHDTOPO_LIBRARIES} ${SPE_LIBRARIES})
#
# Defines SPE_FOUND, SPE_INCLUDES, SPE_LIBRARIES, SHDTOPO_LIBRARIES.
find_path(SPE_INCLUDES NAMES spe.h shd_topology_spe.h
          HINTS ${SPE_ROOT}/include $ENV{SPE_ROOT}/include)
find_library(SPE_LIBRARIES NAMES spe
             HINTS ${SPE_ROOT}/lib ${SPE_ROOT}/shadow_amd $ENV{SPE_ROOT}/lib $ENV{SPE_ROOT}/shadow_amd)
find_library(SHDTOPO_LIBRARIES NAMES shdtopo
             HINTS ${SPE_ROOT}/lib ${SPE_ROOT}/shadow_amd $ENV{SPE_ROOT}/lib $ENV{SPE_ROOT}/shadow_amd)
include(FindPackageHandleStandardArgs)
find_package_handle_standard_args(SPE DEFAULT_MSG SPE_INCLUDES SPE_LIBRARIES SHDTOPO_LIBRARIES)
mark_as_advanced(SPE_INCLUDES SPE_LIBRARIES SHDTOPO_LIBRARIES)
