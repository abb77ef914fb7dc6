// Private to the halo workload's translation units (halo*.cpp): shared includes and the box
// geometry helper every transport uses.
#pragma once

#include "workloads.hpp"

#include "core/numeric.hpp"
#include "core/util.hpp"
#include "hip/hip_runtime.hpp"
#include "hip/rccl_comm.hpp"

#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>

namespace tz {
namespace halo_detail {
/// the sub-box of direction d: interior slab facing d (ghost = false) or the ghost slab on
/// side d (ghost = true), in grid element offsets
kern::BoxDesc make_box(const HaloArgs &a, const HaloExchange::Dir &d, bool ghost, int64_t xoff,
                       int64_t sy, int64_t sz, int64_t sq);
/// the device-side wait limit of the transport preflights (seconds; preflight_limit_s)
inline double preflight_wait_s() { return preflight_limit_s(3.0); }
} // namespace halo_detail
using halo_detail::preflight_wait_s;
using halo_detail::make_box;
} // namespace tz
