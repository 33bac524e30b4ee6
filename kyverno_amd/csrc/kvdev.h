// Device-side views of a compiled policy set and an ingested batch, shared by
// the HIP kernels (kvkernel.hip) and the host runtime (kvapi.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kv_layout.h"
#include "kvdevtypes.h"

namespace kv {

// Launch one pass over rules [rule_begin, rule_end) for every resource.
// P and B point to device-resident copies of the views (uniform scalar loads).
hipError_t launch_validate(const DevPS* P, const DevBatch* B, uint32_t n_res, const DevOut& O, uint32_t rule_begin,
                           uint32_t rule_end, hipStream_t stream);

}  // namespace kv
