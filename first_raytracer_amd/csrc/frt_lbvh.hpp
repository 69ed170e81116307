// frt_lbvh.hpp -- GPU BVH builders (frt_lbvh.hip: PLOC, linear BVH), internal to libfrt.so.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <string>

namespace frt {
// n >= 2 primitive boxes (box6: lo xyz, hi xyz per prim, fp32 rounded outward)
// -> n-1 internal nodes: child2 (internal index >= 0 or ~sorted leaf position),
// node_box6 (per internal node), order (sorted leaf position -> prim index),
// ms = device time of the build passes.  Runs on `st` (current device).
// Returns 0, or -1 with `err` set.
// algo: kGpuBvhPloc (PLOC clustering, the default), kGpuBvhLbvh (Karras) or
// kGpuBvhSah (top-down binned SAH; leaves are prims, `order` the identity).
constexpr int kGpuBvhPloc = 0, kGpuBvhLbvh = 1, kGpuBvhSah = 2;
int lbvh_build(hipStream_t st, int n, const float *box6, int32_t *child2, float *node_box6, int32_t *order, float *ms,
               std::string &err, int algo = kGpuBvhPloc);
}  // namespace frt
