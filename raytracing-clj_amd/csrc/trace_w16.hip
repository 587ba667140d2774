// trace_w16.hip — variant 26's kernel (trace_kernel.h: the compact 4-body
// image in 16-wave workgroups, 8 waves per SIMD), compiled on its own with
// the AMDGPU register-pressure trackers (raytracing-clj_amd/Makefile): the
// default scheduler holds it at 64 VGPRs by spilling three values to scratch
// (the thread index, a compaction slot address and the tile's row magic,
// 662 MB per C4 launch against 468 spill-free); the trackers fit it without.
#include "trace_kernel.h"

namespace rtclj {

const void* trace_kernel_w16() { return RT_KW(SRC_LDS, SCAN_BVHQ7, false, 16); }

}  // namespace rtclj
