// rt_wavefront.hpp — device arena of the breadth-first TraceRay (rt_wavefront.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "rt_internal.hpp"

namespace rtamd {

// Per-level ray counts and first node ids, written by the level kernels (device memory).
struct WfCtl {
    uint32_t count[kMaxDepth + 2];
    uint32_t base[kMaxDepth + 2];
    uint32_t lost;  // some sample's tree overflowed the arena (the fix-up pass has work)
    uint32_t dcount;  // deferred direct-lighting records of the inner levels (queue front)
    uint32_t dleaf;   // ... of the last shading level (queue back, filled backwards)
};

// Node ids [0, n0) are the roots (pixel samples, row-local pixel * aa + sample); deeper nodes
// are allocated level by level up to `cap`.  Structure-of-arrays, each component contiguous.
struct WfArena {
    double* val;      // 3 x cap: value of the node (local colour, then folded)
    double* fw;       // cap: refraction weight transparency·(1 − F)
    double* rw;       // cap: reflection weight
    double* ray;      // 6 x cap_r: origin xyz, direction xyz of node n0 + r
    int32_t* child;   // 2 x cap: refraction child id, reflection child id (−1: none)
    uint32_t* root;   // cap_r: root id of node n0 + r
    uint8_t* redo;    // n0: 1 = the tree of this root overflowed the arena
    // deferred direct lighting (the shadow stage): one record per hit node with transparency
    // < 1, appended by the level kernels — node id, hit code (primitive index | kind << 26 |
    // level << 28), hit distance — and shaded by wf_direct_kernel after the last level; the
    // last shading level's records fill the queue from the back
    uint32_t* dq_id;    // cap (null unless `defer`)
    uint32_t* dq_code;  // cap (null unless `defer`)
    double* dq_t;       // cap (null unless `defer`)
    WfCtl* ctl;
    uint32_t n0, cap, cap_r;
    bool defer;         // the arena holds the deferred-direct queue (wf_defer_selected())
};

// Whether refraction trees take the deferred direct-lighting pass (RTAMD_WF_DEFER=1; read per
// frame, tests switch it).  The arena is sized and laid out for the queue only then.
bool wf_defer_selected();
size_t wf_arena_bytes(size_t n0, size_t cap, bool defer);
WfArena wf_arena_layout(void* mem, size_t n0, size_t cap, WfCtl* ctl, bool defer);
hipError_t launch_wavefront(const TraceParams& p, int path, const WfArena& A, bool lds,
                            size_t lds_bytes, hipStream_t stream);
namespace lean {  // rt_wavefront_lean.hip: scenes without triangles / area light
hipError_t launch_wavefront(const TraceParams& p, int path, const WfArena& A, bool lds,
                            size_t lds_bytes, hipStream_t stream);
}

}  // namespace rtamd
