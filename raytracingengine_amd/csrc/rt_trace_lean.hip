// rt_trace_lean.hip — the per-pixel trace kernels of rt_trace.hip compiled without triangle /
// BVH and area-light support (namespace rtamd::lean), for scenes that use neither: the generic
// kernels' register budget is set by their largest path, and these two are the largest.
#define RT_LEAN_GENERIC 1
#include "rt_trace.hip"
