// rt_wavefront_lean.hip — the breadth-first TraceRay kernels of rt_wavefront.hip compiled without
// triangle / BVH and area-light support (namespace rtamd::lean), for scenes that use neither.
#define RT_LEAN_GENERIC 1
#include "rt_wavefront.hip"
