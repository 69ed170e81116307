// The library's fourth translation unit: the lambertian PSS-MLT chain kernels
// of the octant LDS plan (C5), reached through frt_lds::mlt_oct (frt_render.hip
// "launch plans").  Built with the machine scheduler's iterative-maxocc
// strategy (Makefile, CHAINFLAGS); see the comment at kSplitLds.
#define FRT_TU_CHAIN 1
#undef FRT_DIAG
#ifndef FRT_RENDER_SRC
#define FRT_RENDER_SRC "frt_render.hip"
#endif
#include FRT_RENDER_SRC
