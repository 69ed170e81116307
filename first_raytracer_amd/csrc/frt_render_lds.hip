// The library's third translation unit: the lambertian path kernels of the
// octant LDS plan (C2), reached through frt_lds::path_oct (frt_render.hip
// "launch plans").  Built with the machine
// scheduler's max-memory-clause strategy (Makefile, LDSFLAGS); see the comment
// at kSplitLds.
#define FRT_TU_LDS 1
#undef FRT_DIAG
#ifndef FRT_RENDER_SRC
#define FRT_RENDER_SRC "frt_render.hip"
#endif
#include FRT_RENDER_SRC
