// The library's second translation unit: every kernel compiled with a
// material set (MATS != kMatsNone), reached through frt_mats::pick /
// frt_mats::mlt (frt_render.hip "launch plans").  Built with the basic SGPR
// register allocator (Makefile, MATSFLAGS); see DESIGN.md "Register-cap hazard".
#define FRT_TU_MATS 1
#undef FRT_DIAG
#ifndef FRT_RENDER_SRC
#define FRT_RENDER_SRC "frt_render.hip"
#endif
#include FRT_RENDER_SRC
