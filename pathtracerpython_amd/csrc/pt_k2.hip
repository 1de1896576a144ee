// pt_k2.hip — the K2 kernel, k_render<false, false, false> (f32 filter, no
// counters, no BVH: the Cornell-box configurations and the bench line), in a
// translation unit of its own.  build.py compiles this unit with K2_FLAGS:
// LLVM's iterative ILP scheduler orders its unit loop for fewer dependency
// stalls (K2 -2.8%, the same instructions and frame), while it slows the BVH
// walk kernels of pt_hip.hip (+11-18%), which keep the default scheduler
// (DESIGN.md §11, round 6).
#include "pt_render.h"

#if PT_K2_OWN_TU
template __global__ void k_render<false, false, false>(SceneK, RenderK, void*, StatsDev*);
#endif
