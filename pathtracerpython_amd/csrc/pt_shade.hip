// pt_shade.hip — the wavefront path's shade step (k_wf_shade, pt_shade.h) in a
// translation unit of its own: build.py compiles it with LLVM's iterative ILP
// scheduler (its unit pass is the K2 kernel's), while the walk kernels of
// pt_hip.hip keep the default scheduler.
#define PT_SHADE_UNIT 1
#include "pt_shade.h"
