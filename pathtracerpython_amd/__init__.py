"""MI355X-native (gfx950) path tracer with the capabilities of
thiagoald/pathtracerpython's hot path: the per-pixel Monte-Carlo radiance
loop (main.py:186-280) runs as one HIP kernel behind a C-ABI (include/pt_capi.h),
while scene ingest keeps the reference's SDL/OBJ semantics (scene_reader).

    from pathtracerpython_amd import Scene, render
    fb = render(Scene("scenes/cornell/cornellroom.sdl"), 512, 512, spp=64, bounces=4)

Importing the package needs no GPU; the HIP library is loaded on first use
and there is no CPU fallback.
"""
from .scene_reader import Obj, Scene  # noqa: F401
from .render import Renderer, from_list_order, render, to_list_order  # noqa: F401
from .progressive import Checkpoint, render_progressive  # noqa: F401
from .utils import framebuffer_to_image, make_image, make_rays, make_screen_pts  # noqa: F401
