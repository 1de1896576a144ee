/*
 * pt_capi.h — C-ABI of the MI355X path-tracing library (libpt_hip.so).
 *
 * Drop-in boundary for the reference's per-pixel radiance loop
 * (/root/reference/main.py:186-271).  The reference has no native FFI: its
 * only operator seam is two Python callables handed to
 * multiprocessing.Pool.apply_async —
 *     intersect_objects(ray, objects, light_obj)      main.py:83, :200-201
 *     compute_color(scene, obj, point, normal)        main.py:142, :218-219
 * — driven by the spp x bounce loop of main.py:186-271.  This header replaces
 * that whole loop (pt_render*), and exposes the two callables as batched
 * entry points (pt_intersect_objects, pt_compute_color) so a caller can swap
 * them in one at a time.  Python binds it with ctypes
 * (pathtracerpython_amd/_native.py); INTEGRATION.md shows the binding.
 *
 * Conventions: plain C types only.  Return 0 on success, a negative
 * PT_E* code on failure; pt_last_error() gives a thread-local message.  Input
 * arrays are caller-owned and read-only; the library copies what it needs to
 * device memory at pt_scene_create.  Output buffers are caller-allocated.
 * A pt_scene handle is not re-entrant (one call at a time per handle); the
 * library orders the launches made on one handle (each waits on the GPU for
 * the previous one, whatever stream either was issued on), because they share
 * the handle's device scratch.
 */
#ifndef PT_CAPI_H
#define PT_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_API_VERSION 7

/* error codes */
#define PT_OK 0
#define PT_EINVAL (-1)     /* bad argument (shape, range, null pointer) */
#define PT_EHIP (-2)       /* HIP runtime error */
#define PT_ENOMEM (-3)     /* device or host allocation failed */
#define PT_ENODEV (-4)     /* no usable gfx950 device */
#define PT_EUNSUPPORTED (-5) /* pt_obj_load: input outside the fast reader's subset */
#define PT_ETIMEOUT (-6)   /* pt_wait_flags: the flags did not arrive in time */

/* pt_render flags */
#define PT_FLAG_RR (1u << 0)           /* Russian roulette (build extension) */
#define PT_FLAG_FORCE_F64 (1u << 1)    /* send every intersection test to the
                                          f64 evaluator (self-check mode) */
#define PT_FLAG_COUNT (1u << 2)        /* fill pt_stats counters (slower) */
#define PT_FLAG_OUT_F64 (1u << 3)      /* framebuffer elements are float64
                                          (default float32)              */
#define PT_FLAG_MEGAKERNEL (1u << 4)   /* scenes with a BVH: render with the
                                          single kernel instead of the
                                          wavefront kernels (same result) */
#define PT_FLAG_WALK_COUNT (1u << 5)   /* wavefront renders (BVH scenes): count
                                          the walks' queries, node visits and
                                          leaf-unit tests into pt_stats
                                          (counting kernels; synchronous)  */
#define PT_FLAG_KERNEL_TIMES (1u << 6) /* wavefront renders: per-kernel HIP-event
                                          times into pt_stats (synchronous; the
                                          two walks of a step run one after the
                                          other, so each time is its own)   */
/* bit 7: reserved (v4's PT_FLAG_TREE_WALK, retired in v5 with the grid-walk
   experiment it selected against; the library rejects it)                */
#define PT_FLAG_RESERVED7 (1u << 7)

/*
 * Flattened scene, as produced by scene_reader.Scene
 * (/root/reference/scene_reader.py:107-188).  Triangles are ordered exactly
 * as the reference iterates them in intersect_objects (main.py:91-96):
 * every object's triangles in scene order, then the light's triangles.
 */
typedef struct pt_scene_desc {
    int32_t n_tri;           /* all triangles (objects + light)               */
    int32_t n_obj_tri;       /* leading triangles that belong to objects      */
    int32_t n_obj;           /* objects (materials); light has index n_obj    */
    int32_t reserved;
    const double* tri_v;     /* [n_tri][3][3] vertices v1,v2,v3 as read       */
    const double* tri_n;     /* [n_tri][3] Obj.normals (scene_reader.py:5-8)  */
    const double* tri_area;  /* [n_tri]    Obj.areas  (vector.py:164-165)     */
    const int32_t* tri_obj;  /* [n_tri] object index; light triangles: n_obj  */
    const double* mat;       /* [n_obj][8] red green blue ka kd ks kt n       */
    double eye[3];           /* Scene.eye       scene_reader.py:151-152       */
    double ortho[4];         /* Scene.ortho     x0 y0 x1 y1                   */
    double ambient;          /* Scene.ambient                                 */
    double light_rgb[3];     /* Scene.light_color                             */
} pt_scene_desc;

/* Render parameters.  Pixel k = ix*height + iy is the reference's list order
 * (utils.py:64-69).  Rows: a launch renders the image rows iy with
 * row_begin <= iy < row_end and iy % row_step == row_phase, which covers
 * contiguous bands (row_step 1) and the interleaved bands used for
 * multi-GPU balance.  Output: image orientation, float32 (float64 with
 * PT_FLAG_OUT_F64) out[(height-1-iy)][ix][3] restricted to the launched rows,
 * in launch order (see pt_band_rows), one output row every out_row_stride
 * elements (0: packed, width*3) — a band can be written straight into its
 * rows of a whole frame (out = the frame's row of the band's top iy, stride =
 * row_step*width*3).  Values are the averaged radiance before make_image's
 * min-max normalisation (main.py:274-280).
 *
 * lanes_per_pixel: 0 lets the library choose the work-items per pixel of the
 * launch (from the launch's size and the device: one rank's band of an N-GPU
 * split gets more lanes per pixel than the whole frame); a power of two
 * <= min(64, spp) fixes it.  A pixel's samples are summed in an order that
 * follows its lane count, so two launches covering a pixel give bit-identical
 * values when they use the same lanes_per_pixel, and values within ~1e-15
 * relative of each other otherwise.                                        */
typedef struct pt_render_params {
    int32_t width, height;
    int32_t spp;             /* main.py -r                                     */
    int32_t bounces;         /* main.py -b                                     */
    uint64_t seed;           /* RNG key (SDL `seed`, unused by the reference) */
    uint32_t flags;          /* PT_FLAG_*                                      */
    int32_t rr_depth;        /* first bounce that may be terminated by RR     */
    int32_t row_begin, row_end, row_step, row_phase;
    int32_t sample_begin;    /* first sample index (spp-split renders)        */
    int32_t out_row_stride;  /* elements between output rows (0: width*3)     */
    int32_t lanes_per_pixel; /* 0: chosen per launch; else fixed (see above)  */
    int32_t reserved;        /* 0 */
} pt_render_params;

/* Work counters (PT_FLAG_COUNT); reference-semantics test counts are those
 * the reference loop would execute (shadow rays stop at the first occluding
 * object, main.py:42-55).                                                   */
typedef struct pt_stats {
    uint64_t closest_tests;   /* intersect calls of intersect_objects        */
    uint64_t shadow_tests;    /* intersect calls of compute_shadow_rays      */
    uint64_t ray_bounces;     /* non-None rays traced                        */
    uint64_t shading_points;  /* compute_color calls                         */
    uint64_t light_hits;
    uint64_t escapes;
    uint64_t f64_fallbacks;   /* single tests re-evaluated in f64 (filter)   */
    uint64_t f64_rescans;     /* closest-hit queries re-run fully in f64     */
    /* PT_FLAG_WALK_COUNT (wavefront renders of BVH scenes): the walk kernels'
     * work — queries taken, 4-wide node visits, BVH leaf units tested      */
    uint64_t shadow_queries, shadow_node_visits, shadow_leaf_units;
    uint64_t closest_queries, closest_node_visits, closest_leaf_units;
    /* PT_FLAG_KERNEL_TIMES (wavefront renders): summed HIP-event time (ms)
     * and launch count of each wavefront kernel                            */
    double shade_ms, shadow_ms, closest_ms;
    uint64_t shade_launches, shadow_launches, closest_launches;
    /* (v7) the shadow list's counting sort between the shade and the shadow
     * walks (its four kernels per step) */
    double sort_ms;
    uint64_t sort_launches;
} pt_stats;

typedef struct pt_scene pt_scene;

int pt_api_version(void);
const char* pt_last_error(void);
/* Content hash (16 hex digits) of the sources the library was compiled from
 * (the .h and .hip files of csrc/ and this header; pathtracerpython_amd/build.py).  The
 * Python binding refuses a library whose id is not the hash of the sources on
 * disk, and measurements name the loaded library's id.  (v6) */
const char* pt_build_id(void);

/* number of HIP devices visible to the library */
int pt_device_count(int32_t* count);

/* Upload a scene to the current HIP device.  Replaces Scene(path)'s role as
 * the thing the workers receive by pickle (main.py:201, :219). */
int pt_scene_create(const pt_scene_desc* desc, pt_scene** out);
/* Same, on HIP device `device` (the current device is left unchanged). */
int pt_scene_create_on(const pt_scene_desc* desc, int32_t device, pt_scene** out);
void pt_scene_destroy(pt_scene* scene);

/* Number of rows a launch with these params renders. */
int pt_band_rows(const pt_render_params* p, int32_t* rows);

/* Whole loop main.py:186-280 for the selected rows.  out_rgb_dev is a DEVICE
 * pointer (rows*width*3 float32, or float64 with PT_FLAG_OUT_F64), written on
 * `stream` (a hipStream_t, or NULL for the null stream).  Asynchronous unless
 * stats are requested with PT_FLAG_COUNT; pt_last_kernel_ms() reads the
 * HIP-event time of the most recent launch. */
int pt_render_device(pt_scene* scene, const pt_render_params* p,
                     void* out_rgb_dev, void* stream, pt_stats* stats);

/* Same, synchronous, with a host output buffer (rows*width*3 elements, or
 * rows rows of out_row_stride elements). */
int pt_render(pt_scene* scene, const pt_render_params* p, void* out_rgb_host,
              pt_stats* stats);

/* Several GPUs from one process (SURVEY.md §8(b) pt_render_multi; the
 * reference's only parallelism is its process pool over rays,
 * main.py:197-231).  scenes[i] is a handle of the same scene created on its
 * own device (pt_scene_create_on).  The rows row_begin <= iy < row_end of p
 * (p->row_step must be 1) are dealt out interleaved: handle i renders the
 * rows with (iy - row_begin) % n == i, all devices concurrently, and each
 * band is copied with one strided device-to-host copy straight into its rows
 * of out_rgb_host ((row_end-row_begin) x width x 3, the layout pt_render
 * writes for the whole range; p->out_row_stride must be 0).  Bit-identical to
 * pt_render of the same range on one device when p->lanes_per_pixel is set
 * (the same value for both); with 0 each band's launch chooses its own
 * lanes per pixel and values agree to ~1e-15 relative (see
 * pt_render_params).  Synchronous.  On an error the devices already launched
 * are drained before it returns, so the handles and out_rgb_host are free
 * for reuse.  stats (optional) receives the per-device sums of every field
 * (PT_FLAG_COUNT / PT_FLAG_WALK_COUNT / PT_FLAG_KERNEL_TIMES renders then run
 * one device at a time). */
int pt_render_multi(pt_scene* const* scenes, int32_t n, const pt_render_params* p,
                    void* out_rgb_host, pt_stats* stats);

/* Kernel time (ms) of the last pt_render_device launch on this handle. */
int pt_last_kernel_ms(pt_scene* scene, float* ms);

/* Batched replacement of intersect_objects (main.py:83-122).
 * rays: [n][6] f64 (origin, direction — direction need not be normalised).
 * out_tri [n]: closest triangle index or -1 (None); out_p [n][3]: hit point.
 * The light flag of the reference is out_tri >= n_obj_tri. */
int pt_intersect_objects(pt_scene* scene, const double* rays, int64_t n,
                         int32_t* out_tri, double* out_p);

/* Batched replacement of compute_color (main.py:142-145 + :23-80) with the
 * 12 light-sampling uniforms given explicitly per point (slots 0..11).
 * obj [n]: object index; point [n][3]; normal [n][3]; u [n][12];
 * out_rgb [n][3] f64. */
int pt_compute_color(pt_scene* scene, const int32_t* obj, const double* point,
                     const double* normal, const double* u, int64_t n,
                     double* out_rgb);

/* Frame assembly after the multi-GPU gather (replaces the
 * reference's collection of Pool results, main.py:224-231): tiles_dev is the
 * gathered (world, max_rows, width, 3) array whose band r is what
 * pt_render_device writes for row_step = world, row_phase = r over the whole
 * image (rows iy % world == r, top-first; max_rows >= ceil(height / world));
 * out_dev receives the (height, width, 3) framebuffer in image orientation.
 * Elements are float32, or float64 with PT_FLAG_OUT_F64 in flags.
 * Asynchronous on `stream`. */
int pt_assemble_bands_device(const void* tiles_dev, int32_t world, int32_t max_rows,
                             int32_t width, int32_t height, uint32_t flags, void* out_dev,
                             void* stream);

/* Host frames (the metric's framebuffer ends in host
 * memory; §8(e): the N ranks' bands make one frame).  The reference collects
 * the pool workers' colours into the parent's list through pipes
 * (main.py:204, :224-231); here each GPU writes its band straight into its
 * rows of one frame in page-locked host memory — shared by the rank
 * processes of one node (e.g. a /dev/shm mapping) — through a band render
 * with out = pt_host_map's device address of the band's first row and
 * out_row_stride = row_step*width*3, so the framebuffer crosses PCIe while the
 * kernel runs, each GPU over its own link.  Completion is a flag per rank in
 * the same memory: pt_signal writes it on the render's stream after the
 * render (system-scope release, so the band's stores are visible first), the
 * consumer waits for all flags with pt_wait_flags.
 *
 * pt_host_map page-locks [host, host+bytes) (caller-owned, page-aligned, e.g.
 * an mmap) for every device of the process and returns the address kernels
 * use for it; pt_host_unmap releases it (after the work using it is done). */
int pt_host_map(void* host, uint64_t bytes, void** dev_ptr);
int pt_host_unmap(void* host);
/* After all work queued on `stream` so far: *flag_dev = value (64-bit store,
 * system scope, release).  flag_dev: a pt_host_map address or device memory. */
int pt_signal(uint64_t* flag_dev, uint64_t value, void* stream);
/* Host: spin until flags[i * stride] >= value for i < n (relaxed loads, then
 * an acquire fence), or PT_ETIMEOUT after timeout_s seconds. */
int pt_wait_flags(const uint64_t* flags, int32_t n, int32_t stride, uint64_t value, double timeout_s);

/* Image finalisation of make_image (utils.py:150-161) on the device:
 * global min over the whole height x width x 3 array, shift, divide by the
 * shifted maximum, x255, truncate to uint8 — in f64, as numpy does (a NaN
 * anywhere, or a constant image, gives 0s like numpy's cast on x86).
 * fb: a full framebuffer as pt_render* writes it (image orientation, f32, or
 * f64 with PT_FLAG_OUT_F64 in flags); out: height*width*3 uint8 in the same
 * layout, which is make_image's array for the square images the reference
 * supports (for width != height its placement, utils.py:154-156, indexes out
 * of range).  The _device form is asynchronous on `stream`. */
int pt_image_u8_device(const void* fb_dev, int32_t width, int32_t height, uint32_t flags,
                       void* out_u8_dev, void* stream);
int pt_image_u8(const void* fb_host, int32_t width, int32_t height, uint32_t flags,
                uint8_t* out_u8_host);

/* Native OBJ reader (host only, no GPU needed) with the semantics of the
 * reference's Obj (scene_reader.py:49-104, vector.py:143-173): comment and
 * token rules, `v` / `f` records, negative indices, fan triangulation, and
 * the per-triangle normal and area computed in the reference's operation
 * order (bit-identical doubles).  Other commands are skipped; their raw line
 * byte ranges are returned so a caller can report them as the reference
 * prints them.  Returns PT_EUNSUPPORTED for inputs it does not mirror byte
 * for byte (e.g. "1/2/3" face tokens, hex or underscore numbers, vertices
 * with other than 3 coordinates, out-of-range indices, a zero-area
 * triangle): the caller then falls back to the Python reader, which raises
 * what the reference raises.  The mesh is owned by the library until
 * pt_mesh_free. */
typedef struct pt_mesh {
    int64_t n_vert, n_tri, n_skip;
    const double* vert;       /* [n_vert][3] */
    const int64_t* face;      /* [n_tri][3] vertex indices as Obj.faces holds them */
    const double* tri_v;      /* [n_tri][3][3] */
    const double* tri_n;      /* [n_tri][3] */
    const double* tri_area;   /* [n_tri] */
    const int64_t* skip_off;  /* [n_skip] byte offset of each skipped line */
    const int64_t* skip_len;  /* [n_skip] its length */
} pt_mesh;
int pt_obj_load(const char* path, pt_mesh** out);
void pt_mesh_free(pt_mesh* mesh);

/* Test hook (v6): the next pt_render_multi calls fail with PT_EHIP while
 * dealing band `multi_band`, after bands 0..multi_band-1 were launched (the
 * error path's drain); -1 (the default) turns it off.  Process-wide. */
int pt_test_fault_inject(int32_t multi_band);

#ifdef __cplusplus
}
#endif
#endif /* PT_CAPI_H */
