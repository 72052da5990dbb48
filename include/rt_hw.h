/* rt_hw.h — C ABI of the MI355X path-tracing core (librt_hw_amd.so).
 *
 * The reference (Korinin38/raytracing-hw) has no plugin API; its hot path is reached
 * through three C++ calls made by src/main.cpp:46-57.  Each entry point below replaces
 * one of them (plain pointers and sizes, no C++ or torch types, never throws):
 *
 *   rt_scene_load_gltf   <- parse_scene_gltf            src/io/scene_parser.cpp:25-350
 *                           + Scene::Scene (BVH build, light list)  src/core/scene.cpp:197-249
 *   rt_render / rt_render_device
 *                        <- Scene::render sample loop   src/core/scene.cpp:17-52
 *                           (per-pixel float RGB sums = sample_canvas, scene.cpp:20,42)
 *   rt_render_frame      <- the same loop over every GPU of the node (one row-block shard
 *                           per device), finished to 8 bits on each device and gathered
 *                           device-to-device onto one GPU (scene.cpp:17-64, canvas.h:76-89)
 *   rt_render_multi      <- the float frame of the same split (ABI 3 entry)
 *   rt_tonemap_u8        <- Scene::render frame finish  src/core/scene.cpp:54-64
 *   rt_tonemap_u8_device <- the same finish on the GPU   src/core/scene.cpp:54-64
 *   rt_write_ppm         <- Canvas::write_to            src/render/canvas.h:76-89
 *   rt_last_error        <- the reference's std::runtime_error messages (23 throw sites);
 *                           the host wrappers re-throw them (drop-in failure behaviour).
 *
 * RNG convention: pixel (i,j) runs minstd_rand seeded with j*W+i
 * (pixel 0 -> state 1) and a polar-normal cache reset at the pixel start, so output does
 * not depend on threads, GPUs or the pixel partition.
 *
 * Status codes: 0 = OK, < 0 = error (message in rt_last_error(), thread-local).
 */
#ifndef RT_HW_H
#define RT_HW_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 6   /* 6: RT_FLAG_POOL and RT_SCHED_POOL removed (the path pool, round 5) */

enum rt_status {
    RT_OK = 0,
    RT_ERR_ARG = -1,      /* bad argument / NULL pointer */
    RT_ERR_IO = -2,       /* file missing or unreadable */
    RT_ERR_FORMAT = -3,   /* glTF / image content not supported (reference throws the same) */
    RT_ERR_DEVICE = -4,   /* HIP runtime error or no device */
    RT_ERR_LIMIT = -5     /* scene exceeds a device limit (e.g. BVH deeper than the stack) */
};

typedef struct rt_scene rt_scene; /* opaque: host arrays + lazily uploaded device copies */

/* Read-only view of the flattened scene (the layout the kernels read from HBM).
 * Triangles and BVH nodes are in the reference's post-build order (bvh.cpp:166 reorders
 * `objects` in place), so object ids equal the reference's Intersection::object_id. */
typedef struct {
    int32_t width, height, samples, ray_depth; /* canvas, spp (scene_parser.cpp:16-22)   */
    float max_distance;                        /* camera zfar or 1e9 (scene_parser.cpp:119) */
    float cam_pos[3];                          /* camera.h position_                        */
    float cam_axes[9];                         /* right, up, forward (camera.h axes_)       */
    float cam_fov[2];                          /* fov_x, fov_y radians                      */
    float tan_half_fov[2];                     /* tanf(fov/2) as camera.cpp:51-52 computes  */
    uint32_t n_tris;
    const float *tri;       /* n_tris x 12: v0.xyz, U.xyz, V.xyz, geometric normal.xyz       */
    const float *tri_attr;  /* n_tris x 16: normal[3].xyz, texcoord[3].xy, mesh_id (int bits) */
    const float *tri_tan;   /* n_tris x 12: tangent[3].xyzw                                   */
    uint32_t n_nodes;
    const float *node;      /* n_nodes x 8: aabb min.xyz, max.xyz, a, b (int bits):
                               internal: a = left child (right = left+1), b = split_dim
                               leaf:     a = first primitive, b = 3 | count << 2           */
    uint32_t bvh_depth;     /* max root-to-leaf depth (root = 0)                            */
    uint32_t n_lights;
    const float *light;     /* n_lights x 16: v0.xyz, U.xyz, V.xyz, geo normal.xyz, area, 0,0,0
                               (ManyLightsDistribution objects, light-BVH order)          */
    uint32_t n_light_nodes;
    const float *light_node; /* same format as node */
    uint32_t light_bvh_depth;
    uint32_t n_meshes;
    const float *mesh_f;     /* n_meshes x 12: base_color.xyz, emission.xyz, metallic,
                                roughness2, alpha, ior, 0, 0                               */
    const int32_t *mesh_tex; /* n_meshes x 4: base_color_i, normal_i, metallic_roughness_i,
                                emission_i (-1 = none)                                     */
    const double *mesh_normal_transform; /* n_meshes x 16 (column-major matrix4d)          */
    uint32_t n_textures;
    const uint32_t *tex_info; /* n_textures x 4: texel offset, width, height, channels     */
    const uint8_t *texels;    /* RGBA8, all textures concatenated                          */
    uint64_t n_texel_bytes;
} rt_scene_view;

typedef struct {
    int32_t spp;          /* samples per pixel (0 = the scene's)                         */
    int32_t rank, world;  /* pixel-row partition: rows whose (row / row_block) % world == rank */
    int32_t row_block;    /* rows per interleave block (default 8)                       */
    int32_t count;        /* 1 = accumulate ray / AABB / triangle test counters          */
    int32_t kernel;       /* RT_KERNEL_LANE (0, default) or RT_KERNEL_WAVEFRONT (4)      */
    int32_t flags;        /* RT_FLAG_* */
    int32_t fast_chunk;   /* RT_FLAG_FAST: samples per work unit (0 = 2; raised so a pixel
                             has at most 128 units)                                      */
    int32_t device;       /* HIP device to render on (rt_render uploads the scene there;
                             rt_render_device needs rt_scene_upload(scene, device) first) */
} rt_params;

/* rt_params.kernel: two schedules of the same per-pixel arithmetic (same bits) */
#define RT_KERNEL_LANE 0       /* lane-resident persistent kernel (rt_mega.h)            */
#define RT_KERNEL_WAVEFRONT 4  /* wavefront: init / extend / shade launches (rt_wavefront.h) */

/* rt_params.flags */
#define RT_FLAG_KERNEL_TIMES 1  /* wavefront path (kernel 4): time every extend / shade launch (HIP events) */
/* Fast mode (kernel 0 only): every (pixel, sample) draws from its own
 * stream (Philox4x32-10 keyed by pixel j*W+i, counter = sample, seeds the sample's minstd
 * stream; normal cache empty per sample), so a pixel's samples are independent work units
 * of fast_chunk samples that any lane may run.  The pixel sum is the chunk partials added in
 * chunk order: deterministic for a given (spp, fast_chunk), statistically equivalent to the
 * reference, NOT bit-identical to it (the parity mode is the default). */
#define RT_FLAG_FAST 2
/* Light-split kernel (kernel 0, parity mode): the light pdf's light-BVH
 * walk as its own traversal state between two shading passes.  Same bits; measured slower
 * on every scene tried, so off by default. */
#define RT_FLAG_LIGHT_SPLIT 4
/* Parity mode at spp >= 128 renders pixels heaviest-first: a counting pre-pass of 1 sample
 * per pixel (its own Philox streams), a box filter, a radix sort and a spread over the
 * waves, all inside the call and inside render_ms.  Below 128 spp it renders in row-major
 * order (the pre-pass would cost more than it gains).  NATURAL_ORDER always renders in
 * row-major order, HEAVY_ORDER always builds the heaviest-first order; same bits either way,
 * and the two flags exclude each other (RT_ERR_ARG). */
#define RT_FLAG_NATURAL_ORDER 8
#define RT_FLAG_HEAVY_ORDER 32
/* Parity mode, once the pixel queue is empty, runs the next samples of a wave's unfinished
 * pixels on its idle lanes before their start state is known, and adds only those whose
 * start state is proven equal to the sequential chain's (rt_mega.h, speculative sample
 * runahead): same bits, shorter frame tail.  A shard of at most two pixels per resident lane
 * runs on the runahead kernel throughout; a larger one runs on the plain kernel, which hands
 * its sparse tail waves' pixels to the runahead kernel at a sample boundary (the hand-off:
 * schedule = RT_SCHED_LANE | RT_SCHED_RUNAHEAD).  This flag turns both off.  (Counting
 * renders, count = 1, never use it: their counters are those of the sequential chain.) */
#define RT_FLAG_NO_RUNAHEAD 16
/* Every defined flag; a call with any other bit set fails with RT_ERR_ARG (e.g. ABI 5's
 * RT_FLAG_POOL = 64, removed in ABI 6). */
#define RT_FLAG_ALL (RT_FLAG_KERNEL_TIMES | RT_FLAG_FAST | RT_FLAG_LIGHT_SPLIT | RT_FLAG_NATURAL_ORDER | \
                     RT_FLAG_NO_RUNAHEAD | RT_FLAG_HEAVY_ORDER)

typedef struct {
    uint64_t pixels;        /* pixels rendered by this call                               */
    uint64_t samples;       /* pixels x spp                                               */
    uint64_t rays;          /* scene closest-hit queries (calls of BVH::intersect)         */
    uint64_t aabb_tests;    /* AABB::intersect calls inside those queries                 */
    uint64_t tri_tests;     /* Primitive::intersect calls inside those queries            */
    uint64_t light_queries; /* BVH::intersectAll calls (light pdf)                        */
    uint64_t light_aabb_tests;
    uint64_t light_tri_tests;
    uint64_t shading_hits;  /* scene hits that were shaded (texture / attribute fetches)  */
    double render_ms;       /* device time of the whole render (order pre-pass included), HIP events;
                               rt_render_frame / _multi: the slowest device (its shards summed) */
    /* RT_FLAG_KERNEL_TIMES (wavefront path): summed launch durations and launch counts   */
    double extend_ms, shade_ms;
    uint64_t extend_launches, shade_launches;
    uint64_t extend_rays;   /* rays traced by the extend launches (always filled)          */
    double order_ms;        /* part of render_ms spent building the pixel order            */
    double gather_ms;       /* rt_render_frame / _multi: device-to-device copies of the slowest
                               device + assembly on the root device + the copy to the host  */
    uint64_t devices;       /* devices that rendered                                       */
    uint64_t schedule;      /* RT_SCHED_* bits of the kernels that rendered (ABI 5; for
                               rt_render_frame / _multi the union over the shards)          */
} rt_stats;

/* rt_stats.schedule bits: which instantiation of the sample loop ran */
#define RT_SCHED_LANE 1         /* lane-resident kernel (rt_mega.h), no runahead            */
#define RT_SCHED_RUNAHEAD 2     /* lane-resident kernel with speculative sample runahead
                                   (both bits: the plain kernel's tail handed to it)        */
#define RT_SCHED_FAST 4         /* fast mode (RT_FLAG_FAST)                                 */
#define RT_SCHED_LIGHT_SPLIT 8  /* light-split kernel (RT_FLAG_LIGHT_SPLIT)                 */
#define RT_SCHED_WAVEFRONT 16   /* wavefront launches (RT_KERNEL_WAVEFRONT)                 */

/* --- scene ------------------------------------------------------------------------ */
int rt_scene_load_gltf(const char *path, int32_t width, int32_t height, int32_t samples, rt_scene **out);
/* Builds a scene from already-flattened arrays (same layout as rt_scene_view; copied).
 * This is the seam for a host that keeps its own loader: e.g. the reference's parsed and
 * BVH-built `Scene` (scene.h:14-38) flattened field by field. */
int rt_scene_from_view(const rt_scene_view *view, rt_scene **out);
int rt_scene_get_view(const rt_scene *scene, rt_scene_view *view);
void rt_scene_free(rt_scene *scene);

/* --- render ----------------------------------------------------------------------- */
/* Copies the scene to `device` (once per device; later calls reuse it).  One render per
 * (scene, device) may be in flight at a time; different devices render independently. */
int rt_scene_upload(rt_scene *scene, int32_t device);
/* Number of pixels a (rank, world, row_block) shard owns, and their row-major order:
 * rows_out (may be NULL) receives the owned row indices, ascending. */
int64_t rt_shard_rows(int32_t height, int32_t rank, int32_t world, int32_t row_block, int32_t *rows_out);
/* Renders the shard into host memory: out_sum[k*W*3 + i*3 + c] for the k-th owned row. */
int rt_render(rt_scene *scene, const rt_params *params, float *out_sum, rt_stats *stats);
/* Same into device memory (d_out_sum on the scene's device, same layout) on HIP stream
 * `stream` (NULL = default stream); returns after the launch (asynchronous) unless
 * stats != NULL, in which case it waits and fills the counters and kernel time. */
int rt_render_device(rt_scene *scene, const rt_params *params, float *d_out_sum, void *stream, rt_stats *stats);
/* The whole frame on devices 0 .. n_devices-1 (n_devices <= 0: every visible device), one
 * host thread per device, device d rendering the shard (rank d, world n_devices,
 * params->row_block); params->rank / world / device are ignored.  out_sum: W*H*3 floats,
 * host memory, row-major.  Bits do not depend on n_devices. */
int rt_render_multi(rt_scene *scene, const rt_params *params, int32_t n_devices, float *out_sum, rt_stats *stats);
/* The whole frame as shards 0 .. n_shards-1 of a (world = n_shards, params->row_block) split,
 * shard r rendered on device devices[r] (devices NULL: device r; a device given several shards
 * renders them one after another).  Each shard is rendered and finished to 8 bits on its own
 * device (scene.cpp:54-64), then copied device-to-device (hipMemcpyPeerAsync, xGMI between
 * MI355X) to devices[0], which places the rows in frame order; the frame leaves the devices
 * in one copy per output.  out_rgb: W*H*3 bytes, the reference's canvas (canvas.h:76-89);
 * out_sum: W*H*3 floats (sample_canvas, scene.cpp:20,42); either may be NULL, not both.
 * params->rank / world / device are ignored.  Bits do not depend on n_shards or devices. */
int rt_render_frame(rt_scene *scene, const rt_params *params, int32_t n_shards, const int32_t *devices,
                    uint8_t *out_rgb, float *out_sum, rt_stats *stats);

/* Closest hit + light pdf for n explicit rays (BVH::intersect bvh.cpp:239-243 and
 * ManyLightsDistribution::pdf random.cpp:179-188; origin/dir as given to Ray::Ray, which
 * normalises dir).  Host arrays: org/dir n x 3; out_f n x 4 (t, u, v, light_pdf);
 * out_i n x 6 (hit, object id or -1, AABB tests, triangle tests, light AABB tests,
 * light triangle tests). */
int rt_intersect_rays(rt_scene *scene, int64_t n, const float *org, const float *dir, float *out_f, int64_t *out_i);

/* --- frame finish / output (host) ---------------------------------------------------- */
/* mean -> ACES -> powf(1/2.2) -> roundf(clamp(v*255)) per scene.cpp:54-64, vector.h:222-233, :400-407 */
int rt_tonemap_u8(const float *sum, int32_t width, int32_t height, int32_t spp, uint8_t *rgb_out);
/* The same finish on the device (current HIP device, asynchronous on `stream`): d_sum and
 * d_rgb are device pointers; bit-identical to rt_tonemap_u8 (the gamma quantizer is glibc
 * powf's, as exact thresholds). */
int rt_tonemap_u8_device(const float *d_sum, int32_t width, int32_t height, int32_t spp, uint8_t *d_rgb, void *stream);
/* "P6\n{W} {H}\n255\n" + raw RGB (canvas.h:76-89) */
int rt_write_ppm(const char *path, const uint8_t *rgb, int32_t width, int32_t height);

/* --- misc --------------------------------------------------------------------------- */
const char *rt_last_error(void);
int32_t rt_abi_version(void);
int32_t rt_device_count(void);
int rt_device_synchronize(void);
/* Device self-check of hardware-dependent arithmetic the kernels rely on for exactness
 * (no reference counterpart; test entry).  which 0: the traversal's fast reciprocal
 * (rt_wavefront.h rcp_ieee) against IEEE division over every float with a normal
 * reciprocal; which 1: the computed linear texel decode (rt_path.h unorm8) against
 * (float)b / 255.f for every byte, and the packed LDS RNG word round trip over every minstd
 * state and both normal-cache flags; which 2: the cooperative leaf step (rt_wavefront.h
 * trav_step_coop) against the per-lane in-order strict-< loop over 2^16 synthetic leaves rich
 * in equal-t ties, NaN and infinite vertices (four launches); *mismatches = values (cases)
 * that differ (0 = exact). */
int rt_device_selfcheck(int32_t which, uint64_t *mismatches);

#ifdef __cplusplus
}
#endif
#endif /* RT_HW_H */
