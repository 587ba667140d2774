/*
 * rt.h — C ABI of the MI355X-native per-pixel render loop.
 *
 * This is the drop-in boundary for the reference's hot path
 * (keychera/raytracing-clj, Clojure, no FFI of its own). It replaces:
 *
 *   compute-pixel + the row-chunk executor   src/raytracing.clj:141-171
 *     └ ray-color (recursive bounce)         src/raytracing.clj:45-58
 *        └ hit-anything (closest-hit scan)   src/raytracing.clj:33-43
 *           └ sphere ::hit-fn                src/hittable.clj:7-31
 *        └ material ::scatter-fn             src/material.clj:13-46
 *           (lambertian :13-19, metal :21-28, dielectric :34-46)
 *        └ vec3a math + rand samplers        src/vec3a.clj:56-101
 *
 * Scene definition (raytracing.clj:63-78), camera set-up (:101-139) and the
 * PPM writer (:19-26, :172-175) stay on the host; helpers for them are
 * exported here too (rt_camera_setup, rt_quantize, rt_write_ppm) so a
 * Clojure/JNI, C++ or Python host can reuse them.
 *
 * Conventions: plain pointers and sizes, no ownership transfer (the library
 * never retains a caller pointer past the call), 0 = OK, negative = error
 * (see rt_status; message via rt_last_error(), thread-local).
 */
#ifndef RT_H
#define RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The library is built with -fvisibility=hidden: exactly the functions
 * declared here are exported. */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

/* ABI revision of this header (rt_abi_version() of the loaded library must
 * equal it; INTEGRATION.md lists the breaks).  3: rt_stats grew to 112 bytes
 * (set-up/enqueue/wait/scatter/other/D2H timers). */
#define RT_ABI_VERSION 3

/* ---- status codes ------------------------------------------------------ */
typedef enum rt_status {
  RT_OK = 0,
  RT_E_ARG = -1,        /* bad argument (NULL, size, range)                      */
  RT_E_MATERIAL = -2,   /* unsupported material kind                             */
  RT_E_TOO_MANY = -3,   /* sphere list larger than the LDS-resident limit        */
  RT_E_HIP = -4,        /* HIP runtime error (message has the HIP error string)  */
  RT_E_NODEV = -5,      /* no GPU visible / device index out of range            */
  RT_E_IO = -6,         /* file I/O (rt_write_ppm, rt_write_png, rt_ppm_to_png)  */
  RT_E_ALLOC = -7       /* host memory exhausted (the JNI shim's frame buffer)   */
} rt_status;

/* ---- material kinds: material.clj:13 (lambertian), :21 (metal), :34 (dielectric).
 * RT_NONE: a body merged with no material: ray-color finds no scatter-fn and
 * returns black (raytracing.clj:49-54). */
enum { RT_LAMBERTIAN = 0, RT_METAL = 1, RT_DIELECTRIC = 2, RT_NONE = 3 };

/* Maximum spheres per scene (LDS-resident sphere table, 16 B each). */
#define RT_MAX_SPHERES 8192

/* Maximum samples per pixel of one call (the pixel's fixed-point colour sums,
 * 2^-24 units per sample, stay below 2^64; larger counts: several calls with
 * sample_begin). */
#define RT_MAX_SPP (1 << 24)

/* ---- scene: the reference's `hittables` vector (raytracing.clj:63-78) -----
 * Bodies are tested in array order; on equal t the earlier body wins, exactly
 * as hit-anything's strict `root < closest-so-far` (raytracing.clj:35-42,
 * hittable.clj:17-23). */
typedef struct rt_scene {
  int n;                  /* number of bodies                                  */
  const float* sphere;    /* n x 4: center x,y,z, radius  (hittable.clj:7)     */
  const int* mat_kind;    /* n: RT_LAMBERTIAN | RT_METAL | RT_DIELECTRIC | RT_NONE */
  const float* mat;       /* n x 4: albedo r,g,b, then fuzz (metal) or
                             refraction index (dielectric); unused lanes 0     */
} rt_scene;

/* ---- camera: the values -main derives at raytracing.clj:117-139 ---------- */
typedef struct rt_camera {
  float center[3];        /* camera-center = look-from          (:126)          */
  float p00[3];           /* pixel-00-loc                       (:135)          */
  float du[3];            /* pixel-du                           (:129)          */
  float dv[3];            /* pixel-dv                           (:130)          */
  float disk_u[3];        /* defocus-disk-u                     (:138)          */
  float disk_v[3];        /* defocus-disk-v                     (:139)          */
  int defocus;            /* defocus-angle > 0                  (:147)          */
} rt_camera;

/* ---- render parameters -----------------------------------------------------
 * Pixel (i, j) of sample k gets its own RNG stream keyed by (seed, j*width+i,
 * sample_begin+k): results do not depend on tiling, device count or launch
 * shape.  spp / max_depth are the reference's CLI args (raytracing.clj:96-97).
 *
 * Output rows: the rendered rows are [row_begin, row_end).  With
 * tile_step == 0 they are written contiguously.  With tile_step > 0 the call
 * renders only the interleaved row tiles  tile_first, tile_first+tile_step,
 * ... (tile height row_tile, tiles counted from row_begin) and writes them
 * compacted, in order; rt_rows_out() gives the row count. */
typedef struct rt_params {
  int width, height;      /* full image; height = int(width/aspect) (:105-107) */
  int row_begin, row_end; /* global rows to render                             */
  int spp;                /* samples per pixel in this call                    */
  int max_depth;          /* ray-color depth budget                            */
  uint64_t seed;          /* RNG key                                           */
  int sample_begin;       /* first sample index (sample stripes), usually 0    */
  int n_devices;          /* rt_render fan-out: 0 = all visible devices        */
  int row_tile;           /* interleaved tile height (rows); 0 -> 8            */
  int tile_first;         /* rt_launch: first tile of this shard               */
  int tile_step;          /* rt_launch: tile stride (0 = contiguous rows)      */
  int flags;              /* 0, RT_FLAG_REALM, RT_FLAG_REJECTION_SAMPLERS,
                             RT_FLAG_SHARDS_ON_DEVICE0 (rt_render),
                             RT_FLAG_STREAMED (rt_launch), ored                 */
} rt_params;

/* rt_render: split into n_devices interleaved-tile shards exactly as for n
 * GPUs, but run every shard on device 0 (exercises the multi-GPU fan-out and
 * host gather on a one-GPU machine).  n_devices must be > 0. */
#define RT_FLAG_SHARDS_ON_DEVICE0 1

/* rt_launch / rt_render: the semantics of the reference's second namespace,
 * realm.raytracing (`clojure -M:realm`, src/realm/raytracing.clj) instead of
 * raytracing (`-M:main`): lambertian scatter without the near-zero fallback
 * (:137-143), dielectric without Schlick reflectance and its draw (:158-177),
 * and the pixel as sum * (1/spp) rather than sum / spp (:25, :276).  Its
 * camera (no defocus, focal length |lookfrom - lookat|) is an rt_camera like
 * any other (rt_camera_setup with defocus_angle 0). */
#define RT_FLAG_REALM 2

/* rt_launch only: the caller keeps launches of consecutive frames in flight
 * on two (or more) streams of the device, so the next frame's workgroups fill
 * the slots this launch's tail frees.  A launch of few tiles then splits its
 * tiles' samples for two rounds of workgroups instead of three (fewer, longer
 * sample pools: each pool's end idles lanes; the tail no longer waits alone).
 * Timing only: the bits never depend on it.  (tools/shard_time.py
 * --inflight; bench.py's frames in flight) */
#define RT_FLAG_STREAMED 4

/* rt_launch / rt_render: draw vec3a/random-unit-vec3 and random-in-unit-disk
 * by the reference's own rejection loops (vec3a.clj:74-86: three or two
 * uniforms per trip until the point falls inside the unit ball / disk).
 * Without the flag (the default) the kernel draws the same distributions
 * with a fixed number of draws -- uniform on the sphere as z = 2 xi1 - 1,
 * r = sqrt(1 - z^2), at the angle 2 pi xi2; uniform in the disk as
 * r = sqrt(xi1) at 2 pi xi2 -- so a wave no longer waits for its slowest
 * lane's rejection trips (C1 5.23 -> 4.75 ms per frame).
 * The reference's rand is unseeded, so either choice matches its renders
 * statistically (tests/test_oracle_pinning.py); each equals its own fp32
 * mirror in the oracle bit for bit.  Mixed within one frame never. */
#define RT_FLAG_REJECTION_SAMPLERS 8

/* ---- per-call statistics (device-side counters, host timers) ------------ */
typedef struct rt_stats {
  uint64_t segments;      /* hit-anything calls (raytracing.clj:48)            */
  uint64_t samples;       /* compute-pixel loop iterations (:142-154)          */
  double kernel_ms;       /* max over devices of the trace-kernel time         */
  double total_ms;        /* wall time of the whole call incl. H2D/D2H         */
  int n_devices;          /* devices used                                      */
  int scene_cached;       /* devices whose scene came from the library's cache */
  double upload_ms;       /* max over devices: the wait for the scene's upload +
                             BVH builds (a cache miss; they run beside the
                             render-context set-up, this is what is left)      */
  double gather_ms;       /* max over devices: D2H of the device's row tiles
                             into their rows of out_rgb (strided copies)       */
  double kernel_ms_mean;  /* mean over devices of the trace-kernel time
                             (load imbalance = kernel_ms / kernel_ms_mean)     */
  /* Where the wall time of the slowest device's share went (host clocks, in
   * order): setup_ms, upload_ms above, then the others; the rest of total_ms
   * (argument checks, thread fan-out and join) is other_ms.  A first call
   * shows its one-time costs here: setup_ms (events, device framebuffer,
   * pinned counters; a device's first context runs on its NULL stream, a
   * created stream costs 5-7 ms), upload_ms (what the scene upload and BVH
   * builds add beyond the set-up they run beside) and enqueue_ms (the first
   * launch loads the kernels' code object).                                  */
  double setup_ms;        /* render context set-up                             */
  double enqueue_ms;      /* rt_launch + D2H enqueue                           */
  double wait_ms;         /* host wait for the device: kernel + D2H            */
  double scatter_ms;      /* host scatter of row tiles: 0 since ABI 3's
                             strided copies place the rows                    */
  double other_ms;        /* total_ms - upload - setup - enqueue - wait - scatter */
  double d2h_ms;          /* max over devices: event-timed D2H of the frame    */
} rt_stats;

/* ========================= host-side helpers =========================== */

/* Camera basis exactly as -main computes it, in double, rounded to float at
 * the end (raytracing.clj:105-139; deg->rad :60-61).  vfov/defocus_angle in
 * degrees.  Viewport width uses image_width/image_height, not the aspect
 * ratio (:120). */
int rt_camera_setup(int image_width, int image_height, double vfov,
                    const double look_from[3], const double look_at[3],
                    const double vup[3], double defocus_angle,
                    double focus_dist, rt_camera* out);

/* write-color! per channel (raytracing.clj:19-26):
 * out = int(256 * clamp(c > 0 ? sqrt(c) : 0, 0, 0.999)); NaN -> 0.  n = channel count. */
int rt_quantize(const float* lin, uint8_t* out, size_t n);

/* PPM P3, one "r g b\n" per pixel, rows top->bottom (raytracing.clj:172-175). */
int rt_write_ppm(const char* path, const uint8_t* rgb, int width, int height);

/* PNG, 8-bit truecolour RGB, adaptive per-row filters, deflate: the same
 * pixels as rt_write_ppm (the format src/ppm2png.clj:35-87 converts to). */
int rt_write_png(const char* path, const uint8_t* rgb, int width, int height);

/* ppm->png (src/ppm2png.clj:35-87): read a P3 file (max value <= 255, w*h
 * pixels of 3 values) and write it as rt_write_png does.  RT_E_ARG on a
 * malformed PPM, RT_E_IO on file errors. */
int rt_ppm_to_png(const char* src_ppm, const char* dst_png);

/* Number of output rows a (row_begin,row_end,row_tile,tile_first,tile_step)
 * selection produces (0 on bad args). */
int rt_rows_out(const rt_params* p);

/* ---- scene builders (host) ----------------------------------------------
 * Both write up to `cap` bodies into sphere (x4), kind, mat (x4) and return
 * the body count (the needed count when the arrays are NULL / cap too small).
 *
 * rt_scene_reference: the reference's five bodies, in order
 *   (raytracing.clj:63-78): ground, center, left (glass), bubble, right (metal).
 * rt_scene_cover: the RTIOW "final render" cover scene (book §14; the
 *   reference has no such scene): ground r=1000, a
 *   (2*grid)^2 jittered field of r=0.2 bodies (80 % lambertian, 15 % metal,
 *   5 % glass; skipped within 0.9 of (4,0.2,0)), then three r=1 bodies.
 *   Deterministic in `seed` (splitmix64 stream, 53-bit doubles). */
int rt_scene_reference(float* sphere, int* kind, float* mat, int cap);
int rt_scene_cover(int grid, uint64_t seed, float* sphere, int* kind, float* mat, int cap);

/* ============================ rendering ================================ */

/* Render into a caller-owned host buffer of linear RGB fp32, row-major,
 * rows_out x width x 3, the mean over spp (compute-pixel's accum/spp,
 * raytracing.clj:155).  Fans out over p->n_devices GPUs inside the call
 * (a host worker per device from a persistent pool, interleaved row tiles,
 * each device's rows copied straight into their place; no collectives).  tile_first/tile_step must be 0 here.  stats may be NULL.
 *
 * The device copy of the scene (tables + BVHs) is cached per device by the
 * scene's content (a hash, then a byte compare): a repeated call with the
 * same bodies skips the upload and the BVH builds, and its launches reuse
 * the per-device stream whose adaptive tile order (rt_set_schedule) the
 * previous call recorded.  The library keeps copies, never caller pointers.
 * Output bits never depend on the cache. */
int rt_render(const rt_scene* s, const rt_camera* c, const rt_params* p,
              float* out_rgb, size_t out_len, rt_stats* stats);

/* rt_render, then rt_quantize on the device: out_rgb8 (rows_out x width x 3
 * bytes) holds exactly the bytes rt_quantize gives for rt_render's floats,
 * the write-color! bytes of the -main loop (raytracing.clj:160-175), at a
 * quarter of the copy back.  stats->d2h_ms includes the quantiser. */
int rt_render_u8(const rt_scene* s, const rt_camera* c, const rt_params* p,
                 uint8_t* out_rgb8, size_t out_len, rt_stats* stats);

/* ---- frames in flight: a host drawing a sequence of frames ---------------
 * rt_render_submit starts the frame rt_render would render -- the same
 * shards, scene cache, devices and bits -- and returns without waiting for
 * the devices; rt_render_wait blocks until the frame's rows are in out_rgb
 * (which the caller leaves alone until then), fills stats as rt_render does
 * and frees the frame.  Frames submitted before earlier ones are waited on
 * run concurrently: each frame in flight holds its own render context
 * (stream, device buffers) per device, and its launches split their tiles'
 * samples for two rounds of workgroups (RT_FLAG_STREAMED), so the next
 * frame's workgroups fill this one's tail.  Every submitted frame must be
 * waited on exactly once, from any thread.  (raytracing.clj:157-171's
 * executor hands its futures back the same way: submit, then .get in order.)
 * The _u8 form delivers rt_render_u8's bytes. */
typedef struct rt_frame rt_frame;
int rt_render_submit(const rt_scene* s, const rt_camera* c, const rt_params* p, float* out_rgb,
                     size_t out_len, rt_frame** frame);
int rt_render_submit_u8(const rt_scene* s, const rt_camera* c, const rt_params* p, uint8_t* out_rgb8,
                        size_t out_len, rt_frame** frame);
int rt_render_wait(rt_frame* frame, rt_stats* stats);

/* Drop rt_render's cached device scenes and render contexts (streams,
 * buffers; those not in use by a concurrent call).  Returns the number of
 * scenes dropped. */
int rt_cache_clear(void);

/* Device-resident path (inputs already in HBM; used by the benchmark). */
typedef struct rt_dscene rt_dscene;
int rt_scene_upload(int device, const rt_scene* s, rt_dscene** out);
int rt_scene_free(rt_dscene* ds);
/* Asynchronous: enqueue one trace launch on hip_stream (NULL = default
 * stream) of ds's device.  d_out: device buffer of rt_rows_out(p) x width x 3
 * floats.  d_counters: NULL or device u64[2] += {segments, samples}.
 * A launch of fewer 8 x 8 tiles than 3 x the workgroups the device holds at
 * once (a multi-GPU shard, a small frame) splits every tile's samples over
 * several workgroups; their integer pixel sums are added by a second kernel
 * on the same stream, from a scratch buffer the library keeps per scene and
 * stream (splits x rows x width x 3 x 8 bytes).  Bits never depend on it. */
int rt_launch(const rt_dscene* ds, const rt_camera* c, const rt_params* p,
              float* d_out, uint64_t* d_counters, void* hip_stream);

/* Asynchronous: enqueue rt_quantize on hip_stream's device for n channels
 * already in HBM (d_lin: n floats, d_out: n bytes, device pointers): the same
 * bytes as rt_quantize for every float (NaN, infinities and denormals
 * included), through a table of the 255 float thresholds between bytes that
 * the host derives from rt_quantize's own arithmetic. */
int rt_quantize_device(const float* d_lin, uint8_t* d_out, size_t n, void* hip_stream);

/* Kernel variant selector (all variants give identical bits).  The product
 * library holds: 0 = default (22 where it applies, else 16; when the 4-body
 * tree's LDS image would cap a CU below 5 workgroups and the 8-body tree's
 * is smaller: 26 where 22 applies and two of its 16-wave workgroups fit a
 * CU, else 24 where three of its 8-wave workgroups fit, else 18);
 * 16 = BVH traversal, 4 bodies per leaf, nodes and leaf bodies in LDS;
 * 18 = the same with 8 bodies per leaf, in 512-thread workgroups (one LDS
 * image per 8 waves); 22 = 16 in a compact LDS image (u8 node-index stack,
 * u32 pixel sums that count their wraps above 255 spp: seven workgroups per
 * CU; 0 selects it wherever spp < 65536, every albedo lies in [-1, 1], the
 * tree has <= 256 nodes and no frame side exceeds 65536, else 16); 24 = 22's
 * image in 512-thread workgroups (one per 8 waves; 16 where 22 does not
 * apply); 26 = the same in 1024-thread workgroups (8 waves per SIMD); 12 = BVH
 * with 2 bodies per leaf read from global memory (the fallback for a tree
 * too big for LDS); 5 = linear scan, bodies in groups of 4 through the
 * scalar cache (the fallback for a tree too deep for the stack).  The
 * diagnostic build lib/librtclj_diag.so (make diag) adds: 1 / 2 = simple
 * scan, table in LDS / scalar cache; 4 = grouped scan, table in LDS
 * (north_star's LDS-staged sphere list); 8 / 9 = packed-fp32 scan, LDS /
 * scalar; 11 = BVH in LDS, 2 bodies per leaf; 20 / 21 = direction-sorted
 * 8-wave lock-step workgroups (octant sort / live-path packing); and the
 * statistics builds 3, 6, 7, 10, 13, 17, 19 (= 1, 4, 5, 9, 11, 16, 18 with
 * wave-level counters, rt_debug_stats).  Returns the previous value, or
 * RT_E_ARG for a variant this build does not hold.  Applies to subsequent
 * launches in this
 * process (an atomic, read once per launch). */
int rt_set_variant(int variant);

/* The kernel variant the current selector resolves to for ds (the default
 * resolved for this scene, or a fallback when a tree does not fit), before
 * the per-launch choice of the compact image (16 -> 22, 18 -> 26 / 24), which also
 * depends on the launch (spp < 65536, frame size): rt_launch_occupancy's
 * out4[3] reports the variant a given launch runs.  For reading the matching
 * statistics build.  -1 on a NULL scene. */
int rt_resolve_variant(const rt_dscene* ds);

/* Occupancy of the launch rt_launch would make for (ds, p) under the current
 * selectors (diagnostic): out4 = {256-thread workgroups per CU (HIP occupancy
 * query with the launch's dynamic LDS), VGPRs per lane, LDS bytes per
 * workgroup, the variant}. */
int rt_launch_occupancy(const rt_dscene* ds, const rt_params* p, int* out4);

/* Tile dispatch order of rt_launch.  0 (default) = adaptive: every launch
 * adds how long each 8 x 8 pixel tile's waves ran to half the tile's earlier
 * record, and a one-block sort enqueued after it (same stream, no host sync)
 * turns that into a longest-first order; the next launch on the same scene and stream with the
 * same launch shape (width, row selection; camera, spp, seed, flags and the
 * kernel variant may differ) dispatches its tiles in that order, so the slow
 * tiles do not trail the kernel's end.  A launch of another shape runs in
 * plain order and re-keys the record (per scene, up to 8 streams; launches on
 * further streams are unscheduled).  1 = always plain order.  Changes timing
 * only: every pixel is computed the same way in any order (bit-identical
 * output).  Returns the previous value, RT_E_ARG for another mode. */
int rt_set_schedule(int mode);

/* Diagnostic counters of the stats variants (diagnostic build) since the
 * last call (then cleared), summed over devices, 32 values: [0] wave loop
 * iterations, [1] active lanes summed over them, [2] body tests per wave
 * (scan) / node visits per lane (BVH), [3] candidate blocks per wave (scan) /
 * leaf tests per lane (BVH), [4] lanes in candidate blocks / exact body
 * tests (BVH), [5] waves, [6] BVH wave-level traversal iterations, [7] lanes
 * active in them, [8..11] shader clocks per wave spent in camera sampling,
 * hit search, shading, accumulation (s_memtime; summed over waves), [12] BVH
 * wave-level leaf passes, [13] wave-level exact-test passes, [14] / [15]
 * wave-level trips of the random-unit-vec3 / defocus-disk rejection loops,
 * [16] / [17] wave-level camera-sample blocks / lanes in them, [18] executed
 * fp32 flops (per lane, fma = 2), [19] / [20] wave-level
 * dielectric shading blocks / lanes in them, [21] / [22] wave-level
 * lambertian-or-metal shading blocks / lanes in them, [23..31] 0.
 * Synchronises the devices. */
int rt_debug_stats(uint64_t* out32);

/* Diagnostic wave timeline of the stats variants' last launches on `device`
 * (of every variant's when the diagnostic build is loaded with
 * RTCLJ_TIMELINE=1):
 * n_waves x {start, end (s_memrealtime, 100 MHz), HW_ID, XCC_ID}; returns
 * the count. */
int rt_debug_waves(int device, uint64_t* out, size_t n_waves);

/* Sample stealing of rt_launch (diagnostic): the launches on (ds, hip_stream)
 * since the last call made out2[0] steals of out2[1] samples in all (a
 * workgroup that finds no tile left to start takes free samples of another
 * workgroup's tile).  Waits for the stream, then clears the
 * counts.  Timing only: the bits never depend on it. */
int rt_steal_stats(const rt_dscene* ds, void* hip_stream, uint64_t* out2);

/* Path export of rt_launch's split launches (diagnostic; RTCLJ_EXPORT=1):
 * out2[0] = the launches on (ds, hip_stream) since the last call that wrote
 * their waves' last paths out for a sweep launch, out2[1] =
 * the records the latest of them wrote.  Waits for the stream.  Timing
 * only: the bits never depend on it. */
int rt_export_stats(const rt_dscene* ds, void* hip_stream, uint64_t* out2);

/* A device's one-time start-up, done ahead of the first render so that a
 * one-frame process (-main, raytracing.clj:95-177) can overlap it with its
 * own work (rt_main starts it on a thread at process start): the device
 * context, the kernels' code object, the NULL stream's hardware queue and
 * the runtime's staging for pageable copies.  out_ms4 (nullable) = the
 * milliseconds of those four steps.  Idempotent; rt_render does the same
 * work lazily when it was not called. */
int rt_prepare(int device, double* out_ms4);

int rt_device_count(void);
const char* rt_last_error(void);
const char* rt_version(void);
int rt_abi_version(void);   /* RT_ABI_VERSION the library was built with */

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}
#endif
#endif /* RT_H */
