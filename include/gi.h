/*
 * gi.h -- C-ABI drop-in boundary of the MI355X-native photon-mapping renderer.
 *
 * Plain C: pointers, sizes and POD structs only (no C++ / torch types). One context owns one
 * HIP device, the uploaded scene, the photon maps (device-resident) and all scratch buffers.
 * Calls are synchronous and NOT re-entrant per context. Errors are integer status codes; the
 * library never calls exit(); the message of the last failure is returned by gi_last_error().
 *
 * Each entry point names the reference interface it replaces (ReillyBova/Global-Illumination,
 * paths relative to src/):
 *
 *   gi_parse_args           ParseArgs             utils/io_utils.cpp:16-212 (flag set, defaults
 *                                                  photonmap.cpp:27-106)
 *   gi_read_scene           ReadScene / R3Scene::ReadFile (.scn Princeton + .off)
 *                                                  utils/io_utils.cpp:219-250,
 *                                                  R3Graphics/R3Scene.cpp:514-587, 1462-1953
 *   gi_map_photons          static void MapPhotons(void)           photonmap.cpp:260-436
 *   gi_render_image         R2Image *RenderImage(int aa,int w,int h) render.cpp:155-259
 *   gi_render_tiles         the column interleave of Threadable_RayTracer (render.cpp:90)
 *                           re-cut as an image-tile shard for multi-GPU ranks
 *   gi_estimate_radiance_batch   EstimateRadiance(...)     utils/photon_utils.cpp:72-162
 *   gi_knn_batch            R3Kdtree<Photon*>::FindClosestQuick  R3Shapes/R3Kdtree.cpp:688-848
 *   gi_intersect_batch      R3Scene::Intersects(ray, ...)        R3Graphics/R3Scene.cpp:471-479
 *   gi_write_image          WriteImage / R2Image::Write (png: row flip R2Image.cpp:1430, ppm)
 *
 * The photon record is the exchange format of the photon maps (20 B; on device it is split
 * into a 16-B position stream and a 4-B RGBE stream, DESIGN.md "Data layout"): positions are fp32 (reference: fp64 R3Point,
 * render.h:17-21), power in Ward RGBE (as the reference), direction as the reference's
 * 8+8-bit spherical code (photon_utils.cpp:56-60).
 */
#ifndef GI_H
#define GI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------------------- */
enum {
  GI_OK = 0,
  GI_ERR_ARG = 1,         /* bad argument / flag (reference: "Invalid program argument", exit 1) */
  GI_ERR_IO = 2,          /* scene / image file error (reference: exit(-1)) */
  GI_ERR_HIP = 3,         /* HIP runtime failure */
  GI_ERR_STATE = 4,       /* call out of order (e.g. render before scene) */
  GI_ERR_UNSUPPORTED = 5, /* feature not available on the device path */
  GI_ERR_ALLOC = 6        /* device / host allocation failure */
};

enum { GI_FILTER_DISK = 0, GI_FILTER_CONE = 1, GI_FILTER_GAUSS = 2 }; /* render.h Filter_Type */
enum { GI_MAP_GLOBAL = 0, GI_MAP_CAUSTIC = 1 };                      /* render.h Photon_Type */

/* ---- parameters: one field per reference global (photonmap.cpp:40-106, render.h:27-81) -- */
typedef struct gi_params {
  int32_t verbose;              /* VERBOSE                        -v            */
  int32_t threads;              /* THREADS (host CPU threads)     -threads N    */
  int32_t fresnel;              /* FRESNEL                        -no_fresnel   */
  int32_t ambient;              /* AMBIENT                        -no_ambient   */
  int32_t direct_illum;         /* DIRECT_ILLUM                   -no_direct    */
  int32_t transmissive_illum;   /* TRANSMISSIVE_ILLUM             -no_transmissive */
  int32_t specular_illum;       /* SPECULAR_ILLUM                 -no_specular  */
  int32_t indirect_illum;       /* INDIRECT_ILLUM                 -no_indirect  */
  int32_t caustic_illum;        /* CAUSTIC_ILLUM                  -no_caustic   */
  int32_t direct_photon_illum;  /* DIRECT_PHOTON_ILLUM            -photon_viz   */
  int32_t fast_global;          /* FAST_GLOBAL                    -fast_global  */
  int32_t irradiance_cache;     /* IRRADIANCE_CACHE               -cache        */
  int32_t shadows;              /* SHADOWS                        -no_shadow    */
  int32_t soft_shadows;         /* SOFT_SHADOWS                   -no_ss        */
  int32_t light_test;           /* LIGHT_TEST                     -lt N         */
  int32_t shadow_test;          /* SHADOW_TEST                    -ss N         */
  int32_t monte_carlo;          /* MONTE_CARLO                    -no_monte     */
  int32_t max_monte_depth;      /* MAX_MONTE_DEPTH                -md N         */
  int32_t recursive_shadows;    /* RECURSIVE_SHADOWS              -no_rs        */
  int32_t distrib_transmissive; /* DISTRIB_TRANSMISSIVE           -no_dt        */
  int32_t transmissive_test;    /* TRANSMISSIVE_TEST              -tt N         */
  int32_t distrib_specular;     /* DISTRIB_SPECULAR               -no_ds        */
  int32_t specular_test;        /* SPECULAR_TEST                  -st N         */
  int32_t depth_of_field;       /* DEPTH_OF_FIELD                 -dof N D R    */
  int32_t dof_test;             /* DOF_TEST                                     */
  int32_t global_photon_count;  /* GLOBAL_PHOTON_COUNT            -global N     */
  int32_t caustic_photon_count; /* CAUSTIC_PHOTON_COUNT           -caustic N    */
  int32_t max_photon_depth;     /* MAX_PHOTON_DEPTH               -pd N         */
  int32_t indirect_test;        /* INDIRECT_TEST                  -it N         */
  int32_t global_estimate_size; /* GLOBAL_ESTIMATE_SIZE           -gs N         */
  int32_t global_filter;        /* GLOBAL_FILTER                  -gf cone K | gauss */
  int32_t caustic_estimate_size;/* CAUSTIC_ESTIMATE_SIZE          -cs N         */
  int32_t caustic_filter;       /* CAUSTIC_FILTER                 -cf cone K | gauss */
  int32_t gpus;                 /* extension: devices of the drop-in CLI (-gpus N); 0/1 = one */
  double ir_air;                /* IR_AIR                         -ir F         */
  double prob_absorb;           /* PROB_ABSORB                    -absorb F     */
  double focus_depth;           /* FOCUS_DEPTH                                  */
  double aperture_radius;       /* APERTURE_RADIUS                              */
  double global_estimate_dist;  /* GLOBAL_ESTIMATE_DIST           -gd F         */
  double caustic_estimate_dist; /* CAUSTIC_ESTIMATE_DIST          -cd F         */
  double filter_const_a;        /* FILTER_CONST_A (0.918)                       */
  double filter_const_b;        /* FILTER_CONST_B (1.953)                       */
  double filter_const_k;        /* FILTER_CONST_K                               */
  uint64_t seed;                /* extension: RNG seed (-seed S); reference RNG is unseeded */
} gi_params;

/* ---- photon record (exchange format, 20 bytes; device layout is SoA) -------- */
typedef struct gi_photon {
  float pos[3];       /* hit point, fp32 (reference: R3Point fp64)            */
  uint8_t rgbe[4];    /* Ward RGBE power (graphics_utils.cpp:50-77)           */
  uint16_t dir;       /* phi*256+theta travel direction (photon_utils.cpp:56) */
  uint16_t flags;     /* reserved (0)                                         */
} gi_photon;

/* ---- EstimateRadiance test-seam query (photon_utils.h:32-35 argument list) ------------- */
typedef struct gi_radiance_query {
  double point[3];
  double normal[3];
  double exact_bounce[3];
  double cos_theta;
  double kd[3];        /* brdf->Diffuse()   */
  double ks[3];        /* brdf->Specular()  */
  double shininess;    /* brdf->Shininess() */
  double max_dist;     /* estimate_dist     */
  int32_t k;           /* estimate_size     */
  int32_t filter;      /* GI_FILTER_*       */
} gi_radiance_query;

typedef struct gi_photon_stats {
  int64_t global_stored, caustic_stored;
  int64_t global_emitted, caustic_emitted;
  /* trace_s: emission rounds + power rescale; kd_s: kd builds and the k-NN kernels' per-photon
   * K-th distance bound pass; irradiance_s: the -cache pass and replication over a device set */
  double total_s, trace_s, kd_s, irradiance_s;
} gi_photon_stats;

/* Counters mirror the -v report of render.cpp:224-255 */
typedef struct gi_render_stats {
  uint64_t screen_rays, shadow_rays, monte_carlo_rays, transmissive_samples;
  uint64_t specular_samples, indirect_samples, caustic_samples;
  uint64_t knn_queries, knn_photons;   /* sum over queries of photons returned */
  uint64_t knn_visited;                /* photons distance-tested by the k-NN search */
  double render_s;                     /* wall time of the render phase       */
  double knn_kernel_ms;                /* summed k-NN kernel time (HIP events) */
  double knn_kernel_launches;
  /* the same split per photon map (0 = global, 1 = caustic) */
  uint64_t knn_map_queries[2], knn_map_photons[2], knn_map_visited[2];
  double knn_map_kernel_ms[2], knn_map_launches[2];
  /* chunk k-NN path, within knn_map_kernel_ms: time and queries of the final fallback kernel
   * (per-lane for K <= 64, query-per-wave for K > 64): the queries neither chunk pass resolved */
  double knn_map_fallback_ms[2];
  uint64_t knn_map_fallback_queries[2];
  /* k-NN launch sequence the last batch ran per map (-1 none): 7 lane-select chunk kernel +
   * per-lane fallback, 8 large-K chunk kernel (+ second chunk pass) + query-per-wave fallback,
   * 3 per-lane, 1 query-per-wave, 0 per-lane with global heaps, 9 irradiance-cache lookup */
  int32_t knn_map_kind[2];
  /* chunk k-NN path: time of the second chunk pass (larger LDS candidate set) and the queries
   * the first pass handed to it (those it did not resolve are in knn_map_fallback_queries) */
  double knn_map_pass2_ms[2];
  uint64_t knn_map_pass2_queries[2];
  /* device sets (gi_create_devices): the slowest and fastest device's render phase and the
   * tile gather onto the first device after the last one finished (0 on one device) */
  double device_render_s_max, device_render_s_min, gather_s;
} gi_render_stats;

typedef struct gi_ctx gi_ctx;

/* ---- host-side flag parsing (drop-in ParseArgs) --------------------------------------- */
void gi_params_default(gi_params *p);
/* returns GI_OK, or GI_ERR_ARG with the reference's message in *err (static storage) */
int gi_parse_args(int argc, char **argv, gi_params *p, const char **scene_path,
                  const char **output_path, int *width, int *height, int *aa,
                  int *real_material, const char **err);

/* ---- context ----------------------------------------------------------------------- */
int gi_create(gi_ctx **out, int hip_device);
/* One context over several HIP devices (SURVEY.md 8(b) gi_create(gi_ctx**, const
 * gi_device_set*); render.cpp:90's thread interleave re-cut as a device shard). Every call on
 * it drives all of them: the scene and photon maps are replicated (photon emission ranges are
 * split across the devices, the maps built once), gi_render_image deals 16x16 output tiles
 * (tx, ty) to device (tx + ty) % count and gathers the tiles onto devices[0] (RCCL send/recv over xGMI when the
 * devices are distinct, else a peer copy). Test seams (gi_*_batch) run on devices[0]. */
#define GI_MAX_DEVICES 64
typedef struct gi_device_set {
  int32_t count;
  int32_t devices[GI_MAX_DEVICES];
} gi_device_set;
int gi_create_devices(gi_ctx **out, const gi_device_set *set);
/* What a context really drives, so that a multi-GPU run can prove it (no reference
 * counterpart: the reference's threads share one host). *ndev = the context's device count;
 * for each (up to max): devices[k] = its HIP ordinal, pci_bus[k] = that device's PCI bus id
 * (hipDeviceAttributePciBusId; -1 if unknown), comm_rank[k] = ncclCommUserRank of its RCCL
 * communicator (-1 without one). *comm_count = ncclCommCount of the first communicator (0 when
 * the set gathers without RCCL: one device, or entries naming the same device). */
int gi_device_info(const gi_ctx *ctx, int max, int *ndev, int *devices, int *pci_bus,
                   int *comm_rank, int *comm_count);
void gi_destroy(gi_ctx *ctx);
const char *gi_last_error(const gi_ctx *ctx);
int gi_set_params(gi_ctx *ctx, const gi_params *p);
/* Progress reports (the reference's PrintProgress calls, io_utils.cpp:257-268): stage 0 =
 * RenderImage, progress = output pixels done / total after each batch (render.cpp:80-87, 201);
 * stage 1 / 2 = the global / caustic map's emission rounds, progress = stored / goal
 * (photonmap.cpp:193-197, 244-248). Called on the thread that made the gi_ call; null = off. */
typedef void (*gi_progress_fn)(int stage, double progress, void *user);
int gi_set_progress(gi_ctx *ctx, gi_progress_fn fn, void *user);
int gi_read_scene(gi_ctx *ctx, const char *path, int real_material);
/* scene summary: nodes, lights, radius, ambient/background */
int gi_scene_info(gi_ctx *ctx, int *nnodes, int *nlights, int *nprims, double *radius);

/* ---- photon maps ---------------------------------------------------------------------- */
int gi_map_photons(gi_ctx *ctx, gi_photon_stats *stats);
/* Replace a photon map with caller photons (kd build + upload); n == 0 disables the map. */
int gi_set_photon_map(gi_ctx *ctx, int map, const gi_photon *photons, int64_t n);
/* Copy a photon map back in storage (emission) order. */
int gi_get_photon_map(gi_ctx *ctx, int map, gi_photon *out, int64_t capacity, int64_t *n);
/* Test seam: the map's kd tree as the k-NN kernels read it (the R3Kdtree the reference builds
 * in R3Kdtree.cpp:1552-1671). nodes: 8 floats per node of the implicit tree (node v = 1 ..
 * 2 * nleaves - 1; {lo.xyz, split}, {hi.xyz, axis bits}); perm: kd-order position -> emission
 * index. Null outputs only report the sizes. */
int gi_get_kd_tree(gi_ctx *ctx, int map, float *nodes, int64_t node_floats, int32_t *perm,
                   int64_t perm_capacity, int32_t *nleaves, int64_t *n);

/* ---- rendering ------------------------------------------------------------------------ */
/* Full frame; rgb8 is W*H*3 bytes row-major with row 0 = image row y=0 (bottom, as R2Image);
 * rgbf (optional) receives the clamped box-filtered colour in [0,1]. */
int gi_render_image(gi_ctx *ctx, int aa, int width, int height, uint8_t *rgb8, float *rgbf,
                    gi_render_stats *stats);
/* Shard: render only the output tiles (tile_px x tile_px pixels; tile column tx, row ty) with
 * (tx + ty) % nshards == shard (a diagonal deal: every run of nshards tiles along a row or a
 * column meets every shard), packed shards in row-major tile order; rgbf is the full W*H*3 image, untouched outside the shard. */
int gi_render_tiles(gi_ctx *ctx, int aa, int width, int height, int tile_px, int shard,
                    int nshards, float *rgbf, gi_render_stats *stats);
/* Shard left on the device (one-process-per-GPU ranks, e.g. torchrun): renders the same tiles
 * as gi_render_tiles and writes them packed into `packed`, a DEVICE pointer on the context's
 * device holding `capacity` pixels: 16 B per pixel of the shard, in the shard's tile order
 * (f32 r, g, b; the u8 r, g, b in the low 24 bits of the fourth word). *npix receives the
 * shard's pixel count (packed == NULL only reports it). Synchronous: the buffer is complete on
 * return. */
int gi_render_tiles_packed(gi_ctx *ctx, int aa, int width, int height, int tile_px, int shard,
                           int nshards, void *packed, int64_t capacity, int64_t *npix,
                           gi_render_stats *stats);
/* Compose the frame from every shard's packed pixels: `packed` is a DEVICE pointer on the
 * context's device to nshards buffers of `stride` pixels (16 B each), shard s at s * stride
 * (the layout of a gather of gi_render_tiles_packed outputs); the caller must have allocated
 * all stride * nshards * 16 bytes (each shard's pixel count must be <= stride, checked).
 * rgb8 / rgbf (host, optional) receive the full image as gi_render_image returns it.
 * Both packed entry points restore the calling thread's current HIP device on return. */
int gi_compose_tiles(gi_ctx *ctx, int width, int height, int tile_px, int nshards,
                     const void *packed, int64_t stride, uint8_t *rgb8, float *rgbf);
/* Quantise a full float image like RenderImage's SetPixelRGB (truncate 255*c). */
int gi_quantize(int width, int height, const float *rgbf, uint8_t *rgb8);

/* ---- test seams ----------------------------------------------------------------------- */
/* n <= 2^26 queries per call (GI_ERR_ARG above). */
int gi_estimate_radiance_batch(gi_ctx *ctx, int map, int64_t n, const gi_radiance_query *q,
                               double *rgb_out, int32_t *nfound, float *max_d2);
int gi_knn_batch(gi_ctx *ctx, int map, int64_t n, const double *points, int k, double max_dist,
                 int32_t *idx_out, float *d2_out, int32_t *nfound);
/* Diagnostics: time the k-NN estimate kernel over n resident queries (Morton-ordered as in
 * rendering; mode 0 radiance, 1 irradiance, 2 list) for `iters` launches with the given
 * kernel (-1 = default; else a GI_KNN_KERNEL kind of gi_host.cpp run_knn). Uses the context's
 * estimate size / distance / filter for `map`. Outputs average ms per launch and the
 * photons found / visited per query. No reference counterpart (measurement only). */
int gi_knn_bench(gi_ctx *ctx, int map, int64_t n, const double *points, const double *normals,
                 const int32_t *materials, int mode, int kernel, int iters, double *ms_per_launch,
                 double *found_per_query, double *visited_per_query);
int gi_intersect_batch(gi_ctx *ctx, int64_t n, const double *org, const double *dir,
                       int32_t *hit, double *t, double *point, double *normal, int32_t *material);
/* Test seam: the device's fp64 math on host inputs, fn = 0 acos(x), 1 sin(x), 2 cos(x),
 * 3 pow(x, y), 4 atan2(x, y), 5 sqrt(x), 6 tan(x), 7 asin(x) (y ignored except by 3 and 4): the
 * functions the photon tracer, samplers and Phong terms call (graphics_utils.cpp:95-216,
 * photon_utils.cpp:56-60), gi_math.h's sequences, for comparing the device's results with the
 * oracle's (the same sequences on the host) and the host C library's one for one. */
int gi_math_probe(gi_ctx *ctx, int fn, int64_t n, const double *x, const double *y, double *out);

/* Free the context's render and photon-tracing device scratch (all devices of a device set),
 * keeping the scene, the photon maps and their kd trees; the next render or map build
 * re-allocates what it needs. For a long-lived context that must share the GPU with another
 * large one. No reference counterpart (the reference's buffers are host memory). */
int gi_release_scratch(gi_ctx *ctx);

/* ---- output --------------------------------------------------------------------------- */
int gi_write_image(const char *path, int width, int height, const uint8_t *rgb8);

#ifdef __cplusplus
}
#endif
#endif /* GI_H */
