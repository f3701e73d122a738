// gi_kernels.h -- kernel argument blocks and host-callable launchers (gi_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gi_device.h"

namespace gi {

// device-written photon record; byte-identical to gi_photon (gi.h) on little-endian
struct gi_photon_dev {
  float pos[3];
  uint32_t rgbe;   // r | g<<8 | b<<16 | e<<24
  uint16_t dir;
  uint16_t flags;
};
static_assert(sizeof(gi_photon_dev) == 20, "photon record is 20 bytes");

// per primary sample: the RayTrace state the sample paths need (raytracer.cpp:174-233)
struct Spawn {
  double p[3], n[3], v[3];
  double ct, R;
  double base[3];    // ambient + direct (+ background on a miss)
  int32_t mat, hit;
  int32_t n_t, n_s, n_i;  // transmissive / specular / indirect sample counts
  int32_t q_glob, q_caus; // primary-hit photon-map queries (photon_viz / caustic)
  int32_t tri;            // triangle hit (gi_device.h Hit::tri): the sample paths leave from it
  double wt[3];           // indirect paths' outer weight kd / n_i (raytracer.cpp:112-135)
};

// shading half of a photon-map query (search half is float4 {x, y, z, meta})
// an indirect sample path whose first bounce hit a material with a specular or transmissive
// term: the state of MonteCarlo_IndirectSample's loop (montecarlo.cpp:177-305) at that hit,
// queued so the shading and the rest of the path run compacted in ind_cont_kernel
// Two kinds share the record (and ind_cont_kernel):
//   mat >= 0: an indirect sample path queued at its first hit (hp, hn, mat) by ind_kernel;
//   mat == -1: the IndirectIllumination(inMC) sub-path of a Monte Carlo path (montecarlo.cpp:
//   144-152), queued by mc_kernel as a ray (org, direction in hp) with its path's query count j;
//   its contribution is added to the path's base (the last term of that path's sum).
struct IndCont {
  double org[3];          // origin of the traced ray (the loop's ray_start)
  double hp[3], hn[3];    // hit point and normal (mat >= 0); hp = ray direction (mat == -1)
  double w[3];            // outer weight W (throughput is still 1)
  uint64_t rkey, rctr;    // RNG stream position
  uint32_t g, prim;       // path slot, primary sample
  uint32_t pslot, qslot;  // slot within the primary, global-query slot (~0: append)
  int32_t mat;
  uint32_t j;             // queries already issued by the path (mat == -1)
  int32_t tri;            // triangle the continued ray leaves from (-1: none), Hit::tri
  int32_t sub;            // 1: a Monte Carlo path's indirect sub-path queued at its first hit
};

// continuation queue stripes: wave w appends to stripe w % IND_QS (one atomic per wave on a
// counter shared by 1/IND_QS of the waves)
constexpr int IND_QS = 64;
// IndCont::g of an empty entry of the dense Monte Carlo sub-path queue (mc_persist_kernel)
constexpr uint32_t IND_EMPTY = 0xffffffffu;
// chunk k-NN fallback list stripes: block b appends to stripe b % FB_QS
constexpr int FB_QS = 64;

struct QShade {
  double n[3];   // surface normal
  double ex[3];  // exact reflection direction (Phong lobe term)
  double w[3];   // path weight multiplying the estimate
};

enum {
  ST_RAY = 0, ST_SHADOW, ST_MONTE, ST_TRANS, ST_SPEC, ST_INDIRECT, ST_CAUSTIC,
  ST_KNN, ST_KNN_PHOTONS, ST_KNN_VISITED,        // global map (caustic map: + ST_KNN_MAP)
  ST_KNN_C, ST_KNN_C_PHOTONS, ST_KNN_C_VISITED,
  ST_GEN_MISS,   // queries an instance without the general estimate form met (host re-runs)
  ST_PHASE = 16,                                 // 16 diagnostic counters (GI_KNN_DBG & 16)
  ST_COUNT = 32
};
enum { ST_KNN_MAP = ST_KNN_C - ST_KNN
};

struct RenderArgs {
  SceneView S;
  Flags F;
  const int2 *pixels;   // output pixels of this batch
  int32_t npix;
  int32_t af;           // 2^aa
  int32_t W, H;         // supersampled viewport (render.cpp:177-178)
  int32_t dof_test;
  int32_t out_w;
  int64_t nprim;        // npix * af^2 * dof_test
  int64_t total_paths;
  Spawn *spawn;
  uint32_t *npaths;     // [nprim] 1 + transmissive + specular paths (CSR base slots; the
                        // indirect paths' are tiled, ind_rows)
  uint32_t *nmc;        // [nprim] transmissive + specular (Monte Carlo path) samples
  uint32_t *nind;       // [nprim] indirect samples
  const uint32_t *path_off;  // [nprim + 1] exclusive scans of the three counts
  const uint32_t *mc_off;
  const uint32_t *ind_off;
  const uint64_t *ind_row_info;  // [rows] tile << 32 | sample index of each 64-entry row of
                                 // the tiled indirect slots
  const uint32_t *mc_tab;    // same for the Monte Carlo paths
  int64_t total_mc, total_ind;
  int64_t tind;               // tiled indirect entries (64 per row, >= total_ind; RenderArgs::ind_rows)
  int32_t dbg;          // diagnostics: 1 = skip the indirect trace, 2 = skip diffuse sampling too
  int32_t split_ind;    // 1: indirect paths trace their first bounce, continuations are queued
  int32_t tiled_skip;   // 1: unused tiled indirect slots keep whatever they hold instead of QMETA_NONE
                        // (the global list's k-NN order comes from the row masks; nothing reads them)
  IndCont *ind_cont;    // continuation queue: IND_QS stripes of ind_cap_s entries
  uint32_t *ind_ncont;  // fill of stripe s at [s * 32] (one 128-B line per counter)
  uint32_t ind_cap_s;
  IndCont *mc_cont;     // Monte Carlo paths' indirect sub-paths, striped the same way
  uint32_t *mc_ncont;
  uint32_t mc_cap_s;
  uint32_t *mc_next;    // mc_persist_kernel's path counter (null: mc_kernel, one path per lane)
  int32_t mc_persist_blocks;  // its grid
  IndCont *mc_cont2;    // ... those whose first bounce hit glass / a mirror (mc_sub_kernel),
  uint32_t *mc_ncont2;  // at that hit, same stripes and capacity
  // Indirect paths' slots, tiled: primaries b in tiles of 64 (T = b / 64); tile T holds
  // ind_rows[T+1] - ind_rows[T] = max n_i over its primaries rows of 64 entries, and indirect
  // path s of primary b is entry tau(b, s) = 64 * (ind_rows[T] + s) + b % 64 (ind_tau). Its
  // base is base slot ind_g0 + tau, its query (global list) slot qind_base + tau. The indirect
  // path kernel runs one thread per entry (a wave = one row: sample s of 64 primaries) and the
  // reduction one per primary, so both read and write rows as 64 contiguous entries.
  int64_t qind_base;
  const uint32_t *ind_rows;  // [ntiles + 1] exclusive scan of the tiles' row counts
  int64_t ind_g0;            // first base slot of the tiled region (= the CSR paths' total)
  uint64_t *ind_qmask;       // [rows] bit l of row r: entry 64 r + l holds a query
  uint64_t *ind_bmask;       // [rows] ... holds a stored base (not +0; unstored bases are +0)
  // query lists (0 = global map, 1 = caustic map). Deterministic slots first: list l slot p
  // = primary sample p's own query (slot-0 path), then (global list only) slot
  // qind_base + t = indirect path t's single query; unused ones hold QMETA_NONE. Monte Carlo
  // paths append after those with a wave-aggregated atomic counter. Each query carries key =
  // path_slot << 20 | index-in-path so the per-pixel reduction can sum them in a
  // deterministic order after a key sort (empty slots: key ~0).
  float4 *qpos[2];
  QShade *qshade[2];
  uint64_t *qkey[2];
  uint32_t *qcount;     // [2] device counters
  uint32_t qcap[2];
  uint32_t qapp[2];           // first Monte Carlo (appended) slot of each list
  const uint64_t *skey[2];    // sorted keys of the appended slots [qapp, nq)
  const uint32_t *sslot[2];   // slot - qapp of each sorted key
  uint32_t *qseg[2];          // [nprim + 1]: sorted appends of primary b are [qseg[b], qseg[b+1])
  uint32_t nq[2];
  double *base;         // [total_paths * 3]
  double *prim_rgb;     // [nprim * 3] per-primary sums (reduce_prim_kernel -> reduce_kernel)
  const double *qout[2];       // k-NN contributions per slot
  float *rgbf;
  uint8_t *rgb8;
  unsigned long long *stats;
};

// kd node record (KdView::nodes): lo = {min xyz, split}, hi = {max xyz, axis bits}
struct KdNode {
  float4 lo, hi;
};

// The maps are read-only during a k-NN launch. Reading a node through the constant address
// space lets wave-uniform node reads compile to scalar loads into SGPRs (through a generic
// pointer, which could alias the kernel's own writes, the compiler emits vector loads into
// VGPRs). The host compilation pass has no address spaces.
__device__ __forceinline__ KdNode ld_node(const float *nodes, int n) {
  KdNode r;
#if __HIP_DEVICE_COMPILE__
  typedef __attribute__((address_space(4))) const float cfloat;
  cfloat *p = (cfloat *)nodes + 8 * n;
  r.lo = make_float4(p[0], p[1], p[2], p[3]);
  r.hi = make_float4(p[4], p[5], p[6], p[7]);
#else
  r = reinterpret_cast<const KdNode *>(nodes)[n];
#endif
  return r;
}

// squared distance from q to a node's tight box, evaluated with the same fp32 operation
// sequence as the photon metric (d2 = fma(dz,dz, fma(dy,dy, dx*dx))): every rounding step is
// monotone, so box_d2 <= metric d2 of every photon inside the box -- pruning on
// box_d2 > bound never drops a photon the exact search would keep.
__device__ __forceinline__ float kd_box_d2(const float4 &lo, const float4 &hi, float qx, float qy,
                                           float qz) {
  float gx = fmaxf(fmaxf(lo.x - qx, qx - hi.x), 0.0f);
  float gy = fmaxf(fmaxf(lo.y - qy, qy - hi.y), 0.0f);
  float gz = fmaxf(fmaxf(lo.z - qz, qz - hi.z), 0.0f);
  return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, __fmul_rn(gx, gx)));
}

__device__ __forceinline__ float kd_axis_q(int axis, float qx, float qy, float qz) {
  return (axis == 0) ? qx : ((axis == 1) ? qy : qz);
}

// Stackless backtrack: move to the far sibling of the deepest near child on the path from
// the root to `node`; false when the walk is complete.
__device__ __forceinline__ bool kd_next(const KdNode *nodes, int &node, float qx, float qy,
                                        float qz) {
  while (node != 1) {
    const KdNode &pn = nodes[node >> 1];
    float q = kd_axis_q(__float_as_int(pn.hi.w), qx, qy, qz);
    int near_is_right = (q - pn.lo.w >= 0.0f) ? 1 : 0;
    if ((node & 1) == near_is_right) break;
    node >>= 1;
  }
  if (node == 1) return false;
  node ^= 1;
  return true;
}

// pow behind a call: the estimates' specular and Gaussian-filter branches would otherwise inline
// one fp64 pow per unrolled photon (code size, registers) for paths most scenes never take
static __device__ __noinline__ double pow_call(double x, double y) { return gm::pow(x, y); }

// d-ary max-heap of u64 keys in LDS laid out [slot][lane] (stride 64): sift-down, Floyd build,
// and accept (append unordered until K, heapify once, then replace the root)
template <int ARY>
__device__ __forceinline__ void heapn_sift(uint64_t *h, int n, int c, uint64_t key) {
  while (true) {
    int f = ARY * c + 1;
    if (f >= n) break;
    uint64_t kk[ARY];
#pragma unroll
    for (int j = 0; j < ARY; j++) kk[j] = (f + j < n) ? h[(f + j) * 64] : 0ull;
    int m = f;
    uint64_t mk = kk[0];
#pragma unroll
    for (int j = 1; j < ARY; j++)
      if (kk[j] > mk) { mk = kk[j]; m = f + j; }
    if (key >= mk) break;
    h[c * 64] = mk;
    c = m;
  }
  h[c * 64] = key;
}

template <int ARY>
__device__ __forceinline__ void heapn_build(uint64_t *h, int n) {
  for (int i = (n - 2) / ARY; i >= 0; i--) heapn_sift<ARY>(h, n, i, h[i * 64]);
}

// accept one candidate (key < lim already checked)
template <int ARY>
__device__ __forceinline__ void heapn_accept(uint64_t *h, int &size, int K, uint64_t key,
                                             uint64_t &lim) {
  if (size < K) {
    h[size * 64] = key;
    size++;
    if (size == K) {
      heapn_build<ARY>(h, K);
      lim = h[0];
    }
  } else {
    heapn_sift<ARY>(h, K, 0, key);
    lim = h[0];
  }
}

// The -v counters live in ST_STRIPES copies of ST_COUNT words (the host sums them). One
// counter word takes ~10^8 atomics/s (MI355X_MICROARCH.md): a launch of ~500k waves adding to
// one word would serialise for ~5 ms, so each wave adds to the copy its global wave id selects.
constexpr int ST_STRIPES = 64;
__device__ __forceinline__ unsigned long long *stat_stripe(unsigned long long *stats) {
  uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  return stats + (size_t)(w & (ST_STRIPES - 1)) * ST_COUNT;
}

// wave-level counter reduction (one atomic per wave, on the wave's stripe; dst points into
// stripe 0)
__device__ __forceinline__ void wave_add(unsigned long long *dst, uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0 && v) {
    uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    atomicAdd(dst + (size_t)(w & (ST_STRIPES - 1)) * ST_COUNT, (unsigned long long)v);
  }
}

// query-list slot with no query (deterministic slots a path did not use): qpos.w bits
constexpr uint32_t QMETA_NONE = 0xffffffffu;
// a query's qpos.w bits: side of the surface (bits 0-1), material (bits 2-27), and the face of
// its normal for the launch order (bits 28-30: dominant axis * 2 + negative; gi_sort.hip
// surface_key); bit 31 is clear, so no query's bits equal QMETA_NONE
constexpr uint32_t QMETA_MAT_MASK = 0x03ffffffu;
constexpr int QMETA_MAX_MATS = 1 << 26;
__host__ __device__ __forceinline__ uint32_t qmeta_mat(uint32_t meta) { return (meta >> 2) & QMETA_MAT_MASK; }

enum { KNN_MODE_RADIANCE = 0, KNN_MODE_IRRADIANCE = 1, KNN_MODE_LIST = 2, KNN_MODE_DK = 3 };

struct KnnArgs {
  KdView map;
  const float4 *qpos;
  const QShade *qshade;
  const uint32_t *perm;    // optional query order (spatial sort)
  const DMaterial *mats;
  const double *lut;       // 65536 x 3 direction table
  int64_t nq;              // queries in this launch
  int64_t q0;              // first (sorted) query position of this launch
  int32_t K;
  int32_t filter;
  int32_t mode;
  int32_t stat_off;        // 0 (global map) or ST_KNN_MAP (caustic map)
  int32_t sel_slack;       // query-per-wave kernel: re-select once K + slack candidates held
  int32_t chunk_minsub;    // chunk kernel: smallest query group an overflowing chunk is split to
  int32_t dk_exact;        // large-K chunk kernel: refine the dk bound of the centre to the exact d_K(c)
  int32_t qpl;             // per-lane kernel: consecutive (sorted) queries per lane
  int32_t dbg;             // diagnostics: chunk kernel phase skips (timing only)
  int32_t general;         // 1: a query may need EstimateRadiance's general form (pow: specular
                           // term, cone / Gauss filter); 0: host-checked that the disk filter and
                           // diffuse-only materials serve every query (knn_general), and the
                           // kernels run instances without the general form (fewer registers)
  float r2f;               // (float)(r*r) accept radius
  double rmax;
  double fa, fb, fk;       // FILTER_CONST_A/B/K
  double *out;             // [nq*3]
  int32_t *out_n;          // optional
  float *out_maxd2;        // optional
  float *out_dk;           // KNN_MODE_DK: per query, the K-th distance bound (KdView::dk)
  int32_t *out_idx;        // KNN_MODE_LIST
  float *out_d2;
  int32_t *list_idx;       // query-per-wave kernel: K-best lists [nq][K] (kd-order index)
  float *list_d2;          //   and their d2; -1 past list_n[q]
  int32_t *list_n;
  uint32_t *fb_list;       // chunk kernel: queries (original slots) handed to the fallback,
  uint32_t *fb_count;      // FB_QS stripes of fb_cap_s entries; fill of stripe s at [s * 32]
  uint32_t fb_cap_s;
  float *gheap_d2;         // global heap scratch (K > 64)
  int32_t *gheap_idx;
  unsigned long long *stats;
};

struct PhotonArgs {
  SceneView S;
  Flags F;
  int32_t light;
  int32_t caustic;
  int64_t e0;     // first emission index
  int64_t n;      // photons in this launch
  uint32_t *counts;        // PM_COUNT: photons each emitted photon stores
  const uint32_t *offsets; // PM_EMIT: their exclusive scan
  gi_photon_dev *out;
  uint32_t *cursor;        // PM_APPEND: slot counter (one atomic per wave per bounce)
  uint64_t *keys;          // PM_APPEND: (emission index << obits) | store ordinal per slot
  uint32_t cap;            // PM_APPEND: slots in out / keys
  int32_t obits;           // PM_APPEND: bits of the store ordinal (max_photon_depth)
};
enum { PM_COUNT = 0, PM_EMIT = 1, PM_APPEND = 2 };

struct ScanTemp {
  uint32_t *level[8];
  uint32_t *level_out[8];
  int depth;
};

hipError_t launch_scan(const uint32_t *in, uint32_t *out, int64_t n, ScanTemp &tmp,
                       hipStream_t st);
void launch_primary(const RenderArgs &a, hipStream_t st);
// wait_join = false: the join event is recorded on st2 but st does not wait for it (the caller
// makes st wait later, after work that reads only the deterministic query slots)
void launch_path(const RenderArgs &a, hipStream_t st, hipStream_t st2 = nullptr,
                 hipEvent_t fork = nullptr, hipEvent_t join = nullptr, bool wait_join = true);
// float4 queries {x, y, z, 0} at the photons of a map (KNN_MODE_DK input)
void launch_photon_queries(const float *pos4, int64_t n, float4 *q, hipStream_t st);
// dense copy of the striped chunk fallback list; total length to *total
void launch_fb_compact(const uint32_t *list, const uint32_t *count, uint32_t cap_s, uint32_t *dense,
                       uint32_t *total, hipStream_t st);  // slot0 + indirect + Monte Carlo
void launch_reduce(const RenderArgs &a, hipStream_t st);
void launch_owner_table(const uint32_t *off, int64_t n, uint32_t *tab, hipStream_t st);
void launch_ind_tiles(const uint32_t *nind, int64_t nprim, uint32_t *rows, hipStream_t st);
void launch_ind_row_tile(const uint32_t *rows, int64_t ntiles, uint64_t *tab, hipStream_t st);
void launch_ind_pad(const RenderArgs &a, hipStream_t st);
// device-set gather: pixels (x, y int32 pairs) packed 16 B each / scattered back
void launch_pack_pixels(const int32_t *pix_xy, int64_t n, int w, const float *rgbf,
                        const uint8_t *rgb8, void *out, hipStream_t st);
void launch_unpack_pixels(const int32_t *pix_xy, int64_t n, int w, const void *in, float *rgbf,
                          uint8_t *rgb8, hipStream_t st);
void launch_segments(const uint64_t *skeys, uint32_t n, uint32_t nprim, uint32_t *seg,
                     hipStream_t st);
// generic per-lane kernel with its heaps in global scratch (any K; used beyond the LDS kernels)
void launch_knn(const KnnArgs &a, hipStream_t st);
bool launch_knn_wave(const KnnArgs &a, int cap_mul, hipStream_t st);
bool launch_knn_lane(const KnnArgs &a, hipStream_t st);
bool launch_knn_chunk(const KnnArgs &a, hipStream_t st);  // K <= 64, lane select
bool launch_knn_chunk2(const KnnArgs &a, hipStream_t st);  // its 480-candidate second pass
bool launch_knn_chunk_big(const KnnArgs &a, int cap, hipStream_t st);  // K > 64, needs a.map.dk
// blocks of the chunk kernels (one 64-query chunk each, grid-stride)
unsigned knn_chunk_grid(int64_t nq);
void launch_list_estimate(const KnnArgs &a, hipStream_t st);
void launch_cached(const KnnArgs &a, hipStream_t st);
void launch_photons(const PhotonArgs &a, int mode, hipStream_t st);
void launch_photon_gather(const gi_photon_dev *src, const uint32_t *slot, int64_t n,
                          gi_photon_dev *dst, hipStream_t st);
void launch_photon_rescale(gi_photon_dev *ph, int64_t n, double pp, hipStream_t st);
void launch_math_probe(int fn, int64_t n, const double *x, const double *y, double *out,
                       hipStream_t st);
void launch_intersect(const SceneView &S, int64_t n, const double *org, const double *dir,
                      int32_t *hit, double *t, double *point, double *normal, int32_t *mat,
                      hipStream_t st);

}  // namespace gi
