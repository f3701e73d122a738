// gi_host.cpp -- host orchestration of the MI355X renderer and the C-ABI of include/gi.h.
//
// Replaces the reference's host-side driver code: MapPhotons (photonmap.cpp:260-436) and
// RenderImage (render.cpp:155-259). The CPU threads of the reference become batched
// wavefront launches; host code only sequences kernels, runs the adaptive photon-emission
// bookkeeping and builds the kd-tree (kd build on the GPU is SURVEY.md §8(f) row f1).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include "../../include/gi.h"
#include "gi_kdbuild.h"
#include "gi_kernels.h"
#include "gi_scene.h"
#include "gi_sort.h"

using namespace gi;

namespace {

// ---------------------------------------------------------------------------------------
// small device-buffer helper
// ---------------------------------------------------------------------------------------
// Device buffer that only grows. A growth re-allocates with 1.5x headroom: hipMalloc of tens of
// GB takes seconds on MI355X, and a frame whose batches grow a little at a time (C5's first
// render: query lists 365 M -> 431 M -> 449 M) would otherwise pay that at every step
// (the batch log showed 3.9 s and 3.2 s batches; C5 shard 1/8 cold 64.0 s vs 16.5 s warm).
// Environment knobs: tests and measurements only (every default is the measured best). All of
// them are read here, through env_num: GI_LOG (bit 1 device allocations >= 64 MiB, bit 2 one
// line per batch, bit 4 one line per chunk k-NN launch; stderr), GI_KNN_DBG (k-NN kernel
// diagnostics, KnnArgs::dbg), GI_DBG (render-kernel diagnostics, RenderArgs::dbg), GI_SLOT_LIMIT,
// and the exactness-tested alternatives gi_create lists (the tests select them to show that the
// default's result does not depend on them).
static double env_num(const char *name, double def) {
  const char *s = getenv(name);
  return (s && *s) ? atof(s) : def;
}
static int log_bits() {
  static const int bits = (int)env_num("GI_LOG", 0);
  return bits;
}
static bool alloc_log() { return (log_bits() & 1) != 0; }
struct DBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes, int line = __builtin_LINE()) {
    if (bytes <= cap && p) return hipSuccess;
    if (alloc_log() && bytes >= ((size_t)64 << 20)) {
      auto t0 = std::chrono::steady_clock::now();
      size_t old = cap;
      hipError_t e = grow(bytes);
      fprintf(stderr, "[gi] alloc %.2f GB (was %.2f GB) at gi_host.cpp:%d: %.1f ms\n", cap / 1e9,
              old / 1e9, line,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
      return e;
    }
    return grow(bytes);
  }
  hipError_t grow(size_t bytes) {
    // headroom for a buffer that has grown before: at least 1/8 above the request and at least
    // twice the old capacity. Freed device memory is cleared by the driver before it is handed
    // out again, and an allocation that finds no clean memory waits for it: C5's first frame
    // (fresh box, first process) grew its buffers in 1/8 steps to 467 GB of cumulative
    // allocation, 377 GB of it freed again, and one 32.9 GB step then waited 6.0 s (DESIGN.md
    // 3.3). Doubling (capped at 1.5x the request, so that a buffer that needs just over its old
    // capacity does not take twice that: C2's 33 GB shading list) keeps the steps few.
    size_t grown = cap ? std::max(std::min(cap * 2, bytes + bytes / 2), bytes + bytes / 8) : 0;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (grown > bytes) {  // headroom only while a quarter of the device stays free after it
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < grown + tot / 4) grown = 0;
    }
    size_t want = std::max(std::max(bytes, grown), (size_t)256);
    hipError_t e = hipMalloc(&p, want);
    if (e != hipSuccess && want > bytes) {  // no room for the headroom: exactly what is asked
      (void)hipGetLastError();
      want = std::max(bytes, (size_t)256);
      e = hipMalloc(&p, want);
    }
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

// RNRgb_to_RGBE / RGBE_to_RNRgb (graphics_utils.cpp:50-77), host side
void rgbe_enc(const double c[3], uint8_t *out) {
  double mx = 0;
  for (int i = 0; i < 3; i++)
    if (c[i] > mx) mx = c[i];
  if (!(mx > 0)) { out[0] = out[1] = out[2] = out[3] = 0; return; }
  int e;
  double m = frexp(mx, &e);
  out[0] = (uint8_t)(256.0 * c[0] / mx * m);
  out[1] = (uint8_t)(256.0 * c[1] / mx * m);
  out[2] = (uint8_t)(256.0 * c[2] / mx * m);
  out[3] = (uint8_t)(e + 128);
}
void rgbe_dec(const uint8_t *in, double c[3]) {
  if (!in[3]) { c[0] = c[1] = c[2] = 0; return; }
  double inv = ldexp(1.0, ((int)in[3]) - 128 - 8);
  for (int i = 0; i < 3; i++) c[i] = (double)in[i] * inv;
}

// ---------------------------------------------------------------------------------------
// photon map: host kd build of an implicit complete tree (leaf l holds photons
// [l*n/L, (l+1)*n/L)); split = median of the node's range along its longest bbox axis.
// Any kd-tree gives the same k-NN set (up to ties at the k-th distance, broken here by
// (d2, kd-order index)); the reference's tree is R3Kdtree.cpp:1552-1671.
// ---------------------------------------------------------------------------------------
struct HostMap {
  std::vector<gi_photon> storage;  // emission order
  std::vector<int32_t> perm;       // kd order -> storage index
  std::vector<float> pos4;
  std::vector<uint32_t> rgbe;
  std::vector<float> nodes;  // 8 floats per node: {lo.xyz, split}, {hi.xyz, axis bits}
  int nleaves = 1, levels = 0;
  float bmin[3] = {0, 0, 0}, bmax[3] = {0, 0, 0};
};

void kd_rec(HostMap &M, int node, int a, int b, int depth_par) {
  int64_t n = (int64_t)M.storage.size();
  int L = M.nleaves;
  if (node >= L) return;
  int64_t lo = (int64_t)a * n / L, hi = (int64_t)b * n / L;
  int midleaf = (a + b) / 2;
  int64_t mid = (int64_t)midleaf * n / L;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  for (int64_t i = lo; i < hi; i++) {
    const float *p = M.storage[M.perm[i]].pos;
    for (int k = 0; k < 3; k++) { mn[k] = std::min(mn[k], p[k]); mx[k] = std::max(mx[k], p[k]); }
  }
  int axis = 0;
  float ext = mx[0] - mn[0];
  if (mx[1] - mn[1] > ext) { axis = 1; ext = mx[1] - mn[1]; }
  if (mx[2] - mn[2] > ext) axis = 2;
  float split = 0.f;
  if (hi > lo && mid < hi) {
    std::nth_element(M.perm.begin() + lo, M.perm.begin() + mid, M.perm.begin() + hi,
                     [&](int x, int y) { return M.storage[x].pos[axis] < M.storage[y].pos[axis]; });
    split = M.storage[M.perm[mid]].pos[axis];
  } else if (hi > lo) {
    split = mx[axis];
  }
  M.nodes[8 * node + 3] = split;
  int ai = axis;
  memcpy(&M.nodes[8 * node + 7], &ai, 4);
  if (depth_par > 0) {
    std::thread t([&]() { kd_rec(M, 2 * node, a, midleaf, depth_par - 1); });
    kd_rec(M, 2 * node + 1, midleaf, b, depth_par - 1);
    t.join();
  } else {
    kd_rec(M, 2 * node, a, midleaf, 0);
    kd_rec(M, 2 * node + 1, midleaf, b, 0);
  }
}

void kd_build(HostMap &M, int leaf_size, int threads) {
  int64_t n = (int64_t)M.storage.size();
  M.nleaves = 1;
  M.levels = 0;
  while ((int64_t)M.nleaves * leaf_size < n) { M.nleaves *= 2; M.levels++; }
  M.perm.resize(n);
  for (int64_t i = 0; i < n; i++) M.perm[i] = (int32_t)i;
  const int L = M.nleaves;
  M.nodes.assign(8 * 2 * (size_t)L, 0.0f);
  int par = 0;
  while ((1 << par) < threads && par < 4) par++;
  if (n > 0) kd_rec(M, 1, 0, L, par);
  M.pos4.resize(4 * (size_t)n);
  M.rgbe.resize(n);
  for (int k = 0; k < 3; k++) { M.bmin[k] = FLT_MAX; M.bmax[k] = -FLT_MAX; }
  for (int64_t i = 0; i < n; i++) {
    const gi_photon &p = M.storage[M.perm[i]];
    uint32_t w = (uint32_t)p.dir | ((uint32_t)p.flags << 16);
    M.pos4[4 * i] = p.pos[0];
    M.pos4[4 * i + 1] = p.pos[1];
    M.pos4[4 * i + 2] = p.pos[2];
    memcpy(&M.pos4[4 * i + 3], &w, 4);
    memcpy(&M.rgbe[i], p.rgbe, 4);
    for (int k = 0; k < 3; k++) {
      M.bmin[k] = std::min(M.bmin[k], p.pos[k]);
      M.bmax[k] = std::max(M.bmax[k], p.pos[k]);
    }
  }
  // tight boxes: leaves from their photons, internal nodes as the union of their children
  // (an empty leaf gets lo = +inf, hi = -inf: its box distance is +inf)
  for (int l = 0; l < L; l++) {
    float *b = &M.nodes[8 * (size_t)(L + l)];
    b[0] = b[1] = b[2] = INFINITY;
    b[4] = b[5] = b[6] = -INFINITY;
    int64_t s0 = (int64_t)l * n / L, s1 = (int64_t)(l + 1) * n / L;
    for (int64_t i = s0; i < s1; i++)
      for (int k = 0; k < 3; k++) {
        b[k] = std::min(b[k], M.pos4[4 * i + k]);
        b[4 + k] = std::max(b[4 + k], M.pos4[4 * i + k]);
      }
  }
  for (int v = L - 1; v >= 1; v--) {
    float *b = &M.nodes[8 * (size_t)v];
    const float *c0 = &M.nodes[8 * (size_t)(2 * v)], *c1 = &M.nodes[8 * (size_t)(2 * v + 1)];
    for (int k = 0; k < 3; k++) {
      b[k] = std::min(c0[k], c1[k]);
      b[4 + k] = std::max(c0[4 + k], c1[4 + k]);
    }
  }
}

struct DevMap {
  DBuf pos4, rgbe, nodes;
  DBuf dk;               // per-photon K-th distance bounds (KdView::dk), valid for dk_k / dk_r2
  int dk_k = -1;
  float dk_r2 = -1.0f;
  int64_t n = 0;
  int nleaves = 1, levels = 0;
  KdView view() const {
    KdView v;
    v.pos4 = pos4.as<float>();
    v.rgbe = rgbe.as<uint32_t>();
    v.nodes = nodes.as<float>();
    v.n = n;
    v.nleaves = nleaves;
    v.levels = levels;
    for (int k = 0; k < 3; k++) v.bmin[k] = v.bmax[k] = 0;
    v.dk = nullptr;
    return v;
  }
};

}  // namespace

// =======================================================================================
// RCCL, opened at run time by multi-device contexts only (gi_create_devices with distinct
// devices): the single-device library carries no RCCL dependency, and a torch process that
// loads it keeps its own copy.
struct Rccl {
  bool tried = false, ok = false;
  ncclResult_t (*commInitAll)(ncclComm_t *, int, const int *) = nullptr;
  ncclResult_t (*commDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*groupStart)() = nullptr;
  ncclResult_t (*groupEnd)() = nullptr;
  ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char *(*errString)(ncclResult_t) = nullptr;
  ncclResult_t (*commCount)(const ncclComm_t, int *) = nullptr;
  ncclResult_t (*commUserRank)(const ncclComm_t, int *) = nullptr;
  bool load() {
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    if (tried) return ok;
    tried = true;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return false;
    commInitAll = (decltype(commInitAll))dlsym(h, "ncclCommInitAll");
    commDestroy = (decltype(commDestroy))dlsym(h, "ncclCommDestroy");
    groupStart = (decltype(groupStart))dlsym(h, "ncclGroupStart");
    groupEnd = (decltype(groupEnd))dlsym(h, "ncclGroupEnd");
    send = (decltype(send))dlsym(h, "ncclSend");
    recv = (decltype(recv))dlsym(h, "ncclRecv");
    errString = (decltype(errString))dlsym(h, "ncclGetErrorString");
    commCount = (decltype(commCount))dlsym(h, "ncclCommCount");
    commUserRank = (decltype(commUserRank))dlsym(h, "ncclCommUserRank");
    ok = commInitAll && commDestroy && groupStart && groupEnd && send && recv && errString;
    return ok;
  }
};
Rccl g_rccl;

// =======================================================================================
// Execution state of one photon map's k-NN launches (stream, timing events, scratch). One per
// map, so the two maps' estimates can run concurrently on two streams during a render.
struct MapExec {
  hipStream_t st = nullptr;        // the ctx stream, or the side stream while maps overlap
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;  // chunk pass | second
                                   // chunk pass | fallback split timing (ev0 ev2 ev3 ev1)
  SortScratch sorter;              // Morton order of the query list
  DBuf list_idx, list_d2, list_n;  // K-best lists of the query-per-wave k-NN path
  DBuf gheap_d2, gheap_idx;        // global-memory heaps (K > 64 per-lane kernel)
  DBuf fb_list, fb_count, fb_dense;     // chunk k-NN fallback queries (striped, compacted)
  DBuf fb_list2, fb_count2, fb_dense2;  // large-K chunk k-NN: second pass's fallback queries
  DBuf dk_q;                       // photon positions as queries (ensure_dk)
  uint64_t fb_total = 0;
};

struct gi_ctx {
  int device = 0;
  // Device set (gi_create_devices): this context drives the first device and forwards every
  // call to one context per further device. Output tile (tx, ty) goes to device (tx + ty) % ndev
  // (shard_pixels' diagonal deal); photon emission ranges are split across the devices; the maps
  // are built once and replicated.
  std::vector<gi_ctx *> peers;
  std::vector<ncclComm_t> comms;     // [ndev] RCCL communicators (distinct devices), else empty
  DBuf pack;                         // this device's shard pixels, packed for the gather
  std::vector<DBuf> recv, peer_pix;  // first device: each peer's packed pixels and pixel list
  std::mutex err_mu;                 // err is written by the map worker threads too
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;     // side stream: Monte Carlo paths beside the indirect paths
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  MapExec mx[2];
  std::string err;
  gi_params P;
  bool have_params = false;
  bool have_scene = false;
  HostScene scene;
  // device scene
  DBuf d_nodes, d_elems, d_shapes, d_tris, d_bvh, d_mats, d_lights, d_lut, d_stats;
  // photon maps
  HostMap hmap[2];
  DevMap dmap[2];
  bool map_valid[2] = {false, false};
  int leaf_size[2] = {64, 256};  // photons per kd leaf, per map (global, caustic)
  bool gpu_kd = true;            // kd trees built on the device (gi_kdbuild.hip); GI_HOST_KD=1: host
  KdBuildScratch kdb;            // its scratch
  DBuf kd_ph;                    // emission-ordered photons uploaded for the device build
  int wave_cap_mul = 1;
  int chunk_cap_big = 512;        // large-K chunk kernel: LDS candidates of the first pass
  // large-K chunk kernel: the centre's dk bound refined to the exact d_K(c) (GI_CHUNK_DK_EXACT,
  // default on: C4 shard caustic k-NN 154.7 -> 145.1 ms per launch, C2 / C3 frames -0.7 / -1.0 %;
  // profiles/r05_dk_exact_ab.txt)
  bool chunk_dk_exact = true;
  int chunk_minsub_big = 64;      // large-K chunk kernel: overflowing chunks retried down to this (64: none, measured best)
  int chunk_minsub = 32;          // chunk kernel: overflowing chunks retried as halves (measured best with the dk bound)
  double fb_ms[2] = {0, 0};       // final fallback kernel's time and queries per map (since the
  uint64_t fb_q[2] = {0, 0};      // last reset)
  double p2_ms[2] = {0, 0};       // second chunk pass's time and queries per map
  uint64_t p2_q[2] = {0, 0};
  int last_kind[2] = {-1, -1};
  bool knn_log = false;            // GI_LOG & 4: one stderr line per chunk k-NN launch
  int knn_dbg = 0;                 // GI_KNN_DBG: k-NN kernel diagnostics (KnnArgs::dbg)
  int render_dbg = 0;              // GI_DBG: render-kernel diagnostics (RenderArgs::dbg)
  int64_t slot_limit = 0;          // GI_SLOT_LIMIT: path slots per batch (tests; 0 = 2^31)
  int elem_pretest = -1;           // GI_ELEM_PRETEST: -1 auto (make_view), 0 off, 1 on
  gi_progress_fn progress = nullptr;  // gi_set_progress
  void *progress_user = nullptr;
  int64_t progress_done = 0, progress_total = 0;  // output pixels of the current RenderImage     // k-NN kind run_knn chose last, per map (gi_render_stats)
  int sel_slack = 64;
  int knn_qpl = 1;
  DBuf ind_cont, ind_ncont;       // indirect paths that continue past their first bounce
  DBuf mc_cont, mc_ncont;         // Monte Carlo paths' indirect sub-paths
  DBuf mc_cont2, mc_ncont2;       // ... those continuing past a glass / mirror first hit
  bool mc_sub = true;             // sub-paths' first bounce in mc_sub_kernel (GI_MC_SUB=0: all in ind_cont_kernel)
  int mc_persist = -1;            // Monte Carlo paths in mc_persist_kernel with this many blocks
                                  // (GI_MC_PERSIST; 0: mc_kernel, one path per lane; -1: auto)
  DBuf prim_rgb;                  // per-primary sums of the reduction
  DBuf ind_tab, mc_tab;           // row -> tile of the tiled indirect entries; owner of MC path 64k
  DBuf ind_trows, ind_rows;       // indirect paths' tiled slots: rows per tile, their scan
  DBuf ind_masks;                 // their rows' query and base masks
  bool split_ind = true;          // continuation queue for indirect paths (else one loop per lane)
  double ind_frac = 0.25;         // continuation queue size, as a fraction of its worst case
  // render scratch
  DBuf spawn, npaths, path_off, nmc, mc_off, nind, ind_off, base, pixels, rgbf, rgb8, qcount, stats_bak;
  DBuf qpos[2], qshade[2], qkey[2], qout[2];
  bool chunk_big2 = true;            // large-K chunk k-NN: further chunk passes
  // ... the second pass's LDS candidates (1024) and a third pass's (GI_CHUNK_CAP_BIG3, test knob;
  // 0: none). r05: a 576-candidate pass at two waves per SIMD, alone or before the 1024 one, was
  // not faster (profiles/r05_chunk_pass_chain_ab.txt)
  int chunk_cap_big2 = 1024;
  int chunk_cap_big3 = 0;
  bool chunk_lane2 = true;           // lane-select chunk k-NN: second pass (480; without it C5 +1.8 %, C2 / C4 +0.4-0.6 %, r06)
  int chunk_minsub_big2 = 64;        // ... its overflowing chunks retried down to this group size
  bool chunk_dk = true;            // chunk kernel (K <= 64): centre bound from the dk bounds (measured: fewer fallbacks)
  bool chunk_fb_all = false;       // test knob: the lane-select chunk kernel hands every query to its fallback
  // k-NN instances: 0 auto (knn_general), 1 the general estimate form only (GI_KNN_GENERAL=1,
  // and after an instance without it met a query that needed it), -1 test knob: claim that no
  // render query needs it (GI_KNN_GENERAL=-1; exercises render_common's re-run)
  int knn_general_mode = 0;
  // launch-order cells per axis for the global / caustic list (> 10: 64-bit keys, gi_sort.hip
  // curve64_valid_kernel). The caustic queries crowd into foci far smaller than
  // a 10-bit cell of the scene box, where a cell's queries stay in slot order: 16-bit cells cut
  // the C4 shard's caustic k-NN 207 -> 155 ms per launch (second-pass queries 37.8 % -> 14.9 %).
  // The global list (C2: 400 M slots, one query per ~cell) keeps 32-bit keys: a 64-bit sort
  // would cost more than it saves (profiles/r05_key_bits_ab.txt).
  int key_bits[2] = {10, 16};
  // GI_ROW_ORDER (default 1): the global list's valid slots compacted from the row masks before
  // the sort (gi_sort.h curve_order_rows) instead of sorting every slot with the empty ones last
  bool row_order = true;
  bool surf_key = true;             // global list: surface keys (gi_sort.hip surface_key) instead of the 3-D curve
  bool surf_key_c = true;           // caustic list: 64-bit surface keys (surf64_valid_kernel)
  bool fb_wave = true;              // chunk kernel's last fallback: the query-per-wave kernel (r06; the per-lane one: GI_FB_WAVE=0)
  bool use_dk = true;              // wave k-NN kernel starts from per-photon K-th bounds
  DBuf qseg[2];  // K-best lists of the query-per-wave k-NN path
  size_t qcap_hint[2] = {0, 0};
  KeySortScratch keysort[2];
  int knn_kernel_kind = -1;  // -1 auto; run_knn lists the kinds
  DBuf scan_lvl[8], scan_out[8];
  // photon tracing scratch
  DBuf pcounts, poffs, pbuf;
  DBuf pkeys, pcursor, ptmp;      // single pass: slot keys, slot counter, sorted photons (host sink)
  DBuf pacc, pglob;               // maps being traced on the device (emission order), held global map
  int64_t pacc_n = 0;
  KeySortScratch psort;
  double prate[2] = {2.0, 2.0};   // stored per emitted photon in the last launch, per map
  bool photon_2pass = false;      // GI_PHOTON_2PASS=1: count pass + scan + re-trace (r03)
  // Primary samples per batch. Denser query batches make the chunk k-NN's 64 Morton-adjacent
  // queries span less of a K-neighbourhood (fewer LDS candidates per query): C2 at 2^19 / 2^20 /
  // 2^21 / 2^22 ran 6.85 / 7.44 / 7.89 / 7.69 Mpixel-samples/s. A batch is also capped by the
  // query budget below (queries per primary sample vary ~10x between scenes).
  int64_t prim_per_batch = 1 << 21;
  int64_t batch_reruns = 0;          // batches re-run smaller for 32-bit path slots (render_pixels)
  bool batch_log = false;            // GI_LOG & 2: per-batch sizes and times on stderr
  int64_t query_budget = 400000000;  // photon-map queries per batch (~120 B each: ~48 GB)
  double q_per_prim = 0.0;           // largest queries per primary sample seen so far
  double mc_app_rate[2] = {0.0, 0.0};  // per list: largest appends per Monte Carlo path seen
  float sbmin[3] = {0, 0, 0}, sbmax[3] = {1, 1, 1};
};

static void set_err(gi_ctx *c, const std::string &msg) {
  std::lock_guard<std::mutex> g(c->err_mu);
  c->err = msg;
}

#define HIPCHK(ctx, call)                                                                   \
  do {                                                                                      \
    hipError_t _e = (call);                                                                 \
    if (_e != hipSuccess) {                                                                 \
      set_err((ctx), std::string("HIP error: ") + hipGetErrorString(_e) + " at " + __FILE__ + \
                         ":" + std::to_string(__LINE__));                                   \
      return GI_ERR_HIP;                                                                    \
    }                                                                                       \
  } while (0)

namespace {

int fail(gi_ctx *c, int code, const std::string &msg) {
  set_err(c, msg);
  return code;
}

Flags make_flags(const gi_params &P) {
  Flags F;
  memset(&F, 0, sizeof F);
  F.ambient = P.ambient; F.direct = P.direct_illum; F.transmissive = P.transmissive_illum;
  F.specular = P.specular_illum; F.indirect = P.indirect_illum; F.caustic = P.caustic_illum;
  F.photon_viz = P.direct_photon_illum; F.fast_global = P.fast_global;
  F.cache = P.irradiance_cache; F.shadows = P.shadows; F.soft_shadows = P.soft_shadows;
  F.light_test = P.light_test; F.shadow_test = P.shadow_test; F.monte_carlo = P.monte_carlo;
  F.max_monte_depth = P.max_monte_depth; F.recursive_shadows = P.recursive_shadows;
  F.distrib_trans = P.distrib_transmissive; F.trans_test = P.transmissive_test;
  F.distrib_spec = P.distrib_specular; F.spec_test = P.specular_test; F.fresnel = P.fresnel;
  F.indirect_test = P.indirect_test; F.dof = P.depth_of_field; F.dof_test = P.dof_test;
  F.max_photon_depth = P.max_photon_depth;
  F.ir_air = P.ir_air;
  F.prob_absorb = P.prob_absorb;
  F.seed = P.seed;
  return F;
}

SceneView make_view(gi_ctx *c) {
  SceneView S;
  memset(&S, 0, sizeof S);
  const HostScene &H = c->scene;
  S.nodes = c->d_nodes.as<DNode>();
  S.elems = c->d_elems.as<DElement>();
  S.shapes = c->d_shapes.as<DShape>();
  S.tris = c->d_tris.as<DTri>();
  S.bvh = c->d_bvh.as<DBvhNode>();
  S.mats = c->d_mats.as<DMaterial>();
  S.lights = c->d_lights.as<DLight>();
  S.nnodes = (int)H.nodes.size();
  S.nelems = (int)H.elems.size();
  S.nlights = (int)H.lights.size();
  S.kinds = 0;
  for (const DShape &sh : H.shapes) S.kinds |= 1u << sh.kind;
  S.hard_lights = 1;
  for (const DLight &L : H.lights)
    if (L.kind == LK_AREA || L.kind == LK_RECT) S.hard_lights = 0;
  // the division-free element pre-test pays where soft lights cast many shadow rays (C3 jensen
  // +3 %) and costs where every light is hard (C2 cornell -2 %, r02 A/B); GI_ELEM_PRETEST=0/1
  S.elem_pretest = c->elem_pretest >= 0 ? c->elem_pretest : (S.hard_lights ? 0 : 1);
  // rigid scene graph: every node's 3x3 part orthonormal (then R3SceneNode's t rescale stays 1
  // and a hit's t is its world distance, which the bounded shadow walk relies on)
  S.rigid = 1;
  for (const DNode &nd : H.nodes) {
    if (nd.identity) continue;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double g = nd.T[4 * 0 + i] * nd.T[4 * 0 + j] + nd.T[4 * 1 + i] * nd.T[4 * 1 + j] +
                   nd.T[4 * 2 + i] * nd.T[4 * 2 + j];
        if (std::fabs(g - (i == j ? 1.0 : 0.0)) > 1e-12) S.rigid = 0;
      }
  }
  S.radius = H.radius;
  for (int i = 0; i < 3; i++) {
    S.centroid[i] = H.centroid[i];
    S.ambient[i] = H.ambient[i];
    S.background[i] = H.background[i];
  }
  // render.cpp:67-77
  const gi_params &P = c->P;
  double tx = tan(H.xfov), ty = tan(H.yfov);
  double ul = sqrt(H.up[0] * H.up[0] + H.up[1] * H.up[1] + H.up[2] * H.up[2]);
  double rl = sqrt(H.right[0] * H.right[0] + H.right[1] * H.right[1] + H.right[2] * H.right[2]);
  for (int i = 0; i < 3; i++) {
    S.cam.eye[i] = H.eye[i];
    S.cam.far_org[i] = H.eye[i] + H.towards[i] * P.focus_depth;
    S.cam.far_right[i] = H.right[i] * tx * P.focus_depth;
    S.cam.far_up[i] = H.up[i] * ty * P.focus_depth;
    S.cam.dof_u[i] = (ul == 0.0 ? H.up[i] : H.up[i] / ul) * P.aperture_radius;
    S.cam.dof_v[i] = (rl == 0.0 ? H.right[i] : H.right[i] / rl) * P.aperture_radius;
  }
  return S;
}

// BuildDirectionLookupTable, photon_utils.cpp:253-272
void build_lut(std::vector<double> &lut) {
  lut.assign(65536 * 3, 0.0);
  const double PI = 3.14159265358979323846;
  for (int phi = 0; phi < 256; phi++)
    for (int th = 0; th < 256; th++) {
      double tp = (phi * (2.0 * PI) / 255.0) - PI;
      double tt = (th * PI / 255.0);
      double x = sin(tt) * cos(tp), y = sin(tt) * sin(tp), z = cos(tt);
      double l = sqrt((x * x) + (y * y) + (z * z));
      if (l != 0.0) { x /= l; y /= l; z /= l; }
      int i = 256 * phi + th;
      lut[3 * i] = x; lut[3 * i + 1] = y; lut[3 * i + 2] = z;
    }
}

hipError_t upload(DBuf &b, const void *src, size_t bytes, hipStream_t st) {
  hipError_t e = b.ensure(bytes);
  if (e != hipSuccess) return e;
  if (bytes) return hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, st);
  return hipSuccess;
}

ScanTemp scan_temp(gi_ctx *c, int64_t n) {
  ScanTemp t;
  memset(&t, 0, sizeof t);
  int64_t m = n;
  for (int l = 0; l < 8; l++) {
    m = (m + 1023) / 1024;
    c->scan_lvl[l].ensure((size_t)(m + 2) * 4);
    c->scan_out[l].ensure((size_t)(m + 2) * 4);
    t.level[l] = c->scan_lvl[l].as<uint32_t>();
    t.level_out[l] = c->scan_out[l].as<uint32_t>();
  }
  t.depth = 0;
  return t;
}

int upload_map(gi_ctx *c, int mi) {
  HostMap &H = c->hmap[mi];
  DevMap &D = c->dmap[mi];
  int64_t n = (int64_t)H.storage.size();
  HIPCHK(c, upload(D.pos4, H.pos4.data(), H.pos4.size() * 4, c->stream));
  HIPCHK(c, upload(D.rgbe, H.rgbe.data(), H.rgbe.size() * 4, c->stream));
  HIPCHK(c, upload(D.nodes, H.nodes.data(), H.nodes.size() * 4, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  D.n = n;
  D.nleaves = H.nleaves;
  D.levels = H.levels;
  D.dk_k = -1;
  c->map_valid[mi] = n > 0;
  return GI_OK;
}

// the device build (f1): the emission-ordered photons go up once, the tree, the kd-order
// arrays and the permutation come back (perm only to the host, for the test seams' indices)
int build_map_device(gi_ctx *c, int mi, bool upload_storage = true) {
  HostMap &H = c->hmap[mi];
  DevMap &D = c->dmap[mi];
  const int64_t n = (int64_t)H.storage.size();
  static_assert(sizeof(gi_photon) == sizeof(KdPhoton), "photon record layout");
  if (upload_storage)  // else kd_ph already holds H.storage (traced on this device)
    HIPCHK(c, upload(c->kd_ph, H.storage.data(), (size_t)n * sizeof(gi_photon), c->stream));
  int64_t L = 1;
  while (L * c->leaf_size[mi] < n) L *= 2;
  HIPCHK(c, D.pos4.ensure((size_t)n * 16));
  HIPCHK(c, D.rgbe.ensure((size_t)n * 4));
  HIPCHK(c, D.nodes.ensure((size_t)L * 16 * 4));
  H.perm.resize(n);
  H.pos4.clear();
  H.rgbe.clear();
  H.nodes.clear();
  HIPCHK(c, kd_build_device(c->kd_ph.as<KdPhoton>(), n, c->leaf_size[mi], c->kdb, D.pos4.as<float>(),
                            D.rgbe.as<uint32_t>(), D.nodes.as<float>(),
                            reinterpret_cast<uint32_t *>(H.perm.data()), &H.nleaves, &H.levels,
                            c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  D.n = n;
  D.nleaves = H.nleaves;
  D.levels = H.levels;
  D.dk_k = -1;
  c->map_valid[mi] = n > 0;
  return GI_OK;
}

// kd tree + device arrays of map mi from its emission-ordered photons (hmap[mi].storage)
int build_map(gi_ctx *c, int mi) {
  if (c->gpu_kd) return build_map_device(c, mi);
  kd_build(c->hmap[mi], c->leaf_size[mi], std::max(1, c->P.threads));
  return upload_map(c, mi);
}

int set_map(gi_ctx *c, int mi, const gi_photon *ph, int64_t n) {
  HostMap &H = c->hmap[mi];
  H = HostMap();
  H.storage.assign(ph, ph + n);
  return build_map(c, mi);
}

// map mi from n emission-ordered photons already in device buffer `dev` (traced here): one copy
// to the host (the map's storage order, gi_get_photon_map) and, for the device build, `dev`
// becomes the build's input buffer without a re-upload
int set_map_device(gi_ctx *c, int mi, DBuf &dev, int64_t n) {
  HostMap &H = c->hmap[mi];
  H = HostMap();
  H.storage.resize(n);
  if (n) {
    HIPCHK(c, hipMemcpyAsync(H.storage.data(), dev.p, (size_t)n * sizeof(gi_photon),
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  if (!c->gpu_kd) return build_map(c, mi);
  std::swap(c->kd_ph, dev);
  return build_map_device(c, mi, false);
}

// grow a device buffer to `want` bytes keeping its first `used` bytes
hipError_t grow_keep(DBuf &b, size_t used, size_t want, hipStream_t st) {
  if (want <= b.cap && b.p) return hipSuccess;
  DBuf nb;
  hipError_t e = nb.ensure(std::max(want, b.cap + b.cap / 2));
  if (e != hipSuccess) return e;
  if (used) e = hipMemcpyAsync(nb.p, b.p, used, hipMemcpyDeviceToDevice, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  b.release();
  b = nb;
  return e;
}

// LightPower, graphics_utils.cpp:223-258
double light_power(const HostScene &S, const DLight &L) {
  const double PI = 3.14159265358979323846;
  double area = 1.0, flux = 4.0 * PI;
  if (L.kind == LK_DIR) {
    area = PI * pow(S.radius, 2.0);
    flux = 1.0;
  } else if (L.kind == LK_AREA) {
    area = PI * pow(L.radius, 2.0);
    flux /= 2.0;
  } else if (L.kind == LK_RECT) {
    double a1[3], a2[3];
    for (int i = 0; i < 3; i++) { a1[i] = L.a1[i] * L.len1; a2[i] = L.a2[i] * L.len2; }
    double cx = a1[1] * a2[2] - a1[2] * a2[1], cy = a1[2] * a2[0] - a1[0] * a2[2],
           cz = a1[0] * a2[1] - a1[1] * a2[0];
    area = sqrt((cx * cx) + (cy * cy) + (cz * cz));
    flux /= 2.0;
  } else if (L.kind == LK_SPOT) {
    double s = L.dropoff;
    flux = (2.0 * PI) / (s + 1.0) * (1.0 - pow(cos(L.cutoff), s + 1.0));
  }
  return (L.color[0] + L.color[1] + L.color[2]) * area * flux;
}

// trace photons [e0, e0+n) of one light on this context's device and append the stored ones in
// emission order: to `host` when given (device sets concatenate their parts there), else to the
// device map being built (pacc / pacc_n).
//
// One pass (PhotonTrace, photontracer.cpp:28-176): every stored photon takes a slot from one
// atomic per wave (StorePhoton's local buffer + flush, photon_utils.cpp:19-65, re-cut as a wave
// ballot + prefix) with the key (emission index, store ordinal); a radix sort of the keys and a
// gather restore emission order, so the map is the same photon for photon as the count pass +
// scan + re-trace (GI_PHOTON_2PASS=1) it replaces. A launch that stores more photons than the
// slots it was given is re-run with room (the RNG is keyed by emission index: same photons).
int trace_batch_dev(gi_ctx *c, int caustic, int light, int64_t e0, int64_t n,
                    std::vector<gi_photon> *host) {
  const int64_t CH = 1 << 22;
  for (int64_t s = 0; s < n; s += CH) {
    int64_t m = std::min(CH, n - s);
    PhotonArgs a;
    memset(&a, 0, sizeof a);
    a.S = make_view(c);
    a.F = make_flags(c->P);
    a.light = light;
    a.caustic = caustic;
    a.e0 = e0 + s;
    a.n = m;
    uint32_t total = 0;
    gi_photon_dev *sorted = nullptr;  // emission-ordered photons of this launch (device)
    if (c->photon_2pass) {
      HIPCHK(c, c->pcounts.ensure((size_t)m * 4));
      HIPCHK(c, c->poffs.ensure((size_t)(m + 1) * 4));
      a.counts = c->pcounts.as<uint32_t>();
      a.offsets = c->poffs.as<uint32_t>();
      launch_photons(a, PM_COUNT, c->stream);
      HIPCHK(c, hipGetLastError());
      ScanTemp t = scan_temp(c, m);
      HIPCHK(c, launch_scan(c->pcounts.as<uint32_t>(), c->poffs.as<uint32_t>(), m, t, c->stream));
      HIPCHK(c, hipMemcpyAsync(&total, c->poffs.as<uint32_t>() + m, 4, hipMemcpyDeviceToHost,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      if (total == 0) continue;
      HIPCHK(c, c->pbuf.ensure((size_t)total * sizeof(gi_photon_dev)));
      a.out = c->pbuf.as<gi_photon_dev>();
      launch_photons(a, PM_EMIT, c->stream);
      HIPCHK(c, hipGetLastError());
      sorted = c->pbuf.as<gi_photon_dev>();
    } else {
      int obits = 1;
      while (obits < 40 && (1LL << obits) < (int64_t)c->P.max_photon_depth) obits++;
      int jbits = 1;
      while ((1LL << jbits) < m) jbits++;
      double want = (double)m * (c->prate[caustic] * 1.25 + 0.02) + 4096.0;
      uint32_t cap = (uint32_t)std::min(want, 4.0e9);
      HIPCHK(c, c->pcursor.ensure(4));
      for (;;) {
        HIPCHK(c, c->pbuf.ensure((size_t)cap * sizeof(gi_photon_dev)));
        HIPCHK(c, c->pkeys.ensure((size_t)cap * 8));
        HIPCHK(c, hipMemsetAsync(c->pcursor.p, 0, 4, c->stream));
        a.out = c->pbuf.as<gi_photon_dev>();
        a.keys = c->pkeys.as<uint64_t>();
        a.cursor = c->pcursor.as<uint32_t>();
        a.cap = cap;
        a.obits = obits;
        launch_photons(a, PM_APPEND, c->stream);
        HIPCHK(c, hipGetLastError());
        HIPCHK(c, hipMemcpyAsync(&total, c->pcursor.p, 4, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        if (total <= cap) break;
        if ((double)total * 1.1 + 4096.0 > 4.0e9)
          return fail(c, GI_ERR_ALLOC, "photon launch stores more than 2^32 photons");
        cap = (uint32_t)((double)total * 1.1 + 4096.0);
      }
      c->prate[caustic] = (double)total / (double)m;
      if (total == 0) continue;
      uint64_t *skeys = nullptr;
      uint32_t *slots = nullptr;
      HIPCHK(c, key_order(c->pkeys.as<uint64_t>(), total, jbits + obits, c->psort, &skeys,
                          &slots, c->stream));
      gi_photon_dev *dst;
      if (host) {
        HIPCHK(c, c->ptmp.ensure((size_t)total * sizeof(gi_photon_dev)));
        dst = c->ptmp.as<gi_photon_dev>();
      } else {
        HIPCHK(c, grow_keep(c->pacc, (size_t)c->pacc_n * sizeof(gi_photon_dev),
                            (size_t)(c->pacc_n + total) * sizeof(gi_photon_dev), c->stream));
        dst = c->pacc.as<gi_photon_dev>() + c->pacc_n;
      }
      launch_photon_gather(c->pbuf.as<gi_photon_dev>(), slots, total, dst, c->stream);
      HIPCHK(c, hipGetLastError());
      sorted = dst;
    }
    if (host) {
      size_t old = host->size();
      host->resize(old + total);
      HIPCHK(c, hipMemcpyAsync(host->data() + old, sorted, (size_t)total * sizeof(gi_photon),
                               hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    } else if (sorted != c->pacc.as<gi_photon_dev>() + c->pacc_n) {  // 2-pass: append the launch
      HIPCHK(c, grow_keep(c->pacc, (size_t)c->pacc_n * sizeof(gi_photon_dev),
                          (size_t)(c->pacc_n + total) * sizeof(gi_photon_dev), c->stream));
      HIPCHK(c, hipMemcpyAsync(c->pacc.as<gi_photon_dev>() + c->pacc_n, sorted,
                               (size_t)total * sizeof(gi_photon_dev), hipMemcpyDeviceToDevice,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      c->pacc_n += total;
    } else {
      c->pacc_n += total;
    }
  }
  return GI_OK;
}

// Run fn(k, ctx_k) for every device of the set (k = 0 is this context, run on the calling
// thread, so its progress callbacks arrive where gi.h promises; each peer on a host thread of
// its own); returns the first failure, with that device's message copied into c->err.
template <typename Fn>
int on_devices(gi_ctx *c, Fn fn) {
  const int nd = 1 + (int)c->peers.size();
  if (nd == 1) return fn(0, c);
  std::vector<int> rc(nd, GI_OK);
  auto run = [&](int k, gi_ctx *d) {
    if (hipSetDevice(d->device) != hipSuccess) {
      rc[k] = fail(d, GI_ERR_HIP, "hipSetDevice failed");
      return;
    }
    try {
      rc[k] = fn(k, d);
    } catch (const std::bad_alloc &) {
      rc[k] = fail(d, GI_ERR_ALLOC, "host allocation failed");
    } catch (...) {
      rc[k] = fail(d, GI_ERR_HIP, "unexpected exception");
    }
  };
  std::vector<std::thread> th;
  for (int k = 1; k < nd; k++) th.emplace_back(run, k, c->peers[k - 1]);
  run(0, c);
  for (auto &t : th) t.join();
  hipSetDevice(c->device);
  for (int k = 0; k < nd; k++)
    if (rc[k] != GI_OK) {
      if (k) set_err(c, "device " + std::to_string(c->peers[k - 1]->device) + ": " + c->peers[k - 1]->err);
      return rc[k];
    }
  return GI_OK;
}

// trace photons [e0, e0+n) of one light: on a device set the range is cut into one contiguous
// piece per device (the RNG is keyed by emission index, so the concatenation in device order
// is the one-device result photon for photon)
int trace_batch(gi_ctx *c, int caustic, int light, int64_t e0, int64_t n,
                std::vector<gi_photon> *out) {
  const int nd = 1 + (int)c->peers.size();
  if (nd == 1 || n < 4096 * (int64_t)nd) return trace_batch_dev(c, caustic, light, e0, n, out);
  std::vector<std::vector<gi_photon>> part(nd);
  int rc = on_devices(c, [&](int k, gi_ctx *d) -> int {
    int64_t a = e0 + n * k / nd, b = e0 + n * (k + 1) / nd;
    return trace_batch_dev(d, caustic, light, a, b - a, &part[k]);
  });
  if (rc) return rc;
  for (auto &p : part) out->insert(out->end(), p.begin(), p.end());
  return GI_OK;
}

// adaptive emission rounds of Threadable_PhotonTracer (photonmap.cpp:145-257), one emitter.
// The map grows in `map` (device sets) or, when `map` is null, on this device (pacc / pacc_n).
int trace_map(gi_ctx *c, int caustic, int64_t goal, const std::vector<double> &powers,
              double total_power, std::vector<gi_photon> *map, int64_t &emitted) {
  int64_t stored = 0;
  if (!map) c->pacc_n = 0;
  emitted = 0;
  double rate = caustic ? (double)c->P.max_photon_depth : 4.0;
  double slowdown = 1.0;
  int attempts = 10;
  int nl = (int)c->scene.lights.size();
  while (stored < goal && attempts > 0) {
    int emit_goal = (int)((double)(int)(goal - stored) / rate / slowdown + 1);
    int64_t assigned = 0;
    for (int i = 0; i < nl; i++) {
      int num = (int)ceil(emit_goal * (powers[i] / total_power));
      if (c->scene.lights[i].active && num) {
        int rc = trace_batch(c, caustic, i, emitted + assigned, num, map);
        if (rc) return rc;
      }
      assigned += num;
    }
    emitted += assigned;
    stored = map ? (int64_t)map->size() : c->pacc_n;
    if (c->progress && goal > 0) c->progress(caustic ? 2 : 1, (double)stored / goal, c->progress_user);
    if (stored > 0 && emitted > 0) {
      rate = (double)stored / emitted;
      double frac = caustic ? (double)stored / goal : (double)stored / emitted;
      slowdown = (frac < 0.75) ? 2.0 : 1.0;
    } else {
      rate /= 2.0;
      attempts--;
    }
  }
  return GI_OK;
}

// device counters: ST_STRIPES copies of ST_COUNT words (gi_kernels.h wave_add), summed here
constexpr size_t ST_BYTES = (size_t)ST_STRIPES * ST_COUNT * 8;
hipError_t read_stats(gi_ctx *c, unsigned long long *out) {
  std::vector<unsigned long long> all((size_t)ST_STRIPES * ST_COUNT);
  hipError_t e = hipMemcpyAsync(all.data(), c->d_stats.p, ST_BYTES, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  for (int i = 0; i < ST_COUNT; i++) {
    out[i] = 0;
    for (int s = 0; s < ST_STRIPES; s++) out[i] += all[(size_t)s * ST_COUNT + i];
  }
  return e;
}

// KnnArgs::general: 0 when the map's filter is the disk and no material a query can carry (kd or
// the diffuse flag: queries sit on diffuse hits) has a specular term -- the device's test for the
// estimate's common form (photon_utils.cpp:98-158; gi_knn.hip wave_estimate) -- so the k-NN
// kernels can run their instances without pow
// (every_material: also those no render query can carry -- the estimate seam's per-query ones)
static int knn_general(const std::vector<DMaterial> &mats, int filter, bool every_material = false) {
  if (filter != 0) return 1;
  for (const DMaterial &m : mats) {
    if (!every_material && !(m.flags & MF_DIFFUSE) && m.max_kd == 0.0) continue;
    const bool spec = (m.flags & MF_SPECULAR) || (m.n < 0);
    if (spec || !std::isfinite(m.ks[0]) || !std::isfinite(m.ks[1]) || !std::isfinite(m.ks[2]))
      return 1;
  }
  return 0;
}

KnnArgs knn_args(gi_ctx *c, int mi) {
  KnnArgs k;
  memset(&k, 0, sizeof k);
  k.map = c->dmap[mi].view();
  k.mats = c->d_mats.as<DMaterial>();
  k.lut = c->d_lut.as<double>();
  const gi_params &P = c->P;
  k.K = mi == GI_MAP_GLOBAL ? P.global_estimate_size : P.caustic_estimate_size;
  double r = mi == GI_MAP_GLOBAL ? P.global_estimate_dist : P.caustic_estimate_dist;
  k.filter = mi == GI_MAP_GLOBAL ? P.global_filter : P.caustic_filter;
  k.r2f = (float)(r * r);
  k.rmax = r;
  k.fa = P.filter_const_a;
  k.fb = P.filter_const_b;
  k.fk = P.filter_const_k;
  k.stats = c->d_stats.as<unsigned long long>();
  k.stat_off = mi == GI_MAP_GLOBAL ? 0 : ST_KNN_MAP;
  k.sel_slack = c->sel_slack;
  k.chunk_minsub = c->chunk_minsub;
  k.qpl = c->knn_qpl;
  k.general = c->knn_general_mode > 0 ? 1 : c->knn_general_mode < 0 ? 0 : knn_general(c->scene.mats, k.filter);
  k.dbg = c->knn_dbg;
  return k;
}

// Per-photon K-th distance bounds of map mi for this launch's K and r (KdView::dk): one
// KNN_MODE_DK pass of the wave kernel with the photons themselves as queries, computed once
// per map and (K, r). The wave kernel then starts each query from the bound of the photons in
// its leaf instead of from r.
int ensure_dk(gi_ctx *c, KnnArgs &k) {
  MapExec &X = c->mx[k.stat_off ? 1 : 0];
  int mi = k.stat_off ? 1 : 0;
  DevMap &D = c->dmap[mi];
  if (!c->use_dk || D.n == 0 || k.K <= 0) return GI_OK;
  if (D.dk_k != k.K || D.dk_r2 != k.r2f) {
    D.dk_k = -1;
    HIPCHK(c, X.dk_q.ensure((size_t)D.n * 16));
    HIPCHK(c, D.dk.ensure((size_t)D.n * 4));
    launch_photon_queries(D.pos4.as<float>(), D.n, X.dk_q.as<float4>(), X.st);
    KnnArgs d = k;
    d.mode = KNN_MODE_DK;
    d.map.dk = nullptr;
    d.qpos = X.dk_q.as<float4>();
    d.qshade = nullptr;
    d.perm = nullptr;
    d.nq = D.n;
    d.q0 = 0;
    d.out_dk = D.dk.as<float>();
    d.stats = nullptr;
    d.dbg = 0;
    if (!launch_knn_wave(d, c->wave_cap_mul, X.st))
      return fail(c, GI_ERR_ARG, "k-NN bound pass: unsupported estimate size");
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(X.st));
    D.dk_k = k.K;
    D.dk_r2 = k.r2f;
  }
  k.map.dk = D.dk.as<float>();
  return GI_OK;
}

// run a k-NN launch over nq queries (chunked when the heap lives in global scratch)
int run_knn(gi_ctx *c, KnnArgs k, int64_t nq, double *ms) {
  MapExec &X = c->mx[k.stat_off ? 1 : 0];
  // Kernel choice (GI_KNN_KERNEL overrides; -1 = auto):
  //   7  chunk kernel with lane select + per-lane fallback (K <= 64, estimates): the default
  //   3  per-lane kernel, LDS heaps (K <= 128; list mode)
  //   8  large-K chunk kernel + query-per-wave fallback (K > 64, estimates; needs dk bounds)
  //   1  query-per-wave kernel (K + 64 <= 1024)
  //   0  per-lane kernel with global-memory heaps (any K)
  int kind = c->knn_kernel_kind;
  const bool list = k.mode == KNN_MODE_LIST, dkm = k.mode == KNN_MODE_DK;
  int auto_kind = (k.K <= 64) ? (list ? 3 : 7) : ((list || !c->use_dk) ? 1 : 8);
  if (kind < 0) kind = auto_kind;
  // an override that cannot serve this launch falls back to the automatic choice
  if (kind == 7 && (k.K > 64 || list)) kind = auto_kind;
  if (kind == 8 && (list || dkm || k.K + 64 > 1024 || !c->use_dk)) kind = auto_kind == 8 ? 1 : auto_kind;
  if (kind == 3 && (size_t)k.K * 512 > 64 * 1024) kind = auto_kind;
  if (kind == 1 && k.K + 64 > 1024) kind = 0;
  if (!dkm) c->last_kind[k.stat_off ? 1 : 0] = kind;
  if (kind == 8) {
    // large-K chunk kernel, then the query-per-wave kernel on what it hands over
    int rc = ensure_dk(c, k);
    if (rc) return rc;
    int64_t chunks = (nq + 63) / 64;
    int64_t grid = knn_chunk_grid(nq);
    uint32_t cap_s = (uint32_t)(64 * ((chunks + grid - 1) / grid) * ((grid + FB_QS - 1) / FB_QS));
    HIPCHK(c, X.fb_list.ensure((size_t)FB_QS * cap_s * 4));
    HIPCHK(c, X.fb_dense.ensure((size_t)nq * 4 + 4));
    HIPCHK(c, X.fb_count.ensure(FB_QS * 32 * 4));
    HIPCHK(c, hipMemsetAsync(X.fb_count.p, 0, FB_QS * 32 * 4, X.st));
    k.nq = nq;
    k.q0 = 0;
    k.fb_list = X.fb_list.as<uint32_t>();
    k.fb_count = X.fb_count.as<uint32_t>();
    k.fb_cap_s = cap_s;
    k.chunk_minsub = c->chunk_minsub_big;
    k.dk_exact = c->chunk_dk_exact ? 1 : 0;
    HIPCHK(c, hipEventRecord(X.ev0, X.st));
    if (!launch_knn_chunk_big(k, c->chunk_cap_big, X.st))
      return fail(c, GI_ERR_ARG, "k-NN launch: large-K chunk kernel unavailable");
    HIPCHK(c, hipGetLastError());
    uint32_t *dense = X.fb_dense.as<uint32_t>();
    launch_fb_compact(k.fb_list, k.fb_count, cap_s, dense, dense + nq, X.st);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(X.ev2, X.st));
    uint32_t nfb = 0;
    HIPCHK(c, hipMemcpyAsync(&nfb, dense + nq, 4, hipMemcpyDeviceToHost, X.st));
    HIPCHK(c, hipStreamSynchronize(X.st));
    X.fb_total += nfb;
    uint32_t nfb2 = nfb;
    bool ran2 = false;
    // further chunk passes over the overflowing chunks' queries, with more LDS candidates each
    // (chunk_cap_big2: 1024 by default; chunk_cap_big3 > 0 adds a third); the compacted lists
    // keep each chunk's queries together, in Morton order. What overflows the last one goes to
    // the query-per-wave kernel. Pass i reads `dense` and writes the other list (ping-pong:
    // the first pass's list is free once the second has read it).
    const int caps2[2] = {c->chunk_cap_big2, c->chunk_cap_big3};
    for (int pi = 0; pi < 2 && nfb2 && c->chunk_big2 && caps2[pi] > 0; pi++) {
      ran2 = true;
      const uint32_t nin = nfb2;
      DBuf &L = pi == 0 ? X.fb_list2 : X.fb_list;
      DBuf &Dn = pi == 0 ? X.fb_dense2 : X.fb_dense;
      DBuf &Cn = pi == 0 ? X.fb_count2 : X.fb_count;
      int64_t chunks2 = ((int64_t)nin + 63) / 64;
      int64_t grid2 = knn_chunk_grid(nin);
      uint32_t cap2 = (uint32_t)(64 * ((chunks2 + grid2 - 1) / grid2) * ((grid2 + FB_QS - 1) / FB_QS));
      HIPCHK(c, L.ensure((size_t)FB_QS * cap2 * 4));
      HIPCHK(c, Dn.ensure((size_t)nin * 4 + 4));
      HIPCHK(c, Cn.ensure(FB_QS * 32 * 4));
      HIPCHK(c, hipMemsetAsync(Cn.p, 0, FB_QS * 32 * 4, X.st));
      KnnArgs s2 = k;
      s2.perm = dense;
      s2.nq = nin;
      s2.q0 = 0;
      s2.fb_list = L.as<uint32_t>();
      s2.fb_count = Cn.as<uint32_t>();
      s2.fb_cap_s = cap2;
      s2.dbg &= ~16;
      s2.chunk_minsub = c->chunk_minsub_big2;
      if (!launch_knn_chunk_big(s2, caps2[pi], X.st))
        return fail(c, GI_ERR_ARG, "k-NN launch: large-K chunk kernel unavailable");
      HIPCHK(c, hipGetLastError());
      dense = Dn.as<uint32_t>();
      launch_fb_compact(s2.fb_list, s2.fb_count, cap2, dense, dense + nin, X.st);
      HIPCHK(c, hipGetLastError());
      HIPCHK(c, hipMemcpyAsync(&nfb2, dense + nin, 4, hipMemcpyDeviceToHost, X.st));
      HIPCHK(c, hipStreamSynchronize(X.st));
    }
    HIPCHK(c, hipEventRecord(X.ev3, X.st));
    if (nfb2) {
      KnnArgs f = k;
      f.perm = dense;
      f.nq = nfb2;
      f.q0 = 0;
      if (!launch_knn_wave(f, c->wave_cap_mul, X.st))
        return fail(c, GI_ERR_ARG, "k-NN launch: unsupported estimate size for this kernel");
      HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(X.ev1, X.st));
    if (ms) {
      HIPCHK(c, hipEventSynchronize(X.ev1));
      float t = 0, tf = 0, t2 = 0;
      HIPCHK(c, hipEventElapsedTime(&t, X.ev0, X.ev1));
      HIPCHK(c, hipEventElapsedTime(&tf, X.ev3, X.ev1));
      HIPCHK(c, hipEventElapsedTime(&t2, X.ev2, X.ev3));
      *ms += t;
      int mi = k.stat_off ? 1 : 0;
      c->fb_ms[mi] += tf;
      c->fb_q[mi] += nfb2;
      c->p2_ms[mi] += t2;
      c->p2_q[mi] += ran2 ? nfb : 0;
      if (c->knn_log)
        fprintf(stderr, "[gi] knn map %d kind 8: nq %lld chunk pass %.2f ms, second pass %u (%.2f ms), wave %u (%.2f ms)\n",
                mi, (long long)nq, t - tf - t2, nfb, t2, nfb2, tf);
    }
    return GI_OK;
  }
  if (kind == 7) {
    // chunk kernel, then the per-lane kernel on the chunks that overflowed its LDS gather
    // striped fallback list (gi_knn_chunk.hip to_fallback): block b -> stripe b % FB_QS, at most
    // 64 queries per chunk, ceil(chunks / grid) chunks per block
    int64_t chunks = (nq + 63) / 64;
    int64_t grid = knn_chunk_grid(nq);
    uint32_t cap_s = (uint32_t)(64 * ((chunks + grid - 1) / grid) * ((grid + FB_QS - 1) / FB_QS));
    HIPCHK(c, X.fb_list.ensure((size_t)FB_QS * cap_s * 4));
    HIPCHK(c, X.fb_dense.ensure((size_t)nq * 4 + 4));
    HIPCHK(c, X.fb_count.ensure(FB_QS * 32 * 4));
    HIPCHK(c, hipMemsetAsync(X.fb_count.p, 0, FB_QS * 32 * 4, X.st));
    k.nq = nq;
    k.q0 = 0;
    k.fb_list = X.fb_list.as<uint32_t>();
    k.fb_count = X.fb_count.as<uint32_t>();
    k.fb_cap_s = cap_s;
    // per-photon K-th distance bounds: the fallback's starting bound; the chunk kernel's centre
    // bound uses them only with chunk_dk (else the exact d_K(c) gather)
    const float *fb_dk = nullptr;
    if (c->use_dk && k.mode != KNN_MODE_DK) {
      int rc = ensure_dk(c, k);
      if (rc) return rc;
      fb_dk = k.map.dk;
      if (!c->chunk_dk) k.map.dk = nullptr;
    }
    const int dbg0 = k.dbg;
    if (c->chunk_fb_all) k.dbg |= 4;  // lane select skipped: all to the fallback
    HIPCHK(c, hipEventRecord(X.ev0, X.st));
    launch_knn_chunk(k, X.st);
    k.dbg = dbg0;
    HIPCHK(c, hipGetLastError());
    uint32_t *dense = X.fb_dense.as<uint32_t>();
    launch_fb_compact(k.fb_list, k.fb_count, cap_s, dense, dense + nq, X.st);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(X.ev2, X.st));
    uint32_t nfb = 0;
    HIPCHK(c, hipMemcpyAsync(&nfb, dense + nq, 4, hipMemcpyDeviceToHost, X.st));
    HIPCHK(c, hipStreamSynchronize(X.st));
    X.fb_total += nfb;
    uint32_t nfb2 = nfb;
    bool ran2 = false;
    if (nfb && c->chunk_lane2 && !c->chunk_fb_all) {
      ran2 = true;
      // second chunk pass, 480 LDS candidates, over the overflowing chunks' queries (the
      // compacted list keeps each chunk's queries together, in Morton order)
      int64_t chunks2 = ((int64_t)nfb + 63) / 64;
      int64_t grid2 = knn_chunk_grid(nfb);
      uint32_t cap2 = (uint32_t)(64 * ((chunks2 + grid2 - 1) / grid2) * ((grid2 + FB_QS - 1) / FB_QS));
      HIPCHK(c, X.fb_list2.ensure((size_t)FB_QS * cap2 * 4));
      HIPCHK(c, X.fb_dense2.ensure((size_t)nfb * 4 + 4));
      HIPCHK(c, X.fb_count2.ensure(FB_QS * 32 * 4));
      HIPCHK(c, hipMemsetAsync(X.fb_count2.p, 0, FB_QS * 32 * 4, X.st));
      KnnArgs s2 = k;
      s2.perm = dense;
      s2.nq = nfb;
      s2.q0 = 0;
      s2.fb_list = X.fb_list2.as<uint32_t>();
      s2.fb_count = X.fb_count2.as<uint32_t>();
      s2.fb_cap_s = cap2;
      s2.dbg &= ~16;
      launch_knn_chunk2(s2, X.st);
      HIPCHK(c, hipGetLastError());
      dense = X.fb_dense2.as<uint32_t>();
      launch_fb_compact(s2.fb_list, s2.fb_count, cap2, dense, dense + nfb, X.st);
      HIPCHK(c, hipGetLastError());
      HIPCHK(c, hipMemcpyAsync(&nfb2, dense + nfb, 4, hipMemcpyDeviceToHost, X.st));
      HIPCHK(c, hipStreamSynchronize(X.st));
    }
    HIPCHK(c, hipEventRecord(X.ev3, X.st));
    if (nfb2) {
      KnnArgs f = k;
      f.perm = dense;
      f.nq = nfb2;
      f.q0 = 0;
      f.map.dk = fb_dk;
      if (c->fb_wave) {
        if (!launch_knn_wave(f, c->wave_cap_mul, X.st))
          return fail(c, GI_ERR_ARG, "k-NN launch: unsupported estimate size for this kernel");
      } else {
        launch_knn_lane(f, X.st);
      }
      HIPCHK(c, hipGetLastError());
    }
    HIPCHK(c, hipEventRecord(X.ev1, X.st));
    if (ms) {
      HIPCHK(c, hipEventSynchronize(X.ev1));
      float t = 0, tf = 0, t2 = 0;
      HIPCHK(c, hipEventElapsedTime(&t, X.ev0, X.ev1));
      HIPCHK(c, hipEventElapsedTime(&tf, X.ev3, X.ev1));
      HIPCHK(c, hipEventElapsedTime(&t2, X.ev2, X.ev3));
      *ms += t;
      int mi = k.stat_off ? 1 : 0;
      c->fb_ms[mi] += tf;
      c->fb_q[mi] += nfb2;
      c->p2_ms[mi] += t2;
      c->p2_q[mi] += ran2 ? nfb : 0;
      if (c->knn_log)
        fprintf(stderr, "[gi] knn map %d kind 7: nq %lld chunk %.2f ms, second pass %u (%.2f ms), per-lane %u (%.2f ms)\n",
                mi, (long long)nq, t - tf - t2, nfb, t2, nfb2, tf);
    }
    return GI_OK;
  }
  if (kind == 3) {
    k.nq = nq;
    k.q0 = 0;
    HIPCHK(c, hipEventRecord(X.ev0, X.st));
    launch_knn_lane(k, X.st);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(X.ev1, X.st));
    if (ms) {
      HIPCHK(c, hipEventSynchronize(X.ev1));
      float t = 0;
      HIPCHK(c, hipEventElapsedTime(&t, X.ev0, X.ev1));
      *ms += t;
    }
    return GI_OK;
  }
  if (kind == 1) {
    // one query per wave; the search writes per-query K-best lists in list / DK mode (and when
    // the estimate is not fused into it), a second kernel estimates from them
    k.nq = nq;
    k.q0 = 0;
    if (k.mode == KNN_MODE_LIST) {
      k.list_idx = k.out_idx;
      k.list_d2 = k.out_d2;
      k.list_n = k.out_n;
    } else {
      size_t slots = (size_t)nq * (size_t)k.K;
      HIPCHK(c, X.list_idx.ensure(slots * 4));
      HIPCHK(c, X.list_d2.ensure(slots * 4));
      HIPCHK(c, X.list_n.ensure((size_t)nq * 4));
      k.list_idx = X.list_idx.as<int32_t>();
      k.list_d2 = X.list_d2.as<float>();
      k.list_n = X.list_n.as<int32_t>();
    }
    int rc = ensure_dk(c, k);
    if (rc) return rc;
    HIPCHK(c, hipEventRecord(X.ev0, X.st));
    if (!launch_knn_wave(k, c->wave_cap_mul, X.st))
      return fail(c, GI_ERR_ARG, "k-NN launch: unsupported estimate size for this kernel");
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(X.ev1, X.st));
    if (ms) {
      HIPCHK(c, hipEventSynchronize(X.ev1));
      float t = 0;
      HIPCHK(c, hipEventElapsedTime(&t, X.ev0, X.ev1));
      *ms += t;
    }
    return GI_OK;
  }
  // kind 0: per-lane heaps in global scratch, launched in slices of 2^20 queries
  const int64_t CH = (int64_t)(1 << 20);
  for (int64_t s = 0; s < nq; s += CH) {
    int64_t m = std::min(CH, nq - s);
    KnnArgs a = k;
    a.nq = m;
    a.q0 = s;
    {
      size_t slots = (size_t)((m + 63) / 64) * 64 * (size_t)k.K;
      HIPCHK(c, X.gheap_d2.ensure(slots * 4));
      HIPCHK(c, X.gheap_idx.ensure(slots * 4));
      a.gheap_d2 = X.gheap_d2.as<float>();
      a.gheap_idx = X.gheap_idx.as<int32_t>();
    }
    HIPCHK(c, hipEventRecord(X.ev0, X.st));
    launch_knn(a, X.st);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(X.ev1, X.st));
    if (ms) {
      HIPCHK(c, hipEventSynchronize(X.ev1));
      float t = 0;
      HIPCHK(c, hipEventElapsedTime(&t, X.ev0, X.ev1));
      *ms += t;
    }
  }
  return GI_OK;
}

// run the k-NN estimate of one query list into out[slot] (Morton-ordered launch)
// the global list's slot layout (render_pixels): primary slots, tiled indirect slots with their
// query row masks, appends from qbase (gi_sort.h curve_order_rows)
struct ListRows {
  int64_t nprim;
  const uint64_t *qmask;
  int64_t trows;
  uint32_t qbase;
};

int knn_list(gi_ctx *c, int mi, const float4 *qpos, const QShade *qshade, int64_t nq,
             double *out, double *ms, const ListRows *rows = nullptr) {
  MapExec &X = c->mx[mi];
  KnnArgs k = knn_args(c, mi);
  k.qpos = qpos;
  k.qshade = qshade;
  k.out = out;
  k.nq = nq;
  if (c->P.irradiance_cache && mi == GI_MAP_GLOBAL) {
    // the cached-radiance lookup runs thread per list slot (it reads no permutation)
    c->last_kind[mi] = 9;
    launch_cached(k, X.st);
    HIPCHK(c, hipGetLastError());
    return GI_OK;
  }
  {
    // only the valid queries are sorted and searched: the empty deterministic slots (indirect
    // paths absorbed, escaped, or whose continuation left no query; primaries without their own
    // query; Monte Carlo paths that deferred none) are ~46 % of C2's global list, and the
    // reduction never reads their outputs (their keys / row-mask bits mark them).
    uint32_t *perm = nullptr;
    if (rows && c->row_order && c->key_bits[mi] <= 10) {
      // compacted from the row masks: the empty slots are never read or sorted
      int64_t nv = 0;
      HIPCHK(c, curve_order_rows(qpos, rows->nprim, rows->qmask, rows->trows, rows->qbase, nq,
                                 c->sbmin, c->sbmax, X.sorter, &perm, &nv, X.st,
                                 c->surf_key));
      nq = nv;
      k.nq = nv;
      if (nv == 0) return GI_OK;
    } else {
      int64_t nv = 0;
      HIPCHK(c, morton_order_valid(qpos, nq, c->sbmin, c->sbmax, X.sorter, &perm, &nv, X.st,
                                   c->key_bits[mi], c->surf_key_c));
      nq = nv;
      k.nq = nv;
      if (nv == 0) return GI_OK;
    }
    k.perm = perm;
  }
  return run_knn(c, k, nq, ms);
}

// render the given output pixels into the device image buffers
int render_pixels(gi_ctx *c, int aa, int w, int h, const std::vector<int32_t> &pix_xy,
                  gi_render_stats *rs) {
  const gi_params &P = c->P;
  int af = 1 << aa;
  int dof = std::max(1, P.dof_test);
  int64_t per_pix = (int64_t)af * af * dof;
  int64_t npix_total = (int64_t)pix_xy.size() / 2;
  double knn_ms[2] = {0, 0}, launches[2] = {0, 0};
  HIPCHK(c, upload(c->pixels, pix_xy.data(), pix_xy.size() * 4, c->stream));
  HIPCHK(c, c->qcount.ensure(16));
  HIPCHK(c, c->stats_bak.ensure(ST_BYTES));
  // path slots are 32-bit: a batch whose paths (with the indirect tiles' padding) would not fit
  // is re-run at half the primary samples, as often as needed (slot_limit: GI_SLOT_LIMIT, tests)
  int64_t shrink = 1;
  uint64_t slot_limit = 0xFFFFFFF0ull;
  if (c->slot_limit > 0) slot_limit = (uint64_t)c->slot_limit;
  int64_t nbatch = 0;
  for (int64_t p0 = 0, npix = 0; p0 < npix_total; p0 += npix) {
    auto tb0 = std::chrono::steady_clock::now();
    int attempts_used = 0;
    // batch size: prim_per_batch primary samples, fewer when the query rate seen so far would
    // exceed the query budget (the first batch of a scene starts at 1/8 to measure that rate)
    int64_t prim_cap = c->prim_per_batch;
    if (c->q_per_prim > 0.0)
      prim_cap = std::min<int64_t>(prim_cap, (int64_t)(c->query_budget / c->q_per_prim));
    else
      prim_cap = std::max<int64_t>(1, prim_cap / 8);
    prim_cap = std::max<int64_t>(1, prim_cap / shrink);
    const int64_t pix_batch = std::max<int64_t>(1, prim_cap / per_pix);
    npix = std::min(pix_batch, npix_total - p0);
    int64_t nprim = npix * per_pix;
    RenderArgs a;
    memset(&a, 0, sizeof a);
    a.S = make_view(c);
    a.F = make_flags(P);
    a.pixels = c->pixels.as<int2>() + p0;
    a.npix = (int)npix;
    a.af = af;
    a.W = w * af;
    a.H = h * af;
    a.dof_test = dof;
    a.out_w = w;
    a.nprim = nprim;
    a.stats = c->d_stats.as<unsigned long long>();
    a.split_ind = c->split_ind;
    a.dbg = c->render_dbg;
    HIPCHK(c, c->spawn.ensure((size_t)nprim * sizeof(Spawn)));
    HIPCHK(c, c->npaths.ensure((size_t)nprim * 4));
    HIPCHK(c, c->path_off.ensure((size_t)(nprim + 1) * 4));
    HIPCHK(c, c->nmc.ensure((size_t)nprim * 4));
    HIPCHK(c, c->mc_off.ensure((size_t)(nprim + 1) * 4));
    HIPCHK(c, c->nind.ensure((size_t)nprim * 4));
    HIPCHK(c, c->ind_off.ensure((size_t)(nprim + 1) * 4));
    a.spawn = c->spawn.as<Spawn>();
    a.npaths = c->npaths.as<uint32_t>();
    a.nmc = c->nmc.as<uint32_t>();
    a.nind = c->nind.as<uint32_t>();
    a.path_off = c->path_off.as<uint32_t>();
    a.mc_off = c->mc_off.as<uint32_t>();
    a.ind_off = c->ind_off.as<uint32_t>();
    // counters before the primary kernel, restored if the batch is re-run smaller
    HIPCHK(c, hipMemcpyAsync(c->stats_bak.p, c->d_stats.p, ST_BYTES, hipMemcpyDeviceToDevice,
                             c->stream));
    launch_primary(a, c->stream);
    HIPCHK(c, hipGetLastError());
    ScanTemp t = scan_temp(c, nprim);
    HIPCHK(c, launch_scan(a.npaths, c->path_off.as<uint32_t>(), nprim, t, c->stream));
    HIPCHK(c, launch_scan(a.nmc, c->mc_off.as<uint32_t>(), nprim, t, c->stream));
    HIPCHK(c, launch_scan(a.nind, c->ind_off.as<uint32_t>(), nprim, t, c->stream));
    uint32_t totals[3] = {0, 0, 0};
    HIPCHK(c, hipMemcpyAsync(&totals[0], c->path_off.as<uint32_t>() + nprim, 4,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&totals[1], c->mc_off.as<uint32_t>() + nprim, 4,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipMemcpyAsync(&totals[2], c->ind_off.as<uint32_t>() + nprim, 4,
                             hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    uint32_t total_paths = totals[0];
    a.total_paths = total_paths;
    a.total_mc = totals[1];
    a.total_ind = totals[2];
    // owner tables: the path kernels find their waves' primary sample in one load
    if (a.total_mc > 0) {
      HIPCHK(c, c->mc_tab.ensure(((size_t)a.total_mc / 64 + 2) * 4));
      launch_owner_table(c->mc_off.as<uint32_t>(), nprim, c->mc_tab.as<uint32_t>(), c->stream);
      a.mc_tab = c->mc_tab.as<uint32_t>();
    }
    // the indirect paths' tiled slots (RenderArgs::ind_rows): rows per 64-primary tile, scanned
    const int64_t ntiles = (nprim + 63) / 64;
    HIPCHK(c, c->ind_trows.ensure((size_t)(ntiles + 1) * 4));
    HIPCHK(c, c->ind_rows.ensure((size_t)(ntiles + 1) * 4));
    launch_ind_tiles(a.nind, nprim, c->ind_trows.as<uint32_t>(), c->stream);
    HIPCHK(c, launch_scan(c->ind_trows.as<uint32_t>(), c->ind_rows.as<uint32_t>(), ntiles, t, c->stream));
    uint32_t trows = 0;
    HIPCHK(c, hipMemcpyAsync(&trows, c->ind_rows.as<uint32_t>() + ntiles, 4, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    const uint64_t tind = 64ull * trows;  // tiled entries (>= total_ind)
    if ((uint64_t)total_paths + tind + (uint64_t)nprim > slot_limit) {
      if (npix == 1)
        return fail(c, GI_ERR_ALLOC, "one output pixel's samples need more than 2^32 path slots");
      HIPCHK(c, hipMemcpyAsync(c->d_stats.p, c->stats_bak.p, ST_BYTES, hipMemcpyDeviceToDevice,
                               c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      shrink *= 2;
      c->batch_reruns++;
      npix = 0;  // same pixels again, half as many per batch
      continue;
    }
    a.ind_rows = c->ind_rows.as<uint32_t>();
    a.ind_g0 = total_paths;
    a.tind = (int64_t)tind;
    HIPCHK(c, c->ind_tab.ensure(((size_t)trows + 1) * 8));
    launch_ind_row_tile(a.ind_rows, ntiles, c->ind_tab.as<uint64_t>(), c->stream);
    a.ind_row_info = c->ind_tab.as<uint64_t>();
    HIPCHK(c, c->ind_masks.ensure(((size_t)trows + 1) * 16));
    a.ind_qmask = c->ind_masks.as<uint64_t>();
    a.ind_bmask = a.ind_qmask + trows + 1;
    HIPCHK(c, c->base.ensure(((size_t)total_paths + tind) * 24));
    a.base = c->base.as<double>();
    // continuation queue: stripe s takes the appends of waves w with w % IND_QS == s (<= 64
    // paths per wave, so `full` entries per stripe can never overflow); sized from the fill
    // seen so far (c->ind_frac of full), re-run with more room when a stripe overflows
    const uint64_t ind_full = 64 * ((((uint64_t)a.tind + 63) / 64 + IND_QS - 1) / IND_QS);
    if (a.split_ind && a.total_ind > 0) HIPCHK(c, c->ind_ncont.ensure(IND_QS * 32 * 4));
    // Monte Carlo paths' indirect sub-paths: at most one per path, so the worst case is sized
    if (a.split_ind && a.total_mc > 0 && a.F.indirect) {
      const uint64_t full = 64 * ((((uint64_t)a.total_mc + 63) / 64 + IND_QS - 1) / IND_QS);
      HIPCHK(c, c->mc_cont.ensure((size_t)IND_QS * full * sizeof(IndCont)));
      HIPCHK(c, c->mc_ncont.ensure(IND_QS * 32 * 4));
      a.mc_cont = c->mc_cont.as<IndCont>();
      a.mc_ncont = c->mc_ncont.as<uint32_t>();
      a.mc_cap_s = (uint32_t)full;
      // mc_persist_kernel (path counter in the spare qcount word): always with a grid given,
      // and by default (-1) where a bounce's direct light is a soft-shadow fan, the only case it
      // was measured faster (C3 +5.5 %; with hard lights the plain kernel wins: C2 -0.4 %, C4
      // -7.4 %, since the persistent waves hold every SIMD's registers while the indirect kernel
      // on the other stream waits)
      if (c->mc_persist > 0 || (c->mc_persist < 0 && !a.S.hard_lights)) {
        a.mc_next = c->qcount.as<uint32_t>() + 2;
        a.mc_persist_blocks = c->mc_persist > 0 ? c->mc_persist : 1024;
      }
      if (c->mc_sub) {
        HIPCHK(c, c->mc_cont2.ensure((size_t)IND_QS * full * sizeof(IndCont)));
        HIPCHK(c, c->mc_ncont2.ensure(IND_QS * 32 * 4));
        a.mc_cont2 = c->mc_cont2.as<IndCont>();
        a.mc_ncont2 = c->mc_ncont2.as<uint32_t>();
      }
    }
    // single Monte Carlo pass; grow the query lists and re-run on overflow
    uint32_t nq[2] = {0, 0};
    HIPCHK(c, hipMemcpyAsync(c->stats_bak.p, c->d_stats.p, ST_BYTES,
                             hipMemcpyDeviceToDevice, c->stream));
    // deterministic slots: [0, nprim) per primary sample, then (global list) the indirect
    // paths' tiled slots; Monte Carlo paths append after qbase[l]
    uint32_t qbase[2] = {(uint32_t)(nprim + tind), (uint32_t)nprim};
    a.qind_base = nprim;
    // the empty tiled slots need their QMETA_NONE only where something reads every slot: the
    // global list's sort over all slots (no row masks: GI_ROW_ORDER=0, or no indirect paths in a
    // tiled batch) and the -cache lookup (thread per slot). C5 writes ~390 M of them per batch.
    a.tiled_skip = c->row_order && c->key_bits[0] <= 10 && !P.irradiance_cache && a.ind_qmask &&
                   (a.total_ind > 0 || tind == 0);
    for (int attempt = 0; attempt < 3; attempt++) {
      for (int l = 0; l < 2; l++) {
        // capacity: the largest list seen so far (+25 %), or this batch's primaries at the
        // largest per-primary rate seen (+25 %), so that a batch larger than the ones before (the
        // first full batch after the 1/8 probe, a batch where the scene fills more of the frame)
        // does not overflow and re-run its path pass; before any rate is known, the
        // deterministic slots plus 8 appends per primary
        size_t cap = std::max<size_t>(c->qcap_hint[l], (size_t)qbase[l] + 1024);
        if (attempt == 0) {
          // the deterministic slots are known (qbase); the appends come from the batch's
          // Monte Carlo paths, whose count is known too (total_mc): at the largest appends per
          // Monte Carlo path seen so far (at least 2), +25 %
          const double per_mc = std::max(2.0, c->mc_app_rate[l]);
          size_t pred = (size_t)qbase[l] + (size_t)(1.25 * per_mc * (double)a.total_mc) + 1024;
          cap = std::max(cap, std::min<size_t>(pred, 0xFFFFFFF0u));
        }
        HIPCHK(c, c->qpos[l].ensure(cap * 16));
        HIPCHK(c, c->qshade[l].ensure(cap * sizeof(QShade)));
        HIPCHK(c, c->qkey[l].ensure(cap * 8));
        a.qpos[l] = c->qpos[l].as<float4>();
        a.qshade[l] = c->qshade[l].as<QShade>();
        a.qkey[l] = c->qkey[l].as<uint64_t>();
        a.qcap[l] = (uint32_t)std::min<size_t>(cap, 0xFFFFFFF0u);
      }
      if (a.split_ind && a.total_ind > 0) {
        uint64_t cap_s = std::min<uint64_t>(ind_full, 64 * ((uint64_t)(ind_full * c->ind_frac) / 64 + 1));
        HIPCHK(c, c->ind_cont.ensure((size_t)IND_QS * cap_s * sizeof(IndCont)));
        a.ind_cap_s = (uint32_t)cap_s;
        a.ind_cont = c->ind_cont.as<IndCont>();
        a.ind_ncont = c->ind_ncont.as<uint32_t>();
      }
      a.qcount = c->qcount.as<uint32_t>();
      HIPCHK(c, hipMemcpyAsync(c->qcount.p, qbase, 8, hipMemcpyHostToDevice, c->stream));
      if (!a.tiled_skip && tind > (uint64_t)a.total_ind) launch_ind_pad(a, c->stream);  // (never when tind = 0)
      launch_path(a, c->stream, c->stream2, c->ev_fork, c->ev_join, true);
      HIPCHK(c, hipGetLastError());
      HIPCHK(c, hipMemcpyAsync(nq, c->qcount.p, 8, hipMemcpyDeviceToHost, c->stream));
      uint32_t fills[IND_QS * 32];
      if (a.split_ind && a.total_ind > 0)
        HIPCHK(c, hipMemcpyAsync(fills, c->ind_ncont.p, sizeof fills, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      attempts_used = attempt + 1;
      bool ok = nq[0] <= a.qcap[0] && nq[1] <= a.qcap[1];
      if (a.split_ind && a.total_ind > 0) {
        uint32_t mx = 0;
        for (int q = 0; q < IND_QS; q++) mx = std::max(mx, fills[q * 32]);
        c->ind_frac = std::max(c->ind_frac, std::min(1.0, 1.25 * mx / (double)ind_full));
        if (mx > a.ind_cap_s) ok = false;
      }
      for (int l = 0; l < 2; l++)
        c->qcap_hint[l] = std::max<size_t>(c->qcap_hint[l], (size_t)(nq[l] * 1.25) + 1024);
      c->q_per_prim = std::max(c->q_per_prim, (double)((uint64_t)nq[0] + nq[1]) / (double)nprim);
      if (a.total_mc > 0)
        for (int l = 0; l < 2; l++)
          c->mc_app_rate[l] = std::max(c->mc_app_rate[l], (double)(nq[l] - qbase[l]) / (double)a.total_mc);
      if (ok) break;
      if (attempt == 2) return fail(c, GI_ERR_ALLOC, "query list overflow");
      HIPCHK(c, hipMemcpyAsync(c->d_stats.p, c->stats_bak.p, ST_BYTES,
                               hipMemcpyDeviceToDevice, c->stream));
    }
    // photon-map estimates, then a deterministic order of each list for the reduction. The
    // deterministic slots (a primary's own query at slot b; its indirect paths' at tiled slots)
    // are located by (primary, slot-in-primary); only the Monte Carlo appends after
    // qbase[l] are key-sorted and indexed per primary (CSR over the sorted keys).
    bool run[2] = {false, false};
    for (int l = 0; l < 2; l++) {
      a.nq[l] = nq[l];
      a.qapp[l] = qbase[l];
      a.qout[l] = nullptr;
      if (nq[l]) {
        HIPCHK(c, c->qout[l].ensure((size_t)nq[l] * 24));
        a.qout[l] = c->qout[l].as<double>();
        if (!c->map_valid[l])
          HIPCHK(c, hipMemsetAsync(c->qout[l].p, 0, (size_t)nq[l] * 24, c->stream));
        else
          run[l] = true;
      }
    }
    // the two maps' estimates, one after the other on the render stream (running the caustic
    // one in a worker thread on a second stream measured no faster: r02)
    int rcm[2] = {GI_OK, GI_OK};
    for (int l = 0; l < 2; l++) {
      if (!run[l]) continue;
      // the global list's launch order from its row masks (GI_ROW_ORDER, default on)
      ListRows lr{nprim, a.ind_qmask, (int64_t)(tind / 64), qbase[0]};
      const bool use_rows = l == 0 && a.ind_qmask && (a.total_ind > 0 || tind == 0);
      rcm[l] = knn_list(c, l, a.qpos[l], a.qshade[l], nq[l], c->qout[l].as<double>(),
                        rs ? &knn_ms[l] : nullptr, use_rows ? &lr : nullptr);
      if (rcm[l]) break;
    }
    for (int l = 0; l < 2; l++) {
      if (rcm[l]) return rcm[l];
      if (run[l]) launches[l]++;
    }
    for (int l = 0; l < 2; l++) {
      HIPCHK(c, c->qseg[l].ensure((size_t)(nprim + 1) * 4));
      a.qseg[l] = c->qseg[l].as<uint32_t>();
      const int64_t napp = (int64_t)nq[l] - (int64_t)qbase[l];
      if (napp <= 0) {  // no appends: empty segments for every primary
        HIPCHK(c, hipMemsetAsync(c->qseg[l].p, 0, (size_t)(nprim + 1) * 4, c->stream));
        a.skey[l] = nullptr;
        a.sslot[l] = nullptr;
        continue;
      }
      uint64_t *sk = nullptr;
      uint32_t *ss = nullptr;
      // keys: primary << 32 | slot in primary << 16 | query in path (empty slots: ~0)
      int bits = 32;
      while (bits < 64 && ((uint64_t)nprim >> (bits - 32)) != 0) bits++;
      if (bits < 64) bits++;  // room for the empty-slot key's top bits
      HIPCHK(c, key_order(a.qkey[l] + qbase[l], napp, bits, c->keysort[l], &sk, &ss, c->stream));
      a.skey[l] = sk;
      a.sslot[l] = ss;  // slots relative to qbase[l]
      launch_segments(sk, (uint32_t)napp, (uint32_t)nprim, a.qseg[l], c->stream);
      HIPCHK(c, hipGetLastError());
    }
    a.rgbf = c->rgbf.as<float>();
    a.rgb8 = c->rgb8.as<uint8_t>();
    HIPCHK(c, c->prim_rgb.ensure((size_t)nprim * 24));
    a.prim_rgb = c->prim_rgb.as<double>();
    launch_reduce(a, c->stream);
    HIPCHK(c, hipGetLastError());
    if (c->progress) c->progress(0, (double)(p0 + npix) / (double)npix_total, c->progress_user);
    if (c->batch_log) {  // GI_LOG & 2: one stderr line per batch (synchronises the batch)
      HIPCHK(c, hipStreamSynchronize(c->stream));
      double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count();
      fprintf(stderr, "[gi] batch %lld: pixels %lld primaries %lld paths %u tiled %llu mc %lld "
              "queries %u + %u, path passes %d, %.1f ms\n", (long long)nbatch, (long long)npix,
              (long long)nprim, total_paths, (unsigned long long)tind, (long long)a.total_mc,
              nq[0], nq[1], attempts_used, ms);
    }
    nbatch++;
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (rs) {
    for (int l = 0; l < 2; l++) {
      rs->knn_map_kernel_ms[l] += knn_ms[l];
      rs->knn_map_launches[l] += launches[l];
      rs->knn_kernel_ms += knn_ms[l];
      rs->knn_kernel_launches += launches[l];
    }
  }
  return GI_OK;
}

int upload_scene(gi_ctx *c) {
  HostScene &H = c->scene;
  if (H.mats.size() >= (size_t)QMETA_MAX_MATS) return fail(c, GI_ERR_UNSUPPORTED, "more than 2^26 materials");
  HIPCHK(c, upload(c->d_nodes, H.nodes.data(), H.nodes.size() * sizeof(DNode), c->stream));
  HIPCHK(c, upload(c->d_elems, H.elems.data(), H.elems.size() * sizeof(DElement), c->stream));
  HIPCHK(c, upload(c->d_shapes, H.shapes.data(), H.shapes.size() * sizeof(DShape), c->stream));
  HIPCHK(c, upload(c->d_tris, H.tris.data(), H.tris.size() * sizeof(DTri), c->stream));
  HIPCHK(c, upload(c->d_bvh, H.bvh.data(), H.bvh.size() * sizeof(DBvhNode), c->stream));
  HIPCHK(c, upload(c->d_mats, H.mats.data(), H.mats.size() * sizeof(DMaterial), c->stream));
  HIPCHK(c, upload(c->d_lights, H.lights.data(), H.lights.size() * sizeof(DLight), c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->have_scene = true;
  c->map_valid[0] = c->map_valid[1] = false;
  c->q_per_prim = 0.0;  // the batch size is re-measured on the new scene
  c->mc_app_rate[0] = c->mc_app_rate[1] = 0.0;
  for (int i = 0; i < 3; i++) {
    c->sbmin[i] = (float)H.bmin[i];
    c->sbmax[i] = (float)H.bmax[i];
  }
  return GI_OK;
}

// the first device's photon maps (host copies + kd trees) and parameters onto the others
int replicate_maps(gi_ctx *c) {
  if (c->peers.empty()) return GI_OK;
  return on_devices(c, [&](int k, gi_ctx *d) -> int {
    if (k == 0) return GI_OK;
    d->P = c->P;
    for (int m = 0; m < 2; m++) {
      d->hmap[m] = c->hmap[m];
      // a host-built tree is uploaded; a device-built one is rebuilt on each device (the build
      // is a deterministic function of the photons: the same tree everywhere)
      int rc = d->hmap[m].pos4.empty() && !d->hmap[m].storage.empty() ? build_map_device(d, m)
                                                                        : upload_map(d, m);
      if (rc) return rc;
    }
    return (int)GI_OK;
  });
}

int check_ready(gi_ctx *c) {
  if (!c->have_scene) return fail(c, GI_ERR_STATE, "no scene loaded (gi_read_scene)");
  if (c->scene.unsupported_depth)
    return fail(c, GI_ERR_UNSUPPORTED, "scene graph deeper than 16 levels");
  if (c->scene.unsupported_shapes)
    return fail(c, GI_ERR_UNSUPPORTED,
                "scene contains cone shapes: not yet on the device path");
  return GI_OK;
}

}  // namespace

// =======================================================================================
// C-ABI
// =======================================================================================
extern "C" {

int gi_create(gi_ctx **out, int dev) {
  *out = nullptr;
  gi_ctx *c = new gi_ctx();
  c->device = dev;
  gi_params_default(&c->P);
  if (hipSetDevice(dev) != hipSuccess) { delete c; return GI_ERR_HIP; }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return GI_ERR_HIP; }
  // (stream priorities for either stream measured no different: r06)
  if (hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess) c->stream2 = nullptr;
  hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming);
  hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming);
  for (int m = 0; m < 2; m++) {
    c->mx[m].st = c->stream;
    hipEventCreate(&c->mx[m].ev0);
    hipEventCreate(&c->mx[m].ev1);
    hipEventCreate(&c->mx[m].ev2);
    hipEventCreate(&c->mx[m].ev3);
  }
  std::vector<double> lut;
  build_lut(lut);
  if (upload(c->d_lut, lut.data(), lut.size() * 8, c->stream) != hipSuccess ||
      c->d_stats.ensure(ST_BYTES) != hipSuccess) {
    delete c;
    return GI_ERR_HIP;
  }
  hipStreamSynchronize(c->stream);
  // diagnostics and the exactness-tested alternatives (tests/test_gpu_*.py select them)
  c->batch_log = (log_bits() & 2) != 0;
  c->knn_log = (log_bits() & 4) != 0;
  c->knn_dbg = (int)env_num("GI_KNN_DBG", 0);
  c->render_dbg = (int)env_num("GI_DBG", 0);
  c->slot_limit = (int64_t)env_num("GI_SLOT_LIMIT", 0);
  if (const int ls = (int)env_num("GI_LEAF_SIZE", 0); ls > 0) c->leaf_size[0] = c->leaf_size[1] = ls;
  c->gpu_kd = env_num("GI_HOST_KD", 0) == 0;                      // 1: the host kd build
  c->photon_2pass = env_num("GI_PHOTON_2PASS", c->photon_2pass) != 0;
  c->prate[0] = c->prate[1] = std::max(0.0, env_num("GI_PHOTON_RATE0", c->prate[0]));
  c->chunk_minsub_big = std::min(64, std::max(1, (int)env_num("GI_CHUNK_MINSUB_BIG", c->chunk_minsub_big)));
  c->chunk_dk_exact = env_num("GI_CHUNK_DK_EXACT", c->chunk_dk_exact) != 0;
  c->chunk_cap_big3 = (int)env_num("GI_CHUNK_CAP_BIG3", c->chunk_cap_big3);
  c->chunk_minsub = std::min(64, std::max(1, (int)env_num("GI_CHUNK_MINSUB", c->chunk_minsub)));
  c->split_ind = env_num("GI_SPLIT_IND", c->split_ind) != 0;
  c->knn_general_mode = std::max(-1, std::min(1, (int)env_num("GI_KNN_GENERAL", c->knn_general_mode)));
  c->use_dk = env_num("GI_KNN_DK", c->use_dk) != 0;
  c->chunk_dk = env_num("GI_CHUNK_DK", c->chunk_dk) != 0;
  c->mc_sub = env_num("GI_MC_SUB", c->mc_sub) != 0;
  c->mc_persist = std::max(-1, (int)env_num("GI_MC_PERSIST", c->mc_persist));
  c->elem_pretest = env_num("GI_ELEM_PRETEST", c->elem_pretest) != 0;
  c->chunk_fb_all = env_num("GI_CHUNK_FB_ALL", c->chunk_fb_all) != 0;
  c->ind_frac = std::min(1.0, std::max(1e-6, env_num("GI_IND_FRAC", c->ind_frac)));
  c->knn_kernel_kind = (int)env_num("GI_KNN_KERNEL", c->knn_kernel_kind);
  c->row_order = env_num("GI_ROW_ORDER", c->row_order) != 0;
  c->surf_key = env_num("GI_SURF_KEY", c->surf_key) != 0;
  c->surf_key_c = env_num("GI_SURF_KEY_C", c->surf_key_c) != 0;
  c->fb_wave = env_num("GI_FB_WAVE", c->fb_wave) != 0;
  *out = c;
  return GI_OK;
}

int gi_create_devices(gi_ctx **out, const gi_device_set *set) {
  if (!out || !set || set->count < 1 || set->count > GI_MAX_DEVICES) return GI_ERR_ARG;
  *out = nullptr;
  gi_ctx *c = nullptr;
  int rc = gi_create(&c, set->devices[0]);
  if (rc) return rc;
  bool distinct = true;
  for (int k = 1; k < set->count; k++) {
    gi_ctx *d = nullptr;
    rc = gi_create(&d, set->devices[k]);
    if (rc) {
      gi_destroy(c);
      return rc;
    }
    c->peers.push_back(d);
    for (int j = 0; j < k; j++) distinct = distinct && set->devices[j] != set->devices[k];
  }
  if (set->count > 1 && distinct) {
    if (!g_rccl.load()) {
      gi_destroy(c);
      return GI_ERR_UNSUPPORTED;
    }
    c->comms.assign(set->count, nullptr);
    ncclResult_t r = g_rccl.commInitAll(c->comms.data(), set->count, set->devices);
    if (r != ncclSuccess) {
      c->comms.clear();
      gi_destroy(c);
      return GI_ERR_HIP;
    }
  }
  hipSetDevice(c->device);
  *out = c;
  return GI_OK;
}

int gi_device_info(const gi_ctx *c, int max, int *ndev, int *devices, int *pci_bus,
                   int *comm_rank, int *comm_count) {
  if (!c || !ndev || max < 0) return GI_ERR_ARG;
  const int nd = 1 + (int)c->peers.size();
  *ndev = nd;
  for (int k = 0; k < nd && k < max; k++) {
    const gi_ctx *d = k ? c->peers[k - 1] : c;
    if (devices) devices[k] = d->device;
    if (pci_bus) {
      int bus = -1;
      if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, d->device) != hipSuccess) bus = -1;
      pci_bus[k] = bus;
    }
    if (comm_rank) {
      int r = -1;
      if (k < (int)c->comms.size() && c->comms[k] && g_rccl.commUserRank &&
          g_rccl.commUserRank(c->comms[k], &r) != ncclSuccess)
        r = -1;
      comm_rank[k] = r;
    }
  }
  if (comm_count) {
    int n = 0;
    if (!c->comms.empty() && c->comms[0] && g_rccl.commCount &&
        g_rccl.commCount(c->comms[0], &n) != ncclSuccess)
      n = 0;
    *comm_count = n;
  }
  return GI_OK;
}

// the calling thread's current HIP device, restored on scope exit (the packed entry points run
// inside processes whose torch shares that device setting)
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    hipSetDevice(d);
  }
  ~DeviceScope() {
    if (prev >= 0) hipSetDevice(prev);
  }
};

// the render's and the photon tracer's device scratch (everything but the scene, the maps, the
// counters and the streams); the next call re-allocates what it needs
static void release_scratch(gi_ctx *c) {
  DBuf *bufs[] = {&c->spawn, &c->npaths, &c->path_off, &c->nmc, &c->mc_off, &c->nind,
                  &c->ind_off, &c->base, &c->pixels, &c->rgbf, &c->rgb8, &c->stats_bak,
                  &c->pcounts, &c->poffs, &c->pbuf, &c->pkeys, &c->pcursor, &c->ptmp, &c->pacc,
                  &c->pglob, &c->ind_cont, &c->ind_ncont, &c->mc_cont, &c->mc_ncont,
                  &c->mc_cont2, &c->mc_ncont2, &c->prim_rgb, &c->ind_tab, &c->mc_tab,
                  &c->ind_trows, &c->ind_rows, &c->ind_masks, &c->pack};
  for (DBuf *b : bufs) b->release();
  for (auto &b : c->recv) b.release();
  for (auto &b : c->peer_pix) b.release();
  for (int m = 0; m < 2; m++) {
    MapExec &X = c->mx[m];
    DBuf *xb[] = {&X.list_idx, &X.list_d2, &X.list_n, &X.gheap_d2, &X.gheap_idx, &X.fb_list, &X.fb_count,
                  &X.fb_dense, &X.fb_list2, &X.fb_count2, &X.fb_dense2, &X.dk_q};
    for (DBuf *b : xb) b->release();
    sort_scratch_release(X.sorter);
  }
  for (int l = 0; l < 2; l++) {
    c->qpos[l].release(); c->qshade[l].release(); c->qkey[l].release(); c->qout[l].release();
    c->qseg[l].release();
    sort_scratch_release(c->keysort[l]);
  }
  sort_scratch_release(c->psort);
  for (int l = 0; l < 8; l++) { c->scan_lvl[l].release(); c->scan_out[l].release(); }
  c->kdb.release();
  c->kd_ph.release();
}

int gi_release_scratch(gi_ctx *c) {
  if (!c) return GI_ERR_ARG;
  DeviceScope scope(c->device);  // the caller's current device is restored on return
  for (gi_ctx *d : c->peers) {
    hipSetDevice(d->device);
    hipDeviceSynchronize();
    release_scratch(d);
  }
  hipSetDevice(c->device);
  hipDeviceSynchronize();
  release_scratch(c);
  return GI_OK;
}

void gi_destroy(gi_ctx *c) {
  if (!c) return;
  for (ncclComm_t m : c->comms)
    if (m) g_rccl.commDestroy(m);
  c->comms.clear();
  for (gi_ctx *d : c->peers) gi_destroy(d);
  c->peers.clear();
  hipSetDevice(c->device);
  release_scratch(c);
  DBuf *bufs[] = {&c->d_nodes, &c->d_elems, &c->d_shapes, &c->d_tris, &c->d_bvh, &c->d_mats,
                  &c->d_lights, &c->d_lut, &c->d_stats, &c->qcount};
  for (DBuf *b : bufs) b->release();
  for (int m = 0; m < 2; m++) {
    MapExec &X = c->mx[m];
    if (X.ev0) hipEventDestroy(X.ev0);
    if (X.ev1) hipEventDestroy(X.ev1);
    if (X.ev2) hipEventDestroy(X.ev2);
    if (X.ev3) hipEventDestroy(X.ev3);
  }
  for (int m = 0; m < 2; m++) {
    c->dmap[m].pos4.release();
    c->dmap[m].rgbe.release();
    c->dmap[m].nodes.release();
    c->dmap[m].dk.release();
  }
  if (c->ev_fork) hipEventDestroy(c->ev_fork);
  if (c->ev_join) hipEventDestroy(c->ev_join);
  if (c->stream2) hipStreamDestroy(c->stream2);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

const char *gi_last_error(const gi_ctx *c) { return c ? c->err.c_str() : "null context"; }

int gi_set_progress(gi_ctx *c, gi_progress_fn fn, void *user) {
  if (!c) return GI_ERR_ARG;
  c->progress = fn;  // device 0 reports for a device set (its share of the pixels)
  c->progress_user = user;
  return GI_OK;
}

int gi_set_params(gi_ctx *c, const gi_params *p) {
  if (!c || !p) return GI_ERR_ARG;
  c->P = *p;
  c->have_params = true;
  for (gi_ctx *d : c->peers) {
    d->P = *p;
    d->have_params = true;
  }
  return GI_OK;
}

int gi_read_scene(gi_ctx *c, const char *path, int real) {
  if (!c || !path) return GI_ERR_ARG;
  hipSetDevice(c->device);
  std::string err;
  HostScene S;
  if (!load_scene(path, real != 0, S, err)) return fail(c, GI_ERR_IO, err);
  c->scene = std::move(S);
  // the device set shares the host scene; every device gets its own copy of the arrays
  return on_devices(c, [&](int k, gi_ctx *d) -> int {
    if (k) d->scene = c->scene;
    return upload_scene(d);
  });
}

int gi_scene_info(gi_ctx *c, int *nnodes, int *nlights, int *nprims, double *radius) {
  if (!c || !c->have_scene) return GI_ERR_STATE;
  if (nnodes) *nnodes = (int)c->scene.nodes.size();
  if (nlights) *nlights = (int)c->scene.lights.size();
  if (nprims) *nprims = (int)c->scene.shapes.size();
  if (radius) *radius = c->scene.radius;
  return GI_OK;
}

// MapPhotons, photonmap.cpp:260-436
int gi_map_photons(gi_ctx *c, gi_photon_stats *st) {
  if (!c) return GI_ERR_ARG;
  hipSetDevice(c->device);
  int rc = check_ready(c);
  if (rc) return rc;
  auto t0 = std::chrono::steady_clock::now();
  gi_params &P = c->P;
  for (int m = 0; m < 2; m++) { c->hmap[m] = HostMap(); c->map_valid[m] = false; }
  int nl = (int)c->scene.lights.size();
  int64_t gem = 0, cem = 0;
  if (st) memset(st, 0, sizeof *st);
  if (nl <= 0) return GI_OK;
  std::vector<double> powers(nl, 0.0);
  double total = 0;
  for (int i = 0; i < nl; i++) {
    if (!c->scene.lights[i].active) continue;
    powers[i] = light_power(c->scene, c->scene.lights[i]);
    total += powers[i];
  }
  if (total <= 0) return GI_OK;
  // one device: the maps grow on the device across the emission rounds (pacc; the global map is
  // then held in pglob while the caustic map is traced); device sets: on the host
  const bool on_dev = c->peers.empty();
  std::vector<gi_photon> gph, cph;
  int64_t gn = 0, cn = 0;
  if (P.indirect_illum || P.direct_photon_illum) {
    rc = trace_map(c, 0, P.global_photon_count, powers, total, on_dev ? nullptr : &gph, gem);
    if (rc) return rc;
    gn = on_dev ? c->pacc_n : (int64_t)gph.size();
    if (on_dev) std::swap(c->pglob, c->pacc);
  }
  if (P.caustic_illum) {
    rc = trace_map(c, 1, P.caustic_photon_count, powers, total, on_dev ? nullptr : &cph, cem);
    if (rc) return rc;
    cn = on_dev ? c->pacc_n : (int64_t)cph.size();
  }
  auto t1 = std::chrono::steady_clock::now();
  // power rescale (Q9), photonmap.cpp:339-361: RGBE -> colour * total / emitted -> RGBE
  auto rescale = [&](std::vector<gi_photon> &v, DBuf &dv, int64_t n, int64_t emitted) -> int {
    double pp = total / (double)emitted;
    if (on_dev) {
      launch_photon_rescale(dv.as<gi_photon_dev>(), n, pp, c->stream);
      HIPCHK(c, hipGetLastError());
      return GI_OK;
    }
    for (auto &p : v) {
      double col[3];
      rgbe_dec(p.rgbe, col);
      for (int i = 0; i < 3; i++) col[i] *= pp;
      rgbe_enc(col, p.rgbe);
    }
    return GI_OK;
  };
  if ((P.indirect_illum || P.direct_photon_illum) && gn > 0) {
    P.global_photon_count = (int)gn;
    if ((rc = rescale(gph, c->pglob, gn, gem))) return rc;
  } else if (P.indirect_illum || P.direct_photon_illum) {
    P.indirect_illum = 0;
    P.direct_photon_illum = 0;
  }
  if (P.caustic_illum && cn > 0) {
    P.caustic_photon_count = (int)cn;
    if ((rc = rescale(cph, c->pacc, cn, cem))) return rc;
  } else if (P.caustic_illum) {
    P.caustic_illum = 0;
  }
  if (on_dev) {
    rc = set_map_device(c, GI_MAP_GLOBAL, c->pglob, gn);
    if (rc) return rc;
    rc = set_map_device(c, GI_MAP_CAUSTIC, c->pacc, cn);
    if (rc) return rc;
    // tracing scratch is not needed by the render
    DBuf *rel[] = {&c->pbuf, &c->pkeys, &c->ptmp, &c->pacc, &c->pglob};
    for (DBuf *b : rel) b->release();
    sort_scratch_release(c->psort);
    c->pacc_n = 0;
  } else {
    rc = set_map(c, GI_MAP_GLOBAL, gph.data(), (int64_t)gph.size());
    if (rc) return rc;
    rc = set_map(c, GI_MAP_CAUSTIC, cph.data(), (int64_t)cph.size());
    if (rc) return rc;
  }
  auto t2 = std::chrono::steady_clock::now();
  // irradiance cache, photonmap.cpp:381-413: irradiance = own power + EstimateIrradiance
  if (P.irradiance_cache && (P.indirect_illum || P.direct_photon_illum) && gn > 0) {
    HostMap &H = c->hmap[GI_MAP_GLOBAL];
    int64_t n = (int64_t)H.storage.size();
    std::vector<float> q(4 * n);
    for (int64_t i = 0; i < n; i++) {
      q[4 * i] = H.storage[i].pos[0];
      q[4 * i + 1] = H.storage[i].pos[1];
      q[4 * i + 2] = H.storage[i].pos[2];
      q[4 * i + 3] = 0;
    }
    DBuf dq, dout;
    HIPCHK(c, upload(dq, q.data(), q.size() * 4, c->stream));
    HIPCHK(c, dout.ensure((size_t)n * 24));
    KnnArgs k = knn_args(c, GI_MAP_GLOBAL);
    k.mode = KNN_MODE_IRRADIANCE;
    k.qpos = dq.as<float4>();
    k.out = dout.as<double>();
    k.stats = nullptr;
    // Morton order, as for the render's queries: the chunk kernel's 64-query chunks are then
    // spatial neighbourhoods (emission order scatters them over the scene)
    uint32_t *iperm = nullptr;
    HIPCHK(c, morton_order(dq.as<float4>(), n, c->sbmin, c->sbmax, c->mx[0].sorter, &iperm, c->stream));
    k.perm = iperm;
    rc = run_knn(c, k, n, nullptr);
    if (rc) return rc;
    std::vector<double> irr(3 * n);
    HIPCHK(c, hipMemcpyAsync(irr.data(), dout.p, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    dq.release();
    dout.release();
    std::vector<gi_photon> cached = H.storage;
    for (int64_t i = 0; i < n; i++) {
      double col[3];
      rgbe_dec(cached[i].rgbe, col);
      for (int j = 0; j < 3; j++) col[j] += irr[3 * i + j];
      rgbe_enc(col, cached[i].rgbe);
    }
    rc = set_map(c, GI_MAP_GLOBAL, cached.data(), n);
    if (rc) return rc;
  }
  rc = replicate_maps(c);
  if (rc) return rc;
  auto t3 = std::chrono::steady_clock::now();
  // the k-NN kernels' per-photon K-th distance bounds (ensure_dk), for the estimate sizes and
  // distances the render will use: part of building the maps, so timed here and not inside
  // the first RenderImage
  rc = on_devices(c, [&](int, gi_ctx *d) -> int {
    for (int m = 0; m < 2; m++) {
      if (!d->map_valid[m] || d->dmap[m].n == 0) continue;
      KnnArgs k = knn_args(d, m);
      if (k.K <= 0 || k.K + 64 > 1024) continue;  // only the per-lane global-heap kernel
      int r = ensure_dk(d, k);
      if (r) return r;
    }
    return (int)GI_OK;
  });
  if (rc) return rc;
  auto t4 = std::chrono::steady_clock::now();
  if (st) {
    st->global_stored = (int64_t)c->hmap[0].storage.size();
    st->caustic_stored = (int64_t)c->hmap[1].storage.size();
    st->global_emitted = gem;
    st->caustic_emitted = cem;
    st->trace_s = std::chrono::duration<double>(t1 - t0).count();
    // kd_s: the tree builds, their replication and the k-NN bound pass
    st->kd_s = std::chrono::duration<double>((t2 - t1) + (t4 - t3)).count();
    st->irradiance_s = std::chrono::duration<double>(t3 - t2).count();
    st->total_s = std::chrono::duration<double>(t4 - t0).count();
  }
  return GI_OK;
}

int gi_set_photon_map(gi_ctx *c, int map, const gi_photon *ph, int64_t n) {
  if (!c || map < 0 || map > 1 || (n > 0 && !ph)) return GI_ERR_ARG;
  hipSetDevice(c->device);
  int rc = set_map(c, map, ph, n);
  if (rc) return rc;
  return replicate_maps(c);
}

int gi_get_photon_map(gi_ctx *c, int map, gi_photon *out, int64_t cap, int64_t *n) {
  if (!c || map < 0 || map > 1) return GI_ERR_ARG;
  const auto &v = c->hmap[map].storage;
  if (n) *n = (int64_t)v.size();
  if (out) {
    if ((int64_t)v.size() > cap) return fail(c, GI_ERR_ARG, "capacity too small");
    memcpy(out, v.data(), v.size() * sizeof(gi_photon));
  }
  return GI_OK;
}

int gi_get_kd_tree(gi_ctx *c, int map, float *nodes, int64_t node_floats, int32_t *perm,
                   int64_t perm_cap, int32_t *nleaves, int64_t *n) {
  if (!c || map < 0 || map > 1) return GI_ERR_ARG;
  hipSetDevice(c->device);
  const HostMap &H = c->hmap[map];
  const DevMap &D = c->dmap[map];
  const int64_t nn = (int64_t)H.storage.size();
  if (n) *n = nn;
  if (nleaves) *nleaves = H.nleaves;
  const int64_t nf = (int64_t)16 * H.nleaves;
  if (nodes) {
    if (node_floats < nf) return fail(c, GI_ERR_ARG, "node capacity too small");
    if (D.nodes.p && D.nodes.cap >= (size_t)nf * 4) {
      HIPCHK(c, hipMemcpyAsync(nodes, D.nodes.p, (size_t)nf * 4, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    } else {
      memset(nodes, 0, (size_t)nf * 4);
    }
  }
  if (perm) {
    if (perm_cap < nn) return fail(c, GI_ERR_ARG, "capacity too small");
    memcpy(perm, H.perm.data(), (size_t)nn * 4);
  }
  return GI_OK;
}

static int render_common(gi_ctx *c, int aa, int w, int h, const std::vector<int32_t> &pix,
                         uint8_t *rgb8, float *rgbf, gi_render_stats *st, bool keep_rgbf) {
  int rc = check_ready(c);
  if (rc) return rc;
  if (aa < 0 || w <= 0 || h <= 0) return fail(c, GI_ERR_ARG, "bad image size");
  auto t0 = std::chrono::steady_clock::now();
  size_t npx = (size_t)w * h * 3;
  HIPCHK(c, c->rgbf.ensure(npx * 4));
  HIPCHK(c, c->rgb8.ensure(npx));
  if (keep_rgbf && rgbf) {
    HIPCHK(c, hipMemcpyAsync(c->rgbf.p, rgbf, npx * 4, hipMemcpyHostToDevice, c->stream));
  } else {
    HIPCHK(c, hipMemsetAsync(c->rgbf.p, 0, npx * 4, c->stream));
  }
  HIPCHK(c, hipMemsetAsync(c->rgb8.p, 0, npx, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_stats.p, 0, ST_BYTES, c->stream));
  c->fb_ms[0] = c->fb_ms[1] = 0;
  c->fb_q[0] = c->fb_q[1] = 0;
  c->p2_ms[0] = c->p2_ms[1] = 0;
  c->p2_q[0] = c->p2_q[1] = 0;
  c->last_kind[0] = c->last_kind[1] = -1;
  gi_render_stats local;
  unsigned long long s[ST_COUNT];
  for (int pass = 0;; pass++) {
    memset(&local, 0, sizeof local);
    rc = render_pixels(c, aa, w, h, pix, &local);
    if (rc) return rc;
    HIPCHK(c, read_stats(c, s));
    if (s[ST_GEN_MISS] == 0) break;
    // a k-NN instance without the general estimate form (KnnArgs::general == 0, knn_general)
    // met a query that needed it and wrote NaN: the host's material check missed a query site.
    // Render again with the general instances only (kept for this context), never return NaN.
    if (pass > 0 || c->knn_general_mode > 0)
      return fail(c, GI_ERR_STATE, "k-NN estimate: general-form query in a general instance");
    fprintf(stderr, "[gi] %llu k-NN queries needed the general estimate form; re-rendering with "
            "the general k-NN instances\n", s[ST_GEN_MISS]);
    c->knn_general_mode = 1;
    if (keep_rgbf && rgbf) {
      HIPCHK(c, hipMemcpyAsync(c->rgbf.p, rgbf, npx * 4, hipMemcpyHostToDevice, c->stream));
    } else {
      HIPCHK(c, hipMemsetAsync(c->rgbf.p, 0, npx * 4, c->stream));
    }
    HIPCHK(c, hipMemsetAsync(c->rgb8.p, 0, npx, c->stream));
    HIPCHK(c, hipMemsetAsync(c->d_stats.p, 0, ST_BYTES, c->stream));
    c->fb_ms[0] = c->fb_ms[1] = 0;
    c->fb_q[0] = c->fb_q[1] = 0;
    c->p2_ms[0] = c->p2_ms[1] = 0;
    c->p2_q[0] = c->p2_q[1] = 0;
  }
  if (rgbf) HIPCHK(c, hipMemcpyAsync(rgbf, c->rgbf.p, npx * 4, hipMemcpyDeviceToHost, c->stream));
  if (rgb8) HIPCHK(c, hipMemcpyAsync(rgb8, c->rgb8.p, npx, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->knn_dbg & 16) {
    fprintf(stderr, "[gi] k-NN phase cycles (sum over waves):");
    for (int i = 0; i < 16; i++) fprintf(stderr, " %llu", s[ST_PHASE + i]);
    fprintf(stderr, "\n");
  }
  if (st) {
    st->screen_rays = s[ST_RAY];
    st->shadow_rays = s[ST_SHADOW];
    st->monte_carlo_rays = s[ST_MONTE];
    st->transmissive_samples = s[ST_TRANS];
    st->specular_samples = s[ST_SPEC];
    st->indirect_samples = s[ST_INDIRECT];
    st->caustic_samples = s[ST_CAUSTIC];
    for (int m = 0; m < 2; m++) {
      st->knn_map_queries[m] = s[ST_KNN + m * ST_KNN_MAP];
      st->knn_map_photons[m] = s[ST_KNN_PHOTONS + m * ST_KNN_MAP];
      st->knn_map_visited[m] = s[ST_KNN_VISITED + m * ST_KNN_MAP];
      st->knn_map_kernel_ms[m] = local.knn_map_kernel_ms[m];
      st->knn_map_launches[m] = local.knn_map_launches[m];
      st->knn_map_fallback_ms[m] = c->fb_ms[m];
      st->knn_map_fallback_queries[m] = c->fb_q[m];
      st->knn_map_pass2_ms[m] = c->p2_ms[m];
      st->knn_map_pass2_queries[m] = c->p2_q[m];
      st->knn_map_kind[m] = c->last_kind[m];
    }
    st->knn_queries = st->knn_map_queries[0] + st->knn_map_queries[1];
    st->knn_photons = st->knn_map_photons[0] + st->knn_map_photons[1];
    st->knn_visited = st->knn_map_visited[0] + st->knn_map_visited[1];
    st->knn_kernel_ms = local.knn_kernel_ms;
    st->knn_kernel_launches = local.knn_kernel_launches;
    st->render_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  return GI_OK;
}

// output pixels of the tiles (tile x tile, row-major tile id t = ty * tx + tx_i) that shard owns:
// tile (tx_i, ty_i) goes to shard (tx_i + ty_i) % nshards, a diagonal deal, so every run of
// nshards tiles along a row or a column meets every shard (t % nshards with tx a multiple of
// nshards deals whole tile columns, and a compact expensive region -- the glass sphere -- then
// lands on a few shards in proportion to the columns it spans)
static std::vector<int32_t> shard_pixels(int w, int h, int tile, int shard, int nshards) {
  int tx = (w + tile - 1) / tile, ty = (h + tile - 1) / tile;
  std::vector<int32_t> pix;
  for (int t = 0; t < tx * ty; t++) {
    if (((t % tx) + (t / tx)) % nshards != shard) continue;
    int x0 = (t % tx) * tile, y0 = (t / tx) * tile;
    for (int y = y0; y < std::min(h, y0 + tile); y++)
      for (int x = x0; x < std::min(w, x0 + tile); x++) {
        pix.push_back(x);
        pix.push_back(y);
      }
  }
  return pix;
}

// RenderImage on a device set: device k renders the 16x16 output tiles of
// shard k (shard_pixels: the reference's column interleave, render.cpp:90, re-cut as diagonally
// dealt tiles), packs its
// pixels (16 B each) and sends them to the first device: ncclSend / ncclRecv in one group over
// xGMI when the devices are distinct (each peer's stream feeds its own link into device 0), a
// peer copy otherwise. Device 0 scatters them into the image; nothing else is exchanged.
static int render_multi(gi_ctx *c, int aa, int w, int h, uint8_t *rgb8, float *rgbf,
                        gi_render_stats *st) {
  const int nd = 1 + (int)c->peers.size();
  const int tile = 16;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::vector<int32_t>> pix(nd);
  std::vector<gi_render_stats> ls(nd);
  for (int k = 0; k < nd; k++) {
    pix[k] = shard_pixels(w, h, tile, k, nd);
    memset(&ls[k], 0, sizeof ls[k]);
  }
  int rc = on_devices(c, [&](int k, gi_ctx *d) -> int {
    int r = render_common(d, aa, w, h, pix[k], nullptr, nullptr, &ls[k], false);
    if (r || k == 0) return r;
    const int64_t n = (int64_t)pix[k].size() / 2;
    HIPCHK(d, d->pack.ensure((size_t)n * 16));
    launch_pack_pixels(d->pixels.as<int32_t>(), n, w, d->rgbf.as<float>(), d->rgb8.as<uint8_t>(),
                       d->pack.p, d->stream);
    HIPCHK(d, hipGetLastError());
    HIPCHK(d, hipStreamSynchronize(d->stream));
    return (int)GI_OK;
  });
  if (rc) return rc;
  auto tg = std::chrono::steady_clock::now();
  if ((int)c->recv.size() < nd) c->recv.resize(nd);
  if ((int)c->peer_pix.size() < nd) c->peer_pix.resize(nd);
  for (int k = 1; k < nd; k++) {
    const int64_t n = (int64_t)pix[k].size() / 2;
    HIPCHK(c, c->recv[k].ensure((size_t)n * 16));
    HIPCHK(c, upload(c->peer_pix[k], pix[k].data(), pix[k].size() * 4, c->stream));
  }
  if (!c->comms.empty()) {
    ncclResult_t r = g_rccl.groupStart();
    for (int k = 1; k < nd && r == ncclSuccess; k++) {
      const size_t bytes = pix[k].size() / 2 * 16;
      gi_ctx *d = c->peers[k - 1];
      r = g_rccl.send(d->pack.p, bytes, ncclUint8, 0, c->comms[k], d->stream);
      if (r == ncclSuccess) r = g_rccl.recv(c->recv[k].p, bytes, ncclUint8, k, c->comms[0], c->stream);
    }
    ncclResult_t r2 = g_rccl.groupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      return fail(c, GI_ERR_HIP, std::string("RCCL tile gather: ") +
                                     g_rccl.errString(r != ncclSuccess ? r : r2));
  } else {
    for (int k = 1; k < nd; k++) {
      gi_ctx *d = c->peers[k - 1];
      HIPCHK(c, hipMemcpyPeerAsync(c->recv[k].p, c->device, d->pack.p, d->device,
                                   pix[k].size() / 2 * 16, c->stream));
    }
  }
  for (int k = 1; k < nd; k++)
    launch_unpack_pixels(c->peer_pix[k].as<int32_t>(), (int64_t)pix[k].size() / 2, w,
                         c->recv[k].p, c->rgbf.as<float>(), c->rgb8.as<uint8_t>(), c->stream);
  HIPCHK(c, hipGetLastError());
  const size_t npx = (size_t)w * h * 3;
  if (rgbf) HIPCHK(c, hipMemcpyAsync(rgbf, c->rgbf.p, npx * 4, hipMemcpyDeviceToHost, c->stream));
  if (rgb8) HIPCHK(c, hipMemcpyAsync(rgb8, c->rgb8.p, npx, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (st) {
    memset(st, 0, sizeof *st);
    for (int k = 0; k < nd; k++) {
      const gi_render_stats &a = ls[k];
      st->screen_rays += a.screen_rays; st->shadow_rays += a.shadow_rays;
      st->monte_carlo_rays += a.monte_carlo_rays; st->transmissive_samples += a.transmissive_samples;
      st->specular_samples += a.specular_samples; st->indirect_samples += a.indirect_samples;
      st->caustic_samples += a.caustic_samples; st->knn_queries += a.knn_queries;
      st->knn_photons += a.knn_photons; st->knn_visited += a.knn_visited;
      st->knn_kernel_ms += a.knn_kernel_ms; st->knn_kernel_launches += a.knn_kernel_launches;
      for (int m = 0; m < 2; m++) {
        st->knn_map_queries[m] += a.knn_map_queries[m];
        st->knn_map_photons[m] += a.knn_map_photons[m];
        st->knn_map_visited[m] += a.knn_map_visited[m];
        st->knn_map_kernel_ms[m] += a.knn_map_kernel_ms[m];
        st->knn_map_launches[m] += a.knn_map_launches[m];
        st->knn_map_fallback_ms[m] += a.knn_map_fallback_ms[m];
        st->knn_map_fallback_queries[m] += a.knn_map_fallback_queries[m];
        st->knn_map_pass2_ms[m] += a.knn_map_pass2_ms[m];
        st->knn_map_pass2_queries[m] += a.knn_map_pass2_queries[m];
        if (k == 0) st->knn_map_kind[m] = a.knn_map_kind[m];
      }
      st->device_render_s_max = k ? std::max(st->device_render_s_max, a.render_s) : a.render_s;
      st->device_render_s_min = k ? std::min(st->device_render_s_min, a.render_s) : a.render_s;
    }
    const auto t1 = std::chrono::steady_clock::now();
    st->gather_s = std::chrono::duration<double>(t1 - tg).count();
    st->render_s = std::chrono::duration<double>(t1 - t0).count();
  }
  return GI_OK;
}

// RenderImage, render.cpp:155-259
int gi_render_image(gi_ctx *c, int aa, int w, int h, uint8_t *rgb8, float *rgbf,
                    gi_render_stats *st) {
  if (!c) return GI_ERR_ARG;
  hipSetDevice(c->device);
  if (!c->peers.empty()) {
    int rc = check_ready(c);
    if (rc) return rc;
    if (aa < 0 || w <= 0 || h <= 0) return fail(c, GI_ERR_ARG, "bad image size");
    return render_multi(c, aa, w, h, rgb8, rgbf, st);
  }
  std::vector<int32_t> pix((size_t)w * h * 2);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      pix[2 * ((size_t)y * w + x)] = x;
      pix[2 * ((size_t)y * w + x) + 1] = y;
    }
  return render_common(c, aa, w, h, pix, rgb8, rgbf, st, false);
}

int gi_render_tiles(gi_ctx *c, int aa, int w, int h, int tile, int shard, int nshards,
                    float *rgbf, gi_render_stats *st) {
  if (!c || tile <= 0 || nshards <= 0 || shard < 0 || shard >= nshards || !rgbf) return GI_ERR_ARG;
  hipSetDevice(c->device);
  std::vector<int32_t> pix = shard_pixels(w, h, tile, shard, nshards);
  return render_common(c, aa, w, h, pix, nullptr, rgbf, st, true);
}

// One rank's shard, left on the device and packed (torchrun: each rank gathers these buffers to
// rank 0 over RCCL and rank 0 composes them with gi_compose_tiles; nothing else crosses).
int gi_render_tiles_packed(gi_ctx *c, int aa, int w, int h, int tile, int shard, int nshards,
                           void *packed, int64_t cap, int64_t *npix, gi_render_stats *st) {
  if (!c || !npix || tile <= 0 || nshards <= 0 || shard < 0 || shard >= nshards || w <= 0 || h <= 0)
    return GI_ERR_ARG;
  DeviceScope dev(c->device);
  std::vector<int32_t> pix = shard_pixels(w, h, tile, shard, nshards);
  const int64_t n = (int64_t)pix.size() / 2;
  *npix = n;
  if (!packed) return GI_OK;
  if (cap < n) return fail(c, GI_ERR_ARG, "packed buffer holds fewer pixels than the shard");
  if (!c->peers.empty()) return fail(c, GI_ERR_STATE, "packed shards are for one-device contexts");
  int rc = render_common(c, aa, w, h, pix, nullptr, nullptr, st, false);
  if (rc) return rc;
  launch_pack_pixels(c->pixels.as<int32_t>(), n, w, c->rgbf.as<float>(), c->rgb8.as<uint8_t>(),
                     packed, c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GI_OK;
}

int gi_compose_tiles(gi_ctx *c, int w, int h, int tile, int nshards, const void *packed,
                     int64_t stride, uint8_t *rgb8, float *rgbf) {
  if (!c || !packed || tile <= 0 || nshards <= 0 || w <= 0 || h <= 0) return GI_ERR_ARG;
  DeviceScope dev(c->device);
  const size_t npx = (size_t)w * h * 3;
  HIPCHK(c, c->rgbf.ensure(npx * 4));
  HIPCHK(c, c->rgb8.ensure(npx));
  if ((int)c->peer_pix.size() < nshards) c->peer_pix.resize(nshards);
  for (int s = 0; s < nshards; s++) {
    std::vector<int32_t> pix = shard_pixels(w, h, tile, s, nshards);
    const int64_t n = (int64_t)pix.size() / 2;
    if (n > stride) return fail(c, GI_ERR_ARG, "packed stride smaller than a shard");
    HIPCHK(c, upload(c->peer_pix[s], pix.data(), pix.size() * 4, c->stream));
    launch_unpack_pixels(c->peer_pix[s].as<int32_t>(), n, w,
                         (const uint8_t *)packed + (size_t)s * stride * 16, c->rgbf.as<float>(),
                         c->rgb8.as<uint8_t>(), c->stream);
    HIPCHK(c, hipGetLastError());
  }
  if (rgbf) HIPCHK(c, hipMemcpyAsync(rgbf, c->rgbf.p, npx * 4, hipMemcpyDeviceToHost, c->stream));
  if (rgb8) HIPCHK(c, hipMemcpyAsync(rgb8, c->rgb8.p, npx, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GI_OK;
}

int gi_quantize(int w, int h, const float *rgbf, uint8_t *rgb8) {
  if (!rgbf || !rgb8) return GI_ERR_ARG;
  for (size_t i = 0; i < (size_t)w * h * 3; i++) rgb8[i] = (uint8_t)(255 * (double)rgbf[i]);
  return GI_OK;
}

int gi_estimate_radiance_batch(gi_ctx *c, int map, int64_t n, const gi_radiance_query *q,
                               double *rgb_out, int32_t *nfound, float *maxd2) {
  if (!c || map < 0 || map > 1 || (n > 0 && (!q || !rgb_out))) return GI_ERR_ARG;
  if (n == 0) return GI_OK;
  for (int64_t i = 1; i < n; i++)
    if (q[i].k != q[0].k || q[i].max_dist != q[0].max_dist || q[i].filter != q[0].filter)
      return fail(c, GI_ERR_ARG, "estimate_size / estimate_dist / filter must be uniform");
  if (n > QMETA_MAX_MATS) return fail(c, GI_ERR_ARG, "at most 2^26 queries per call");
  // one material per query carries its brdf terms
  std::vector<DMaterial> mats(n);
  std::vector<float> qp(4 * n);
  std::vector<QShade> qs(n);
  for (int64_t i = 0; i < n; i++) {
    DMaterial &m = mats[i];
    memset(&m, 0, sizeof m);
    for (int j = 0; j < 3; j++) { m.kd[j] = q[i].kd[j]; m.ks[j] = q[i].ks[j]; }
    m.n = q[i].shininess;
    bool spec = !(m.ks[0] == 0.0 && m.ks[1] == 0.0 && m.ks[2] == 0.0);
    m.flags = spec ? MF_SPECULAR : 0;
    double ct = q[i].cos_theta;
    uint32_t sign = (ct > 0) ? 1u : ((ct < 0) ? 2u : 0u);
    uint32_t meta = sign | ((uint32_t)i << 2);
    qp[4 * i] = (float)q[i].point[0];
    qp[4 * i + 1] = (float)q[i].point[1];
    qp[4 * i + 2] = (float)q[i].point[2];
    memcpy(&qp[4 * i + 3], &meta, 4);
    for (int j = 0; j < 3; j++) {
      qs[i].n[j] = q[i].normal[j];
      qs[i].ex[j] = q[i].exact_bounce[j];
      qs[i].w[j] = 1.0;
    }
  }
  DBuf dm, dq, ds, dout, dn, dmd;
  HIPCHK(c, upload(dm, mats.data(), mats.size() * sizeof(DMaterial), c->stream));
  HIPCHK(c, upload(dq, qp.data(), qp.size() * 4, c->stream));
  HIPCHK(c, upload(ds, qs.data(), qs.size() * sizeof(QShade), c->stream));
  HIPCHK(c, dout.ensure((size_t)n * 24));
  HIPCHK(c, dn.ensure((size_t)n * 4));
  HIPCHK(c, dmd.ensure((size_t)n * 4));
  KnnArgs k = knn_args(c, map);
  k.mats = dm.as<DMaterial>();
  k.K = q[0].k;
  k.filter = q[0].filter;
  k.general = c->knn_general_mode > 0 ? 1 : knn_general(mats, k.filter, true);  // the batch's own materials
  k.r2f = (float)(q[0].max_dist * q[0].max_dist);
  k.rmax = q[0].max_dist;
  k.qpos = dq.as<float4>();
  k.qshade = ds.as<QShade>();
  k.out = dout.as<double>();
  k.out_n = dn.as<int32_t>();
  k.out_maxd2 = dmd.as<float>();
  // an instance without the general estimate form counts the queries it cannot answer
  // (ST_GEN_MISS; the batch's own materials decide, so none is expected): re-run those batches
  // with the general instances instead of returning NaN
  unsigned long long *miss = c->d_stats.as<unsigned long long>() + ST_GEN_MISS;
  for (int pass = 0;; pass++) {
    HIPCHK(c, hipMemsetAsync(miss, 0, 8, c->stream));
    int rc = run_knn(c, k, n, nullptr);
    if (rc) return rc;
    unsigned long long nm = 0;
    HIPCHK(c, hipMemcpyAsync(&nm, miss, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (nm == 0) break;
    if (pass > 0 || k.general) return fail(c, GI_ERR_STATE, "k-NN estimate: general-form miss");
    k.general = 1;
  }
  HIPCHK(c, hipMemcpyAsync(rgb_out, dout.p, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
  if (nfound) HIPCHK(c, hipMemcpyAsync(nfound, dn.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  if (maxd2) HIPCHK(c, hipMemcpyAsync(maxd2, dmd.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  DBuf *bs[] = {&dm, &dq, &ds, &dout, &dn, &dmd};
  for (DBuf *b : bs) b->release();
  return GI_OK;
}

int gi_knn_batch(gi_ctx *c, int map, int64_t n, const double *pts, int K, double max_dist,
                 int32_t *idx_out, float *d2_out, int32_t *nfound) {
  if (!c || map < 0 || map > 1 || K <= 0 || (n > 0 && (!pts || !idx_out || !d2_out || !nfound)))
    return GI_ERR_ARG;
  if (n == 0) return GI_OK;
  std::vector<float> qp(4 * n, 0.0f);
  for (int64_t i = 0; i < n; i++)
    for (int j = 0; j < 3; j++) qp[4 * i + j] = (float)pts[3 * i + j];
  DBuf dq, di, dd, dn;
  HIPCHK(c, upload(dq, qp.data(), qp.size() * 4, c->stream));
  HIPCHK(c, di.ensure((size_t)n * K * 4));
  HIPCHK(c, dd.ensure((size_t)n * K * 4));
  HIPCHK(c, dn.ensure((size_t)n * 4));
  KnnArgs k = knn_args(c, map);
  k.mode = KNN_MODE_LIST;
  k.K = K;
  k.r2f = (float)(max_dist * max_dist);
  k.rmax = max_dist;
  k.qpos = dq.as<float4>();
  k.out_idx = di.as<int32_t>();
  k.out_d2 = dd.as<float>();
  k.out_n = dn.as<int32_t>();
  k.stats = nullptr;
  int rc = run_knn(c, k, n, nullptr);
  if (rc) return rc;
  std::vector<int32_t> idx((size_t)n * K);
  HIPCHK(c, hipMemcpyAsync(idx.data(), di.p, idx.size() * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(d2_out, dd.p, (size_t)n * K * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(nfound, dn.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // kd order -> storage (emission) order indices
  const auto &perm = c->hmap[map].perm;
  for (size_t i = 0; i < idx.size(); i++) idx_out[i] = idx[i] >= 0 ? perm[idx[i]] : -1;
  dq.release(); di.release(); dd.release(); dn.release();
  return GI_OK;
}

int gi_knn_bench(gi_ctx *c, int map, int64_t n, const double *pts, const double *nrm,
                 const int32_t *mat, int mode, int kernel, int iters, double *ms_out,
                 double *found_out, double *visited_out) {
  if (!c || map < 0 || map > 1 || n <= 0 || !pts || iters <= 0 || mode < 0 || mode > 2)
    return GI_ERR_ARG;
  if (mode == KNN_MODE_RADIANCE && (!nrm || !mat || !c->have_scene))
    return fail(c, GI_ERR_STATE, "radiance mode needs normals, materials and a scene");
  std::vector<float> qp(4 * n, 0.0f);
  std::vector<QShade> qs(n);
  for (int64_t i = 0; i < n; i++) {
    for (int j = 0; j < 3; j++) qp[4 * i + j] = (float)pts[3 * i + j];
    uint32_t meta = mat ? ((uint32_t)std::max(0, mat[i]) << 2) : 0u;
    memcpy(&qp[4 * i + 3], &meta, 4);
    for (int j = 0; j < 3; j++) {
      qs[i].n[j] = nrm ? nrm[3 * i + j] : 0.0;
      qs[i].ex[j] = nrm ? nrm[3 * i + j] : 0.0;
      qs[i].w[j] = 1.0;
    }
  }
  KnnArgs k = knn_args(c, map);
  DBuf dq, ds, dout, di, dd, dn;
  HIPCHK(c, upload(dq, qp.data(), qp.size() * 4, c->stream));
  HIPCHK(c, upload(ds, qs.data(), qs.size() * sizeof(QShade), c->stream));
  HIPCHK(c, dout.ensure((size_t)n * 24));
  k.qpos = dq.as<float4>();
  k.qshade = ds.as<QShade>();
  k.out = dout.as<double>();
  k.mode = mode;
  if (mode == KNN_MODE_LIST) {
    HIPCHK(c, di.ensure((size_t)n * k.K * 4));
    HIPCHK(c, dd.ensure((size_t)n * k.K * 4));
    HIPCHK(c, dn.ensure((size_t)n * 4));
    k.out_idx = di.as<int32_t>();
    k.out_d2 = dd.as<float>();
    k.out_n = dn.as<int32_t>();
  }
  float bmin[3], bmax[3];
  for (int j = 0; j < 3; j++) { bmin[j] = FLT_MAX; bmax[j] = -FLT_MAX; }
  for (int64_t i = 0; i < n; i++)
    for (int j = 0; j < 3; j++) {
      bmin[j] = std::min(bmin[j], qp[4 * i + j]);
      bmax[j] = std::max(bmax[j], qp[4 * i + j]);
    }
  uint32_t *perm = nullptr;
  HIPCHK(c, morton_order(dq.as<float4>(), n, bmin, bmax, c->mx[0].sorter, &perm, c->stream));
  k.perm = perm;
  int saved = c->knn_kernel_kind;
  if (kernel >= 0) c->knn_kernel_kind = kernel;
  HIPCHK(c, hipMemsetAsync(c->d_stats.p, 0, ST_BYTES, c->stream));
  double ms = 0;
  int rc = GI_OK;
  for (int it = 0; it < iters && rc == GI_OK; it++) rc = run_knn(c, k, n, &ms);
  c->knn_kernel_kind = saved;
  if (rc) return rc;
  unsigned long long st[ST_COUNT];
  HIPCHK(c, read_stats(c, st));
  // a measurement over wrong (NaN) estimates would be meaningless
  if (st[ST_GEN_MISS]) return fail(c, GI_ERR_STATE, "k-NN bench: queries needed the general estimate form");
  if (c->knn_dbg & 16) {
    fprintf(stderr, "[gi] k-NN phase cycles (sum over waves):");
    for (int i = 0; i < 16; i++) fprintf(stderr, " %llu", st[ST_PHASE + i]);
    fprintf(stderr, "\n");
  }
  if (ms_out) *ms_out = ms / iters;
  int so = map * ST_KNN_MAP;
  double nqd = (double)std::max<unsigned long long>(1, st[ST_KNN + so]);
  if (found_out) *found_out = (double)st[ST_KNN_PHOTONS + so] / nqd;
  if (visited_out) *visited_out = (double)st[ST_KNN_VISITED + so] / nqd;
  return GI_OK;
}

int gi_math_probe(gi_ctx *c, int fn, int64_t n, const double *x, const double *y, double *out) {
  if (!c || n < 0 || fn < 0 || fn > 7 || (n > 0 && (!x || !y || !out))) return GI_ERR_ARG;
  if (n == 0) return GI_OK;
  DeviceScope scope(c->device);
  DBuf dx, dy, dout;
  HIPCHK(c, upload(dx, x, (size_t)n * 8, c->stream));
  HIPCHK(c, upload(dy, y, (size_t)n * 8, c->stream));
  HIPCHK(c, dout.ensure((size_t)n * 8));
  launch_math_probe(fn, n, dx.as<double>(), dy.as<double>(), dout.as<double>(), c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, dout.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  dx.release();
  dy.release();
  dout.release();
  return GI_OK;
}

int gi_intersect_batch(gi_ctx *c, int64_t n, const double *org, const double *dir, int32_t *hit,
                       double *t, double *point, double *normal, int32_t *material) {
  if (!c) return GI_ERR_ARG;
  if (!c->have_scene) return fail(c, GI_ERR_STATE, "no scene loaded");
  if (n == 0) return GI_OK;
  DBuf dorg, ddir, dhit, dt, dp, dn, dm;
  HIPCHK(c, upload(dorg, org, (size_t)n * 24, c->stream));
  HIPCHK(c, upload(ddir, dir, (size_t)n * 24, c->stream));
  HIPCHK(c, dhit.ensure((size_t)n * 4));
  HIPCHK(c, dt.ensure((size_t)n * 8));
  HIPCHK(c, dp.ensure((size_t)n * 24));
  HIPCHK(c, dn.ensure((size_t)n * 24));
  HIPCHK(c, dm.ensure((size_t)n * 4));
  launch_intersect(make_view(c), n, dorg.as<double>(), ddir.as<double>(), dhit.as<int32_t>(),
                   dt.as<double>(), dp.as<double>(), dn.as<double>(), dm.as<int32_t>(), c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(hit, dhit.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(t, dt.p, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(point, dp.p, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(normal, dn.p, (size_t)n * 24, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(material, dm.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  DBuf *bs[] = {&dorg, &ddir, &dhit, &dt, &dp, &dn, &dm};
  for (DBuf *b : bs) b->release();
  return GI_OK;
}

}  // extern "C"
