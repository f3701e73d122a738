// gi_kernels.hip -- HIP kernels of the MI355X photon-mapping renderer (gfx950).
//
// Render pipeline for one batch of output pixels (all their 4^aa * DOF_TEST primary samples):
//   primary_kernel   camera ray + RayTrace prologue (ambient, direct) and the sample fan-out
//                    counts of raytracer.cpp:47-135 (transmissive / specular / indirect)
//   path_kernel<0>   count k-NN queries each sample path will issue   (Monte Carlo loops,
//   path_kernel<1>   emit them + the path's non-photon colour          montecarlo.cpp:16-305)
//   knn_kernel       k nearest photons + EstimateRadiance (photon_utils.cpp:72-162) per query,
//                    multiplied by the query's path weight
//   reduce_kernel    per pixel: sum paths and queries per primary sample, DOF average, clamp,
//                    box filter, 8-bit truncation (render.cpp:205-221)
// The decomposition is exact: every k-NN estimate enters the pixel linearly (colour += w*est),
// so deferring the estimates into a query list changes only the fp summation order.
#include <hip/hip_runtime.h>
#include "gi_device.h"
#include "gi_kernels.h"

namespace gi {

// ---------------------------------------------------------------------------------------
// exclusive scan of uint32 -> uint32 (n+1 outputs, last = total)
// ---------------------------------------------------------------------------------------
constexpr int SCAN_BLOCK = 256, SCAN_ITEMS = 4, SCAN_TILE = SCAN_BLOCK * SCAN_ITEMS;

__global__ __launch_bounds__(SCAN_BLOCK) void scan_tile_kernel(const uint32_t *in, uint32_t *out,
                                                                uint32_t *block_sums, int64_t n) {
  __shared__ uint32_t s[SCAN_BLOCK];
  int64_t base = (int64_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint32_t sum = 0;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; i++) {
    int64_t k = base + i;
    v[i] = (k < n) ? in[k] : 0u;
    sum += v[i];
  }
  s[threadIdx.x] = sum;
  __syncthreads();
  for (int off = 1; off < SCAN_BLOCK; off <<= 1) {
    uint32_t t = (threadIdx.x >= (unsigned)off) ? s[threadIdx.x - off] : 0u;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - sum;
#pragma unroll
  for (int i = 0; i < SCAN_ITEMS; i++) {
    int64_t k = base + i;
    if (k < n) out[k] = run;
    run += v[i];
  }
  if (threadIdx.x == SCAN_BLOCK - 1) block_sums[blockIdx.x] = s[SCAN_BLOCK - 1];
}

__global__ void scan_add_kernel(uint32_t *out, const uint32_t *block_off, int64_t n) {
  int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) out[k] += block_off[k / SCAN_TILE];
}

// ---------------------------------------------------------------------------------------
// Render: primary samples
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void decode_primary(const RenderArgs &a, int64_t b, int &pix, int &i,
                                               int &j, int &k, uint64_t &psample) {
  // b < nprim <= 2^31 per batch: 32-bit division (64-bit integer division is a long routine)
  uint32_t af2 = (uint32_t)(a.af * a.af), dof = (uint32_t)a.dof_test, ub = (uint32_t)b;
  k = (int)(ub % dof);
  uint32_t r = ub / dof;
  int sub = (int)(r % af2);
  pix = (int)(r / af2);
  int2 pc = a.pixels[pix];
  i = pc.x * a.af + (sub % a.af);
  j = pc.y * a.af + (sub / a.af);
  psample = ((uint64_t)j * (uint64_t)a.W + (uint64_t)i) * (uint64_t)a.dof_test + (uint64_t)k;
}

// Threadable_RayTracer body (render.cpp:96-132) + RayTrace (raytracer.cpp:174-233) up to the
// sample fan-outs. Writes the spawn record the path kernels expand.
// Occupancy target: left free, the soft-light call chain (direct_illumination -> soft_light ->
// illum_test) took 256 VGPRs + 110 AGPRs, one wave per SIMD; at 2 (32 VGPRs spilled) the C3
// frame (jensen.scn, 128 + 128 shadow rays per primary hit) is 10 % faster (3 waves: 5 %), the
// images unchanged; C2 (one hard shadow ray) is indifferent.
#ifndef PRIMARY_WPE
#define PRIMARY_WPE 2
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PRIMARY_WPE))) void primary_kernel(RenderArgs a) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t c_ray = 0, c_shadow = 0, c_ind = 0;
  if (b < a.nprim) {
    const SceneView &S = a.S;
    const Flags &F = a.F;
    int pix, i, j, k;
    uint64_t psample;
    decode_primary(a, b, pix, i, j, k, psample);
    Rng rng;
    rng.init(F.seed, KIND_PRIMARY, psample, 0);
    double dx = (double)(2 * (i - a.W / 2)) / (double)a.W;
    double dy = (double)(2 * (j - a.H / 2)) / (double)a.H;
    V far_point = ld3(S.cam.far_org) + (ld3(S.cam.far_right) * dx) + (ld3(S.cam.far_up) * dy);
    V eye = ld3(S.cam.eye);
    V org = eye;
    if (F.dof) {
      double r1, r2;
      do {
        r1 = (rng.next() * 2.0) - 1.0;
        r2 = (rng.next() * 2.0) - 1.0;
      } while (r1 * r1 + r2 * r2 > 1.0);
      org = eye + r1 * ld3(S.cam.dof_u) + r2 * ld3(S.cam.dof_v);
    }
    V dir = normalize(far_point - org);
    Spawn sp;
    sp.hit = 0;
    sp.tri = -1;
    sp.n_t = sp.n_s = sp.n_i = 0;
    sp.q_glob = sp.q_caus = 0;
    Hit h;
    Counts cnt = {0, 0, 0, 0, 0, 0};
    if (!scene_intersect(S, org, dir, h)) {
      C3 bg = ldc(S.background);
      sp.base[0] = bg.r; sp.base[1] = bg.g; sp.base[2] = bg.b;
    } else {
      c_ray = 1;
      const DMaterial &m = S.mats[h.mat];
      C3 color = rgb(0, 0, 0);
      if (F.ambient) color += ldc(S.ambient);
      V view = normalize(h.p - eye);
      double ct = dot(h.n, -view);
      double R = 0;
      if (F.ambient && (m.flags & MF_AMBIENT)) color += ldc(m.ka);
      if (F.direct && (m.flags & (MF_DIFFUSE | MF_SPECULAR)))
        direct_illumination(S, F, h.p, h.n, eye, color, m, ct, false, rng, cnt);
      if (F.transmissive && (m.flags & MF_TRANSPARENT)) {
        if (F.specular && F.fresnel) R = reflection_coeff(F.ir_air, ct, m.ir);
        if (R < 1.0) {
          C3 tw = (1.0 - R) * ldc(m.kt);
          sp.n_t = (int)ceil((F.trans_test * maxch(tw) + F.trans_test) / 2.0);
        }
      }
      if (F.specular && ((m.flags & MF_SPECULAR) || R > 0)) {
        C3 tw = ldc(m.kt) * R + ldc(m.ks);
        sp.n_s = (int)ceil((F.spec_test * maxch(tw) + F.spec_test) / 2.0);
      }
      if (F.indirect && (m.flags & MF_DIFFUSE)) {
        sp.n_i = (int)ceil((F.indirect_test * m.max_kd + F.indirect_test) / 2.0);
        const C3 wt = ldc(m.kd) / (double)sp.n_i;
        sp.wt[0] = wt.r; sp.wt[1] = wt.g; sp.wt[2] = wt.b;
      }
      if (F.caustic && (m.flags & MF_DIFFUSE)) sp.q_caus = 1;
      if (F.photon_viz && (m.flags & MF_DIFFUSE)) {
        sp.q_glob = 1;
        if (!F.cache) c_ind = 1;
      }
      sp.hit = 1;
      sp.p[0] = h.p.x; sp.p[1] = h.p.y; sp.p[2] = h.p.z;
      sp.n[0] = h.n.x; sp.n[1] = h.n.y; sp.n[2] = h.n.z;
      sp.v[0] = view.x; sp.v[1] = view.y; sp.v[2] = view.z;
      sp.ct = ct;
      sp.R = R;
      sp.mat = h.mat;
      sp.tri = h.tri;
      sp.base[0] = color.r; sp.base[1] = color.g; sp.base[2] = color.b;
    }
    a.spawn[b] = sp;
    a.npaths[b] = 1u + (uint32_t)(sp.n_t + sp.n_s);
    a.nmc[b] = (uint32_t)(sp.n_t + sp.n_s);
    a.nind[b] = (uint32_t)sp.n_i;
    c_shadow = cnt.shadow;
  }
  wave_add(&a.stats[ST_RAY], c_ray);
  wave_add(&a.stats[ST_SHADOW], c_shadow);
  wave_add(&a.stats[ST_INDIRECT], c_ind);
}

// Out-of-line optics for the path kernels' glass/mirror branches (transcendental-heavy; inlined,
// they set the register footprint: mc_kernel 294 -> 252 registers, 1 -> 2 waves per SIMD,
// 2.5x faster; ind_cont_kernel 256 + scratch -> 168 at 3 waves per SIMD). The RNG state is
// passed by value (a reference would put it in scratch); each sampler draws exactly two
// numbers, so the caller advances its counter by 2.
__device__ __noinline__ double reflection_coeff_nc(double ir_air, double ct, double ir_mat) {
  return reflection_coeff(ir_air, ct, ir_mat);
}
__device__ __noinline__ V transmissive_bounce_nc(double ir_air, V n, V view, double ct, double ir_mat) {
  return transmissive_bounce(ir_air, n, view, ct, ir_mat);
}
__device__ __noinline__ V specular_sample_nc(V ex, double nsh, double ct, uint64_t key, uint64_t ctr) {
  Rng r;
  r.key = key;
  r.ctr = ctr;
  return specular_sample(ex, nsh, ct, r);
}
__device__ __noinline__ V diffuse_sample_nc(V n, double ct, uint64_t key, uint64_t ctr) {
  Rng r;
  r.key = key;
  r.ctr = ctr;
  return diffuse_sample(n, ct, r);
}
__device__ __forceinline__ V specular_sample_call(V ex, double nsh, double ct, Rng &rng) {
  V v = specular_sample_nc(ex, nsh, ct, rng.key, rng.ctr);
  rng.ctr += 2;
  return v;
}
__device__ __forceinline__ V diffuse_sample_call(V n, double ct, Rng &rng) {
  V v = diffuse_sample_nc(n, ct, rng.key, rng.ctr);
  rng.ctr += 2;
  return v;
}

struct PathCtx {
  const SceneView *S;
  const Flags *F;
  const RenderArgs *A;
  uint64_t g;       // path slot
  uint32_t prim;    // primary sample of the path (within the batch)
  uint32_t pslot;   // slot of the path within its primary sample (0 = the primary's own)
  uint32_t j;       // queries issued so far by this path
  C3 base;
  Counts cnt;
  int64_t fixed[2]; // deterministic query slot per list (>= 0), -1 append, -2 used
  int hint;         // triangle the path's current ray leaves from (ray_mesh_bvh), -1 none
  uint32_t qstripe; // mc_cont stripe of the path's deferred sub-path (gi_host.cpp sizes a stripe
                    // for the paths of every IND_QS-th group of 64)
  int64_t cont_slot;  // >= 0: the sub-path's fixed mc_cont entry (mc_persist_kernel: the path's
                      // index, so the queue stays in path order); -1: striped append
};

// the indirect paths' tiled global-list slots carry no key: the reduction reads their row
// masks (RenderArgs::ind_qmask) instead
__device__ __forceinline__ bool keyed_slot(const RenderArgs &a, int list, int64_t slot) {
  return list != 0 || slot < a.qind_base || slot >= a.qind_base + a.tind;
}

__device__ __forceinline__ void put_none(const RenderArgs &a, int list, int64_t slot) {
  if (a.tiled_skip && !keyed_slot(a, list, slot)) return;  // a tiled slot nothing reads
  a.qpos[list][slot] = make_float4(0.f, 0.f, 0.f, __uint_as_float(QMETA_NONE));
  if (keyed_slot(a, list, slot)) a.qkey[list][slot] = ~0ull;
}

// append one photon-map query (list 0 = global, 1 = caustic): search half (point as f32 +
// meta) and shading half (normal, exact bounce, path weight)
__device__ __forceinline__ void put_query(PathCtx &P, int list, V p, V n, V ex, double ct,
                                          int mat, C3 w) {
  const RenderArgs &a = *P.A;
  uint32_t slot;
  if (P.fixed[list] >= 0) {
    slot = (uint32_t)P.fixed[list];
    P.fixed[list] = -2;
  } else {
    // one atomic per wave for all lanes that emit here (a single counter word serialises
    // ~10^8 atomics/s, MI355X_MICROARCH.md 'dequeue')
    uint64_t act = __ballot(1);
    int lane = (int)(threadIdx.x & 63);
    int leader = __ffsll((long long)act) - 1;
    uint32_t rank = (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&a.qcount[list], (uint32_t)__popcll(act));
    base = (uint32_t)__shfl((int)base, leader, 64);
    slot = base + rank;
  }
  // order key: (primary, slot in primary, query in path) -- the per-pixel reduction sums each
  // primary's queries in this order; segments per primary come from one boundary pass
  uint64_t key = ((uint64_t)P.prim << 32) | ((uint64_t)(P.pslot & 0xffffu) << 16) |
                 (uint64_t)(P.j++ & 0xffffu);
  if (slot >= a.qcap[list]) return;  // overflow: the host grows the lists and re-runs
  uint32_t sign = (ct > 0) ? 1u : ((ct < 0) ? 2u : 0u);
  const double ax = fabs(n.x), ay = fabs(n.y), az = fabs(n.z);
  const bool a0 = ax >= ay && ax >= az, a1 = !a0 && ay >= az;
  const double nw = a0 ? n.x : a1 ? n.y : n.z;
  const uint32_t face = (a0 ? 0u : a1 ? 2u : 4u) + (nw < 0.0 ? 1u : 0u);
  uint32_t meta = sign | ((uint32_t)mat << 2) | (face << 28);
  a.qpos[list][slot] = make_float4((float)p.x, (float)p.y, (float)p.z, __uint_as_float(meta));
  QShade q;
  q.n[0] = n.x; q.n[1] = n.y; q.n[2] = n.z;
  q.ex[0] = ex.x; q.ex[1] = ex.y; q.ex[2] = ex.z;
  q.w[0] = w.r; q.w[1] = w.g; q.w[2] = w.b;
  a.qshade[list][slot] = q;
  if (keyed_slot(a, list, slot)) a.qkey[list][slot] = key;
}

// global-map lookup at a diffuse hit: EstimateRadiance or (with -cache) the cached radiance
__device__ __forceinline__ void global_query(PathCtx &P, V p, V n, V ex, double ct, int mat, C3 w) {
  put_query(P, 0, p, n, ex, ct, mat, w);
}

// The shading half of one iteration of MonteCarlo_IndirectSample's loop, montecarlo.cpp:
// 177-305, at hit h of the ray from org (W = outer weight of the path, tw = throughput so far;
// org is also the loop's ray_start). Returns true when the path continues with the bounced ray
// in (org, dir). DIFFUSE_ONLY: the material has no specular/transmissive term (kt = ks = 0,
// opaque): R = pt = ps = 0 exactly, so only the query/absorb outcomes remain and the branches
// with pow/acos/asin/tan are not compiled in.
template <bool DIFFUSE_ONLY>
__device__ __forceinline__ bool ind_shade(PathCtx &P, const Hit &h, V &org, V &dir, Rng &rng, C3 W,
                                          C3 &tw) {
  const SceneView &S = *P.S;
  const Flags &F = *P.F;
  const DMaterial &m = S.mats[h.mat];
  V view = normalize(h.p - org);
  double ct = dot(h.n, -view);
  double R = 0;
  if (!DIFFUSE_ONLY && F.fresnel && (m.flags & MF_TRANSPARENT)) R = reflection_coeff_nc(F.ir_air, ct, m.ir);
  double pd = m.max_kd, pt = m.max_kt;
  double ps = m.max_ks + R * pt;
  pt *= (1.0 - R);
  double pterm = m.max_e + F.prob_absorb;
  double ptot = pd + pt + ps + pterm;
  double rnd = rng.next();
  if (ptot > 1.0) rnd *= ptot;
  if (rnd < pd) {
    V ex = reflective_bounce(h.n, view, ct);
    global_query(P, h.p, h.n, ex, ct, h.mat, W * (ldc(m.kd) * tw / pd));
    return false;
  }
  if (DIFFUSE_ONLY) return false;
  V sb;
  if (rnd < pd + pt) {
    V ex = transmissive_bounce_nc(F.ir_air, h.n, view, ct, m.ir);
    sb = F.distrib_trans ? specular_sample_call(ex, m.n, ct, rng) : ex;
    P.cnt.trans++;
    tw *= (1.0 - R) * ldc(m.kt) / pt;
  } else if (rnd < pd + pt + ps) {
    V ex = reflective_bounce(h.n, view, ct);
    sb = F.distrib_spec ? specular_sample_call(ex, m.n, ct, rng) : ex;
    P.cnt.spec++;
    tw *= (ldc(m.ks) + R * ldc(m.kt)) / ps;
  } else {
    return false;
  }
  org = h.p + sb * kEps;
  dir = sb;
  return true;
}

__device__ __forceinline__ bool diffuse_only(const DMaterial &m) {
  return !(m.flags & MF_TRANSPARENT) && m.max_kt == 0.0 && m.max_ks == 0.0;
}

// one full iteration: trace, then shade (background on a miss)
template <uint32_t KINDS = KINDS_ALL>
__device__ __forceinline__ bool ind_bounce(PathCtx &P, V &org, V &dir, Rng &rng, C3 W, C3 &tw) {
  Hit h;
  if (!scene_intersect<KINDS>(*P.S, org, dir, h, P.hint)) {
    P.base += W * (tw * ldc(P.S->background));
    return false;
  }
  P.cnt.monte++;
  P.hint = h.tri;
  return ind_shade<false>(P, h, org, dir, rng, W, tw);
}

// MonteCarlo_IndirectSample, montecarlo.cpp:177-305 (W = outer weight of this path)
template <uint32_t KINDS = KINDS_ALL>
__device__ __forceinline__ void mc_indirect_body(PathCtx &P, V org, V dir, Rng &rng, C3 W) {
  C3 tw = rgb(1, 1, 1);
  for (int iter = 0; iter < P.F->max_monte_depth; iter++)
    if (!ind_bounce<KINDS>(P, org, dir, rng, W, tw)) break;
}

template <uint32_t KINDS = KINDS_ALL>
__device__ __noinline__ void mc_indirect(PathCtx &P, V org, V dir, Rng &rng, C3 W) {
  mc_indirect_body<KINDS>(P, org, dir, rng, W);
}

// MonteCarlo_PathTrace's loop state (montecarlo.cpp:16-171): the current ray, the loop's
// ray_start, the throughput, the path's outer weight and RNG stream, the iteration count
struct McLoop {
  V org, dir, ray_start;
  C3 tw, W;
  Rng rng;
  int iter;
};

__device__ __forceinline__ void mc_begin(McLoop &L, V org, V dir, const Rng &rng, C3 W) {
  L.org = org;
  L.dir = dir;
  L.ray_start = org;
  L.tw = rgb(1, 1, 1);
  L.W = W;
  L.rng = rng;
  L.iter = 0;
}

// One iteration of MonteCarlo_PathTrace's loop (DEFER: indirect sub-paths go to the mc_cont
// queue). Returns false when the path has ended.
template <uint32_t KINDS = KINDS_ALL, bool DEFER = false, bool HARD = false>
__device__ __forceinline__ bool mc_step(PathCtx &P, McLoop &L) {
  const SceneView &S = *P.S;
  const Flags &F = *P.F;
  if (L.iter >= F.max_monte_depth) return false;
  L.iter++;
  const C3 W = L.W;
  Rng &rng = L.rng;
  C3 &tw = L.tw;
  Hit h;
  if (!scene_intersect<KINDS>(S, L.org, L.dir, h, P.hint)) {
    P.base += W * (tw * ldc(S.background));
    return false;
  }
  P.cnt.monte++;
  P.hint = h.tri;
  const DMaterial &m = S.mats[h.mat];
  C3 cb = rgb(0, 0, 0);
  if (F.ambient) cb += ldc(S.ambient);
  V view = normalize(h.p - L.ray_start);
  double ct = dot(h.n, -view);
  if (m.flags & (MF_DIFFUSE | MF_SPECULAR)) {
    if (HARD) direct_illumination_hard<KINDS>(S, F, h.p, h.n, L.ray_start, cb, m, ct, true, P.cnt);
    else direct_illumination<KINDS>(S, F, h.p, h.n, L.ray_start, cb, m, ct, true, rng, P.cnt);
  }
  if (F.caustic && (m.flags & MF_DIFFUSE)) {
    V ex = reflective_bounce(h.n, view, ct);
    put_query(P, 1, h.p, h.n, ex, ct, h.mat, W * tw);
    P.cnt.caustic++;
  }
  P.base += W * (cb * tw);
  double R = 0;
  if (F.specular && F.transmissive && F.fresnel && (m.flags & MF_TRANSPARENT))
    R = reflection_coeff_nc(F.ir_air, ct, m.ir);
  double pd = m.max_kd, pt = m.max_kt;
  double ps = m.max_ks + R * pt;
  pt *= (1.0 - R);
  double pterm = m.max_e + F.prob_absorb;
  double ptot = pd + pt + ps + pterm;
  double rnd = rng.next();
  if (ptot > 1.0) rnd *= ptot;
  V sb;
  if (rnd < pd) {
    C3 kd = ldc(m.kd);
    if (F.indirect) {
      // IndirectIllumination(inMC): one sample continuing this path's stream. Queued (the
      // path ends here, so its trace is this path's last work and its background term the
      // last addition to the path's sum) and traced compacted in ind_cont_kernel.
      V s2 = diffuse_sample_call(h.n, ct, rng);
      C3 w2 = W * ((kd * kd * tw) / pd);
      if (DEFER) {
        V o2 = h.p + s2 * kEps;
        size_t e;
        if (P.cont_slot >= 0) {
          e = (size_t)P.cont_slot;  // mc_persist_kernel: the entry of path t is slot t
        } else {  // mc_kernel: one atomic per wave on its stripe
          int lane = (int)(threadIdx.x & 63);
          uint64_t act = __ballot(1);
          int leader = __ffsll((long long)act) - 1;
          uint32_t qb = 0;
          if (lane == leader) qb = atomicAdd(&P.A->mc_ncont[P.qstripe * 32], (uint32_t)__popcll(act));
          qb = (uint32_t)__shfl((int)qb, leader, 64);
          e = (size_t)P.qstripe * P.A->mc_cap_s + qb + (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
        }
        IndCont &q = P.A->mc_cont[e];
        q.org[0] = o2.x; q.org[1] = o2.y; q.org[2] = o2.z;
        q.hp[0] = s2.x; q.hp[1] = s2.y; q.hp[2] = s2.z;
        q.w[0] = w2.r; q.w[1] = w2.g; q.w[2] = w2.b;
        q.rkey = rng.key;
        q.rctr = rng.ctr;
        q.g = (uint32_t)P.g;
        q.prim = P.prim;
        q.pslot = P.pslot;
        q.qslot = P.fixed[0] >= 0 ? (uint32_t)P.fixed[0] : 0xffffffffu;
        q.mat = -1;
        q.j = P.j;
        q.tri = h.tri;
        q.sub = 0;
        P.fixed[0] = -2;  // the sub-path owns the global slot now
      } else {
        mc_indirect<KINDS>(P, h.p + s2 * kEps, s2, rng, w2);
      }
      P.cnt.indirect++;
    } else if (F.fast_global) {
      V ex = reflective_bounce(h.n, view, ct);
      global_query(P, h.p, h.n, ex, ct, h.mat, W * (kd * tw / pd));
      if (!F.cache) P.cnt.indirect++;
    }
    return false;
  } else if (rnd < pd + pt) {
    if (!F.transmissive) return false;
    V ex = transmissive_bounce_nc(F.ir_air, h.n, view, ct, m.ir);
    sb = F.distrib_trans ? specular_sample_call(ex, m.n, ct, rng) : ex;
    P.cnt.trans++;
    tw *= (1.0 - R) * ldc(m.kt) / pt;
  } else if (rnd < pd + pt + ps) {
    if (!F.specular) return false;
    V ex = reflective_bounce(h.n, view, ct);
    sb = F.distrib_spec ? specular_sample_call(ex, m.n, ct, rng) : ex;
    P.cnt.spec++;
    tw *= (ldc(m.ks) + R * ldc(m.kt)) / ps;
  } else {
    return false;
  }
  L.ray_start = h.p + sb * kEps;
  L.org = L.ray_start;
  L.dir = sb;
  return true;
}

// MonteCarlo_PathTrace, montecarlo.cpp:16-171
template <uint32_t KINDS = KINDS_ALL, bool DEFER = false, bool HARD = false>
__device__ __forceinline__ void mc_path(PathCtx &P, V org, V dir, Rng &rng, C3 W) {
  if (!P.F->monte_carlo) return;
  McLoop L;
  mc_begin(L, org, dir, rng, W);
  while (mc_step<KINDS, DEFER, HARD>(P, L)) {
  }
  rng = L.rng;
}

// last p in [0, n) with off[p] <= t (off is an exclusive scan, off[0] = 0)
__device__ __forceinline__ int64_t scan_owner(const uint32_t *off, int64_t n, int64_t t) {
  int64_t lo = 0, hi = n;
  while (hi - lo > 1) {
    int64_t mid = (lo + hi) >> 1;
    if ((int64_t)off[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

// scan_owner for a whole wave: the owner of the wave's first path, then each lane steps forward
// (a wave's 64 consecutive paths span only a few primary samples). With an owner table
// (tab[k] = owner of path 64k, owner_table_kernel) the first owner is one load; without it, a
// binary search (19 dependent loads for 2^19 primaries).
__device__ __forceinline__ int64_t wave_owner(const uint32_t *off, int64_t n, int64_t t,
                                              int64_t total, const uint32_t *tab) {
  int64_t t0 = (int64_t)__builtin_amdgcn_readfirstlane((int)t);
  if (t0 > t) t0 = t;
  int64_t p;
  if (tab) p = (int64_t)tab[t0 >> 6];
  else p = scan_owner(off, n, t0 < total ? t0 : total - 1);
  while (p + 1 < n && (int64_t)off[p + 1] <= t) p++;
  return p;
}

// tab[k] = the primary owning path 64k of an exclusive scan off[0..n] (thread per primary)
__global__ void owner_table_kernel(const uint32_t *off, int64_t n, uint32_t *tab) {
  int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint32_t lo = off[p], hi = off[p + 1];
  for (uint32_t k = (lo + 63) >> 6; (k << 6) < hi; k++) tab[k] = (uint32_t)p;
}

// a path base that is +0 in every channel adds nothing to a sum that starts at +0 (such a sum is
// never -0: x + (+0) == x for every x other than -0), so it need not be stored or read
__device__ __forceinline__ bool base_is_pzero(const C3 &c) {
  return __double_as_longlong(c.r) == 0 && __double_as_longlong(c.g) == 0 &&
         __double_as_longlong(c.b) == 0;
}

// tiled entry of indirect path s of primary b (RenderArgs::ind_rows)
__device__ __forceinline__ int64_t ind_tau(const RenderArgs &a, int64_t b, int s) {
  return 64 * ((int64_t)a.ind_rows[b >> 6] + s) + (b & 63);
}

// rows[T] = max n_i over tile T's primaries (one wave per tile); scanned into ind_rows after
__global__ __launch_bounds__(64) void ind_tile_rows_kernel(const uint32_t *nind, int64_t nprim,
                                                          uint32_t *rows) {
  const int64_t b = (int64_t)blockIdx.x * 64 + threadIdx.x;
  uint32_t v = b < nprim ? nind[b] : 0u;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  if (threadIdx.x == 0) rows[blockIdx.x] = v;
}

// the tiled entries past a primary's own n_i (its tile's other primaries have more), and every
// entry of the last tile's lanes past nprim: empty global-list query slots (the k-NN skips them;
// the reduction never reads them). One thread per lane of every tile.
__global__ __launch_bounds__(256) void ind_pad_kernel(RenderArgs a) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= ((a.nprim + 63) & ~(int64_t)63)) return;
  const int rows = (int)(a.ind_rows[(b >> 6) + 1] - a.ind_rows[b >> 6]);
  for (int s = b < a.nprim ? (int)a.nind[b] : 0; s < rows; s++) {
    const int64_t sl = a.qind_base + ind_tau(a, b, s);
    a.qpos[0][sl] = make_float4(0.f, 0.f, 0.f, __uint_as_float(QMETA_NONE));
  }
}

__device__ __forceinline__ void path_init(PathCtx &P, const RenderArgs &a, int64_t g, int64_t prim,
                                          int pslot) {
  P.S = &a.S;
  P.F = &a.F;
  P.A = &a;
  P.g = (uint64_t)g;
  P.prim = (uint32_t)prim;
  P.pslot = (uint32_t)pslot;
  P.j = 0;
  P.base = rgb(0, 0, 0);
  Counts z = {0, 0, 0, 0, 0, 0};
  P.cnt = z;
  P.fixed[0] = P.fixed[1] = -1;
  P.hint = -1;
  P.qstripe = ((blockIdx.x * blockDim.x + threadIdx.x) >> 6) & (IND_QS - 1);
  P.cont_slot = -1;
}

// the six -v counters of a wave, two per 64-bit word through three wave reductions instead of
// six (a lane's counts are below 2^25, so 64 of them cannot carry into the upper half; a wave
// with a larger count, never seen, takes the six reductions)
__device__ __forceinline__ void path_stats(const RenderArgs &a, const Counts &cnt) {
  const uint32_t any = cnt.shadow | cnt.monte | cnt.trans | cnt.spec | cnt.indirect | cnt.caustic;
  if (__ballot((any >> 25) != 0u)) {
    wave_add(&a.stats[ST_SHADOW], cnt.shadow);
    wave_add(&a.stats[ST_MONTE], cnt.monte);
    wave_add(&a.stats[ST_TRANS], cnt.trans);
    wave_add(&a.stats[ST_SPEC], cnt.spec);
    wave_add(&a.stats[ST_INDIRECT], cnt.indirect);
    wave_add(&a.stats[ST_CAUSTIC], cnt.caustic);
    return;
  }
  uint64_t v0 = (uint64_t)cnt.shadow | ((uint64_t)cnt.monte << 32);
  uint64_t v1 = (uint64_t)cnt.trans | ((uint64_t)cnt.spec << 32);
  uint64_t v2 = (uint64_t)cnt.indirect | ((uint64_t)cnt.caustic << 32);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v0 += __shfl_xor(v0, o, 64);
    v1 += __shfl_xor(v1, o, 64);
    v2 += __shfl_xor(v2, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    unsigned long long *sd = stat_stripe(a.stats);
    const uint64_t v[6] = {v0 & 0xffffffffu, v0 >> 32, v1 & 0xffffffffu, v1 >> 32,
                           v2 & 0xffffffffu, v2 >> 32};
    const int id[6] = {ST_SHADOW, ST_MONTE, ST_TRANS, ST_SPEC, ST_INDIRECT, ST_CAUSTIC};
#pragma unroll
    for (int i = 0; i < 6; i++)
      if (v[i]) atomicAdd(sd + id[i], (unsigned long long)v[i]);
  }
}

// Path slots of primary sample p are [path_off[p], path_off[p+1]): slot 0 = the sample's own
// photon-map queries (CausticIllumination / EstimateGlobalIllumination at the primary hit) and
// base colour; then n_t transmissive, n_s specular and n_i indirect sample paths
// (raytracer.cpp:47-135). The three kinds run as separate launches so the ~90 % of paths
// that are indirect samples (one bounce to a diffuse hit, then a query) get a lean,
// call-free kernel instead of the Monte Carlo megakernel's register footprint.
__global__ __launch_bounds__(256) void slot0_kernel(RenderArgs a) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Counts cnt = {0, 0, 0, 0, 0, 0};
  if (b < a.nprim) {
    int64_t g = a.path_off[b];
    const Spawn &sp = a.spawn[b];
    PathCtx P;
    path_init(P, a, g, b, 0);
    P.fixed[0] = P.fixed[1] = b;
    P.base = ldc(sp.base);
    if (sp.hit) {
      V p = ld3(sp.p), n = ld3(sp.n), view = ld3(sp.v);
      V ex = reflective_bounce(n, view, sp.ct);
      if (sp.q_caus) {
        put_query(P, 1, p, n, ex, sp.ct, sp.mat, rgb(1, 1, 1));
        P.cnt.caustic++;
      }
      if (sp.q_glob) put_query(P, 0, p, n, ex, sp.ct, sp.mat, rgb(1, 1, 1));
    }
    if (P.fixed[0] >= 0) put_none(a, 0, b);
    if (P.fixed[1] >= 0) put_none(a, 1, b);
    a.base[3 * g] = P.base.r;
    a.base[3 * g + 1] = P.base.g;
    a.base[3 * g + 2] = P.base.b;
    cnt = P.cnt;
  }
  path_stats(a, cnt);
}

// IndirectIllumination sample s of primary pb (raytracer.cpp:112-135). With split_ind the
// kernel traces the first bounce and shades it only when the hit material is diffuse-only.
// Nearly every wave has a lane or two whose ray hits the glass, and shading that inline would
// make all 64 lanes execute the Fresnel pow, refraction trig and Phong-lobe sampling (and hold
// them idle through the glass bounces). Such paths are queued at the hit (wave-aggregated
// append) and finish compacted in ind_cont_kernel; the arithmetic and RNG stream are unchanged.
template <int W, bool SPLIT, uint32_t KINDS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(W))) void ind_kernel(RenderArgs a) {
  // thread t = tiled entry t (RenderArgs::ind_rows): row t / 64 of tile T, lane = primary
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Counts cnt = {0, 0, 0, 0, 0, 0};
  bool queue = false, hasq = false, hasb = false;
  // one row-table load gives the tile and the sample index; the spawn record (n_i, the weight)
  // and the pixel come next, side by side: two dependent loads before the path's arithmetic
  const uint64_t ri = t < a.tind ? a.ind_row_info[t >> 6] : 0ull;
  const int64_t pb = 64 * (int64_t)(ri >> 32) + (t & 63);
  const int s = (int)(uint32_t)ri;
  const Spawn &sp = a.spawn[pb < a.nprim ? pb : 0];
  if (t < a.tind && pb < a.nprim && s < sp.n_i) {
    int pslot = 1 + sp.n_t + sp.n_s + s;
    const int64_t tau = t;
    int64_t g = a.ind_g0 + tau;
    int pix, i, j, k;
    uint64_t psample;
    decode_primary(a, pb, pix, i, j, k, psample);
    PathCtx P;
    path_init(P, a, g, pb, pslot);
    P.fixed[0] = a.qind_base + tau;  // at most one (global) query per indirect path
    P.hint = sp.tri;
    Rng rng;
    rng.init(a.F.seed, KIND_IND, psample, (uint64_t)s);
    V p = ld3(sp.p), n = ld3(sp.n);
    V sb = (a.dbg >= 2) ? n : diffuse_sample(n, sp.ct, rng);
    C3 Wt = ldc(sp.wt);  // kd / n_i (primary_kernel)
    if (a.dbg != 0) {
      P.base = rgb(sb.x, sb.y, sb.z);
    } else if (!SPLIT) {
      mc_indirect_body(P, p + sb * kEps, sb, rng, Wt);
    } else if (a.F.max_monte_depth > 0) {
      V org = p + sb * kEps, dir = sb;
      C3 tw = rgb(1, 1, 1);
      Hit h;
      if (!scene_intersect<KINDS>(a.S, org, dir, h, sp.tri)) {
        P.base += Wt * (tw * ldc(a.S.background));
      } else {
        P.cnt.monte++;
        if (diffuse_only(a.S.mats[h.mat])) {
          ind_shade<true>(P, h, org, dir, rng, Wt, tw);
        } else {
          // glass / mirror hit: shaded in ind_cont_kernel (wave-aggregated append)
          queue = true;
          uint64_t act = __ballot(1);
          int lane = (int)(threadIdx.x & 63);
          int leader = __ffsll((long long)act) - 1;
          const uint32_t stripe = (uint32_t)(t >> 6) & (IND_QS - 1);
          uint32_t base = 0;
          if (lane == leader) base = atomicAdd(&a.ind_ncont[stripe * 32], (uint32_t)__popcll(act));
          base = (uint32_t)__shfl((int)base, leader, 64);
          const uint32_t slot = base + (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
          // a full stripe drops the entry; the host sees the fill and re-runs the batch
          IndCont &q = a.ind_cont[(size_t)stripe * a.ind_cap_s + (slot < a.ind_cap_s ? slot : 0)];
          if (slot < a.ind_cap_s) {
          q.org[0] = org.x; q.org[1] = org.y; q.org[2] = org.z;
          q.hp[0] = h.p.x; q.hp[1] = h.p.y; q.hp[2] = h.p.z;
          q.hn[0] = h.n.x; q.hn[1] = h.n.y; q.hn[2] = h.n.z;
          q.w[0] = Wt.r; q.w[1] = Wt.g; q.w[2] = Wt.b;
          q.rkey = rng.key;
          q.rctr = rng.ctr;
          q.g = (uint32_t)g;
          q.prim = (uint32_t)pb;
          q.pslot = (uint32_t)pslot;
          q.qslot = (uint32_t)P.fixed[0];
          q.mat = h.mat;
          q.tri = h.tri;
          q.sub = 0;
          }
        }
      }
    }
    P.cnt.indirect++;
    if (!queue) {
      hasq = P.fixed[0] == -2;
      if (P.fixed[0] >= 0) put_none(a, 0, P.fixed[0]);
      hasb = !base_is_pzero(P.base);
      if (hasb) {
        a.base[3 * g] = P.base.r;
        a.base[3 * g + 1] = P.base.g;
        a.base[3 * g + 2] = P.base.b;
      }
    }
    cnt = P.cnt;
  }
  // the row's masks (a wave is one row; tind is a multiple of 64): which entries hold a query,
  // which a base other than +0 (only those bases are stored). Queued paths set theirs in
  // ind_cont_kernel.
  const uint64_t qm = __ballot(hasq), bm = __ballot(hasb);
  if (t < a.tind && (threadIdx.x & 63) == 0) {
    a.ind_qmask[t >> 6] = qm;
    a.ind_bmask[t >> 6] = bm;
  }
  path_stats(a, cnt);
}

// the queued indirect paths, one per thread: block b serves stripe b % IND_QS, striding over its
// fill (the fills are known only on the device). At-hit entries (mat >= 0): shading of the
// first hit, then MonteCarlo_IndirectSample's loop from iteration 1 on; ray entries
// (mat == -1): the whole loop, its contribution added to the Monte Carlo path's base.
// occupancy: 3 waves per SIMD; scenes with meshes / boxes (C4: 148 VGPRs spilled at 3) get 2
template <uint32_t KINDS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu((KINDS & ~KINDS_TRI_SPHERE) ? 2 : 3)))
void ind_cont_kernel(RenderArgs a, const IndCont *queue, const uint32_t *fill, uint32_t cap_s) {
  const uint32_t stripe = blockIdx.x % IND_QS, part = blockIdx.x / IND_QS;
  const uint32_t parts = gridDim.x / IND_QS;
  const uint32_t n = min(fill[stripe * 32], cap_s);
  Counts tot = {0, 0, 0, 0, 0, 0};
  const uint32_t rounds = (n + parts * blockDim.x - 1) / (parts * blockDim.x);
  for (uint32_t r = 0; r < rounds; r++) {
    uint32_t idx = (r * parts + part) * blockDim.x + threadIdx.x;
    if (idx >= n) continue;
    const IndCont &q = queue[(size_t)stripe * cap_s + idx];
    if (q.g == IND_EMPTY) continue;  // a Monte Carlo path that deferred no sub-path
    PathCtx P;
    path_init(P, a, q.g, q.prim, (int)q.pslot);
    P.fixed[0] = (q.qslot == 0xffffffffu) ? -1 : (int64_t)q.qslot;
    P.hint = q.tri;
    Rng rng;
    rng.key = q.rkey;
    rng.ctr = q.rctr;
    C3 tw = rgb(1, 1, 1), W = ldc(q.w);
    V org = ld3(q.org), dir = org;
    bool go;
    int iter0;
    const bool sub = q.sub != 0;  // a Monte Carlo sub-path, its first bounce done (mc_sub_kernel)
    if (sub) P.j = q.j;
    if (q.mat >= 0) {
      Hit h;
      h.p = ld3(q.hp);
      h.n = ld3(q.hn);
      h.t = 0.0;
      h.mat = q.mat;
      h.tri = q.tri;
      go = ind_shade<false>(P, h, org, dir, rng, W, tw);
      iter0 = 1;
    } else {
      P.j = q.j;
      dir = ld3(q.hp);
      go = true;
      iter0 = 0;
    }
    if (go)
      for (int iter = iter0; iter < a.F.max_monte_depth; iter++)
        if (!ind_bounce<KINDS>(P, org, dir, rng, W, tw)) break;
    const bool used = P.fixed[0] == -2;
    if (P.fixed[0] >= 0) put_none(a, 0, P.fixed[0]);
    double *bp = a.base + 3 * (int64_t)q.g;
    if (q.mat >= 0 && !sub) {
      // an indirect path's tiled entry (q.qslot = qind_base + tau): its mask bits
      const int64_t tau = (int64_t)q.qslot - a.qind_base;
      const unsigned long long bit = 1ull << (tau & 63);
      if (used) atomicOr((unsigned long long *)&a.ind_qmask[tau >> 6], bit);
      if (!base_is_pzero(P.base)) {
        bp[0] = P.base.r;
        bp[1] = P.base.g;
        bp[2] = P.base.b;
        atomicOr((unsigned long long *)&a.ind_bmask[tau >> 6], bit);
      }
    } else {  // the sub-path's background term is the last addition to the path's sum
      bp[0] = bp[0] + P.base.r;
      bp[1] = bp[1] + P.base.g;
      bp[2] = bp[2] + P.base.b;
    }
    tot.shadow += P.cnt.shadow; tot.monte += P.cnt.monte; tot.trans += P.cnt.trans;
    tot.spec += P.cnt.spec; tot.indirect += P.cnt.indirect; tot.caustic += P.cnt.caustic;
  }
  path_stats(a, tot);
}

// The Monte Carlo paths' indirect sub-paths (mc_path's deferred IndirectIllumination sample,
// montecarlo.cpp:177-305 from a diffuse hit): their first bounce, one per thread, in the lean
// shape of ind_kernel. A sub-path that hits a diffuse-only material ends there (its query, or
// its background term), as most do; one that hits glass or a mirror is queued at that hit to
// mc_cont2 (flag `sub`) and finished by ind_cont_kernel with the Fresnel / refraction / lobe
// sampling code. Same arithmetic, RNG stream and order of additions to the path's base as
// ind_cont_kernel's whole-loop ray entries, so the same image; the 4-wave lean kernel replaces
// the 3-wave general loop for the common one-bounce case: C2 1,554 -> 1,536 ms per frame, C3
// 2,769 -> 2,730 ms, images identical (GI_MC_SUB=0 restores the single queue).
#ifndef MC_SUB_WPE
#define MC_SUB_WPE 4  // 3 measured equal (C2 1,536 vs 1,539 ms)
#endif
template <uint32_t KINDS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(MC_SUB_WPE)))
void mc_sub_kernel(RenderArgs a, const IndCont *queue, const uint32_t *fill, uint32_t cap_s) {
  const uint32_t stripe = blockIdx.x % IND_QS, part = blockIdx.x / IND_QS;
  const uint32_t parts = gridDim.x / IND_QS;
  const uint32_t n = min(fill[stripe * 32], cap_s);
  Counts tot = {0, 0, 0, 0, 0, 0};
  const uint32_t rounds = (n + parts * blockDim.x - 1) / (parts * blockDim.x);
  for (uint32_t r = 0; r < rounds; r++) {
    const uint32_t idx = (r * parts + part) * blockDim.x + threadIdx.x;
    bool on = idx < n;
    bool queue_it = false;
    Hit h;
    // the entry is read where its fields are used (a register copy of all 128 B spilled)
    const IndCont &q = queue[(size_t)stripe * cap_s + (on ? idx : 0u)];
    if (on && q.g == IND_EMPTY) on = false;  // a Monte Carlo path that deferred no sub-path
    PathCtx P;
    Rng rng;
    C3 W = rgb(0, 0, 0);
    V org = mk(0, 0, 0);
    if (on) {
      path_init(P, a, q.g, q.prim, (int)q.pslot);
      P.fixed[0] = (q.qslot == 0xffffffffu) ? -1 : (int64_t)q.qslot;
      P.hint = q.tri;
      P.j = q.j;
      rng.key = q.rkey;
      rng.ctr = q.rctr;
      W = ldc(q.w);
      org = ld3(q.org);
      V dir = ld3(q.hp);
      C3 tw = rgb(1, 1, 1);
      if (a.F.max_monte_depth > 0) {
        if (!scene_intersect<KINDS>(a.S, org, dir, h, P.hint)) {
          P.base += W * (tw * ldc(a.S.background));
        } else {
          P.cnt.monte++;
          P.hint = h.tri;
          if (diffuse_only(a.S.mats[h.mat])) ind_shade<true>(P, h, org, dir, rng, W, tw);
          else queue_it = true;
        }
      }
    }
    // glass / mirror first hits: wave-aggregated append to the same stripe of mc_cont2 (at most
    // this stripe's fill, so within its capacity)
    const uint64_t act = __ballot(queue_it);
    if (act) {
      const int lane = (int)(threadIdx.x & 63);
      const int leader = __ffsll((long long)act) - 1;
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(&a.mc_ncont2[stripe * 32], (uint32_t)__popcll(act));
      base = (uint32_t)__shfl((int)base, leader, 64);
      if (queue_it) {
        IndCont &o = a.mc_cont2[(size_t)stripe * cap_s + base +
                                (uint32_t)__popcll(act & ((1ull << lane) - 1ull))];
        o.org[0] = org.x; o.org[1] = org.y; o.org[2] = org.z;
        o.hp[0] = h.p.x; o.hp[1] = h.p.y; o.hp[2] = h.p.z;
        o.hn[0] = h.n.x; o.hn[1] = h.n.y; o.hn[2] = h.n.z;
        o.w[0] = W.r; o.w[1] = W.g; o.w[2] = W.b;
        o.rkey = rng.key;
        o.rctr = rng.ctr;
        o.g = q.g;
        o.prim = q.prim;
        o.pslot = q.pslot;
        o.qslot = q.qslot;
        o.mat = h.mat;
        o.j = P.j;
        o.tri = h.tri;
        o.sub = 1;
      }
    }
    if (on && !queue_it) {
      if (P.fixed[0] >= 0) put_none(a, 0, P.fixed[0]);
      // the sub-path's background term is the last addition to the path's sum
      double *bp = a.base + 3 * (int64_t)q.g;
      bp[0] = bp[0] + P.base.r;
      bp[1] = bp[1] + P.base.g;
      bp[2] = bp[2] + P.base.b;
    }
    if (on) {
      tot.shadow += P.cnt.shadow; tot.monte += P.cnt.monte; tot.trans += P.cnt.trans;
      tot.spec += P.cnt.spec; tot.indirect += P.cnt.indirect; tot.caustic += P.cnt.caustic;
    }
  }
  path_stats(a, tot);
}

#ifndef MC_WPE
#define MC_WPE 2  // mc_kernel occupancy target (waves per SIMD; 3 measured slower: spills)
#endif
// TransmissiveIllumination / SpecularIllumination sample (raytracer.cpp:47-109)
template <uint32_t KINDS, bool DEFER, bool HARD>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(MC_WPE))) void mc_kernel(RenderArgs a) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Counts cnt = {0, 0, 0, 0, 0, 0};
  if (t < a.total_mc) {
    int64_t pb = wave_owner(a.mc_off, a.nprim, t, a.total_mc, a.mc_tab);
    int s = (int)(t - a.mc_off[pb]);
    const Spawn &sp = a.spawn[pb];
    int64_t g = (int64_t)a.path_off[pb] + 1 + s;
    int pix, i, j, k;
    uint64_t psample;
    decode_primary(a, pb, pix, i, j, k, psample);
    const SceneView &S = a.S;
    const Flags &F = a.F;
    const DMaterial &m = S.mats[sp.mat];
    V p = ld3(sp.p), n = ld3(sp.n), view = ld3(sp.v);
    double ct = sp.ct, R = sp.R;
    PathCtx P;
    path_init(P, a, g, pb, 1 + s);
    P.hint = sp.tri;
    Rng rng;
    if (s < sp.n_t) {
      rng.init(F.seed, KIND_TRANS, psample, (uint64_t)s);
      V ex = transmissive_bounce_nc(F.ir_air, n, view, ct, m.ir);
      C3 tw = (1.0 - R) * ldc(m.kt);
      V sb = F.distrib_trans ? specular_sample_call(ex, m.n, ct, rng) : ex;
      mc_path<KINDS, DEFER, HARD>(P, p + sb * kEps, sb, rng, tw / (double)sp.n_t);
      P.cnt.trans++;
    } else {
      s -= sp.n_t;
      rng.init(F.seed, KIND_SPEC, psample, (uint64_t)s);
      V ex = reflective_bounce(n, view, ct);
      C3 tw = ldc(m.kt) * R + ldc(m.ks);
      V sb = F.distrib_spec ? specular_sample_call(ex, m.n, ct, rng) : ex;
      mc_path<KINDS, DEFER, HARD>(P, p + sb * kEps, sb, rng, tw / (double)sp.n_s);
      P.cnt.spec++;
    }
    a.base[3 * g] = P.base.r;
    a.base[3 * g + 1] = P.base.g;
    a.base[3 * g + 2] = P.base.b;
    cnt = P.cnt;
  }
  path_stats(a, cnt);
}

// The same Monte Carlo paths with a lane that finishes its path taking the next one (Aila &
// Laine's persistent "while-while" loop): every lane of a wave runs one iteration of
// MonteCarlo_PathTrace per trip, whatever path and depth it is at, instead of the wave running
// as long as its longest path with the finished lanes idle. Paths are handed out in order by one
// atomic per wave per refill (mc_next); a path's arithmetic, RNG stream, query keys and base
// slot do not depend on the lane that runs it, so the image and counters equal mc_kernel's.
template <uint32_t KINDS, bool DEFER, bool HARD>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(MC_WPE)))
void mc_persist_kernel(RenderArgs a) {
  const int lane = (int)(threadIdx.x & 63);
  const SceneView &S = a.S;
  const Flags &F = a.F;
  Counts cnt = {0, 0, 0, 0, 0, 0};
  PathCtx P;
  McLoop L;
  bool active = false, more = true;
  if (DEFER && blockIdx.x == 0 && threadIdx.x < IND_QS) {
    // the dense queue as the striped consumers read it: stripe s = paths [s cap, (s + 1) cap)
    const int64_t lo = (int64_t)threadIdx.x * a.mc_cap_s;
    const int64_t nf = a.total_mc - lo;
    a.mc_ncont[threadIdx.x * 32] = (uint32_t)(nf < 0 ? 0 : (nf > a.mc_cap_s ? a.mc_cap_s : nf));
  }
  while (true) {
    if (!active && more) {
      uint64_t need = __ballot(1);
      int leader = __ffsll((long long)need) - 1;
      uint32_t b = 0;
      if (lane == leader) b = atomicAdd(a.mc_next, (uint32_t)__popcll(need));
      b = (uint32_t)__shfl((int)b, leader, 64);
      int64_t t = (int64_t)b + __popcll(need & ((1ull << lane) - 1ull));
      if (t < a.total_mc) {
        // mc_kernel's prologue: the path's primary, its first (transmissive / specular) sample
        int64_t pb = wave_owner(a.mc_off, a.nprim, t, a.total_mc, a.mc_tab);
        int s = (int)(t - a.mc_off[pb]);
        const Spawn &sp = a.spawn[pb];
        int64_t g = (int64_t)a.path_off[pb] + 1 + s;
        int pix, i, j, k;
        uint64_t psample;
        decode_primary(a, pb, pix, i, j, k, psample);
        const DMaterial &m = S.mats[sp.mat];
        V p = ld3(sp.p), n = ld3(sp.n), view = ld3(sp.v);
        double ct = sp.ct, R = sp.R;
        path_init(P, a, g, pb, 1 + s);
        P.hint = sp.tri;
        P.cont_slot = t;
        Rng rng;
        V sb;
        C3 w;
        if (s < sp.n_t) {
          rng.init(F.seed, KIND_TRANS, psample, (uint64_t)s);
          V ex = transmissive_bounce_nc(F.ir_air, n, view, ct, m.ir);
          sb = F.distrib_trans ? specular_sample_call(ex, m.n, ct, rng) : ex;
          w = ((1.0 - R) * ldc(m.kt)) / (double)sp.n_t;
          P.cnt.trans++;
        } else {
          s -= sp.n_t;
          rng.init(F.seed, KIND_SPEC, psample, (uint64_t)s);
          V ex = reflective_bounce(n, view, ct);
          sb = F.distrib_spec ? specular_sample_call(ex, m.n, ct, rng) : ex;
          w = (ldc(m.kt) * R + ldc(m.ks)) / (double)sp.n_s;
          P.cnt.spec++;
        }
        mc_begin(L, p + sb * kEps, sb, rng, w);
        if (!F.monte_carlo) L.iter = F.max_monte_depth;  // MonteCarlo_PathTrace returns at once
        active = true;
      } else {
        more = false;  // the counter only grows: this lane will find no more paths
      }
    }
    if (!__any(active)) break;
    if (active && !mc_step<KINDS, DEFER, HARD>(P, L)) {
      // a path that deferred no sub-path marks its mc_cont entry empty (P.fixed[0] == -2 after
      // a deferral)
      if (DEFER && P.fixed[0] != -2) a.mc_cont[P.cont_slot].g = IND_EMPTY;
      a.base[3 * P.g] = P.base.r;
      a.base[3 * P.g + 1] = P.base.g;
      a.base[3 * P.g + 2] = P.base.b;
      cnt.shadow += P.cnt.shadow; cnt.monte += P.cnt.monte; cnt.trans += P.cnt.trans;
      cnt.spec += P.cnt.spec; cnt.indirect += P.cnt.indirect; cnt.caustic += P.cnt.caustic;
      active = false;
    }
  }
  path_stats(a, cnt);
}

// ---------------------------------------------------------------------------------------
// k-NN radiance estimate (R3Kdtree::FindClosestQuick R3Kdtree.cpp:688-784 + EstimateRadiance
// photon_utils.cpp:72-162). One query per lane; stackless nearest-first traversal of the
// implicit complete kd-tree (parent = node>>1, sibling = node^1); per-lane max-heap of the K
// best (d2, index) pairs in LDS laid out [slot][lane] (conflict-free b32 accesses) or, for
// K > 64, in a global scratch laid out the same way.
// ---------------------------------------------------------------------------------------
struct HeapRef {
  float *d2;
  int32_t *idx;
  int stride;  // elements between consecutive slots of one lane
};

__device__ __forceinline__ bool heap_less(float da, int ia, float db, int ib) {
  return da < db || (da == db && ia < ib);
}

// 0-based binary max-heap on (d2, idx)
__device__ __forceinline__ void heap_push(HeapRef h, int &size, float d, int id) {
  int c = size++;
  while (c > 0) {
    int p = (c - 1) >> 1;
    float pd = h.d2[p * h.stride];
    int pi = h.idx[p * h.stride];
    if (!heap_less(pd, pi, d, id)) break;
    h.d2[c * h.stride] = pd;
    h.idx[c * h.stride] = pi;
    c = p;
  }
  h.d2[c * h.stride] = d;
  h.idx[c * h.stride] = id;
}
__device__ __forceinline__ void heap_replace_top(HeapRef h, int size, float d, int id) {
  int c = 0;
  while (true) {
    int l = 2 * c + 1;
    if (l >= size) break;
    float ld = h.d2[l * h.stride];
    int li = h.idx[l * h.stride];
    int r = l + 1;
    if (r < size) {
      float rd = h.d2[r * h.stride];
      int ri = h.idx[r * h.stride];
      if (heap_less(ld, li, rd, ri)) { l = r; ld = rd; li = ri; }
    }
    if (!heap_less(d, id, ld, li)) break;
    h.d2[c * h.stride] = ld;
    h.idx[c * h.stride] = li;
    c = l;
  }
  h.d2[c * h.stride] = d;
  h.idx[c * h.stride] = id;
}

__device__ __forceinline__ float metric_d2(float qx, float qy, float qz, float4 p) {
  float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
  return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
}

// Find the K best photons of query (qx,qy,qz) within r2; returns heap size.
// "While-while" structure: each lane walks internal nodes until it holds its next leaf
// (or finishes); only then does the wave run the leaf loop, for all lanes at once. A single
// loop mixing descend and leaf steps would re-run the 64-photon leaf loop whenever any one
// lane reached a leaf (measured ~15x instruction overhead from divergence).
__device__ __forceinline__ int knn_search(const KdView &M, float qx, float qy, float qz, float r2,
                                          int K, HeapRef h, uint32_t &visited) {
  int size = 0;
  float maxd2 = r2;
  float topd = 0.f;
  int topi = 0;
  if (M.n == 0) return 0;
  const KdNode *nodes = reinterpret_cast<const KdNode *>(M.nodes);
  const float4 *pos = reinterpret_cast<const float4 *>(M.pos4);
  const int L = M.nleaves;
  int node = 1;
  bool live = true;
  while (true) {
    // walk to the next leaf whose tight box is within the current bound
    int leaf = -1;
    while (live) {
      KdNode nd = nodes[node];
      if (kd_box_d2(nd.lo, nd.hi, qx, qy, qz) <= maxd2) {
        if (node < L) {
          float q = kd_axis_q(__float_as_int(nd.hi.w), qx, qy, qz);
          node = 2 * node + ((q - nd.lo.w >= 0.0f) ? 1 : 0);
          continue;
        }
        leaf = node - L;
        break;
      }
      live = kd_next(nodes, node, qx, qy, qz);
    }
    if (leaf < 0) break;
    int64_t s0 = ((int64_t)leaf * M.n) / L, s1 = ((int64_t)(leaf + 1) * M.n) / L;
    for (int64_t ii = s0; ii < s1; ii += 4) {
      float4 p[4];
#pragma unroll
      for (int u = 0; u < 4; u++) p[u] = pos[(ii + u < s1) ? ii + u : s1 - 1];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        float d2 = metric_d2(qx, qy, qz, p[u]);
        if (ii + u < s1 && d2 <= maxd2) {
          int id = (int)(ii + u);
          if (size < K) {
            heap_push(h, size, d2, id);
            if (size == K) {
              topd = h.d2[0];
              topi = h.idx[0];
              maxd2 = topd;
            }
          } else if (heap_less(d2, id, topd, topi)) {
            heap_replace_top(h, size, d2, id);
            topd = h.d2[0];
            topi = h.idx[0];
            maxd2 = topd;
          }
        }
      }
    }
    visited += (uint32_t)(s1 - s0);
    live = kd_next(nodes, node, qx, qy, qz);
  }
  return size;
}

// Each lane answers a.qpl Morton-consecutive queries (q = (block*qpl + it)*64 + lane). After
// the first, the search starts from a proven bound instead of r^2: the K photons found for
// the previous query p all lie within d_K(p) + |q - p| of q (triangle inequality), so
// d_K(q)^2 <= (d_K(p) + |q - p|)^2. A 1e-5 relative margin covers the fp32 metric's
// rounding; the bound only prunes, the result set is unchanged.
// The heaps live in global scratch, so any K works: this is the path for estimate sizes beyond
// the LDS kernels (K + 64 > 1024 photons per query-per-wave candidate buffer).
__global__ __launch_bounds__(64) void knn_kernel(KnnArgs a) {
  int lane = threadIdx.x;
  uint64_t nfound_total = 0, visited_total = 0, nq_done = 0;
  HeapRef h;
  {
    int64_t t = (int64_t)blockIdx.x * 64 + lane;
    h.d2 = a.gheap_d2 + t;
    h.idx = a.gheap_idx + t;
    h.stride = (int)((int64_t)gridDim.x * 64);
  }
  float px = 0.f, py = 0.f, pz = 0.f, pk2 = -1.0f;  // previous query and its K-th d2
  for (int it = 0; it < a.qpl; it++) {
    int64_t q = ((int64_t)blockIdx.x * a.qpl + it) * 64 + lane;
    if (q >= a.nq) break;
    int64_t qg = a.q0 + q;
    int64_t qi = a.perm ? (int64_t)a.perm[qg] : qg;
    float4 qp = a.qpos[qi];
    if (__float_as_uint(qp.w) == QMETA_NONE) continue;  // empty deterministic slot
    float bound = a.r2f;
    if (pk2 >= 0.0f) {
      double dx = (double)qp.x - px, dy = (double)qp.y - py, dz = (double)qp.z - pz;
      double rb = (sqrt((double)pk2) + sqrt(dx * dx + dy * dy + dz * dz)) * (1.0 + 1e-5);
      float b2 = __double2float_ru(rb * rb);
      if (b2 < bound) bound = b2;
    }
    uint32_t visited = 0;
    int num = knn_search(a.map, qp.x, qp.y, qp.z, bound, a.K, h, visited);
    px = qp.x; py = qp.y; pz = qp.z;
    pk2 = (num == a.K) ? h.d2[0] : -1.0f;
    nfound_total += num;
    visited_total += visited;
    nq_done += 1;
    if (a.mode == KNN_MODE_LIST) {
      for (int s = 0; s < a.K; s++) {
        a.out_idx[qi * a.K + s] = (s < num) ? h.idx[s * h.stride] : -1;
        a.out_d2[qi * a.K + s] = (s < num) ? h.d2[s * h.stride] : -1.0f;
      }
      a.out_n[qi] = num;
    } else {
      double o0 = 0, o1 = 0, o2 = 0;
      double maxd2 = kEps;
      if (num > 0) {
        if (num < a.K) {
          maxd2 = a.rmax * a.rmax;
        } else {
          for (int s = 0; s < num; s++) {
            double d = (double)h.d2[s * h.stride];
            if (d > maxd2) maxd2 = d;
          }
        }
        if (a.mode == KNN_MODE_IRRADIANCE) {
          // EstimateIrradiance, photon_utils.cpp:209-246
          for (int s = 0; s < num; s++) {
            uint32_t e = a.map.rgbe[h.idx[s * h.stride]];
            uint32_t ex = e >> 24;
            if (ex) {
              double inv = ldexp(1.0, (int)ex - 128 - 8);
              o0 += (double)(e & 255u) * inv;
              o1 += (double)((e >> 8) & 255u) * inv;
              o2 += (double)((e >> 16) & 255u) * inv;
            }
          }
          double den = kPi * maxd2;
          o0 /= den; o1 /= den; o2 /= den;
        } else {
          const QShade &sh = a.qshade[qi];
          uint32_t meta = __float_as_uint(qp.w);
          uint32_t sign = meta & 3u;
          const DMaterial &m = a.mats[qmeta_mat(meta)];
          double N0 = sh.n[0], N1 = sh.n[1], N2 = sh.n[2];
          double E0 = sh.ex[0], E1 = sh.ex[1], E2 = sh.ex[2];
          bool spec = (m.flags & MF_SPECULAR) || (m.n < 0);
          double c1 = 1.0, c2 = 1.0, tot_w = 0;
          if (a.filter == 1) c1 = 1.0 / (a.fk * sqrt(maxd2));
          else if (a.filter == 2) {
            c1 = gm::pow(2.7182818284590452354, -a.fb);
            c2 = 1.0 / (2.0 * maxd2);
          }
          for (int s = 0; s < num; s++) {
            int id = h.idx[s * h.stride];
            uint32_t dcode = __float_as_uint(a.map.pos4[4 * (int64_t)id + 3]) & 0xffffu;
            double ix = a.lut[3 * dcode], iy = a.lut[3 * dcode + 1], iz = a.lut[3 * dcode + 2];
            double perp = N0 * ix + N1 * iy + N2 * iz;
            if ((sign == 2u && perp < 0) || (sign == 1u && perp > 0)) continue;
            uint32_t e = a.map.rgbe[id];
            uint32_t ee = e >> 24;
            double inv = ee ? ldexp(1.0, (int)ee - 128 - 8) : 0.0;
            double p0 = ee ? (double)(e & 255u) * inv : 0.0;
            double p1 = ee ? (double)((e >> 8) & 255u) * inv : 0.0;
            double p2 = ee ? (double)((e >> 16) & 255u) * inv : 0.0;
            double ca = E0 * -ix + E1 * -iy + E2 * -iz;
            if (ca < 0) ca = 0;
            double ap = fabs(perp);
            double pw = spec ? gm::pow(ca, m.n) : 0.0;
            p0 *= ap * m.kd[0] + pw * m.ks[0];
            p1 *= ap * m.kd[1] + pw * m.ks[1];
            p2 *= ap * m.kd[2] + pw * m.ks[2];
            if (a.filter == 1) {
              double f = (1.0 - c1 * sqrt((double)h.d2[s * h.stride]));
              p0 *= f; p1 *= f; p2 *= f;
            } else if (a.filter == 2) {
              double w = (1.0 - (1.0 - gm::pow(c1, c2 * (double)h.d2[s * h.stride])) / (1.0 - c1));
              p0 *= w; p1 *= w; p2 *= w;
              tot_w += w;
            }
            o0 += p0; o1 += p1; o2 += p2;
          }
          // photon_utils.cpp:149-158 normalisation
          bool ok = true;
          if (a.filter == 0 && maxd2 > 0) {
            double den = kPi * maxd2;
            o0 /= den; o1 /= den; o2 /= den;
          } else if (a.filter == 1 && maxd2 > 0) {
            double den = (1.0 - 2.0 / 3.0 / a.fk) * kPi * maxd2;
            o0 /= den; o1 /= den; o2 /= den;
          } else if (a.filter == 2 && tot_w > 0 && maxd2 > 0) {
            double sc = a.fa * (num / tot_w) / (kPi * maxd2);
            o0 *= sc; o1 *= sc; o2 *= sc;
          } else {
            ok = false;
          }
          if (ok) {
            o0 *= sh.w[0]; o1 *= sh.w[1]; o2 *= sh.w[2];
          } else {
            o0 = o1 = o2 = 0;
          }
        }
      }
      a.out[3 * qi] = o0;
      a.out[3 * qi + 1] = o1;
      a.out[3 * qi + 2] = o2;
      if (a.out_n) a.out_n[qi] = num;
      if (a.out_maxd2) a.out_maxd2[qi] = (num > 0) ? (float)maxd2 : 0.0f;
    }
  }
  if (a.stats) {
    wave_add(&a.stats[ST_KNN + a.stat_off], nq_done);
    wave_add(&a.stats[ST_KNN_PHOTONS + a.stat_off], nfound_total);
    wave_add(&a.stats[ST_KNN_VISITED + a.stat_off], visited_total);
  }
}

// EstimateCachedRadiance (photon_utils.cpp:165-205) with FindClosest (R3Kdtree.cpp:317-445):
// nearest photon at distance >= previous + 1e-6 until one passes the side test (Q8 guarded).
__global__ __launch_bounds__(64) void cached_kernel(KnnArgs a) {
  int64_t q = (int64_t)blockIdx.x * 64 + threadIdx.x;
  uint64_t nq_done = 0;
  if (q < a.nq && __float_as_uint(a.qpos[q].w) != QMETA_NONE) {
    float4 qp = a.qpos[q];
    nq_done = 1;
    const QShade &sh = a.qshade[q];
    uint32_t meta = __float_as_uint(qp.w);
    uint32_t sign = meta & 3u;
    const DMaterial &m = a.mats[qmeta_mat(meta)];
    double N0 = sh.n[0], N1 = sh.n[1], N2 = sh.n[2];
    double out0 = 0, out1 = 0, out2 = 0;
    double closest = 0;
    const KdNode *nodes = reinterpret_cast<const KdNode *>(a.map.nodes);
    const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
    const int L = a.map.nleaves;
    for (int guard = 0; guard < 1 << 20 && a.map.n > 0; guard++) {
      double mn = closest + kEps;
      float min2 = (float)(mn * mn);
      float best2 = a.r2f;
      int best = -1;
      int node = 1;
      while (true) {
        KdNode nd = nodes[node];
        if (kd_box_d2(nd.lo, nd.hi, qp.x, qp.y, qp.z) <= best2) {
          if (node < L) {
            float qq = kd_axis_q(__float_as_int(nd.hi.w), qp.x, qp.y, qp.z);
            node = 2 * node + ((qq - nd.lo.w >= 0.0f) ? 1 : 0);
            continue;
          }
          int leaf = node - L;
          int64_t s0 = ((int64_t)leaf * a.map.n) / L, s1 = ((int64_t)(leaf + 1) * a.map.n) / L;
          for (int64_t ii = s0; ii < s1; ii++) {
            float d2 = metric_d2(qp.x, qp.y, qp.z, pos[ii]);
            if (d2 >= min2 && d2 <= best2 && (d2 < best2 || best < 0 || (int)ii < best)) {
              best2 = d2;
              best = (int)ii;
            }
          }
        }
        while (node != 1) {
          const KdNode &pn = nodes[node >> 1];
          float qq = kd_axis_q(__float_as_int(pn.hi.w), qp.x, qp.y, qp.z);
          int near_is_right = (qq - pn.lo.w >= 0.0f) ? 1 : 0;
          if ((node & 1) == near_is_right) break;
          node >>= 1;
        }
        if (node == 1) break;
        node ^= 1;
      }
      closest = sqrt((double)best2);
      if (best < 0) break;
      uint32_t dcode = __float_as_uint(a.map.pos4[4 * (int64_t)best + 3]) & 0xffffu;
      double ix = a.lut[3 * dcode], iy = a.lut[3 * dcode + 1], iz = a.lut[3 * dcode + 2];
      double perp = N0 * ix + N1 * iy + N2 * iz;
      if ((sign == 2u && perp < 0) || (sign == 1u && perp > 0)) continue;
      uint32_t e = a.map.rgbe[best];
      uint32_t ee = e >> 24;
      double inv = ee ? ldexp(1.0, (int)ee - 128 - 8) : 0.0;
      double p0 = ee ? (double)(e & 255u) * inv : 0.0;
      double p1 = ee ? (double)((e >> 8) & 255u) * inv : 0.0;
      double p2 = ee ? (double)((e >> 16) & 255u) * inv : 0.0;
      double ca = sh.ex[0] * -ix + sh.ex[1] * -iy + sh.ex[2] * -iz;
      if (ca < 0) ca = 0;
      double ap = fabs(perp);
      double pw = gm::pow(ca, m.n);
      p0 *= ap * m.kd[0] + pw * m.ks[0];
      p1 *= ap * m.kd[1] + pw * m.ks[1];
      p2 *= ap * m.kd[2] + pw * m.ks[2];
      out0 = p0 * sh.w[0];
      out1 = p1 * sh.w[1];
      out2 = p2 * sh.w[2];
      break;
    }
    a.out[3 * q] = out0;
    a.out[3 * q + 1] = out1;
    a.out[3 * q + 2] = out2;
  }
  if (a.stats) wave_add(&a.stats[ST_KNN + a.stat_off], nq_done);
}

// CSR offsets of the key-sorted query list by primary sample: seg[b] = the first position whose
// primary is >= b (empty slots, key ~0, count as primary nprim), b = 0 .. nprim. One thread per
// primary, a binary search over the sorted keys: the Monte Carlo appends of a batch cluster on
// the few rows through glass, and filling the gaps from the positions' side left one thread
// writing every primary after the last append (27 ms in the r02 trace).
__global__ void segments_kernel(const uint64_t *skeys, uint32_t n, uint32_t nprim, uint32_t *seg) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b > (int64_t)nprim) return;
  auto prim_of = [&](int64_t k) -> int64_t {
    uint64_t key = skeys[k];
    if (key == ~0ull) return nprim;
    uint64_t p = key >> 32;
    return p < nprim ? (int64_t)p : (int64_t)nprim;
  };
  int64_t lo = 0, hi = n;  // first k in [0, n] with prim_of(k) >= b (prim_of(n) = nprim)
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (prim_of(mid) >= b) hi = mid;
    else lo = mid + 1;
  }
  seg[b] = (uint32_t)lo;
}

void launch_segments(const uint64_t *skeys, uint32_t n, uint32_t nprim, uint32_t *seg,
                     hipStream_t st) {
  segments_kernel<<<(unsigned)(((int64_t)nprim + 1 + 255) / 256), 256, 0, st>>>(skeys, n, nprim, seg);
}

// ---------------------------------------------------------------------------------------
// Per-pixel reduction: RenderImage's DOF average + ClampColor + box filter + SetPixelRGB
// (render.cpp:130-135, 205-221; R2Image.cpp:205-208)
// ---------------------------------------------------------------------------------------
// lane i's value of a wave-uniform index i (two readlanes)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int i) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, i);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), i);
  return ((uint64_t)hi << 32) | lo;
}

// the sum over the tiled rows [r0, r0 + M) of one mask array: lane l (primary 64 T + l) adds
// entry 64 r + l of vals where bit l of mask[r] is set, rows in order. The masks of 64 rows come
// in with one load (lane i: row r0 + s0 + i) and are read back with readlane; four rows' entries
// are loaded before they are added.
__device__ __forceinline__ void tiled_row_sum(const uint64_t *mask, const double *vals, int64_t r0, int M,
                                              int lane, double &c0, double &c1, double &c2) {
  for (int s0 = 0; s0 < M; s0 += 64) {
    const int n = M - s0 < 64 ? M - s0 : 64;
    const uint64_t mk = lane < n ? mask[r0 + s0 + lane] : 0ull;
    for (int j = 0; j < n; j += 4) {
      bool on[4];
      double v[12];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        on[u] = j + u < n && ((readlane64(mk, j + u < n ? j + u : 0) >> lane) & 1ull);
        v[3 * u] = v[3 * u + 1] = v[3 * u + 2] = 0.0;
        if (on[u]) {  // unflagged entries are not read
          const double *e = vals + 3 * (64 * (r0 + s0 + j + u) + lane);
          v[3 * u] = e[0];
          v[3 * u + 1] = e[1];
          v[3 * u + 2] = e[2];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; u++)
        if (on[u]) {
          c0 += v[3 * u];
          c1 += v[3 * u + 1];
          c2 += v[3 * u + 2];
        }
    }
  }
}

// Pass 1, one thread per primary sample b: c(b) = sum of b's path bases, then of its queries,
// in the oracle's order (a sequential fp64 sum). The CSR runs (slot-0 and Monte Carlo path bases)
// are short. The indirect paths are tiled (RenderArgs::ind_rows): a wave is one tile, its lanes
// its 64 primaries, and row s's masks say which lanes have a stored base (the others are +0,
// which adds nothing) and which a query; only those entries are read, 64 contiguous per row
// (a lane's entries past its own n_i are padding, never flagged).
__global__ __launch_bounds__(256) void reduce_prim_kernel(RenderArgs a) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t T = b >> 6;  // wave-uniform: blocks of whole waves
  if (T * 64 >= a.nprim) return;
  const bool own = b < a.nprim;
  const int lane = (int)(b & 63);
  const int64_t r0 = (int64_t)a.ind_rows[T];
  const int M = (int)((int64_t)a.ind_rows[T + 1] - r0);
  double c0 = 0, c1 = 0, c2 = 0;
  const double *bs = a.base;
  // RB entries' loads are issued before their additions (the sums stay in order): a primary on
  // the glass has hundreds of Monte Carlo paths and appends, and one dependent memory round trip
  // per entry made it the batch's longest thread
#ifndef REDUCE_RB
#define REDUCE_RB 8
#endif
  constexpr int RB = REDUCE_RB;
  if (own)
    for (uint32_t g0 = a.path_off[b], p1 = a.path_off[b + 1]; g0 < p1; g0 += RB) {
      double v[3 * RB];
#pragma unroll
      for (int u = 0; u < RB; u++) {
        const int64_t g = g0 + u < p1 ? (int64_t)g0 + u : (int64_t)g0;
        v[3 * u] = bs[3 * g];
        v[3 * u + 1] = bs[3 * g + 1];
        v[3 * u + 2] = bs[3 * g + 2];
      }
#pragma unroll
      for (int u = 0; u < RB; u++)
        if (g0 + u < p1) {
          c0 += v[3 * u];
          c1 += v[3 * u + 1];
          c2 += v[3 * u + 2];
        }
    }
  tiled_row_sum(a.ind_bmask, bs + 3 * a.ind_g0, r0, M, lane, c0, c1, c2);
  // each list in (primary, slot in primary, query in path) order: the primary's own query
  // (slot b), its Monte Carlo paths' appends (sorted), then (global list) its indirect paths'
  // queries (tiled slots, in path order); empty slots skipped
  for (int l = 0; l < 2; l++) {
    if (!a.qout[l]) continue;
    const uint64_t *qk = a.qkey[l];
    const double *qo = a.qout[l];
    auto add = [&](int64_t sl) {
      if (qk[sl] == ~0ull) return;
      c0 += qo[3 * sl];
      c1 += qo[3 * sl + 1];
      c2 += qo[3 * sl + 2];
    };
    if (own) {
      add(b);
      const uint32_t q0 = a.qseg[l][b], q1 = a.qseg[l][b + 1];
      const uint32_t *ss = a.sslot[l];
      const int64_t qa = (int64_t)a.qapp[l];
      for (uint32_t qb = q0; qb < q1; qb += RB) {
        int64_t sl[RB];
        bool on[RB];
        double v[3 * RB];
#pragma unroll
        for (int u = 0; u < RB; u++) sl[u] = qa + ss[qb + u < q1 ? qb + u : qb];
#pragma unroll
        for (int u = 0; u < RB; u++) on[u] = qb + u < q1 && qk[sl[u]] != ~0ull;
#pragma unroll
        for (int u = 0; u < RB; u++) {
          v[3 * u] = v[3 * u + 1] = v[3 * u + 2] = 0.0;
          if (on[u]) {
            v[3 * u] = qo[3 * sl[u]];
            v[3 * u + 1] = qo[3 * sl[u] + 1];
            v[3 * u + 2] = qo[3 * sl[u] + 2];
          }
        }
#pragma unroll
        for (int u = 0; u < RB; u++)
          if (on[u]) {
            c0 += v[3 * u];
            c1 += v[3 * u + 1];
            c2 += v[3 * u + 2];
          }
      }
    }
    if (l == 0) tiled_row_sum(a.ind_qmask, qo + 3 * a.qind_base, r0, M, lane, c0, c1, c2);
  }
  if (own) {
    a.prim_rgb[3 * b] = c0;
    a.prim_rgb[3 * b + 1] = c1;
    a.prim_rgb[3 * b + 2] = c2;
  }
}

// Pass 2, one thread per output pixel
__global__ __launch_bounds__(64) void reduce_kernel(RenderArgs a) {
  int pix = blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= a.npix) return;
  int af2 = a.af * a.af;
  double acc0 = 0, acc1 = 0, acc2 = 0;
  // row-major subsample order inside the pixel block (render.cpp:207-214 sums j-outer)
  for (int sub = 0; sub < af2; sub++) {
    double s0 = 0, s1 = 0, s2 = 0;
    for (int k = 0; k < a.dof_test; k++) {
      int64_t b = ((int64_t)pix * af2 + sub) * a.dof_test + k;
      s0 += a.prim_rgb[3 * b];
      s1 += a.prim_rgb[3 * b + 1];
      s2 += a.prim_rgb[3 * b + 2];
    }
    s0 /= a.dof_test; s1 /= a.dof_test; s2 /= a.dof_test;
    s0 = s0 < 0 ? 0 : (s0 > 1.0 ? 1.0 : s0);
    s1 = s1 < 0 ? 0 : (s1 > 1.0 ? 1.0 : s1);
    s2 = s2 < 0 ? 0 : (s2 > 1.0 ? 1.0 : s2);
    acc0 += s0; acc1 += s1; acc2 += s2;
  }
  double bw = 1.0 / a.af / a.af;
  double r = bw * acc0, g = bw * acc1, b = bw * acc2;
  int2 pc = a.pixels[pix];
  int64_t o = ((int64_t)pc.y * a.out_w + pc.x) * 3;
  if (a.rgbf) {
    a.rgbf[o] = (float)r;
    a.rgbf[o + 1] = (float)g;
    a.rgbf[o + 2] = (float)b;
  }
  if (a.rgb8) {
    a.rgb8[o] = (uint8_t)(255 * r);
    a.rgb8[o + 1] = (uint8_t)(255 * g);
    a.rgb8[o + 2] = (uint8_t)(255 * b);
  }
}

// ---------------------------------------------------------------------------------------
// Photon tracing (photontracer.cpp:28-373)
// ---------------------------------------------------------------------------------------
// RNRgb_to_RGBE, graphics_utils.cpp:50-61
__device__ __forceinline__ uint32_t rgbe_encode(C3 c) {
  double mx = maxch(c);
  if (!(mx > 0)) return 0u;
  int e;
  double m = frexp(mx, &e);
  uint32_t r = (uint8_t)(256.0 * c.r / mx * m);
  uint32_t g = (uint8_t)(256.0 * c.g / mx * m);
  uint32_t b = (uint8_t)(256.0 * c.b / mx * m);
  uint32_t x = (uint8_t)(e + 128);
  return r | (g << 8) | (b << 16) | (x << 24);
}

struct PhotonOut {
  gi_photon_dev *out;
  uint32_t off;     // PM_EMIT: this photon's first slot (scan of the PM_COUNT pass)
  uint32_t count;   // photons stored so far by this emitted photon (its store ordinal)
  // PM_APPEND
  uint32_t *cursor;
  uint64_t *keys;
  uint32_t cap;
  uint32_t obits;
  uint64_t j;       // emission index within the launch
};

// StorePhoton, photon_utils.cpp:40-65. PM_COUNT only counts; PM_EMIT writes at the slot the
// scan of the count pass gave; PM_APPEND takes a slot from one atomic per wave (ballot of the
// lanes storing at this bounce, prefix by popcount) and records the (emission index, store
// ordinal) key that restores emission order afterwards (photon_sort).
__device__ __forceinline__ void store_photon(int mode, PhotonOut &o, C3 power, V inc, V p) {
  if (mode != PM_COUNT) {
    gi_photon_dev ph;
    ph.pos[0] = (float)p.x;
    ph.pos[1] = (float)p.y;
    ph.pos[2] = (float)p.z;
    ph.rgbe = rgbe_encode(power);
    int phi = (uint8_t)(255.0 * (gm::atan2(inc.y, inc.x) + kPi) / (2.0 * kPi));
    double z = inc.z < -1.0 ? -1.0 : (inc.z > 1.0 ? 1.0 : inc.z);
    int theta = (uint8_t)(255.0 * gm::acos(z) / kPi);
    ph.dir = (uint16_t)(phi * 256 + theta);
    ph.flags = 0;
    if (mode == PM_EMIT) {
      o.out[o.off + o.count] = ph;
    } else {
      uint64_t act = __ballot(1);
      int lane = (int)(threadIdx.x & 63);
      int leader = __ffsll((long long)act) - 1;
      uint32_t rank = (uint32_t)__popcll(act & ((1ull << lane) - 1ull));
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(o.cursor, (uint32_t)__popcll(act));
      base = (uint32_t)__shfl((int)base, leader, 64);
      uint32_t slot = base + rank;
      if (slot < o.cap) {   // an overflowing launch is re-run with room (trace_batch_dev)
        o.out[slot] = ph;
        o.keys[slot] = (o.j << o.obits) | (uint64_t)o.count;
      }
    }
  }
  o.count++;
}

// PhotonTrace, photontracer.cpp:28-176
__device__ __noinline__ void photon_trace(const SceneView &S, const Flags &F, V org, V dir,
                                          C3 photon, bool caustic, Rng &rng, int mode,
                                          PhotonOut &o) {
  bool store = (!caustic && !F.fast_global);
  V ray_start = org;
  int hint = -1;  // the triangle each bounce leaves from (ray_mesh_bvh)
  for (int iter = 0; iter < F.max_photon_depth; iter++) {
    Hit h;
    if (!scene_intersect(S, org, dir, h, hint)) break;
    hint = h.tri;
    const DMaterial &m = S.mats[h.mat];
    V view = normalize(h.p - ray_start);
    double ct = dot(h.n, -view);
    if ((m.flags & MF_DIFFUSE) && store) store_photon(mode, o, photon, view, h.p);
    double R = 0;
    if (F.fresnel && (m.flags & MF_TRANSPARENT)) R = reflection_coeff(F.ir_air, ct, m.ir);
    double mc = maxch(photon);
    double pd = maxch(ldc(m.kd) * photon) / mc;
    double pt = maxch(ldc(m.kt) * photon) / mc;
    double ps = (maxch(ldc(m.ks) * photon) / mc) + R * pt;
    pt *= (1.0 - R);
    double ptot = pd + pt + ps + F.prob_absorb;
    double rnd = rng.next();
    if (ptot > 1.0) rnd *= ptot;
    V sb;
    if (rnd < pd) {
      if (caustic) break;
      store = true;
      sb = diffuse_sample(h.n, ct, rng);
      photon *= ldc(m.kd) / pd;
    } else if (rnd < pd + pt) {
      if (caustic) store = true;
      V ex = transmissive_bounce(F.ir_air, h.n, view, ct, m.ir);
      sb = F.distrib_trans ? specular_sample(ex, m.n, ct, rng) : ex;
      photon *= (1.0 - R) * ldc(m.kt) / pt;
    } else if (rnd < pd + pt + ps) {
      if (caustic) store = true;
      V ex = reflective_bounce(h.n, view, ct);
      sb = F.distrib_spec ? specular_sample(ex, m.n, ct, rng) : ex;
      photon *= (ldc(m.ks) + R * ldc(m.kt)) / ps;
    } else {
      break;
    }
    ray_start = h.p + sb * kEps;
    org = ray_start;
    dir = sb;
  }
}

// EmitPhotons, photontracer.cpp:182-373, one photon per lane (emission index e0 + lane)
template <int MODE>
__global__ __launch_bounds__(128) void photon_kernel(PhotonArgs a) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= a.n) return;
  const SceneView &S = a.S;
  const Flags &F = a.F;
  const DLight &L = S.lights[a.light];
  Rng rng;
  rng.init(F.seed, a.caustic ? KIND_PHOTON_CAUSTIC : KIND_PHOTON_GLOBAL, (uint64_t)(a.e0 + j), 0);
  C3 photon = ldc(L.color);
  double tot = photon.r + photon.g + photon.b;  // NormalizeColor, graphics_utils.cpp:25-36
  if (tot > 0) photon = photon / tot;
  V org, dir;
  if (L.kind == LK_DIR) {
    V ln = ld3(L.dir);
    V center = ld3(S.centroid) - ln * S.radius * 3.0;
    double r1, r2;
    do {
      r1 = rng.next() * 2.0 - 1.0;
      r2 = rng.next() * 2.0 - 1.0;
    } while (r1 * r1 + r2 * r2 > 1.0);
    org = ((r1 * ld3(L.su) + r2 * ld3(L.sv)) + center) + ln * kEps;
    dir = ln;
  } else if (L.kind == LK_POINT) {
    double x, y, z;
    do {
      x = rng.next() * 2.0 - 1.0;
      y = rng.next() * 2.0 - 1.0;
      z = rng.next() * 2.0 - 1.0;
    } while (x * x + y * y + z * z > 1.0);
    org = ld3(L.pos);
    dir = normalize(mk(x, y, z));
  } else if (L.kind == LK_SPOT) {
    V ln = ld3(L.dir);
    double cutoff = fabs(gm::cos(L.cutoff));
    int attempts_left = 20;
    V sd;
    do {
      sd = specular_sample(ln, L.dropoff, 1.0, rng);
    } while (dot(sd, ln) < cutoff && attempts_left-- > 0);
    if (attempts_left == 0) sd = specular_sample(ln, L.dropoff, cutoff, rng);
    org = ld3(L.pos);
    dir = sd;
  } else if (L.kind == LK_AREA) {
    V ln = ld3(L.dir);
    double r1, r2;
    do {
      r1 = rng.next() * 2.0 - 1.0;
      r2 = rng.next() * 2.0 - 1.0;
    } while (r1 * r1 + r2 * r2 > 1.0);
    org = ((r1 * ld3(L.su) + r2 * ld3(L.sv)) + ld3(L.pos)) + ln * kEps;
    dir = diffuse_sample(ln, 1.0, rng);
  } else {
    V ln = ld3(L.dir);
    double r1 = rng.next() - 0.5;
    double r2 = rng.next() - 0.5;
    org = ((r1 * ld3(L.su) + r2 * ld3(L.sv)) + ld3(L.pos)) + ln * kEps;
    dir = diffuse_sample(ln, 1.0, rng);
  }
  PhotonOut o;
  o.out = a.out;
  o.off = MODE == PM_EMIT ? a.offsets[j] : 0u;
  o.count = 0;
  o.cursor = a.cursor;
  o.keys = a.keys;
  o.cap = a.cap;
  o.obits = (uint32_t)a.obits;
  o.j = (uint64_t)j;
  photon_trace(S, F, org, dir, photon, a.caustic != 0, rng, MODE, o);
  if (MODE == PM_COUNT) a.counts[j] = o.count;
}

// the appended photons in (emission index, store ordinal) order: dst[i] = src[slot[i]]
__global__ __launch_bounds__(256) void photon_gather_kernel(const gi_photon_dev *src,
                                                            const uint32_t *slot, int64_t n,
                                                            gi_photon_dev *dst) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[slot[i]];
}

// power rescale (Q9, photonmap.cpp:339-361) of a device map: RGBE -> RNRgb, * pp, -> RGBE
__global__ __launch_bounds__(256) void photon_rescale_kernel(gi_photon_dev *ph, int64_t n,
                                                             double pp) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t v = ph[i].rgbe;
  uint32_t e = v >> 24;
  C3 c = rgb(0.0, 0.0, 0.0);
  if (e) {
    double inv = ldexp(1.0, (int)e - 128 - 8);   // RGBE_to_RNRgb, graphics_utils.cpp:64-77
    c = rgb((double)(v & 255u) * inv, (double)((v >> 8) & 255u) * inv,
            (double)((v >> 16) & 255u) * inv);
  }
  c = c * pp;
  ph[i].rgbe = rgbe_encode(c);
}

// directional-light disk basis needs the scene radius: computed on host (gi_host.cpp)

// ---------------------------------------------------------------------------------------
// R3Scene::Intersects test seam
// ---------------------------------------------------------------------------------------
__global__ void intersect_kernel(SceneView S, int64_t n, const double *org, const double *dir,
                                 int32_t *hit, double *t, double *point, double *normal,
                                 int32_t *mat) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Hit h;
  bool ok = scene_intersect(S, ld3(org + 3 * i), ld3(dir + 3 * i), h);
  hit[i] = ok;
  t[i] = ok ? h.t : 0.0;
  point[3 * i] = ok ? h.p.x : 0; point[3 * i + 1] = ok ? h.p.y : 0; point[3 * i + 2] = ok ? h.p.z : 0;
  normal[3 * i] = ok ? h.n.x : 0; normal[3 * i + 1] = ok ? h.n.y : 0; normal[3 * i + 2] = ok ? h.n.z : 0;
  mat[i] = ok ? h.mat : -2;
}

// ---------------------------------------------------------------------------------------
// host-callable launchers
// ---------------------------------------------------------------------------------------
static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

hipError_t launch_scan(const uint32_t *in, uint32_t *out, int64_t n, ScanTemp &tmp,
                       hipStream_t st) {
  // out has n+1 entries; out[n] = total
  if (n <= 0) {
    return hipMemsetAsync(out, 0, sizeof(uint32_t), st);
  }
  int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  uint32_t *sums = tmp.level[tmp.depth];
  uint32_t *soff = tmp.level_out[tmp.depth];
  // write total via an extra padded element: scan n+1 with in[n] treated as 0
  scan_tile_kernel<<<nblk(n, SCAN_TILE), SCAN_BLOCK, 0, st>>>(in, out, sums, n);
  if (nb > 1) {
    tmp.depth++;
    hipError_t e = launch_scan(sums, soff, nb, tmp, st);
    tmp.depth--;
    if (e != hipSuccess) return e;
    scan_add_kernel<<<nblk(n, 256), 256, 0, st>>>(out, soff, n);
    // total = soff[nb]
    return hipMemcpyAsync(out + n, soff + nb, sizeof(uint32_t), hipMemcpyDeviceToDevice, st);
  }
  return hipMemcpyAsync(out + n, sums, sizeof(uint32_t), hipMemcpyDeviceToDevice, st);
}

void launch_primary(const RenderArgs &a, hipStream_t st) {
  primary_kernel<<<nblk(a.nprim, 256), 256, 0, st>>>(a);
}
// occupancy: 4 waves per SIMD where the kernel fits 128 VGPRs without spills (triangles and
// spheres only; C2 ind_kernel 37.8 -> 31.3 ms, frame -2.6 %), else 3 (the 4-wave instances of
// the other element sets spill 74-129 VGPRs; 3 or 5 waves for triangles and spheres measured
// slower, profiles/r05_ind_waves_ab.txt)
template <uint32_t KINDS>
void launch_ind(const RenderArgs &a, unsigned g, hipStream_t st) {
  if (KINDS == KINDS_TRI_SPHERE) ind_kernel<4, true, KINDS><<<g, 128, 0, st>>>(a);
  else ind_kernel<3, true, KINDS><<<g, 128, 0, st>>>(a);
}
void launch_cont(const RenderArgs &a, const IndCont *q, const uint32_t *fill, uint32_t cap_s,
                 hipStream_t st) {
  if ((a.S.kinds & ~KINDS_TRI_SPHERE) == 0)
    ind_cont_kernel<KINDS_TRI_SPHERE><<<IND_QS * 32, 128, 0, st>>>(a, q, fill, cap_s);
  else if ((a.S.kinds & ~KINDS_POLY) == 0)
    ind_cont_kernel<KINDS_POLY><<<IND_QS * 32, 128, 0, st>>>(a, q, fill, cap_s);
  else
    ind_cont_kernel<KINDS_ALL><<<IND_QS * 32, 128, 0, st>>>(a, q, fill, cap_s);
}
static void launch_mc_sub(const RenderArgs &a, hipStream_t st) {
  if ((a.S.kinds & ~KINDS_TRI_SPHERE) == 0)
    mc_sub_kernel<KINDS_TRI_SPHERE><<<IND_QS * 32, 128, 0, st>>>(a, a.mc_cont, a.mc_ncont, a.mc_cap_s);
  else if ((a.S.kinds & ~KINDS_POLY) == 0)
    mc_sub_kernel<KINDS_POLY><<<IND_QS * 32, 128, 0, st>>>(a, a.mc_cont, a.mc_ncont, a.mc_cap_s);
  else
    mc_sub_kernel<KINDS_ALL><<<IND_QS * 32, 128, 0, st>>>(a, a.mc_cont, a.mc_ncont, a.mc_cap_s);
}
// Path expansion of one batch. The Monte Carlo paths (mc_kernel: few, long, one wave per SIMD
// by its registers) run on the side stream st2 when given, concurrently with the indirect paths
// on st, so their waves share the CUs instead of running as a low-occupancy tail; st waits for
// them before returning (fork/join events). The two kernels write disjoint path slots and
// append queries through the same atomic counters.
void launch_path(const RenderArgs &a, hipStream_t st, hipStream_t st2, hipEvent_t fork,
                 hipEvent_t join, bool wait_join) {
  const bool side = st2 && fork && join && a.total_mc > 0;
  hipStream_t ms = side ? st2 : st;
  // the Monte Carlo queues' counters are zeroed on st before the fork: a fill on the side stream
  // waits for a CU slot behind st's kernels (rocprof: single fills of 42 ms at C2 and 170 ms
  // at C3 with the persistent kernel), and the side stream's kernels wait behind it
  if (a.total_mc > 0 && a.mc_cont) {
    (void)hipMemsetAsync(a.mc_ncont, 0, IND_QS * 32 * sizeof(uint32_t), st);
    if (a.mc_next) (void)hipMemsetAsync(a.mc_next, 0, sizeof(uint32_t), st);
    if (a.mc_cont2) (void)hipMemsetAsync(a.mc_ncont2, 0, IND_QS * 32 * sizeof(uint32_t), st);
  }
  // the same for the indirect continuation queue's counters: cleared before the fork, not after
  // it on st, where the fill waited for the persistent Monte Carlo kernel (whose 1,024 blocks of
  // 256-VGPR waves take every SIMD's registers) to release a CU -- C3's 40-162 ms single fills,
  // 725 ms over two frames
  if (a.total_ind > 0 && a.split_ind)
    (void)hipMemsetAsync(a.ind_ncont, 0, IND_QS * 32 * sizeof(uint32_t), st);
  if (side) {
    (void)hipEventRecord(fork, st);
    (void)hipStreamWaitEvent(st2, fork, 0);
  }
  // the primaries' own slots first: enqueued behind the Monte Carlo kernel, this small kernel
  // waited for CU slots until that kernel's blocks drained (cold C2 frame: 47 ms), holding back
  // the indirect kernel behind it on st; it reads and writes nothing the Monte Carlo paths touch
  if (a.nprim > 0) slot0_kernel<<<nblk(a.nprim, 256), 256, 0, st>>>(a);
  if (a.total_mc > 0) {
    unsigned g = nblk(a.total_mc, 128);
    if (a.mc_cont && a.mc_next) {
      // persistent: enough blocks to fill the chip at MC_WPE waves per SIMD, or one per 128 paths
      unsigned gp = std::min(g, (unsigned)(a.mc_persist_blocks > 0 ? a.mc_persist_blocks : 1024));
      if ((a.S.kinds & ~KINDS_TRI_SPHERE) == 0) {
        if (a.S.hard_lights) mc_persist_kernel<KINDS_TRI_SPHERE, true, true><<<gp, 128, 0, ms>>>(a);
        else mc_persist_kernel<KINDS_TRI_SPHERE, true, false><<<gp, 128, 0, ms>>>(a);
      } else if ((a.S.kinds & ~KINDS_POLY) == 0) {
        if (a.S.hard_lights) mc_persist_kernel<KINDS_POLY, true, true><<<gp, 128, 0, ms>>>(a);
        else mc_persist_kernel<KINDS_POLY, true, false><<<gp, 128, 0, ms>>>(a);
      } else {
        mc_persist_kernel<KINDS_ALL, true, false><<<gp, 128, 0, ms>>>(a);
      }
    } else if (a.mc_cont) {
      if ((a.S.kinds & ~KINDS_TRI_SPHERE) == 0) {
        if (a.S.hard_lights) mc_kernel<KINDS_TRI_SPHERE, true, true><<<g, 128, 0, ms>>>(a);
        else mc_kernel<KINDS_TRI_SPHERE, true, false><<<g, 128, 0, ms>>>(a);
      } else if ((a.S.kinds & ~KINDS_POLY) == 0) {
        if (a.S.hard_lights) mc_kernel<KINDS_POLY, true, true><<<g, 128, 0, ms>>>(a);
        else mc_kernel<KINDS_POLY, true, false><<<g, 128, 0, ms>>>(a);
      } else {
        mc_kernel<KINDS_ALL, true, false><<<g, 128, 0, ms>>>(a);
      }
    }
    if (a.mc_cont) {
      if (a.mc_cont2) {
        launch_mc_sub(a, ms);
        launch_cont(a, a.mc_cont2, a.mc_ncont2, a.mc_cap_s, ms);
      } else {
        launch_cont(a, a.mc_cont, a.mc_ncont, a.mc_cap_s, ms);
      }
    } else {
      mc_kernel<KINDS_ALL, false, false><<<g, 128, 0, ms>>>(a);
    }
  }
  if (a.total_ind > 0) {
    unsigned g = nblk(a.tind, 128);
    if (!a.split_ind) ind_kernel<2, false, KINDS_ALL><<<g, 128, 0, st>>>(a);
    else if ((a.S.kinds & ~KINDS_TRI_SPHERE) == 0) launch_ind<KINDS_TRI_SPHERE>(a, g, st);
    else if ((a.S.kinds & ~KINDS_POLY) == 0) launch_ind<KINDS_POLY>(a, g, st);
    else launch_ind<KINDS_ALL>(a, g, st);
    // continuations: 32 blocks per stripe stride over its fill
    if (a.split_ind) launch_cont(a, a.ind_cont, a.ind_ncont, a.ind_cap_s, st);
  }
  if (side) {
    (void)hipEventRecord(join, st2);
    if (wait_join) (void)hipStreamWaitEvent(st, join, 0);
  }
}
// Shard gather of a device set (gi_host.cpp render_multi): a device's output pixels packed in
// its pixel-list order as {r, g, b, rgb8 bytes} (16 B), and their scatter on the first device.
__global__ void pack_pixels_kernel(const int2 *pix, int64_t n, int w, const float *rgbf,
                                   const uint8_t *rgb8, uint4 *out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int2 p = pix[i];
  size_t o = 3 * ((size_t)p.y * w + p.x);
  uint32_t b = (uint32_t)rgb8[o] | ((uint32_t)rgb8[o + 1] << 8) | ((uint32_t)rgb8[o + 2] << 16);
  out[i] = make_uint4(__float_as_uint(rgbf[o]), __float_as_uint(rgbf[o + 1]),
                      __float_as_uint(rgbf[o + 2]), b);
}
__global__ void unpack_pixels_kernel(const int2 *pix, int64_t n, int w, const uint4 *in,
                                     float *rgbf, uint8_t *rgb8) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int2 p = pix[i];
  size_t o = 3 * ((size_t)p.y * w + p.x);
  uint4 v = in[i];
  rgbf[o] = __uint_as_float(v.x);
  rgbf[o + 1] = __uint_as_float(v.y);
  rgbf[o + 2] = __uint_as_float(v.z);
  rgb8[o] = (uint8_t)(v.w & 255u);
  rgb8[o + 1] = (uint8_t)((v.w >> 8) & 255u);
  rgb8[o + 2] = (uint8_t)((v.w >> 16) & 255u);
}
void launch_pack_pixels(const int32_t *pix_xy, int64_t n, int w, const float *rgbf,
                        const uint8_t *rgb8, void *out, hipStream_t st) {
  if (n == 0) return;
  pack_pixels_kernel<<<nblk(n, 256), 256, 0, st>>>(reinterpret_cast<const int2 *>(pix_xy), n, w,
                                                   rgbf, rgb8, reinterpret_cast<uint4 *>(out));
}
void launch_unpack_pixels(const int32_t *pix_xy, int64_t n, int w, const void *in, float *rgbf,
                          uint8_t *rgb8, hipStream_t st) {
  if (n == 0) return;
  unpack_pixels_kernel<<<nblk(n, 256), 256, 0, st>>>(reinterpret_cast<const int2 *>(pix_xy), n, w,
                                                     reinterpret_cast<const uint4 *>(in), rgbf,
                                                     rgb8);
}
void launch_ind_tiles(const uint32_t *nind, int64_t nprim, uint32_t *rows, hipStream_t st) {
  ind_tile_rows_kernel<<<(unsigned)((nprim + 63) / 64), 64, 0, st>>>(nind, nprim, rows);
}

// tab[r] = T << 32 | s for row r = ind_rows[T] + s of the tiled indirect entries (thread per tile)
__global__ void ind_row_tile_kernel(const uint32_t *rows, int64_t ntiles, uint64_t *tab) {
  const int64_t T = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (T >= ntiles) return;
  const uint32_t r0 = rows[T];
  for (uint32_t r = r0; r < rows[T + 1]; r++) tab[r] = ((uint64_t)T << 32) | (r - r0);
}

void launch_ind_row_tile(const uint32_t *rows, int64_t ntiles, uint64_t *tab, hipStream_t st) {
  if (ntiles > 0) ind_row_tile_kernel<<<nblk(ntiles, 256), 256, 0, st>>>(rows, ntiles, tab);
}

void launch_ind_pad(const RenderArgs &a, hipStream_t st) {
  ind_pad_kernel<<<nblk((a.nprim + 63) & ~(int64_t)63, 256), 256, 0, st>>>(a);
}

void launch_owner_table(const uint32_t *off, int64_t n, uint32_t *tab, hipStream_t st) {
  if (n > 0) owner_table_kernel<<<nblk(n, 256), 256, 0, st>>>(off, n, tab);
}
void launch_reduce(const RenderArgs &a, hipStream_t st) {
  reduce_prim_kernel<<<nblk((a.nprim + 63) & ~(int64_t)63, 256), 256, 0, st>>>(a);
  reduce_kernel<<<nblk(a.npix, 64), 64, 0, st>>>(a);
}
void launch_knn(const KnnArgs &a, hipStream_t st) {
  if (a.nq == 0) return;
  knn_kernel<<<nblk(a.nq, 64 * a.qpl), 64, 0, st>>>(a);
}
void launch_cached(const KnnArgs &a, hipStream_t st) {
  if (a.nq == 0) return;
  cached_kernel<<<nblk(a.nq, 64), 64, 0, st>>>(a);
}
void launch_photons(const PhotonArgs &a, int mode, hipStream_t st) {
  if (a.n == 0) return;
  if (mode == PM_EMIT) photon_kernel<PM_EMIT><<<nblk(a.n, 128), 128, 0, st>>>(a);
  else if (mode == PM_COUNT) photon_kernel<PM_COUNT><<<nblk(a.n, 128), 128, 0, st>>>(a);
  else photon_kernel<PM_APPEND><<<nblk(a.n, 128), 128, 0, st>>>(a);
}
void launch_photon_gather(const gi_photon_dev *src, const uint32_t *slot, int64_t n,
                          gi_photon_dev *dst, hipStream_t st) {
  if (n > 0) photon_gather_kernel<<<nblk(n, 256), 256, 0, st>>>(src, slot, n, dst);
}
void launch_photon_rescale(gi_photon_dev *ph, int64_t n, double pp, hipStream_t st) {
  if (n > 0) photon_rescale_kernel<<<nblk(n, 256), 256, 0, st>>>(ph, n, pp);
}
// gi_math_probe: the device's fp64 math as the path kernels call it (gi_math.h; sqrt: the
// correctly rounded hardware sequence)
__global__ void math_probe_kernel(int fn, int64_t n, const double *x, const double *y,
                                  double *out) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = x[i], b = y[i], r = 0.0;
  switch (fn) {
    case 0: r = gm::acos(a); break;
    case 1: r = gm::sin(a); break;
    case 2: r = gm::cos(a); break;
    case 3: r = gm::pow(a, b); break;
    case 4: r = gm::atan2(a, b); break;
    case 6: r = gm::tan(a); break;
    case 7: r = gm::asin(a); break;
    default: r = sqrt(a); break;
  }
  out[i] = r;
}
void launch_math_probe(int fn, int64_t n, const double *x, const double *y, double *out,
                       hipStream_t st) {
  if (n > 0) math_probe_kernel<<<nblk(n, 256), 256, 0, st>>>(fn, n, x, y, out);
}
void launch_intersect(const SceneView &S, int64_t n, const double *org, const double *dir,
                      int32_t *hit, double *t, double *point, double *normal, int32_t *mat,
                      hipStream_t st) {
  if (n == 0) return;
  intersect_kernel<<<nblk(n, 128), 128, 0, st>>>(S, n, org, dir, hit, t, point, normal, mat);
}

}  // namespace gi
