// gi_knn.hip -- wave-cooperative k-nearest-photon radiance estimate (the dominant kernel).
//
// Re-expresses R3Kdtree<Photon*>::FindClosestQuick (R3Kdtree.cpp:688-784) + EstimateRadiance
// (photon_utils.cpp:72-162) for CDNA4: ONE QUERY PER WAVE.
//   * traversal of the implicit kd-tree is wave-uniform: node ids, split planes and leaf
//     ranges live in SGPRs (scalar loads), nearest-first, stackless (parent = node>>1);
//   * leaves hold <= 64 photons: one photon per lane, one coalesced 16-B load per lane;
//   * candidates with key = (d2 bits << 32 | photon index) below the current threshold are
//     appended to an LDS buffer by ballot/mbcnt compaction; when the buffer cannot take the
//     next leaf, a radix select (LDS histograms) keeps the K best and tightens the threshold
//     (the reference's delayed make_heap + replace-max, R3Kdtree.cpp:753-782, as a batched
//     selection). Result set: the K smallest (d2, index) pairs with d2 <= r2 -- identical
//     to the reference's set up to ties at the K-th distance.
//   * the estimate sums the K photons across lanes and reduces in registers.
// LDS per wave: CAP * 8 bytes (1 KiB for K <= 64, 4 KiB for K <= 448), so occupancy is set
// by registers, not by a per-lane heap.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include "gi_device.h"
#include "gi_kernels.h"

namespace gi {

__device__ __forceinline__ uint32_t ufirst(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ float ffirst(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wave-level radix select over the candidate buffer buf[0, count): find the K-th smallest
// key T, keep exactly the keys <= T (compacted to buf[0, K)) and set thr = T (a later
// candidate must be < T). Digits: the 4 bytes of the d2 bits, MSB first, each a 256-bin LDS
// histogram + wave prefix scan; the index bytes are resolved only when several keys share
// the K-th distance. Keys are re-read from LDS on every pass (no per-lane key arrays: the
// register budget sets this kernel's occupancy).
__device__ __forceinline__ uint32_t radix_pick(uint32_t *hist, int lane, uint32_t &need) {
  uint32_t c0 = hist[4 * lane], c1 = hist[4 * lane + 1], c2 = hist[4 * lane + 2],
           c3 = hist[4 * lane + 3];
  uint32_t sum = c0 + c1 + c2 + c3, inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = (uint32_t)__shfl_up((int)inc, o, 64);
    if (lane >= o) inc += t;
  }
  uint32_t exc = inc - sum;
  uint64_t hit = __ballot(exc < need && need <= inc);
  int L = __ffsll((long long)hit) - 1;
  uint32_t d = 0, before = exc;
  if (lane == L) {
    if (need <= before + c0) d = 0;
    else if (need <= before + c0 + c1) { d = 1; before += c0; }
    else if (need <= before + c0 + c1 + c2) { d = 2; before += c0 + c1; }
    else { d = 3; before += c0 + c1 + c2; }
    d = 4 * (uint32_t)lane + d;
  }
  need -= (uint32_t)__shfl((int)before, L, 64);
  return (uint32_t)__shfl((int)d, L, 64);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// Narrow [lo, hi] (inclusive, u32 digit values of the keys that pass `member`) to the single
// value of the need-th smallest, with 256-bin LDS histograms over the live range: pass p bins
// by (v - lo) >> shift with 2^shift the smallest power of two giving <= 256 bins. Unlike fixed
// radix bytes, the bins always span the keys actually present (a fixed top byte of nearby d2
// values is one exponent: every lane's LDS atomic would hit one or two bins).
template <typename Digit, typename Member>
__device__ __forceinline__ uint32_t range_select(const uint64_t *buf, uint32_t *hist, int lane,
                                                 uint32_t count, uint32_t &need, uint32_t lo,
                                                 uint32_t hi, Digit digit, Member member) {
  while (hi > lo) {
    uint32_t span = hi - lo;
    int shift = 32 - __clz((int)span) - 8;
    if (shift < 0) shift = 0;
    hist[4 * lane] = hist[4 * lane + 1] = hist[4 * lane + 2] = hist[4 * lane + 3] = 0u;
    __syncthreads();
    for (uint32_t s = (uint32_t)lane; s < count; s += 64) {
      uint64_t k = buf[s];
      uint32_t v = digit(k);
      if (member(k) && v >= lo && v <= hi) atomicAdd(&hist[(v - lo) >> shift], 1u);
    }
    __syncthreads();
    uint32_t B = radix_pick(hist, lane, need);
    __syncthreads();
    uint32_t nlo = lo + (B << shift);
    uint32_t w = (shift >= 32) ? 0xffffffffu : ((1u << shift) - 1u);
    hi = (hi - nlo > w) ? nlo + w : hi;
    lo = nlo;
  }
  return lo;
}

// Wave-level selection over the candidate buffer buf[0, count): find the K-th smallest key T,
// keep exactly the keys <= T (compacted to buf[0, K)) and set thr = T (a later candidate must
// be < T). The d2 bits are resolved by range_select; the index bits only when several keys
// share the K-th distance. Keys are re-read from LDS on every pass (no per-lane key arrays:
// the register budget sets this kernel's occupancy).
template <int CAP>
__device__ __forceinline__ void select_k(uint64_t *buf, uint32_t *hist, int lane, uint32_t &count,
                                         int K, uint64_t &thr) {
  uint32_t lo = 0xffffffffu, hi = 0u;
  for (uint32_t s = (uint32_t)lane; s < count; s += 64) {
    uint32_t h = (uint32_t)(buf[s] >> 32);
    lo = min(lo, h);
    hi = max(hi, h);
  }
  lo = wave_min_u32(lo);
  hi = wave_max_u32(hi);
  uint32_t need = (uint32_t)K;
  const uint32_t prefix = range_select(buf, hist, lane, count, need, lo, hi,
                                       [](uint64_t k) { return (uint32_t)(k >> 32); },
                                       [](uint64_t) { return true; });
  // prefix = d2 bits of the K-th key; `need` of the keys with exactly that d2 are kept
  uint32_t eq = 0, ilo = 0xffffffffu, ihi = 0u;
  for (uint32_t s0 = 0; s0 < count; s0 += 64) {
    uint32_t s = s0 + (uint32_t)lane;
    uint64_t k = (s < count) ? buf[s] : ~0ull;
    bool e = s < count && (uint32_t)(k >> 32) == prefix;
    if (e) {
      ilo = min(ilo, (uint32_t)k);
      ihi = max(ihi, (uint32_t)k);
    }
    eq += (uint32_t)__popcll(__ballot(e));
  }
  uint32_t tidx = 0xffffffffu;
  if (need < eq)
    tidx = range_select(buf, hist, lane, count, need, wave_min_u32(ilo), wave_max_u32(ihi),
                        [](uint64_t k) { return (uint32_t)k; },
                        [prefix](uint64_t k) { return (uint32_t)(k >> 32) == prefix; });
  uint64_t T = ((uint64_t)prefix << 32) | (uint64_t)tidx;
  // compact the keys <= T (exactly K) to buf[0, K); writes never pass unread entries
  uint32_t base = 0;
  for (uint32_t s0 = 0; s0 < count; s0 += 64) {
    uint32_t s = s0 + (uint32_t)lane;
    uint64_t k = (s < count) ? buf[s] : ~0ull;
    bool keep = (s < count) && k <= T;
    uint64_t m = __ballot(keep);
    if (keep) buf[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = k;
    base += (uint32_t)__popcll(m);
  }
  __syncthreads();
  count = base;  // == K
  thr = T;
}

// EstimateRadiance / EstimateIrradiance (photon_utils.cpp:72-162, 209-246) of one query from its
// num K-best photons (fetch_id(s), fetch_d2(s) for s < num), one wave per query: photons spread
// over the lanes, fp64 partial sums reduced across the wave (butterfly). Shared by the
// list-estimate kernel and the wave kernel's fused estimate, so both sum in the same order.
template <bool GEN = true, typename FetchId, typename FetchD2>
__device__ __forceinline__ void wave_estimate(const KnnArgs &a, int64_t qi, float4 qp, int num,
                                              FetchId fetch_id, FetchD2 fetch_d2) {
  const int lane = threadIdx.x;
  const int K = a.K;
  double maxd2 = kEps;
  double o0 = 0, o1 = 0, o2 = 0;
  if (num > 0) {
    if (num < K) {
      maxd2 = a.rmax * a.rmax;
    } else {
      double lm = 0.0;
      for (int s = lane; s < num; s += 64) {
        double d = (double)fetch_d2(s);
        lm = d > lm ? d : lm;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        double t = __shfl_xor(lm, o, 64);
        lm = t > lm ? t : lm;
      }
      if (lm > maxd2) maxd2 = lm;
    }
    if (a.mode == KNN_MODE_IRRADIANCE) {
      for (int s = lane; s < num; s += 64) {
        uint32_t e = a.map.rgbe[fetch_id(s)];
        uint32_t ee = e >> 24;
        if (ee) {
          double inv = ldexp(1.0, (int)ee - 128 - 8);
          o0 += (double)(e & 255u) * inv;
          o1 += (double)((e >> 8) & 255u) * inv;
          o2 += (double)((e >> 16) & 255u) * inv;
        }
      }
      o0 = wave_sum(o0); o1 = wave_sum(o1); o2 = wave_sum(o2);
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
      // without the specular term, ap * kd + 0 * ks == ap * kd up to the sign of a zero (for
      // finite ks), and the sums start at +0, so dropping the 0 * ks products changes no result
      const bool diff_only = !spec && isfinite(m.ks[0]) && isfinite(m.ks[1]) && isfinite(m.ks[2]);
      double c1 = 1.0, c2 = 1.0, tw = 0;
      if (a.filter == 1) c1 = 1.0 / (a.fk * sqrt(maxd2));
      else if (a.filter == 2) {
        c1 = pow_call(2.7182818284590452354, -a.fb);
        c2 = 1.0 / (2.0 * maxd2);
      }
      if (a.filter == 0 && diff_only) {
        // common case (disk filter, no specular term): the lane's photons s, s + 64, ... in
        // groups of four, their list, direction-code, rgbe and LUT loads in flight together;
        // each lane still sums its photons in increasing s
        for (int s0 = lane; s0 < num; s0 += 256) {
          uint32_t ids[4], ee[4], dcs[4];
          double lx[4], ly[4], lz[4];
#pragma unroll
          for (int u = 0; u < 4; u++) ids[u] = fetch_id(s0 + 64 * u < num ? s0 + 64 * u : s0);
#pragma unroll
          for (int u = 0; u < 4; u++) {
            dcs[u] = __float_as_uint(a.map.pos4[4 * (int64_t)ids[u] + 3]) & 0xffffu;
            ee[u] = a.map.rgbe[ids[u]];
          }
#pragma unroll
          for (int u = 0; u < 4; u++) {
            lx[u] = a.lut[3 * dcs[u]];
            ly[u] = a.lut[3 * dcs[u] + 1];
            lz[u] = a.lut[3 * dcs[u] + 2];
          }
#pragma unroll
          for (int u = 0; u < 4; u++) {
            if (s0 + 64 * u >= num) break;
            double perp = N0 * lx[u] + N1 * ly[u] + N2 * lz[u];
            if ((sign == 2u && perp < 0) || (sign == 1u && perp > 0)) continue;
            uint32_t e = ee[u];
            uint32_t x = e >> 24;
            double inv = x ? ldexp(1.0, (int)x - 128 - 8) : 0.0;
            double p0 = x ? (double)(e & 255u) * inv : 0.0;
            double p1 = x ? (double)((e >> 8) & 255u) * inv : 0.0;
            double p2 = x ? (double)((e >> 16) & 255u) * inv : 0.0;
            double ap = fabs(perp);
            p0 *= ap * m.kd[0];
            p1 *= ap * m.kd[1];
            p2 *= ap * m.kd[2];
            o0 += p0; o1 += p1; o2 += p2;
          }
        }
      } else if constexpr (!GEN) {
        o0 = o1 = o2 = __builtin_nan("");  // see chunk_estimate: the host's check failed
        if (a.stats) atomicAdd(a.stats + ST_GEN_MISS, 1ull);
      } else
      for (int s = lane; s < num; s += 64) {
        uint32_t id = fetch_id(s);
        double d2 = (double)fetch_d2(s);
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
        if (diff_only) {
          p0 *= ap * m.kd[0];
          p1 *= ap * m.kd[1];
          p2 *= ap * m.kd[2];
        } else {
          double pw = spec ? pow_call(ca, m.n) : 0.0;
          p0 *= ap * m.kd[0] + pw * m.ks[0];
          p1 *= ap * m.kd[1] + pw * m.ks[1];
          p2 *= ap * m.kd[2] + pw * m.ks[2];
        }
        if (a.filter == 1) {
          double f = (1.0 - c1 * sqrt(d2));
          p0 *= f; p1 *= f; p2 *= f;
        } else if (a.filter == 2) {
          double w = (1.0 - (1.0 - pow_call(c1, c2 * d2)) / (1.0 - c1));
          p0 *= w; p1 *= w; p2 *= w;
          tw += w;
        }
        o0 += p0; o1 += p1; o2 += p2;
      }
      o0 = wave_sum(o0); o1 = wave_sum(o1); o2 = wave_sum(o2);
      if (a.filter == 2) tw = wave_sum(tw);
      bool ok = true;
      if (a.filter == 0 && maxd2 > 0) {
        double den = kPi * maxd2;
        o0 /= den; o1 /= den; o2 /= den;
      } else if (a.filter == 1 && maxd2 > 0) {
        double den = (1.0 - 2.0 / 3.0 / a.fk) * kPi * maxd2;
        o0 /= den; o1 /= den; o2 /= den;
      } else if (a.filter == 2 && tw > 0 && maxd2 > 0) {
        double sc = a.fa * (num / tw) / (kPi * maxd2);
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
  if (lane == 0) {
    a.out[3 * qi] = o0;
    a.out[3 * qi + 1] = o1;
    a.out[3 * qi + 2] = o2;
    if (a.out_n) a.out_n[qi] = num;
    if (a.out_maxd2) a.out_maxd2[qi] = (num > 0) ? (float)maxd2 : 0.0f;
  }
}

#ifndef WAVE_WPE
#define WAVE_WPE 6  // fused query-per-wave kernel: occupancy target (80 VGPRs)
#endif
// Leaf sweep height (SWEEP instances): a subtree of at most 2^SWEEP_H leaves is not walked node
// by node; its leaf boxes are read at once, one per lane, and the leaves within the bound are
// scanned nearest first.
#ifndef SWEEP_H
#define SWEEP_H 6
#endif
// a sweep reads one leaf box per lane: at most 64 leaves (SWEEP_H 7 gave wrong sets, r05)
static_assert(SWEEP_H >= 0 && SWEEP_H <= 6, "leaf sweep: one leaf per lane of a 64-wide wave");
template <int CAP, int LB, bool PROF, bool FUSE, bool SWEEP, bool GEN = true>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(FUSE ? WAVE_WPE : 1)))
void knn_wave_kernel(KnnArgs a) {
  __shared__ uint64_t buf[CAP];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t stk[64];   // traversal stack: pending far children and their box distances
  __shared__ float sdist[64];
  const int lane = threadIdx.x;
  const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
  const int L = a.map.nleaves;
  const int64_t N = a.map.n;
  const int K = a.K;
  uint64_t st_q = 0, st_found = 0, st_vis = 0;
  // GI_KNN_DBG & 16: cycle counters ST_PHASE + 10.. (traversal, leaf scans, selects, select
  // calls, node visits, whole queries)
  const bool prof = PROF;  // a template argument: the counters cost registers
  uint64_t pc[6] = {0, 0, 0, 0, 0, 0}, pt = 0, pq = 0;
  for (int64_t qq = blockIdx.x; qq < a.nq; qq += gridDim.x) {
    int64_t qg = a.q0 + qq;
    int64_t qi = a.perm ? (int64_t)a.perm[qg] : qg;
    float4 qp = a.qpos[qi];
    if (__float_as_uint(qp.w) == QMETA_NONE) {  // empty deterministic slot
      if (FUSE) {
        if (lane == 0) {
          a.out[3 * qi] = a.out[3 * qi + 1] = a.out[3 * qi + 2] = 0.0;
          if (a.out_n) a.out_n[qi] = 0;
          if (a.out_maxd2) a.out_maxd2[qi] = 0.0f;
        }
      } else if (lane == 0 && a.list_n) {
        a.list_n[qi] = 0;
      }
      continue;
    }
    float qx = ffirst(qp.x), qy = ffirst(qp.y), qz = ffirst(qp.z);
    uint32_t count = 0;
    // keys accepted while key < thr; start: every d2 <= r2
    uint64_t thr = ((uint64_t)__float_as_uint(a.r2f) << 32) + 0x100000000ull;
    uint32_t visited = 0;
    bool tight = false;
    if (prof) { pt = clock64(); pq = pt; }
    if (SWEEP) {
      // Walk with leaf sweeps: nodes above sweep height are expanded near child first (both
      // children's boxes in one scalar load, the far one pushed with its box distance); a node
      // at sweep height has its <= 2^SWEEP_H leaf boxes read in one vector load (lane i: leaf
      // i), and the leaves within the bound are scanned nearest first. The first leaf scanned
      // (the nearest to q) also gives the start bound from the per-photon K-th distances (for
      // any photon p: d_K(q) <= |q - p| + d_K(p)), computed from the same loads.
      // The walk replaces the bottom SWEEP_H levels' dependent node loads (most of a query's
      // node visits) by one round trip per subtree. The result set is order independent.
      if (N > 0) {
        const int levels = a.map.levels;
        const KdNode *nodesv = reinterpret_cast<const KdNode *>(a.map.nodes);
        bool need_dk = (a.map.dk != nullptr) && K > 0;
        int sp = 0;
        int node = 0;
        {
          KdNode r = ld_node(a.map.nodes, 1);
          if (prof) pc[4]++;
          if (kd_box_d2(r.lo, r.hi, qx, qy, qz) <= __uint_as_float((uint32_t)((thr - 1ull) >> 32)))
            node = 1;
        }
        while (true) {
          float pr = __uint_as_float((uint32_t)((thr - 1ull) >> 32));
          if (!node) {
            while (sp > 0) {
              sp--;
              if (ffirst(sdist[sp]) <= pr) {
                node = (int)ufirst(stk[sp]);
                break;
              }
            }
            if (!node) break;
          }
          node = __builtin_amdgcn_readfirstlane(node);
          const int h = levels - (31 - __clz(node));
          if (h > SWEEP_H) {
            KdNode c0 = ld_node(a.map.nodes, 2 * node), c1 = ld_node(a.map.nodes, 2 * node + 1);
            if (prof) pc[4]++;
            float d0 = kd_box_d2(c0.lo, c0.hi, qx, qy, qz), d1 = kd_box_d2(c1.lo, c1.hi, qx, qy, qz);
            int nn = 2 * node, fn = nn + 1;
            if (d1 < d0) {
              float t = d0; d0 = d1; d1 = t;
              nn = fn; fn = 2 * node;
            }
            if (d1 <= pr) {
              stk[sp] = (uint32_t)fn;  // every lane stores the same value
              sdist[sp] = d1;
              sp++;
            }
            node = (d0 <= pr) ? nn : 0;
            continue;
          }
          // sweep: leaf boxes of the 2^h leaves under node, lane i holding leaf i
          const int nl = 1 << h;
          const int lf0 = node << h;  // node index of the first leaf
          float ldist = INFINITY;
          if (lane < nl) {
            KdNode b = nodesv[lf0 + lane];
            ldist = kd_box_d2(b.lo, b.hi, qx, qy, qz);
          }
          if (prof) pc[4]++;
          uint64_t lm = __ballot(ldist <= pr);
          while (lm) {
            pr = __uint_as_float((uint32_t)((thr - 1ull) >> 32));
            const uint32_t cb = ((lm >> lane) & 1ull) ? __float_as_uint(ldist) : 0xffffffffu;
            const uint32_t mn = wave_min_u32(cb);
            if (__uint_as_float(mn) > pr) break;  // the rest are farther than the bound
            const int li = __ffsll((long long)__ballot(cb == mn)) - 1;
            lm &= ~(1ull << li);
            const int leaf = lf0 + li - L;
            int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
            if (need_dk) {
              need_dk = false;
              double best = INFINITY;
              for (int64_t b = s0; b < s1; b += 64) {
                int64_t ii = b + lane;
                if (ii < s1) {
                  float4 p = pos[ii];
                  float dkp = a.map.dk[ii];
                  float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
                  float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
                  if (dkp < INFINITY) best = fmin(best, sqrt((double)d2 * (1.0 + 1e-5)) + (double)dkp);
                }
              }
#pragma unroll
              for (int o = 32; o > 0; o >>= 1) best = fmin(best, __shfl_xor(best, o, 64));
              if (best < INFINITY) {
                double U = best * (1.0 + 1e-6) + 1e-12;
                float U2 = __double2float_ru(U * U * (1.0 + 1e-5));
                if (U2 < a.r2f) thr = ((uint64_t)__float_as_uint(U2) << 32) + 0x100000000ull;
                tight = true;
              }
            }
            visited += (uint32_t)(s1 - s0);
            if (prof) { uint64_t n = clock64(); pc[0] += n - pt; pt = n; }
            for (int64_t base0 = s0; base0 < s1; base0 += 64 * LB) {
              float4 pf[LB];
#pragma unroll
              for (int u = 0; u < LB; u++) {
                int64_t ii = base0 + u * 64 + lane;
                pf[u] = pos[ii < s1 ? ii : s0];
              }
#pragma unroll
              for (int u = 0; u < LB; u++) {
              const int64_t base = base0 + u * 64;
              if (base >= s1) break;
              int64_t ii = base + lane;
              uint64_t key = ~0ull;
              if (ii < s1) {
                float4 p = pf[u];
                float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
                float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
                key = ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)(uint32_t)ii;
              }
              bool pass = key < thr;
              uint64_t m = __ballot(pass);
              uint32_t nnew = (uint32_t)__popcll(m);
              if (nnew == 0) continue;
              if (count + nnew > (uint32_t)CAP) {
                if (prof) { uint64_t n = clock64(); pc[1] += n - pt; pt = n; pc[3]++; }
                select_k<CAP>(buf, hist, lane, count, K, thr);
                if (prof) { uint64_t n = clock64(); pc[2] += n - pt; pt = n; }
                pass = key < thr;
                m = __ballot(pass);
                nnew = (uint32_t)__popcll(m);
                if (nnew == 0) continue;
              }
              if (pass) {
                uint32_t off = count + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                buf[off] = key;
              }
              count += nnew;
              __syncthreads();
              }
            }
            // first time K candidates are held: select now so the prune bound tightens from
            // r^2 to the K-th distance early (otherwise it stays r^2 until the buffer fills)
            if (prof) { uint64_t n = clock64(); pc[1] += n - pt; pt = n; }
            if (K > 0 && count >= (uint32_t)K + (tight ? (uint32_t)a.sel_slack : 0u)) {
              select_k<CAP>(buf, hist, lane, count, K, thr);
              tight = true;
              if (prof) { uint64_t n = clock64(); pc[2] += n - pt; pt = n; pc[3]++; }
            }
          }
          node = 0;
        }
      }
    } else {
    if (a.map.dk && N > 0 && K > 0) {
        // Start from a bound instead of r: for any photon p, d_K(q) <= |q - p| + d_K(p)
        // (triangle inequality; the map's per-photon dk holds d_K(p)). The photons of the leaf
        // containing q give a bound within a few percent of d_K(q), so the walk prunes to the
        // K-neighbourhood from the first leaf on and the buffer rarely needs a select before
        // the final one.
        int node = 1;
        while (node < L) {
          KdNode nd = ld_node(a.map.nodes, node);
          float qa = kd_axis_q(__float_as_int(nd.hi.w), qx, qy, qz);
          node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
        }
        int leaf = node - L;
        int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
        double best = INFINITY;
        for (int64_t b = s0; b < s1; b += 64) {
          int64_t ii = b + lane;
          if (ii < s1) {
            float4 p = pos[ii];
            float dkp = a.map.dk[ii];
            float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
            float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
            // fp32 metric -> true distance: 1e-5 relative margin
            if (dkp < INFINITY) best = fmin(best, sqrt((double)d2 * (1.0 + 1e-5)) + (double)dkp);
          }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) best = fmin(best, __shfl_xor(best, o, 64));
        if (best < INFINITY) {
          double U = best * (1.0 + 1e-6) + 1e-12;
          float U2 = __double2float_ru(U * U * (1.0 + 1e-5));
          if (U2 < a.r2f) thr = ((uint64_t)__float_as_uint(U2) << 32) + 0x100000000ull;
          tight = true;
        }
      }
      // Traversal with a per-wave LDS stack: expanding a node loads both children's tight boxes
      // (adjacent 32-B records, one scalar load) and pushes the far child with its box distance,
      // so backtracking re-reads nothing from memory (the stackless walk re-read one parent per
      // level climbed, each a dependent round trip). Near child = the smaller box distance; the
      // visiting order does not change the result set.
      if (N > 0) {
        int sp = 0;
        int node = 0;
        {
          KdNode r = ld_node(a.map.nodes, 1);
          if (prof) pc[4]++;
          if (kd_box_d2(r.lo, r.hi, qx, qy, qz) <= __uint_as_float((uint32_t)((thr - 1ull) >> 32)))
            node = 1;
        }
        while (node) {
          node = __builtin_amdgcn_readfirstlane(node);  // wave-uniform: scalar node loads
          if (node < L) {
            KdNode c0 = ld_node(a.map.nodes, 2 * node), c1 = ld_node(a.map.nodes, 2 * node + 1);
            if (prof) pc[4]++;
            float pr = __uint_as_float((uint32_t)((thr - 1ull) >> 32));
            float d0 = kd_box_d2(c0.lo, c0.hi, qx, qy, qz), d1 = kd_box_d2(c1.lo, c1.hi, qx, qy, qz);
            int nn = 2 * node, fn = nn + 1;
            if (d1 < d0) {
              float t = d0; d0 = d1; d1 = t;
              nn = fn; fn = 2 * node;
            }
            if (d1 <= pr) {
              stk[sp] = (uint32_t)fn;  // every lane stores the same value: no cross-lane LDS hazard
              sdist[sp] = d1;
              sp++;
            }
            if (d0 <= pr) {
              node = nn;
              continue;
            }
          } else {
            int leaf = node - L;
            int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
            visited += (uint32_t)(s1 - s0);
            if (prof) { uint64_t n = clock64(); pc[0] += n - pt; pt = n; }
            // the leaf's photons, LB batches of 64 loaded before any is used: one memory round
            // trip per leaf instead of one per batch (a wave's traversal is a dependent chain,
            // and ~7 waves per SIMD cannot hide a round trip per 64 photons)
            for (int64_t base0 = s0; base0 < s1; base0 += 64 * LB) {
              float4 pf[LB];
#pragma unroll
              for (int u = 0; u < LB; u++) {
                int64_t ii = base0 + u * 64 + lane;
                pf[u] = pos[ii < s1 ? ii : s0];
              }
#pragma unroll
              for (int u = 0; u < LB; u++) {
              const int64_t base = base0 + u * 64;
              if (base >= s1) break;
              int64_t ii = base + lane;
              uint64_t key = ~0ull;
              if (ii < s1) {
                float4 p = pf[u];
                float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
                float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
                key = ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)(uint32_t)ii;
              }
              bool pass = key < thr;
              uint64_t m = __ballot(pass);
              uint32_t nnew = (uint32_t)__popcll(m);
              if (nnew == 0) continue;
              if (count + nnew > (uint32_t)CAP) {
                if (prof) { uint64_t n = clock64(); pc[1] += n - pt; pt = n; pc[3]++; }
                select_k<CAP>(buf, hist, lane, count, K, thr);
                if (prof) { uint64_t n = clock64(); pc[2] += n - pt; pt = n; }
                pass = key < thr;
                m = __ballot(pass);
                nnew = (uint32_t)__popcll(m);
                if (nnew == 0) continue;
              }
              if (pass) {
                uint32_t off = count + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                buf[off] = key;
              }
              count += nnew;
              __syncthreads();
              }
            }
            // first time K candidates are held: select now so the prune bound tightens from
            // r^2 to the K-th distance early (otherwise it stays r^2 until the buffer fills)
            if (prof) { uint64_t n = clock64(); pc[1] += n - pt; pt = n; }
            if (K > 0 && count >= (uint32_t)K + (tight ? (uint32_t)a.sel_slack : 0u)) {
              select_k<CAP>(buf, hist, lane, count, K, thr);
              tight = true;
              if (prof) { uint64_t n = clock64(); pc[2] += n - pt; pt = n; pc[3]++; }
            }
          }
          // pop the nearest pending subtree still within the (possibly tightened) bound
          node = 0;
          float pr = __uint_as_float((uint32_t)((thr - 1ull) >> 32));
          while (sp > 0) {
            sp--;
            if (ffirst(sdist[sp]) <= pr) {  // uniform: keeps the walk in scalar registers
              node = (int)ufirst(stk[sp]);
              break;
            }
          }
        }
      }
    }
    // exact K best
    if (prof) { uint64_t n = clock64(); pc[0] += n - pt; pt = n; }
    if (count > (uint32_t)K) {
      select_k<CAP>(buf, hist, lane, count, K, thr);
      if (prof) { uint64_t n = clock64(); pc[2] += n - pt; pt = n; pc[3]++; }
    }
    int num = (int)count;
    st_q += 1;
    st_found += (uint64_t)num;
    st_vis += visited;
    if (a.mode == KNN_MODE_DK) {
      // true-distance upper bound of the K-th neighbour: K-th fp32 metric, 1e-5 margin, round up
      float km = 0.0f;
      for (int s = lane; s < num; s += 64) km = fmaxf(km, __uint_as_float((uint32_t)(buf[s] >> 32)));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) km = fmaxf(km, __shfl_xor(km, o, 64));
      if (lane == 0)
        a.out_dk[qi] = (num < K) ? INFINITY : __double2float_ru(sqrt((double)km * (1.0 + 1e-5)));
    } else if (FUSE) {
      // the estimate straight from the K best keys in LDS (no list round trip through HBM)
      wave_estimate<GEN>(a, qi, qp, num, [&](int s) { return (uint32_t)buf[s]; },
                    [&](int s) { return __uint_as_float((uint32_t)(buf[s] >> 32)); });
    } else {
      for (int s = lane; s < K; s += 64) {
        bool v = s < num;
        a.list_idx[qi * K + s] = v ? (int32_t)(uint32_t)buf[s] : -1;
        a.list_d2[qi * K + s] = v ? __uint_as_float((uint32_t)(buf[s] >> 32)) : -1.0f;
      }
      if (lane == 0) a.list_n[qi] = num;
    }
    __syncthreads();
    if (prof) pc[5] += clock64() - pq;
  }
  if (prof && a.stats)
    for (int i = 0; i < 6; i++) wave_add(&a.stats[ST_PHASE + 10 + i], pc[i]);
  if (a.stats && lane == 0) {
    unsigned long long *sd = stat_stripe(a.stats);
    if (st_q) atomicAdd(&sd[ST_KNN + a.stat_off], (unsigned long long)st_q);
    if (st_found) atomicAdd(&sd[ST_KNN_PHOTONS + a.stat_off], (unsigned long long)st_found);
    if (st_vis) atomicAdd(&sd[ST_KNN_VISITED + a.stat_off], (unsigned long long)st_vis);
  }
}

// the estimate over the K-best lists written by knn_wave_kernel in list mode (kept for
// the group kernel); split from the search so the search kernel keeps a
// small register footprint
__global__ __launch_bounds__(64) void knn_list_estimate_kernel(KnnArgs a) {
  const int K = a.K;
  for (int64_t qq = blockIdx.x; qq < a.nq; qq += gridDim.x) {
    int64_t qg = a.q0 + qq;
    int64_t qi = a.perm ? (int64_t)a.perm[qg] : qg;
    float4 qp = a.qpos[qi];
    wave_estimate(a, qi, qp, a.list_n[qi],
                  [&](int s) { return (uint32_t)a.list_idx[qi * K + s]; },
                  [&](int s) { return a.list_d2[qi * K + s]; });
  }
}

__device__ __forceinline__ void kheap_push(uint64_t *h, int size, uint64_t key) {
  int c = size;
  while (c > 0) {
    int p = (c - 1) >> 1;
    uint64_t pk = h[p * 64];
    if (pk >= key) break;
    h[c * 64] = pk;
    c = p;
  }
  h[c * 64] = key;
}

__device__ __forceinline__ void kheap_replace_top(uint64_t *h, int size, uint64_t key) {
  int c = 0;
  while (true) {
    int l = 2 * c + 1;
    if (l >= size) break;
    uint64_t lk = h[l * 64];
    if (l + 1 < size) {
      uint64_t rk = h[(l + 1) * 64];
      if (rk > lk) { l = l + 1; lk = rk; }
    }
    if (key >= lk) break;
    h[c * 64] = lk;
    c = l;
  }
  h[c * 64] = key;
}

// ---------------------------------------------------------------------------------------
// Per-lane k-NN (the default for K <= 64): one query per lane, exact K-best keys
// (d2 bits << 32 | kd-order index) in a 4-ary max-heap in LDS laid out [slot][lane].
// Measured: this kernel is bound by dependent LDS round trips in the heap updates, at the
// ~6 waves/CU that the heaps' LDS allows. So:
//   * the first K accepted keys are appended unordered and heapified once (Floyd), instead
//     of K sift-ups that each run at the SIMD-max depth;
//   * the heap is 4-ary: a replacement sifts ~3 levels for K = 50 (binary: ~6), and the 4
//     child loads of a level are in flight together;
//   * the walk is "while-while": lanes step through internal nodes until each holds a leaf,
//     then the wave runs the leaf loop together, CH photon loads in flight per lane.
// Result set: the K smallest (d2, index) keys with d2 <= r2 (R3Kdtree.cpp:688-784 semantics).
// ---------------------------------------------------------------------------------------
template <int CH, int ARY>
__global__ __launch_bounds__(64) void knn_lane_kernel(KnnArgs a) {
  extern __shared__ uint64_t lsm[];
  const int lane = threadIdx.x;
  const int K = a.K;
  uint64_t *h = lsm + lane;  // [K][64]
  const KdNode *nodes = reinterpret_cast<const KdNode *>(a.map.nodes);
  const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
  const int L = a.map.nleaves;
  const int64_t N = a.map.n;
  const int64_t q = (int64_t)blockIdx.x * 64 + lane;
  bool valid = q < a.nq;
  int64_t qi = 0;
  float4 qp = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
    int64_t qg = a.q0 + q;
    qi = a.perm ? (int64_t)a.perm[qg] : qg;
    qp = a.qpos[qi];
    valid = __float_as_uint(qp.w) != QMETA_NONE;  // empty deterministic slot
  }
  int size = 0;
  // accept key < lim; start: every d2 <= r2
  uint64_t lim = ((uint64_t)__float_as_uint(a.r2f) + 1ull) << 32;
  uint32_t visited = 0;
  int node = 1;
  bool live = valid && N > 0 && K > 0;
  // first leaf (usually q's own): its photons p also give d_K(q) <= |q - p| + d_K(p)
  // (KdView::dk, triangle inequality, as knn_wave_kernel's start), which caps lim from the
  // second leaf on, so the rest of the walk prunes to about the K-neighbourhood
  bool seed = a.map.dk != nullptr;
  float sb = INFINITY, sd2 = 0.0f, sdk = INFINITY;
  while (__ballot(live)) {
    // walk to the next leaf within the bound
    int leaf = -1;
    float pr = __uint_as_float((uint32_t)((lim - 1ull) >> 32));
    while (live) {
      KdNode nd = nodes[node];
      if (kd_box_d2(nd.lo, nd.hi, qp.x, qp.y, qp.z) <= pr) {
        if (node < L) {
          float qa = kd_axis_q(__float_as_int(nd.hi.w), qp.x, qp.y, qp.z);
          node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
          continue;
        }
        leaf = node - L;
        break;
      }
      live = kd_next(nodes, node, qp.x, qp.y, qp.z);
    }
    int64_t s0 = 0, s1 = 0;
    if (leaf >= 0) {
      s0 = ((int64_t)leaf * N) / L;
      s1 = ((int64_t)(leaf + 1) * N) / L;
      visited += (uint32_t)(s1 - s0);
    }
    // converged leaf loop: CH photon loads in flight per lane
    int steps = (int)((s1 - s0 + CH - 1) / CH);
    int msteps = steps;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) msteps = max(msteps, __shfl_xor(msteps, o, 64));
    for (int st = 0; st < msteps; st++) {
      if (st < steps) {
        int64_t ii = s0 + CH * (int64_t)st;
        float4 p[CH];
#pragma unroll
        for (int u = 0; u < CH; u++) p[u] = pos[(ii + u < s1) ? ii + u : s1 - 1];
        float dk[CH];
        if (seed) {
#pragma unroll
          for (int u = 0; u < CH; u++) dk[u] = a.map.dk[(ii + u < s1) ? ii + u : s1 - 1];
        }
#pragma unroll
        for (int u = 0; u < CH; u++) {
          float dx = qp.x - p[u].x, dy = qp.y - p[u].y, dz = qp.z - p[u].z;
          float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
          uint64_t key = ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)(uint32_t)(ii + u);
          if (ii + u < s1 && key < lim) heapn_accept<ARY>(h, size, K, key, lim);
          if (seed) {
            float v = sqrtf(d2) + dk[u];
            if (v < sb) { sb = v; sd2 = d2; sdk = dk[u]; }
          }
        }
      }
    }
    if (seed && leaf >= 0) {
      // the photon minimising |q - p| + d_K(p) is picked in f32; the bound is computed with
      // its rounding margins in f64 for that photon (any photon gives a valid bound)
      seed = false;
      if (sdk < INFINITY) {
        double U = (sqrt((double)sd2 * (1.0 + 1e-5)) + (double)sdk) * (1.0 + 1e-6) + 1e-12;
        uint64_t ul = ((uint64_t)__float_as_uint(__double2float_ru(U * U * (1.0 + 1e-5))) + 1ull) << 32;
        if (ul < lim) lim = ul;
      }
    }
    if (leaf >= 0) live = kd_next(nodes, node, qp.x, qp.y, qp.z);
  }
  int num = size;
  if (valid) {
    if (a.mode == KNN_MODE_LIST) {
      for (int s = 0; s < K; s++) {
        bool v = s < num;
        uint64_t key = v ? h[s * 64] : 0ull;
        a.out_idx[qi * K + s] = v ? (int32_t)(uint32_t)key : -1;
        a.out_d2[qi * K + s] = v ? __uint_as_float((uint32_t)(key >> 32)) : -1.0f;
      }
      a.out_n[qi] = num;
    } else {
      double o0 = 0, o1 = 0, o2 = 0;
      double maxd2 = kEps;
      if (num > 0) {
        // max-heap root = K-th distance (photon_utils.cpp:108-111); r_max^2 if fewer (Q4)
        maxd2 = (num < K) ? a.rmax * a.rmax : (double)__uint_as_float((uint32_t)(h[0] >> 32));
        if (num == K && maxd2 < kEps) maxd2 = kEps;
        if (a.mode == KNN_MODE_IRRADIANCE) {
          // EstimateIrradiance, photon_utils.cpp:209-246
          for (int s = 0; s < num; s++) {
            uint32_t e = a.map.rgbe[(uint32_t)h[s * 64]];
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
          // EstimateRadiance, photon_utils.cpp:113-158
          const QShade &sh = a.qshade[qi];
          uint32_t meta = __float_as_uint(qp.w);
          uint32_t sign = meta & 3u;
          const DMaterial &m = a.mats[qmeta_mat(meta)];
          double N0 = sh.n[0], N1 = sh.n[1], N2 = sh.n[2];
          double E0 = sh.ex[0], E1 = sh.ex[1], E2 = sh.ex[2];
          bool spec = (m.flags & MF_SPECULAR) || (m.n < 0);
          // without the specular term, ap * kd + 0 * ks == ap * kd up to the sign of a zero (for
          // finite ks), and the sums start at +0, so dropping the 0 * ks products changes no result
          const bool diff_only = !spec && isfinite(m.ks[0]) && isfinite(m.ks[1]) && isfinite(m.ks[2]);
          double c1 = 1.0, c2 = 1.0, tw = 0;
          if (a.filter == 1) c1 = 1.0 / (a.fk * sqrt(maxd2));
          else if (a.filter == 2) {
            c1 = pow_call(2.7182818284590452354, -a.fb);
            c2 = 1.0 / (2.0 * maxd2);
          }
          if (a.filter == 0 && diff_only) {
            // common case (disk filter, no specular term): photons in groups of four, the heap
            // slot, direction-code, rgbe and LUT loads of a group in flight together; the sum
            // runs in slot order as in the general loop below
            for (int s0 = 0; s0 < num; s0 += 4) {
              uint32_t ids[4], ee[4];
              double lx[4], ly[4], lz[4];
#pragma unroll
              for (int u = 0; u < 4; u++) ids[u] = (uint32_t)h[(s0 + u < num ? s0 + u : s0) * 64];
              uint32_t dcs[4];
#pragma unroll
              for (int u = 0; u < 4; u++) {
                dcs[u] = __float_as_uint(a.map.pos4[4 * (int64_t)ids[u] + 3]) & 0xffffu;
                ee[u] = a.map.rgbe[ids[u]];
              }
#pragma unroll
              for (int u = 0; u < 4; u++) {
                lx[u] = a.lut[3 * dcs[u]];
                ly[u] = a.lut[3 * dcs[u] + 1];
                lz[u] = a.lut[3 * dcs[u] + 2];
              }
#pragma unroll
              for (int u = 0; u < 4; u++) {
                if (s0 + u >= num) break;
                double perp = N0 * lx[u] + N1 * ly[u] + N2 * lz[u];
                if ((sign == 2u && perp < 0) || (sign == 1u && perp > 0)) continue;
                uint32_t e = ee[u];
                uint32_t x = e >> 24;
                double inv = x ? ldexp(1.0, (int)x - 128 - 8) : 0.0;
                double p0 = x ? (double)(e & 255u) * inv : 0.0;
                double p1 = x ? (double)((e >> 8) & 255u) * inv : 0.0;
                double p2 = x ? (double)((e >> 16) & 255u) * inv : 0.0;
                double ap = fabs(perp);
                p0 *= ap * m.kd[0];
                p1 *= ap * m.kd[1];
                p2 *= ap * m.kd[2];
                o0 += p0; o1 += p1; o2 += p2;
              }
            }
          } else
          for (int s = 0; s < num; s++) {
            uint64_t key = h[s * 64];
            uint32_t id = (uint32_t)key;
            double d2 = (double)__uint_as_float((uint32_t)(key >> 32));
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
            if (diff_only) {
              p0 *= ap * m.kd[0];
              p1 *= ap * m.kd[1];
              p2 *= ap * m.kd[2];
            } else {
              double pw = spec ? pow_call(ca, m.n) : 0.0;
              p0 *= ap * m.kd[0] + pw * m.ks[0];
              p1 *= ap * m.kd[1] + pw * m.ks[1];
              p2 *= ap * m.kd[2] + pw * m.ks[2];
            }
            if (a.filter == 1) {
              double f = (1.0 - c1 * sqrt(d2));
              p0 *= f; p1 *= f; p2 *= f;
            } else if (a.filter == 2) {
              double w = (1.0 - (1.0 - pow_call(c1, c2 * d2)) / (1.0 - c1));
              p0 *= w; p1 *= w; p2 *= w;
              tw += w;
            }
            o0 += p0; o1 += p1; o2 += p2;
          }
          bool ok = true;
          if (a.filter == 0 && maxd2 > 0) {
            double den = kPi * maxd2;
            o0 /= den; o1 /= den; o2 /= den;
          } else if (a.filter == 1 && maxd2 > 0) {
            double den = (1.0 - 2.0 / 3.0 / a.fk) * kPi * maxd2;
            o0 /= den; o1 /= den; o2 /= den;
          } else if (a.filter == 2 && tw > 0 && maxd2 > 0) {
            double sc = a.fa * (num / tw) / (kPi * maxd2);
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
    wave_add(&a.stats[ST_KNN + a.stat_off], valid ? 1ull : 0ull);
    wave_add(&a.stats[ST_KNN_PHOTONS + a.stat_off], valid ? (uint64_t)num : 0ull);
    wave_add(&a.stats[ST_KNN_VISITED + a.stat_off], valid ? (uint64_t)visited : 0ull);
  }
}

// 8 photon loads in flight per lane and a 4-ary heap: the measured best
bool launch_knn_lane(const KnnArgs &a, hipStream_t st) {
  if (a.nq == 0) return true;
  size_t lds = (size_t)(a.K > 0 ? a.K : 1) * 64 * sizeof(uint64_t);
  if (lds > 64 * 1024) return false;
  unsigned grid = (unsigned)((a.nq + 63) / 64);
  knn_lane_kernel<8, 4><<<grid, 64, lds, st>>>(a);
  return true;
}

void launch_list_estimate(const KnnArgs &a, hipStream_t st) {
  if (a.nq == 0) return;
  int64_t grid = a.nq < (1 << 16) ? a.nq : (1 << 16);
  knn_list_estimate_kernel<<<(unsigned)grid, 64, 0, st>>>(a);
}

#ifndef WAVE_LB
#define WAVE_LB 1  // leaf batches of 64 photons loaded together by the 512/1024 instances
#endif
template <bool PROF, bool FUSE, bool SWEEP>
bool wave_launch(const KnnArgs &a, int need, unsigned grid, hipStream_t st) {
  if (!PROF && FUSE && SWEEP && !a.general) {  // without the estimate's general form
    if (need <= 128) knn_wave_kernel<128, 1, false, true, true, false><<<grid, 64, 0, st>>>(a);
    else if (need <= 256) knn_wave_kernel<256, 1, false, true, true, false><<<grid, 64, 0, st>>>(a);
    else if (need <= 512) knn_wave_kernel<512, WAVE_LB, false, true, true, false><<<grid, 64, 0, st>>>(a);
    else if (need <= 1024) knn_wave_kernel<1024, WAVE_LB, false, true, true, false><<<grid, 64, 0, st>>>(a);
    else return false;
    return true;
  }
  if (need <= 128) knn_wave_kernel<128, 1, PROF, FUSE, SWEEP><<<grid, 64, 0, st>>>(a);
  else if (need <= 256) knn_wave_kernel<256, 1, PROF, FUSE, SWEEP><<<grid, 64, 0, st>>>(a);
  else if (need <= 512) knn_wave_kernel<512, WAVE_LB, PROF, FUSE, SWEEP><<<grid, 64, 0, st>>>(a);
  else if (need <= 1024) knn_wave_kernel<1024, WAVE_LB, PROF, FUSE, SWEEP><<<grid, 64, 0, st>>>(a);
  else return false;
  return true;
}
template <bool PROF, bool FUSE>
bool wave_launch(const KnnArgs &a, int need, unsigned grid, hipStream_t st) {
  // GI_KNN_DBG & 1024: the node-by-node walk (A/B measurements)
  return (a.dbg & 1024) ? wave_launch<PROF, FUSE, false>(a, need, grid, st)
                        : wave_launch<PROF, FUSE, true>(a, need, grid, st);
}

bool launch_knn_wave(const KnnArgs &a, int cap_mul, hipStream_t st) {
  if (a.nq == 0) return true;
  int need = (a.K + 64) * cap_mul;
  int64_t grid = a.nq < (1 << 16) ? a.nq : (1 << 16);
  // GI_KNN_DBG & 16 selects the instance with phase cycle counters
  // the estimate fused into the search (list and dk modes write lists / bounds instead)
  const bool est = a.mode != KNN_MODE_LIST && a.mode != KNN_MODE_DK;
  bool ok;
  if (est) {
    ok = (a.dbg & 16) ? wave_launch<true, true>(a, need, (unsigned)grid, st)
                      : wave_launch<false, true>(a, need, (unsigned)grid, st);
  } else {
    ok = (a.dbg & 16) ? wave_launch<true, false>(a, need, (unsigned)grid, st)
                      : wave_launch<false, false>(a, need, (unsigned)grid, st);
  }
  if (!ok) return false;
  return true;
}

__global__ void photon_queries_kernel(const float4 *pos, int64_t n, float4 *q) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    float4 p = pos[i];
    q[i] = make_float4(p.x, p.y, p.z, 0.0f);
  }
}

void launch_photon_queries(const float *pos4, int64_t n, float4 *q, hipStream_t st) {
  if (n == 0) return;
  photon_queries_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
      reinterpret_cast<const float4 *>(pos4), n, q);
}

}  // namespace gi
