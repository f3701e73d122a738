// gi_knn_chunk.hip -- k-NN radiance estimate for chunks of 64 Morton-adjacent queries.
//
// Same result as R3Kdtree<Photon*>::FindClosestQuick (R3Kdtree.cpp:688-784) + EstimateRadiance
// (photon_utils.cpp:72-162) per query: the K smallest (d2, kd-order index) keys with d2 <= r2.
// The work is reorganised around the density of the queries. A frame issues ~150 M of them, and
// 64 consecutive sorted queries span far less than one K-neighbourhood. One wave per chunk:
//   1. bound: c = centre of the chunk's box B, rho = max |q - c|. Photons are on surfaces, so
//      the kd leaf reached from c holds >= K photons; the K-th smallest metric d2 among them
//      bounds d_K(c). Every query then has d_K(q) <= U = d_K(c) + rho (triangle inequality),
//      and every photon of its K-NN lies within U of B.
//   2. gather: one wave-uniform kd traversal (box-to-box pruning) copies every photon within U
//      of B into LDS (position, dir bits, rgbe, index), ballot-compacted.
//   3. per query: each lane computes the keys of its LDS candidates into registers. A wave
//      radix select (four 256-bin LDS histogram passes over the d2 bits, index bits only on
//      exact ties) finds the K-th key. The kept photons' estimate terms are reduced across the
//      wave in a fixed order.
// There is no per-query traversal and no per-query heap. The only global traffic per query is
// its record and the LUT rows of the photons it keeps. Chunks whose gather exceeds the LDS
// capacity (Morton jumps, sparse regions) go to a fallback list, and the per-lane kernel
// (gi_knn.hip) answers those queries.
#include <hip/hip_runtime.h>
#include "gi_device.h"
#include "gi_kernels.h"

namespace gi {

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wmaxf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wminf(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// ascending bitonic sort of one float per lane across the wave
__device__ __forceinline__ float wave_sort(float v, int lane) {
#pragma unroll
  for (int k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      float o = __shfl_xor(v, j, 64);
      bool up = (lane & k) == 0;
      bool lower = (lane & j) == 0;
      v = (lower == up) ? fminf(v, o) : fmaxf(v, o);
    }
  }
  return v;
}

// squared gap between a point/box and box B, same fp32 operation order as the photon metric
__device__ __forceinline__ float gap2(float lx, float ly, float lz, float hx, float hy, float hz,
                                      const float *bl, const float *bh) {
  float gx = fmaxf(fmaxf(lx - bh[0], bl[0] - hx), 0.0f);
  float gy = fmaxf(fmaxf(ly - bh[1], bl[1] - hy), 0.0f);
  float gz = fmaxf(fmaxf(lz - bh[2], bl[2] - hz), 0.0f);
  return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, __fmul_rn(gx, gx)));
}

// one radix digit over the register keys (PER per lane); returns the digit, updates need
template <int PER>
__device__ __forceinline__ uint32_t chunk_digit(uint32_t *hist, int lane, const uint64_t (&key)[PER],
                                                bool low, int shift, uint32_t prefix,
                                                uint32_t dprefix, uint32_t &need) {
  hist[4 * lane] = hist[4 * lane + 1] = hist[4 * lane + 2] = hist[4 * lane + 3] = 0u;
  __syncthreads();
  uint32_t hm = (shift == 24) ? 0u : (0xffffffffu << (shift + 8));
#pragma unroll
  for (int u = 0; u < PER; u++) {
    if (key[u] == ~0ull) continue;
    uint32_t hi = (uint32_t)(key[u] >> 32), lo = (uint32_t)key[u];
    uint32_t part = low ? lo : hi;
    bool m = ((part ^ prefix) & hm) == 0u;
    if (low) m = m && hi == dprefix;
    if (m) atomicAdd(&hist[(part >> shift) & 255u], 1u);
  }
  __syncthreads();
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
  uint32_t digit = (uint32_t)__shfl((int)d, L, 64);
  __syncthreads();
  return digit;
}

// Keep exactly the K smallest (d2, kd index) of the wave's register keys (key = d2 bits << 32 |
// LDS slot, ~0 = none; more than K valid). Value-range buckets: b(d2) = (d2 - min) *
// 255 / (max - min) is monotone in d2, so the K-th key lies in the first bucket whose
// cumulative count reaches K. That bucket usually holds 1-3 keys, and the exact (d2, index)
// order is resolved only there. LDS histogram atomics stay spread: a d2-bit radix would pile
// every key of a neighbourhood onto one exponent byte.
template <int PER>
__device__ __forceinline__ void wave_select_k(uint64_t (&key)[PER], int K, float mn, float mx,
                                              uint32_t *hist, const uint32_t *cidx, int lane) {
        // value-range buckets: b(d2) = (d2 - min) * 255/(max - min) is monotone in d2, so the
      // K-th key lies in the first bucket whose cumulative count reaches K
      mn = wminf(mn);
      mx = wmaxf(mx);
      float scale = (mx > mn) ? 255.0f / (mx - mn) : 0.0f;
      hist[4 * lane] = hist[4 * lane + 1] = hist[4 * lane + 2] = hist[4 * lane + 3] = 0u;
      __syncthreads();
      uint32_t bk[PER];
#pragma unroll
      for (int u = 0; u < PER; u++) {
        bk[u] = 256u;
        if (key[u] != ~0ull) {
          float d2 = __uint_as_float((uint32_t)(key[u] >> 32));
          bk[u] = min(255u, (uint32_t)((d2 - mn) * scale));
          atomicAdd(&hist[bk[u]], 1u);
        }
      }
      __syncthreads();
      uint32_t c0 = hist[4 * lane], c1 = hist[4 * lane + 1], c2 = hist[4 * lane + 2],
               c3 = hist[4 * lane + 3];
      uint32_t sum = c0 + c1 + c2 + c3, inc = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        uint32_t tt = (uint32_t)__shfl_up((int)inc, o, 64);
        if (lane >= o) inc += tt;
      }
      uint32_t exc = inc - sum, need = (uint32_t)K;
      uint64_t hit = __ballot(exc < need && need <= inc);
      int Lh = __ffsll((long long)hit) - 1;
      uint32_t d = 0, before = exc, cb = 0;
      if (lane == Lh) {
        if (need <= before + c0) { d = 0; cb = c0; }
        else if (need <= before + c0 + c1) { d = 1; before += c0; cb = c1; }
        else if (need <= before + c0 + c1 + c2) { d = 2; before += c0 + c1; cb = c2; }
        else { d = 3; before += c0 + c1 + c2; cb = c3; }
        d = 4 * (uint32_t)lane + d;
      }
      uint32_t B = (uint32_t)__shfl((int)d, Lh, 64);
      uint32_t m = need - (uint32_t)__shfl((int)before, Lh, 64);  // keys needed from bucket B
      cb = (uint32_t)__shfl((int)cb, Lh, 64);
      __syncthreads();
      // keep buckets < B, drop buckets > B; in B keep the m smallest (d2, kd index)
      uint32_t take = 0;  // bit u: key u of this lane is in B and kept
      if (m < cb) {
        uint32_t cand = 0;
#pragma unroll
        for (int u = 0; u < PER; u++) cand |= (bk[u] == B) ? (1u << u) : 0u;
        for (uint32_t it = 0; it < m; it++) {
          uint64_t best = ~0ull;
          int bu = -1;
#pragma unroll
          for (int u = 0; u < PER; u++) {
            if (!((cand >> u) & 1u)) continue;
            uint64_t rk = (key[u] & 0xffffffff00000000ull) | (uint64_t)cidx[(uint32_t)key[u]];
            if (rk < best) { best = rk; bu = u; }
          }
          uint64_t wbest = best;
#pragma unroll
          for (int o = 32; o > 0; o >>= 1) {
            uint64_t ob = (uint64_t)__shfl_xor((long long)wbest, o, 64);
            wbest = ob < wbest ? ob : wbest;
          }
          if (bu >= 0 && best == wbest) {
            take |= 1u << bu;
            cand &= ~(1u << bu);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < PER; u++) {
        if (key[u] == ~0ull) continue;
        bool keep = bk[u] < B || (bk[u] == B && (m >= cb || ((take >> u) & 1u)));
        if (!keep) key[u] = ~0ull;
      }
    }

template <int CAPC>
__global__ __launch_bounds__(64) void knn_chunk_kernel(KnnArgs a) {
  constexpr int PER = CAPC / 64;
  __shared__ float4 cpos[CAPC];
  __shared__ uint32_t cidx[CAPC];
  __shared__ uint32_t crgbe[CAPC];
  __shared__ uint32_t hist[256];
  __shared__ uint16_t sel[64 * 64];   // kept LDS slots per query of the chunk (K <= 64)
  __shared__ float smax[64];          // per query: K-th d2 (or -1 when fewer than K kept)
  __shared__ int snum[64];
  const int lane = threadIdx.x;
  const KdNode *nodes = reinterpret_cast<const KdNode *>(a.map.nodes);
  const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
  const int L = a.map.nleaves;
  const int64_t N = a.map.n;
  const int K = a.K;
  uint64_t st_q = 0, st_found = 0, st_vis = 0;
  for (int64_t chunk = blockIdx.x; chunk * 64 < a.nq; chunk += gridDim.x) {
    // ---- 1. the chunk's queries, their box and the K-th distance bound
    int64_t qs = chunk * 64 + lane;
    bool valid = qs < a.nq;
    int64_t qi = 0;
    float4 qp = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) {
      qi = a.perm ? (int64_t)a.perm[a.q0 + qs] : a.q0 + qs;
      qp = a.qpos[qi];
      valid = __float_as_uint(qp.w) != QMETA_NONE;
    }
    uint64_t vmask = __ballot(valid);
    if (vmask == 0) continue;
    float bl[3], bh[3];
    bl[0] = wminf(valid ? qp.x : INFINITY); bh[0] = wmaxf(valid ? qp.x : -INFINITY);
    bl[1] = wminf(valid ? qp.y : INFINITY); bh[1] = wmaxf(valid ? qp.y : -INFINITY);
    bl[2] = wminf(valid ? qp.z : INFINITY); bh[2] = wmaxf(valid ? qp.z : -INFINITY);
    float cx = 0.5f * (bl[0] + bh[0]), cy = 0.5f * (bl[1] + bh[1]), cz = 0.5f * (bl[2] + bh[2]);
    double rho = 0.0;
    if (valid) {
      double dx = (double)qp.x - cx, dy = (double)qp.y - cy, dz = (double)qp.z - cz;
      rho = sqrt(dx * dx + dy * dy + dz * dz);
    }
    rho = wmax(rho);
    // U: r_max, tightened by the K-th metric d2 from c among the photons of c's leaf
    double U = a.rmax;
    double dkc = -1.0;  // exact d_K(c) (true-distance upper bound), when found
    if (N > 0 && K > 0) {
      int node = 1;
      while (node < L) {
        KdNode nd = nodes[node];
        float qa = kd_axis_q(__float_as_int(nd.hi.w), cx, cy, cz);
        node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
      }
      int leaf = node - L;
      int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
      if (s1 - s0 >= K && K <= 64) {
        float d2 = INFINITY;
        if (s0 + lane < s1) {
          float4 p = pos[s0 + lane];
          float dx = cx - p.x, dy = cy - p.y, dz = cz - p.z;
          d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
        }
        float sorted = wave_sort(d2, lane);
        float dk2 = __shfl(sorted, K - 1, 64);  // >= d_K(c): K-th over a subset of photons
        // exact d_K(c): gather the photons within that radius of c and select the K-th
        float RA2 = __double2float_ru((double)dk2 * (1.0 + 1e-5));
        uint32_t na = 0;
        bool ovf = false;
        int nd = 1;
        while (true) {
          KdNode b = nodes[nd];
          if (kd_box_d2(b.lo, b.hi, cx, cy, cz) <= RA2) {
            if (nd < L) {
              float qa = kd_axis_q(__float_as_int(b.hi.w), cx, cy, cz);
              nd = 2 * nd + ((qa - b.lo.w >= 0.0f) ? 1 : 0);
              continue;
            }
            int lf = nd - L;
            int64_t a0 = ((int64_t)lf * N) / L, a1 = ((int64_t)(lf + 1) * N) / L;
            for (int64_t bb = a0; bb < a1; bb += 64) {
              int64_t ii = bb + lane;
              bool take = false;
              float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
              if (ii < a1) {
                p = pos[ii];
                float dx = cx - p.x, dy = cy - p.y, dz = cz - p.z;
                take = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx))) <= RA2;
              }
              uint64_t m = __ballot(take);
              uint32_t nn = (uint32_t)__popcll(m);
              if (na + nn > (uint32_t)CAPC) { ovf = true; break; }
              if (take) {
                uint32_t off = na + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                cpos[off] = p;
                cidx[off] = (uint32_t)ii;
              }
              na += nn;
            }
            if (ovf) break;
          }
          while (nd != 1) {
            const KdNode &pn = nodes[nd >> 1];
            float qa = kd_axis_q(__float_as_int(pn.hi.w), cx, cy, cz);
            if ((nd & 1) == ((qa - pn.lo.w >= 0.0f) ? 1 : 0)) break;
            nd >>= 1;
          }
          if (nd == 1) break;
          nd ^= 1;
        }
        __syncthreads();
        if (!ovf && na >= (uint32_t)K) {
          uint64_t kc[PER];
          float mn = INFINITY, mx = -INFINITY;
#pragma unroll
          for (int u = 0; u < PER; u++) {
            uint32_t s = (uint32_t)(u * 64 + lane);
            kc[u] = ~0ull;
            if (s < na) {
              float4 p = cpos[s];
              float dx = cx - p.x, dy = cy - p.y, dz = cz - p.z;
              float dd = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
              kc[u] = ((uint64_t)__float_as_uint(dd) << 32) | (uint64_t)s;
              mn = fminf(mn, dd);
              mx = fmaxf(mx, dd);
            }
          }
          if (na > (uint32_t)K) wave_select_k<PER>(kc, K, wminf(mn), wmaxf(mx), hist, cidx, lane);
          float km = 0.0f;
#pragma unroll
          for (int u = 0; u < PER; u++)
            if (kc[u] != ~0ull) km = fmaxf(km, __uint_as_float((uint32_t)(kc[u] >> 32)));
          dk2 = wmaxf(km);
        }
        __syncthreads();
        // metric -> true distance: 1e-5 relative margin covers the fp32 rounding
        dkc = sqrt((double)dk2 * (1.0 + 1e-5));
        double ub = dkc + rho * (1.0 + 1e-6) + 1e-12;
        if (ub < U) U = ub;
      }
    }
    float U2 = __double2float_ru(U * U * (1.0 + 1e-5));
    // ---- 2. gather every photon within U of the chunk's box into LDS
    uint32_t count = 0;
    bool overflow = false;
    if (N > 0 && K > 0) {
      int node = 1;
      while (true) {
        KdNode nd = nodes[node];
        if (gap2(nd.lo.x, nd.lo.y, nd.lo.z, nd.hi.x, nd.hi.y, nd.hi.z, bl, bh) <= U2) {
          if (node < L) {
            float qa = kd_axis_q(__float_as_int(nd.hi.w), cx, cy, cz);
            node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
            continue;
          }
          int leaf = node - L;
          int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
          for (int64_t b = s0; b < s1; b += 64) {
            int64_t ii = b + lane;
            bool take = false;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ii < s1) {
              p = pos[ii];
              take = gap2(p.x, p.y, p.z, p.x, p.y, p.z, bl, bh) <= U2;
            }
            uint64_t m = __ballot(take);
            uint32_t nn = (uint32_t)__popcll(m);
            if (count + nn > (uint32_t)CAPC) {
              overflow = true;
              break;
            }
            if (take) {
              uint32_t off = count + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
              cpos[off] = p;
              cidx[off] = (uint32_t)ii;
              crgbe[off] = a.map.rgbe[ii];
            }
            count += nn;
          }
          if (overflow) break;
        }
        // stackless backtrack (near side by c)
        while (node != 1) {
          const KdNode &pn = nodes[node >> 1];
          float qa = kd_axis_q(__float_as_int(pn.hi.w), cx, cy, cz);
          int near_is_right = (qa - pn.lo.w >= 0.0f) ? 1 : 0;
          if ((node & 1) == near_is_right) break;
          node >>= 1;
        }
        if (node == 1) break;
        node ^= 1;
      }
    }
    if (overflow) {
      // hand the chunk's queries to the per-lane fallback kernel
      uint32_t nv = (uint32_t)__popcll(vmask);
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(a.fb_count, nv);
      base = (uint32_t)__shfl((int)base, 0, 64);
      if (valid) a.fb_list[base + (uint32_t)__popcll(vmask & ((1ull << lane) - 1ull))] = (uint32_t)qi;
      __syncthreads();
      continue;
    }
    __syncthreads();
    // ---- 3. each query of the chunk against the LDS candidates
    for (int j = 0; j < 64 && !(a.dbg & 4); j++) {
      if (!((vmask >> j) & 1ull)) continue;
      float qx = __shfl(qp.x, j, 64), qy = __shfl(qp.y, j, 64), qz = __shfl(qp.z, j, 64);
      int64_t qj = (int64_t)__shfl((int)(qi & 0xffffffff), j, 64) |
                   ((int64_t)__shfl((int)(qi >> 32), j, 64) << 32);
      uint32_t meta = __float_as_uint(__shfl(qp.w, j, 64));
      // this query's own bound d_K(q) <= d_K(c) + |q - c| (tighter than the chunk's U)
      float lim2 = a.r2f;
      if (dkc >= 0.0) {
        double ex = (double)qx - cx, ey = (double)qy - cy, ez = (double)qz - cz;
        double uq = dkc + sqrt(ex * ex + ey * ey + ez * ez) * (1.0 + 1e-6) + 1e-12;
        float uq2 = __double2float_ru(uq * uq * (1.0 + 1e-5));
        if (uq2 < lim2) lim2 = uq2;
      }
      // key = d2 bits << 32 | LDS slot; ~0 = not a candidate (beyond the bound or past count)
      uint64_t key[PER];
      uint32_t nvalid = 0;
      float mn = INFINITY, mx = -INFINITY;
#pragma unroll
      for (int u = 0; u < PER; u++) {
        uint32_t s = (uint32_t)(u * 64 + lane);
        key[u] = ~0ull;
        if (s < count) {
          float4 p = cpos[s];
          float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
          float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
          if (d2 <= lim2) {
            key[u] = ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)s;
            mn = fminf(mn, d2);
            mx = fmaxf(mx, d2);
          }
        }
        nvalid += (uint32_t)__popcll(__ballot(key[u] != ~0ull));
      }
      if (nvalid > (uint32_t)K && !(a.dbg & 1)) wave_select_k<PER>(key, K, mn, mx, hist, cidx, lane);
      int num = (int)(nvalid > (uint32_t)K ? (uint32_t)K : nvalid);
      // record the kept slots of query j (order: slot-major, then lane) and its K-th d2
      float km = 0.0f;
      uint32_t base = 0;
#pragma unroll
      for (int u = 0; u < PER; u++) {
        bool kp = key[u] != ~0ull;
        uint64_t bm = __ballot(kp);
        if (kp) {
          sel[j * 64 + base + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull))] =
              (uint16_t)(uint32_t)key[u];
          km = fmaxf(km, __uint_as_float((uint32_t)(key[u] >> 32)));
        }
        base += (uint32_t)__popcll(bm);
      }
      km = wmaxf(km);
      if (lane == 0) {
        snum[j] = num;
        smax[j] = km;
        st_q += 1;
        st_found += (uint64_t)num;
        st_vis += count;
      }
    }
    __syncthreads();
    // ---- 4. estimates, one query per lane (photon data from LDS; latencies overlap across
    //         the 64 lanes). EstimateRadiance photon_utils.cpp:72-162 / Irradiance :209-246
    if (valid && !(a.dbg & 2)) {
      int num = snum[lane];
      double maxd2 = kEps;
      double o0 = 0, o1 = 0, o2 = 0, tw = 0;
      if (num > 0) {
        maxd2 = (num < K) ? a.rmax * a.rmax : (double)smax[lane];
        if (num == K && maxd2 < kEps) maxd2 = kEps;
        if (a.mode == KNN_MODE_IRRADIANCE) {
          for (int s = 0; s < num; s++) {
            uint32_t e = crgbe[sel[lane * 64 + s]];
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
          const DMaterial &mt = a.mats[meta >> 2];
          double N0 = sh.n[0], N1 = sh.n[1], N2 = sh.n[2];
          double E0 = sh.ex[0], E1 = sh.ex[1], E2 = sh.ex[2];
          bool spec = (mt.flags & MF_SPECULAR) || (mt.n < 0);
          double c1 = 1.0, c2 = 1.0;
          if (a.filter == 1) c1 = 1.0 / (a.fk * sqrt(maxd2));
          else if (a.filter == 2) {
            c1 = pow(2.7182818284590452354, -a.fb);
            c2 = 1.0 / (2.0 * maxd2);
          }
          for (int s = 0; s < num; s++) {
            uint32_t slot = sel[lane * 64 + s];
            float4 p = cpos[slot];
            float dx = qp.x - p.x, dy = qp.y - p.y, dz = qp.z - p.z;
            double d2 = (double)__builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
            uint32_t dcode = __float_as_uint(p.w) & 0xffffu;
            double ix = a.lut[3 * dcode], iy = a.lut[3 * dcode + 1], iz = a.lut[3 * dcode + 2];
            double perp = N0 * ix + N1 * iy + N2 * iz;
            if ((sign == 2u && perp < 0) || (sign == 1u && perp > 0)) continue;
            uint32_t e = crgbe[slot];
            uint32_t ee = e >> 24;
            double inv = ee ? ldexp(1.0, (int)ee - 128 - 8) : 0.0;
            double p0 = ee ? (double)(e & 255u) * inv : 0.0;
            double p1 = ee ? (double)((e >> 8) & 255u) * inv : 0.0;
            double p2 = ee ? (double)((e >> 16) & 255u) * inv : 0.0;
            double ca = E0 * -ix + E1 * -iy + E2 * -iz;
            if (ca < 0) ca = 0;
            double ap = fabs(perp);
            double pw = spec ? pow(ca, mt.n) : 0.0;
            p0 *= ap * mt.kd[0] + pw * mt.ks[0];
            p1 *= ap * mt.kd[1] + pw * mt.ks[1];
            p2 *= ap * mt.kd[2] + pw * mt.ks[2];
            if (a.filter == 1) {
              double f = (1.0 - c1 * sqrt(d2));
              p0 *= f; p1 *= f; p2 *= f;
            } else if (a.filter == 2) {
              double w = (1.0 - (1.0 - pow(c1, c2 * d2)) / (1.0 - c1));
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
            double scl = a.fa * (num / tw) / (kPi * maxd2);
            o0 *= scl; o1 *= scl; o2 *= scl;
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
    __syncthreads();
  }
  if (a.stats && lane == 0) {
    if (st_q) atomicAdd(&a.stats[ST_KNN + a.stat_off], (unsigned long long)st_q);
    if (st_found) atomicAdd(&a.stats[ST_KNN_PHOTONS + a.stat_off], (unsigned long long)st_found);
    if (st_vis) atomicAdd(&a.stats[ST_KNN_VISITED + a.stat_off], (unsigned long long)st_vis);
  }
}

// ascending bitonic sort of PER*64 u64 keys held as key[u] at index u*64 + lane
template <int PER>
__device__ __forceinline__ void wave_bitonic_sort(uint64_t (&k)[PER], int lane) {
  constexpr int N = PER * 64;
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int us = stride >> 6;
#pragma unroll
        for (int u = 0; u < PER; u++) {
          int pu = u ^ us;
          if (pu <= u) continue;
          bool asc = (((u * 64 + lane) & size) == 0);
          uint64_t x = k[u], y = k[pu];
          if ((x > y) == asc) { k[u] = y; k[pu] = x; }
        }
      } else {
#pragma unroll
        for (int u = 0; u < PER; u++) {
          bool asc = (((u * 64 + lane) & size) == 0);
          uint64_t o = (uint64_t)__shfl_xor((long long)k[u], stride, 64);
          bool lower = (lane & stride) == 0;
          k[u] = (lower == asc) ? (k[u] < o ? k[u] : o) : (k[u] > o ? k[u] : o);
        }
      }
    }
  }
}

template <int CAPC>
__global__ __launch_bounds__(64) void knn_chunk_heap_kernel(KnnArgs a) {
  constexpr int PER = CAPC / 64;
  __shared__ float4 cpos[CAPC];
  __shared__ uint32_t cidx[CAPC];
  __shared__ uint32_t crgbe[CAPC];
  __shared__ uint32_t hist[256];
  __shared__ uint16_t ord[CAPC];      // candidate slots sorted by distance to the chunk centre
  extern __shared__ uint64_t hsm[];   // per-lane 4-ary heaps [K][64]
  uint64_t *h = hsm + threadIdx.x;
  const int lane = threadIdx.x;
  const KdNode *nodes = reinterpret_cast<const KdNode *>(a.map.nodes);
  const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
  const int L = a.map.nleaves;
  const int64_t N = a.map.n;
  const int K = a.K;
  uint64_t st_q = 0, st_found = 0, st_vis = 0;
  for (int64_t chunk = blockIdx.x; chunk * 64 < a.nq; chunk += gridDim.x) {
    // ---- 1. the chunk's queries, their box and the K-th distance bound
    int64_t qs = chunk * 64 + lane;
    bool valid = qs < a.nq;
    int64_t qi = 0;
    float4 qp = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) {
      qi = a.perm ? (int64_t)a.perm[a.q0 + qs] : a.q0 + qs;
      qp = a.qpos[qi];
      valid = __float_as_uint(qp.w) != QMETA_NONE;
    }
    uint64_t vmask = __ballot(valid);
    if (vmask == 0) continue;
    float bl[3], bh[3];
    bl[0] = wminf(valid ? qp.x : INFINITY); bh[0] = wmaxf(valid ? qp.x : -INFINITY);
    bl[1] = wminf(valid ? qp.y : INFINITY); bh[1] = wmaxf(valid ? qp.y : -INFINITY);
    bl[2] = wminf(valid ? qp.z : INFINITY); bh[2] = wmaxf(valid ? qp.z : -INFINITY);
    float cx = 0.5f * (bl[0] + bh[0]), cy = 0.5f * (bl[1] + bh[1]), cz = 0.5f * (bl[2] + bh[2]);
    double rho = 0.0;
    if (valid) {
      double dx = (double)qp.x - cx, dy = (double)qp.y - cy, dz = (double)qp.z - cz;
      rho = sqrt(dx * dx + dy * dy + dz * dz);
    }
    rho = wmax(rho);
    // U: r_max, tightened by the K-th metric d2 from c among the photons of c's leaf
    double U = a.rmax;
    double dkc = -1.0;  // exact d_K(c) (true-distance upper bound), when found
    if (N > 0 && K > 0) {
      int node = 1;
      while (node < L) {
        KdNode nd = nodes[node];
        float qa = kd_axis_q(__float_as_int(nd.hi.w), cx, cy, cz);
        node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
      }
      int leaf = node - L;
      int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
      if (s1 - s0 >= K && K <= 64) {
        float d2 = INFINITY;
        if (s0 + lane < s1) {
          float4 p = pos[s0 + lane];
          float dx = cx - p.x, dy = cy - p.y, dz = cz - p.z;
          d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
        }
        float sorted = wave_sort(d2, lane);
        float dk2 = __shfl(sorted, K - 1, 64);  // >= d_K(c): K-th over a subset of photons
        // exact d_K(c): gather the photons within that radius of c and select the K-th
        float RA2 = __double2float_ru((double)dk2 * (1.0 + 1e-5));
        uint32_t na = 0;
        bool ovf = false;
        int nd = 1;
        while (true) {
          KdNode b = nodes[nd];
          if (kd_box_d2(b.lo, b.hi, cx, cy, cz) <= RA2) {
            if (nd < L) {
              float qa = kd_axis_q(__float_as_int(b.hi.w), cx, cy, cz);
              nd = 2 * nd + ((qa - b.lo.w >= 0.0f) ? 1 : 0);
              continue;
            }
            int lf = nd - L;
            int64_t a0 = ((int64_t)lf * N) / L, a1 = ((int64_t)(lf + 1) * N) / L;
            for (int64_t bb = a0; bb < a1; bb += 64) {
              int64_t ii = bb + lane;
              bool take = false;
              float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
              if (ii < a1) {
                p = pos[ii];
                float dx = cx - p.x, dy = cy - p.y, dz = cz - p.z;
                take = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx))) <= RA2;
              }
              uint64_t m = __ballot(take);
              uint32_t nn = (uint32_t)__popcll(m);
              if (na + nn > (uint32_t)CAPC) { ovf = true; break; }
              if (take) {
                uint32_t off = na + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
                cpos[off] = p;
                cidx[off] = (uint32_t)ii;
              }
              na += nn;
            }
            if (ovf) break;
          }
          while (nd != 1) {
            const KdNode &pn = nodes[nd >> 1];
            float qa = kd_axis_q(__float_as_int(pn.hi.w), cx, cy, cz);
            if ((nd & 1) == ((qa - pn.lo.w >= 0.0f) ? 1 : 0)) break;
            nd >>= 1;
          }
          if (nd == 1) break;
          nd ^= 1;
        }
        __syncthreads();
        if (!ovf && na >= (uint32_t)K) {
          uint64_t kc[PER];
          float mn = INFINITY, mx = -INFINITY;
#pragma unroll
          for (int u = 0; u < PER; u++) {
            uint32_t s = (uint32_t)(u * 64 + lane);
            kc[u] = ~0ull;
            if (s < na) {
              float4 p = cpos[s];
              float dx = cx - p.x, dy = cy - p.y, dz = cz - p.z;
              float dd = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
              kc[u] = ((uint64_t)__float_as_uint(dd) << 32) | (uint64_t)s;
              mn = fminf(mn, dd);
              mx = fmaxf(mx, dd);
            }
          }
          if (na > (uint32_t)K) wave_select_k<PER>(kc, K, wminf(mn), wmaxf(mx), hist, cidx, lane);
          float km = 0.0f;
#pragma unroll
          for (int u = 0; u < PER; u++)
            if (kc[u] != ~0ull) km = fmaxf(km, __uint_as_float((uint32_t)(kc[u] >> 32)));
          dk2 = wmaxf(km);
        }
        __syncthreads();
        // metric -> true distance: 1e-5 relative margin covers the fp32 rounding
        dkc = sqrt((double)dk2 * (1.0 + 1e-5));
        double ub = dkc + rho * (1.0 + 1e-6) + 1e-12;
        if (ub < U) U = ub;
      }
    }
    float U2 = __double2float_ru(U * U * (1.0 + 1e-5));
    // ---- 2. gather every photon within U of the chunk's box into LDS
    uint32_t count = 0;
    bool overflow = false;
    if (N > 0 && K > 0) {
      int node = 1;
      while (true) {
        KdNode nd = nodes[node];
        if (gap2(nd.lo.x, nd.lo.y, nd.lo.z, nd.hi.x, nd.hi.y, nd.hi.z, bl, bh) <= U2) {
          if (node < L) {
            float qa = kd_axis_q(__float_as_int(nd.hi.w), cx, cy, cz);
            node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
            continue;
          }
          int leaf = node - L;
          int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
          for (int64_t b = s0; b < s1; b += 64) {
            int64_t ii = b + lane;
            bool take = false;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
            if (ii < s1) {
              p = pos[ii];
              take = gap2(p.x, p.y, p.z, p.x, p.y, p.z, bl, bh) <= U2;
            }
            uint64_t m = __ballot(take);
            uint32_t nn = (uint32_t)__popcll(m);
            if (count + nn > (uint32_t)CAPC) {
              overflow = true;
              break;
            }
            if (take) {
              uint32_t off = count + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
              cpos[off] = p;
              cidx[off] = (uint32_t)ii;
              crgbe[off] = a.map.rgbe[ii];
            }
            count += nn;
          }
          if (overflow) break;
        }
        // stackless backtrack (near side by c)
        while (node != 1) {
          const KdNode &pn = nodes[node >> 1];
          float qa = kd_axis_q(__float_as_int(pn.hi.w), cx, cy, cz);
          int near_is_right = (qa - pn.lo.w >= 0.0f) ? 1 : 0;
          if ((node & 1) == near_is_right) break;
          node >>= 1;
        }
        if (node == 1) break;
        node ^= 1;
      }
    }
    if (overflow) {
      // hand the chunk's queries to the per-lane fallback kernel
      uint32_t nv = (uint32_t)__popcll(vmask);
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(a.fb_count, nv);
      base = (uint32_t)__shfl((int)base, 0, 64);
      if (valid) a.fb_list[base + (uint32_t)__popcll(vmask & ((1ull << lane) - 1ull))] = (uint32_t)qi;
      __syncthreads();
      continue;
    }
    __syncthreads();
    // ---- 3. sort the candidates by distance to c, then every lane scans them for its own
    //         query into its LDS heap: all lanes read the same candidate (LDS broadcast), and
    //         near-first order keeps replacements rare after the Floyd-built fill
    {
      uint64_t kc[PER];
#pragma unroll
      for (int u = 0; u < PER; u++) {
        uint32_t s = (uint32_t)(u * 64 + lane);
        kc[u] = ~0ull;
        if (s < count) {
          float4 p = cpos[s];
          float dx = cx - p.x, dy = cy - p.y, dz = cz - p.z;
          float dd = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
          kc[u] = ((uint64_t)__float_as_uint(dd) << 32) | (uint64_t)s;
        }
      }
      wave_bitonic_sort<PER>(kc, lane);
#pragma unroll
      for (int u = 0; u < PER; u++) {
        uint32_t i = (uint32_t)(u * 64 + lane);
        if (i < count) ord[i] = (uint16_t)(uint32_t)kc[u];
      }
    }
    __syncthreads();
    int size = 0;
    if (!(a.dbg & 4)) {
      float lim2 = a.r2f;
      if (valid && dkc >= 0.0) {
        double ex = (double)qp.x - cx, ey = (double)qp.y - cy, ez = (double)qp.z - cz;
        double uq = dkc + sqrt(ex * ex + ey * ey + ez * ez) * (1.0 + 1e-6) + 1e-12;
        float uq2 = __double2float_ru(uq * uq * (1.0 + 1e-5));
        if (uq2 < lim2) lim2 = uq2;
      }
      uint64_t lim = valid ? (((uint64_t)__float_as_uint(lim2) + 1ull) << 32) : 0ull;
      for (uint32_t i = 0; i < count; i++) {
        uint32_t slot = ord[i];
        float4 p = cpos[slot];
        float dx = qp.x - p.x, dy = qp.y - p.y, dz = qp.z - p.z;
        float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
        uint64_t key = ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)cidx[slot];
        if (key < lim) heapn_accept<4>(h, size, K, key, lim);
      }
    }
    // ---- 4. estimate from the lane's heap (EstimateRadiance photon_utils.cpp:72-162)
    if (valid && !(a.dbg & 2)) {
      int num = size;
      double maxd2 = kEps;
      double o0 = 0, o1 = 0, o2 = 0, tw = 0;
      if (num > 0) {
        maxd2 = (num < K) ? a.rmax * a.rmax : (double)__uint_as_float((uint32_t)(h[0] >> 32));
        if (num == K && maxd2 < kEps) maxd2 = kEps;
        if (a.mode == KNN_MODE_IRRADIANCE) {
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
          const QShade &sh = a.qshade[qi];
          uint32_t meta = __float_as_uint(qp.w);
          uint32_t sign = meta & 3u;
          const DMaterial &mt = a.mats[meta >> 2];
          double N0 = sh.n[0], N1 = sh.n[1], N2 = sh.n[2];
          double E0 = sh.ex[0], E1 = sh.ex[1], E2 = sh.ex[2];
          bool spec = (mt.flags & MF_SPECULAR) || (mt.n < 0);
          double c1 = 1.0, c2 = 1.0;
          if (a.filter == 1) c1 = 1.0 / (a.fk * sqrt(maxd2));
          else if (a.filter == 2) {
            c1 = pow(2.7182818284590452354, -a.fb);
            c2 = 1.0 / (2.0 * maxd2);
          }
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
            double pw = spec ? pow(ca, mt.n) : 0.0;
            p0 *= ap * mt.kd[0] + pw * mt.ks[0];
            p1 *= ap * mt.kd[1] + pw * mt.ks[1];
            p2 *= ap * mt.kd[2] + pw * mt.ks[2];
            if (a.filter == 1) {
              double f = (1.0 - c1 * sqrt(d2));
              p0 *= f; p1 *= f; p2 *= f;
            } else if (a.filter == 2) {
              double w = (1.0 - (1.0 - pow(c1, c2 * d2)) / (1.0 - c1));
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
            double scl = a.fa * (num / tw) / (kPi * maxd2);
            o0 *= scl; o1 *= scl; o2 *= scl;
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
    if (valid) {
      st_q += 1;
      st_found += (uint64_t)size;
      st_vis += count;
    }
    __syncthreads();
  }
  if (a.stats) {
    wave_add(&a.stats[ST_KNN + a.stat_off], st_q);
    wave_add(&a.stats[ST_KNN_PHOTONS + a.stat_off], st_found);
    wave_add(&a.stats[ST_KNN_VISITED + a.stat_off], st_vis);
  }
}

bool launch_knn_chunk(const KnnArgs &a, int cap, bool lane_heaps, hipStream_t st) {
  if (a.nq == 0) return true;
  if (a.mode == KNN_MODE_LIST || a.K > 64) return false;
  int64_t chunks = (a.nq + 63) / 64;
  unsigned grid = (unsigned)(chunks < (1 << 17) ? chunks : (1 << 17));
  if (lane_heaps) {
    size_t lds = (size_t)a.K * 64 * sizeof(uint64_t);
    if (cap <= 256) knn_chunk_heap_kernel<256><<<grid, 64, lds, st>>>(a);
    else knn_chunk_heap_kernel<512><<<grid, 64, lds, st>>>(a);
    return true;
  }
  if (cap <= 256) knn_chunk_kernel<256><<<grid, 64, 0, st>>>(a);
  else if (cap <= 512) knn_chunk_kernel<512><<<grid, 64, 0, st>>>(a);
  else knn_chunk_kernel<1024><<<grid, 64, 0, st>>>(a);
  return true;
}

}  // namespace gi
