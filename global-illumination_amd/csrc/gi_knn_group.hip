// gi_knn_group.hip -- k-nearest-photon search with G = 64/L queries per wave, L lanes each.
//
// The same result set as R3Kdtree<Photon*>::FindClosestQuick (R3Kdtree.cpp:688-784): the K
// smallest (d2, kd-order index) keys with d2 <= r2. The search is re-cut for CDNA4 between
// two measured extremes:
//   * one query per lane (knn_kernel): LDS max-heaps cap occupancy at ~6 waves/CU, and the
//     sift loops are dependent LDS chains that run divergently;
//   * one query per wave (knn_wave_kernel): no per-candidate chains, but a single traversal
//     per wave leaves the dependent node-load latency exposed.
// Here each group of L lanes walks the kd-tree for its own query. The walk is the stackless
// near-first descent with tight-box pruning, and it is group-uniform. The groups of a wave
// overlap their node-load latencies; the walk is "while-while", so leaves are processed
// together. A leaf's photons are spread over the group's lanes, and candidates below the
// group's threshold are appended to its LDS buffer with a group-masked ballot. When the
// buffer is full, a group radix select (4 byte-digit histogram passes over the d2 bits, plus
// the index bits on exact ties) keeps the K best and tightens the threshold. The K-best lists
// go to HBM; knn_list_estimate_kernel (gi_knn.hip) turns them into radiance estimates.
//
// Synchronisation: a workgroup is one wave and groups diverge, so there is no s_barrier.
// LDS hand-offs between lanes use a workgroup fence + wave barrier (lds_sync).
#include <hip/hip_runtime.h>
#include "gi_device.h"
#include "gi_kernels.h"

namespace gi {

__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int L>
__device__ __forceinline__ uint64_t group_bits(uint64_t m, int g) {
  if constexpr (L == 64) return m;
  else return (m >> (g * L)) & ((1ull << L) - 1ull);
}

// one radix digit for group g: histogram of ((key_part >> shift) & 255) over the keys whose
// higher digits match `prefix` (and whose d2 matches `dprefix` when resolving the index)
template <int L, int CAP, bool LOW>
__device__ __forceinline__ uint32_t group_digit(const uint64_t *buf, uint32_t *hist, int g, int r,
                                                uint32_t count, int shift, uint32_t prefix,
                                                uint32_t dprefix, uint32_t &need) {
  constexpr int B = 256 / L;  // bins per lane
#pragma unroll
  for (int b = 0; b < B; b++) hist[r * B + b] = 0u;
  lds_sync();
  uint32_t hm = (shift == 24) ? 0u : (0xffffffffu << (shift + 8));
  for (uint32_t s = (uint32_t)r; s < count; s += L) {
    uint64_t k = buf[s];
    uint32_t part = LOW ? (uint32_t)k : (uint32_t)(k >> 32);
    bool m = ((part ^ prefix) & hm) == 0u;
    if (LOW) m = m && (uint32_t)(k >> 32) == dprefix;
    if (m) atomicAdd(&hist[(part >> shift) & 255u], 1u);
  }
  lds_sync();
  uint32_t c[B];
  uint32_t sum = 0;
#pragma unroll
  for (int b = 0; b < B; b++) {
    c[b] = hist[r * B + b];
    sum += c[b];
  }
  uint32_t inc = sum;
#pragma unroll
  for (int o = 1; o < L; o <<= 1) {
    uint32_t t = (uint32_t)__shfl_up((int)inc, o, L);
    if (r >= o) inc += t;
  }
  uint32_t exc = inc - sum;
  uint64_t hit = group_bits<L>(__ballot(exc < need && need <= inc), g);
  int l0 = __ffsll((long long)hit) - 1;  // group-relative lane holding the digit
  uint32_t d = 0, before = exc;
  if (r == l0) {
    uint32_t run = exc;
#pragma unroll
    for (int b = 0; b < B; b++) {
      if (need > run && need <= run + c[b]) { d = (uint32_t)(r * B + b); before = run; }
      run += c[b];
    }
  }
  int src = g * L + l0;
  need -= (uint32_t)__shfl((int)before, src, 64);
  uint32_t digit = (uint32_t)__shfl((int)d, src, 64);
  lds_sync();
  return digit;
}

// keep exactly the K smallest keys of buf[0, count) in buf[0, K); thr = the K-th key
template <int L, int CAP>
__device__ __forceinline__ void group_select(uint64_t *buf, uint32_t *hist, int g, int r,
                                             uint32_t &count, int K, uint64_t &thr) {
  uint32_t need = (uint32_t)K, prefix = 0;
#pragma unroll 1
  for (int shift = 24; shift >= 0; shift -= 8)
    prefix |= group_digit<L, CAP, false>(buf, hist, g, r, count, shift, prefix, 0u, need) << shift;
  uint32_t eq = 0;
  for (uint32_t s0 = 0; s0 < count; s0 += L) {
    uint32_t s = s0 + (uint32_t)r;
    bool e = s < count && (uint32_t)(buf[s < count ? s : 0] >> 32) == prefix;
    eq += (uint32_t)__popcll(group_bits<L>(__ballot(e), g));
  }
  uint32_t tidx = 0xffffffffu;
  if (need < eq) {
    uint32_t lp = 0;
#pragma unroll 1
    for (int shift = 24; shift >= 0; shift -= 8)
      lp |= group_digit<L, CAP, true>(buf, hist, g, r, count, shift, lp, prefix, need) << shift;
    tidx = lp;
  }
  uint64_t T = ((uint64_t)prefix << 32) | (uint64_t)tidx;
  uint32_t base = 0;
  uint64_t below = (r == 0) ? 0ull : ((1ull << r) - 1ull);
  for (uint32_t s0 = 0; s0 < count; s0 += L) {
    uint32_t s = s0 + (uint32_t)r;
    uint64_t k = (s < count) ? buf[s] : ~0ull;
    bool keep = (s < count) && k <= T;
    uint64_t m = group_bits<L>(__ballot(keep), g);
    if (keep) buf[base + (uint32_t)__popcll(m & below)] = k;
    base += (uint32_t)__popcll(m);
  }
  lds_sync();
  count = base;  // == K
  thr = T;
}

template <int L, int CAP>
__global__ __launch_bounds__(64) void knn_group_kernel(KnnArgs a) {
  constexpr int G = 64 / L;
  __shared__ uint64_t sbuf[G][CAP];
  __shared__ uint32_t shist[G][256];
  const int lane = threadIdx.x;
  const int g = lane / L, r = lane % L;
  uint64_t *buf = sbuf[g];
  uint32_t *hist = shist[g];
  const uint64_t below = (r == 0) ? 0ull : ((1ull << r) - 1ull);
  const KdNode *nodes = reinterpret_cast<const KdNode *>(a.map.nodes);
  const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
  const int Lv = a.map.nleaves;
  const int64_t N = a.map.n;
  const int K = a.K;
  uint64_t st_q = 0, st_found = 0, st_vis = 0;
  for (int64_t base = (int64_t)blockIdx.x * G; base < a.nq; base += (int64_t)gridDim.x * G) {
    const int64_t qq = base + g;
    bool valid = qq < a.nq;
    int64_t qi = 0;
    float4 qp = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) {
      int64_t qg = a.q0 + qq;
      qi = a.perm ? (int64_t)a.perm[qg] : qg;
      qp = a.qpos[qi];
      if (__float_as_uint(qp.w) == QMETA_NONE) {  // empty deterministic slot
        if (r == 0) a.list_n[qi] = 0;
        valid = false;
      }
    }
    uint32_t count = 0, visited = 0;
    uint64_t thr = ((uint64_t)__float_as_uint(a.r2f) + 1ull) << 32;  // accept key < thr
    bool tight = false;
    int node = 1;
    bool live = valid && N > 0 && K > 0;
    while (__ballot(live)) {
      int leaf = -1;
      float pr = __uint_as_float((uint32_t)((thr - 1ull) >> 32));
      while (live) {
        KdNode nd = nodes[node];
        if (kd_box_d2(nd.lo, nd.hi, qp.x, qp.y, qp.z) <= pr) {
          if (node < Lv) {
            float qa = kd_axis_q(__float_as_int(nd.hi.w), qp.x, qp.y, qp.z);
            node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
            continue;
          }
          leaf = node - Lv;
          break;
        }
        live = kd_next(nodes, node, qp.x, qp.y, qp.z);
      }
      if (leaf >= 0) {
        int64_t s0 = ((int64_t)leaf * N) / Lv, s1 = ((int64_t)(leaf + 1) * N) / Lv;
        visited += (uint32_t)(s1 - s0);
        for (int64_t b = s0; b < s1; b += L) {
          int64_t ii = b + r;
          uint64_t key = ~0ull;
          if (ii < s1) {
            float4 p = pos[ii];
            float dx = qp.x - p.x, dy = qp.y - p.y, dz = qp.z - p.z;
            float d2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
            key = ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)(uint32_t)ii;
          }
          bool pass = key < thr;
          uint64_t m = group_bits<L>(__ballot(pass), g);
          uint32_t nnew = (uint32_t)__popcll(m);
          if (count + nnew > (uint32_t)CAP) {
            group_select<L, CAP>(buf, hist, g, r, count, K, thr);
            tight = true;
            pass = key < thr;
            m = group_bits<L>(__ballot(pass), g);
            nnew = (uint32_t)__popcll(m);
          }
          if (pass) buf[count + (uint32_t)__popcll(m & below)] = key;
          count += nnew;
        }
        lds_sync();
        // tighten the bound as soon as K candidates are held, then every `slack` more
        if (count >= (uint32_t)K + (tight ? (uint32_t)a.sel_slack : 0u)) {
          group_select<L, CAP>(buf, hist, g, r, count, K, thr);
          tight = true;
        }
        live = kd_next(nodes, node, qp.x, qp.y, qp.z);
      }
    }
    if (valid && count > (uint32_t)K) group_select<L, CAP>(buf, hist, g, r, count, K, thr);
    int num = valid ? (int)count : 0;
    if (valid) {
      for (int s = r; s < K; s += L) {
        bool v = s < num;
        uint64_t k = v ? buf[s] : 0ull;
        a.list_idx[qi * K + s] = v ? (int32_t)(uint32_t)k : -1;
        a.list_d2[qi * K + s] = v ? __uint_as_float((uint32_t)(k >> 32)) : -1.0f;
      }
      if (r == 0) a.list_n[qi] = num;
      if (r == 0) {
        st_q += 1;
        st_found += (uint64_t)num;
        st_vis += visited;
      }
    }
    lds_sync();
  }
  if (a.stats) {
    wave_add(&a.stats[ST_KNN + a.stat_off], st_q);
    wave_add(&a.stats[ST_KNN_PHOTONS + a.stat_off], st_found);
    wave_add(&a.stats[ST_KNN_VISITED + a.stat_off], st_vis);
  }
}

bool launch_knn_group(const KnnArgs &a, int lanes, hipStream_t st) {
  if (a.nq == 0) return true;
  int need = a.K + lanes;  // a full buffer must still take one more leaf slice
  int64_t waves = (a.nq + (64 / lanes) - 1) / (64 / lanes);
  unsigned grid = (unsigned)(waves < (1 << 16) ? waves : (1 << 16));
#define GI_GROUP_LAUNCH(LL, CC) knn_group_kernel<LL, CC><<<grid, 64, 0, st>>>(a)
  if (lanes == 8) {
    if (need <= 64) GI_GROUP_LAUNCH(8, 64);
    else if (need <= 128) GI_GROUP_LAUNCH(8, 128);
    else return false;
  } else if (lanes == 16) {
    if (need <= 128) GI_GROUP_LAUNCH(16, 128);
    else if (need <= 256) GI_GROUP_LAUNCH(16, 256);
    else if (need <= 512) GI_GROUP_LAUNCH(16, 512);
    else return false;
  } else if (lanes == 32) {
    if (need <= 128) GI_GROUP_LAUNCH(32, 128);
    else if (need <= 256) GI_GROUP_LAUNCH(32, 256);
    else if (need <= 512) GI_GROUP_LAUNCH(32, 512);
    else return false;
  } else {
    return false;
  }
#undef GI_GROUP_LAUNCH
  if (a.mode != KNN_MODE_LIST) launch_list_estimate(a, st);
  return true;
}

}  // namespace gi
