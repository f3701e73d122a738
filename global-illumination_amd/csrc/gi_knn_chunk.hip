// gi_knn_chunk.hip -- k-NN radiance estimate for chunks of 64 Morton-adjacent queries.
//
// Same result as R3Kdtree<Photon*>::FindClosestQuick (R3Kdtree.cpp:688-784) + EstimateRadiance
// (photon_utils.cpp:72-162) per query: the K smallest (d2, kd-order index) keys with d2 <= r2.
// The work is reorganised around the density of the queries. A frame issues ~150 M of them, and
// 64 consecutive sorted queries span far less than one K-neighbourhood. One wave per chunk:
//   1. bound: c = centre of the chunk's box B, rho = max |q - c|. The exact d_K(c) is found from
//      the photons near c (c's leaf gives a first radius, a gather within it the exact K-th).
//      Every query then has d_K(q) <= d_K(c) + |q - c| <= U = d_K(c) + rho (triangle
//      inequality), and every photon of its K-NN lies within U of B.
//   2. gather: one wave-uniform kd traversal (box-to-box pruning) copies every photon within U
//      of B into LDS (position, dir bits, rgbe, index), ballot-compacted.
//   3. lane select (knn_chunk_lane_kernel): lane j owns query j. Counting passes over the LDS
//      candidates (every read is an LDS broadcast) narrow a d2 bracket with 16 value-range bins
//      each, until the K-th key's bracket holds few photons; a collect pass then keeps
//      everything below the bracket and sorts the bracket by (d2, index). All 64 queries
//      advance together.
//   4. estimate: each lane estimates its own query from the LDS-staged photons it kept.
// There is no per-query traversal and no per-query heap. The only global traffic per query is
// its record and the LUT rows of the photons it keeps. Chunks whose gather exceeds the LDS
// capacity (Morton jumps, sparse regions) go to a fallback list, and the per-lane kernel
// (gi_knn.hip) answers those queries.
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <type_traits>
#include "gi_device.h"
#include "gi_kernels.h"

namespace gi {

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

#ifndef CHUNK_EST_EB
#define CHUNK_EST_EB 4         // photons per LDS/LUT round trip in the chunk estimate
#endif
#ifndef EST_GROUPS
#define EST_GROUPS 3           // (normal, side) groups per chunk estimated from shared photon terms
#endif

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

// photon metric: the reference's squared distance in fp32, one fixed operation order
__device__ __forceinline__ float metric(float qx, float qy, float qz, const float4 &p) {
  float dx = qx - p.x, dy = qy - p.y, dz = qz - p.z;
  return __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, __fmul_rn(dx, dx)));
}

// The chunk's LDS candidates, structure of arrays: x[CAPC], y[CAPC], z[CAPC], w[CAPC] (w = the
// photon's dir | flags bits). The select loops read four consecutive candidates' x (y, z) with
// one broadcast ds_read_b128 (4 LDS cycles; a float4 per candidate would be a ds_read_b96 at 8
// cycles each, MI355X_MICROARCH.md LDS table).
template <int CAPC>
struct Cands {
  float *b;
  __device__ __forceinline__ float4 get(uint32_t s) const {
    return make_float4(b[s], b[CAPC + s], b[2 * CAPC + s], b[3 * CAPC + s]);
  }
  __device__ __forceinline__ void put(uint32_t s, const float4 &p) const {
    b[s] = p.x; b[CAPC + s] = p.y; b[2 * CAPC + s] = p.z; b[3 * CAPC + s] = p.w;
  }
  __device__ __forceinline__ float wbits(uint32_t s) const { return b[3 * CAPC + s]; }
  // candidates s0 .. s0 + 3 (s0 % 4 == 0) of coordinate c
  __device__ __forceinline__ float4 quad(int c, uint32_t s0) const {
    return *reinterpret_cast<const float4 *>(b + c * CAPC + s0);
  }
  __device__ __forceinline__ float d2(float qx, float qy, float qz, uint32_t s) const {
    return metric(qx, qy, qz, make_float4(b[s], b[CAPC + s], b[2 * CAPC + s], 0.0f));
  }
};

// d2 of the 8 candidates s0 .. s0 + 7 (s0 % 8 == 0, s0 + 8 <= CAPC): six broadcast reads
template <int CAPC>
__device__ __forceinline__ void cand_d2x8(const Cands<CAPC> &C, uint32_t s0, float qx, float qy,
                                          float qz, float (&d)[8]) {
  const float4 x0 = C.quad(0, s0), x1 = C.quad(0, s0 + 4);
  const float4 y0 = C.quad(1, s0), y1 = C.quad(1, s0 + 4);
  const float4 z0 = C.quad(2, s0), z1 = C.quad(2, s0 + 4);
  // metric() in packed pairs, each operation on all four pairs before the next one: no packed
  // result is read by the next instruction (the dependent v_pk_* pairs otherwise take s_nop)
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 qx2 = {qx, qx}, qy2 = {qy, qy}, qz2 = {qz, qz};
  const f2 X[4] = {{x0.x, x0.y}, {x0.z, x0.w}, {x1.x, x1.y}, {x1.z, x1.w}};
  const f2 Y[4] = {{y0.x, y0.y}, {y0.z, y0.w}, {y1.x, y1.y}, {y1.z, y1.w}};
  const f2 Z[4] = {{z0.x, z0.y}, {z0.z, z0.w}, {z1.x, z1.y}, {z1.z, z1.w}};
  f2 dx[4], dy[4], dz[4], r[4];
#pragma unroll
  for (int i = 0; i < 4; i++) dx[i] = qx2 - X[i];
#pragma unroll
  for (int i = 0; i < 4; i++) dy[i] = qy2 - Y[i];
#pragma unroll
  for (int i = 0; i < 4; i++) dz[i] = qz2 - Z[i];
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = dx[i] * dx[i];
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = __builtin_elementwise_fma(dy[i], dy[i], r[i]);
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = __builtin_elementwise_fma(dz[i], dz[i], r[i]);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    d[2 * i] = r[i].x;
    d[2 * i + 1] = r[i].y;
  }
}

// squared gap between a point/box and box B, same fp32 operation order as the photon metric
__device__ __forceinline__ float gap2(float lx, float ly, float lz, float hx, float hy, float hz,
                                      const float *bl, const float *bh) {
  float gx = fmaxf(fmaxf(lx - bh[0], bl[0] - hx), 0.0f);
  float gy = fmaxf(fmaxf(ly - bh[1], bl[1] - hy), 0.0f);
  float gz = fmaxf(fmaxf(lz - bh[2], bl[2] - hz), 0.0f);
  return __builtin_fmaf(gz, gz, __builtin_fmaf(gy, gy, __fmul_rn(gx, gx)));
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

// ---------------------------------------------------------------------------------------------
// phases 1-2, shared by the chunk kernels
// ---------------------------------------------------------------------------------------------
struct ChunkGeom {
  float bl[3], bh[3];  // the chunk's query box B
  float cx, cy, cz;    // its centre c
  double dkc;          // d_K(c) as a true-distance upper bound; -1 when not found
  bool dkc_exact;      // dkc is d_K(c) itself (within rounding), not a looser upper bound
  uint32_t count;      // candidates gathered into LDS
  bool overflow;       // more than `cap` candidates: the chunk goes to the fallback
};

// Diagnostic counters of GI_KNN_DBG & 16 (ST_PHASE + i, summed over waves):
//   0 bound cycles, 1 gather cycles, 2 select cycles, 3 estimate cycles, 4 bound+gather cycles
//   of overflowing chunks, 5 kd nodes read by the bound, 6 by the gather, 7 chunks,
//   8 counting passes (lane select), 9 queries handed to the fallback by the lane select
struct ChunkProf {
  bool on;
  uint64_t t;
  uint64_t c[10];
  __device__ __forceinline__ void lap(int i) {
    if (on) {
      uint64_t n = clock64();
      c[i] += n - t;
      t = n;
    }
  }
};

// Wave-uniform walk over every kd leaf whose node box passes boxd(node) <= bound, with a
// per-wave LDS stack (stk, >= tree depth entries): an expansion reads both children's boxes
// (scalar loads, ld_node) and pushes one, so backtracking reads nothing from memory. leaf(l)
// returns true to stop the walk. Returns the number of node records read.
//
// Two levels per round trip: an expansion whose children are internal also reads the four grandchildren (128
// contiguous bytes, issued with the children's 64): two levels per dependent round trip. A
// grandchild is taken when its parent and its own box pass, as two single-level expansions
// would take it, and the in-grandchildren are pushed right to left, so leaves are still visited
// left to right: the callers' LDS candidate order, and so every estimate sum, is unchanged.
// Stack: at most three entries per two levels.
//
// Leaf sweep: a node with at most 2^CHUNK_SWEEP_H leaves below it is not expanded further; its
// leaf boxes are read in one vector load (lane i: leaf i) and the passing leaves are visited in
// index order. A leaf's tight box lies inside every ancestor's and boxd is monotone under
// containment (the same fp operation sequence, every rounding monotone), so the leaves that
// pass are exactly those the node-by-node walk reaches, in the same left-to-right order: the
// candidate order, and every result, are unchanged; the bottom levels' dependent node loads
// become one round trip per subtree.
#ifndef CHUNK_SWEEP_H
#define CHUNK_SWEEP_H 6
#endif
static_assert(CHUNK_SWEEP_H >= 0 && CHUNK_SWEEP_H <= 6, "leaf sweep: one leaf per lane of a 64-wide wave");
template <typename BoxD, typename Leaf>
__device__ __forceinline__ uint32_t walk_within(const float *nodes, int L, float bound, uint32_t *stk,
                                                BoxD boxd, Leaf leaf, int root = 1) {
  const int levels = 31 - __clz(L);
  const int lane = threadIdx.x & 63;
  uint32_t reads = 1;
  int sp = 0;
  int node = (boxd(ld_node(nodes, root)) <= bound) ? root : 0;
  while (node) {
    node = __builtin_amdgcn_readfirstlane(node);
    const int h = levels - (31 - __clz(node));
    if (h <= CHUNK_SWEEP_H) {
      const int lf0 = node << h;
      bool in = false;
      if (lane < (1 << h)) in = boxd(reinterpret_cast<const KdNode *>(nodes)[lf0 + lane]) <= bound;
      reads += 1u << h;
      uint64_t m = __ballot(in);
      while (m) {
        const int li = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        if (leaf(lf0 + li - L)) return reads;
      }
    } else {
      const int c = 2 * node;
      KdNode c0 = ld_node(nodes, c), c1 = ld_node(nodes, c + 1);
      if (h > CHUNK_SWEEP_H + 1) {
        KdNode g0 = ld_node(nodes, 2 * c), g1 = ld_node(nodes, 2 * c + 1);
        KdNode g2 = ld_node(nodes, 2 * c + 2), g3 = ld_node(nodes, 2 * c + 3);
        reads += 6;
        const bool in0 = boxd(c0) <= bound, in1 = boxd(c1) <= bound;
        const bool i0 = in0 && boxd(g0) <= bound, i1 = in0 && boxd(g1) <= bound;
        const bool i2 = in1 && boxd(g2) <= bound, i3 = in1 && boxd(g3) <= bound;
        const int nxt = i0 ? 2 * c : (i1 ? 2 * c + 1 : (i2 ? 2 * c + 2 : (i3 ? 2 * c + 3 : 0)));
        // every lane stores the same values
        if (i3 && nxt != 2 * c + 3) stk[sp++] = (uint32_t)(2 * c + 3);
        if (i2 && nxt != 2 * c + 2) stk[sp++] = (uint32_t)(2 * c + 2);
        if (i1 && nxt != 2 * c + 1) stk[sp++] = (uint32_t)(2 * c + 1);
        if (nxt) { node = nxt; continue; }
      } else {
        reads += 2;
        bool in0 = boxd(c0) <= bound, in1 = boxd(c1) <= bound;
        if (in0 && in1) {
          stk[sp] = (uint32_t)(c + 1);  // every lane stores the same value
          sp++;
        }
        if (in0) { node = c; continue; }
        if (in1) { node = c + 1; continue; }
      }
    }
    node = 0;
    if (sp > 0) {
      sp--;
      node = (int)__builtin_amdgcn_readfirstlane((int)stk[sp]);
    }
  }
  return reads;
}

// the exact K-th distance from c (the chunk centre): every photon within RA2 (an upper bound of
// d_K(c)^2) gathered into the LDS candidate arrays, then a wave select; false (dk2 untouched)
// when they overflow the arrays or fewer than K lie within RA2
#ifndef DK_EXACT_MAXCAP
#define DK_EXACT_MAXCAP 1024  // the large-K instances that refine the centre bound (KnnArgs::dk_exact)
#endif
template <int CAPC>
__device__ __forceinline__ bool exact_dk2(const KnnArgs &a, int lane, float cx, float cy, float cz,
                                          float RA2, const Cands<CAPC> &cpos, uint32_t *cidx,
                                          uint32_t *hist, uint32_t *stk, ChunkProf &P,
                                          float &dk2) {
  constexpr int PER = (CAPC + 63) / 64;
  const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
  const int L = a.map.nleaves;
  const int64_t N = a.map.n;
  const int K = a.K;
  // exact d_K(c): gather the photons within that radius of c and select the K-th
  uint32_t na = 0;
  bool ovf = false;
  uint32_t rd = walk_within(a.map.nodes, L, RA2, stk,
      [&](const KdNode &b) { return kd_box_d2(b.lo, b.hi, cx, cy, cz); },
      [&](int lf) {
        int64_t a0 = ((int64_t)lf * N) / L, a1 = ((int64_t)(lf + 1) * N) / L;
        for (int64_t bb = a0; bb < a1; bb += 64) {
          int64_t ii = bb + lane;
          bool take = false;
          float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ii < a1) {
            p = pos[ii];
            take = metric(cx, cy, cz, p) <= RA2;
          }
          uint64_t m = __ballot(take);
          uint32_t nn = (uint32_t)__popcll(m);
          if (na + nn > (uint32_t)CAPC) { ovf = true; return true; }
          if (take) {
            uint32_t off = na + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
            cpos.put(off, p);
            cidx[off] = (uint32_t)ii;
          }
          na += nn;
        }
        return false;
      });
  if (P.on) P.c[5] += rd;
  __syncthreads();
  if (!ovf && na >= (uint32_t)K) {
    uint64_t kc[PER];
    float mn = INFINITY, mx = -INFINITY;
#pragma unroll
    for (int u = 0; u < PER; u++) {
      uint32_t s = (uint32_t)(u * 64 + lane);
      kc[u] = ~0ull;
      if (s < na) {
        float dd = cpos.d2(cx, cy, cz, s);
        kc[u] = ((uint64_t)__float_as_uint(dd) << 32) | (uint64_t)s;
        mn = fminf(mn, dd);
        mx = fmaxf(mx, dd);
      }
    }
    if (na > (uint32_t)K) wave_select_k<PER>(kc, K, mn, mx, hist, cidx, lane);
    float km = 0.0f;
#pragma unroll
    for (int u = 0; u < PER; u++)
      if (kc[u] != ~0ull) km = fmaxf(km, __uint_as_float((uint32_t)(kc[u] >> 32)));
    dk2 = wmaxf(km);
  }
  __syncthreads();
  return !ovf && na >= (uint32_t)K;
}

template <int CAPC>
__device__ __forceinline__ void chunk_bound_gather(const KnnArgs &a, int lane, bool valid, float4 qp,
                                                   uint32_t cap, const Cands<CAPC> &cpos, uint32_t *cidx,
                                                   uint32_t *crgbe, uint32_t *hist, uint32_t *stk,
                                                   ChunkGeom &G, ChunkProf &P) {
  constexpr int PER = (CAPC + 63) / 64;
  const float4 *pos = reinterpret_cast<const float4 *>(a.map.pos4);
  const int L = a.map.nleaves;
  const int64_t N = a.map.n;
  const int K = a.K;
  float *bl = G.bl, *bh = G.bh;
  bl[0] = wminf(valid ? qp.x : INFINITY); bh[0] = wmaxf(valid ? qp.x : -INFINITY);
  bl[1] = wminf(valid ? qp.y : INFINITY); bh[1] = wmaxf(valid ? qp.y : -INFINITY);
  bl[2] = wminf(valid ? qp.z : INFINITY); bh[2] = wmaxf(valid ? qp.z : -INFINITY);
  const float cx = 0.5f * (bl[0] + bh[0]), cy = 0.5f * (bl[1] + bh[1]), cz = 0.5f * (bl[2] + bh[2]);
  G.cx = cx; G.cy = cy; G.cz = cz;
  double rho = 0.0;
  if (valid) {
    double dx = (double)qp.x - cx, dy = (double)qp.y - cy, dz = (double)qp.z - cz;
    rho = sqrt(dx * dx + dy * dy + dz * dz);
  }
  rho = wmax(rho);
  // ---- 1. U: r_max, tightened by the exact d_K(c)
  double U = a.rmax;
  G.dkc = -1.0;
  G.dkc_exact = false;
  // the descent's splits, lane k holding depth k's (for the gather's subtree root below)
  float path_split = 0.0f;
  int path_axis = 0, depth = 0, cleaf = 1;
  if (N > 0 && K > 0) {
    int node = 1;
    while (node < L) {
      // the node's children are read with it: two levels per round trip
      KdNode nd = ld_node(a.map.nodes, node), k0, k1;
      const bool two = 2 * node < L;
      if (two) { k0 = ld_node(a.map.nodes, 2 * node); k1 = ld_node(a.map.nodes, 2 * node + 1); }
      const int ax = __float_as_int(nd.hi.w);
      if (lane == depth) { path_split = nd.lo.w; path_axis = ax; }
      float qa = kd_axis_q(ax, cx, cy, cz);
      node = 2 * node + ((qa - nd.lo.w >= 0.0f) ? 1 : 0);
      depth++;
      if (P.on) P.c[5]++;
      if (two) {
        const KdNode &kn = (node & 1) ? k1 : k0;
        const int kax = __float_as_int(kn.hi.w);
        if (lane == depth) { path_split = kn.lo.w; path_axis = kax; }
        float ka = kd_axis_q(kax, cx, cy, cz);
        node = 2 * node + ((ka - kn.lo.w >= 0.0f) ? 1 : 0);
        depth++;
      }
    }
    cleaf = node;
    int leaf = node - L;
    int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
    if (a.map.dk) {
      // d_K(c) <= |c - p| + d_K(p) for every photon p of c's leaf (per-photon bounds, KdView::dk)
      double best = INFINITY;
      for (int64_t b = s0; b < s1; b += 64) {
        int64_t ii = b + lane;
        if (ii < s1) {
          float dkp = a.map.dk[ii];
          if (dkp < INFINITY)
            best = fmin(best, sqrt((double)metric(cx, cy, cz, pos[ii]) * (1.0 + 1e-5)) + (double)dkp);
        }
      }
      best = -wmax(-best);
      if (best < INFINITY) {
        G.dkc = best * (1.0 + 1e-6) + 1e-12;
        // large-K chunk kernel (KnnArgs::dk_exact): the bound refined to the exact d_K(c) from
        // the photons within it, so U = d_K(c) + rho as in the lane kernel (a tighter gather,
        // fewer overflowing chunks); the dk bound stays when they overflow the LDS arrays
        if (CAPC <= DK_EXACT_MAXCAP && a.dk_exact && K <= (int)CAPC) {
          float dk2 = 0.0f;
          const float RA2 = __double2float_ru(G.dkc * G.dkc * (1.0 + 1e-5));
          if (exact_dk2<CAPC>(a, lane, cx, cy, cz, RA2, cpos, cidx, hist, stk, P, dk2)) {
            G.dkc = sqrt((double)dk2 * (1.0 + 1e-5));
            G.dkc_exact = true;
          }
        }
        double ub = G.dkc + rho * (1.0 + 1e-6) + 1e-12;
        if (ub < U) U = ub;
      }
    } else if (s1 - s0 >= K && K <= 64) {
      float d2 = INFINITY;
      if (s0 + lane < s1) d2 = metric(cx, cy, cz, pos[s0 + lane]);
      float sorted = wave_sort(d2, lane);
      float dk2 = __shfl(sorted, K - 1, 64);  // >= d_K(c): K-th over a subset of photons
      // exact d_K(c): gather the photons within that radius of c and select the K-th
      float RA2 = __double2float_ru((double)dk2 * (1.0 + 1e-5));
      const bool ex = exact_dk2<CAPC>(a, lane, cx, cy, cz, RA2, cpos, cidx, hist, stk, P, dk2);
      // metric -> true distance: 1e-5 relative margin covers the fp32 rounding
      G.dkc = sqrt((double)dk2 * (1.0 + 1e-5));
      G.dkc_exact = ex;
      double ub = G.dkc + rho * (1.0 + 1e-6) + 1e-12;
      if (ub < U) U = ub;
    }
  }
  const float U2 = __double2float_ru(U * U * (1.0 + 1e-5));
  // Subtree root of the gather: the first node on c's descent whose split plane the region
  // {x : |x - B| <= U} touches. Above it the region lies strictly on the descent's side of every
  // split, so no photon of the region (a photon equal to a split may sit on either side, but
  // none lies in the region) is outside that subtree; the walk starts there instead of at the
  // root (saving two node reads per level above it). The test margin covers the fp32 metric.
  int groot = 1;
  if (N > 0 && K > 0 && depth <= 64) {
    const double Ut = U * (1.0 + 1e-4) + 1e-6;
    const float lo_ax = path_axis == 0 ? bl[0] : (path_axis == 1 ? bl[1] : bl[2]);
    const float hi_ax = path_axis == 0 ? bh[0] : (path_axis == 1 ? bh[1] : bh[2]);
    const bool touch = lane < depth && (double)lo_ax - Ut <= (double)path_split &&
                       (double)hi_ax + Ut >= (double)path_split;
    const uint64_t tm = __ballot(touch);
    const int kr = tm ? __ffsll((long long)tm) - 1 : depth;
    groot = cleaf >> (depth - kr);
    if (a.dbg & 512) groot = 1;
  }
  P.lap(0);
  // ---- 2. gather every photon within U of the chunk's box into LDS
  uint32_t count = 0;
  bool overflow = false;
  if (N > 0 && K > 0) {
    uint32_t rd = walk_within(a.map.nodes, L, U2, stk,
        [&](const KdNode &b) {
          return gap2(b.lo.x, b.lo.y, b.lo.z, b.hi.x, b.hi.y, b.hi.z, bl, bh);
        },
        [&](int leaf) {
          int64_t s0 = ((int64_t)leaf * N) / L, s1 = ((int64_t)(leaf + 1) * N) / L;
          for (int64_t b = s0; b < s1; b += 64) {
            int64_t ii = b + lane;
            bool take = false;
            float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
            uint32_t e = 0u;
            if (ii < s1) {
              p = pos[ii];
              e = a.map.rgbe[ii];  // issued with the position: no second round trip per leaf
              take = gap2(p.x, p.y, p.z, p.x, p.y, p.z, bl, bh) <= U2;
            }
            uint64_t m = __ballot(take);
            uint32_t nn = (uint32_t)__popcll(m);
            if (count + nn > cap) {
              overflow = true;
              return true;
            }
            if (take) {
              uint32_t off = count + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
              cpos.put(off, p);
              cidx[off] = (uint32_t)ii;
              crgbe[off] = e;
            }
            count += nn;
          }
          return false;
        }, groot);
    if (P.on) P.c[6] += rd;
  }
  // +inf positions after the last candidate, up to the next multiple of 8: the select loops
  // read whole groups of 8, and d2 = +inf is never below a bound or inside a bracket
  if (!overflow && lane < 8 && (count & 7u) != 0u && count + lane < ((count + 7u) & ~7u))
    cpos.put(count + lane, make_float4(INFINITY, INFINITY, INFINITY, 0.0f));
  G.count = count;
  G.overflow = overflow;
  if (P.on) {
    uint64_t n = clock64();
    P.c[overflow ? 4 : 1] += n - P.t;
    P.t = n;
    P.c[7]++;
  }
}

// this query's own bound d_K(q) <= d_K(c) + |q - c| (tighter than the chunk's U), as an fp32
// metric bound, capped by the accept radius
__device__ __forceinline__ float query_lim2(const KnnArgs &a, const ChunkGeom &G, float qx, float qy,
                                            float qz) {
  float lim2 = a.r2f;
  if (G.dkc >= 0.0) {
    double ex = (double)qx - G.cx, ey = (double)qy - G.cy, ez = (double)qz - G.cz;
    double uq = G.dkc + sqrt(ex * ex + ey * ey + ez * ez) * (1.0 + 1e-6) + 1e-12;
    float uq2 = __double2float_ru(uq * uq * (1.0 + 1e-5));
    if (uq2 < lim2) lim2 = uq2;
  }
  return lim2;
}

// hand the wave's valid queries to the per-lane fallback kernel
__device__ __forceinline__ void to_fallback(const KnnArgs &a, uint64_t vmask, bool valid, int64_t qi,
                                            int lane) {
  // one atomic per wave, on the block's stripe (a single counter would serialise the waves)
  uint32_t nv = (uint32_t)__popcll(vmask);
  const uint32_t s = blockIdx.x & (FB_QS - 1);
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(&a.fb_count[s * 32], nv);
  base = (uint32_t)__shfl((int)base, 0, 64);
  if (valid)
    a.fb_list[(size_t)s * a.fb_cap_s + base + (uint32_t)__popcll(vmask & ((1ull << lane) - 1ull))] =
        (uint32_t)qi;
}

// ---- 4. the estimate of one query from LDS-staged photons (slot_at(s) = s-th kept slot).
//         EstimateRadiance photon_utils.cpp:72-162 / irradiance :209-246
template <bool GEN, int CAPC, typename SlotAt>
__device__ __forceinline__ void chunk_estimate(const KnnArgs &a, int64_t qi, float4 qp, int num,
                                               float km, const Cands<CAPC> &cpos, const uint32_t *crgbe,
                                               SlotAt slot_at) {
  const int K = a.K;
  double maxd2 = kEps;
  double o0 = 0, o1 = 0, o2 = 0, tw = 0;
  if (num > 0) {
    maxd2 = (num < K) ? a.rmax * a.rmax : (double)km;
    if (num == K && maxd2 < kEps) maxd2 = kEps;
    if (a.mode == KNN_MODE_IRRADIANCE) {
      for (int s = 0; s < num; s++) {
        uint32_t e = crgbe[slot_at(s)];
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
      const DMaterial &mt = a.mats[qmeta_mat(meta)];
      double N0 = sh.n[0], N1 = sh.n[1], N2 = sh.n[2];
      bool spec = (mt.flags & MF_SPECULAR) || (mt.n < 0);
      // without the specular term, ap * kd + 0 * ks == ap * kd up to the sign of a zero (for
      // finite ks), and the sums start at +0, so dropping the 0 * ks products changes no result
      const bool diff_only = !spec && isfinite(mt.ks[0]) && isfinite(mt.ks[1]) && isfinite(mt.ks[2]);
      double c1 = 1.0, c2 = 1.0;
      if (a.filter == 1) c1 = 1.0 / (a.fk * sqrt(maxd2));
      else if (a.filter == 2) {
        c1 = pow_call(2.7182818284590452354, -a.fb);
        c2 = 1.0 / (2.0 * maxd2);
      }
      // photons in groups of EB: the LDS slot reads and direction-LUT loads of a group are
      // issued before its arithmetic (one memory round trip per group, not per photon); the
      // sums still run in photon order
      constexpr int EB = CHUNK_EST_EB;
      if (a.filter == 0 && diff_only) {
        // the common case (disk filter, no specular term): neither d2 nor the exact bounce is
        // needed, so only the direction code (w bits) and the rgbe word are read
        const double kd0 = mt.kd[0], kd1 = mt.kd[1], kd2 = mt.kd[2];
        for (int s0 = 0; s0 < num; s0 += EB) {
          uint32_t eg[EB];
          double lg[EB][3];
#pragma unroll
          for (int u = 0; u < EB; u++) {
            uint32_t slot = slot_at(s0 + u < num ? s0 + u : s0);
            eg[u] = crgbe[slot];
            uint32_t dc = __float_as_uint(cpos.wbits(slot)) & 0xffffu;
            lg[u][0] = a.lut[3 * dc];
            lg[u][1] = a.lut[3 * dc + 1];
            lg[u][2] = a.lut[3 * dc + 2];
          }
          // per photon (byte * 2^(e - 136)) * |perp|; kd multiplies the sums once per query
          // (re-associated like the sum order: relative 1e-16 per term). The same terms as
          // chunk_estimate_shared's, bit for bit.
#pragma unroll
          for (int u = 0; u < EB; u++) {
            if (s0 + u >= num) break;
            double ix = lg[u][0], iy = lg[u][1], iz = lg[u][2];
            double perp = N0 * ix + N1 * iy + N2 * iz;
            if ((sign == 2u && perp < 0) || (sign == 1u && perp > 0)) continue;
            uint32_t e = eg[u];
            uint32_t ee = e >> 24;
            double inv = ee ? ldexp(1.0, (int)ee - 128 - 8) : 0.0;
            double p0 = ee ? (double)(e & 255u) * inv : 0.0;
            double p1 = ee ? (double)((e >> 8) & 255u) * inv : 0.0;
            double p2 = ee ? (double)((e >> 16) & 255u) * inv : 0.0;
            double ap = fabs(perp);
            p0 *= ap; p1 *= ap; p2 *= ap;
            o0 += p0; o1 += p1; o2 += p2;
          }
        }
        o0 *= kd0; o1 *= kd1; o2 *= kd2;
      } else if constexpr (!GEN) {
        // an instance without the general form (KnnArgs::general == 0) met a query that needs
        // it: the host's check failed. Count it (the host re-runs the render with the general
        // instances, gi_host.cpp render_common) and make the result unmistakable meanwhile
        o0 = o1 = o2 = __builtin_nan("");
        if (a.stats) atomicAdd(a.stats + ST_GEN_MISS, 1ull);
      } else {
      // one photon per step here: this path calls pow (specular term, Gauss filter), and a
      // group of photons held across those calls would cost the whole kernel registers
      constexpr int EB1 = 1;
      const double E0 = sh.ex[0], E1 = sh.ex[1], E2 = sh.ex[2];
      for (int s0 = 0; s0 < num; s0 += EB1) {
      float4 pg[EB1];
      uint32_t eg[EB1];
      double lg[EB1][3];
#pragma unroll
      for (int u = 0; u < EB1; u++) {
        uint32_t slot = slot_at(s0 + u < num ? s0 + u : s0);
        pg[u] = cpos.get(slot);
        eg[u] = crgbe[slot];
        uint32_t dc = __float_as_uint(pg[u].w) & 0xffffu;
        lg[u][0] = a.lut[3 * dc];
        lg[u][1] = a.lut[3 * dc + 1];
        lg[u][2] = a.lut[3 * dc + 2];
      }
#pragma unroll
      for (int u = 0; u < EB1; u++) {
        if (s0 + u >= num) break;
        float4 p = pg[u];
        double d2 = (double)metric(qp.x, qp.y, qp.z, p);
        double ix = lg[u][0], iy = lg[u][1], iz = lg[u][2];
        double perp = N0 * ix + N1 * iy + N2 * iz;
        if ((sign == 2u && perp < 0) || (sign == 1u && perp > 0)) continue;
        uint32_t e = eg[u];
        uint32_t ee = e >> 24;
        double inv = ee ? ldexp(1.0, (int)ee - 128 - 8) : 0.0;
        double p0 = ee ? (double)(e & 255u) * inv : 0.0;
        double p1 = ee ? (double)((e >> 8) & 255u) * inv : 0.0;
        double p2 = ee ? (double)((e >> 16) & 255u) * inv : 0.0;
        double ca = E0 * -ix + E1 * -iy + E2 * -iz;
        if (ca < 0) ca = 0;
        double ap = fabs(perp);
        if (diff_only) {
          p0 *= ap * mt.kd[0];
          p1 *= ap * mt.kd[1];
          p2 *= ap * mt.kd[2];
        } else {
          double pw = spec ? pow_call(ca, mt.n) : 0.0;
          p0 *= ap * mt.kd[0] + pw * mt.ks[0];
          p1 *= ap * mt.kd[1] + pw * mt.ks[1];
          p2 *= ap * mt.kd[2] + pw * mt.ks[2];
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
      }
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

// ---- 4b. the estimate of the chunk's queries that share a surface normal and side, on the
//          common path (disk filter, materials without a specular term). For such queries a
//          photon's term (byte * 2^(e - 136)) * |N . I| does not depend on the query, so it is
//          computed once per candidate (lanes over candidates, 4 per lane) into LDS over the
//          candidate arrays (tp, [3][CAPC] doubles: the arrays are no longer needed), and each
//          query sums its kept slots: 3 LDS reads and 3 adds per photon instead of ~45
//          instructions. Up to EST_GROUPS groups (a chunk on one wall: one); the other queries
//          estimate per lane first (they still read the candidate arrays). Bit-identical to
//          chunk_estimate's per-lane sums (same terms, same slot order); GI_KNN_DBG & 256 turns
//          the sharing off.
template <int CAPC, typename SlotAt, typename PerLane>
__device__ __forceinline__ void chunk_estimate_shared(const KnnArgs &a, int lane, bool col, int64_t qi,
                                                      float4 qp, int num, float km, uint32_t count,
                                                      const Cands<CAPC> &cpos, const uint32_t *crgbe,
                                                      double *tp, SlotAt slot_at, PerLane per_lane) {
  bool shp = false;
  double N0 = 0.0, N1 = 0.0, N2 = 0.0;
  uint32_t sign = 0u;
  const DMaterial *mt = nullptr;
  if (col && num > 0 && a.mode == KNN_MODE_RADIANCE && a.filter == 0 && !(a.dbg & 256)) {
    const uint32_t meta = __float_as_uint(qp.w);
    mt = &a.mats[qmeta_mat(meta)];
    const bool spec = (mt->flags & MF_SPECULAR) || (mt->n < 0);
    shp = !spec && isfinite(mt->ks[0]) && isfinite(mt->ks[1]) && isfinite(mt->ks[2]);
    if (shp) {
      const QShade &sh = a.qshade[qi];
      N0 = sh.n[0]; N1 = sh.n[1]; N2 = sh.n[2];
      sign = meta & 3u;
    }
  }
  // groups: equal normal bits and side flags (a NaN normal never forms a group: bounded loop)
  uint64_t rem = __ballot(shp);
  int gi = -1, ng = 0;
  int lead[EST_GROUPS];
#pragma unroll
  for (int g = 0; g < EST_GROUPS; g++) {
    lead[g] = 0;
    if (!rem) continue;  // wave-uniform
    const int L0 = __ffsll((long long)rem) - 1;
    const long long l0 = __shfl(__double_as_longlong(N0), L0, 64);
    const long long l1 = __shfl(__double_as_longlong(N1), L0, 64);
    const long long l2 = __shfl(__double_as_longlong(N2), L0, 64);
    const uint32_t ls = (uint32_t)__shfl((int)sign, L0, 64);
    const bool in = ((rem >> lane) & 1ull) && __double_as_longlong(N0) == l0 &&
                    __double_as_longlong(N1) == l1 && __double_as_longlong(N2) == l2 && sign == ls;
    const uint64_t m = __ballot(in);
    if (in) gi = g;
    lead[g] = L0;
    rem &= ~m;
    rem &= ~(1ull << L0);
    ng = g + 1;
  }
  if (col && gi < 0) per_lane();
  if (ng == 0) return;
  constexpr int PC = (CAPC + 63) / 64;
  uint32_t cw[PC], ce[PC];
#pragma unroll
  for (int i = 0; i < PC; i++) {
    const uint32_t s = (uint32_t)(i * 64 + lane);
    cw[i] = s < count ? (__float_as_uint(cpos.wbits(s)) & 0xffffu) : 0u;
    ce[i] = s < count ? crgbe[s] : 0u;
  }
  double o0 = 0.0, o1 = 0.0, o2 = 0.0;
#pragma unroll
  for (int g = 0; g < EST_GROUPS; g++) {
    if (g >= ng) break;  // wave-uniform
    const int L0 = lead[g];
    const double g0 = __shfl(N0, L0, 64), g1 = __shfl(N1, L0, 64), g2 = __shfl(N2, L0, 64);
    const uint32_t gs = (uint32_t)__shfl((int)sign, L0, 64);
    __syncthreads();  // readers of the candidate arrays / of the previous group's terms are done
#pragma unroll
    for (int i = 0; i < PC; i++) {
      const uint32_t s = (uint32_t)(i * 64 + lane);
      if (s < count) {
        const double ix = a.lut[3 * cw[i]], iy = a.lut[3 * cw[i] + 1], iz = a.lut[3 * cw[i] + 2];
        const double perp = g0 * ix + g1 * iy + g2 * iz;
        double p0 = 0.0, p1 = 0.0, p2 = 0.0;
        const uint32_t e = ce[i], ee = e >> 24;
        if (!((gs == 2u && perp < 0) || (gs == 1u && perp > 0)) && ee) {
          const double inv = ldexp(1.0, (int)ee - 128 - 8), ap = fabs(perp);
          p0 = (double)(e & 255u) * inv;
          p1 = (double)((e >> 8) & 255u) * inv;
          p2 = (double)((e >> 16) & 255u) * inv;
          p0 *= ap; p1 *= ap; p2 *= ap;
        }
        tp[s] = p0;
        tp[CAPC + s] = p1;
        tp[2 * CAPC + s] = p2;
      }
    }
    __syncthreads();
    if (gi == g) {
      constexpr int EB = 4;  // slots, then their terms, four photons per LDS round trip
      for (int k0 = 0; k0 < num; k0 += EB) {
        uint32_t sl[EB];
#pragma unroll
        for (int u = 0; u < EB; u++) sl[u] = slot_at(k0 + u < num ? k0 + u : k0);
        double t[EB][3];
#pragma unroll
        for (int u = 0; u < EB; u++) {
          t[u][0] = tp[sl[u]];
          t[u][1] = tp[CAPC + sl[u]];
          t[u][2] = tp[2 * CAPC + sl[u]];
        }
#pragma unroll
        for (int u = 0; u < EB; u++) {
          if (k0 + u >= num) break;
          o0 += t[u][0]; o1 += t[u][1]; o2 += t[u][2];
        }
      }
    }
  }
  if (gi >= 0) {
    const int K = a.K;
    double maxd2 = (num < K) ? a.rmax * a.rmax : (double)km;
    if (num == K && maxd2 < kEps) maxd2 = kEps;
    o0 *= mt->kd[0]; o1 *= mt->kd[1]; o2 *= mt->kd[2];
    if (maxd2 > 0) {
      const double den = kPi * maxd2;
      o0 /= den; o1 /= den; o2 /= den;
      const QShade &sh = a.qshade[qi];
      o0 *= sh.w[0]; o1 *= sh.w[1]; o2 *= sh.w[2];
    } else {
      o0 = o1 = o2 = 0.0;
    }
    a.out[3 * qi] = o0;
    a.out[3 * qi + 1] = o1;
    a.out[3 * qi + 2] = o2;
    if (a.out_n) a.out_n[qi] = num;
    if (a.out_maxd2) a.out_maxd2[qi] = (float)maxd2;
  }
}

__device__ __forceinline__ void chunk_load_query(const KnnArgs &a, int64_t chunk, int lane, bool &valid,
                                                 int64_t &qi, float4 &qp) {
  int64_t qs = chunk * 64 + lane;
  valid = qs < a.nq;
  qi = 0;
  qp = make_float4(0.f, 0.f, 0.f, 0.f);
  if (valid) {
    qi = a.perm ? (int64_t)a.perm[a.q0 + qs] : a.q0 + qs;
    qp = a.qpos[qi];
    valid = __float_as_uint(qp.w) != QMETA_NONE;
  }
}

__device__ __forceinline__ void chunk_flush_stats(const KnnArgs &a, const ChunkProf &P, uint64_t q,
                                                  uint64_t found, uint64_t vis) {
  if (P.on && a.stats)
    for (int i = 0; i < 10; i++) wave_add(&a.stats[ST_PHASE + i], P.c[i]);
  if (a.stats) {
    wave_add(&a.stats[ST_KNN + a.stat_off], q);
    wave_add(&a.stats[ST_KNN_PHOTONS + a.stat_off], found);
    wave_add(&a.stats[ST_KNN_VISITED + a.stat_off], vis);
  }
}

// ---------------------------------------------------------------------------------------------
// lane select: one query per lane, counting passes over the LDS candidates
// ---------------------------------------------------------------------------------------------
#ifndef LS_BR_B
#define LS_BR_B 16             // bracket photons resolved by the collect pass (large-K kernel)
#endif
#ifndef LS_NBB
#define LS_NBB 32              // value-range bins per counting pass of the large-K kernel
#endif
#ifndef LS_BR_L
#define LS_BR_L 12             // the same for the lane-select kernel (bracket kept in its LDS slot list; measured best)
#endif
constexpr int LS_PASSES = 10;  // counting passes before a query goes to the fallback
#ifndef LS_NB
#define LS_NB 64               // value-range bins per counting pass of the lane-select kernel
#endif
#ifndef LS_UNROLL
#define LS_UNROLL 8            // candidates per loop trip in the counting / collect loops (fixed by cand_d2x8)
#endif

// value-range bin (of NB) of d2 in the bracket binning of [lo, hi]: sc = NB / (hi - lo), off =
// -lo * sc. fma + clamp + truncate: monotone non-decreasing in d2 (any monotone map works:
// bin_floor inverts this same function), 0 at lo and NB - 1 at hi. sc = 0 (an empty bracket)
// puts all in bin 0.
template <int NB>
__device__ __forceinline__ uint32_t binN(float d2, float sc, float off) {
  return (uint32_t)__builtin_amdgcn_fmed3f(__builtin_fmaf(d2, sc, off), 0.0f, (float)(NB - 1));
}
template <int NB>
__device__ __forceinline__ void bin_setup(float lo, float hi, float &sc, float &off) {
  sc = (hi > lo) ? (float)NB / (hi - lo) : 0.0f;
  off = -lo * sc;
}

// smallest float x in (lo, hi] with binN(x) >= b, for 1 <= b <= NB - 1, lo < hi,
// binN(hi) == NB - 1
template <int NB>
__device__ __forceinline__ float bin_floor(uint32_t b, float lo, float hi, float sc, float off) {
  uint32_t l = __float_as_uint(lo), h = __float_as_uint(hi);  // bin(l) < b <= bin(h)
  float g = lo + (float)b / sc;
  if (g > lo && g < hi) {
    uint32_t gb = __float_as_uint(g);
    uint32_t gl = (gb - l > 64u) ? gb - 64u : l;
    uint32_t gh = (h - gb > 64u) ? gb + 64u : h;
    if (binN<NB>(__uint_as_float(gl), sc, off) < b) l = gl;
    if (binN<NB>(__uint_as_float(gh), sc, off) >= b) h = gh;
  }
  while (h - l > 1u) {
    uint32_t m = l + ((h - l) >> 1);
    if (binN<NB>(__uint_as_float(m), sc, off) >= b) h = m;
    else l = m;
  }
  return __uint_as_float(h);
}

// d2 in [A, B] as one unsigned compare on the float bits (d2 >= 0): ab = bits(A), span =
// bits(B) - bits(A); a lane that counts nothing passes ab = ~0, span = 0 (only a NaN matches)
__device__ __forceinline__ bool in_bracket(float d2, uint32_t ab, uint32_t span) {
  return __float_as_uint(d2) - ab <= span;
}

__device__ __forceinline__ float next_up(float x) { return __uint_as_float(__float_as_uint(x) + 1u); }
__device__ __forceinline__ float next_down(float x) { return __uint_as_float(__float_as_uint(x) - 1u); }

// CAPC = 240 (first pass): 10,112 B of LDS per wave, so 16 waves (4 per SIMD, the VGPR limit)
// fit in a CU's 160 KiB (256 candidates took 10,752 B: 14 waves); u8 slots and u8 counters.
// CAPC = 480 (second pass over the first's overflowing chunks): u16 slots and counters, 19.8 KB.
template <int WPE, bool PROF, int CAPC = 240, bool GEN = true>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE)))
void knn_chunk_lane_kernel(KnnArgs a) {
  using SlotT = typename std::conditional<(CAPC < 256), uint8_t, uint16_t>::type;
  constexpr int SB = sizeof(SlotT);      // bytes per slot and per bin counter
  constexpr int NWC = LS_NB * SB / 4;    // counter words per lane (64 bins)
  // candidates: x, y, z, w [4][CAPC], index, rgbe; the shared estimate's terms reuse the same
  // 24 B per candidate ([3][CAPC] doubles, chunk_estimate_shared)
  __shared__ __attribute__((aligned(16))) double cand_lds[3 * CAPC];
  float *const cbase = reinterpret_cast<float *>(cand_lds);
  const Cands<CAPC> cpos{cbase};
  uint32_t *const cidx = reinterpret_cast<uint32_t *>(cbase + 4 * CAPC);
  uint32_t *const crgbe = cidx + CAPC;
  // kept LDS slots [s][lane] (K <= 64, u8) during the collect and the estimate; during the
  // counting passes the lanes' bin counters [w][lane] (u32, four u8 bins each), and during the
  // bound phase the centre select's 256-bin histogram. One spare slot row (row 64): a lane that
  // keeps exactly K = 64 photons without a bracket stores its later, unkept candidates there
  // (the collect's branch-free store always writes entry n).
  // counting-pass layout (r05): lane-major with a stride of NWC + 1 words (coprime with
  // the banks: conflict-free), so a counter's address is base + (b & ~(PERW - 1)) / PERW words
  // -- one and + add instead of the word-major layout's shift, and, add
  constexpr int CST = NWC + 1;   // counter row stride (words)
  __shared__ uint32_t selh[(16 * SB * 64 + 16 * SB) > 64 * (NWC + 1) ? (16 * SB * 64 + 16 * SB) : 64 * (NWC + 1)];
  SlotT *sel = reinterpret_cast<SlotT *>(selh);
  uint32_t *hist = selh;
  // kd walk stack (walk_within): the last 64 words of selh, live only during the gather walk,
  // when neither the counters nor the slot lists are (the bound phase's histogram is words
  // 0-255)
  uint32_t *const stk = selh + (sizeof(selh) / sizeof(uint32_t) - 64);
  const int lane = threadIdx.x;
  const int K = a.K;
  uint64_t st_q = 0, st_found = 0, st_vis = 0;
  ChunkProf P;
  P.on = PROF;  // a template argument: the counters cost registers
  P.t = 0;
  for (int i = 0; i < 10; i++) P.c[i] = 0;
  const int minsub = a.chunk_minsub > 0 ? a.chunk_minsub : 64;
  for (int64_t chunk = blockIdx.x; chunk * 64 < a.nq; chunk += gridDim.x) {
    bool valid;
    int64_t qi;
    float4 qp;
    chunk_load_query(a, chunk, lane, valid, qi, qp);
    uint64_t vmask = __ballot(valid);
    if (vmask == 0) continue;
    // A chunk whose gather overflows is retried as halves, quarters, ... down to minsub
    // Morton-adjacent queries (smaller boxes gather fewer photons); what still overflows goes
    // to the per-lane kernel. Lanes outside the current group idle through its select.
    uint64_t pending = vmask;
    for (int sub = 64; sub >= minsub && pending; sub >>= 1) {
    for (int g0 = 0; g0 < 64; g0 += sub) {
    const uint64_t gm = (sub == 64) ? ~0ull : (((1ull << sub) - 1ull) << g0);
    if (!(pending & gm)) continue;
    const bool act = valid && ((gm >> lane) & 1ull);
    if (P.on) P.t = clock64();
    ChunkGeom G;
    // u8 slot lists below: at most 255 candidates per chunk
    chunk_bound_gather<CAPC>(a, lane, act, qp, CAPC - 1, cpos, cidx, crgbe, hist, stk, G, P);
    __syncthreads();
    if (G.overflow) continue;
    pending &= ~gm;
    const uint32_t count = G.count;
    const float qx = qp.x, qy = qp.y, qz = qp.z;
    // ---- 3. lane select. State: every valid candidate with d2 < A is kept; `need` more come
    //         from the bracket [A, B] (smallest (d2, kd index) first); above B nothing is kept.
    float A = 0.0f, B = query_lim2(a, G, qx, qy, qz);
    // Bin origin of the first pass: with the exact d_K(c), d_K(q) >= d_K(c) - |q - c|, so the
    // K-th key lies in [O, B] with O = (d_K(c) - |q - c|)^2; bin 0 takes everything below O.
    // The origin only shapes the bins (any O < B gives the same result), so no rounding
    // margin. From a looser upper bound on d_K(c) (the dk bounds) the same O can lie above the
    // K-th key (all of it in bin 0, a second pass): those bins start at 0 (GI_KNN_DBG & 32
    // restores the old origin for measurements).
    float O = A;
    if (G.dkc >= 0.0 && (G.dkc_exact || (a.dbg & 32))) {
      double ex = (double)qx - G.cx, ey = (double)qy - G.cy, ez = (double)qz - G.cz;
      double lo = G.dkc - sqrt(ex * ex + ey * ey + ez * ez);
      if (lo > 0.0) {
        float o = (float)(lo * lo);
        if (o < B) O = o;
      }
    }
    int need = (act && K > 0) ? K : 0;
    int mode = need > 0 ? 1 : 0;  // 1 counting, 2 bracket resolved by the collect pass, 0 done
    if (!(a.dbg & 4)) {
      for (int pass = 0; pass < LS_PASSES && __ballot(mode == 1); pass++) {
        if (P.on) P.c[8]++;
        const bool on = mode == 1;
        float sc, off;
        bin_setup<LS_NB>(O, B, sc, off);
        const uint32_t ab = on ? __float_as_uint(A) : ~0u;
        const uint32_t span = on ? __float_as_uint(B) - __float_as_uint(A) : 0u;
        // LS_NB = 64 bins per lane: u8 counters packed four per LDS word [w][lane] (w = bin / 4;
        // conflict-free, one ds_add per candidate; at most 255 members, so no byte carries)
#pragma unroll
        for (int w = 0; w < NWC; w++) selh[lane * CST + w] = 0u;
        // groups of 8 candidates: the group's (broadcast) LDS reads are issued together and the
        // loop body has no branches (non-members, and the +inf padding past `count`, add 0)
        constexpr uint32_t PERW = 4 / SB;  // counters per word
        for (uint32_t s0 = 0; s0 < count; s0 += 8) {
          float dg[8];
          cand_d2x8(cpos, s0, qx, qy, qz, dg);
#pragma unroll
          for (int u = 0; u < 8; u++) {
            const uint32_t b = binN<LS_NB>(dg[u], sc, off);
            const uint32_t inc = in_bracket(dg[u], ab, span) ? (1u << ((b & (PERW - 1u)) * 8u * SB)) : 0u;
            atomicAdd(&selh[lane * CST + b / PERW], inc);
          }
        }
        if (on) {
          // the K-th key's bin: word sums first, counters inside the word
          uint32_t before = 0, bs = LS_NB, cb = 0;
          constexpr uint32_t CM = SB == 1 ? 255u : 65535u;
#pragma unroll
          for (int w = 0; w < NWC; w++) {
            const uint32_t c4 = selh[lane * CST + w];
            const uint32_t ws = SB == 1 ? __builtin_amdgcn_sad_u8(c4, 0u, 0u) : (c4 & 65535u) + (c4 >> 16);
            if (bs == LS_NB) {
              if (before + ws >= (uint32_t)need) {
#pragma unroll
                for (int j = 0; j < (int)PERW; j++) {
                  const uint32_t c = (c4 >> (8 * SB * j)) & CM;
                  if (bs == LS_NB) {
                    if (before + c >= (uint32_t)need) { bs = (uint32_t)(PERW * w + j); cb = c; }
                    else before += c;
                  }
                }
              } else {
                before += ws;
              }
            }
          }
          if (bs == LS_NB) {
            // fewer members than needed (first pass: fewer than K within the bound): keep all
            A = next_up(B);
            need = 0;
            mode = 0;
          } else {
            need -= (int)before;
            float nA = (bs == 0) ? A : bin_floor<LS_NB>(bs, O, B, sc, off);
            float nB = (bs == LS_NB - 1) ? B : next_down(bin_floor<LS_NB>(bs + 1, O, B, sc, off));
            if (cb == (uint32_t)need) {
              A = next_up(nB);
              need = 0;
              mode = 0;
            } else {
              A = nA;
              B = nB;
              // the collect keeps the K - need photons below A at the front of the lane's
              // slot list and the bracket's cb at its back: both must fit its 64 entries with
              // a gap of two (the collect's stores of unkept candidates land on the next free
              // entry of each end)
              if (cb <= (uint32_t)LS_BR_L && (uint32_t)(K - need) + cb <= 62u) mode = 2;
              else if (!(B > A)) mode = 3;  // more than LS_BR_L photons tied at one d2
            }
          }
        }
        O = A;
      }
    }
    // queries the counting passes did not resolve go to the exact per-lane kernel
    const bool fb = mode == 1 || mode == 3;
    uint64_t fbm = __ballot(fb);
    if (fbm) {
      to_fallback(a, fbm, fb, qi, lane);
      if (P.on) P.c[9] += (uint64_t)__popcll(fbm);
    }
    const bool col = act && !fb && !(a.dbg & 4);
    // collect: everything below A to the front of the lane's slot list (sel[n][lane]), the
    // bracket's photons to its back (sel[63 - m][lane]); the bracket is then sorted in registers
    int n = 0, m = 0;
    float km = 0.0f;
    const bool inb_on = col && need > 0;
    // branch-free like the counting passes: a candidate that is not kept is written to the next
    // free entry of its end of the list (overwritten by the next kept one, or never read)
    const float acol = col ? A : 0.0f;  // kept: d2 < acol
    const uint32_t ab = inb_on ? __float_as_uint(A) : ~0u;
    const uint32_t span = inb_on ? __float_as_uint(B) - __float_as_uint(A) : 0u;
    int bm = 63;  // next bracket entry, from the back
    for (uint32_t s0 = 0; s0 < count; s0 += 8) {
      float dg[8];
      cand_d2x8(cpos, s0, qx, qy, qz, dg);
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t s = s0 + u;
        const float d2 = dg[u];
        const bool kf = d2 < acol;
        const bool kb = in_bracket(d2, ab, span);
        // one store per candidate: a bracket member to the back entry bm, anything else to the
        // front entry n (a kept one stays there, an unkept one is overwritten by the next kept
        // one or never read; a lane without a bracket may fill all 64 entries, row 64 spare)
        sel[(kb ? bm : n) * 64 + lane] = (SlotT)s;
        n += kf ? 1 : 0;
        bm -= kb ? 1 : 0;
        km = fmaxf(km, kf ? d2 : 0.0f);
      }
    }
    m = 63 - bm;
    // keep the `need` smallest (d2, kd index) of the bracket, appended in that order: each
    // member's rank among the lane's members (keys are unique: kd indices differ) is its offset
    // in the kept list. Unrolled over LS_BR_L entries, but every step past the wave's largest
    // bracket is skipped by a uniform branch, so a wave pays mw (mw - 1) / 2 compares for its
    // largest bracket mw instead of a full sorting network.
    {
      int mw = inb_on ? m : 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mw = max(mw, __shfl_xor(mw, o, 64));
      uint64_t fk[LS_BR_L];
      uint32_t sl[LS_BR_L], rk[LS_BR_L];
#pragma unroll
      for (int i = 0; i < LS_BR_L; i++) {
        sl[i] = 0u;
        fk[i] = ~0ull;
        rk[i] = 0u;
        if (i >= mw) continue;
        if (inb_on && i < m) {
          sl[i] = sel[(63 - i) * 64 + lane];
          float d2 = cpos.d2(qx, qy, qz, sl[i]);
          fk[i] = ((uint64_t)__float_as_uint(d2) << 32) | (uint64_t)cidx[sl[i]];
        }
      }
#pragma unroll
      for (int i = 1; i < LS_BR_L; i++) {
        if (i < mw) {
#pragma unroll
          for (int j = 0; j < i; j++) {
            const bool lt = fk[j] < fk[i];
            rk[i] += lt ? 1u : 0u;
            rk[j] += lt ? 0u : 1u;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < LS_BR_L; i++) {
        if (i < mw && inb_on && i < m && rk[i] < (uint32_t)need) {
          sel[(n + (int)rk[i]) * 64 + lane] = (SlotT)sl[i];
          km = fmaxf(km, __uint_as_float((uint32_t)(fk[i] >> 32)));
        }
      }
      if (inb_on) n += need;
    }
    P.lap(2);
    // ---- 4. estimate
    if (!(a.dbg & 2)) {
      auto slot_at = [&](int s) { return (uint32_t)sel[s * 64 + lane]; };
      chunk_estimate_shared<CAPC>(a, lane, col, qi, qp, n, km, count, cpos, crgbe, cand_lds, slot_at,
                                  [&]() { chunk_estimate<GEN>(a, qi, qp, n, km, cpos, crgbe, slot_at); });
    }
    if (col) {
      st_q += 1;
      st_found += (uint64_t)n;
      st_vis += count;
    }
    __syncthreads();
    P.lap(3);
    }
    }
    if (pending) {
      to_fallback(a, pending, valid && ((pending >> lane) & 1ull), qi, lane);
    }
  }
  chunk_flush_stats(a, P, st_q, st_found, st_vis);
}

// ---------------------------------------------------------------------------------------------
// lane select for large K (the caustic map's 225): no per-query slot lists in LDS. The kept
// candidates of a query are a bitmask over the chunk's LDS slots (NW words per lane), and the
// bin counters are 16 bits wide (a chunk may gather more than 255 photons). The chunk bound
// comes from the per-photon K-th distance bounds (KdView::dk), which the host requires here.
// Overflowing chunks and unresolved queries go to the one-query-per-wave kernel.
// ---------------------------------------------------------------------------------------------
#ifndef BIG_WPE
#define BIG_WPE 3  // large-K chunk kernel occupancy target (waves per SIMD)
#endif
template <int CAPC, bool PROF, bool GEN = true>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BIG_WPE)))
void knn_chunk_big_kernel(KnnArgs a) {
  constexpr int NW = CAPC / 32;
  // bracket list length: 8 keeps the 512-candidate kernel at 17.6 KB of LDS (9 waves per CU)
  constexpr int BRB = CAPC <= 512 ? 8 : LS_BR_B;
  __shared__ __attribute__((aligned(16))) double cand_lds[3 * CAPC];  // as in the lane kernel
  float *const cbase = reinterpret_cast<float *>(cand_lds);
  const Cands<CAPC> cpos{cbase};
  uint32_t *const cidx = reinterpret_cast<uint32_t *>(cbase + 4 * CAPC);
  uint32_t *const crgbe = cidx + CAPC;
  __shared__ uint32_t stk[64];
  // kept-candidate bitmask [word][lane] during the collect and the estimate; during the counting
  // passes the lanes' LS_NBB 16-bit bin counters, two per word [w][lane]
  __shared__ uint32_t selw[(NW > LS_NBB / 2 ? NW : LS_NBB / 2) * 64];
  __shared__ uint16_t brl[(BRB + 1) * 64];  // bracket list [i][lane] of the collect
  const int lane = threadIdx.x;
  const int K = a.K;
  const int minsub = a.chunk_minsub > 0 ? a.chunk_minsub : 64;
  uint64_t st_q = 0, st_found = 0, st_vis = 0;
  ChunkProf P;
  P.on = PROF;
  P.t = 0;
  for (int i = 0; i < 10; i++) P.c[i] = 0;
  for (int64_t chunk = blockIdx.x; chunk * 64 < a.nq; chunk += gridDim.x) {
    bool valid;
    int64_t qi;
    float4 qp;
    chunk_load_query(a, chunk, lane, valid, qi, qp);
    uint64_t vmask = __ballot(valid);
    if (vmask == 0) continue;
    // an overflowing chunk is retried as halves, quarters, ... down to minsub queries (the
    // query-per-wave fallback costs several times a lane-select query even at 1/8 occupancy)
    uint64_t pending = vmask;
    for (int sub = 64; sub >= minsub && pending; sub >>= 1) {
    for (int g0 = 0; g0 < 64; g0 += sub) {
    const uint64_t gm = (sub == 64) ? ~0ull : (((1ull << sub) - 1ull) << g0);
    if (!(pending & gm)) continue;
    const bool act = valid && ((gm >> lane) & 1ull);
    if (P.on) P.t = clock64();
    ChunkGeom G;
    // selw (>= 256 words, idle until the counting passes) is the exact bound's select scratch
    chunk_bound_gather<CAPC>(a, lane, act, qp, CAPC, cpos, cidx, crgbe, selw, stk, G, P);
    __syncthreads();
    if (G.overflow || G.dkc < 0.0) continue;
    pending &= ~gm;
    const uint32_t count = G.count;
    const float qx = qp.x, qy = qp.y, qz = qp.z;
    // ---- lane select (see knn_chunk_lane_kernel): LS_NBB value-range bins per counting pass,
    //      16-bit counters packed two per LDS word [w][lane] (a chunk gathers <= 1024 photons)
    float A = 0.0f, B = query_lim2(a, G, qx, qy, qz);
    // bins from 0 unless GI_KNN_DBG & 64: dkc here is the dk upper bound, and the origin
    // (dkc - |q - c|)^2 from it can lie above the K-th key (measured 33.3 -> 32.1 ms/launch)
    float O = A;
    if (G.dkc_exact || (a.dbg & 64)) {
      double ex = (double)qx - G.cx, ey = (double)qy - G.cy, ez = (double)qz - G.cz;
      double lo = G.dkc - sqrt(ex * ex + ey * ey + ez * ez);
      if (lo > 0.0) {
        float o = (float)(lo * lo);
        if (o < B) O = o;
      }
    }
    int need = (act && K > 0) ? K : 0;
    int mode = need > 0 ? 1 : 0;
    for (int pass = 0; pass < LS_PASSES && __ballot(mode == 1); pass++) {
      if (P.on) P.c[8]++;
      const bool on = mode == 1;
      float sc, off;
      bin_setup<LS_NBB>(O, B, sc, off);
      const uint32_t ab = on ? __float_as_uint(A) : ~0u;
      const uint32_t span = on ? __float_as_uint(B) - __float_as_uint(A) : 0u;
#pragma unroll
      for (int w = 0; w < LS_NBB / 2; w++) selw[w * 64 + lane] = 0u;
      // branch-free groups of 8, as in the lane kernel (non-members and the +inf padding add 0)
      for (uint32_t s0 = 0; s0 < count; s0 += 8) {
        float dg[8];
        cand_d2x8(cpos, s0, qx, qy, qz, dg);
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const uint32_t b = binN<LS_NBB>(dg[u], sc, off);
          const uint32_t inc = in_bracket(dg[u], ab, span) ? (1u << ((b & 1u) << 4)) : 0u;
          atomicAdd(&selw[(b >> 1) * 64 + lane], inc);
        }
      }
      if (on) {
        uint32_t before = 0, bs = LS_NBB, cb = 0;
#pragma unroll
        for (int w = 0; w < LS_NBB / 2; w++) {
          const uint32_t c2 = selw[w * 64 + lane];
#pragma unroll
          for (int j = 0; j < 2; j++) {
            const uint32_t c = (c2 >> (16 * j)) & 0xffffu;
            if (bs == LS_NBB) {
              if (before + c >= (uint32_t)need) { bs = (uint32_t)(2 * w + j); cb = c; }
              else before += c;
            }
          }
        }
        if (bs == LS_NBB) {
          A = next_up(B);
          need = 0;
          mode = 0;
        } else {
          need -= (int)before;
          float nA = (bs == 0) ? A : bin_floor<LS_NBB>(bs, O, B, sc, off);
          float nB = (bs == LS_NBB - 1) ? B : next_down(bin_floor<LS_NBB>(bs + 1, O, B, sc, off));
          if (cb == (uint32_t)need) {
            A = next_up(nB);
            need = 0;
            mode = 0;
          } else {
            A = nA;
            B = nB;
            if (cb <= (uint32_t)BRB) mode = 2;
            else if (!(B > A)) mode = 3;
          }
        }
      }
      O = A;
    }
    const bool fb = mode == 1 || mode == 3;
    uint64_t fbm = __ballot(fb);
    if (fbm) {
      to_fallback(a, fbm, fb, qi, lane);
      if (P.on) P.c[9] += (uint64_t)__popcll(fbm);
    }
    const bool col = act && !fb;
    // ---- collect, branch-free: bitmask words of the candidates below A; the bracket's photons
    //      (<= BRB) to a per-lane LDS list, each candidate stored at the list's next free entry
    //      (a member advances it), then sorted by (d2, kd index) in registers
    int n = 0;
    float km = 0.0f;
    const bool inb_on = col && need > 0;
    const float acol = col ? A : 0.0f;
    const uint32_t cab = inb_on ? __float_as_uint(A) : ~0u;
    const uint32_t cspan = inb_on ? __float_as_uint(B) - __float_as_uint(A) : 0u;
    int m = 0;
    for (uint32_t w0 = 0; w0 < (count + 31) / 32; w0++) {
      uint32_t bits = 0;
#pragma unroll
      for (uint32_t j0 = 0; j0 < 32; j0 += 8) {
        const uint32_t s0 = w0 * 32 + j0;
        if (s0 >= count) break;  // wave-uniform
        float dg[8];
        cand_d2x8(cpos, s0, qx, qy, qz, dg);
#pragma unroll
        for (int u = 0; u < 8; u++) {
          const bool kf = dg[u] < acol;
          const bool kb = in_bracket(dg[u], cab, cspan);
          bits |= kf ? (1u << (j0 + u)) : 0u;
          km = fmaxf(km, kf ? dg[u] : 0.0f);
          brl[m * 64 + lane] = (uint16_t)(s0 + u);
          m += kb ? 1 : 0;
        }
      }
      selw[w0 * 64 + lane] = bits;
      n += __popc(bits);
    }
    // the `need` smallest (d2, kd index) of the bracket by rank (the kept set is a bitmask, so
    // only membership matters); steps past the wave's largest bracket skipped (uniform branch)
    {
      int mw = inb_on ? m : 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mw = max(mw, __shfl_xor(mw, o, 64));
      uint64_t fk[BRB];
      uint32_t sl[BRB], rk[BRB];
#pragma unroll
      for (int i = 0; i < BRB; i++) {
        sl[i] = 0u;
        fk[i] = ~0ull;
        rk[i] = 0u;
        if (i >= mw) continue;
        if (inb_on && i < m) {
          sl[i] = brl[i * 64 + lane];
          fk[i] = ((uint64_t)__float_as_uint(cpos.d2(qx, qy, qz, sl[i])) << 32) | (uint64_t)cidx[sl[i]];
        }
      }
#pragma unroll
      for (int i = 1; i < BRB; i++) {
        if (i < mw) {
#pragma unroll
          for (int j = 0; j < i; j++) {
            const bool lt = fk[j] < fk[i];
            rk[i] += lt ? 1u : 0u;
            rk[j] += lt ? 0u : 1u;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < BRB; i++) {
        if (i < mw && inb_on && i < m && rk[i] < (uint32_t)need) {
          selw[(sl[i] / 32) * 64 + lane] |= 1u << (sl[i] % 32);
          km = fmaxf(km, __uint_as_float((uint32_t)(fk[i] >> 32)));
        }
      }
      if (inb_on) n += need;
    }
    P.lap(2);
    // ---- estimate: the lane walks its bitmask in slot order
    {
      uint32_t wi = 0, bits = selw[lane];
      auto slot_at = [&](int) -> uint32_t {
        while (!bits && wi + 1 < (uint32_t)NW) {
          wi++;
          bits = selw[wi * 64 + lane];
        }
        if (!bits) return 0u;
        uint32_t b = (uint32_t)__ffs(bits) - 1u;
        bits &= bits - 1u;
        return wi * 32u + b;
      };
      chunk_estimate_shared<CAPC>(a, lane, col, qi, qp, n, km, count, cpos, crgbe, cand_lds, slot_at,
                                  [&]() { chunk_estimate<GEN>(a, qi, qp, n, km, cpos, crgbe, slot_at); });
    }
    if (col) {
      st_q += 1;
      st_found += (uint64_t)n;
      st_vis += count;
    }
    __syncthreads();
    P.lap(3);
    }
    }
    if (pending) to_fallback(a, pending, valid && ((pending >> lane) & 1ull), qi, lane);
  }
  chunk_flush_stats(a, P, st_q, st_found, st_vis);
}

// dense copy of the striped fallback list: block b copies stripe b % FB_QS after the fills of
// the stripes before it
__global__ __launch_bounds__(256) void fb_compact_kernel(const uint32_t *list, const uint32_t *count,
                                                         uint32_t cap_s, uint32_t *dense,
                                                         uint32_t *total) {
  const uint32_t s = blockIdx.x % FB_QS, part = blockIdx.x / FB_QS, parts = gridDim.x / FB_QS;
  uint32_t off = 0;
  for (uint32_t i = 0; i < s; i++) off += count[i * 32];
  const uint32_t n = count[s * 32];
  for (uint32_t idx = part * blockDim.x + threadIdx.x; idx < n; idx += parts * blockDim.x)
    dense[off + idx] = list[(size_t)s * cap_s + idx];
  if (s == FB_QS - 1 && part == 0 && threadIdx.x == 0) *total = off + n;
}

void launch_fb_compact(const uint32_t *list, const uint32_t *count, uint32_t cap_s, uint32_t *dense,
                       uint32_t *total, hipStream_t st) {
  fb_compact_kernel<<<FB_QS * 8, 256, 0, st>>>(list, count, cap_s, dense, total);
}

// chunk kernels' grid: one 64-query chunk per block, at most 2^17 blocks (grid-stride beyond)
unsigned knn_chunk_grid(int64_t nq) {
  int64_t chunks = (nq + 63) / 64;
  return (unsigned)(chunks < (1 << 17) ? chunks : (1 << 17));
}

// large-K chunk kernel (needs a.map.dk); cap = LDS candidates per chunk (384, 512 or 1024)
bool launch_knn_chunk_big(const KnnArgs &a, int cap, hipStream_t st) {
  if (a.nq == 0) return true;
  if (a.mode == KNN_MODE_LIST || a.mode == KNN_MODE_DK || !a.map.dk) return false;
  unsigned grid = knn_chunk_grid(a.nq);
  bool prof = (a.dbg & 16) != 0;
  if (cap <= 384) {
    if (prof) knn_chunk_big_kernel<384, true><<<grid, 64, 0, st>>>(a);
    else knn_chunk_big_kernel<384, false><<<grid, 64, 0, st>>>(a);
  } else if (cap <= 512) {
    if (prof) knn_chunk_big_kernel<512, true><<<grid, 64, 0, st>>>(a);
    else if (a.general) knn_chunk_big_kernel<512, false><<<grid, 64, 0, st>>>(a);
    else knn_chunk_big_kernel<512, false, false><<<grid, 64, 0, st>>>(a);
  } else {
    // second pass over the first pass's overflowing chunks: 32 KiB of LDS per wave
    if (a.general) knn_chunk_big_kernel<1024, false><<<grid, 64, 0, st>>>(a);
    else knn_chunk_big_kernel<1024, false, false><<<grid, 64, 0, st>>>(a);
  }
  return true;
}

// second lane-select pass (K <= 64) over the first pass's overflowing chunks' queries: 480 LDS
// candidates, u16 slots and counters
bool launch_knn_chunk2(const KnnArgs &a, hipStream_t st) {
  if (a.nq == 0) return true;
  if (a.mode == KNN_MODE_LIST || a.K > 64) return false;
  if (a.general) knn_chunk_lane_kernel<2, false, 480><<<knn_chunk_grid(a.nq), 64, 0, st>>>(a);
  else knn_chunk_lane_kernel<2, false, 480, false><<<knn_chunk_grid(a.nq), 64, 0, st>>>(a);
  return true;
}

// lane-select chunk kernel (K <= 64), 4 waves per SIMD (3 and 2 measured +4 % and +40 %)
#ifndef LANE_WPE
#define LANE_WPE 4
#endif
bool launch_knn_chunk(const KnnArgs &a, hipStream_t st) {
  if (a.nq == 0) return true;
  if (a.mode == KNN_MODE_LIST || a.K > 64) return false;
  unsigned grid = knn_chunk_grid(a.nq);
  // GI_KNN_DBG & 128: phase counters from the large-K kernel only
  if ((a.dbg & 16) && !(a.dbg & 128)) knn_chunk_lane_kernel<3, true><<<grid, 64, 0, st>>>(a);
  else if (a.general) knn_chunk_lane_kernel<LANE_WPE, false><<<grid, 64, 0, st>>>(a);
  else knn_chunk_lane_kernel<LANE_WPE, false, 240, false><<<grid, 64, 0, st>>>(a);
  return true;
}

}  // namespace gi
