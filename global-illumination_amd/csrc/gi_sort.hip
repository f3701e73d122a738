// gi_sort.hip -- spatial ordering of photon-map queries.
//
// The reference answers k-NN queries one at a time in path order (photon_utils.cpp:79), so
// consecutive queries land anywhere in the scene. On the GPU a wave runs 64 queries in
// lock-step: ordering queries along a 30-bit Morton curve over the scene box makes a wave's
// lanes walk the same kd-tree nodes and leaves (coherent control flow, L1/L2 reuse). The
// results are written back to each query's original slot, so the order is invisible to the
// per-pixel reduction.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include "gi_sort.h"

namespace gi {

__device__ __forceinline__ uint32_t spread10(uint32_t v) {
  v &= 0x3ffu;
  v = (v | (v << 16)) & 0x030000FFu;
  v = (v | (v << 8)) & 0x0300F00Fu;
  v = (v | (v << 4)) & 0x030C30C3u;
  v = (v | (v << 2)) & 0x09249249u;
  return v;
}

// 30-bit space-filling-curve key of a 10-bit cell (x, y, z): the 3-D Hilbert curve
// (Skilling's axes-to-transpose, "Programming the Hilbert curve", AIP Conf. Proc. 707, 2004),
// its transposed bits interleaved as Morton's are: consecutive keys are face-adjacent cells, so
// a 64-query chunk of the sorted list is more compact than a Z-order run (a floor patch at C2's
// query density: chunk radius 0.00170 -> 0.00133, photons gathered per chunk 87 -> 77;
// tools/sim_chunks.py). Only the order of the k-NN launches changes, never a result.
__device__ __forceinline__ uint32_t curve_key10(uint32_t x, uint32_t y, uint32_t z) {
  uint32_t X[3] = {x, y, z};
  for (uint32_t Q = 1u << 9; Q > 1u; Q >>= 1) {
    const uint32_t P = Q - 1u;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      if (X[i] & Q) {
        X[0] ^= P;  // invert
      } else {      // exchange
        const uint32_t t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  X[1] ^= X[0];
  X[2] ^= X[1];
  uint32_t t = 0;
  for (uint32_t Q = 1u << 9; Q > 1u; Q >>= 1)
    if (X[2] & Q) t ^= Q - 1u;
  X[0] ^= t;
  X[1] ^= t;
  X[2] ^= t;
  return (spread10(X[0]) << 2) | (spread10(X[1]) << 1) | spread10(X[2]);
}

// the same curve on B bits per axis (11 <= B <= 20) as a 64-bit key (3B bits)
__device__ __forceinline__ uint64_t spread21(uint32_t x) {
  uint64_t v = x & 0x1fffffu;
  v = (v | (v << 32)) & 0x1f00000000ffffull;
  v = (v | (v << 16)) & 0x1f0000ff0000ffull;
  v = (v | (v << 8)) & 0x100f00f00f00f00full;
  v = (v | (v << 4)) & 0x10c30c30c30c30c3ull;
  v = (v | (v << 2)) & 0x1249249249249249ull;
  return v;
}
template <int B>
__device__ __forceinline__ uint64_t curve_key64(uint32_t x, uint32_t y, uint32_t z) {
  uint32_t X[3] = {x, y, z};
  for (uint32_t Q = 1u << (B - 1); Q > 1u; Q >>= 1) {
    const uint32_t P = Q - 1u;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      if (X[i] & Q) {
        X[0] ^= P;
      } else {
        const uint32_t t = (X[0] ^ X[i]) & P;
        X[0] ^= t;
        X[i] ^= t;
      }
    }
  }
  X[1] ^= X[0];
  X[2] ^= X[1];
  uint32_t t = 0;
  for (uint32_t Q = 1u << (B - 1); Q > 1u; Q >>= 1)
    if (X[2] & Q) t ^= Q - 1u;
  return (spread21(X[0] ^ t) << 2) | (spread21(X[1] ^ t) << 1) | spread21(X[2] ^ t);
}

// 30-bit surface key (r06): the query surface's dominant normal axis and side (6 faces, 3 bits),
// its coordinate along that axis in 32 slabs of the scene box (5 bits), and the 2-D Hilbert
// curve of the other two coordinates on square 11-bit cells (22 bits). Queries on a plane (every
// global-map query of a cornell wall) then follow a 2-D curve in that plane instead of the plane's
// cut through the 3-D curve, which leaves and re-enters it: 64 consecutive queries cover a
// more compact patch, and the chunk gathers fewer photons.
template <int B>
__device__ __forceinline__ uint64_t hilbert2(uint32_t x, uint32_t y) {
  uint64_t d = 0;
  for (uint32_t s = 1u << (B - 1); s > 0u; s >>= 1) {
    const uint32_t rx = (x & s) ? 1u : 0u, ry = (y & s) ? 1u : 0u;
    d += (uint64_t)s * s * ((3u * rx) ^ ry);
    if (ry == 0u) {
      if (rx == 1u) {
        x = s - 1u - (x & (s - 1u));
        y = s - 1u - (y & (s - 1u));
      }
      const uint32_t t = x;
      x = y;
      y = t;
    }
  }
  return d;
}
__device__ __forceinline__ uint32_t hilbert2_11(uint32_t x, uint32_t y) { return (uint32_t)hilbert2<11>(x, y); }
// the face / slab / in-plane cells of a surface key with B-bit in-plane cells
struct SurfCell {
  uint32_t face, dep, cu, cv;
};
__device__ __forceinline__ SurfCell surface_cell(const float4 &p, float ox, float oy, float oz,
                                                 const float sdep[3], float siso, float cmax) {
  // the face comes with the query (qpos.w bits 28-30, put_query); selects, not indexed arrays
  // (a lane-varying index into a local or kernel-argument array goes through scratch memory)
  SurfCell c;
  c.face = (__float_as_uint(p.w) >> 28) & 7u;
  const bool a0 = c.face < 2u, a1 = c.face == 2u || c.face == 3u;
  const float cx = p.x - ox, cy = p.y - oy, cz = p.z - oz;
  const float cw = a0 ? cx * sdep[0] : a1 ? cy * sdep[1] : cz * sdep[2];
  const float u = a0 ? cy : cx, v = (a0 || a1) ? cz : cy;
  c.dep = (uint32_t)fminf(fmaxf(cw, 0.0f), 31.0f);
  c.cu = (uint32_t)fminf(fmaxf(u * siso, 0.0f), cmax);
  c.cv = (uint32_t)fminf(fmaxf(v * siso, 0.0f), cmax);
  return c;
}
__global__ void morton_kernel(const float4 *q, int64_t n, float ox, float oy, float oz,
                              float sx, float sy, float sz, float cmax, uint32_t *keys, uint32_t *vals) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float4 p = q[i];
  float fx = fminf(fmaxf((p.x - ox) * sx, 0.0f), cmax);
  float fy = fminf(fmaxf((p.y - oy) * sy, 0.0f), cmax);
  float fz = fminf(fmaxf((p.z - oz) * sz, 0.0f), cmax);
  keys[i] = curve_key10((uint32_t)fx, (uint32_t)fy, (uint32_t)fz);
  vals[i] = (uint32_t)i;
}

// A sort scratch buffer that only grows, with the headroom rule of gi_host.cpp's DBuf: at least
// 1/8 above the request and twice the old capacity, none when the device is short of memory.
static hipError_t grow_scratch(void *&p, size_t &cap, size_t bytes) {
  if (bytes <= cap && p) return hipSuccess;
  size_t want = cap ? std::max(std::min(cap * 2, bytes + bytes / 2), bytes + bytes / 8) : bytes;
  if (p) hipFree(p);
  p = nullptr;
  cap = 0;
  if (want > bytes) {
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < want + tot / 4) want = bytes;
  }
  hipError_t r = hipMalloc(&p, want);
  if (r != hipSuccess && want > bytes) {
    (void)hipGetLastError();
    want = bytes;
    r = hipMalloc(&p, want);
  }
  if (r == hipSuccess) cap = want;
  return r;
}

hipError_t morton_order(const float4 *q, int64_t n, const float bmin[3], const float bmax[3],
                        SortScratch &s, uint32_t **perm_out, hipStream_t st) {
  *perm_out = nullptr;
  if (n <= 0) return hipSuccess;
  hipError_t e;
  auto grow = grow_scratch;
  size_t b4 = (size_t)n * 4;
  if ((e = grow(s.k0, s.k0_cap, b4)) != hipSuccess) return e;
  if ((e = grow(s.k1, s.k1_cap, b4)) != hipSuccess) return e;
  if ((e = grow(s.v0, s.v0_cap, b4)) != hipSuccess) return e;
  if ((e = grow(s.v1, s.v1_cap, b4)) != hipSuccess) return e;
  // 2^10 cells per axis: a 30-bit code, four 8-bit radix passes
  constexpr int bits = 10;
  const float cmax = (float)((1 << bits) - 1);
  float sc[3];
  for (int i = 0; i < 3; i++) {
    float ext = bmax[i] - bmin[i];
    sc[i] = ext > 0 ? cmax / ext : 0.0f;
  }
  morton_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
      q, n, bmin[0], bmin[1], bmin[2], sc[0], sc[1], sc[2], cmax, (uint32_t *)s.k0, (uint32_t *)s.v0);
  size_t tb = 0;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t *)s.k0, (uint32_t *)s.k1,
                                         (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0, 3 * bits,
                                         st);
  if (e != hipSuccess) return e;
  if ((e = grow(s.tmp, s.tmp_cap, tb + 256)) != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortPairs(s.tmp, tb, (const uint32_t *)s.k0, (uint32_t *)s.k1,
                                         (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0, 3 * bits,
                                         st);
  if (e != hipSuccess) return e;
  *perm_out = (uint32_t *)s.v1;
  return hipSuccess;
}

// Morton keys of the valid queries (meta != QMETA_NONE) and, for the empty slots, the key 2^30
// (above every 30-bit code): the stable sort puts the valid queries first, in the order
// morton_order gives them, and the empty ones after them
__global__ void morton_valid_kernel(const float4 *q, int64_t n, float ox, float oy, float oz,
                                    float sx, float sy, float sz, float cmax, uint32_t *keys,
                                    uint32_t *vals) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float4 p = q[i];
  const bool valid = __float_as_uint(p.w) != 0xffffffffu;  // QMETA_NONE (gi_kernels.h)
  float fx = fminf(fmaxf((p.x - ox) * sx, 0.0f), cmax);
  float fy = fminf(fmaxf((p.y - oy) * sy, 0.0f), cmax);
  float fz = fminf(fmaxf((p.z - oz) * sz, 0.0f), cmax);
  keys[i] = valid ? curve_key10((uint32_t)fx, (uint32_t)fy, (uint32_t)fz) : (1u << 30);
  vals[i] = (uint32_t)i;
}

// morton_valid_kernel with B-bit cells (64-bit keys; the empty slots get 2^(3B))
template <int B>
__global__ void curve64_valid_kernel(const float4 *q, int64_t n, float ox, float oy, float oz,
                                     float sx, float sy, float sz, float cmax, uint64_t *keys,
                                     uint32_t *vals) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float4 p = q[i];
  const bool valid = __float_as_uint(p.w) != 0xffffffffu;  // QMETA_NONE (gi_kernels.h)
  float fx = fminf(fmaxf((p.x - ox) * sx, 0.0f), cmax);
  float fy = fminf(fmaxf((p.y - oy) * sy, 0.0f), cmax);
  float fz = fminf(fmaxf((p.z - oz) * sz, 0.0f), cmax);
  keys[i] = valid ? curve_key64<B>((uint32_t)fx, (uint32_t)fy, (uint32_t)fz) : (1ull << (3 * B));
  vals[i] = (uint32_t)i;
}
// the surface key with B-bit in-plane cells as a 64-bit key (8 + 2B bits: face, slab, 2-D curve;
// the empty slots get 2^(8 + 2B))
template <int B>
__global__ void surf64_valid_kernel(const float4 *q, int64_t n, KeyGeom g, uint64_t *keys,
                                    uint32_t *vals) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float4 p = q[i];
  const bool valid = __float_as_uint(p.w) != 0xffffffffu;  // QMETA_NONE (gi_kernels.h)
  uint64_t key = 1ull << (8 + 2 * B);
  if (valid) {
    const SurfCell c = surface_cell(p, g.o[0], g.o[1], g.o[2], g.sdep, g.siso, (float)((1u << B) - 1u));
    key = ((uint64_t)c.face << (5 + 2 * B)) | ((uint64_t)c.dep << (2 * B)) | hilbert2<B>(c.cu, c.cv);
  }
  keys[i] = key;
  vals[i] = (uint32_t)i;
}
// first sorted key >= empty (the valid keys sort before the empty slots' key): one wave, 64
// probes per round
template <typename KeyT>
__global__ void __launch_bounds__(64) first_empty_kernel(const KeyT *k, int64_t n, KeyT empty,
                                                         unsigned long long *out) {
  int64_t lo = 0, hi = n;  // the answer lies in [lo, hi]
  const int lane = threadIdx.x;
  while (lo < hi) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t p = lo + lane * step;
    const uint64_t m = __ballot(p >= hi || k[p] >= empty);
    if (m == 0) {  // every probe valid: past lane 63's
      lo += 63 * step + 1;
      continue;
    }
    const int f = __ffsll((unsigned long long)m) - 1;
    const int64_t nhi = lo + f * step;
    lo = f ? lo + (f - 1) * step + 1 : lo;
    hi = nhi < hi ? nhi : hi;
  }
  if (lane == 0) *out = (unsigned long long)lo;
}

// curve_order_rows: bit b of row r = primary slot 64 r + b holds a query (one wave per row)
__global__ void prim_rows_kernel(const float4 *q, int64_t nprim, uint64_t *rows) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool v = i < nprim && __float_as_uint(q[i].w) != 0xffffffffu;  // QMETA_NONE
  const uint64_t m = __ballot(v);
  if ((threadIdx.x & 63) == 0 && i < nprim) rows[i >> 6] = m;
}
__global__ void row_popc_kernel(const uint64_t *rows, int64_t R, uint32_t *cnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r < R) cnt[r] = (uint32_t)__popcll(rows[r]);
}
__device__ __forceinline__ uint32_t surface_key(const float4 &p, const KeyGeom &g) {
  const SurfCell c = surface_cell(p, g.o[0], g.o[1], g.o[2], g.sdep, g.siso, 2047.0f);
  return (c.face << 27) | (c.dep << 22) | hilbert2_11(c.cu, c.cv);
}

// the scatter and the keys in one pass (r05): lane b of row r's wave writes the key and slot of
// its query at the query's compacted position (its rank among the row's set bits after the
// rows before it); the appends get theirs in append_keys_kernel
__device__ __forceinline__ uint32_t slot_key10(const float4 *q, uint32_t slot, const KeyGeom &g) {
  const float4 p = q[slot];
  const bool valid = __float_as_uint(p.w) != 0xffffffffu;  // (always, by the masks)
  if (!valid) return 1u << 30;
  if (g.surf) return surface_key(p, g);
  float fx = fminf(fmaxf((p.x - g.o[0]) * g.s[0], 0.0f), g.cmax);
  float fy = fminf(fmaxf((p.y - g.o[1]) * g.s[1], 0.0f), g.cmax);
  float fz = fminf(fmaxf((p.z - g.o[2]) * g.s[2], 0.0f), g.cmax);
  return curve_key10((uint32_t)fx, (uint32_t)fy, (uint32_t)fz);
}
// one wave per 64 rows (r06; was one wave per row: C2's 6 M rows per list, half of them empty,
// cost 2.1 ms per launch in wave dispatch): the lanes load the group's row masks and offsets
// together, then the wave visits its non-empty rows two at a time (both rows' query loads issued
// before either key is computed)
__device__ __forceinline__ void row_put(const float4 *__restrict__ q, const KeyGeom &g, uint64_t m,
                                        uint32_t o, int64_t r, int64_t Rp, int64_t nprim, int lane,
                                        uint32_t *__restrict__ keys, uint32_t *__restrict__ vals) {
  if ((m >> lane) & 1ull) {
    const uint32_t at = o + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    const uint32_t slot = (uint32_t)(r < Rp ? 64 * r + lane : nprim + 64 * (r - Rp) + lane);
    keys[at] = slot_key10(q, slot, g);
    vals[at] = slot;
  }
}
__global__ __launch_bounds__(256) void row_keys_kernel(const uint64_t *rows, const uint32_t *off,
                                                       int64_t Rp, int64_t R, int64_t nprim,
                                                       const float4 *__restrict__ q, KeyGeom g,
                                                       uint32_t *__restrict__ keys,
                                                       uint32_t *__restrict__ vals) {
  const int64_t r0 = 64 * ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (r0 >= R) return;
  const int64_t rl = r0 + lane;
  const uint64_t mine = rl < R ? rows[rl] : 0ull;
  const uint32_t moff = rl < R ? off[rl] : 0u;
  uint64_t todo = __ballot(mine != 0ull);
  while (todo) {
    const int j = __ffsll((unsigned long long)todo) - 1;
    todo &= todo - 1ull;
    const uint64_t m1 = __shfl(mine, j, 64);
    const uint32_t o1 = (uint32_t)__shfl((int)moff, j, 64);
    if (todo) {
      const int j2 = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1ull;
      const uint64_t m2 = __shfl(mine, j2, 64);
      const uint32_t o2 = (uint32_t)__shfl((int)moff, j2, 64);
      row_put(q, g, m1, o1, r0 + j, Rp, nprim, lane, keys, vals);
      row_put(q, g, m2, o2, r0 + j2, Rp, nprim, lane, keys, vals);
    } else {
      row_put(q, g, m1, o1, r0 + j, Rp, nprim, lane, keys, vals);
    }
  }
}
__global__ void append_keys_kernel(const float4 *q, uint32_t qbase, int64_t napp, int64_t ndet,
                                   KeyGeom g, uint32_t *keys, uint32_t *vals) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= napp) return;
  const uint32_t slot = qbase + (uint32_t)i;
  keys[ndet + i] = slot_key10(q, slot, g);
  vals[ndet + i] = slot;
}

// the number of valid queries = the first sorted key >= 2^30, by a 64-way search in one wave
// (a per-wave atomic count in morton_valid_kernel serialised 6M same-address atomics: r05i,
// +32 ms per list)

// the row path's 30-bit key sort: three onesweep passes of 10 bits (rocprim's gfx950 default for
// 32-bit pairs is 8 bits: four passes). C2's 214 M pairs per launch: 5.8 -> 5.1 ms per launch,
// frame -8 ms; 11 bits (two passes of 11, one of 8) and sort blocks of 512 x 16 were slower, 1024
// x 12 the same (r06, profiles/r06_row_sort_ab.jsonl)
static hipError_t row_sort(void *tmp, size_t &tb, const uint32_t *k0, uint32_t *k1, const uint32_t *v0,
                           uint32_t *v1, int64_t n, hipStream_t st) {
  using cfg = rocprim::radix_sort_config<
      rocprim::default_config, rocprim::default_config,
      rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 16>, rocprim::kernel_config<1024, 16>, 10,
                                          rocprim::block_radix_rank_algorithm::match>>;
  return rocprim::radix_sort_pairs<cfg>(tmp, tb, k0, k1, v0, v1, (size_t)n, 0, 30, st);
}
// the caustic list's 41-bit surface keys in 64-bit words: hipcub's default (8-bit passes; 10-bit
// passes measured the same at C2 / C3 / C4)
static hipError_t wide_sort(void *tmp, size_t &tb, const uint64_t *k0, uint64_t *k1, const uint32_t *v0,
                            uint32_t *v1, int64_t n, int bits, hipStream_t st) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, tb, k0, k1, v0, v1, (int)n, 0, bits, st);
}

hipError_t morton_order_valid(const float4 *q, int64_t n, const float bmin[3], const float bmax[3],
                              SortScratch &s, uint32_t **perm_out, int64_t *nvalid, hipStream_t st,
                              int key_bits, bool surf) {
  *perm_out = nullptr;
  *nvalid = 0;
  if (n <= 0) return hipSuccess;
  hipError_t e;
  auto grow = grow_scratch;
  size_t b4 = (size_t)n * 4;
  const bool wide = key_bits > 10;
  const size_t kb = wide ? 2 * b4 : b4;
  if ((e = grow(s.k0, s.k0_cap, kb + 16)) != hipSuccess) return e;
  if ((e = grow(s.k1, s.k1_cap, kb)) != hipSuccess) return e;
  if ((e = grow(s.v0, s.v0_cap, b4)) != hipSuccess) return e;
  if ((e = grow(s.v1, s.v1_cap, b4)) != hipSuccess) return e;
  // the valid count lives past the keys (8 B, aligned)
  auto *d_cnt = reinterpret_cast<unsigned long long *>((char *)s.k0 + ((kb + 7) & ~(size_t)7));
  if (wide && surf) {
    // surface keys with 16-bit in-plane cells: 8 + 32 key bits and the empty slots' bit, six
    // radix passes (the 3-D curve's 16-bit cells take seven)
    constexpr int B = 16;
    KeyGeom g;
    float emax = 0.0f;
    for (int i = 0; i < 3; i++) {
      float ext = bmax[i] - bmin[i];
      g.o[i] = bmin[i];
      g.sdep[i] = ext > 0 ? 32.0f / ext : 0.0f;
      emax = std::max(emax, ext);
    }
    g.siso = emax > 0 ? (float)(1u << B) / emax : 0.0f;
    surf64_valid_kernel<B><<<(unsigned)((n + 255) / 256), 256, 0, st>>>(q, n, g, (uint64_t *)s.k0,
                                                                        (uint32_t *)s.v0);
    size_t tb = 0;
    e = wide_sort(nullptr, tb, (const uint64_t *)s.k0, (uint64_t *)s.k1, (const uint32_t *)s.v0,
                  (uint32_t *)s.v1, n, 8 + 2 * B + 1, st);
    if (e != hipSuccess) return e;
    if ((e = grow(s.tmp, s.tmp_cap, tb + 256)) != hipSuccess) return e;
    e = wide_sort(s.tmp, tb, (const uint64_t *)s.k0, (uint64_t *)s.k1, (const uint32_t *)s.v0,
                  (uint32_t *)s.v1, n, 8 + 2 * B + 1, st);
    if (e != hipSuccess) return e;
    first_empty_kernel<uint64_t><<<1, 64, 0, st>>>((const uint64_t *)s.k1, n, 1ull << (8 + 2 * B), d_cnt);
  } else if (wide) {
    // B-bit cells, 64-bit keys: 3B + 1 key bits, (3B + 1) / 8 rounded up radix passes
    const int B = key_bits > 20 ? 20 : key_bits;
    const float cm = (float)((1 << B) - 1);
    float sw[3];
    for (int i = 0; i < 3; i++) {
      float ext = bmax[i] - bmin[i];
      sw[i] = ext > 0 ? cm / ext : 0.0f;
    }
    const unsigned g = (unsigned)((n + 255) / 256);
#define CURVE64_CASE(b)                                                                      \
  case b:                                                                                    \
    curve64_valid_kernel<b><<<g, 256, 0, st>>>(q, n, bmin[0], bmin[1], bmin[2], sw[0], sw[1], \
                                               sw[2], cm, (uint64_t *)s.k0, (uint32_t *)s.v0); \
    break;
    switch (B) {
      CURVE64_CASE(11) CURVE64_CASE(12) CURVE64_CASE(13) CURVE64_CASE(14) CURVE64_CASE(15)
      CURVE64_CASE(16) CURVE64_CASE(17) CURVE64_CASE(18) CURVE64_CASE(19) default:
      CURVE64_CASE(20)
    }
#undef CURVE64_CASE
    size_t tb = 0;
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint64_t *)s.k0, (uint64_t *)s.k1,
                                           (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0,
                                           3 * B + 1, st);
    if (e != hipSuccess) return e;
    if ((e = grow(s.tmp, s.tmp_cap, tb + 256)) != hipSuccess) return e;
    e = hipcub::DeviceRadixSort::SortPairs(s.tmp, tb, (const uint64_t *)s.k0, (uint64_t *)s.k1,
                                           (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0,
                                           3 * B + 1, st);
    if (e != hipSuccess) return e;
    first_empty_kernel<uint64_t><<<1, 64, 0, st>>>((const uint64_t *)s.k1, n, 1ull << (3 * B), d_cnt);
  } else {
  constexpr int bits = 10;
  const float cmax = (float)((1 << bits) - 1);
  float sc[3];
  for (int i = 0; i < 3; i++) {
    float ext = bmax[i] - bmin[i];
    sc[i] = ext > 0 ? cmax / ext : 0.0f;
  }
  morton_valid_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>(
      q, n, bmin[0], bmin[1], bmin[2], sc[0], sc[1], sc[2], cmax, (uint32_t *)s.k0,
      (uint32_t *)s.v0);
  size_t tb = 0;
  // 31 key bits: the 30-bit code and the empty slots' 2^30 (four 8-bit passes, as for 30 bits)
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, (const uint32_t *)s.k0, (uint32_t *)s.k1,
                                         (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0,
                                         3 * bits + 1, st);
  if (e != hipSuccess) return e;
  if ((e = grow(s.tmp, s.tmp_cap, tb + 256)) != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortPairs(s.tmp, tb, (const uint32_t *)s.k0, (uint32_t *)s.k1,
                                         (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0,
                                         3 * bits + 1, st);
  if (e != hipSuccess) return e;
  first_empty_kernel<uint32_t><<<1, 64, 0, st>>>((const uint32_t *)s.k1, n, 1u << 30, d_cnt);
  }
  unsigned long long nv = 0;
  if ((e = hipMemcpyAsync(&nv, d_cnt, 8, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  *nvalid = (int64_t)nv;
  *perm_out = (uint32_t *)s.v1;
  return hipSuccess;
}

__global__ void iota_kernel(uint32_t *v, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

hipError_t key_order(const uint64_t *keys, int64_t n, int key_bits, KeySortScratch &s,
                     uint64_t **skeys, uint32_t **sslots, hipStream_t st) {
  *skeys = nullptr;
  *sslots = nullptr;
  if (n <= 0) return hipSuccess;
  hipError_t e;
  auto grow = grow_scratch;
  if ((e = grow(s.k1, s.k1_cap, (size_t)n * 8)) != hipSuccess) return e;
  if ((e = grow(s.v0, s.v0_cap, (size_t)n * 4)) != hipSuccess) return e;
  if ((e = grow(s.v1, s.v1_cap, (size_t)n * 4)) != hipSuccess) return e;
  iota_kernel<<<(unsigned)((n + 255) / 256), 256, 0, st>>>((uint32_t *)s.v0, n);
  size_t tb = 0;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys, (uint64_t *)s.k1,
                                         (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0,
                                         key_bits, st);
  if (e != hipSuccess) return e;
  if ((e = grow(s.tmp, s.tmp_cap, tb + 256)) != hipSuccess) return e;
  e = hipcub::DeviceRadixSort::SortPairs(s.tmp, tb, keys, (uint64_t *)s.k1,
                                         (const uint32_t *)s.v0, (uint32_t *)s.v1, (int)n, 0,
                                         key_bits, st);
  if (e != hipSuccess) return e;
  *skeys = (uint64_t *)s.k1;
  *sslots = (uint32_t *)s.v1;
  return hipSuccess;
}

void sort_scratch_release(KeySortScratch &s) {
  void *ps[] = {s.k1, s.v0, s.v1, s.tmp};
  for (void *p : ps)
    if (p) hipFree(p);
  s = KeySortScratch();
}

void sort_scratch_release(SortScratch &s) {
  void *ps[] = {s.k0, s.k1, s.v0, s.v1, s.tmp, s.rows, s.cnt};
  for (void *p : ps)
    if (p) hipFree(p);
  s = SortScratch();
}

hipError_t curve_order_rows(const float4 *q, int64_t nprim, const uint64_t *qmask, int64_t trows,
                            uint32_t qbase, int64_t nq, const float bmin[3], const float bmax[3],
                            SortScratch &s, uint32_t **perm_out, int64_t *nvalid, hipStream_t st,
                            bool surf) {
  *perm_out = nullptr;
  *nvalid = 0;
  if (nq <= 0) return hipSuccess;
  hipError_t e;
  auto grow = grow_scratch;
  const int64_t Rp = (nprim + 63) / 64, R = Rp + trows;
  if ((e = grow(s.rows, s.rows_cap, (size_t)(R + 1) * 8)) != hipSuccess) return e;
  if ((e = grow(s.cnt, s.cnt_cap, (size_t)(2 * R + 2) * 4)) != hipSuccess) return e;
  uint64_t *rows = (uint64_t *)s.rows;
  uint32_t *cnt = (uint32_t *)s.cnt, *off = cnt + (R + 1);
  if (nprim > 0) prim_rows_kernel<<<(unsigned)((nprim + 255) / 256), 256, 0, st>>>(q, nprim, rows);
  if (trows > 0 &&
      (e = hipMemcpyAsync(rows + Rp, qmask, (size_t)trows * 8, hipMemcpyDeviceToDevice, st)) != hipSuccess)
    return e;
  if (R > 0) row_popc_kernel<<<(unsigned)((R + 255) / 256), 256, 0, st>>>(rows, R, cnt);
  // exclusive offsets of the rows' counts, the total at off[R]
  if ((e = hipMemsetAsync(cnt + R, 0, 4, st)) != hipSuccess) return e;
  size_t tb = 0;
  e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, off, (int)(R + 1), st);
  if (e != hipSuccess) return e;
  if ((e = grow(s.tmp, s.tmp_cap, tb + 256)) != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(s.tmp, tb, cnt, off, (int)(R + 1), st);
  if (e != hipSuccess) return e;
  uint32_t ndet = 0;
  if ((e = hipMemcpyAsync(&ndet, off + R, 4, hipMemcpyDeviceToHost, st)) != hipSuccess) return e;
  if ((e = hipStreamSynchronize(st)) != hipSuccess) return e;
  const int64_t napp = nq > (int64_t)qbase ? nq - (int64_t)qbase : 0;
  const int64_t n = (int64_t)ndet + napp;
  if (n == 0) return hipSuccess;
  size_t b4 = (size_t)n * 4;
  if ((e = grow(s.k0, s.k0_cap, b4 + 16)) != hipSuccess) return e;
  if ((e = grow(s.k1, s.k1_cap, b4)) != hipSuccess) return e;
  if ((e = grow(s.v0, s.v0_cap, b4)) != hipSuccess) return e;
  if ((e = grow(s.v1, s.v1_cap, b4)) != hipSuccess) return e;
  constexpr int bits = 10;
  KeyGeom g;
  g.cmax = (float)((1 << bits) - 1);
  float emax = 0.0f;
  for (int i = 0; i < 3; i++) {
    float ext = bmax[i] - bmin[i];
    g.o[i] = bmin[i];
    g.s[i] = ext > 0 ? g.cmax / ext : 0.0f;
    g.sdep[i] = ext > 0 ? 32.0f / ext : 0.0f;
    emax = std::max(emax, ext);
  }
  g.siso = emax > 0 ? 2048.0f / emax : 0.0f;
  g.surf = surf ? 1 : 0;
  if (R > 0)
    row_keys_kernel<<<(unsigned)((R + 255) / 256), 256, 0, st>>>(rows, off, Rp, R, nprim, q, g,
                                                             (uint32_t *)s.k0, (uint32_t *)s.v0);
  if (napp > 0)
    append_keys_kernel<<<(unsigned)((napp + 255) / 256), 256, 0, st>>>(
        q, qbase, napp, (int64_t)ndet, g, (uint32_t *)s.k0, (uint32_t *)s.v0);
  // every compacted slot holds a query (the masks say so), so every key is below 2^30: 30 key
  // bits, and no count of the valid ones
  tb = 0;
  e = row_sort(nullptr, tb, (const uint32_t *)s.k0, (uint32_t *)s.k1, (const uint32_t *)s.v0,
               (uint32_t *)s.v1, n, st);
  if (e != hipSuccess) return e;
  if ((e = grow(s.tmp, s.tmp_cap, tb + 256)) != hipSuccess) return e;
  e = row_sort(s.tmp, tb, (const uint32_t *)s.k0, (uint32_t *)s.k1, (const uint32_t *)s.v0,
               (uint32_t *)s.v1, n, st);
  if (e != hipSuccess) return e;
  *nvalid = n;
  *perm_out = (uint32_t *)s.v1;
  return hipSuccess;
}

}  // namespace gi
