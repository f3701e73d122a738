// gi_kdbuild.hip -- photon-map kd-tree built on the device.
//
// The reference inserts photons into an R3Kdtree (R3Kdtree.cpp:1552-1671: recursive median
// split of each node's point range along its box's longest axis, random-pivot quickselect). The
// device map keeps the same kind of tree in the layout the k-NN kernels read (gi_host.cpp
// HostMap, KdView): an implicit complete tree over L = 2^levels leaves, leaf l owning kd-order
// positions [l*n/L, (l+1)*n/L), node v's range the union of its leaves'. Node v splits its range
// at the median position along the longest axis of its photons' tight box; its record is
// {lo.xyz, split}, {hi.xyz, axis bits} with the tight box.
//
// Built level by level, one radix sort per level instead of a recursion:
//   level d: (1) tight boxes of the 2^d nodes (segmented min/max over the current order),
//            (2) each node's axis from its box (longest extent, the host rule),
//            (3) a radix sort of all positions by (node, coordinate along the node's axis):
//                every node's range ends up ordered along its axis, so its lower half is the
//                lower child's range,
//            (4) split = the coordinate at the node's median position.
//   then the leaves' tight boxes, and the kd-order position / rgbe arrays.
// Equal coordinates are ordered by a hash of the emission index (step 3), so the tree is a
// deterministic function of the emission-ordered photons (the host build's nth_element gives
// another equally valid order inside a node; the k-NN set is the same up to ties at the K-th
// distance, which both orders break by kd-order index).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <stdint.h>
#include "gi_kdbuild.h"

namespace gi {

namespace {

__device__ __forceinline__ uint32_t f2o(float f) {  // order-preserving float -> u32
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float o2f(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// leaf of kd-order position i: the largest l with floor(l * n / L) <= i
__device__ __forceinline__ int64_t leaf_of(int64_t i, int64_t n, int64_t L) {
  return ((i + 1) * L - 1) / n;
}

// (1) tight boxes of the level-d nodes: orderable min/max per axis, one atomic per wave and
//     value when the wave's 64 positions share a node (all but the node boundaries)
__global__ __launch_bounds__(256) void kd_box_kernel(const KdPhoton *ph, const uint32_t *perm, int64_t n,
                                                     int64_t L, int levels, int d, uint32_t *box) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = i < n;
  int64_t v = 0;
  uint32_t o[3] = {0u, 0u, 0u};
  if (ok) {
    v = ((L + leaf_of(i, n, L)) >> (levels - d)) - ((int64_t)1 << d);
    const KdPhoton &p = ph[perm[i]];
    for (int k = 0; k < 3; k++) o[k] = f2o(p.pos[k]);
  }
  const int64_t v0 = __shfl((long long)v, 0, 64);
  const bool uniform = __ballot(ok && v == v0) == __ballot(1);
  if (uniform) {
    uint32_t mn[3], mx[3];
    for (int k = 0; k < 3; k++) {
      mn[k] = ok ? o[k] : 0xffffffffu;
      mx[k] = ok ? o[k] : 0u;
    }
    for (int off = 32; off > 0; off >>= 1)
      for (int k = 0; k < 3; k++) {
        mn[k] = min(mn[k], (uint32_t)__shfl_xor((int)mn[k], off, 64));
        mx[k] = max(mx[k], (uint32_t)__shfl_xor((int)mx[k], off, 64));
      }
    if ((threadIdx.x & 63) == 0 && __ballot(ok) != 0)
      for (int k = 0; k < 3; k++) {
        atomicMin(&box[6 * v0 + k], mn[k]);
        atomicMax(&box[6 * v0 + 3 + k], mx[k]);
      }
  } else if (ok) {
    for (int k = 0; k < 3; k++) {
      atomicMin(&box[6 * v + k], o[k]);
      atomicMax(&box[6 * v + 3 + k], o[k]);
    }
  }
}

__global__ void kd_box_init_kernel(uint32_t *box, int64_t nn) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < 6 * nn) box[j] = (j % 6) < 3 ? 0xffffffffu : 0u;
}

// (2) node records of level d: tight box and axis (the host kd_rec rule: x, then y or z only
//     when strictly longer); an empty node gets the empty box {+inf, -inf} and axis 0
__global__ void kd_node_kernel(const uint32_t *box, int64_t n, int64_t L, int levels, int d,
                               float *nodes, int32_t *axis) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ((int64_t)1 << d)) return;
  const int64_t v = ((int64_t)1 << d) + j;
  const int64_t span = L >> d;
  const int64_t lo = j * span * n / L, hi = (j + 1) * span * n / L;
  float mn[3], mx[3];
  for (int k = 0; k < 3; k++) {
    mn[k] = hi > lo ? o2f(box[6 * j + k]) : INFINITY;
    mx[k] = hi > lo ? o2f(box[6 * j + 3 + k]) : -INFINITY;
  }
  int ax = 0;
  float ext = mx[0] - mn[0];
  if (mx[1] - mn[1] > ext) { ax = 1; ext = mx[1] - mn[1]; }
  if (mx[2] - mn[2] > ext) ax = 2;
  float *r = nodes + 8 * v;
  r[0] = mn[0]; r[1] = mn[1]; r[2] = mn[2]; r[3] = 0.0f;
  r[4] = mx[0]; r[5] = mx[1]; r[6] = mx[2];
  const int32_t a = d < levels ? ax : 0;
  r[7] = __int_as_float(a);
  if (axis) axis[j] = a;
}

// (3) sort keys of level d: node (d bits) above the coordinate along the node's axis, above tb
//     bits of a hash of the photon's emission index. The hash scatters photons with equal
//     coordinates over both halves of a median that falls inside their run (photons on an
//     axis-aligned wall share its coordinate): kept in the previous level's order they would
//     split by another axis, and a query on that plane, which the split-plane descents send to
//     the upper child, would find its first leaf far away (measured: caustic chunk k-NN 670 ->
//     842 candidates per query on cornell); the host's nth_element scatters them too.
__global__ __launch_bounds__(256) void kd_key_kernel(const KdPhoton *ph, const uint32_t *perm, int64_t n,
                                                     int64_t L, int levels, int d, int tb,
                                                     const int32_t *axis, uint64_t *keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t j = ((L + leaf_of(i, n, L)) >> (levels - d)) - ((int64_t)1 << d);
  const uint32_t e = perm[i];
  const uint64_t h = tb ? (uint64_t)((e * 0x9E3779B1u) >> (32 - tb)) : 0ull;
  keys[i] = ((uint64_t)j << (32 + tb)) | ((uint64_t)f2o(ph[e].pos[axis[j]]) << tb) | h;
}

// (4) split of each level-d node: the coordinate at its median position (host kd_rec: the
//     nth_element pivot), the box's upper bound when the upper half is empty, 0 when empty
__global__ void kd_split_kernel(const KdPhoton *ph, const uint32_t *perm, int64_t n, int64_t L, int d,
                                float *nodes, const int32_t *axis) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= ((int64_t)1 << d)) return;
  const int64_t v = ((int64_t)1 << d) + j;
  const int64_t span = L >> d;
  const int64_t lo = j * span * n / L, hi = (j + 1) * span * n / L;
  const int64_t mid = (j * span + span / 2) * n / L;
  float split = 0.0f;
  if (hi > lo && mid < hi) split = ph[perm[mid]].pos[axis[j]];
  else if (hi > lo) split = nodes[8 * v + 4 + axis[j]];
  nodes[8 * v + 3] = split;
}

// kd-order photon arrays: pos4 {x, y, z, bits(dir | flags << 16)} and rgbe
__global__ __launch_bounds__(256) void kd_finish_kernel(const KdPhoton *ph, const uint32_t *perm, int64_t n,
                                                        float4 *pos4, uint32_t *rgbe) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const KdPhoton &p = ph[perm[i]];
  pos4[i] = make_float4(p.pos[0], p.pos[1], p.pos[2],
                        __uint_as_float((uint32_t)p.dir | ((uint32_t)p.flags << 16)));
  rgbe[i] = p.rgbe;
}

__global__ void kd_iota_kernel(uint32_t *v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (uint32_t)i;
}

unsigned blocks(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

}  // namespace

hipError_t kd_build_device(const KdPhoton *ph, int64_t n, int leaf_size, KdBuildScratch &s,
                           float *pos4, uint32_t *rgbe, float *nodes, uint32_t *perm_out, int *nleaves,
                           int *levels_out, hipStream_t st) {
  int64_t L = 1;
  int levels = 0;
  while (L * leaf_size < n) { L *= 2; levels++; }
  *nleaves = (int)L;
  *levels_out = levels;
  hipError_t e = hipMemsetAsync(nodes, 0, (size_t)16 * L * 4, st);
  if (e != hipSuccess || n == 0) {
    if (e == hipSuccess) {  // empty map: the root leaf's empty box (the kernel reads no box)
      kd_node_kernel<<<1, 64, 0, st>>>(nullptr, 0, 1, 0, 0, nodes, nullptr);
      e = hipGetLastError();
    }
    return e;
  }
  if ((e = s.grow(n, L)) != hipSuccess) return e;
  uint32_t *pa = s.perm0, *pb = s.perm1;
  uint64_t *ka = s.key0, *kb = s.key1;
  kd_iota_kernel<<<blocks(n, 256), 256, 0, st>>>(pa, n);
  for (int d = 0; d <= levels; d++) {
    const int64_t nn = (int64_t)1 << d;
    kd_box_init_kernel<<<blocks(6 * nn, 256), 256, 0, st>>>(s.box, nn);
    kd_box_kernel<<<blocks(n, 256), 256, 0, st>>>(ph, pa, n, L, levels, d, s.box);
    kd_node_kernel<<<blocks(nn, 256), 256, 0, st>>>(s.box, n, L, levels, d, nodes, s.axis);
    if (d == levels) break;
    const int hb = std::min(12, 32 - d);  // hash bits below the coordinate
    kd_key_kernel<<<blocks(n, 256), 256, 0, st>>>(ph, pa, n, L, levels, d, hb, s.axis, ka);
    size_t tb = s.tmp_cap;
    e = hipcub::DeviceRadixSort::SortPairs(s.tmp, tb, ka, kb, pa, pb, (int)n, 0, 32 + d + hb, st);
    if (e != hipSuccess) return e;
    std::swap(pa, pb);
    kd_split_kernel<<<blocks(nn, 256), 256, 0, st>>>(ph, pa, n, L, d, nodes, s.axis);
  }
  kd_finish_kernel<<<blocks(n, 256), 256, 0, st>>>(ph, pa, n, reinterpret_cast<float4 *>(pos4), rgbe);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if (perm_out) e = hipMemcpyAsync(perm_out, pa, (size_t)n * 4, hipMemcpyDeviceToHost, st);
  return e;
}

hipError_t KdBuildScratch::grow(int64_t n, int64_t L) {
  auto g = [](void **p, size_t &cap, size_t bytes) -> hipError_t {
    if (bytes <= cap && *p) return hipSuccess;
    if (*p) hipFree(*p);
    *p = nullptr;
    cap = 0;
    hipError_t r = hipMalloc(p, bytes);
    if (r == hipSuccess) cap = bytes;
    return r;
  };
  hipError_t e;
  if ((e = g((void **)&perm0, perm_cap0, (size_t)n * 4)) != hipSuccess) return e;
  if ((e = g((void **)&perm1, perm_cap1, (size_t)n * 4)) != hipSuccess) return e;
  if ((e = g((void **)&key0, key_cap0, (size_t)n * 8)) != hipSuccess) return e;
  if ((e = g((void **)&key1, key_cap1, (size_t)n * 8)) != hipSuccess) return e;
  if ((e = g((void **)&box, box_cap, (size_t)6 * 4 * L)) != hipSuccess) return e;
  if ((e = g((void **)&axis, axis_cap, (size_t)4 * L)) != hipSuccess) return e;
  size_t tb = 0;
  e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, key0, key1, perm0, perm1, (int)n, 0, 64);
  if (e != hipSuccess) return e;
  return g(&tmp, tmp_cap, tb + 256);
}

void KdBuildScratch::release() {
  void *ps[] = {perm0, perm1, key0, key1, box, axis, tmp};
  for (void *p : ps)
    if (p) hipFree(p);
  *this = KdBuildScratch();
}

}  // namespace gi
