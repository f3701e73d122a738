// gi_sort.h -- Morton ordering of query batches (gi_sort.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gi {
struct SortScratch {
  void *k0 = nullptr, *k1 = nullptr, *v0 = nullptr, *v1 = nullptr, *tmp = nullptr;
  size_t k0_cap = 0, k1_cap = 0, v0_cap = 0, v1_cap = 0, tmp_cap = 0;
  // curve_order_rows: the row masks and their counts / offsets
  void *rows = nullptr, *cnt = nullptr;
  size_t rows_cap = 0, cnt_cap = 0;
};
// returns a device permutation (sorted position -> query index) valid until the next call
hipError_t morton_order(const float4 *q, int64_t n, const float bmin[3], const float bmax[3],
                        SortScratch &s, uint32_t **perm_out, hipStream_t st);
// the same with the empty slots (meta == QMETA_NONE) sorted after every valid query: the first
// *nvalid entries of the permutation are the valid queries in morton_order's order, so the k-NN
// launch takes only those (synchronises st for the count)
// key_bits > 10: cells of key_bits (<= 20) bits per axis and 64-bit keys; with surf as well, 64-bit
// surface keys with 16-bit in-plane cells (gi_sort.hip surf64_valid_kernel)
hipError_t morton_order_valid(const float4 *q, int64_t n, const float bmin[3], const float bmax[3],
                              SortScratch &s, uint32_t **perm_out, int64_t *nvalid, hipStream_t st,
                              int key_bits = 10, bool surf = false);
// The global list's launch order built from its slot layout instead of a sort over every slot:
// primary slots [0, nprim) (validity read from q), then the tiled indirect slots [nprim,
// nprim + 64 trows) whose row masks qmask[r] mark the entries holding a query (the reduction's
// own masks, gi_kernels.hip ind_kernel / ind_cont_kernel), then the appends [qbase, nq), all
// valid. The valid slots are compacted (row popcounts, a scan, a scatter: no per-slot pass over
// the empty ones), keyed like morton_order_valid and sorted: the first *nvalid entries of the
// permutation are the same queries, in the same order, as morton_order_valid's. With surf the
// keys are surface keys instead (gi_sort.hip surface_key: the face of the query's normal, a
// depth slab, the 2-D Hilbert curve in the face's plane).
hipError_t curve_order_rows(const float4 *q, int64_t nprim, const uint64_t *qmask, int64_t trows,
                            uint32_t qbase, int64_t nq, const float bmin[3], const float bmax[3],
                            SortScratch &s, uint32_t **perm_out, int64_t *nvalid, hipStream_t st,
                            bool surf = false);
void sort_scratch_release(SortScratch &s);
// key parameters: the 3-D curve's 10-bit cells (origin o, scale s per axis, cmax), or, with surf,
// the surface key's square 11-bit cells (siso) and 32 depth slabs per axis (sdep)
struct KeyGeom {
  float o[3], s[3], cmax;
  float siso, sdep[3];
  int surf;
};

struct KeySortScratch {
  void *k1 = nullptr, *v0 = nullptr, *v1 = nullptr, *tmp = nullptr;
  size_t k1_cap = 0, v0_cap = 0, v1_cap = 0, tmp_cap = 0;
};
// stable order of 64-bit keys: sorted keys + the original slot of each
hipError_t key_order(const uint64_t *keys, int64_t n, int key_bits, KeySortScratch &s,
                     uint64_t **skeys, uint32_t **sslots, hipStream_t st);
void sort_scratch_release(KeySortScratch &s);
}  // namespace gi
