// gi_kdbuild.h -- photon-map kd-tree built on the device (gi_kdbuild.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gi {
// emission-ordered photon record as gi_photon (include/gi.h) / gi_photon_dev: 20 bytes
struct KdPhoton {
  float pos[3];
  uint32_t rgbe;
  uint16_t dir;
  uint16_t flags;
};
static_assert(sizeof(KdPhoton) == 20, "photon record is 20 bytes");

struct KdBuildScratch {
  uint32_t *perm0 = nullptr, *perm1 = nullptr, *box = nullptr;
  uint64_t *key0 = nullptr, *key1 = nullptr;
  int32_t *axis = nullptr;
  void *tmp = nullptr;
  size_t perm_cap0 = 0, perm_cap1 = 0, key_cap0 = 0, key_cap1 = 0, box_cap = 0, axis_cap = 0,
         tmp_cap = 0;
  hipError_t grow(int64_t n, int64_t L);
  void release();
};

// Builds the map's implicit kd tree (leaves of <= leaf_size photons; gi_host.cpp HostMap
// layout) from n emission-ordered photons on the device: pos4 (16 B per photon), rgbe and nodes
// (16 * L floats) in kd order, perm_out (host memory, may be null) = kd order -> emission index.
// Asynchronous on st (perm_out is valid after the stream synchronises).
hipError_t kd_build_device(const KdPhoton *ph, int64_t n, int leaf_size, KdBuildScratch &s,
                           float *pos4, uint32_t *rgbe, float *nodes, uint32_t *perm_out,
                           int *nleaves, int *levels, hipStream_t st);
}  // namespace gi
