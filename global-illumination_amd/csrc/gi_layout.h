// gi_layout.h -- POD layout of the flattened, device-resident scene and photon maps.
//
// The reference walks a pointer-based scene graph (R3SceneNode -> R3SceneElement -> R3Shape,
// R3SceneNode.cpp:420-510, R3SceneElement.cpp:209-243). On the device the graph is flattened
// into arrays in the same depth-first order (so "first element wins ties" semantics are kept):
//   DNode[]    nodes in pre-order; root = 0; world->local transform chain via parent links
//   DElement[] elements in (node pre-order, element order); material + shape range + bbox
//   DShape[]   shapes in element order; triangles / meshes index into DTri[]
//   DTri[]     triangles with precomputed plane and edge planes (R3Cont.cpp:491-512)
//   DBvhNode[] per-mesh linearised BVHs over the mesh's triangles (see DBvhNode)
// Everything geometric is fp64 (RNScalar is double; the 1e-6 tolerances of RNScalar.h:225-316
// need it). Photon maps are fp32 (see DESIGN.md "Data layout").
#pragma once
#include <stdint.h>

namespace gi {

enum ShapeKind { SK_TRI = 0, SK_MESH = 1, SK_SPHERE = 2, SK_BOX = 3, SK_CIRCLE = 4,
                 SK_CYLINDER = 5, SK_CONE = 6 };
enum LightKind { LK_DIR = 0, LK_POINT = 1, LK_SPOT = 2, LK_AREA = 3, LK_RECT = 4 };
enum MatFlags { MF_AMBIENT = 1, MF_DIFFUSE = 2, MF_SPECULAR = 4, MF_TRANSPARENT = 8,
                MF_EMISSIVE = 16 };

struct DTri {
  double p0[3];
  double n[3];       // plane normal
  double d;          // plane offset
  double ev[3][3];   // edge-plane normals  normalize(n x e_i)
  double ed[3];      // edge-plane offsets
  double bmin[3], bmax[3];
  int32_t idx;       // index within its mesh in file order (BVH leaves reorder the triangles;
                     // ties of the mesh's minimum t go to the lowest idx, R3Isect.cpp:813-829)
  int32_t pad;
};

// Linearised BVH of one mesh (R3TriangleArray) in depth-first pre-order: node i's first child is
// i + 1, and `skip` is the node after its subtree (the root's skip = the node count), so a walk
// needs no stack: descend to i + 1 when the ray meets the box, else jump to skip. Leaves hold
// triangles [tri_first, tri_first + tri_count) relative to the mesh's first triangle. Boxes are
// the union of the triangles' boxes widened by a margin larger than the 1e-6 containment
// tolerances of R3Contains(triangle) (R3Cont.cpp:491-512), so no triangle R3Intersects(ray,
// R3TriangleArray) would report is ever culled.
struct DBvhNode {
  double lo[3], hi[3];
  int32_t skip;
  int32_t tri_first;   // leaf: first triangle (mesh-relative); internal: -1
  int32_t tri_count;   // leaf: triangle count; internal: 0
  int32_t pad;
};

struct DShape {
  int32_t kind;
  int32_t tri_first;   // SK_TRI: triangle index; SK_MESH: first triangle
  int32_t tri_count;   // SK_MESH: number of triangles
  int32_t bvh_first;   // SK_MESH: root of its DBvhNode tree, -1 = no tree (small meshes)
  double c[3];         // sphere / circle centre
  double n[3];         // circle normal
  double r;            // radius
  double bmin[3], bmax[3];  // shape bbox (box shape = the box itself)
};

struct DElement {
  int32_t material;    // index into DMaterial[] (defaults are materialised by the loader)
  int32_t node;        // owning node
  int32_t shape_first, shape_count;
  double bmin[3], bmax[3];  // element bbox in node-local coordinates
  // the bbox grown by 1e-5 + 1e-9 |x| per side: a division-free slab test against it rejects
  // only elements R3Intersects(ray, box) + the t <= closest rule would reject too (gi_device.h
  // elem_maybe_hit)
  double pmin[3], pmax[3];
  // 1 when every shape is a triangle, sphere or circle: tests as cheap as the element's box
  // test, so scene_intersect tests the shapes first and the box only for an element that would
  // take a hit (same result: a box test that fails discards the element's hits either way)
  int32_t shapes_first_ok;
  // 1 when the owning node and all its ancestors are the identity: bmin/bmax are world
  // coordinates (soft_light's occluder mask)
  int32_t world;
};

constexpr int GI_MAX_DEPTH = 16;  // scene-graph depth supported on the device

struct DNode {
  double Tinv[12];     // world(parent)->local rows 0..2 of R4Matrix inverse
  double T[12];        // local->parent
  int32_t parent;      // -1 for root
  int32_t identity;    // transform is exactly the identity
  int32_t elem_first, elem_count;
  int32_t depth;       // nodes on the path root..this node
  int32_t chain[GI_MAX_DEPTH];  // that path, root first (precomputed: no per-ray walk)
  int32_t pad;
};

struct DMaterial {
  double ka[3], kd[3], ks[3], kt[3], e[3];
  double n, ir;
  int32_t flags;       // MatFlags (R3Brdf::UpdateFlags, R3Brdf.cpp:338-348)
  int32_t pad;
  // derived per-material constants used by the Monte Carlo loops (montecarlo.cpp:94-99)
  double max_kd, max_kt, max_ks, max_e;
};

struct DLight {
  int32_t kind;
  int32_t active;
  double color[3];
  double intensity;
  double pos[3];
  double dir[3];       // directional dir / spot dir / area normal / rect normal
  double ca, la, qa;
  double dropoff, cutoff;   // spot
  double radius;            // area
  double a1[3], a2[3];      // rect axes (unit)
  double len1, len2;
  // precomputed sampling frames (illumination_utils.cpp:109-119, 281-283)
  double su[3], sv[3];      // area: disk basis scaled by radius; rect: a1*len1, a2*len2
  double area;              // pi r^2 or |a1 x a2|
  double nr_ax1[3], nr_ax2[3];  // no-shadow area sampling axes (R3AreaLight.cpp:145-153)
};

struct DCamera {
  double eye[3];
  double far_org[3], far_right[3], far_up[3];  // render.cpp:67-69
  double dof_u[3], dof_v[3];                   // render.cpp:72-77
};

// Device photon map: SoA in kd-leaf order.
//   pos4[i]   = (x, y, z, bitcast(dir | flags << 16))
//   rgbe[i]   = packed RGBE bytes (r | g<<8 | b<<16 | e<<24)
//   nodes[j]  = (split, bitcast(axis)) for internal node j in [1, nleaves) of the implicit
//               complete tree; leaf l in [nleaves, 2*nleaves) holds photons
//               [start(l - nleaves), start(l - nleaves + 1)), start(j) = j * n / nleaves.
struct KdView {
  const float *pos4;       // float4
  const uint32_t *rgbe;
  const float *nodes;      // 2 x float4 per node (index 0 unused): {lo.xyz, split},
                           // {hi.xyz, axis bits}; nodes [L, 2L) are the leaves
  int64_t n;
  int32_t nleaves;
  int32_t levels;
  float bmin[3], bmax[3];
  // optional, per photon (kd order): an upper bound on the true distance from the photon to
  // its K-th nearest photon within r (the launch's K and r), +inf where fewer than K lie
  // within r; nullptr when not computed for this K / r
  const float *dk;
};

}  // namespace gi
