// gi_device.h -- device-side geometry, RNG and shading for the MI355X path.
//
// Everything here runs inside HIP kernels (gfx950). Geometry and shading are fp64 like the
// reference (RNScalar = double, RNBasics/RNScalar.h:14-18): the 1e-6 absolute tolerances of
// RNScalar.h:225-316 are below fp32 resolution at scene scale. Each function cites the
// reference function it re-expresses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gi_layout.h"
#include "gi_math.h"  // sin / cos / tan / asin / acos / atan2 / pow shared with the oracle

namespace gi {

#define GI_HD __host__ __device__ __forceinline__
// pow out of line: the Phong / spot terms call it from the path megakernels, where gi_math.h's
// inlined pow (log and exp in double-double) made the 256-VGPR kernels spill
__host__ __device__ __attribute__((noinline)) static double pow_ool(double x, double y) {
  return gm::pow(x, y);
}

constexpr double kEps = 1.0e-6;     // RN_EPSILON, RNScalar.cpp:21
constexpr double kInf = 1.0e6;      // RN_INFINITY, RNScalar.cpp:22
constexpr double kPi = 3.14159265358979323846;

// ---------------------------------------------------------------------------------------
// RNG: keyed counter streams (replaces RNThreadableRandomScalar, RNScalar.cpp:99-131).
// One stream per primary sample / spawned sample path / emitted photon, so results do not
// depend on launch geometry, batch size or GPU count.
// ---------------------------------------------------------------------------------------
GI_HD uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
GI_HD uint64_t stream_key(uint64_t seed, uint64_t kind, uint64_t a, uint64_t b) {
  uint64_t k = mix64(seed ^ (kind * 0xA0761D6478BD642FULL));
  k = mix64(k + a * 0xE7037ED1A0B428DBULL + 0x8EBC6AF09C88C6E3ULL);
  k = mix64(k + b * 0x589965CC75374CC3ULL + 0x1D8E4E27C47D124FULL);
  return k;
}
enum { KIND_PRIMARY = 1, KIND_TRANS = 2, KIND_SPEC = 3, KIND_IND = 4,
       KIND_PHOTON_GLOBAL = 5, KIND_PHOTON_CAUSTIC = 6 };
struct Rng {
  uint64_t key, ctr;
  GI_HD void init(uint64_t seed, uint64_t kind, uint64_t a, uint64_t b) {
    key = stream_key(seed, kind, a, b);
    ctr = 0;
  }
  GI_HD double next() {
    ctr++;
    uint64_t u = mix64(key + ctr * 0x9E3779B97F4A7C15ULL);
    return (double)(u >> 11) * (1.0 / 9007199254740992.0);
  }
};

// ---------------------------------------------------------------------------------------
// fp64 vectors
// ---------------------------------------------------------------------------------------
struct V {
  double x, y, z;
};
GI_HD V mk(double a, double b, double c) { V r; r.x = a; r.y = b; r.z = c; return r; }
GI_HD V ld3(const double *p) { return mk(p[0], p[1], p[2]); }
GI_HD V operator+(V a, V b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
GI_HD V operator-(V a, V b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
GI_HD V operator-(V a) { return mk(-a.x, -a.y, -a.z); }
GI_HD V operator*(V a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
GI_HD V operator*(double s, V a) { return mk(s * a.x, s * a.y, s * a.z); }
GI_HD V operator/(V a, double s) { return mk(a.x / s, a.y / s, a.z / s); }
GI_HD double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
GI_HD V cross(V a, V b) {
  return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
GI_HD double len(V a) { return sqrt((a.x * a.x) + (a.y * a.y) + (a.z * a.z)); }
GI_HD V normalize(V a) {  // R3Vector::Normalize, R3Vector.cpp:232-239
  double l = len(a);
  if (l == 0.0) return a;
  return mk(a.x / l, a.y / l, a.z / l);
}
GI_HD double dist(V a, V b) { return len(a - b); }
GI_HD double comp(V a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// RGB in fp64 (RNRgb)
struct C3 {
  double r, g, b;
};
GI_HD C3 rgb(double a, double b, double c) { C3 o; o.r = a; o.g = b; o.b = c; return o; }
GI_HD C3 ldc(const double *p) { return rgb(p[0], p[1], p[2]); }
GI_HD C3 operator+(C3 a, C3 b) { return rgb(a.r + b.r, a.g + b.g, a.b + b.b); }
GI_HD C3 operator*(C3 a, C3 b) { return rgb(a.r * b.r, a.g * b.g, a.b * b.b); }
GI_HD C3 operator*(C3 a, double s) { return rgb(a.r * s, a.g * s, a.b * s); }
GI_HD C3 operator*(double s, C3 a) { return rgb(s * a.r, s * a.g, s * a.b); }
GI_HD C3 operator/(C3 a, double s) { return rgb(a.r / s, a.g / s, a.b / s); }
GI_HD void operator+=(C3 &a, C3 b) { a.r += b.r; a.g += b.g; a.b += b.b; }
GI_HD void operator*=(C3 &a, C3 b) { a.r *= b.r; a.g *= b.g; a.b *= b.b; }
GI_HD void operator*=(C3 &a, double s) { a.r *= s; a.g *= s; a.b *= s; }
GI_HD double maxch(C3 c) {  // MaxChannelVal, graphics_utils.cpp:39-46
  double m = 0;
  if (c.r > m) m = c.r;
  if (c.g > m) m = c.g;
  if (c.b > m) m = c.b;
  return m;
}

// RNScalar.h tolerant predicates
GI_HD bool isPos(double s) { return s > kEps; }
GI_HD bool isNeg(double s) { return s < -kEps; }
GI_HD bool isPosOrZero(double s) { return s >= -kEps; }
GI_HD bool isNegOrZero(double s) { return s <= kEps; }
GI_HD bool isZero(double s) { return isPosOrZero(s) && isNegOrZero(s); }

// ---------------------------------------------------------------------------------------
// Scene view passed to kernels by value
// ---------------------------------------------------------------------------------------
struct SceneView {
  const DNode *nodes;
  const DElement *elems;
  const DShape *shapes;
  const DTri *tris;
  const DBvhNode *bvh;
  const DMaterial *mats;
  const DLight *lights;
  int32_t nnodes, nelems, nlights;
  uint32_t kinds;  // bit k set: the scene holds shapes of ShapeKind k
  int32_t hard_lights;  // every light is a point, spot or directional light
  int32_t elem_pretest; // scene_intersect runs elem_maybe_hit before each element's box test
  int32_t rigid;        // every node transform is rigid: a hit's world t is its distance
  int32_t pad;
  double radius;
  double centroid[3];
  double ambient[3];
  double background[3];
  DCamera cam;
};

// ---------------------------------------------------------------------------------------
// Intersection (R3Isect.cpp, R3Cont.cpp)
// ---------------------------------------------------------------------------------------
GI_HD bool box_contains(const double *mn, const double *mx, V p) {  // R3Cont.cpp:776-787
  if (mn[0] > mx[0] || mn[1] > mx[1] || mn[2] > mx[2]) return false;
  if (isNeg(p.x - mn[0]) || isNeg(p.y - mn[1]) || isNeg(p.z - mn[2])) return false;
  if (isPos(p.x - mx[0]) || isPos(p.y - mx[1]) || isPos(p.z - mx[2])) return false;
  return true;
}

// R3Intersects(ray, box), R3Isect.cpp:883-942
__device__ __forceinline__ bool ray_box(V o, V d, const double *mn, const double *mx, double *t_out,
                                     V *n_out) {
  if (mn[0] > mx[0] || mn[1] > mx[1] || mn[2] > mx[2]) return false;
  bool inside = box_contains(mn, mx, o);
  double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
#pragma unroll
  for (int dim = 0; dim < 3; dim++) {
    double tval;
    if (isPos(dd[dim])) {
      double bc = inside ? mx[dim] : mn[dim];
      double delta = bc - oo[dim];
      if (delta < 0.0) continue;
      tval = delta / dd[dim];
    } else if (isNeg(dd[dim])) {
      double bc = inside ? mn[dim] : mx[dim];
      double delta = bc - oo[dim];
      if (delta > 0.0) continue;
      tval = delta / dd[dim];
    } else {
      continue;
    }
    int d1 = (dim + 1) % 3, d2 = (dim + 2) % 3;
    double p1 = oo[d1] + dd[d1] * tval;
    double p2 = oo[d2] + dd[d2] * tval;
    if (isNegOrZero(p1 - mx[d1]) && isPosOrZero(p1 - mn[d1]) && isNegOrZero(p2 - mx[d2]) &&
        isPosOrZero(p2 - mn[d2])) {
      if (t_out) *t_out = tval;
      if (n_out) {
        double ax[3] = {0, 0, 0};
        ax[dim] = isNeg(dd[dim]) ? 1.0 : -1.0;
        *n_out = mk(ax[0], ax[1], ax[2]);
      }
      return true;
    }
  }
  return false;
}

// Division-free pre-test of an element's box (R3SceneElement::Intersects, R3SceneElement.cpp:
// 209-243, tests R3Contains(bbox, start) || R3Intersects(ray, bbox) with t <= closest). Slab
// test of t in [-2e-6, maxt + 1e-5 + 1e-9 maxt] against the box grown by 1e-5 + 1e-9 |x|
// (DElement::pmin/pmax), with inv = 1 / direction (+-inf on a zero component: the slab then
// spans everything or nothing; a NaN from 0 * inf drops out of fmin/fmax). Every element the
// exact test keeps passes: its hit point, or the ray origin when inside, lies within 1e-6 (the
// RN_EPSILON tolerances of ray_box / box_contains) plus rounding of the box, at a parameter
// within 1e-6 of [0, maxt]. A false here skips the exact test and its three divisions.
__device__ __forceinline__ bool elem_maybe_hit(const DElement &el, V o, V inv, double maxt) {
  double t0 = -2.0e-6, t1 = maxt + 1e-5 + 1e-9 * fabs(maxt);
  double ta = (el.pmin[0] - o.x) * inv.x, tb = (el.pmax[0] - o.x) * inv.x;
  t0 = fmax(t0, fmin(ta, tb));
  t1 = fmin(t1, fmax(ta, tb));
  ta = (el.pmin[1] - o.y) * inv.y; tb = (el.pmax[1] - o.y) * inv.y;
  t0 = fmax(t0, fmin(ta, tb));
  t1 = fmin(t1, fmax(ta, tb));
  ta = (el.pmin[2] - o.z) * inv.z; tb = (el.pmax[2] - o.z) * inv.z;
  t0 = fmax(t0, fmin(ta, tb));
  t1 = fmin(t1, fmax(ta, tb));
  return t0 <= t1;
}

// R3Intersects(ray, triangle) = plane (R3Isect.cpp:700-732) + R3Contains(triangle)
// (R3Cont.cpp:491-512); edge planes precomputed on the host with the same arithmetic.
// tmax: the caller's current closest t. A plane hit beyond it could not be taken by the caller
// (R3SceneElement's t <= closest rule), so the containment tests are skipped: same result, less
// fp64 work. (A division-free rejection of planes behind the ray or beyond tmax, from the
// numerator and |denom| with a 1e-9 margin, is exact but was measured slower, r05: C2 +1.3 %,
// C5 shard +2.9 %: the lanes of a wave of incoherent rays rarely all reject, so the division runs
// anyway and every lane pays the extra compares; profiles/r05_ray_tri_pretest_ab.txt.)
GI_HD bool ray_tri(V o, V d, const DTri &tr, double &t, V &p, double tmax = INFINITY) {
  V n = ld3(tr.n);
  double denom = dot(n, d);
  if (isZero(denom)) return false;
  double s = -(dot(o, n) + tr.d) / denom;
  if (isNeg(s)) return false;
  if (s > tmax) return false;
  V q = o + d * s;
  if (!box_contains(tr.bmin, tr.bmax, q)) return false;
  if (!isZero(q.x * n.x + q.y * n.y + q.z * n.z + tr.d)) return false;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    if (isNeg(q.x * tr.ev[i][0] + q.y * tr.ev[i][1] + q.z * tr.ev[i][2] + tr.ed[i])) return false;
  }
  t = s;
  p = q;
  return true;
}

// R3Intersects(ray, sphere), R3Isect.cpp:975-1021
GI_HD bool ray_sphere(V o, V d, V c, double r, double &t, V &p, V &nrm, double tmax = INFINITY) {
  V v0 = c - o;
  double r2 = r * r;
  double d2 = v0.x * v0.x + v0.y * v0.y + v0.z * v0.z;
  bool inside = isNegOrZero(d2 - r2);
  double v = dot(v0, d);
  if (!inside && isNegOrZero(v)) return false;
  double disc = r2 - (dot(v0, v0) - v * v);
  if (isNeg(disc)) return false;
  double dd = sqrt(disc);
  t = inside ? v + dd : v - dd;
  if (t > tmax) return false;  // beyond the caller's closest hit (see ray_tri)
  p = o + t * d;
  nrm = (p - c) / r;
  return true;
}

// R3Intersects(ray, circle), R3Isect.cpp:837-879
GI_HD bool ray_circle(V o, V d, V c, V n, double r, double &t, V &p) {
  if (r < 0) return false;
  double pd = -(n.x * c.x + n.y * c.y + n.z * c.z);
  double denom = dot(n, d);
  if (isZero(denom)) return false;
  double s = -(dot(o, n) + pd) / denom;
  if (isNeg(s)) return false;
  V q = o + d * s;
  V v = c - q;
  double dd = v.x * v.x + v.y * v.y + v.z * v.z;
  if (isPos(dd - r * r)) return false;
  t = s;
  p = q;
  return true;
}

// R3Intersects(ray, plane, NULL, &t), R3Isect.cpp:700-732: a ray lying in the plane counts
// as an intersection and leaves t unchanged.
GI_HD bool ray_plane_t(V o, V d, V n, double pd, double &t) {
  double denom = dot(n, d);
  double sd = o.x * n.x + o.y * n.y + o.z * n.z + pd;  // R3SignedDistance, R3Dist.cpp:603-607
  if (isZero(denom)) return isZero(sd);
  double s = -(sd) / denom;
  if (isNeg(s)) return false;
  t = s;
  return true;
}

// R3Intersects(ray, R3Cylinder), R3Isect.cpp:1025-1200 (Graphics Gems IV p.356): cylinder
// p1 -> p2 (unit axis, R3Span.cpp:63-70), radius r, cap planes through p1 (normal -A) and p2
// (normal +A) (R3Cylinder / R3Circle / R3Plane constructors). `line` is a radius-1e-3
// cylinder (R3Scene.cpp:1667-1687).
GI_HD bool ray_cylinder(V o, V R, V p1, V p2, double radius, double &t_out, V &p_out, V &n_out) {
  const double INF = 1.0e6;  // RN_INFINITY
  V A = p2 - p1;
  double alen = len(A);
  if (!isZero(alen)) A = A / alen;
  V nT = A, nB = -A;
  double dT = -(nT.x * p2.x + nT.y * p2.y + nT.z * p2.z);
  double dB = -(nB.x * p1.x + nB.y * p1.y + nB.z * p1.z);
  double cyl_t1, cyl_t2;
  V D = cross(R, A);
  double a = len(D);
  if (isZero(a)) {
    double d = len(cross(A, p1 - o));  // R3Distance(point, line), R3Dist.cpp:59-65
    if (!isNegOrZero(d - radius)) return false;
    cyl_t1 = 0.0;
    cyl_t2 = INF;
  } else {
    D = D / a;
    V RC = o - p1;
    double d = dot(RC, D);
    if (d < 0.0) d = -d;
    if (isPos(d - radius)) return false;
    double t = dot(cross(RC, A), D) / -a;
    double s;
    V O = normalize(cross(D, A));
    double b = radius * radius - d * d;
    if (isPos(b)) {
      double e = dot(R, O);
      s = sqrt(b) / e;
      if (s < 0.0) s = -s;
    } else {
      s = 0.0;
    }
    cyl_t2 = t + s;
    if (isNeg(cyl_t2)) return false;
    cyl_t1 = t - s;
    if (cyl_t1 < 0.0) cyl_t1 = 0.0;
  }
  double cap_t1 = 0, cap_t2 = 0;
  double dv = dot(R, A);
  double d_top = o.x * nT.x + o.y * nT.y + o.z * nT.z + dT;
  double d_base = o.x * nB.x + o.y * nB.y + o.z * nB.z + dB;
  if (isPos(d_top)) {
    if (isPosOrZero(dv)) return false;
    if (ray_plane_t(o, R, nT, dT, cap_t1) && isPos(cap_t1 - cyl_t2)) return false;
    else if (ray_plane_t(o, R, -nB, -dB, cap_t2) && isNeg(cap_t2 - cyl_t1)) return false;
    else if (isPos(cap_t1 - cyl_t1)) {
      t_out = cap_t1;
      p_out = o + R * cap_t1;
      n_out = nT;
      return true;
    }
  } else if (isPos(d_base)) {
    if (isNegOrZero(dv)) return false;
    if (ray_plane_t(o, R, nB, dB, cap_t1) && isPos(cap_t1 - cyl_t2)) return false;
    else if (ray_plane_t(o, R, -nT, -dT, cap_t2) && isNeg(cap_t2 - cyl_t1)) return false;
    else if (isPos(cap_t1 - cyl_t1)) {
      t_out = cap_t1;
      p_out = o + R * cap_t1;
      n_out = nB;
      return true;
    }
  } else {
    if (isPos(dv)) {
      if (ray_plane_t(o, R, -nT, -dT, cap_t1) && isNeg(cap_t1 - cyl_t1)) return false;
    } else if (isNeg(dv)) {
      if (ray_plane_t(o, R, -nB, -dB, cap_t1) && isNeg(cap_t1 - cyl_t1)) return false;
    }
  }
  t_out = cyl_t1;
  p_out = o + R * cyl_t1;
  V HB = p_out - p1;
  n_out = (HB - dot(HB, A) * A) / radius;
  return true;
}

// Slab test of a ray against a BVH node box for parameters in [-2e-6, bound] (a mesh hit may
// have t in [-1e-6, 0), Q2). inv = 1 / direction per axis (+-inf on a zero component: the slab
// then spans everything or nothing). The boxes carry a margin (gi_layout.h DBvhNode), so the
// test is conservative for every triangle hit R3Intersects(ray, R3TriangleArray) can report.
__device__ __forceinline__ bool bvh_box(const DBvhNode &b, V o, V inv, double bound) {
  double t0 = -2.0e-6, t1 = bound;
  double ta = (b.lo[0] - o.x) * inv.x, tb = (b.hi[0] - o.x) * inv.x;
  t0 = fmax(t0, fmin(ta, tb));
  t1 = fmin(t1, fmax(ta, tb));
  ta = (b.lo[1] - o.y) * inv.y; tb = (b.hi[1] - o.y) * inv.y;
  t0 = fmax(t0, fmin(ta, tb));
  t1 = fmin(t1, fmax(ta, tb));
  ta = (b.lo[2] - o.z) * inv.z; tb = (b.hi[2] - o.z) * inv.z;
  t0 = fmax(t0, fmin(ta, tb));
  t1 = fmin(t1, fmax(ta, tb));
  return t0 <= t1;
}

// R3Intersects(ray, R3TriangleArray) (R3Isect.cpp:800-833) through the mesh's BVH: the same
// minimum t over every triangle ray_tri accepts (t >= -1e-6, Q2), the same tie rule as the
// file-order loop (equal t: lowest triangle index), visiting only boxes the ray meets below the
// current minimum. Stackless pre-order walk with skip links.
// hint: a triangle (global index into S.tris) tested before the walk -- the one the ray leaves
// from. A ray leaving a mesh meets its own triangle at t ~ -1e-6 (Q2), and with that as the
// current minimum the walk prunes to the boxes around the origin instead of every box the ray
// crosses. The minimum over all triangles and its (t, index) tie rule do not depend on the order
// the triangles are tested in, so the result is unchanged. Returns the winner's global index in
// otri.
__device__ __noinline__ bool ray_mesh_bvh(const SceneView &S, const DShape &sh, V o, V d, double &t,
                                          V &p, V &n, double tmax, int hint, int &otri) {
  const DBvhNode *B = S.bvh + sh.bvh_first;
  const DTri *T = S.tris + sh.tri_first;
  const V inv = mk(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
  bool found = false;
  double mt = 3.40282346638528859811704183484516925440e+38;  // FLT_MAX, as the linear loop
  int32_t midx = 0x7fffffff;
  int mpos = -1;
  if (hint >= sh.tri_first && hint < sh.tri_first + sh.tri_count) {
    const DTri &tr = S.tris[hint];
    double tt;
    V pp;
    if (ray_tri(o, d, tr, tt, pp, tmax)) {
      found = true;
      p = pp;
      n = ld3(tr.n);
      mt = tt;
      midx = tr.idx;
      mpos = hint - sh.tri_first;
    }
  }
  const int end = B[0].skip;
  int i = 0;
  while (i < end) {
    const DBvhNode &nd = B[i];
    const double bound = fmin(mt, tmax);
    if (!bvh_box(nd, o, inv, bound)) {
      i = nd.skip;
      continue;
    }
    for (int k = 0; k < nd.tri_count; k++) {
      const DTri &tr = T[nd.tri_first + k];
      double tt;
      V pp;
      // (a triangle beyond the current minimum cannot win: ray_tri stops after its plane test)
      if (ray_tri(o, d, tr, tt, pp, fmin(mt, tmax)) && (tt < mt || (tt == mt && tr.idx < midx))) {
        found = true;
        p = pp;
        n = ld3(tr.n);
        mt = tt;
        midx = tr.idx;
        mpos = nd.tri_first + k;
      }
    }
    i++;
  }
  t = mt;
  otri = mpos >= 0 ? sh.tri_first + mpos : -1;
  return found;
}

// shape kinds a kernel instance is compiled for (KINDS template argument): the host launches
// the smallest instance covering SceneView::kinds, so scenes of triangles and spheres do not
// carry the mesh/box/cylinder code (registers and instruction cache) through their hot loops
constexpr uint32_t KIND_BIT(int k) { return 1u << k; }
constexpr uint32_t KINDS_ALL = ~0u;
constexpr uint32_t KINDS_TRI_SPHERE = (1u << SK_TRI) | (1u << SK_SPHERE);
constexpr uint32_t KINDS_POLY = (1u << SK_TRI) | (1u << SK_SPHERE) | (1u << SK_MESH) | (1u << SK_BOX);

// R3Shape::Intersects dispatch (R3Shape.cpp:328-329); SK_MESH is R3Intersects(ray,
// R3TriangleArray) (R3Isect.cpp:800-833): min t over ALL triangles, t >= -1e-6 allowed (Q2).
// hint / otri: the triangle a ray leaves from (ray_mesh_bvh) and the triangle hit (global index
// into S.tris, -1 for other shapes), passed on to the next bounce's walk
template <uint32_t KINDS = KINDS_ALL>
__device__ __forceinline__ bool shape_intersect(const SceneView &S, const DShape &sh, V o, V d,
                                             double &t, V &p, V &n, double tmax, int hint,
                                             int &otri) {
  otri = -1;
  if (KINDS == KINDS_TRI_SPHERE) {
    if (sh.kind == SK_TRI) {
      const DTri &tr = S.tris[sh.tri_first];
      if (!ray_tri(o, d, tr, t, p, tmax)) return false;
      n = ld3(tr.n);
      otri = sh.tri_first;
      return true;
    }
    if (sh.kind == SK_SPHERE) return ray_sphere(o, d, ld3(sh.c), sh.r, t, p, n, tmax);
    return false;
  }
  if (!(KINDS & KIND_BIT(sh.kind))) return false;
  switch (sh.kind) {
    case SK_TRI: {
      const DTri &tr = S.tris[sh.tri_first];
      if (!ray_tri(o, d, tr, t, p, tmax)) return false;
      n = ld3(tr.n);
      otri = sh.tri_first;
      return true;
    }
    case SK_MESH: {
      if (!ray_box(o, d, sh.bmin, sh.bmax, nullptr, nullptr)) return false;
      if (sh.bvh_first >= 0) return ray_mesh_bvh(S, sh, o, d, t, p, n, tmax, hint, otri);
      bool found = false;
      double mt = 3.40282346638528859811704183484516925440e+38;  // FLT_MAX
      for (int i = 0; i < sh.tri_count; i++) {
        const DTri &tr = S.tris[sh.tri_first + i];
        double tt;
        V pp;
        if (ray_tri(o, d, tr, tt, pp, tmax)) {  // a mesh hit beyond tmax is not taken either
          if (tt < mt) {
            found = true;
            p = pp;
            n = ld3(tr.n);
            mt = tt;
            otri = sh.tri_first + i;
          }
        }
      }
      t = mt;
      return found;
    }
    case SK_SPHERE:
      return ray_sphere(o, d, ld3(sh.c), sh.r, t, p, n, tmax);
    case SK_BOX: {
      double tt;
      V nn;
      if (!ray_box(o, d, sh.bmin, sh.bmax, &tt, &nn)) return false;
      t = tt;
      p = o + d * tt;
      n = nn;
      return true;
    }
    case SK_CIRCLE:
      if (!ray_circle(o, d, ld3(sh.c), ld3(sh.n), sh.r, t, p)) return false;
      n = ld3(sh.n);
      return true;
    case SK_CYLINDER:  // c = p1, n = p2
      return ray_cylinder(o, d, ld3(sh.c), ld3(sh.n), sh.r, t, p, n);
    default:
      return false;
  }
}

GI_HD V xf_point(const double *m, V p) {
  return mk(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
            m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}
GI_HD V xf_vec(const double *m, V v) {
  return mk(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
            m[8] * v.x + m[9] * v.y + m[10] * v.z);
}

struct Hit {
  V p, n;
  double t;
  int mat;
  int tri;  // triangle hit (global index into SceneView::tris), -1 for other shapes
};

// R3Scene::Intersects (R3Scene.cpp:471-479) -> R3SceneNode::Intersects (R3SceneNode.cpp:
// 420-510) -> R3SceneElement::Intersects (R3SceneElement.cpp:209-243), flattened: elements are
// visited in the graph's pre-order; an element "hits" only if it strictly improves on the
// current closest t (its "closest_t == max_t -> FALSE" rule), so earlier elements win ties.
// Ray direction is renormalised per graph level (R3Line::InverseTransform, R3Line.cpp:140).
// Inlined at every call site: node/element/shape records are wave-uniform (scalar loads) and
// the root-first transform chain is precomputed per node, so nothing lives in scratch.
//
// Elements of triangles / spheres / circles (DElement::shapes_first_ok) test their shapes
// first and the element box only when a shape would improve on closest: the box test gates the
// element's hits, so running it last gives the same result, and most rays miss most elements
// (the plane test of a triangle is cheaper than the box's slab divisions).
//
// Bounded form for shadow rays (illum_test): t_init < kInf starts the search at that world t
// (hits beyond it are not looked for), and the walk returns 2 as soon as an element is taken
// with t < t_exit (closest only decreases, so the final hit is nearer still). 0 = no hit below
// t_init, 1 = hit in h.
// emask: elements 0..63 whose bit is clear are skipped (their box cannot meet the ray segment
// searched; soft_light's occluder mask); elements from 64 on are always tested.
template <uint32_t KINDS = KINDS_ALL>
__device__ __forceinline__ int scene_intersect_b(const SceneView &S, V org, V dir, Hit &h,
                                                 double t_init, double t_exit, int hint = -1,
                                                 uint64_t emask = ~0ull) {
  double closest = t_init;  // world-frame t (rigid transforms keep t; scale handled below)
  bool found = false;
  V hp = mk(0, 0, 0), hn = mk(0, 0, 0);
  int hnode = 0, hmat = -1, htri = -1;
  for (int ni = 0; ni < S.nnodes; ni++) {
    const DNode &nd = S.nodes[ni];
    if (nd.elem_count == 0) continue;
    // local ray: apply the chain root -> node
    V lo = org, ldir = dir;
    double scale = 1.0;
    bool ok = true;
    for (int k = 0; k < nd.depth; k++) {
      const DNode &a = S.nodes[nd.chain[k]];
      double lv;
      if (a.identity) {
        lv = len(ldir);
        ldir = normalize(ldir);
      } else {
        lv = len(xf_vec(a.T, ldir));
        lo = xf_point(a.Tinv, lo);
        ldir = normalize(xf_vec(a.Tinv, ldir));
      }
      if (isNegOrZero(lv)) { ok = false; break; }
      if (!isZero(lv - 1.0)) scale *= lv;
    }
    if (!ok) continue;
    // the pretest's slab reciprocals only when it runs (a wave-uniform flag: hard-light scenes
    // skip three fp64 divisions per node and ray)
    const V linv = S.elem_pretest ? mk(1.0 / ldir.x, 1.0 / ldir.y, 1.0 / ldir.z) : mk(0, 0, 0);
    for (int ei = 0; ei < nd.elem_count; ei++) {
      const int gei = nd.elem_first + ei;
      if (gei < 64 && !((emask >> gei) & 1ull)) continue;
      const DElement &el = S.elems[gei];
      double maxt = closest / scale;
      if (S.elem_pretest && !elem_maybe_hit(el, lo, linv, maxt)) continue;
      auto box_pass = [&]() -> bool {
        if (box_contains(el.bmin, el.bmax, lo)) return true;
        double bt;
        if (!ray_box(lo, ldir, el.bmin, el.bmax, &bt, nullptr)) return false;
        return !isPos(bt - maxt);
      };
      const bool shapes_first = el.shapes_first_ok != 0;
      if (!shapes_first && !box_pass()) continue;
      double ec = maxt;
      V ep = mk(0, 0, 0), en = mk(0, 0, 0);
      int etri = -1;
      for (int si = 0; si < el.shape_count; si++) {
        double t;
        V p, n;
        int st;
        if (shape_intersect<KINDS>(S, S.shapes[el.shape_first + si], lo, ldir, t, p, n, ec, hint,
                                   st)) {
          if ((t >= 0.0) && (t <= ec)) {
            ep = p;
            en = n;
            ec = t;
            etri = st;
          }
        }
      }
      if (ec == maxt) continue;
      if (shapes_first && !box_pass()) continue;
      found = true;
      closest = ec * scale;
      hp = ep;
      hn = en;
      hnode = ni;
      hmat = el.material;
      htri = etri;
      if (closest < t_exit) return 2;
    }
  }
  if (!found) return 0;
  // transform hit point / normal back to world (Q11: normal by the forward affine)
  for (int c = hnode; c >= 0; c = S.nodes[c].parent) {
    const DNode &a = S.nodes[c];
    if (!a.identity) {
      hp = xf_point(a.T, hp);
      hn = xf_vec(a.T, hn);
    }
    hn = normalize(hn);
  }
  h.p = hp;
  h.n = hn;
  h.t = closest;
  h.mat = hmat;
  h.tri = htri;
  return 1;
}

// hint: the triangle the ray leaves from (the previous hit's Hit::tri), -1 for none
template <uint32_t KINDS = KINDS_ALL>
__device__ __forceinline__ bool scene_intersect(const SceneView &S, V org, V dir, Hit &h,
                                                int hint = -1) {
  return scene_intersect_b<KINDS>(S, org, dir, h, kInf, -1.0, hint) == 1;
}

// ---------------------------------------------------------------------------------------
// Optics and sampling (utils/graphics_utils.cpp)
// ---------------------------------------------------------------------------------------
GI_HD double reflection_coeff(double ir_air, double cos_theta, double ir_mat) {  // :95-101
  double r0 = gm::pow2((ir_air - ir_mat) / (ir_air + ir_mat));
  return (r0 + (1.0 - r0) * gm::pow5((1.0 - fabs(cos_theta))));
}
GI_HD V reflective_bounce(V n, V view, double ct) {  // :104-117
  if (ct < 0) { n = -n; ct *= -1.0; }
  V perp = n * ct;
  V r = view + perp * 2.0;
  return normalize(r);
}
GI_HD V transmissive_bounce(double ir_air, V n, V view, double ct, double ir_mat) {  // :121-154
  double eta;
  if (ct < 0) {
    eta = ir_mat / ir_air;
    n = -n;
    ct *= -1.0;
  } else {
    eta = ir_air / ir_mat;
  }
  double theta = gm::acos(ct);
  double sin_phi = eta * gm::sin(theta);
  if (sin_phi < -1.0 || 1.0 < sin_phi) return reflective_bounce(n, view, ct);
  double phi = gm::asin(sin_phi);
  V par = normalize(view + n * ct);
  V refr = par * gm::tan(phi) - n;
  return normalize(refr);
}
GI_HD V rotate(V v, V axis, double theta) {  // R3Vector::Rotate, R3Vector.cpp:352-363
  double st, ct;
  gm::sincos(theta, st, ct);  // = gm::sin(theta), gm::cos(theta), one range reduction
  double d = dot(v, axis);
  V cr = cross(v, axis);
  v = v * ct;
  v = v + axis * d * (1.0 - ct);
  v = v - cr * st;
  return v;
}
GI_HD V diffuse_sample(V n, double ct, Rng &rng) {  // Diffuse_ImportanceSample :162-185
  if (ct < 0) n = -n;
  double theta = gm::acos(sqrt(rng.next()));
  double phi = 2 * kPi * rng.next();
  V perp = mk(n.y, -n.x, 0);
  if (1.0 - fabs(n.z) < 0.1) perp = mk(n.z, 0, -n.x);
  perp = normalize(perp);
  double st, ctt;
  gm::sincos(theta, st, ctt);
  V r = perp * st + n * ctt;
  r = rotate(r, n, phi);
  return normalize(r);
}
GI_HD V specular_sample(V ex, double nsh, double ct, Rng &rng) {  // :189-216
  double lim = (1.0 - gm::acos(fabs(ct)) * 2.0 / kPi);
  double alpha = gm::acos(gm::pow(rng.next(), 1.0 / (nsh + 1.0))) * lim;
  double phi = 2.0 * kPi * rng.next();
  V perp = mk(ex.y, -ex.x, 0);
  if (1.0 - fabs(ex.z) < 0.1) perp = mk(ex.z, 0, -ex.x);
  perp = normalize(perp);
  double sa, ca;
  gm::sincos(alpha, sa, ca);
  V r = perp * sa + ex * ca;
  r = rotate(r, ex, phi);
  return normalize(r);
}

// ---------------------------------------------------------------------------------------
// Direct illumination (utils/illumination_utils.cpp, R3*Light::Reflection)
// ---------------------------------------------------------------------------------------
struct Flags {  // the rendering globals a kernel needs (photonmap.cpp:40-106)
  int32_t ambient, direct, transmissive, specular, indirect, caustic, photon_viz, fast_global;
  int32_t cache, shadows, soft_shadows, light_test, shadow_test, monte_carlo, max_monte_depth;
  int32_t recursive_shadows, distrib_trans, trans_test, distrib_spec, spec_test, fresnel;
  int32_t indirect_test, dof, dof_test, max_photon_depth, pad;
  double ir_air, prob_absorb;
  uint64_t seed;
};

struct Counts {  // per-thread -v counters (render.cpp:26-32)
  uint32_t shadow, monte, trans, spec, indirect, caustic;
};

// RayIlluminationTest, illumination_utils.cpp:16-31 (Q13 distance equality).
// The verdict only needs the closest hit near unocc: a hit farther than unocc + 1e-6 leaves the
// point unlit whatever lies beyond it (so the search starts at that bound), and once any hit is
// taken below unocc - 1e-6 the final one is nearer still (so the walk stops there). The margins
// (1e-8 relative) cover the rounding between the walk's t and the distance of the transformed
// hit point. The no-hit case keeps the reference's l = RN_INFINITY.
template <uint32_t KINDS = KINDS_ALL>
__device__ __forceinline__ bool illum_test_inl(const SceneView &S, V p_scene, V p_light, Counts &cnt,
                                               uint64_t emask = ~0ull) {
  double unocc = dist(p_light, p_scene);
  V d = normalize(p_scene - p_light);
  Hit h;
  // (only in scenes of rigid transforms: under a scaling node R3SceneNode's t rescale,
  // R3SceneNode.cpp:449-458, is not the hit's distance, so no bound is derived from it)
  const double mg = 1e-8 * fmax(1.0, unocc);
  const int r = S.rigid ? scene_intersect_b<KINDS>(S, p_light, d, h, fmin(kInf, unocc + kEps + mg),
                                                   unocc - kEps - mg, -1, emask)
                        : scene_intersect_b<KINDS>(S, p_light, d, h, kInf, -1.0);
  cnt.shadow++;
  if (r == 2) return false;
  double l = (r == 1) ? dist(p_light, h.p) : kInf;
  return fabs(l - unocc) < kEps;
}
template <uint32_t KINDS = KINDS_ALL>
__device__ __noinline__ bool illum_test(const SceneView &S, V p_scene, V p_light, Counts &cnt,
                                        uint64_t emask = ~0ull) {
  return illum_test_inl<KINDS>(S, p_scene, p_light, cnt, emask);
}

// TestLightIntersection, illumination_utils.cpp:35-84
GI_HD int light_self_test(V p, V eye, const DLight &L) {
  if (L.kind == LK_AREA) {
    V v = p - ld3(L.pos);
    double vl = len(v);
    v = normalize(v);
    V nn = ld3(L.dir);
    if (fabs(dot(v, nn)) < kEps && vl <= L.radius) return (dot(nn, eye - p) <= 0) ? -1 : 1;
  } else if (L.kind == LK_RECT) {
    V v = p - ld3(L.pos);
    double c1 = dot(v, ld3(L.a1)), c2 = dot(v, ld3(L.a2));
    v = normalize(v);
    V nn = ld3(L.dir);
    if (fabs(dot(v, nn)) < kEps && fabs(c1 * 2.0) <= L.len1 && fabs(c2 * 2.0) <= L.len2)
      return (dot(nn, eye - p) <= 0) ? -1 : 1;
  }
  return 0;
}

// sample a point on an area (disk, rejection) or rect light (illumination_utils.cpp:150-157,
// 315-319): ((r1*u + r2*v) + center) + n*eps
GI_HD V light_sample_point(const DLight &L, Rng &rng) {
  double r1, r2;
  if (L.kind == LK_AREA) {
    do {
      r1 = (rng.next() * 2.0) - 1.0;
      r2 = (rng.next() * 2.0) - 1.0;
    } while (r1 * r1 + r2 * r2 > 1.0);
  } else {
    r1 = rng.next() - 0.5;
    r2 = rng.next() - 0.5;
  }
  return ((r1 * ld3(L.su) + r2 * ld3(L.sv)) + ld3(L.pos)) + ld3(L.dir) * kEps;
}

// Occluder mask of the shadow rays between p and light L's samples (rigid scenes of <= 64
// elements): bit e clear when element e is in world coordinates and its box cannot meet any
// segment from a sample point to p. Every sample lies in the light's parallelogram (offset by
// kEps along its normal) and every searched segment in the convex hull of that and p, extended
// past p by kEps + 1e-8 (illum_test_inl's bound), so it lies inside the hull's bounding box
// grown by the margin below; an element box disjoint from that box fails R3Intersects(ray, box)
// (every slab interval or the containment test excludes it, with room for their rounding and the
// 1e-6 tolerance of box_contains), and scene_intersect_b takes no element whose box test fails.
// Same result as testing every element.
__device__ __forceinline__ uint64_t occluder_mask(const SceneView &S, const DLight &L, V p) {
  if (!S.rigid || S.nelems > 64) return ~0ull;
  const double h = (L.kind == LK_AREA) ? 1.0 : 0.5;  // sample coefficients in [-h, h]
  const V c = ld3(L.pos) + ld3(L.dir) * kEps, u = ld3(L.su) * h, v = ld3(L.sv) * h;
  double lo[3] = {p.x, p.y, p.z}, hi[3] = {p.x, p.y, p.z};
  for (int k = 0; k < 4; k++) {
    const V q = c + u * ((k & 1) ? 1.0 : -1.0) + v * ((k & 2) ? 1.0 : -1.0);
    const double qq[3] = {q.x, q.y, q.z};
    for (int i = 0; i < 3; i++) {
      lo[i] = fmin(lo[i], qq[i]);
      hi[i] = fmax(hi[i], qq[i]);
    }
  }
  double ext = 0.0;
  for (int i = 0; i < 3; i++) ext = fmax(ext, fmax(fabs(lo[i]), fabs(hi[i])));
  const double mg = 1e-4 + 1e-6 * ext;
  uint64_t m = 0ull;
  for (int e = 0; e < S.nelems; e++) {
    const DElement &el = S.elems[e];
    bool overlap = true;
    for (int i = 0; i < 3; i++)
      if (el.pmax[i] < lo[i] - mg || el.pmin[i] > hi[i] + mg) overlap = false;
    if (!el.world || overlap) m |= 1ull << e;
  }
  return m;
}

// ComputeAreaLightReflection / ComputeRectLightReflection, illumination_utils.cpp:91-417
// (Q1: the whole accumulated colour is scaled by the shadow hit rate)
template <uint32_t KINDS = KINDS_ALL>
__device__ __noinline__ void soft_light(const SceneView &S, const DLight &L, C3 &color,
                                        const DMaterial &m, V eye, V p, V nrm, int nls, int nes,
                                        Rng &rng, Counts &cnt) {
  if (!L.active) return;
  V center = ld3(L.pos), ln = ld3(L.dir);
  if (dot(ln, p - center) < 0) return;
  // (a fan of a few shadow rays, as in a Monte Carlo path's 2 samples, does not repay the mask)
  const uint64_t em = (nls + nes >= 16) ? occluder_mask(S, L, p) : ~0ull;
  int tot_s = 0, tot_h = 0;
  if (m.flags & MF_DIFFUSE) {
    double w = 0;
    int hits = 0;
    for (int i = 0; i < nls; i++) {
      V sp = light_sample_point(L, rng);
      if (illum_test<KINDS>(S, p, sp, cnt, em)) {
        hits++;
        double I = L.intensity;
        double dd = dist(p, sp);
        double den = L.ca;
        den += dd * L.la;
        den += dd * dd * L.qa;
        if (isPos(den)) I /= den;
        V Ld = normalize(sp - p);
        I *= dot(ln, -Ld) * 2.0;
        w += I * fabs(dot(nrm, Ld));
      }
    }
    if (hits > 0) color += w * ldc(m.kd) * ldc(L.color) * L.area / (double)hits;
    tot_h += hits;
    tot_s += nls;
  }
  if (m.flags & MF_SPECULAR) {
    double w = 0;
    int hits = 0;
    int n2 = nls * 2;
    V Vv = normalize(eye - p);
    for (int i = 0; i < n2; i++) {
      V sp = light_sample_point(L, rng);
      if (illum_test<KINDS>(S, p, sp, cnt, em)) {
        hits++;
        double I = L.intensity;
        double dd = dist(p, sp);
        double den = L.ca;
        den += dd * L.la;
        den += dd * dd * L.qa;
        if (isPos(den)) I /= den;
        V Ld = normalize(sp - p);
        I *= dot(ln, -Ld) * 2.0;
        double NL = dot(nrm, Ld);
        V R = (2.0 * NL) * nrm - Ld;
        double VR = dot(Vv, R);
        if (isNegOrZero(VR)) continue;
        w += (I * pow_ool(VR, m.n));
      }
    }
    if (hits > 0) color += w * ldc(m.ks) * ldc(L.color) * L.area / (double)hits;
    tot_h += hits;
    tot_s += n2;
  }
  int hits = 0;
  for (int i = 0; i < nes; i++) {
    V sp = light_sample_point(L, rng);
    if (illum_test<KINDS>(S, p, sp, cnt, em)) hits++;
  }
  tot_h += hits;
  tot_s += nes;
  if (tot_s > 0) color *= ((double)tot_h) / tot_s;
}

// Light::Reflection: point/spot (R3PointLight.cpp:213-244, IntensityAtPoint :111-121,
// R3SpotLight.cpp:105-115), directional (R3DirectionalLight.cpp:134-166), area/rect without
// shadows (R3AreaLight.cpp:122-330, R3RectLight.cpp:150-340)
// the point/spot/directional part (no sampling), also inlined by the hard-light path
__device__ __forceinline__ C3 light_reflection_hard(const DLight &L, const DMaterial &m, V eye, V p,
                                                    V nrm) {
  C3 Dc = ldc(m.kd), Sc = ldc(m.ks), Ic = ldc(L.color);
  double s = m.n;
  if (L.kind == LK_POINT || L.kind == LK_SPOT) {
    V lp = ld3(L.pos);
    double dd = dist(p, lp);
    double den = L.ca;
    den += dd * L.la;
    den += dd * dd * L.qa;
    double I = isZero(den) ? L.intensity : (L.intensity / den);
    if (L.kind == LK_SPOT) {
      V ML = normalize(p - lp);
      double ca = dot(ML, ld3(L.dir));
      if (gm::cos(L.cutoff) > ca) I = 0.0;
      else I = I * pow_ool(ca, L.dropoff);
    }
    V Ld = normalize(lp - p);
    double NL = dot(nrm, Ld);
    V R = (2.0 * NL) * nrm - Ld;
    V Vv = normalize(eye - p);
    double VR = dot(Vv, R);
    C3 o = I * Dc * Ic * fabs(NL);
    if (isPos(VR)) o += (I * pow_ool(VR, s)) * Sc * Ic;
    return o;
  }
  if (L.kind == LK_DIR) {
    double I = L.intensity;
    V Ld = -ld3(L.dir);
    double NL = dot(nrm, Ld);
    V R = (2.0 * NL) * nrm - Ld;
    V Vv = normalize(eye - p);
    double VR = dot(Vv, R);
    C3 o = (I * fabs(NL)) * Dc * Ic;
    if (isPos(VR)) o += (I * pow_ool(VR, s) * Sc * Ic);
    return o;
  }
  return rgb(0, 0, 0);
}

__device__ __noinline__ C3 light_reflection(const DLight &L, const DMaterial &m, V eye, V p,
                                            V nrm, int max_samples, Rng &rng) {
  if (!L.active) return rgb(0, 0, 0);
  if (L.kind == LK_POINT || L.kind == LK_SPOT || L.kind == LK_DIR)
    return light_reflection_hard(L, m, eye, p, nrm);
  C3 Dc = ldc(m.kd), Sc = ldc(m.ks), Ic = ldc(L.color);
  double s = m.n;
  bool area = (L.kind == LK_AREA);
  V dirn = ld3(L.dir), center = ld3(L.pos);
  if (dot(dirn, p - center) < 0) return rgb(0, 0, 0);
  V ax1 = ld3(L.nr_ax1), ax2 = ld3(L.nr_ax2);
  C3 out = rgb(0, 0, 0);
  for (int pass = 0; pass < 2; pass++) {
    bool spec = (pass == 1);
    int count = 0;
    C3 sum = rgb(0, 0, 0);
    int target = spec ? 2 * max_samples : max_samples;
    for (int i = 0; (spec ? i < target : count < target); i++) {
      double r1, r2;
      if (area) {
        r1 = (rng.next() * 2.0) - 1.0;
        r2 = (rng.next() * 2.0) - 1.0;
        if (r1 * r1 + r2 * r2 > 1) continue;
      } else {
        r1 = rng.next() - 0.5;
        r2 = rng.next() - 0.5;
      }
      V sp = center;
      sp = sp + r1 * ax1;
      sp = sp + r2 * ax2;
      count++;
      double I = L.intensity;
      double dd = dist(p, sp);
      double den = L.ca;
      den += dd * L.la;
      den += dd * dd * L.qa;
      if (isPos(den)) I /= den;
      V Ld = normalize(sp - p);
      I *= dot(dirn, -Ld) * 2.0;
      double NL = dot(nrm, Ld);
      if (!spec) {
        sum += (I * fabs(NL)) * Dc * Ic;
      } else {
        V R = (2.0 * NL) * nrm - Ld;
        V Vv = normalize(eye - p);
        double VR = dot(Vv, R);
        if (isNegOrZero(VR)) continue;
        sum += (I * pow_ool(VR, s) * Sc * Ic);
      }
    }
    C3 mean = sum;
    if (count > 0) mean = mean / (double)count;
    out += L.area * mean;
  }
  return out;
}

// ComputeIllumination, illumination_utils.cpp:425-494
template <uint32_t KINDS = KINDS_ALL>
__device__ __noinline__ void compute_illumination(const SceneView &S, const Flags &F, C3 &color,
                                                  const DLight &L, const DMaterial &m, V eye,
                                                  V p, V nrm, double ct, bool inMC, Rng &rng,
                                                  Counts &cnt) {
  bool shadows = F.shadows && (!inMC || (F.recursive_shadows && inMC));
  int nls = F.light_test, nes = F.shadow_test;
  if (inMC) { nls = 2; nes = 0; }  // Q14
  if (!shadows) {
    color += light_reflection(L, m, eye, p, nrm, nls, rng);
    return;
  }
  V pol;
  if (L.kind == LK_DIR) {
    pol = p - ld3(L.dir) * S.radius * 3.0;
  } else if (L.kind == LK_POINT || L.kind == LK_SPOT) {
    pol = ld3(L.pos);
  } else {
    if (!F.soft_shadows) {
      pol = ld3(L.pos) + kEps * ld3(L.dir);
    } else {
      soft_light<KINDS>(S, L, color, m, eye, p, nrm, nls, nes, rng, cnt);
      return;
    }
  }
  double side = dot(nrm, pol - p);
  if ((side > 0 && ct < 0) || (side < 0 && ct > 0)) return;
  if (illum_test<KINDS>(S, p, pol, cnt)) color += light_reflection(L, m, eye, p, nrm, nls, rng);
}

// DirectIllumination, raytracer.cpp:18-44
template <uint32_t KINDS = KINDS_ALL>
__device__ __noinline__ void direct_illumination(const SceneView &S, const Flags &F, V p, V nrm,
                                                 V eye, C3 &color, const DMaterial &m, double ct,
                                                 bool inMC, Rng &rng, Counts &cnt) {
  bool emit = true;
  for (int k = 0; k < S.nlights; k++) {
    const DLight &L = S.lights[k];
    int li = light_self_test(p, eye, L);
    if (li != 0) {
      if (li == -1) emit = false;
      continue;
    }
    compute_illumination<KINDS>(S, F, color, L, m, eye, p, nrm, ct, inMC, rng, cnt);
  }
  if (emit) color += ldc(m.e);
}

// DirectIllumination for scenes whose lights are all point/spot/directional (SceneView::
// hard_lights), inlined: no light sampling, so no calls, and the caller's registers are not
// spilled around them. Same operations as direct_illumination -> compute_illumination ->
// illum_test / light_reflection for those light kinds (TestLightIntersection is 0 for them).
// (r05: the shadow walk out of line where the scene has boxes or meshes cut mc_kernel's spills
// 48 -> 20 VGPRs but ran slower, C4 shard 0/8 5,862 -> 6,271 ms; removed)
template <uint32_t KINDS = KINDS_ALL>
__device__ __forceinline__ void direct_illumination_hard(const SceneView &S, const Flags &F, V p,
                                                         V nrm, V eye, C3 &color,
                                                         const DMaterial &m, double ct, bool inMC,
                                                         Counts &cnt) {
  bool shadows = F.shadows && (!inMC || (F.recursive_shadows && inMC));
  for (int k = 0; k < S.nlights; k++) {
    const DLight &L = S.lights[k];
    if (!shadows) {
      if (L.active) color += light_reflection_hard(L, m, eye, p, nrm);
      continue;
    }
    V pol = (L.kind == LK_DIR) ? p - ld3(L.dir) * S.radius * 3.0 : ld3(L.pos);
    double side = dot(nrm, pol - p);
    if ((side > 0 && ct < 0) || (side < 0 && ct > 0)) continue;
    if (illum_test_inl<KINDS>(S, p, pol, cnt) && L.active)
      color += light_reflection_hard(L, m, eye, p, nrm);
  }
  color += ldc(m.e);
}

}  // namespace gi
