// oracle_scene.cpp -- TEST INFRASTRUCTURE ONLY (checker, never part of the product).
// Restates the reference's .scn/.off loaders and scene-graph ray intersection.
#include "oracle_scene.h"
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <cctype>
#include <map>
#include <array>

namespace oracle {

// R4Matrix::Invert-equivalent (Gauss-Jordan with partial pivoting)
M4 M4::inverse() const {
  double a[4][8];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) a[i][j] = (j < 4) ? m[i][j] : ((j - 4 == i) ? 1.0 : 0.0);
  for (int c = 0; c < 4; c++) {
    int p = c;
    for (int r = c + 1; r < 4; r++)
      if (fabs(a[r][c]) > fabs(a[p][c])) p = r;
    if (p != c)
      for (int j = 0; j < 8; j++) { double t = a[c][j]; a[c][j] = a[p][j]; a[p][j] = t; }
    double d = a[c][c];
    for (int j = 0; j < 8; j++) a[c][j] /= d;
    for (int r = 0; r < 4; r++) {
      if (r == c) continue;
      double f = a[r][c];
      if (f == 0.0) continue;
      for (int j = 0; j < 8; j++) a[r][j] -= f * a[c][j];
    }
  }
  M4 out;
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) out.m[i][j] = a[i][j + 4];
  return out;
}

// R3Triangle::Update (R3Triangle.cpp:476-485): plane through the three vertices
Tri make_tri(V3 a, V3 b, V3 c) {
  Tri t;
  t.p[0] = a; t.p[1] = b; t.p[2] = c;
  V3 v = cross(b - a, c - a);  // R3Plane(p1,p2,p3), R3Plane.cpp
  v = normalize(v);
  t.n = v;
  t.d = -(v.x * a.x + v.y * a.y + v.z * a.z);
  t.box.add(a); t.box.add(b); t.box.add(c);
  return t;
}

// R3Contains(box, point), R3Cont.cpp:776-787
static bool box_contains(const Box &b, V3 p) {
  if (b.empty()) return false;
  for (int i = 0; i < 3; i++) {
    if (isNeg(p[i] - b.mn[i])) return false;
    if (isPos(p[i] - b.mx[i])) return false;
  }
  return true;
}

// R3Intersects(ray, box), R3Isect.cpp:883-942. Returns 1 on hit (R3_SPAN_CLASS_ID).
int ray_box(V3 org, V3 dir, const Box &box, double *hit_t, V3 *hit_normal) {
  if (box.empty()) return 0;
  bool start_inside = box_contains(box, org);
  for (int dim = 0; dim < 3; dim++) {
    double tval;
    if (isPos(dir[dim])) {
      double bc = start_inside ? box.mx[dim] : box.mn[dim];
      double delta = bc - org[dim];
      if (delta < 0.0) continue;
      tval = delta / dir[dim];
    } else if (isNeg(dir[dim])) {
      double bc = start_inside ? box.mn[dim] : box.mx[dim];
      double delta = bc - org[dim];
      if (delta > 0.0) continue;
      tval = delta / dir[dim];
    } else {
      continue;
    }
    int d1 = (dim + 1) % 3, d2 = (dim + 2) % 3;
    V3 p;
    p[dim] = org[dim] + dir[dim] * tval;
    p[d1] = org[d1] + dir[d1] * tval;
    p[d2] = org[d2] + dir[d2] * tval;
    if (isNegOrZero(p[d1] - box.mx[d1]) && isPosOrZero(p[d1] - box.mn[d1]) &&
        isNegOrZero(p[d2] - box.mx[d2]) && isPosOrZero(p[d2] - box.mn[d2])) {
      if (hit_t) *hit_t = tval;
      if (hit_normal) {
        V3 ax(0, 0, 0);
        ax[dim] = 1.0;
        *hit_normal = isNeg(dir[dim]) ? ax : -ax;
      }
      return 1;
    }
  }
  return 0;
}

// R3Intersects(ray, triangle), R3Isect.cpp:700-732 (plane) + 761-796, with
// R3Contains(triangle, point), R3Cont.cpp:491-512
static bool ray_tri(V3 org, V3 dir, const Tri &tr, double &t, V3 &point) {
  double denom = dot(tr.n, dir);
  if (isZero(denom)) return false;  // parallel (in-plane case also returns NULL)
  double s = -(dot(org, tr.n) + tr.d) / denom;
  if (isNeg(s)) return false;
  V3 p = org + dir * s;
  if (!box_contains(tr.box, p)) return false;
  if (!isZero(p.x * tr.n.x + p.y * tr.n.y + p.z * tr.n.z + tr.d)) return false;
  const V3 &p0 = tr.p[0], &p1 = tr.p[1], &p2 = tr.p[2];
  // R3Plane(point, vector1, vector2): v = normalize(vector1 x vector2), d = -v.point
  V3 e[3] = {p1 - p0, p2 - p1, p0 - p2};
  V3 q[3] = {p1, p2, p0};
  for (int i = 0; i < 3; i++) {
    V3 v = normalize(cross(tr.n, e[i]));
    double d = -(v.x * q[i].x + v.y * q[i].y + v.z * q[i].z);
    if (isNeg(p.x * v.x + p.y * v.y + p.z * v.z + d)) return false;
  }
  t = s;
  point = p;
  return true;
}

// R3Intersects(ray, sphere), R3Isect.cpp:975-1021 (+ R3Contains(sphere), R3Cont.cpp:1056-1063)
static bool ray_sphere(V3 org, V3 dir, V3 c, double r, double &t, V3 &point, V3 &normal) {
  V3 v0 = c - org;
  double r2 = r * r;
  double d2 = v0.x * v0.x + v0.y * v0.y + v0.z * v0.z;
  bool start_inside = isNegOrZero(d2 - r2);
  double v = dot(v0, dir);
  if (!start_inside && isNegOrZero(v)) return false;
  double disc = r2 - (dot(v0, v0) - v * v);
  if (isNeg(disc)) return false;
  double d = sqrt(disc);
  t = start_inside ? v + d : v - d;
  point = org + t * dir;
  normal = (point - c) / r;
  return true;
}

// R3Intersects(ray, circle), R3Isect.cpp:837-879
static bool ray_circle(V3 org, V3 dir, V3 c, V3 n, double r, double &t, V3 &point) {
  if (r < 0) return false;
  double pd = -(n.x * c.x + n.y * c.y + n.z * c.z);
  double denom = dot(n, dir);
  if (isZero(denom)) return false;  // in-plane case: reference returns SPAN with no t
  double s = -(dot(org, n) + pd) / denom;
  if (isNeg(s)) return false;
  V3 p = org + dir * s;
  V3 v = c - p;
  double dd = v.x * v.x + v.y * v.y + v.z * v.z;
  if (isPos(dd - r * r)) return false;
  t = s;
  point = p;
  return true;
}

// R3Cylinder::BBox (R3Cylinder.cpp:175-181): union of the cap circles' boxes, each the cube
// centre +- radius (R3Circle.cpp:179-184)
static void cap_cubes_box(Shape &sh) {
  for (int i = 0; i < 3; i++) {
    sh.box.mn[i] = fmin(sh.c[i] - sh.r, sh.axis[i] - sh.r);
    sh.box.mx[i] = fmax(sh.c[i] + sh.r, sh.axis[i] + sh.r);
  }
}

// R3Intersects(ray, plane, NULL, &t), R3Isect.cpp:700-732. A ray lying in the plane counts as
// an intersection and leaves t unchanged (the caller's cap_t stays at its initial 0).
static bool ray_plane_t(V3 o, V3 d, V3 n, double pd, double &t) {
  double denom = dot(n, d);
  double sd = o.x * n.x + o.y * n.y + o.z * n.z + pd;  // R3SignedDistance, R3Dist.cpp:603-607
  if (isZero(denom)) return isZero(sd);
  double s = -(sd) / denom;
  if (isNeg(s)) return false;
  t = s;
  return true;
}

// R3Intersects(ray, R3Cylinder), R3Isect.cpp:1025-1200 (Graphics Gems IV p.356) for the
// cylinder p1 -> p2 (axis R3Span: unit vector, R3Span.cpp:63-70), radius r; caps are the
// planes through p1 (normal -A) and p2 (normal +A) (R3Cylinder.cpp constructors,
// R3Circle.cpp:78-83, R3Plane.cpp:85-90).
static bool ray_cylinder(V3 o, V3 R, V3 p1, V3 p2, double radius, double &t_out, V3 &p_out,
                         V3 &n_out) {
  const double INF = 1.0e6;  // RN_INFINITY
  V3 A = p2 - p1;
  double alen = length(A);
  if (!isZero(alen)) A = A / alen;
  V3 nT = A, nB = -A;
  double dT = -(nT.x * p2.x + nT.y * p2.y + nT.z * p2.z);
  double dB = -(nB.x * p1.x + nB.y * p1.y + nB.z * p1.z);
  double cyl_t1, cyl_t2;
  V3 D = cross(R, A);
  double a = length(D);
  if (isZero(a)) {
    // parallel: R3Distance(point, line), R3Dist.cpp:59-65
    double d = length(cross(A, p1 - o));
    if (!isNegOrZero(d - radius)) return false;
    cyl_t1 = 0.0;
    cyl_t2 = INF;
  } else {
    D = D / a;
    V3 RC = o - p1;
    double d = dot(RC, D);
    if (d < 0.0) d = -d;
    if (isPos(d - radius)) return false;
    double t = dot(cross(RC, A), D) / -a;
    double s;
    V3 O = normalize(cross(D, A));
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
  V3 HB = p_out - p1;
  n_out = (HB - dot(HB, A) * A) / radius;
  return true;
}

// R3Shape::Intersects virtual dispatch (R3Shape.cpp:328-329 -> R3Isect.cpp)
static bool shape_intersect(const Shape &sh, V3 org, V3 dir, double &t, V3 &point, V3 &normal) {
  switch (sh.type) {
    case SH_TRI:
      if (!ray_tri(org, dir, sh.tri, t, point)) return false;
      normal = sh.tri.n;
      return true;
    case SH_MESH: {
      // R3Intersects(ray, R3TriangleArray), R3Isect.cpp:800-833: bbox, then min t over ALL
      // triangles (t may be in [-1e-6, 0): quirk Q2, rejected later by the element)
      if (!ray_box(org, dir, sh.box, nullptr, nullptr)) return false;
      bool found = false;
      double min_t = FLT_MAX;
      for (const Tri &tr : sh.tris) {
        double tt;
        V3 pp;
        if (ray_tri(org, dir, tr, tt, pp)) {
          if (tt < min_t) {
            found = true;
            point = pp;
            normal = tr.n;
            min_t = tt;
          }
        }
      }
      t = min_t;
      return found;
    }
    case SH_SPHERE:
      return ray_sphere(org, dir, sh.c, sh.r, t, point, normal);
    case SH_BOX: {
      double tt;
      V3 nn;
      if (!ray_box(org, dir, sh.box, &tt, &nn)) return false;
      t = tt;
      point = org + dir * tt;
      // R3Isect.cpp:914-916 recomputes the point per coordinate; same expression
      normal = nn;
      return true;
    }
    case SH_CIRCLE:
      if (!ray_circle(org, dir, sh.c, sh.axis, sh.r, t, point)) return false;
      normal = sh.axis;
      return true;
    case SH_CYLINDER:
      return ray_cylinder(org, dir, sh.c, sh.axis, sh.r, t, point, normal);
    default:
      return false;  // cone: used by no input scene
  }
}

// R3SceneElement::Intersects, R3SceneElement.cpp:209-243
static bool element_intersect(const Element &el, V3 org, V3 dir, double min_t, double max_t,
                              double &t_out, V3 &p_out, V3 &n_out) {
  double bbox_t;
  if (!box_contains(el.bbox, org)) {
    if (!ray_box(org, dir, el.bbox, &bbox_t, nullptr)) return false;
    if (isPos(bbox_t - max_t)) return false;
  }
  double closest_t = max_t;
  for (const Shape &sh : el.shapes) {
    double t;
    V3 p, n;
    if (shape_intersect(sh, org, dir, t, p, n)) {
      if ((t >= min_t) && (t <= closest_t)) {
        p_out = p;
        n_out = n;
        t_out = t;
        closest_t = t;
      }
    }
  }
  return !(closest_t == max_t);
}

// R3SceneNode::Intersects, R3SceneNode.cpp:420-510
static bool node_intersect(const Scene &s, int ni, V3 org, V3 dir, double min_t, double max_t,
                           Hit &h) {
  const Node &nd = s.nodes[ni];
  double bbox_t;
  if (!box_contains(nd.bbox, org)) {
    if (!ray_box(org, dir, nd.bbox, &bbox_t, nullptr)) return false;
    if (isPos(bbox_t - max_t)) return false;
  }
  // R3Ray::InverseTransform -> R3Line::InverseTransform (R3Line.cpp:140-146)
  V3 norg = nd.Tinv.point(org);
  V3 ndir = normalize(nd.Tinv.vec(dir));
  double scale = 1.0;
  double length_v = length(nd.T.vec(dir));
  if (isNegOrZero(length_v)) return false;
  double closest_t = max_t;
  if (!isZero(length_v - 1.0)) {
    scale = length_v;
    min_t /= scale;
    closest_t /= scale;
  }
  bool found = false;
  V3 cp, cn;
  int cmat = -1;
  for (const Element &el : nd.elements) {
    double t;
    V3 p, n;
    if (element_intersect(el, norg, ndir, min_t, closest_t, t, p, n)) {
      if ((t >= min_t) && (t <= closest_t)) {
        found = true;
        cp = p; cn = n; cmat = el.material; closest_t = t;
      }
    }
  }
  for (int ci : nd.children) {
    Hit ch;
    if (node_intersect(s, ci, norg, ndir, min_t, closest_t, ch)) {
      if ((ch.t >= min_t) && (ch.t <= closest_t)) {
        found = true;
        cp = ch.point; cn = ch.normal; cmat = ch.material; closest_t = ch.t;
      }
    }
  }
  if (!found) return false;
  h.point = nd.T.point(cp);
  h.t = scale * closest_t;
  h.normal = normalize(nd.T.vec(cn));  // Q11: forward affine, not inverse transpose
  h.material = cmat;
  return true;
}

bool scene_intersect(const Scene &s, V3 org, V3 dir, Hit &h) {
  return node_intersect(s, 0, org, dir, 0.0, RN_INF, h);
}

// ---------------------------------------------------------------------------------------
// Loader
// ---------------------------------------------------------------------------------------

// R3Mesh::ReadOffFile (R3Mesh.cpp:4075-4210) with CreateFace's half-edge rule
// (R3Mesh.cpp:1135-1196): a face whose directed edge is already used is deferred and then
// re-created as (v1,v2,v3), (v1,v3,v2) or with duplicated vertices.
static bool read_off(const std::string &path, std::vector<Tri> &tris, std::string &err) {
  FILE *fp = fopen(path.c_str(), "r");
  if (!fp) { err = "Unable to open file " + path; return false; }
  int nverts = 0, nfaces = 0, nedges = 0, vcount = 0, fcount = 0;
  char buffer[1024], header[64];
  std::vector<V3> verts;
  struct EdgeRec { int v0; bool f0, f1; };
  std::map<std::pair<int, int>, EdgeRec> edges;
  std::vector<std::array<int, 3>> faces;
  std::vector<std::array<int, 3>> deferred;
  auto edge = [&](int a, int b) -> EdgeRec & {
    auto key = std::make_pair(a < b ? a : b, a < b ? b : a);
    auto it = edges.find(key);
    if (it == edges.end()) it = edges.emplace(key, EdgeRec{a, false, false}).first;
    return it->second;
  };
  auto create_face = [&](int a, int b, int c) -> bool {
    EdgeRec &e1 = edge(a, b);
    EdgeRec &e2 = edge(b, c);
    EdgeRec &e3 = edge(c, a);
    if ((e1.v0 == a && e1.f0) || (e1.v0 == b && e1.f1)) return false;
    if ((e2.v0 == b && e2.f0) || (e2.v0 == c && e2.f1)) return false;
    if ((e3.v0 == c && e3.f0) || (e3.v0 == a && e3.f1)) return false;
    if (e1.v0 == a) e1.f0 = true; else e1.f1 = true;
    if (e2.v0 == b) e2.f0 = true; else e2.f1 = true;
    if (e3.v0 == c) e3.f0 = true; else e3.f1 = true;
    faces.push_back({a, b, c});
    return true;
  };
  while (fgets(buffer, 1023, fp)) {
    char *bp = buffer;
    while (isspace((unsigned char)*bp)) bp++;
    if (*bp == '#' || *bp == '\0') continue;
    if (nverts == 0) {
      if (strstr(bp, "OFF")) {
        int tmp;
        if (sscanf(bp, "%63s%d%d%d", header, &tmp, &nfaces, &nedges) == 4) nverts = tmp;
      } else if (sscanf(bp, "%d%d%d", &nverts, &nfaces, &nedges) != 3 || nverts == 0) {
        err = "Syntax error reading header in file " + path;
        fclose(fp);
        return false;
      }
    } else if (vcount < nverts) {
      double x, y, z;
      if (sscanf(bp, "%lf%lf%lf", &x, &y, &z) != 3) {
        err = "Syntax error with vertex coordinates in file " + path;
        fclose(fp);
        return false;
      }
      verts.push_back(V3(x, y, z));
      vcount++;
    } else if (fcount < nfaces) {
      char *tok = strtok(bp, " \t");
      int fn = tok ? atoi(tok) : 0;
      if (!tok) { err = "Syntax error with face in file " + path; fclose(fp); return false; }
      int v1 = -1, v2 = -1, v3 = -1;
      for (int i = 0; i < fn; i++) {
        tok = strtok(NULL, " \t");
        if (!tok) { err = "Syntax error with face in file " + path; fclose(fp); return false; }
        int v = atoi(tok);
        if (v1 < 0) v1 = v; else v3 = v;
        if (v1 >= 0 && v2 >= 0 && v3 >= 0 && v1 != v2 && v2 != v3 && v1 != v3) {
          if (!create_face(v1, v2, v3)) deferred.push_back({v1, v2, v3});
        }
        v2 = v3;
      }
      fcount++;
    } else {
      break;
    }
  }
  fclose(fp);
  for (auto &f : deferred) {
    if (!create_face(f[0], f[1], f[2]))
      if (!create_face(f[0], f[2], f[1])) {
        int n0 = (int)verts.size();
        verts.push_back(verts[f[0]]);
        verts.push_back(verts[f[1]]);
        verts.push_back(verts[f[2]]);
        create_face(n0, n0 + 1, n0 + 2);
      }
  }
  for (auto &f : faces) {
    if (f[0] >= (int)verts.size() || f[1] >= (int)verts.size() || f[2] >= (int)verts.size()) {
      err = "bad vertex index in " + path;
      return false;
    }
    tris.push_back(make_tri(verts[f[0]], verts[f[1]], verts[f[2]]));
  }
  return true;
}

static std::string dir_of(const std::string &f) {
  size_t p = f.rfind('/');
  return (p == std::string::npos) ? std::string() : f.substr(0, p + 1);
}

// FindPrincetonMaterialAndElement, R3Scene.cpp:1401-1441: shapes are grouped per node into
// one element per distinct material, in first-use order; m < 0 uses the group's default
// material (created from R3default_brdf on first use, R3Brdf.cpp:13-15).
static bool find_element(Scene &s, int node, int m, int &group_material, int &cur_material,
                         Element *&el) {
  int mat;
  if (m >= 0) {
    // materials index: parsed materials are numbered from 1 in Scene::materials? no:
    // Scene::materials holds parsed materials in order, plus lazily created defaults.
    mat = m;  // resolved by caller through parsed index table
  } else {
    mat = group_material;
    if (mat < 0) {
      Brdf d;  // R3default_brdf
      d.ka = Rgb(0.2, 0.2, 0.2); d.kd = Rgb(0.8, 0.8, 0.8);
      d.ks = Rgb(0, 0, 0); d.kt = Rgb(0, 0, 0); d.e = Rgb(0, 0, 0);
      d.n = 0.2; d.ir = 1.0;
      s.materials.push_back(d);
      mat = (int)s.materials.size() - 1;
      group_material = mat;
    }
  }
  cur_material = mat;
  Node &nd = s.nodes[node];
  el = nullptr;
  for (auto &e : nd.elements)
    if (e.material == mat) { el = &e; break; }
  if (!el) {
    nd.elements.push_back(Element());
    el = &nd.elements.back();
    el->material = mat;
  }
  return true;
}

// ReadPrinceton, R3Scene.cpp:1446-1953
static bool read_princeton(Scene &s, int root_node, const std::string &filename, bool real,
                           std::vector<int> &parsed, std::string &err) {
  FILE *fp = fopen(filename.c_str(), "r");
  if (!fp) { err = "Unable to open file " + filename; return false; }
  int group_nodes[1024];
  int group_materials[1024];
  for (int i = 0; i < 1024; i++) { group_nodes[i] = -1; group_materials[i] = -1; }
  group_nodes[0] = root_node;
  int depth = 0;
  int cur_material = -1;
  char cmd[128];
  int command_number = 1;
  auto fail = [&](const char *what) {
    char b[512];
    snprintf(b, sizeof b, "Unable to read %s at command %d in file %s", what, command_number,
             filename.c_str());
    err = b;
    fclose(fp);
    return false;
  };
  auto resolve = [&](int m, Element *&el) -> bool {
    int mi = m;
    if (m >= 0) {
      if (m >= (int)parsed.size()) return false;
      mi = parsed[m];
    }
    return find_element(s, group_nodes[depth], mi, group_materials[depth], cur_material, el);
  };
  while (fscanf(fp, "%127s", cmd) == 1) {
    if (cmd[0] == '#') {
      int c;
      do { c = fgetc(fp); } while (c >= 0 && c != '\n');
      continue;
    }
    Element *el = nullptr;
    if (!strcmp(cmd, "tri")) {
      int m;
      double v[9];
      if (fscanf(fp, "%d%lf%lf%lf%lf%lf%lf%lf%lf%lf", &m, &v[0], &v[1], &v[2], &v[3], &v[4],
                 &v[5], &v[6], &v[7], &v[8]) != 10)
        return fail("triangle");
      Shape sh;
      sh.type = SH_TRI;
      sh.tri = make_tri(V3(v[0], v[1], v[2]), V3(v[3], v[4], v[5]), V3(v[6], v[7], v[8]));
      sh.box = sh.tri.box;
      if (!resolve(m, el)) return fail("material id");
      el->shapes.push_back(sh);
    } else if (!strcmp(cmd, "box")) {
      int m;
      double v[6];
      if (fscanf(fp, "%d%lf%lf%lf%lf%lf%lf", &m, &v[0], &v[1], &v[2], &v[3], &v[4], &v[5]) != 7)
        return fail("box");
      for (int i = 0; i < 3; i++)
        if (v[i] > v[i + 3]) { double t = v[i]; v[i] = v[i + 3]; v[i + 3] = t; }
      Shape sh;
      sh.type = SH_BOX;
      sh.box.mn = V3(v[0], v[1], v[2]);
      sh.box.mx = V3(v[3], v[4], v[5]);
      if (!resolve(m, el)) return fail("material id");
      el->shapes.push_back(sh);
    } else if (!strcmp(cmd, "sphere")) {
      int m;
      double c[3], r;
      if (fscanf(fp, "%d%lf%lf%lf%lf", &m, &c[0], &c[1], &c[2], &r) != 5) return fail("sphere");
      Shape sh;
      sh.type = SH_SPHERE;
      sh.c = V3(c[0], c[1], c[2]);
      sh.r = r;
      sh.box.mn = V3(c[0] - r, c[1] - r, c[2] - r);
      sh.box.mx = V3(c[0] + r, c[1] + r, c[2] + r);
      if (!resolve(m, el)) return fail("material id");
      el->shapes.push_back(sh);
    } else if (!strcmp(cmd, "circle")) {
      int m;
      double c[3], d[3], r;
      if (fscanf(fp, "%d%lf%lf%lf%lf%lf%lf%lf", &m, &c[0], &c[1], &c[2], &d[0], &d[1], &d[2],
                 &r) != 8)
        return fail("circle");
      Shape sh;
      sh.type = SH_CIRCLE;
      sh.c = V3(c[0], c[1], c[2]);
      sh.axis = normalize(V3(d[0], d[1], d[2]));
      sh.r = r;
      // R3Circle::BBox (R3Circle.cpp:179-184): the cube centre +- radius
      for (int i = 0; i < 3; i++) {
        sh.box.mn[i] = c[i] - r;
        sh.box.mx[i] = c[i] + r;
      }
      if (!resolve(m, el)) return fail("material id");
      el->shapes.push_back(sh);
    } else if (!strcmp(cmd, "cylinder") || !strcmp(cmd, "cone")) {
      int m;
      double c[3], r, h;
      if (fscanf(fp, "%d%lf%lf%lf%lf%lf", &m, &c[0], &c[1], &c[2], &r, &h) != 6)
        return fail(cmd);
      Shape sh;
      // R3Scene.cpp:1589-1636: p1/p2 = c -/+ 0.5*h*(0,1,0)
      sh.type = !strcmp(cmd, "cylinder") ? SH_CYLINDER : SH_CONE;
      sh.c = V3(c[0], c[1] - 0.5 * h, c[2]);
      sh.axis = V3(c[0], c[1] + 0.5 * h, c[2]);
      sh.r = r;
      cap_cubes_box(sh);
      if (!resolve(m, el)) return fail("material id");
      el->shapes.push_back(sh);
    } else if (!strcmp(cmd, "line")) {
      int m;
      double v[6];
      if (fscanf(fp, "%d%lf%lf%lf%lf%lf%lf", &m, &v[0], &v[1], &v[2], &v[3], &v[4], &v[5]) != 7)
        return fail("line");
      Shape sh;
      // R3Scene.cpp:1667-1687: a line is R3Cylinder(p1, p2, RN_BIG_EPSILON)
      sh.type = SH_CYLINDER;
      sh.c = V3(v[0], v[1], v[2]);
      sh.axis = V3(v[3], v[4], v[5]);
      sh.r = 1e-3;  // RN_BIG_EPSILON (RNScalar.cpp:22)
      cap_cubes_box(sh);
      if (!resolve(m, el)) return fail("material id");
      el->shapes.push_back(sh);
    } else if (!strcmp(cmd, "mesh")) {
      int m;
      char meshname[256];
      if (fscanf(fp, "%d%255s", &m, meshname) != 2) return fail("mesh");
      Shape sh;
      sh.type = SH_MESH;
      std::string e2;
      if (!read_off(dir_of(filename) + meshname, sh.tris, e2)) {
        err = e2;
        fclose(fp);
        return false;
      }
      for (auto &t : sh.tris) sh.box.add(t.box);
      if (!resolve(m, el)) return fail("material id");
      el->shapes.push_back(sh);
    } else if (!strcmp(cmd, "begin")) {
      int m;
      double mm[16];
      if (fscanf(fp, "%d%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf", &m, &mm[0], &mm[1],
                 &mm[2], &mm[3], &mm[4], &mm[5], &mm[6], &mm[7], &mm[8], &mm[9], &mm[10], &mm[11],
                 &mm[12], &mm[13], &mm[14], &mm[15]) != 17)
        return fail("begin");
      if (m >= 0) cur_material = (m < (int)parsed.size()) ? parsed[m] : -1;
      Node nd;
      for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) nd.T.m[i][j] = mm[4 * i + j];
      nd.Tinv = nd.T.inverse();
      s.nodes.push_back(nd);
      int id = (int)s.nodes.size() - 1;
      s.nodes[group_nodes[depth]].children.push_back(id);
      depth++;
      group_nodes[depth] = id;
      group_materials[depth] = cur_material;
    } else if (!strcmp(cmd, "end")) {
      if (depth <= 0) return fail("end (extra end statement)");
      depth--;
    } else if (!strcmp(cmd, "material")) {
      double v[17];
      char tex[256];
      if (fscanf(fp, "%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%255s", &v[0], &v[1],
                 &v[2], &v[3], &v[4], &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11], &v[12],
                 &v[13], &v[14], &v[15], &v[16], tex) != 18)
        return fail("material");
      Brdf b;
      b.ka = Rgb(v[0], v[1], v[2]);
      b.kd = Rgb(v[3], v[4], v[5]);
      b.ks = Rgb(v[6], v[7], v[8]);
      b.kt = Rgb(v[9], v[10], v[11]);
      b.e = Rgb(v[12], v[13], v[14]);
      b.n = v[15];
      b.ir = v[16];
      if (real) {  // R3Scene.cpp:1779-1793 (-real)
        Rgb tot = b.kd + b.ks + b.kt;
        double mx = 1.0;
        for (int i = 0; i < 3; i++)
          if (tot[i] > mx) mx = tot[i];
        if (mx > 1.0) { b.kd = b.kd / mx; b.ks = b.ks / mx; b.kt = b.kt / mx; }
      }
      s.materials.push_back(b);
      parsed.push_back((int)s.materials.size() - 1);
    } else if (!strcmp(cmd, "dir_light")) {
      double v[6];
      if (fscanf(fp, "%lf%lf%lf%lf%lf%lf", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5]) != 6)
        return fail("directional light");
      Light L;
      L.type = L_DIR;
      L.color = Rgb(v[0], v[1], v[2]);
      L.dir = normalize(V3(v[3], v[4], v[5]));
      s.lights.push_back(L);
    } else if (!strcmp(cmd, "point_light")) {
      double v[9];
      if (fscanf(fp, "%lf%lf%lf%lf%lf%lf%lf%lf%lf", &v[0], &v[1], &v[2], &v[3], &v[4], &v[5],
                 &v[6], &v[7], &v[8]) != 9)
        return fail("point light");
      Light L;
      L.type = L_POINT;
      L.color = Rgb(v[0], v[1], v[2]);
      L.pos = V3(v[3], v[4], v[5]);
      L.ca = v[6]; L.la = v[7]; L.qa = v[8];
      s.lights.push_back(L);
    } else if (!strcmp(cmd, "spot_light")) {
      double v[14];
      if (fscanf(fp, "%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf", &v[0], &v[1], &v[2], &v[3],
                 &v[4], &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11], &v[12], &v[13]) != 14)
        return fail("spot light");
      Light L;
      L.type = L_SPOT;
      L.color = Rgb(v[0], v[1], v[2]);
      L.pos = V3(v[3], v[4], v[5]);
      L.dir = normalize(normalize(V3(v[6], v[7], v[8])));
      L.ca = v[9]; L.la = v[10]; L.qa = v[11];
      L.cutoff = v[12];   // sc
      L.dropoff = v[13];  // sd
      s.lights.push_back(L);
    } else if (!strcmp(cmd, "area_light")) {
      double v[13];
      if (fscanf(fp, "%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf", &v[0], &v[1], &v[2], &v[3],
                 &v[4], &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11], &v[12]) != 13)
        return fail("area light");
      Light L;
      L.type = L_AREA;
      L.color = Rgb(v[0], v[1], v[2]);
      L.pos = V3(v[3], v[4], v[5]);
      L.dir = normalize(V3(v[6], v[7], v[8]));
      L.radius = v[9];
      L.ca = v[10]; L.la = v[11]; L.qa = v[12];
      s.lights.push_back(L);
    } else if (!strcmp(cmd, "rect_light")) {
      double v[17];
      if (fscanf(fp, "%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf", &v[0], &v[1],
                 &v[2], &v[3], &v[4], &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11], &v[12],
                 &v[13], &v[14], &v[15], &v[16]) != 17)
        return fail("rect light");
      Light L;
      L.type = L_RECT;
      L.color = Rgb(v[0], v[1], v[2]);
      L.pos = V3(v[3], v[4], v[5]);
      // R3RectLight ctor, R3RectLight.cpp:58-75 (axes normalized twice: loader + ctor)
      L.a1 = normalize(normalize(V3(v[6], v[7], v[8])));
      L.a2 = normalize(normalize(V3(v[9], v[10], v[11])));
      L.dir = normalize(cross(L.a1, L.a2));
      L.len1 = v[12]; L.len2 = v[13];
      L.ca = v[14]; L.la = v[15]; L.qa = v[16];
      s.lights.push_back(L);
    } else if (!strcmp(cmd, "camera")) {
      double v[12];
      if (fscanf(fp, "%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf%lf", &v[0], &v[1], &v[2], &v[3], &v[4],
                 &v[5], &v[6], &v[7], &v[8], &v[9], &v[10], &v[11]) != 12)
        return fail("camera");
      // R3Camera(e, t, u, xfov, xfov, ...), R3Triad(towards, up) R3Triad.cpp:72-79
      Camera c;
      c.eye = V3(v[0], v[1], v[2]);
      V3 z = normalize(-V3(v[3], v[4], v[5]));
      V3 x = normalize(cross(V3(v[6], v[7], v[8]), z));
      V3 y = cross(z, x);
      c.right = x; c.up = y; c.towards = -z;
      c.xfov = v[9]; c.yfov = v[9];  // Q5: yfov = xfov
      s.camera = c;
      s.has_camera = true;
    } else if (!strcmp(cmd, "include")) {
      char name[256];
      if (fscanf(fp, "%255s", name) != 1) return fail("include");
      std::vector<int> sub_parsed;
      if (!read_princeton(s, group_nodes[depth], dir_of(filename) + name, real, sub_parsed,
                          err)) {
        fclose(fp);
        return false;
      }
    } else if (!strcmp(cmd, "background")) {
      double r, g, b;
      if (fscanf(fp, "%lf%lf%lf", &r, &g, &b) != 3) return fail("background");
      s.background = Rgb(r, g, b);
    } else if (!strcmp(cmd, "ambient")) {
      double r, g, b;
      if (fscanf(fp, "%lf%lf%lf", &r, &g, &b) != 3) return fail("ambient");
      s.ambient = Rgb(r, g, b);
    } else {
      char b[512];
      snprintf(b, sizeof b, "Unrecognized command %d in file %s: %s", command_number,
               filename.c_str(), cmd);
      err = b;
      fclose(fp);
      return false;
    }
    command_number++;
  }
  fclose(fp);
  return true;
}

static void update_bbox(Scene &s, int ni) {
  Node &nd = s.nodes[ni];
  nd.bbox = Box();
  auto add_tx = [&](const Box &b) {
    if (b.empty()) return;
    for (int c = 0; c < 8; c++) {
      V3 p((c & 1) ? b.mx.x : b.mn.x, (c & 2) ? b.mx.y : b.mn.y, (c & 4) ? b.mx.z : b.mn.z);
      nd.bbox.add(nd.T.point(p));
    }
  };
  for (auto &el : nd.elements) {
    el.bbox = Box();
    for (auto &sh : el.shapes) el.bbox.add(sh.box);
    add_tx(el.bbox);
  }
  for (int ci : nd.children) {
    update_bbox(s, ci);
    add_tx(s.nodes[ci].bbox);
  }
}

bool read_scene(const std::string &path, bool real_material, Scene &s, std::string &err) {
  s = Scene();
  Node root;
  root.T = M4::identity();
  root.Tinv = M4::identity();
  s.nodes.push_back(root);
  size_t dot_pos = path.rfind('.');
  if (dot_pos == std::string::npos) { err = "Filename " + path + " has no extension"; return false; }
  std::string ext = path.substr(dot_pos);
  if (ext.compare(0, 4, ".scn") == 0) {
    std::vector<int> parsed;
    if (!read_princeton(s, 0, path, real_material, parsed, err)) return false;
  } else if (ext.compare(0, 4, ".off") == 0) {
    // R3Scene::ReadMeshFile: one node, one element (null material -> default)
    Node child;
    child.T = M4::identity();
    child.Tinv = M4::identity();
    Shape sh;
    sh.type = SH_MESH;
    if (!read_off(path, sh.tris, err)) return false;
    for (auto &t : sh.tris) sh.box.add(t.box);
    Element el;
    el.material = -1;
    el.shapes.push_back(sh);
    child.elements.push_back(el);
    s.nodes.push_back(child);
    s.nodes[0].children.push_back(1);
  } else {
    err = "Unable to read file " + path + " (unrecognized extension)";
    return false;
  }
  update_bbox(s, 0);
  s.bbox = s.nodes[0].bbox;
  s.radius = s.bbox.diag_radius();
  s.centroid = s.bbox.centroid();
  // default camera, R3Scene.cpp:557-566
  if (!s.has_camera) {
    double r = s.radius;
    V3 c = s.centroid;
    V3 towards(0, 0, -1), up(0, 1, 0);
    Camera cam;
    cam.eye = c - 3 * r * towards;
    V3 z = normalize(-towards);
    V3 x = normalize(cross(up, z));
    cam.right = x; cam.up = cross(z, x); cam.towards = -z;
    cam.xfov = 0.25; cam.yfov = 0.25;
    s.camera = cam;
  }
  // default lights, R3Scene.cpp:569-583
  if (s.lights.empty()) {
    Light a;
    a.type = L_DIR; a.color = Rgb(1, 1, 1); a.dir = normalize(V3(-3, -4, -5));
    Light b;
    b.type = L_DIR; b.color = Rgb(0.5, 0.5, 0.5); b.dir = normalize(V3(3, 2, 3));
    s.lights.push_back(a);
    s.lights.push_back(b);
  }
  return true;
}

}  // namespace oracle
