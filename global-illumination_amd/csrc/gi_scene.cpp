// gi_scene.cpp -- .scn (Princeton) / .off loader producing the flattened device scene.
//
// Grammar and defaults follow the reference loader ReadPrinceton (R3Graphics/R3Scene.cpp:
// 1446-1953), FindPrincetonMaterialAndElement (:1401-1441), ReadMesh (:1359-1394) and
// R3Mesh::ReadOffFile (R3Shapes/R3Mesh.cpp:4075-4210, CreateFace half-edge rule :1168-1196);
// default camera / lights as R3Scene::ReadFile (:557-583).
#include "gi_scene.h"
#include <array>
#include <cfloat>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cctype>
#include <map>

namespace gi {
namespace {

struct P3 {
  double v[3];
};
static P3 p3(double a, double b, double c) { P3 r; r.v[0] = a; r.v[1] = b; r.v[2] = c; return r; }
static P3 sub(P3 a, P3 b) { return p3(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2]); }
static P3 crs(P3 a, P3 b) {
  return p3(a.v[1] * b.v[2] - a.v[2] * b.v[1], a.v[2] * b.v[0] - a.v[0] * b.v[2],
            a.v[0] * b.v[1] - a.v[1] * b.v[0]);
}
static double nrm(P3 a) { return sqrt((a.v[0] * a.v[0]) + (a.v[1] * a.v[1]) + (a.v[2] * a.v[2])); }
static P3 unit(P3 a) {
  double l = nrm(a);
  if (l == 0.0) return a;
  return p3(a.v[0] / l, a.v[1] / l, a.v[2] / l);
}
static P3 scl(P3 a, double s) { return p3(a.v[0] * s, a.v[1] * s, a.v[2] * s); }

struct Bx {
  double mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  bool empty() const { return mn[0] > mx[0] || mn[1] > mx[1] || mn[2] > mx[2]; }
  void add(const double *p) {
    for (int i = 0; i < 3; i++) {
      if (p[i] < mn[i]) mn[i] = p[i];
      if (p[i] > mx[i]) mx[i] = p[i];
    }
  }
  void add(const Bx &b) {
    if (b.empty()) return;
    add(b.mn);
    add(b.mx);
  }
};

// triangle with plane + edge planes (R3Plane(p0,p1,p2); R3Plane(point, n, edge))
static DTri make_tri(P3 a, P3 b, P3 c) {
  DTri t;
  P3 n = unit(crs(sub(b, a), sub(c, a)));
  for (int i = 0; i < 3; i++) { t.p0[i] = a.v[i]; t.n[i] = n.v[i]; }
  t.d = -(n.v[0] * a.v[0] + n.v[1] * a.v[1] + n.v[2] * a.v[2]);
  P3 e[3] = {sub(b, a), sub(c, b), sub(a, c)};
  P3 q[3] = {b, c, a};
  for (int k = 0; k < 3; k++) {
    P3 v = unit(crs(n, e[k]));
    for (int i = 0; i < 3; i++) t.ev[k][i] = v.v[i];
    t.ed[k] = -(v.v[0] * q[k].v[0] + v.v[1] * q[k].v[1] + v.v[2] * q[k].v[2]);
  }
  Bx bx;
  bx.add(a.v); bx.add(b.v); bx.add(c.v);
  for (int i = 0; i < 3; i++) { t.bmin[i] = bx.mn[i]; t.bmax[i] = bx.mx[i]; }
  return t;
}

struct GShape {
  DShape s;
  std::vector<DTri> tris;
};
struct GElem {
  int mat;
  std::vector<GShape> shapes;
};
struct GNode {
  double T[16], Tinv[16];
  bool identity = true;
  std::vector<GElem> elems;
  std::vector<int> children;
};

struct Graph {
  std::vector<GNode> nodes;
  std::vector<DMaterial> mats;
  std::vector<DLight> lights;
  bool has_camera = false;
  double cam[12];  // eye, towards, up, xfov
  double ambient[3] = {0, 0, 0}, background[3] = {0, 0, 0};
};

static void mat_flags(DMaterial &m) {  // R3Brdf::UpdateFlags, R3Brdf.cpp:338-348
  auto nz = [](const double *c) { return !(c[0] == 0.0 && c[1] == 0.0 && c[2] == 0.0); };
  m.flags = 0;
  if (nz(m.ka)) m.flags |= MF_AMBIENT;
  if (nz(m.kd)) m.flags |= MF_DIFFUSE;
  if (nz(m.ks)) m.flags |= MF_SPECULAR;
  if (nz(m.kt)) m.flags |= MF_TRANSPARENT;
  if (nz(m.e)) m.flags |= MF_EMISSIVE;
  auto mx = [](const double *c) {
    double v = 0;
    for (int i = 0; i < 3; i++)
      if (c[i] > v) v = c[i];
    return v;
  };
  m.max_kd = mx(m.kd); m.max_kt = mx(m.kt); m.max_ks = mx(m.ks); m.max_e = mx(m.e);
}

static DMaterial default_material() {  // R3default_brdf, R3Brdf.cpp:13-15
  DMaterial m;
  memset(&m, 0, sizeof m);
  for (int i = 0; i < 3; i++) { m.ka[i] = 0.2; m.kd[i] = 0.8; }
  m.n = 0.2;
  m.ir = 1.0;
  mat_flags(m);
  return m;
}

static void mat_inverse(const double *m, double *out) {
  double a[4][8];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) a[i][j] = (j < 4) ? m[4 * i + j] : ((j - 4 == i) ? 1.0 : 0.0);
  for (int c = 0; c < 4; c++) {
    int p = c;
    for (int r = c + 1; r < 4; r++)
      if (fabs(a[r][c]) > fabs(a[p][c])) p = r;
    if (p != c)
      for (int j = 0; j < 8; j++) std::swap(a[c][j], a[p][j]);
    double d = a[c][c];
    for (int j = 0; j < 8; j++) a[c][j] /= d;
    for (int r = 0; r < 4; r++) {
      if (r == c) continue;
      double f = a[r][c];
      if (f == 0.0) continue;
      for (int j = 0; j < 8; j++) a[r][j] -= f * a[c][j];
    }
  }
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) out[4 * i + j] = a[i][j + 4];
}

// R3Mesh::ReadOffFile with the half-edge CreateFace rule and deferred re-creation
static bool read_off(const std::string &path, std::vector<DTri> &tris, std::string &err) {
  FILE *fp = fopen(path.c_str(), "r");
  if (!fp) { err = "Unable to open file " + path; return false; }
  std::vector<P3> verts;
  struct ER { int v0; bool f0, f1; };
  std::map<std::pair<int, int>, ER> edges;
  std::vector<std::array<int, 3>> faces, later;
  auto edge = [&](int a, int b) -> ER & {
    auto key = std::make_pair(std::min(a, b), std::max(a, b));
    auto it = edges.find(key);
    if (it == edges.end()) it = edges.emplace(key, ER{a, false, false}).first;
    return it->second;
  };
  auto face = [&](int a, int b, int c) {
    ER &e1 = edge(a, b), &e2 = edge(b, c), &e3 = edge(c, a);
    auto used = [](ER &e, int from) { return (e.v0 == from) ? e.f0 : e.f1; };
    if (used(e1, a) || used(e2, b) || used(e3, c)) return false;
    (e1.v0 == a ? e1.f0 : e1.f1) = true;
    (e2.v0 == b ? e2.f0 : e2.f1) = true;
    (e3.v0 == c ? e3.f0 : e3.f1) = true;
    faces.push_back({a, b, c});
    return true;
  };
  int nv = 0, nf = 0, ne = 0, vc = 0, fc = 0;
  char line[1024], hdr[64];
  while (fgets(line, 1023, fp)) {
    char *s = line;
    while (isspace((unsigned char)*s)) s++;
    if (*s == '#' || *s == '\0') continue;
    if (nv == 0) {
      if (strstr(s, "OFF")) {
        int t;
        if (sscanf(s, "%63s%d%d%d", hdr, &t, &nf, &ne) == 4) nv = t;
      } else if (sscanf(s, "%d%d%d", &nv, &nf, &ne) != 3 || nv == 0) {
        fclose(fp);
        err = "Syntax error reading header in " + path;
        return false;
      }
    } else if (vc < nv) {
      double x, y, z;
      if (sscanf(s, "%lf%lf%lf", &x, &y, &z) != 3) {
        fclose(fp);
        err = "Syntax error with vertex coordinates in " + path;
        return false;
      }
      verts.push_back(p3(x, y, z));
      vc++;
    } else if (fc < nf) {
      char *tok = strtok(s, " \t");
      if (!tok) { fclose(fp); err = "Syntax error with face in " + path; return false; }
      int k = atoi(tok), v1 = -1, v2 = -1, v3 = -1;
      for (int i = 0; i < k; i++) {
        tok = strtok(NULL, " \t");
        if (!tok) { fclose(fp); err = "Syntax error with face in " + path; return false; }
        int v = atoi(tok);
        if (v1 < 0) v1 = v; else v3 = v;
        if (v1 >= 0 && v2 >= 0 && v3 >= 0 && v1 != v2 && v2 != v3 && v1 != v3)
          if (!face(v1, v2, v3)) later.push_back({v1, v2, v3});
        v2 = v3;
      }
      fc++;
    } else {
      break;
    }
  }
  fclose(fp);
  for (auto &f : later) {
    if (face(f[0], f[1], f[2])) continue;
    if (face(f[0], f[2], f[1])) continue;
    int b = (int)verts.size();
    verts.push_back(verts[f[0]]);
    verts.push_back(verts[f[1]]);
    verts.push_back(verts[f[2]]);
    face(b, b + 1, b + 2);
  }
  for (auto &f : faces) {
    for (int i = 0; i < 3; i++)
      if (f[i] < 0 || f[i] >= (int)verts.size()) { err = "bad vertex index in " + path; return false; }
    tris.push_back(make_tri(verts[f[0]], verts[f[1]], verts[f[2]]));
  }
  return true;
}

static std::string folder(const std::string &f) {
  size_t p = f.rfind('/');
  return p == std::string::npos ? std::string() : f.substr(0, p + 1);
}

static bool read_doubles(FILE *fp, double *v, int n) {
  for (int i = 0; i < n; i++)
    if (fscanf(fp, "%lf", &v[i]) != 1) return false;
  return true;
}

// ReadPrinceton, R3Scene.cpp:1446-1953
static bool parse(Graph &G, int root, const std::string &file, bool real, std::string &err) {
  FILE *fp = fopen(file.c_str(), "r");
  if (!fp) { err = "Unable to open file " + file; return false; }
  std::vector<int> parsed;  // this file's materials (each include has its own list)
  int gnode[1024], gmat[1024];
  gnode[0] = root;
  gmat[0] = -1;
  int depth = 0, cur = -1, cmdno = 1;
  char cmd[128];
  auto bad = [&](const char *what) {
    char b[512];
    snprintf(b, sizeof b, "Unable to read %s at command %d in file %s", what, cmdno, file.c_str());
    err = b;
    fclose(fp);
    return false;
  };
  // FindPrincetonMaterialAndElement
  auto elem_for = [&](int m) -> GElem * {
    int mi;
    if (m >= 0) {
      if (m >= (int)parsed.size()) return nullptr;
      mi = parsed[m];
    } else {
      mi = gmat[depth];
      if (mi < 0) {
        G.mats.push_back(default_material());
        mi = (int)G.mats.size() - 1;
        gmat[depth] = mi;
      }
    }
    cur = mi;
    GNode &nd = G.nodes[gnode[depth]];
    for (auto &e : nd.elems)
      if (e.mat == mi) return &e;
    nd.elems.push_back(GElem());
    nd.elems.back().mat = mi;
    return &nd.elems.back();
  };
  auto add_shape = [&](int m, GShape &&s) {
    GElem *e = elem_for(m);
    if (!e) return false;
    e->shapes.push_back(std::move(s));
    return true;
  };
  while (fscanf(fp, "%127s", cmd) == 1) {
    if (cmd[0] == '#') {
      int c;
      do { c = fgetc(fp); } while (c >= 0 && c != '\n');
      continue;
    }
    int m;
    double v[20];
    if (!strcmp(cmd, "tri")) {
      if (fscanf(fp, "%d", &m) != 1 || !read_doubles(fp, v, 9)) return bad("triangle");
      GShape s;
      memset(&s.s, 0, sizeof s.s);
      s.s.kind = SK_TRI;
      s.tris.push_back(make_tri(p3(v[0], v[1], v[2]), p3(v[3], v[4], v[5]), p3(v[6], v[7], v[8])));
      if (!add_shape(m, std::move(s))) return bad("material id");
    } else if (!strcmp(cmd, "box")) {
      if (fscanf(fp, "%d", &m) != 1 || !read_doubles(fp, v, 6)) return bad("box");
      GShape s;
      memset(&s.s, 0, sizeof s.s);
      s.s.kind = SK_BOX;
      for (int i = 0; i < 3; i++) {
        s.s.bmin[i] = std::min(v[i], v[i + 3]);
        s.s.bmax[i] = std::max(v[i], v[i + 3]);
      }
      if (!add_shape(m, std::move(s))) return bad("material id");
    } else if (!strcmp(cmd, "sphere")) {
      if (fscanf(fp, "%d", &m) != 1 || !read_doubles(fp, v, 4)) return bad("sphere");
      GShape s;
      memset(&s.s, 0, sizeof s.s);
      s.s.kind = SK_SPHERE;
      for (int i = 0; i < 3; i++) {
        s.s.c[i] = v[i];
        s.s.bmin[i] = v[i] - v[3];
        s.s.bmax[i] = v[i] + v[3];
      }
      s.s.r = v[3];
      if (!add_shape(m, std::move(s))) return bad("material id");
    } else if (!strcmp(cmd, "circle")) {
      if (fscanf(fp, "%d", &m) != 1 || !read_doubles(fp, v, 7)) return bad("circle");
      GShape s;
      memset(&s.s, 0, sizeof s.s);
      s.s.kind = SK_CIRCLE;
      P3 n = unit(p3(v[3], v[4], v[5]));
      for (int i = 0; i < 3; i++) {
        s.s.c[i] = v[i];
        s.s.n[i] = n.v[i];
        s.s.bmin[i] = v[i] - v[6];  // R3Circle::BBox: centre +- radius (R3Circle.cpp:179-184)
        s.s.bmax[i] = v[i] + v[6];
      }
      s.s.r = v[6];
      if (!add_shape(m, std::move(s))) return bad("material id");
    } else if (!strcmp(cmd, "cylinder") || !strcmp(cmd, "cone") || !strcmp(cmd, "line")) {
      bool line = !strcmp(cmd, "line");
      int nv = line ? 6 : 5;
      if (fscanf(fp, "%d", &m) != 1 || !read_doubles(fp, v, nv)) return bad(cmd);
      GShape s;
      memset(&s.s, 0, sizeof s.s);
      s.s.kind = !strcmp(cmd, "cone") ? SK_CONE : SK_CYLINDER;
      // cylinder/cone (R3Scene.cpp:1589-1636): p1/p2 = c -/+ 0.5*h*(0,1,0);
      // line (:1667-1687): R3Cylinder(p1, p2, RN_BIG_EPSILON = 1e-3)
      double p1[3], p2[3], rad;
      if (line) {
        for (int i = 0; i < 3; i++) { p1[i] = v[i]; p2[i] = v[3 + i]; }
        rad = 1e-3;
      } else {
        for (int i = 0; i < 3; i++) p1[i] = p2[i] = v[i];
        p1[1] = v[1] - 0.5 * v[4];
        p2[1] = v[1] + 0.5 * v[4];
        rad = v[3];
      }
      s.s.r = rad;
      for (int i = 0; i < 3; i++) {
        s.s.c[i] = p1[i];
        s.s.n[i] = p2[i];
        // R3Cylinder::BBox: union of the cap circles' centre +- radius cubes
        s.s.bmin[i] = std::min(p1[i] - rad, p2[i] - rad);
        s.s.bmax[i] = std::max(p1[i] + rad, p2[i] + rad);
      }
      if (!add_shape(m, std::move(s))) return bad("material id");
    } else if (!strcmp(cmd, "mesh")) {
      char name[256];
      if (fscanf(fp, "%d%255s", &m, name) != 2) return bad("mesh");
      GShape s;
      memset(&s.s, 0, sizeof s.s);
      s.s.kind = SK_MESH;
      std::string e2;
      if (!read_off(folder(file) + name, s.tris, e2)) {
        err = e2;
        fclose(fp);
        return false;
      }
      if (!add_shape(m, std::move(s))) return bad("material id");
    } else if (!strcmp(cmd, "begin")) {
      if (fscanf(fp, "%d", &m) != 1 || !read_doubles(fp, v, 16)) return bad("begin");
      if (m >= 0) cur = (m < (int)parsed.size()) ? parsed[m] : -1;
      GNode nd;
      bool ident = true;
      for (int i = 0; i < 16; i++) {
        nd.T[i] = v[i];
        if (v[i] != ((i % 5 == 0) ? 1.0 : 0.0)) ident = false;
      }
      nd.identity = ident;
      mat_inverse(nd.T, nd.Tinv);
      G.nodes.push_back(nd);
      int id = (int)G.nodes.size() - 1;
      G.nodes[gnode[depth]].children.push_back(id);
      depth++;
      gnode[depth] = id;
      gmat[depth] = cur;
    } else if (!strcmp(cmd, "end")) {
      if (depth <= 0) return bad("end (extra end statement)");
      depth--;
    } else if (!strcmp(cmd, "material")) {
      char tex[256];
      if (!read_doubles(fp, v, 17) || fscanf(fp, "%255s", tex) != 1) return bad("material");
      DMaterial mt;
      memset(&mt, 0, sizeof mt);
      for (int i = 0; i < 3; i++) {
        mt.ka[i] = v[i]; mt.kd[i] = v[3 + i]; mt.ks[i] = v[6 + i];
        mt.kt[i] = v[9 + i]; mt.e[i] = v[12 + i];
      }
      mt.n = v[15];
      mt.ir = v[16];
      if (real) {  // -real normalisation, R3Scene.cpp:1779-1793
        double mx = 1.0;
        for (int i = 0; i < 3; i++) mx = std::max(mx, mt.kd[i] + mt.ks[i] + mt.kt[i]);
        if (mx > 1.0)
          for (int i = 0; i < 3; i++) { mt.kd[i] /= mx; mt.ks[i] /= mx; mt.kt[i] /= mx; }
      }
      mat_flags(mt);
      G.mats.push_back(mt);
      parsed.push_back((int)G.mats.size() - 1);
    } else if (!strcmp(cmd, "dir_light") || !strcmp(cmd, "point_light") ||
               !strcmp(cmd, "spot_light") || !strcmp(cmd, "area_light") ||
               !strcmp(cmd, "rect_light")) {
      DLight L;
      memset(&L, 0, sizeof L);
      L.active = 1;
      L.intensity = 1.0;
      if (!strcmp(cmd, "dir_light")) {
        if (!read_doubles(fp, v, 6)) return bad("directional light");
        L.kind = LK_DIR;
        P3 d = unit(p3(v[3], v[4], v[5]));
        for (int i = 0; i < 3; i++) { L.color[i] = v[i]; L.dir[i] = d.v[i]; }
      } else if (!strcmp(cmd, "point_light")) {
        if (!read_doubles(fp, v, 9)) return bad("point light");
        L.kind = LK_POINT;
        for (int i = 0; i < 3; i++) { L.color[i] = v[i]; L.pos[i] = v[3 + i]; }
        L.ca = v[6]; L.la = v[7]; L.qa = v[8];
      } else if (!strcmp(cmd, "spot_light")) {
        if (!read_doubles(fp, v, 14)) return bad("spot light");
        L.kind = LK_SPOT;
        P3 d = unit(unit(p3(v[6], v[7], v[8])));  // loader + R3SpotLight ctor
        for (int i = 0; i < 3; i++) { L.color[i] = v[i]; L.pos[i] = v[3 + i]; L.dir[i] = d.v[i]; }
        L.ca = v[9]; L.la = v[10]; L.qa = v[11];
        L.cutoff = v[12];
        L.dropoff = v[13];
      } else if (!strcmp(cmd, "area_light")) {
        if (!read_doubles(fp, v, 13)) return bad("area light");
        L.kind = LK_AREA;
        P3 d = unit(p3(v[6], v[7], v[8]));
        for (int i = 0; i < 3; i++) { L.color[i] = v[i]; L.pos[i] = v[3 + i]; L.dir[i] = d.v[i]; }
        L.radius = v[9];
        L.ca = v[10]; L.la = v[11]; L.qa = v[12];
      } else {
        if (!read_doubles(fp, v, 17)) return bad("rect light");
        L.kind = LK_RECT;
        P3 a1 = unit(unit(p3(v[6], v[7], v[8]))), a2 = unit(unit(p3(v[9], v[10], v[11])));
        P3 n = unit(crs(a1, a2));  // R3RectLight ctor, R3RectLight.cpp:58-75
        for (int i = 0; i < 3; i++) {
          L.color[i] = v[i]; L.pos[i] = v[3 + i];
          L.a1[i] = a1.v[i]; L.a2[i] = a2.v[i]; L.dir[i] = n.v[i];
        }
        L.len1 = v[12]; L.len2 = v[13];
        L.ca = v[14]; L.la = v[15]; L.qa = v[16];
      }
      G.lights.push_back(L);
    } else if (!strcmp(cmd, "camera")) {
      if (!read_doubles(fp, v, 12)) return bad("camera");
      G.has_camera = true;
      for (int i = 0; i < 10; i++) G.cam[i] = v[i];
    } else if (!strcmp(cmd, "include")) {
      char name[256];
      if (fscanf(fp, "%255s", name) != 1) return bad("include");
      if (!parse(G, gnode[depth], folder(file) + name, real, err)) {
        fclose(fp);
        return false;
      }
    } else if (!strcmp(cmd, "background") || !strcmp(cmd, "ambient")) {
      if (!read_doubles(fp, v, 3)) return bad(cmd);
      double *dst = !strcmp(cmd, "background") ? G.background : G.ambient;
      for (int i = 0; i < 3; i++) dst[i] = v[i];
    } else {
      char b[512];
      snprintf(b, sizeof b, "Unrecognized command %d in file %s: %s", cmdno, file.c_str(), cmd);
      err = b;
      fclose(fp);
      return false;
    }
    cmdno++;
  }
  fclose(fp);
  return true;
}

static void shape_box(GShape &s) {
  if (s.s.kind == SK_TRI || s.s.kind == SK_MESH) {
    Bx b;
    for (auto &t : s.tris) { b.add(t.bmin); b.add(t.bmax); }
    for (int i = 0; i < 3; i++) { s.s.bmin[i] = b.mn[i]; s.s.bmax[i] = b.mx[i]; }
  }
}

static void xform_box(const double *T, const Bx &b, Bx &out) {
  if (b.empty()) return;
  for (int c = 0; c < 8; c++) {
    double p[3] = {(c & 1) ? b.mx[0] : b.mn[0], (c & 2) ? b.mx[1] : b.mn[1],
                   (c & 4) ? b.mx[2] : b.mn[2]};
    double q[3];
    for (int r = 0; r < 3; r++) q[r] = T[4 * r] * p[0] + T[4 * r + 1] * p[1] + T[4 * r + 2] * p[2] + T[4 * r + 3];
    out.add(q);
  }
}

// ---- per-mesh BVH (DBvhNode, gi_layout.h) ----------------------------------------------
// Top-down median split of the triangle centroids along the longest axis of their box, leaves of
// at most BVH_LEAF triangles, nodes emitted in pre-order with skip links. Box margin: the
// containment tolerances of a triangle hit are 1e-6 per coordinate (R3Cont.cpp:491-512), so a
// reported hit point lies within 1e-6 of its triangle's box; 1e-5 + 1e-9 |x| keeps every such
// point strictly inside its node boxes, with room for the slab test's rounding.
constexpr int BVH_LEAF = 4;
constexpr int BVH_MIN_TRIS = 16;  // smaller meshes keep the linear loop

static int bvh_rec(std::vector<DTri> &t, int a, int b, std::vector<DBvhNode> &out) {
  int id = (int)out.size();
  out.push_back(DBvhNode());
  DBvhNode nd;
  memset(&nd, 0, sizeof nd);
  Bx box, cb;
  for (int i = a; i < b; i++) {
    box.add(t[i].bmin);
    box.add(t[i].bmax);
    double c[3];
    for (int k = 0; k < 3; k++) c[k] = (t[i].bmin[k] + t[i].bmax[k]) * 0.5;
    cb.add(c);
  }
  for (int k = 0; k < 3; k++) {
    nd.lo[k] = box.mn[k] - (1e-5 + 1e-9 * fabs(box.mn[k]));
    nd.hi[k] = box.mx[k] + (1e-5 + 1e-9 * fabs(box.mx[k]));
  }
  if (b - a <= BVH_LEAF) {
    nd.tri_first = a;
    nd.tri_count = b - a;
    nd.skip = id + 1;
    out[id] = nd;
    return id;
  }
  int axis = 0;
  double ext = cb.mx[0] - cb.mn[0];
  for (int k = 1; k < 3; k++)
    if (cb.mx[k] - cb.mn[k] > ext) { axis = k; ext = cb.mx[k] - cb.mn[k]; }
  int mid = (a + b) / 2;
  std::nth_element(t.begin() + a, t.begin() + mid, t.begin() + b, [axis](const DTri &x, const DTri &y) {
    double cx = x.bmin[axis] + x.bmax[axis], cy = y.bmin[axis] + y.bmax[axis];
    return cx < cy || (cx == cy && x.idx < y.idx);
  });
  nd.tri_first = -1;
  nd.tri_count = 0;
  bvh_rec(t, a, mid, out);
  bvh_rec(t, mid, b, out);
  nd.skip = (int)out.size();
  out[id] = nd;
  return id;
}

// reorders `tris` into leaf order and appends the mesh's nodes; returns the root index, or -1
static int build_mesh_bvh(std::vector<DTri> &tris, std::vector<DBvhNode> &all) {
  if ((int)tris.size() < BVH_MIN_TRIS) return -1;
  std::vector<DBvhNode> nodes;
  bvh_rec(tris, 0, (int)tris.size(), nodes);
  int base = (int)all.size();
  all.insert(all.end(), nodes.begin(), nodes.end());  // skip links are relative to the root
  return base;
}

// pre-order flatten; returns the node's bbox in parent coordinates (R3SceneNode::UpdateBBox)
static Bx flatten(Graph &G, int gi_idx, int parent, HostScene &S) {
  GNode &g = G.nodes[gi_idx];
  int id = (int)S.nodes.size();
  DNode dn;
  memset(&dn, 0, sizeof dn);
  for (int i = 0; i < 12; i++) { dn.T[i] = g.T[i]; dn.Tinv[i] = g.Tinv[i]; }
  dn.parent = parent;
  dn.identity = g.identity ? 1 : 0;
  dn.elem_first = (int)S.elems.size();
  dn.elem_count = (int)g.elems.size();
  S.nodes.push_back(dn);
  Bx local;
  for (auto &e : g.elems) {
    DElement de;
    memset(&de, 0, sizeof de);
    de.material = e.mat;
    de.node = id;
    de.shape_first = (int)S.shapes.size();
    de.shape_count = (int)e.shapes.size();
    Bx eb;
    de.shapes_first_ok = 1;
    de.world = 1;
    for (int c = id; c >= 0; c = S.nodes[c].parent)
      if (!S.nodes[c].identity) de.world = 0;
    for (auto &s : e.shapes) {
      if (s.s.kind != SK_TRI && s.s.kind != SK_SPHERE && s.s.kind != SK_CIRCLE)
        de.shapes_first_ok = 0;
      shape_box(s);
      DShape ds = s.s;
      ds.bvh_first = -1;
      if (s.s.kind == SK_TRI || s.s.kind == SK_MESH) {
        std::vector<DTri> tris = s.tris;
        for (size_t i = 0; i < tris.size(); i++) tris[i].idx = (int32_t)i;
        if (s.s.kind == SK_MESH) ds.bvh_first = build_mesh_bvh(tris, S.bvh);
        ds.tri_first = (int)S.tris.size();
        ds.tri_count = (int)tris.size();
        S.tris.insert(S.tris.end(), tris.begin(), tris.end());
      }
      if (s.s.kind == SK_CONE) S.unsupported_shapes = true;
      S.shapes.push_back(ds);
      eb.add(s.s.bmin);
      eb.add(s.s.bmax);
    }
    for (int i = 0; i < 3; i++) {
      de.bmin[i] = eb.mn[i];
      de.bmax[i] = eb.mx[i];
      const double m = 1e-5 + 1e-9 * std::max(std::fabs(eb.mn[i]), std::fabs(eb.mx[i]));
      de.pmin[i] = eb.mn[i] - m;  // an empty box (+inf, -inf) stays empty
      de.pmax[i] = eb.mx[i] + m;
    }
    S.elems.push_back(de);
    local.add(eb);
  }
  // elements are contiguous per node only if children are appended after: gather children
  std::vector<int> kids = g.children;
  Bx kb;
  for (int c : kids) {
    Bx cb = flatten(G, c, id, S);
    kb.add(cb);
  }
  local.add(kb);
  Bx out;
  xform_box(g.T, local, out);
  return out;
}

}  // namespace

bool load_scene(const std::string &path, bool real, HostScene &S, std::string &err) {
  S = HostScene();
  Graph G;
  GNode root;
  for (int i = 0; i < 16; i++) root.T[i] = root.Tinv[i] = (i % 5 == 0) ? 1.0 : 0.0;
  G.nodes.push_back(root);
  size_t dp = path.rfind('.');
  if (dp == std::string::npos) { err = "Filename " + path + " has no extension (e.g., .txt)"; return false; }
  std::string ext = path.substr(dp);
  if (ext.compare(0, 4, ".scn") == 0) {
    if (!parse(G, 0, path, real, err)) return false;
  } else if (ext.compare(0, 4, ".off") == 0) {
    GNode child = root;
    GShape s;
    memset(&s.s, 0, sizeof s.s);
    s.s.kind = SK_MESH;
    if (!read_off(path, s.tris, err)) return false;
    G.mats.push_back(default_material());
    GElem e;
    e.mat = 0;
    e.shapes.push_back(std::move(s));
    child.elems.push_back(std::move(e));
    G.nodes.push_back(child);
    G.nodes[0].children.push_back(1);
  } else {
    err = "Unable to read file " + path + " (unrecognized extension: " + ext + ")";
    return false;
  }
  Bx sb = flatten(G, 0, -1, S);
  // per-node transform chain, root first (the device walks it per ray without a stack)
  for (size_t ni = 0; ni < S.nodes.size(); ni++) {
    int path[256];
    int d = 0;
    for (int c = (int)ni; c >= 0 && d < 256; c = S.nodes[c].parent) path[d++] = c;
    if (d > GI_MAX_DEPTH) {
      S.unsupported_depth = true;
      d = GI_MAX_DEPTH;
    }
    S.nodes[ni].depth = d;
    for (int k = 0; k < d; k++) S.nodes[ni].chain[k] = path[d - 1 - k];
  }
  S.mats = G.mats;
  S.lights = G.lights;
  for (int i = 0; i < 3; i++) {
    S.bmin[i] = sb.mn[i];
    S.bmax[i] = sb.mx[i];
    S.centroid[i] = (sb.mn[i] + sb.mx[i]) * 0.5;
    S.ambient[i] = G.ambient[i];
    S.background[i] = G.background[i];
  }
  S.radius = 0.5 * nrm(p3(sb.mx[0] - sb.mn[0], sb.mx[1] - sb.mn[1], sb.mx[2] - sb.mn[2]));
  // camera: R3Camera(e, t, u, xfov, xfov) with R3Triad(towards, up); default R3Scene.cpp:557-566
  P3 eye, towards, up;
  double xfov;
  if (G.has_camera) {
    eye = p3(G.cam[0], G.cam[1], G.cam[2]);
    towards = p3(G.cam[3], G.cam[4], G.cam[5]);
    up = p3(G.cam[6], G.cam[7], G.cam[8]);
    xfov = G.cam[9];
  } else {
    towards = p3(0, 0, -1);
    up = p3(0, 1, 0);
    P3 c = p3(S.centroid[0], S.centroid[1], S.centroid[2]);
    P3 off = scl(towards, 3 * S.radius);
    eye = sub(c, off);
    xfov = 0.25;
  }
  P3 z = unit(scl(towards, -1.0));
  P3 x = unit(crs(up, z));
  P3 y = crs(z, x);
  for (int i = 0; i < 3; i++) {
    S.eye[i] = eye.v[i];
    S.towards[i] = -z.v[i];
    S.right[i] = x.v[i];
    S.up[i] = y.v[i];
  }
  S.xfov = S.yfov = xfov;
  // default lights, R3Scene.cpp:569-583
  if (S.lights.empty()) {
    for (int k = 0; k < 2; k++) {
      DLight L;
      memset(&L, 0, sizeof L);
      L.kind = LK_DIR;
      L.active = 1;
      L.intensity = 1.0;
      P3 d = unit(k == 0 ? p3(-3, -4, -5) : p3(3, 2, 3));
      double c = k == 0 ? 1.0 : 0.5;
      for (int i = 0; i < 3; i++) { L.color[i] = c; L.dir[i] = d.v[i]; }
      S.lights.push_back(L);
    }
  }
  // per-light sampling frames
  for (auto &L : S.lights) {
    P3 n = p3(L.dir[0], L.dir[1], L.dir[2]);
    auto disk = [&](double rad) {  // illumination_utils.cpp:109-119 / photontracer.cpp:207-217
      P3 u = p3(n.v[1], -n.v[0], 0);
      if (1.0 - fabs(n.v[2]) < 0.1) u = p3(n.v[2], 0, -n.v[0]);
      P3 v = crs(u, n);
      u = scl(unit(u), rad);
      v = scl(unit(v), rad);
      for (int i = 0; i < 3; i++) { L.su[i] = u.v[i]; L.sv[i] = v.v[i]; }
    };
    if (L.kind == LK_AREA) {
      disk(L.radius);
      L.area = M_PI * pow(L.radius, 2.0);
      // R3AreaLight::DiffuseReflection axes (MinDimension, R3Vector.cpp:118-129)
      int dim = (fabs(n.v[0]) <= fabs(n.v[1])) ? ((fabs(n.v[0]) <= fabs(n.v[2])) ? 0 : 2)
                                               : ((fabs(n.v[1]) <= fabs(n.v[2])) ? 1 : 2);
      P3 e = p3(0, 0, 0);
      e.v[dim] = 1.0;
      P3 a1 = unit(crs(n, e));
      P3 a2 = unit(crs(n, a1));
      a1 = scl(a1, L.radius);
      a2 = scl(a2, L.radius);
      for (int i = 0; i < 3; i++) { L.nr_ax1[i] = a1.v[i]; L.nr_ax2[i] = a2.v[i]; }
    } else if (L.kind == LK_RECT) {
      P3 a1 = scl(p3(L.a1[0], L.a1[1], L.a1[2]), L.len1);
      P3 a2 = scl(p3(L.a2[0], L.a2[1], L.a2[2]), L.len2);
      for (int i = 0; i < 3; i++) {
        L.su[i] = a1.v[i]; L.sv[i] = a2.v[i];
        L.nr_ax1[i] = a1.v[i]; L.nr_ax2[i] = a2.v[i];
      }
      L.area = nrm(crs(a1, a2));
    } else if (L.kind == LK_DIR) {
      disk(S.radius);  // EmitPhotons directional disk, photontracer.cpp:198-233
    }
  }
  return true;
}

}  // namespace gi
