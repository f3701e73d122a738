// oracle_scene.h -- TEST INFRASTRUCTURE ONLY. Scene graph, .scn/.off loader and ray
// intersection restated from the reference's GAPS R3Graphics / R3Shapes layers.
#pragma once
#include "oracle_core.h"
#include <string>

namespace oracle {

// R3Box (min/max corners); null box = R3null_box
struct Box {
  V3 mn{FLT_MAX, FLT_MAX, FLT_MAX}, mx{-FLT_MAX, -FLT_MAX, -FLT_MAX};
  bool empty() const { return mn.x > mx.x || mn.y > mx.y || mn.z > mx.z; }
  void add(V3 p) {
    for (int i = 0; i < 3; i++) {
      if (p[i] < mn[i]) mn[i] = p[i];
      if (p[i] > mx[i]) mx[i] = p[i];
    }
  }
  void add(const Box &b) {
    if (b.empty()) return;
    add(b.mn);
    add(b.mx);
  }
  V3 centroid() const { return (mn + mx) * 0.5; }
  double diag_radius() const { return 0.5 * length(mx - mn); }
};

// 4x4 affine (R4Matrix row-major, R3Affine)
struct M4 {
  double m[4][4];
  static M4 identity() {
    M4 r;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) r.m[i][j] = (i == j) ? 1.0 : 0.0;
    return r;
  }
  V3 point(V3 p) const {
    return V3(m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3],
              m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3],
              m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3]);
  }
  V3 vec(V3 v) const {
    return V3(m[0][0] * v.x + m[0][1] * v.y + m[0][2] * v.z,
              m[1][0] * v.x + m[1][1] * v.y + m[1][2] * v.z,
              m[2][0] * v.x + m[2][1] * v.y + m[2][2] * v.z);
  }
  M4 inverse() const;
};

struct Tri {
  V3 p[3];
  V3 n;       // plane normal (R3Plane(p0,p1,p2), R3Plane.cpp)
  double d;   // plane offset
  Box box;
};
Tri make_tri(V3 a, V3 b, V3 c);

enum ShapeType { SH_TRI = 0, SH_MESH = 1, SH_SPHERE = 2, SH_BOX = 3, SH_CIRCLE = 4,
                 SH_CYLINDER = 5, SH_CONE = 6 };
struct Shape {
  int type = SH_TRI;
  Tri tri;                 // SH_TRI
  std::vector<Tri> tris;   // SH_MESH (R3TriangleArray)
  V3 c;                    // sphere/circle centre, cylinder/cone base point
  V3 axis;                 // circle normal; cylinder/cone p2
  double r = 0;            // radius
  Box box;                 // shape bbox
};

struct Brdf {
  Rgb ka, kd, ks, kt, e;
  double n = 0, ir = 1;
  bool isAmbient() const { return !ka.black(); }
  bool isDiffuse() const { return !kd.black(); }
  bool isSpecular() const { return !ks.black(); }
  bool isTransparent() const { return !kt.black(); }
};

struct Element {
  int material = -1;  // index into Scene::materials
  std::vector<Shape> shapes;
  Box bbox;
};

struct Node {
  M4 T, Tinv;
  std::vector<Element> elements;
  std::vector<int> children;
  Box bbox;  // in parent coordinates (R3SceneNode::UpdateBBox)
};

enum LightType { L_DIR = 0, L_POINT = 1, L_SPOT = 2, L_AREA = 3, L_RECT = 4 };
struct Light {
  int type = L_POINT;
  Rgb color;
  double intensity = 1.0;
  bool active = true;
  V3 pos, dir;                 // dir: directional / spot / area normal / rect normal
  double ca = 0, la = 0, qa = 0;
  double dropoff = 0, cutoff = 0;  // spot
  double radius = 0;               // area
  V3 a1, a2;                       // rect axes (normalized)
  double len1 = 0, len2 = 0;
};

struct Camera {
  V3 eye, towards, up, right;
  double xfov = 0.25, yfov = 0.25;
};

struct Scene {
  std::vector<Node> nodes;  // nodes[0] = root
  std::vector<Brdf> materials;
  std::vector<Light> lights;
  Camera camera;
  bool has_camera = false;
  Rgb ambient, background;
  Box bbox;
  double radius = 0;
  V3 centroid;
};

// ReadScene (io_utils.cpp:219-250) -> R3Scene::ReadFile (R3Scene.cpp:514-587)
bool read_scene(const std::string &path, bool real_material, Scene &scene, std::string &err);

struct Hit {
  V3 point, normal;
  double t = 0;
  int material = -1;  // -1 => R3default_material
};
// R3Scene::Intersects (R3Scene.cpp:471-479), min_t = 0, max_t = RN_INFINITY
bool scene_intersect(const Scene &s, V3 org, V3 dir, Hit &h);

// R3Intersects(ray, box) (R3Isect.cpp:883-942)
int ray_box(V3 org, V3 dir, const Box &b, double *t, V3 *normal);

}  // namespace oracle
