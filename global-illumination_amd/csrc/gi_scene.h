// gi_scene.h -- host-side scene description (flattened for the device) and loader.
#pragma once
#include <string>
#include <vector>
#include "gi_layout.h"

namespace gi {

struct HostScene {
  std::vector<DNode> nodes;
  std::vector<DElement> elems;
  std::vector<DShape> shapes;
  std::vector<DTri> tris;
  std::vector<DBvhNode> bvh;  // per-mesh BVHs (DShape::bvh_first)
  std::vector<DMaterial> mats;
  std::vector<DLight> lights;
  // camera (R3Camera: eye + triad, R3Triad.cpp:72-79); xfov = yfov (Q5)
  double eye[3], towards[3], right[3], up[3];
  double xfov = 0.25, yfov = 0.25;
  double ambient[3] = {0, 0, 0}, background[3] = {0, 0, 0};
  double bmin[3], bmax[3];
  double radius = 0, centroid[3] = {0, 0, 0};
  bool unsupported_shapes = false;  // cone present
  bool unsupported_depth = false;   // scene graph deeper than GI_MAX_DEPTH
};

// ReadScene (utils/io_utils.cpp:219-250) -> R3Scene::ReadFile (R3Scene.cpp:514-587)
bool load_scene(const std::string &path, bool real_material, HostScene &out, std::string &err);

}  // namespace gi
