// gi_args.cpp -- host-only pieces of the C-ABI: flag parsing (the drop-in CLI surface) and
// image output.
//   gi_params_default   defaults of photonmap.cpp:27-106
//   gi_parse_args       ParseArgs, utils/io_utils.cpp:16-212 (same flags, clamps, messages;
//                       extensions: -seed S, -gpus N)
//   (gi_write_image, R2Image::Write, is in gi_image.cpp)
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include <zlib.h>
#include "../../include/gi.h"

extern "C" {

void gi_params_default(gi_params *P) {
  memset(P, 0, sizeof *P);
  P->verbose = 0;
  P->threads = 1;
  P->fresnel = 1;
  P->ir_air = 1.0;
  P->ambient = 1;
  P->direct_illum = 1;
  P->transmissive_illum = 1;
  P->specular_illum = 1;
  P->indirect_illum = 1;
  P->caustic_illum = 1;
  P->direct_photon_illum = 0;
  P->fast_global = 0;
  P->irradiance_cache = 0;
  P->shadows = 1;
  P->soft_shadows = 1;
  P->light_test = 128;
  P->shadow_test = 128;
  P->monte_carlo = 1;
  P->max_monte_depth = 128;
  P->prob_absorb = 0.005;
  P->recursive_shadows = 1;
  P->distrib_transmissive = 1;
  P->transmissive_test = 128;
  P->distrib_specular = 1;
  P->specular_test = 128;
  P->depth_of_field = 0;
  P->dof_test = 1;
  P->focus_depth = 100.0;
  P->aperture_radius = 0.025;
  P->global_photon_count = 2176;
  P->caustic_photon_count = 10000000;
  P->max_photon_depth = 128;
  P->indirect_test = 256;
  P->global_estimate_size = 50;
  P->global_estimate_dist = 2.5;
  P->global_filter = GI_FILTER_DISK;
  P->caustic_estimate_size = 225;
  P->caustic_estimate_dist = 0.225;
  P->caustic_filter = GI_FILTER_DISK;
  P->filter_const_a = 0.918;
  P->filter_const_b = 1.953;
  P->filter_const_k = 1.0;
  P->seed = 1;
}

int gi_parse_args(int argc, char **argv, gi_params *P, const char **scene, const char **out,
                  int *w, int *h, int *aa, int *real, const char **err) {
  static std::string msg;
  const double EPS = 1.0e-6;
  *scene = nullptr;
  *out = nullptr;
  argc--;
  argv++;
  auto bad = [&](const char *a) {
    msg = std::string("Invalid program argument: ") + a;
    if (err) *err = msg.c_str();
    return GI_ERR_ARG;
  };
  while (argc > 0) {
    const char *a = *argv;
    auto need = [&](int n) { return argc > n; };
    auto next = [&]() { argc--; argv++; return *argv; };
    if (a[0] == '-') {
      if (!strcmp(a, "-v")) P->verbose = 1;
      else if (!strcmp(a, "-threads") && need(1)) { P->threads = (int)atof(next()); if (P->threads <= 0) P->threads = 1; }
      else if (!strcmp(a, "-aa") && need(1)) { *aa = atoi(next()); if (*aa < 0) *aa *= -1; }
      else if (!strcmp(a, "-real")) *real = 1;
      else if (!strcmp(a, "-no_fresnel")) P->fresnel = 0;
      else if (!strcmp(a, "-ir") && need(1)) { P->ir_air = atof(next()); if (P->ir_air <= 0) P->ir_air = EPS; }
      else if (!strcmp(a, "-no_ambient")) P->ambient = 0;
      else if (!strcmp(a, "-no_direct")) P->direct_illum = 0;
      else if (!strcmp(a, "-no_transmissive")) P->transmissive_illum = 0;
      else if (!strcmp(a, "-no_specular")) P->specular_illum = 0;
      else if (!strcmp(a, "-no_indirect")) P->indirect_illum = 0;
      else if (!strcmp(a, "-no_caustic")) P->caustic_illum = 0;
      else if (!strcmp(a, "-photon_viz")) P->direct_photon_illum = 1;
      else if (!strcmp(a, "-fast_global")) { P->fast_global = 1; P->direct_photon_illum = 1; P->indirect_illum = 0; }
      else if (!strcmp(a, "-cache")) P->irradiance_cache = 1;
      else if (!strcmp(a, "-no_monte")) P->monte_carlo = 0;
      else if (!strcmp(a, "-md") && need(1)) { P->max_monte_depth = atoi(next()); if (P->max_monte_depth < 1) P->max_monte_depth = 1; }
      else if (!strcmp(a, "-absorb") && need(1)) { P->prob_absorb = atof(next()); if (P->prob_absorb < 0) P->prob_absorb = 0; }
      else if (!strcmp(a, "-no_rs")) P->recursive_shadows = 0;
      else if (!strcmp(a, "-no_dt")) P->distrib_transmissive = 0;
      else if (!strcmp(a, "-tt") && need(1)) { P->transmissive_test = atoi(next()); if (P->transmissive_test < 1) P->transmissive_test = 1; }
      else if (!strcmp(a, "-no_ds")) P->distrib_specular = 0;
      else if (!strcmp(a, "-st") && need(1)) { P->specular_test = atoi(next()); if (P->specular_test < 1) P->specular_test = 1; }
      else if (!strcmp(a, "-global") && need(1)) { P->global_photon_count = atoi(next()); if (P->global_photon_count < 1) P->global_photon_count = 1; }
      else if (!strcmp(a, "-caustic") && need(1)) { P->caustic_photon_count = atoi(next()); if (P->caustic_photon_count < 1) P->caustic_photon_count = 1; }
      else if (!strcmp(a, "-pd") && need(1)) { P->max_photon_depth = atoi(next()); if (P->max_photon_depth < 1) P->max_photon_depth = 1; }
      else if (!strcmp(a, "-it") && need(1)) { P->indirect_test = atoi(next()); if (P->indirect_test < 1) P->indirect_test = 1; }
      else if (!strcmp(a, "-gs") && need(1)) { P->global_estimate_size = atoi(next()); if (P->global_estimate_size < 1) P->global_estimate_size = 1; }
      else if (!strcmp(a, "-gd") && need(1)) { P->global_estimate_dist = atof(next()); if (P->global_estimate_dist < 0.0) P->global_estimate_dist = EPS; }
      else if (!strcmp(a, "-gf") && need(1)) {
        const char *f = next();
        if (!strcmp(f, "cone") && need(1)) { P->global_filter = GI_FILTER_CONE; P->filter_const_k = atof(next()); if (P->filter_const_k < 1) P->filter_const_k = 1; }
        else if (!strcmp(f, "gauss")) P->global_filter = GI_FILTER_GAUSS;
      }
      else if (!strcmp(a, "-cs") && need(1)) { P->caustic_estimate_size = atoi(next()); if (P->caustic_estimate_size < 1) P->caustic_estimate_size = 1; }
      else if (!strcmp(a, "-cd") && need(1)) { P->caustic_estimate_dist = atof(next()); if (P->caustic_estimate_dist < 0.0) P->caustic_estimate_dist = EPS; }
      else if (!strcmp(a, "-cf") && need(1)) {
        const char *f = next();
        if (!strcmp(f, "cone") && need(1)) { P->caustic_filter = GI_FILTER_CONE; P->filter_const_k = atof(next()); if (P->filter_const_k < 1) P->filter_const_k = 1; }
        else if (!strcmp(f, "gauss")) P->caustic_filter = GI_FILTER_GAUSS;
      }
      else if (!strcmp(a, "-no_shadow")) P->shadows = 0;
      else if (!strcmp(a, "-no_ss")) P->soft_shadows = 0;
      else if (!strcmp(a, "-lt") && need(1)) { P->light_test = atoi(next()); if (P->light_test < 1) P->light_test = 1; }
      else if (!strcmp(a, "-ss") && need(1)) { P->shadow_test = atoi(next()); if (P->shadow_test < 0) P->shadow_test = 0; }
      else if (!strcmp(a, "-dof") && need(3)) {
        P->depth_of_field = 1;
        P->dof_test = atoi(next());
        P->focus_depth = atof(next());
        P->aperture_radius = atof(next());
        if (P->dof_test < 1) P->dof_test = 1;
        if (P->focus_depth < EPS) P->focus_depth = EPS;
        if (P->aperture_radius <= 0) P->aperture_radius = EPS;
      }
      else if (!strcmp(a, "-resolution") && need(2)) {
        *w = atoi(next());
        *h = atoi(next());
        if (*w < 0) *w *= -1;
        if (*h < 0) *h *= -1;
      }
      else if (!strcmp(a, "-seed") && need(1)) P->seed = strtoull(next(), nullptr, 10);
      else if (!strcmp(a, "-gpus") && need(1)) P->gpus = atoi(next());
      else return bad(a);
      argv++;
      argc--;
    } else {
      if (!*scene) *scene = a;
      else if (!*out) *out = a;
      else return bad(a);
      argv++;
      argc--;
    }
  }
  if (!*scene || !*out) {
    msg = "Usage: photonmap inputscenefile outputimagefile [-FLAGS]";
    if (err) *err = msg.c_str();
    return GI_ERR_STATE;
  }
  return GI_OK;
}

}  // extern "C"
