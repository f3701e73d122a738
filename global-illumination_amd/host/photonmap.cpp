// photonmap.cpp -- drop-in CLI: `photonmap src.scn out.png [-FLAGS]` on the MI355X path.
//
// Same control flow and reports as the reference main (photonmap.cpp:442-499):
// ParseArgs -> ReadScene -> MapPhotons (if indirect|caustic|photon_viz) -> RenderImage ->
// WriteImage, with the -v statistics of io_utils.cpp:240-246, photonmap.cpp:416-435 and
// render.cpp:224-255. Exit codes: 1 for a bad flag, -1 (255) for load/render/write failures.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../../include/gi.h"

// PrintProgress (io_utils.cpp:257-268) with the reference's bar width (photonmap.cpp:132);
// a bar is redrawn when its percentage changes (render.cpp:82-86, photontracer.cpp:168-173)
static const int PROGRESS_BAR_WIDTH = 50;
static void PrintProgress(double progress, int width) {
  printf("[");
  int pos = (int)(width * progress);
  for (int j = 0; j < width; j++) printf("%s", j < pos ? "=" : (j == pos ? ">" : " "));
  printf("] %d%%\r", (int)(progress * 100.0));
  fflush(stdout);
}
struct ProgressState {
  bool verbose;
  int last[3];
};
static void OnProgress(int stage, double progress, void *user) {
  ProgressState *s = (ProgressState *)user;
  if (stage > 0 && !s->verbose) return;  // photon-map bars only with -v (photonmap.cpp:193)
  const int v = (int)(progress * 100.0);
  if (stage == 0 && v >= 100) return;  // the final bar is printed after RenderImage returns
  if (v == s->last[stage]) return;
  s->last[stage] = v;
  PrintProgress(progress, PROGRESS_BAR_WIDTH);
}

int main(int argc, char **argv) {
  gi_params P;
  gi_params_default(&P);
  const char *scene = nullptr, *out = nullptr, *err = nullptr;
  int w = 1024, h = 1024, aa = 2, real = 0;
  int rc = gi_parse_args(argc, argv, &P, &scene, &out, &w, &h, &aa, &real, &err);
  if (rc == GI_ERR_ARG) {
    fprintf(stderr, "%s", err);
    return 1;
  }
  if (rc != GI_OK) {
    fprintf(stderr, "%s\n", err);
    return -1;
  }
  // devices: -gpus N takes devices 0..N-1 (the reference's -threads N re-cut as a device
  // shard); GI_DEVICES="a,b,..." names them explicitly, GI_DEVICE the single device
  gi_device_set ds;
  memset(&ds, 0, sizeof ds);
  ds.count = 1;
  if (const char *d = getenv("GI_DEVICE")) ds.devices[0] = atoi(d);
  if (P.gpus > 1) {
    ds.count = P.gpus < GI_MAX_DEVICES ? P.gpus : GI_MAX_DEVICES;
    for (int k = 0; k < ds.count; k++) ds.devices[k] = k;
  }
  if (const char *l = getenv("GI_DEVICES")) {
    ds.count = 0;
    for (const char *q = l; *q && ds.count < GI_MAX_DEVICES;) {
      ds.devices[ds.count++] = atoi(q);
      while (*q && *q != ',') q++;
      if (*q == ',') q++;
    }
    if (ds.count == 0) ds.count = 1;
  }
  gi_ctx *ctx = nullptr;
  if (gi_create_devices(&ctx, &ds) != GI_OK) {
    fprintf(stderr, "Unable to initialise %d HIP device(s) starting at %d\n", ds.count, ds.devices[0]);
    return -1;
  }
  gi_set_params(ctx, &P);
  ProgressState prog = {P.verbose != 0, {-1, -1, -1}};
  gi_set_progress(ctx, OnProgress, &prog);
  auto t0 = std::chrono::steady_clock::now();
  if (gi_read_scene(ctx, scene, real) != GI_OK) {
    fprintf(stderr, "%s\n", gi_last_error(ctx));
    gi_destroy(ctx);
    return -1;
  }
  if (P.verbose) {
    int nn = 0, nl = 0;
    gi_scene_info(ctx, &nn, &nl, nullptr, nullptr);
    printf("Read scene from %s ...\n", scene);
    printf("  Time = %.2f seconds\n",
           std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    printf("  # Nodes = %d\n", nn);
    printf("  # Lights = %d\n", nl);
    fflush(stdout);
  }
  if (P.indirect_illum || P.caustic_illum || P.direct_photon_illum) {
    gi_photon_stats ps;
    if (gi_map_photons(ctx, &ps) != GI_OK) {
      fprintf(stderr, "%s\n", gi_last_error(ctx));
      gi_destroy(ctx);
      return -1;
    }
    if (prog.last[1] >= 0 || prog.last[2] >= 0) printf("\n");  // photonmap.cpp:196
    if (P.verbose) {
      printf("Built photon map ...\n");
      printf("  Total Time = %.2f seconds\n", ps.total_s);
      printf("  Photon Tracing = %.2f seconds\n", ps.trace_s);
      printf("  KdTree Construction = %.2f seconds\n", ps.kd_s);
      if (P.irradiance_cache) printf("  Irradiance Cache Computation = %.2f seconds\n", ps.irradiance_s);
      if (P.indirect_illum || P.direct_photon_illum)
        printf("  # Global Photons Stored = %lld\n", (long long)ps.global_stored);
      if (P.caustic_illum) printf("  # Caustic Photons Stored = %lld\n", (long long)ps.caustic_stored);
      printf("Total Photons Stored: %lld\n", (long long)(ps.global_stored + ps.caustic_stored));
      fflush(stdout);
    }
  }
  std::vector<uint8_t> rgb((size_t)w * h * 3);
  gi_render_stats rs;
  if (P.verbose) printf("Rendering image ...\n");
  if (gi_render_image(ctx, aa, w, h, rgb.data(), nullptr, &rs) != GI_OK) {
    fprintf(stderr, "%s\n", gi_last_error(ctx));
    gi_destroy(ctx);
    return -1;
  }
  PrintProgress(1.0, PROGRESS_BAR_WIDTH);  // render.cpp:201-202
  printf("\n");
  fflush(stdout);
  if (P.verbose) {
    unsigned long long total = rs.screen_rays;
    printf("Rendered image ...\n");
    printf("  Time = %.2f seconds\n", rs.render_s);
    printf("  # Screen Rays = %llu\n", (unsigned long long)rs.screen_rays);
    if (P.shadows) { printf("  # Shadow Rays = %llu\n", (unsigned long long)rs.shadow_rays); total += rs.shadow_rays; }
    if (P.monte_carlo) { printf("  # Monte Carlo Rays = %llu\n", (unsigned long long)rs.monte_carlo_rays); total += rs.monte_carlo_rays; }
    if (P.transmissive_illum) { printf("  # Transmissive Samples = %llu\n", (unsigned long long)rs.transmissive_samples); total += rs.transmissive_samples; }
    if (P.specular_illum) { printf("  # Specular Samples = %llu\n", (unsigned long long)rs.specular_samples); total += rs.specular_samples; }
    if (P.indirect_illum) { printf("  # Indirect Samples = %llu\n", (unsigned long long)rs.indirect_samples); total += rs.indirect_samples; }
    if (P.caustic_illum) { printf("  # Caustic Samples = %llu\n", (unsigned long long)rs.caustic_samples); total += rs.caustic_samples; }
    printf("Total Rays: %llu\n", total);
    fflush(stdout);
  }
  gi_destroy(ctx);
  auto tw = std::chrono::steady_clock::now();
  if (gi_write_image(out, w, h, rgb.data()) != GI_OK) {
    const char *ext = strrchr(out, '.');
    if (ext && !strncmp(ext, ".tif", 4)) fprintf(stderr, "TIFF not supported\n");  // R2Image.cpp:1300
    else fprintf(stderr, "Unable to write image %s\n", out);
    return -1;
  }
  if (P.verbose) {
    printf("Wrote image to %s ...\n", out);
    printf("  Time = %.2f seconds\n",
           std::chrono::duration<double>(std::chrono::steady_clock::now() - tw).count());
    printf("  Width = %d\n", w);
    printf("  Height = %d\n", h);
    fflush(stdout);
  }
  return 0;
}
