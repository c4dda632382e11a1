// dam_capi.cc — flat C ABI over the host adapter (include/deeparc_host.h).
#include <cstring>
#include <exception>
#include <string>
#include <unordered_map>

#include "../../include/deeparc_host.h"
#include "DeepArcManager.hh"
#include "DabScene.hh"
#include "sfm.hh"

struct dam_manager {
  DeepArcManager m;
};

namespace {
thread_local std::string g_err;
template <class F>
int guarded(F&& f) {
  g_err.clear();
  try {
    f();
    return 0;
  } catch (const char* e) {
    g_err = e;
  } catch (const std::exception& e) {
    g_err = e.what();
  } catch (...) {
    g_err = "unknown error";
  }
  return -1;
}
}  // namespace

extern "C" {

const char* dam_last_error(void) { return g_err.c_str(); }

int dam_create(dam_manager** out) {
  return guarded([&] {
    if (!out) throw "null output pointer";
    *out = new dam_manager();
  });
}
int dam_destroy(dam_manager* m) {
  delete m;
  return 0;
}
int dam_read(dam_manager* m, const char* path) { return guarded([&] { m->m.read(path); }); }
int dam_write(dam_manager* m, const char* path) { return guarded([&] { m->m.write(path); }); }
int dam_write_ply(dam_manager* m, const char* path) { return guarded([&] { m->m.writePly(path); }); }

int dam_sizes(dam_manager* m, int32_t* n_blocks, int32_t* n_points, int32_t* n_intr, int32_t* n_ext,
              int32_t* shared, int32_t* n_arc, int32_t* n_ring) {
  return guarded([&] {
    if (n_blocks) *n_blocks = (int32_t)m->m.parameters()->size();
    if (n_points) *n_points = (int32_t)m->m.point3ds()->size();
    if (n_intr) *n_intr = (int32_t)m->m.intrinsics()->size();
    if (n_ext) *n_ext = (int32_t)m->m.extrinsics()->size();
    if (shared) *shared = m->m.isShareExtrinsic() ? 1 : 0;
    if (n_arc) *n_arc = m->m.arcSize();
    if (n_ring) *n_ring = m->m.ringSize();
  });
}

int dam_get_points(dam_manager* m, double* xyz, int32_t* rgb) {
  return guarded([&] {
    auto& pts = *m->m.point3ds();
    for (size_t i = 0; i < pts.size(); ++i) {
      if (xyz) std::memcpy(xyz + 3 * i, pts[i]->position(), 3 * sizeof(double));
      if (rgb) {
        rgb[3 * i] = pts[i]->r();
        rgb[3 * i + 1] = pts[i]->g();
        rgb[3 * i + 2] = pts[i]->b();
      }
    }
  });
}

int dam_get_cameras(dam_manager* m, double* ext, double* intr) {
  return guarded([&] {
    auto& es = *m->m.extrinsics();
    for (size_t i = 0; ext && i < es.size(); ++i) {
      std::memcpy(ext + 6 * i, es[i]->rotation(), 3 * sizeof(double));
      std::memcpy(ext + 6 * i + 3, es[i]->translation(), 3 * sizeof(double));
    }
    auto& ks = *m->m.intrinsics();
    for (size_t i = 0; intr && i < ks.size(); ++i) {
      double* o = intr + 6 * i;
      o[0] = ks[i]->center()[0];
      o[1] = ks[i]->center()[1];
      o[2] = ks[i]->focal()[0];
      o[3] = ks[i]->focal_size() == 2 ? ks[i]->focal()[1] : 0.0;
      o[4] = ks[i]->distrotion_size() >= 1 ? ks[i]->distrotion()[0] : 0.0;
      o[5] = ks[i]->distrotion_size() >= 2 ? ks[i]->distrotion()[1] : 0.0;
    }
  });
}

int dam_get_blocks(dam_manager* m, int32_t* pos_arc, int32_t* pos_ring, int32_t* point_index, double* xy) {
  return guarded([&] {
    auto& pts = *m->m.point3ds();
    std::unordered_map<Point3d*, int32_t> idx;
    for (size_t i = 0; i < pts.size(); ++i) idx[pts[i]] = (int32_t)i;
    auto& bs = *m->m.parameters();
    for (size_t o = 0; o < bs.size(); ++o) {
      if (pos_arc) pos_arc[o] = bs[o]->pos_arc();
      if (pos_ring) pos_ring[o] = bs[o]->pos_ring();
      if (point_index) {
        auto it = idx.find(bs[o]->point3d());
        point_index[o] = it == idx.end() ? -1 : it->second;
      }
      if (xy) {
        xy[2 * o] = bs[o]->point2d()->x();
        xy[2 * o + 1] = bs[o]->point2d()->y();
      }
    }
  });
}

int dam_solve(dam_manager* m, int32_t max_iteration, int32_t max_second, int32_t freeze_camera,
              int32_t linear_solver_type, dab_summary* summary) {
  return guarded([&] {
    dab_options o;
    dab_options_init(&o);
    o.linear_solver_type = linear_solver_type;
    o.max_num_iterations = max_iteration;
    o.max_solver_time_in_seconds = max_second;
    dab_check(solveWith(m->m, o, freeze_camera != 0, summary));
  });
}

int dam_filter(dam_manager* m, double error_boundary, const double center[3], double radius) {
  return guarded([&] {
    double c[3] = {center[0], center[1], center[2]};
    m->m.filterPoint3d(error_boundary, c, radius);
  });
}

int dam_camera_centers(dam_manager* m, double* out, int32_t capacity, int32_t* count) {
  return guarded([&] {
    auto cs = m->m.getCameraCenter();
    if (count) *count = (int32_t)cs.size();
    for (size_t i = 0; out && i < cs.size() && (int32_t)i < capacity; ++i)
      for (int k = 0; k < 3; ++k) out[3 * i + k] = cs[i][k];
  });
}

int dam_fit_hemisphere(const double* centers, int32_t n, double center[3], double* radius, int32_t max_iteration) {
  return guarded([&] {
    std::vector<std::vector<double> > cs((size_t)n, std::vector<double>(3));
    for (int32_t i = 0; i < n; ++i)
      for (int k = 0; k < 3; ++k) cs[i][k] = centers[3 * i + k];
    fitHemisphere(cs, center, radius, max_iteration);
  });
}

int dam_run_pipeline(const char* input, const char* output, const char* ply_prefix, int32_t max_iteration,
                     int32_t max_second, double error_boundary, double hemi_out[4], int32_t counts_out[3]) {
  return guarded([&] {
    PipelineReport r = runPipeline(input, output ? output : "", ply_prefix ? ply_prefix : "", max_iteration,
                                   max_second, error_boundary);
    if (hemi_out) {
      for (int k = 0; k < 3; ++k) hemi_out[k] = r.hemisphere_center[k];
      hemi_out[3] = r.hemisphere_radius;
    }
    if (counts_out) {
      counts_out[0] = r.rounds;
      counts_out[1] = r.final_blocks;
      counts_out[2] = r.final_points;
    }
  });
}

int dam_run_pipeline_report(const char* input, const char* output, const char* ply_prefix, int32_t max_iteration,
                            int32_t max_second, double error_boundary, int32_t quiet, dam_pipeline_report* out) {
  return guarded([&] {
    PipelineReport r = runPipeline(input, output ? output : "", ply_prefix ? ply_prefix : "", max_iteration,
                                   max_second, error_boundary, quiet == 0);
    if (out) {
      for (int k = 0; k < 3; ++k) out->hemisphere_center[k] = r.hemisphere_center[k];
      out->hemisphere_radius = r.hemisphere_radius;
      out->rounds = r.rounds;
      out->final_blocks = r.final_blocks;
      out->final_points = r.final_points;
      out->solves = r.solves;
      out->lm_iterations = r.lm_iterations;
      out->reserved = 0;
      out->final_cost = r.final_cost;
      out->solve_seconds = r.solve_seconds;
      out->filter_seconds = r.filter_seconds;
      out->total_seconds = r.total_seconds;
      out->read_seconds = r.read_seconds;
      out->fit_seconds = r.fit_seconds;
      out->write_seconds = r.write_seconds;
      out->marshal_seconds = r.marshal_seconds;
      out->setup_seconds = r.setup_seconds;
      out->update_seconds = r.update_seconds;
      out->prep_seconds = r.prep_seconds;
      out->lm_seconds = r.lm_seconds;
      out->writeback_seconds = r.writeback_seconds;
      out->filter_device_seconds = r.filter_device_seconds;
      out->filter_host_seconds = r.filter_host_seconds;
    }
  });
}

}  // extern "C"
