// DabScene.cc — DeepArcManager <-> dab_problem marshalling (see DabScene.hh).
#include "DabScene.hh"

#include <chrono>
#include <cstdlib>

double dab_now_seconds() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void dab_check(int rc) {
  if (rc != 0) throw dab_last_error();
}

DabHandle::DabHandle() {
  const char* env = std::getenv("DAB_DEVICE");
  dab_check(dab_create(env ? std::atoi(env) : 0, &h));
}
DabHandle::~DabHandle() {
  if (h) dab_destroy(h);
}

void DabScene::build(DeepArcManager& m, bool freeze_camera) {
  std::vector<ParameterBlock*>& blocks = *m.parameters();
  std::vector<Point3d*>& pts = *m.point3ds();
  std::vector<Extrinsic*>& exts = *m.extrinsics();
  std::vector<Intrinsic*>& ks = *m.intrinsics();
  // index of every parameter in the manager's lists, kept on the objects themselves (one
  // store each, no hashing); a block whose parameter is not at its recorded index in this
  // manager references a foreign parameter
  for (size_t i = 0; i < pts.size(); ++i) pts[i]->slot((int)i);
  for (size_t i = 0; i < exts.size(); ++i) exts[i]->slot((int)i);
  for (size_t i = 0; i < ks.size(); ++i) ks[i]->slot((int)i);
  auto find = [](auto& list, auto* key) {
    const int i = key ? key->slot() : -1;
    if (i < 0 || (size_t)i >= list.size() || list[i] != key)
      throw "Parameter block references a parameter outside the manager";
    return i;
  };
  const size_t N = blocks.size();
  xy.resize(2 * N);
  obs_point.resize(N);
  obs_ext0.resize(N);
  obs_ext1.resize(N);
  obs_intr.resize(N);
  ext_const.assign(exts.size(), 0);
  obs_gauge.resize(N);
  for (size_t o = 0; o < N; ++o) {
    ParameterBlock* b = blocks[o];
    xy[2 * o] = b->point2d()->x();
    xy[2 * o + 1] = b->point2d()->y();
    obs_point[o] = find(pts, b->point3d());
    obs_intr[o] = find(ks, b->intrinsic());
    obs_ext0[o] = find(exts, b->first_extrinsic());
    Extrinsic* e1 = b->second_extrinsic();
    obs_ext1[o] = e1 ? find(exts, e1) : -1;
    // gauge: the extrinsic of a (0,0) block is constant (sfm.cc:50-53)
    obs_gauge[o] = b->pos_arc() == 0 && b->pos_ring() == 0;
    if (obs_gauge[o]) ext_const[obs_ext0[o]] = 1;
  }
  points.resize(3 * pts.size());
  for (size_t i = 0; i < pts.size(); ++i)
    for (int k = 0; k < 3; ++k) points[3 * i + k] = pts[i]->position()[k];
  ext.resize(6 * exts.size());
  for (size_t i = 0; i < exts.size(); ++i)
    for (int k = 0; k < 3; ++k) {
      ext[6 * i + k] = exts[i]->rotation()[k];
      ext[6 * i + 3 + k] = exts[i]->translation()[k];
    }
  intr.assign(6 * ks.size(), 0.0);
  intr_nf.resize(ks.size());
  intr_nk.resize(ks.size());
  for (size_t i = 0; i < ks.size(); ++i) {
    Intrinsic* k = ks[i];
    intr_nf[i] = k->focal_size();
    intr_nk[i] = k->distrotion_size();
    double* o = &intr[6 * i];
    o[0] = k->center()[0];
    o[1] = k->center()[1];
    o[2] = k->focal()[0];
    o[3] = intr_nf[i] == 2 ? k->focal()[1] : 0.0;
    o[4] = intr_nk[i] >= 1 ? k->distrotion()[0] : 0.0;
    o[5] = intr_nk[i] >= 2 ? k->distrotion()[1] : 0.0;
  }
  bind(freeze_camera);
}

void DabScene::bind(bool freeze_camera) {
  problem = dab_problem{};
  problem.num_obs = (int32_t)obs_point.size();
  problem.num_points = (int32_t)(points.size() / 3);
  problem.num_ext = (int32_t)(ext.size() / 6);
  problem.num_intr = (int32_t)intr_nf.size();
  problem.obs_xy = xy.data();
  problem.obs_point = obs_point.data();
  problem.obs_ext0 = obs_ext0.data();
  problem.obs_ext1 = obs_ext1.data();
  problem.obs_intr = obs_intr.data();
  problem.points = points.data();
  problem.ext = ext.data();
  problem.intr = intr.data();
  problem.intr_nf = intr_nf.data();
  problem.intr_nk = intr_nk.data();
  problem.ext_const = ext_const.data();
  problem.freeze_camera = freeze_camera ? 1 : 0;
}

bool DabScene::compact(const uint8_t* keep_obs, const uint8_t* keep_pt) {
  const size_t N = obs_point.size(), NP = points.size() / 3;
  std::vector<int32_t> remap(NP, -1);
  size_t w = 0;
  for (size_t i = 0; i < NP; ++i)
    if (keep_pt[i]) {
      remap[i] = (int32_t)w;
      for (int k = 0; k < 3; ++k) points[3 * w + k] = points[3 * i + k];
      ++w;
    }
  points.resize(3 * w);
  std::fill(ext_const.begin(), ext_const.end(), 0);
  w = 0;
  for (size_t o = 0; o < N; ++o) {
    if (!keep_obs[o]) continue;
    const int32_t p = remap[obs_point[o]];
    if (p < 0) return false;  // an observation of a removed point: the caller rebuilds
    xy[2 * w] = xy[2 * o];
    xy[2 * w + 1] = xy[2 * o + 1];
    obs_point[w] = p;
    obs_ext0[w] = obs_ext0[o];
    obs_ext1[w] = obs_ext1[o];
    obs_intr[w] = obs_intr[o];
    obs_gauge[w] = obs_gauge[o];
    if (obs_gauge[w]) ext_const[obs_ext0[w]] = 1;
    ++w;
  }
  xy.resize(2 * w);
  obs_point.resize(w);
  obs_ext0.resize(w);
  obs_ext1.resize(w);
  obs_intr.resize(w);
  obs_gauge.resize(w);
  return true;
}

void DabScene::refresh_values(DeepArcManager& m) {
  std::vector<Point3d*>& pts = *m.point3ds();
  std::vector<Extrinsic*>& exts = *m.extrinsics();
  for (size_t i = 0; i < pts.size(); ++i)
    for (int k = 0; k < 3; ++k) points[3 * i + k] = pts[i]->position()[k];
  for (size_t i = 0; i < exts.size(); ++i)
    for (int k = 0; k < 3; ++k) {
      ext[6 * i + k] = exts[i]->rotation()[k];
      ext[6 * i + 3 + k] = exts[i]->translation()[k];
    }
}

int DabSession::ensure(DeepArcManager& m, int want_freeze) {
  const bool same = resident && version == m.structureVersion() && n_blocks == m.parameters()->size() &&
                    n_points == m.point3ds()->size() && n_ext == m.extrinsics()->size() &&
                    n_intr == m.intrinsics()->size() && (want_freeze < 0 || (want_freeze != 0) == freeze);
  double t0 = dab_now_seconds();
  if (same) {  // structure resident: the values may have changed on the host
    scene.refresh_values(m);
    const int rc = dab_update_parameters(handle.h, scene.points.data(), scene.ext.data());
    if (rc) resident = false;  // the handle's state is unknown: the next call re-sets the problem
    t.update += dab_now_seconds() - t0;
    return rc;
  }
  resident = false;
  freeze = want_freeze > 0;
  if (scene_valid && scene_version == m.structureVersion() && scene.obs_point.size() == m.parameters()->size() &&
      scene.points.size() == 3 * m.point3ds()->size() && scene.ext.size() == 6 * m.extrinsics()->size() &&
      scene.intr_nf.size() == m.intrinsics()->size()) {
    scene.refresh_values(m);  // the arrays are the compacted ones: only the values may differ
    scene.bind(freeze);
  } else {
    scene_valid = false;
    scene.build(m, freeze);  // throws const char* on a block that references a foreign parameter
    scene_valid = true;
    scene_version = m.structureVersion();
  }
  const double t1 = dab_now_seconds();
  t.marshal += t1 - t0;
  const int rc = dab_set_problem(handle.h, &scene.problem);
  t.setup += dab_now_seconds() - t1;
  if (rc) return rc;
  resident = true;
  version = m.structureVersion();
  n_blocks = m.parameters()->size();
  n_points = m.point3ds()->size();
  n_ext = m.extrinsics()->size();
  n_intr = m.intrinsics()->size();
  return 0;
}

void DabScene::write_back(DeepArcManager& m) {
  std::vector<Point3d*>& pts = *m.point3ds();
  std::vector<Extrinsic*>& exts = *m.extrinsics();
  for (size_t i = 0; i < pts.size(); ++i)
    for (int k = 0; k < 3; ++k) pts[i]->position()[k] = points[3 * i + k];
  for (size_t i = 0; i < exts.size(); ++i)
    for (int k = 0; k < 3; ++k) {
      exts[i]->rotation()[k] = ext[6 * i + k];
      exts[i]->translation()[k] = ext[6 * i + 3 + k];
    }
}

void DabSession::filtered(DeepArcManager& m, unsigned long long old_version, const uint8_t* keep_obs,
                          const uint8_t* keep_pt) {
  // DAB_SCENE_COMPACT=0: always rebuild from the blocks (A/B)
  const char* knob = getenv("DAB_SCENE_COMPACT");
  const bool on = !knob || atoi(knob) != 0;
  if (!on || !scene_valid || scene_version != old_version) {
    scene_valid = false;
    return;
  }
  const double t0 = dab_now_seconds();
  scene_valid = scene.compact(keep_obs, keep_pt);
  scene_version = m.structureVersion();
  t.marshal += dab_now_seconds() - t0;
}
