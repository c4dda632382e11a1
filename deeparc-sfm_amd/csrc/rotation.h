// rotation.h — host-side angle-axis helpers with Ceres rotation.h semantics
// (SURVEY App. B.1). Used by the .deeparc loader (DeepArcManager.cc:141-147 converts
// 3x3 / quaternion input to angle-axis), the camera-centre code (Extrinsic.hh:12-17)
// and the synthetic generator. Device code has its own inline forms in dab_kernels.hip.
#pragma once
#include <cfloat>
#include <cmath>

namespace dab {

// R(row, col) at R[col*3 + row] (column-major, Ceres default).
inline void AngleAxisToRotationMatrix(const double aa[3], double R[9]) {
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > DBL_EPSILON) {
    const double theta = std::sqrt(theta2);
    const double wx = aa[0] / theta, wy = aa[1] / theta, wz = aa[2] / theta;
    const double c = std::cos(theta), s = std::sin(theta), omc = 1.0 - c;
    R[0] = c + wx * wx * omc;
    R[1] = wz * s + wx * wy * omc;
    R[2] = -wy * s + wx * wz * omc;
    R[3] = wx * wy * omc - wz * s;
    R[4] = c + wy * wy * omc;
    R[5] = wx * s + wy * wz * omc;
    R[6] = wy * s + wx * wz * omc;
    R[7] = -wx * s + wy * wz * omc;
    R[8] = c + wz * wz * omc;
  } else {  // first-order: R = I + [aa]x
    R[0] = 1.0; R[1] = aa[2]; R[2] = -aa[1];
    R[3] = -aa[2]; R[4] = 1.0; R[5] = aa[0];
    R[6] = aa[1]; R[7] = -aa[0]; R[8] = 1.0;
  }
}

// q = (w, x, y, z)
inline void QuaternionToAngleAxis(const double q[4], double aa[3]) {
  const double s2 = q[1] * q[1] + q[2] * q[2] + q[3] * q[3];
  if (s2 > 0.0) {
    const double s = std::sqrt(s2), c = q[0];
    const double two_theta = 2.0 * ((c < 0.0) ? std::atan2(-s, -c) : std::atan2(s, c));
    const double k = two_theta / s;
    aa[0] = q[1] * k; aa[1] = q[2] * k; aa[2] = q[3] * k;
  } else {
    aa[0] = 2.0 * q[1]; aa[1] = 2.0 * q[2]; aa[2] = 2.0 * q[3];
  }
}

inline void RotationMatrixToQuaternion(const double R[9], double q[4]) {
  auto M = [&](int r, int c) { return R[c * 3 + r]; };
  const double trace = M(0, 0) + M(1, 1) + M(2, 2);
  if (trace >= 0.0) {
    double t = std::sqrt(trace + 1.0);
    q[0] = 0.5 * t;
    t = 0.5 / t;
    q[1] = (M(2, 1) - M(1, 2)) * t;
    q[2] = (M(0, 2) - M(2, 0)) * t;
    q[3] = (M(1, 0) - M(0, 1)) * t;
  } else {
    int i = 0;
    if (M(1, 1) > M(0, 0)) i = 1;
    if (M(2, 2) > M(i, i)) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    double t = std::sqrt(M(i, i) - M(j, j) - M(k, k) + 1.0);
    q[i + 1] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (M(k, j) - M(j, k)) * t;
    q[j + 1] = (M(j, i) + M(i, j)) * t;
    q[k + 1] = (M(k, i) + M(i, k)) * t;
  }
}

inline void RotationMatrixToAngleAxis(const double R[9], double aa[3]) {
  double q[4];
  RotationMatrixToQuaternion(R, q);
  QuaternionToAngleAxis(q, aa);
}

inline void AngleAxisRotatePoint(const double aa[3], const double pt[3], double out[3]) {
  const double theta2 = aa[0] * aa[0] + aa[1] * aa[1] + aa[2] * aa[2];
  if (theta2 > DBL_EPSILON) {
    const double theta = std::sqrt(theta2);
    const double c = std::cos(theta), s = std::sin(theta), ti = 1.0 / theta;
    const double w[3] = {aa[0] * ti, aa[1] * ti, aa[2] * ti};
    const double wx[3] = {w[1] * pt[2] - w[2] * pt[1], w[2] * pt[0] - w[0] * pt[2],
                          w[0] * pt[1] - w[1] * pt[0]};
    const double tmp = (w[0] * pt[0] + w[1] * pt[1] + w[2] * pt[2]) * (1.0 - c);
    for (int i = 0; i < 3; ++i) out[i] = pt[i] * c + wx[i] * s + w[i] * tmp;
  } else {
    const double wx[3] = {aa[1] * pt[2] - aa[2] * pt[1], aa[2] * pt[0] - aa[0] * pt[2],
                          aa[0] * pt[1] - aa[1] * pt[0]};
    for (int i = 0; i < 3; ++i) out[i] = pt[i] + wx[i];
  }
}

}  // namespace dab
