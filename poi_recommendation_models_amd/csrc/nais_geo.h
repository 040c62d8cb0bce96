// nais_geo.h -- powerLaw.dist (powerLaw.py:7-21) on the device, float64 in the reference's
// operation order; every product/sum an explicit round-to-nearest op (__dmul_rn / __dadd_rn /
// __dsub_rn) so the compiler cannot contract FMAs. Shared by the prior kernel (nais_kernels.hip)
// the pair-distance kernel (nais_disent.hip) and the prior pair tables (nais_pairs.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace nais_geo {

constexpr double kD2R = 0.017453292519943295;  // math.pi / 180.0

struct Geo {
  double lat, lng, sphi, cphi, theta;
};

__device__ __forceinline__ Geo make_geo(double lat, double lng) {
  const double phi = __dmul_rn(__dsub_rn(90.0, lat), kD2R);
  return Geo{lat, lng, sin(phi), cos(phi), __dmul_rn(lng, kD2R)};
}

// powerLaw.dist(loc1, loc2): loc1 = history POI, loc2 = candidate (powerLaw.py:92)
__device__ __forceinline__ double ref_dist(const Geo& p1, const Geo& p2) {
  if (fabs(__dsub_rn(p1.lat, p2.lat)) < 1e-6 && fabs(__dsub_rn(p1.lng, p2.lng)) < 1e-6) return 0.0;
  const double cosv = __dadd_rn(__dmul_rn(__dmul_rn(p1.sphi, p2.sphi), cos(__dsub_rn(p1.theta, p2.theta))),
                                __dmul_rn(p1.cphi, p2.cphi));
  return __dmul_rn(acos(cosv), 6371.0);
}

// PowerLaw.pr_d (powerLaw.py:86-88): a * max(0.01, d) ** b   (Python max(0.01, nan) = 0.01)
__device__ __forceinline__ double ref_pr_d(double a, double b, double d) {
  const double dd = (d > 0.01) ? d : 0.01;
  return __dmul_rn(a, pow(dd, b));
}

}  // namespace nais_geo

using nais_geo::Geo;
using nais_geo::make_geo;
using nais_geo::ref_dist;
using nais_geo::kD2R;
using nais_geo::ref_pr_d;
