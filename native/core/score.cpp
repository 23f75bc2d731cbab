// Native scoring core (host C++, no GPU): the per-device SLO/interference objective of
// the reference's Logic (pkg/plugins/gpu_plugin/gpu_plugins.go:558-757) evaluated for a
// batch of candidate devices in one call, with the same mixed float32/float64 numerics as
// the Go code (see k8s_gpu_scheduler_amd/plugins/gpu/scoring.py), plus the XCD-unit
// best-fit search of the device ledger.
//
// Inputs are flat numpy arrays prepared by the Python layer (which resolves names ->
// configuration predictions and interference sums once per pod, memoised):
//   offsets[d]..offsets[d+1]  residents of device d
//   r_slo, r_pred, r_intf     resident SLO, prediction (NaN = column missing -> skipped),
//                             interference sum already accumulated in float32
//   inc_slo, inc_pred[d]      incoming pod SLO and prediction on device d (-1 = none qualifies)
//   inc_intf[d]               incoming pod's interference sum on device d (float32)
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <cmath>
#include <cstdint>
#include <vector>

namespace py = pybind11;

namespace {

struct Acc {
  double neg = 0, pos = 0;
  int nn = 0, np = 0;
  inline void add(float slo, float pred, float intf) {
    const float eff = pred - intf;
    const float ratio_f = (1.0f / slo) * (slo - eff);
    const double ratio = static_cast<double>(ratio_f);
    if (slo > eff) {
      const double t = std::fabs(ratio) + 1.0;
      neg += 1.0 / (1.0 + t * t);
      ++nn;
    } else {
      pos += 1.0 / (1.0 + std::fabs(ratio));
      ++np;
    }
  }
  inline double score() const {
    const double f = 100.0;
    if (np > 0 && nn > 0) {
      const double k = static_cast<double>(nn) / static_cast<double>(nn + np);
      return f * ((1 - k) * pos / np) + f * (k * neg / nn);
    }
    if (nn > 0) return f * (neg / nn);
    if (np > 0) return f * (pos / np);
    return 0.0;
  }
};

py::array_t<double> slo_scores(py::array_t<int64_t, py::array::c_style | py::array::forcecast> offsets,
                               py::array_t<float, py::array::c_style | py::array::forcecast> r_slo,
                               py::array_t<float, py::array::c_style | py::array::forcecast> r_pred,
                               py::array_t<float, py::array::c_style | py::array::forcecast> r_intf, float inc_slo,
                               py::array_t<float, py::array::c_style | py::array::forcecast> inc_pred,
                               py::array_t<float, py::array::c_style | py::array::forcecast> inc_intf) {
  const auto off = offsets.unchecked<1>();
  const auto slo = r_slo.unchecked<1>();
  const auto pred = r_pred.unchecked<1>();
  const auto intf = r_intf.unchecked<1>();
  const auto ip = inc_pred.unchecked<1>();
  const auto ii = inc_intf.unchecked<1>();
  const py::ssize_t nd = off.shape(0) - 1;
  if (nd < 0 || ip.shape(0) != nd || ii.shape(0) != nd) throw std::runtime_error("slo_scores: shape mismatch");
  if (off(nd) > slo.shape(0) || slo.shape(0) != pred.shape(0) || slo.shape(0) != intf.shape(0))
    throw std::runtime_error("slo_scores: resident arrays mismatch");
  py::array_t<double> out(nd);
  auto o = out.mutable_unchecked<1>();
  {
    py::gil_scoped_release nogil;
    for (py::ssize_t d = 0; d < nd; ++d) {
      Acc a;
      for (int64_t r = off(d); r < off(d + 1); ++r) {
        if (slo(r) == 0.0f || std::isnan(pred(r))) continue;
        a.add(slo(r), pred(r), intf(r));
      }
      if (ip(d) != -1.0f) a.add(inc_slo, ip(d), ii(d));
      o(d) = a.score();
    }
  }
  return out;
}

// Best-fit aligned run of n free units in each device's bitmask (bit u set = used).
// Returns the first unit index per device or -1.
py::array_t<int32_t> find_units(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> used,
                                py::array_t<int32_t, py::array::c_style | py::array::forcecast> units, int n) {
  const auto u = used.unchecked<1>();
  const auto nu = units.unchecked<1>();
  const py::ssize_t nd = u.shape(0);
  py::array_t<int32_t> out(nd);
  auto o = out.mutable_unchecked<1>();
  int align = 1;
  while (align < n) align *= 2;
  for (py::ssize_t d = 0; d < nd; ++d) {
    const int total = nu(d);
    int best = -1, best_free = 1 << 30;
    if (n <= total && n > 0) {
      const uint64_t run = (n >= 64) ? ~0ull : ((1ull << n) - 1);
      for (int s = 0; s + n <= total; s += align) {
        if (u(d) & (run << s)) continue;
        const int blk = std::max(align * 2, 2);
        const int b0 = (s / blk) * blk;
        const int b1 = std::min(b0 + blk, total);
        int free_in_blk = 0;
        for (int k = b0; k < b1; ++k) free_in_blk += !((u(d) >> k) & 1ull);
        if (free_in_blk < best_free) {
          best_free = free_in_blk;
          best = s;
        }
      }
    }
    o(d) = best;
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(_core, m) {
  m.doc() = "native scoring core for the GPU scheduler plugin";
  m.def("slo_scores", &slo_scores, py::arg("offsets"), py::arg("r_slo"), py::arg("r_pred"), py::arg("r_intf"),
        py::arg("inc_slo"), py::arg("inc_pred"), py::arg("inc_intf"));
  m.def("find_units", &find_units, py::arg("used"), py::arg("units"), py::arg("n"));
}
