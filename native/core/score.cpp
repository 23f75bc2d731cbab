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

#include <algorithm>
#include <cmath>
#include <stdexcept>
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

// Joint placement of a burst of pending fractional pods over a node's devices (the
// reference scores one pod at a time, gpu_plugins.go:558-757; a burst placed greedily can
// co-locate workloads that hurt each other).  Objective: number of pods -- incoming and
// resident -- whose predicted throughput minus the summed interference of their
// co-residents still meets their SLO (the reference's violation test, SLO > pred - intf,
// :616,717), subject to every GPU's predicted load staying within `max_load`.
// Deterministic first-improvement pairwise swaps between pods of equal units on
// different devices, in sweeps, until no swap improves (or `sweeps` run out).
//   dev[p]       initial device of incoming pod p (a feasible assignment)
//   units[p]     its units (only equal-unit pods swap, so capacities stay valid)
//   row[p], col[p]  its interference row / column (-1 = none), slo[p], pred[p], work[p]
//   gpu[d]       physical GPU of device d (load is per GPU)
//   res_*        residents: device, row, col, slo, pred (fixed), res_work per GPU via base_load
//   M            interference matrix [rows x cols]
py::array_t<int32_t> plan_assignment(py::array_t<int32_t, py::array::c_style | py::array::forcecast> dev_in,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> units,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> row,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> col,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> slo,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> pred,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> work,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> gpu,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> base_load,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> res_dev,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> res_row,
                                     py::array_t<int32_t, py::array::c_style | py::array::forcecast> res_col,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> res_slo,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> res_pred,
                                     py::array_t<double, py::array::c_style | py::array::forcecast> M,
                                     double max_load, int sweeps, double tolerance, int load_first) {
  const auto U = units.unchecked<1>();
  const auto R = row.unchecked<1>();
  const auto Cc = col.unchecked<1>();
  const auto S = slo.unchecked<1>();
  const auto Pd = pred.unchecked<1>();
  const auto Wk = work.unchecked<1>();
  const auto G = gpu.unchecked<1>();
  const auto BL = base_load.unchecked<1>();
  const auto RD = res_dev.unchecked<1>();
  const auto RR = res_row.unchecked<1>();
  const auto RC = res_col.unchecked<1>();
  const auto RS = res_slo.unchecked<1>();
  const auto RP = res_pred.unchecked<1>();
  const auto Mx = M.unchecked<2>();
  const py::ssize_t P = dev_in.shape(0), D = gpu.shape(0), NR = res_dev.shape(0);
  if (U.shape(0) != P || R.shape(0) != P || Cc.shape(0) != P || S.shape(0) != P || Pd.shape(0) != P ||
      Wk.shape(0) != P)
    throw std::runtime_error("plan_assignment: pod array shapes differ");
  if (RR.shape(0) != NR || RC.shape(0) != NR || RS.shape(0) != NR || RP.shape(0) != NR)
    throw std::runtime_error("plan_assignment: resident array shapes differ");
  int n_gpu = 0;
  for (py::ssize_t d = 0; d < D; ++d) n_gpu = std::max(n_gpu, G(d) + 1);
  if (BL.shape(0) < n_gpu) throw std::runtime_error("plan_assignment: base_load shorter than GPU count");
  std::vector<int32_t> dev(dev_in.data(), dev_in.data() + P);
  for (py::ssize_t p = 0; p < P; ++p)
    if (dev[p] < 0 || dev[p] >= D) throw std::runtime_error("plan_assignment: device index out of range");
  for (py::ssize_t r = 0; r < NR; ++r)
    if (RD(r) < 0 || RD(r) >= D) throw std::runtime_error("plan_assignment: resident device out of range");
  const py::ssize_t MR = Mx.shape(0), MC = Mx.shape(1);
  auto m = [&](int r, int c) -> double { return (r >= 0 && c >= 0 && r < MR && c < MC) ? Mx(r, c) : 0.0; };

  py::array_t<int32_t> out(P);
  {
    py::gil_scoped_release nogil;
    // members of each device: incoming pods (>= 0) and residents (encoded -1 - r)
    std::vector<std::vector<int>> mem(D);
    for (py::ssize_t p = 0; p < P; ++p) mem[dev[p]].push_back((int)p);
    for (py::ssize_t r = 0; r < NR; ++r) mem[RD(r)].push_back(-1 - (int)r);
    // number of SLO-satisfied members of device d, and its interference-adjusted work: an
    // incoming pod's alone work stretched by its predicted slowdown pred / (pred - intf)
    // (capped at 4x) -- co-located pods share the device, so pairing complementary
    // workloads shortens the device's busy time, which is what paces a coupled epoch
    auto eval_dev = [&](int d, int& ok, double& adj) {
      ok = 0;
      adj = 0.0;
      const auto& v = mem[d];
      for (int a : v) {
        const int ra = a >= 0 ? R(a) : RR(-1 - a);
        const double sa = a >= 0 ? S(a) : RS(-1 - a);
        const double pa = a >= 0 ? Pd(a) : RP(-1 - a);
        double intf = 0;
        for (int b : v)
          if (b != a) intf += m(ra, b >= 0 ? Cc(b) : RC(-1 - b));
        ok += sa <= 0 || !(sa > pa - intf);
        if (a >= 0) adj += pa > 0 ? Wk(a) * pa / std::max(pa - intf, 0.25 * pa) : Wk(a);
      }
    };
    std::vector<int> okd(D, 0);
    std::vector<double> adjd(D, 0.0), load(n_gpu, 0.0);
    for (int g = 0; g < n_gpu; ++g) load[g] = BL(g);
    for (py::ssize_t d = 0; d < D; ++d) {
      eval_dev((int)d, okd[d], adjd[d]);
      load[G(d)] += adjd[d];
    }
    double cap = max_load;
    if (tolerance >= 0) cap = (1.0 + tolerance) * *std::max_element(load.begin(), load.end());
    auto swap_in = [&](int d, int from, int to) {
      for (int& x : mem[d])
        if (x == from) { x = to; return; }
    };
    // first-improvement pairwise swaps of equal-size pods on different devices: accept a
    // swap that meets more SLOs without pushing a GPU over the cap (unless it lowers an
    // over-cap GPU), or meets as many and lowers the pair's busier GPU
    for (int sw = 0; sw < sweeps; ++sw) {
      bool improved = false;
      for (py::ssize_t i = 0; i < P; ++i) {
        for (py::ssize_t j = i + 1; j < P; ++j) {
          const int di = dev[i], dj = dev[j];
          if (di == dj || U(i) != U(j)) continue;
          const int gi = G(di), gj = G(dj);
          swap_in(di, (int)i, (int)j);
          swap_in(dj, (int)j, (int)i);
          int oki, okj;
          double ai, aj;
          eval_dev(di, oki, ai);
          eval_dev(dj, okj, aj);
          double li = load[gi] + ai - adjd[di], lj = load[gj] + aj - adjd[dj];
          if (gi == gj) li = lj = load[gi] + ai - adjd[di] + aj - adjd[dj];
          const int before = okd[di] + okd[dj], after = oki + okj;
          const double mb = std::max(load[gi], load[gj]), ma = std::max(li, lj);
          const bool over = (li > cap && li > load[gi] + 1e-12) || (lj > cap && lj > load[gj] + 1e-12);
          // load_first: lower the pair's busier GPU first, SLO count as the tie-break
          const bool take = load_first
                                ? (ma < mb * (1.0 - 1e-9) || (ma <= mb * (1.0 + 1e-9) && after > before))
                                : !over && (after > before || (after == before && ma < mb * (1.0 - 1e-9)));
          if (take) {
            dev[i] = dj;
            dev[j] = di;
            okd[di] = oki;
            okd[dj] = okj;
            adjd[di] = ai;
            adjd[dj] = aj;
            load[gi] = li;
            load[gj] = lj;
            improved = true;
          } else {
            swap_in(di, (int)j, (int)i);
            swap_in(dj, (int)i, (int)j);
          }
        }
      }
      if (!improved) break;
    }
  }
  auto o = out.mutable_unchecked<1>();
  for (py::ssize_t p = 0; p < P; ++p) o(p) = dev[p];
  return out;
}

// Fixed-mode GPU Score of one node (plugins/gpu/plugin.py GPUPlugin._score_cands): every
// candidate device's blend of the SLO/interference objective (scoring.fast_device_score,
// the reference's Logic terms, gpu_plugins.go:558-757, in float64), unit packing, the
// least-predicted-load balance, roofline complementarity and live telemetry -- the same
// terms in the same order of float operations, so the result is bit-identical to the
// Python path.  The node's static part (its devices' resident terms, fill, loads) is a
// NodePack built once per node version; names and interference columns are interned
// integer ids, a resident's interference row a dense vector over column ids (missing = 0).
//   t_off[d]..t_off[d+1]   SLO terms of device d: t_name, t_slo, t_pred, t_base, t_rows[t, :]
//   k_off[d]..k_off[d+1]   (resident name id, column id) of the residents with a column
//   dev_gpu[d]             physical GPU of device d
//   gpu_tot/gpu_used[g]    unit fill per GPU; gpu_load[g] predicted resident work (balance);
//   roof_m/roof_h[g]       residents' MFMA / HBM seconds (complementarity)
struct NodePack {
  // built once per node version (plugins/gpu/plugin.py _node_pack); see score() below
  std::vector<int64_t> t_off, k_off;
  std::vector<int32_t> t_name, k_name, k_col, dev_gpu, gpu_tot, gpu_used;
  std::vector<double> t_slo, t_pred, t_base, t_rows, gpu_load, roof_m, roof_h;
  int64_t n_col = 0;

  template <typename T>
  static std::vector<T> vec(const py::array_t<T, py::array::c_style | py::array::forcecast>& a) {
    return std::vector<T>(a.data(), a.data() + a.size());
  }

  NodePack(py::array_t<int64_t, py::array::c_style | py::array::forcecast> t_off_,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> t_name_,
           py::array_t<double, py::array::c_style | py::array::forcecast> t_slo_,
           py::array_t<double, py::array::c_style | py::array::forcecast> t_pred_,
           py::array_t<double, py::array::c_style | py::array::forcecast> t_base_,
           py::array_t<double, py::array::c_style | py::array::forcecast> t_rows_,
           py::array_t<int64_t, py::array::c_style | py::array::forcecast> k_off_,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> k_name_,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> k_col_,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> dev_gpu_,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> gpu_tot_,
           py::array_t<int32_t, py::array::c_style | py::array::forcecast> gpu_used_,
           py::array_t<double, py::array::c_style | py::array::forcecast> gpu_load_,
           py::array_t<double, py::array::c_style | py::array::forcecast> roof_m_,
           py::array_t<double, py::array::c_style | py::array::forcecast> roof_h_)
      : t_off(vec(t_off_)), k_off(vec(k_off_)), t_name(vec(t_name_)), k_name(vec(k_name_)), k_col(vec(k_col_)),
        dev_gpu(vec(dev_gpu_)), gpu_tot(vec(gpu_tot_)), gpu_used(vec(gpu_used_)), t_slo(vec(t_slo_)),
        t_pred(vec(t_pred_)), t_base(vec(t_base_)), t_rows(vec(t_rows_)), gpu_load(vec(gpu_load_)),
        roof_m(vec(roof_m_)), roof_h(vec(roof_h_)) {
    const size_t D = dev_gpu.size(), T = t_name.size(), K = k_name.size(), G = gpu_tot.size();
    if (t_rows_.ndim() != 2 || (size_t)t_rows_.shape(0) != T) throw std::runtime_error("NodePack: t_rows shape");
    n_col = t_rows_.shape(1);
    if (t_off.size() != D + 1 || k_off.size() != D + 1 || (size_t)t_off[D] != T || (size_t)k_off[D] != K ||
        t_slo.size() != T || t_pred.size() != T || t_base.size() != T || k_col.size() != K || gpu_used.size() != G ||
        gpu_load.size() != G || roof_m.size() != G || roof_h.size() != G)
      throw std::runtime_error("NodePack: array sizes mismatch");
    for (int32_t g : dev_gpu)
      if (g < 0 || (size_t)g >= G) throw std::runtime_error("NodePack: gpu id out of range");
  }

  // Returns (best candidate position or -1, its score); the first maximum wins.
  //   cand[i], x_pred[i]   candidate device index and the incoming pod's prediction there
  //   tele_ok/gfx/vram_free_mb[d]   fresh telemetry sample per device (tele_ok 0 = none)
  //   wt = (w_slo, w_pack, w_balance, w_complement, w_telemetry)
  //   flags: 1 slo term on, 2 binpack (else spread), 4 balance on, 8 complement on
  py::tuple score(py::array_t<int32_t, py::array::c_style | py::array::forcecast> cand,
                  py::array_t<double, py::array::c_style | py::array::forcecast> x_pred,
                  py::array_t<int8_t, py::array::c_style | py::array::forcecast> tele_ok,
                  py::array_t<double, py::array::c_style | py::array::forcecast> gfx,
                  py::array_t<double, py::array::c_style | py::array::forcecast> vram_free_mb,
                  py::array_t<double, py::array::c_style | py::array::forcecast> x_intf, int x_name, int x_col,
                  double x_slo, int units, double work, double top, double xf, double hbm_mb,
                  py::array_t<double, py::array::c_style | py::array::forcecast> wt, int flags) const {
    const auto CA = cand.unchecked<1>();
    const auto XP = x_pred.unchecked<1>();
    const auto TK = tele_ok.unchecked<1>();
    const auto GX = gfx.unchecked<1>();
    const auto VF = vram_free_mb.unchecked<1>();
    const auto XI = x_intf.unchecked<1>();
    const auto W = wt.unchecked<1>();
    const py::ssize_t D = (py::ssize_t)dev_gpu.size(), NC = CA.shape(0), XC = XI.shape(0);
    if (XP.shape(0) != NC || W.shape(0) != 5 || TK.shape(0) != D || GX.shape(0) != D || VF.shape(0) != D)
      throw std::runtime_error("NodePack.score: shape mismatch");
    for (py::ssize_t i = 0; i < NC; ++i)
      if (CA(i) < 0 || CA(i) >= D) throw std::runtime_error("NodePack.score: candidate out of range");
    const double w_slo = W(0), w_pack = W(1), w_bal = W(2), w_comp = W(3), w_tel = W(4);
    int best_i = -1;
    double best_sc = 0.0;
    for (py::ssize_t i = 0; i < NC; ++i) {
      const int d = CA(i);
      double num = 0.0, den = 0.0;
      if (flags & 1) {
        // scoring.fast_device_score, float64, same order of operations
        double neg_sum = 0.0, pos_sum = 0.0;
        int n_neg = 0, n_pos = 0;
        auto add = [&](double slo, double pred, double it) {
          const double dd = (slo - (pred - it)) / slo;
          if (dd > 0) {
            const double q = std::fabs(dd) + 1.0;
            neg_sum += 1.0 / (1.0 + q * q);
            ++n_neg;
          } else {
            pos_sum += 1.0 / (1.0 + std::fabs(dd));
            ++n_pos;
          }
        };
        for (int64_t t = t_off[d]; t < t_off[d + 1]; ++t) {
          double it = t_base[t];
          if (x_col >= 0 && t_name[t] != x_name) it += (x_col < n_col) ? t_rows[t * n_col + x_col] : 0.0;
          add(t_slo[t], t_pred[t], it);
        }
        if (XP(i) != -1 && x_slo > 0) {
          double it = 0.0;
          for (int64_t k = k_off[d]; k < k_off[d + 1]; ++k)
            if (k_name[k] != x_name) it += (k_col[k] >= 0 && k_col[k] < XC) ? XI(k_col[k]) : 0.0;
          add(x_slo, XP(i), it);
        }
        double s = 0.0;
        if (n_pos && n_neg) {
          const double k = (double)n_neg / (double)(n_neg + n_pos);
          s = 100.0 * ((1 - k) * pos_sum / n_pos) + 100.0 * (k * neg_sum / n_neg);
        } else if (n_neg) {
          s = 100.0 * neg_sum / n_neg;
        } else if (n_pos) {
          s = 100.0 * pos_sum / n_pos;
        }
        num += w_slo * s;
        den += w_slo;
      }
      const int g = dev_gpu[d];
      if (w_pack != 0.0) {
        const double frac = (double)(gpu_used[g] + units) / (double)std::max(gpu_tot[g], 1);
        num += w_pack * ((flags & 2) ? 100.0 * frac : 100.0 * (1.0 - frac));
        den += w_pack;
      }
      if (flags & 4) {
        num += w_bal * (top > 0 ? 100.0 * (1.0 - (gpu_load[g] + work) / top) : 100.0);
        den += w_bal;
      }
      if (flags & 8) {
        const double m = roof_m[g] + work * xf, h = roof_h[g] + work * (1.0 - xf);
        const double mx = std::max(m, h);
        num += w_comp * 100.0 * (mx > 0 ? std::min(m, h) / mx : 1.0);
        den += w_comp;
      }
      if (TK(d)) {
        const double hbm_ok = VF(d) >= hbm_mb ? 1.0 : 0.0;
        num += w_tel * 100.0 * (1.0 - std::min(1.0, GX(d))) * hbm_ok;
        den += w_tel;
      }
      const double sc = den > 0 ? num / den : 0.0;
      if (best_i < 0 || sc > best_sc) {
        best_i = (int)i;
        best_sc = sc;
      }
    }
    return py::make_tuple(best_i, best_sc);
  }
};

// Host selection of one scheduling cycle over cached per-node results (framework.fastpath):
// walk the nodes in rotated order from `start`, keep the first `limit` feasible ones (0 = all;
// kube-scheduler's numFeasibleNodesToFind / nextStartNodeIndex), min-max normalise the
// plugins that ask for it (Go integer arithmetic, reference gpu_plugins.go:816-841), sum
// weight x score per node and return the positions (in feasible order) of every node tied
// at the maximum -- the caller draws the winner among them with its own RNG.
//   feasible[n]  1 = passes every filter, 0 = not, -1 = not evaluated yet (lazy)
//   raw[p, n]    plugin p's raw score of node n (only read for feasible nodes)
//   norm[p]      1 = min-max normalise plugin p over the feasible set
// Returns (processed, feasible node indices, totals, tie positions, bad plugin or -1,
// unevaluated): a score outside [0, 100] after normalisation stops the cycle like the
// framework does.  If the scan meets unevaluated nodes before it can close the sample, it
// returns only them (every one the sample could still need: scanning on as if each were
// feasible) -- the caller evaluates those and calls again.
py::tuple select_nodes(py::array_t<int8_t, py::array::c_style | py::array::forcecast> feasible,
                       py::array_t<int64_t, py::array::c_style | py::array::forcecast> raw,
                       py::array_t<int8_t, py::array::c_style | py::array::forcecast> norm,
                       py::array_t<int64_t, py::array::c_style | py::array::forcecast> weights, int64_t start,
                       int64_t limit) {
  const auto F = feasible.unchecked<1>();
  const auto R = raw.unchecked<2>();
  const auto Nm = norm.unchecked<1>();
  const auto Wt = weights.unchecked<1>();
  const py::ssize_t N = F.shape(0), P = R.shape(0);
  if (R.shape(1) != N || Nm.shape(0) != P || Wt.shape(0) != P) throw std::runtime_error("select_nodes: shape mismatch");
  std::vector<int32_t> feas;
  std::vector<int64_t> tot;
  std::vector<int32_t> ties, unknown;
  int64_t processed = 0;
  int bad = -1;
  {
    py::gil_scoped_release nogil;
    const int64_t s0 = N ? ((start % N) + N) % N : 0;
    feas.reserve(limit > 0 ? (size_t)limit : (size_t)N);
    for (py::ssize_t i = 0; i < N; ++i) {
      const int64_t n = (s0 + i) % N;
      ++processed;
      if (F(n) < 0) {
        unknown.push_back((int32_t)n);
      } else if (F(n)) {
        feas.push_back((int32_t)n);
      }
      if (limit > 0 && (int64_t)(feas.size() + unknown.size()) >= limit) break;
    }
    if (!unknown.empty()) feas.clear();
    tot.assign(feas.size(), 0);
    for (py::ssize_t p = 0; p < P && bad < 0; ++p) {
      int64_t lo = 0, hi = 0;
      if (Nm(p) && !feas.empty()) {
        lo = hi = R(p, feas[0]);
        for (int32_t n : feas) {
          lo = std::min(lo, R(p, n));
          hi = std::max(hi, R(p, n));
        }
      }
      for (size_t k = 0; k < feas.size(); ++k) {
        int64_t v = R(p, feas[k]);
        if (Nm(p)) v = (hi == lo) ? 0 : ((v - lo) * 100) / (hi - lo);
        if (v < 0 || v > 100) {
          bad = (int)p;
          break;
        }
        tot[k] += v * Wt(p);
      }
    }
    if (bad < 0 && !feas.empty()) {
      const int64_t best = *std::max_element(tot.begin(), tot.end());
      for (size_t k = 0; k < tot.size(); ++k)
        if (tot[k] == best) ties.push_back((int32_t)k);
    }
  }
  py::array_t<int32_t> f_out(feas.size());
  py::array_t<int64_t> t_out(tot.size());
  py::array_t<int32_t> ties_out(ties.size());
  py::array_t<int32_t> u_out(unknown.size());
  std::copy(feas.begin(), feas.end(), f_out.mutable_data());
  std::copy(tot.begin(), tot.end(), t_out.mutable_data());
  std::copy(ties.begin(), ties.end(), ties_out.mutable_data());
  std::copy(unknown.begin(), unknown.end(), u_out.mutable_data());
  return py::make_tuple(processed, f_out, t_out, ties_out, bad, u_out);
}

}  // namespace

void register_corun(py::module_& m);   // corun.cpp: multi-way co-run model

PYBIND11_MODULE(_core, m) {
  m.doc() = "native scoring core for the GPU scheduler plugin";
  m.def("slo_scores", &slo_scores, py::arg("offsets"), py::arg("r_slo"), py::arg("r_pred"), py::arg("r_intf"),
        py::arg("inc_slo"), py::arg("inc_pred"), py::arg("inc_intf"));
  m.def("find_units", &find_units, py::arg("used"), py::arg("units"), py::arg("n"));
  m.def("plan_assignment", &plan_assignment, py::arg("dev"), py::arg("units"), py::arg("row"), py::arg("col"),
        py::arg("slo"), py::arg("pred"), py::arg("work"), py::arg("gpu"), py::arg("base_load"), py::arg("res_dev"),
        py::arg("res_row"), py::arg("res_col"), py::arg("res_slo"), py::arg("res_pred"), py::arg("M"),
        py::arg("max_load"), py::arg("sweeps") = 8, py::arg("tolerance") = -1.0, py::arg("load_first") = 0);
  py::class_<NodePack>(m, "NodePack")
      .def(py::init<py::array_t<int64_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<int64_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<int32_t, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>,
                    py::array_t<double, py::array::c_style | py::array::forcecast>>())
      .def("score", &NodePack::score);
  m.def("select_nodes", &select_nodes, py::arg("feasible"), py::arg("raw"), py::arg("norm"), py::arg("weights"),
        py::arg("start"), py::arg("limit"));
  register_corun(m);
}
