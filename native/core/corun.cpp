// Multi-way co-run model, native side (host C++): the fluid simulation of a GPU's pod group
// (k8s_gpu_scheduler_amd/models/corun.py documents the model), the Score-time evaluation of
// candidate GPUs, and the joint placement of a burst of pods.
//
// The reference predicts co-location with a pairwise-additive interference table summed over
// co-residents (pkg/plugins/gpu_plugin/gpu_plugins.go:589-612, 695-714).  Here every pod of a
// group carries work W_i (iterations x alone whole-GPU ms per iteration) and, while the set A
// of pods is active, progresses at r_i = 1 / (1 + sum_{j in A, j != i} c[w_i][w_j]) work-ms
// per wall-ms; c = U V^T is fitted on measured MI355X co-run groups.  Between events (a pod
// starts or finishes) rates are constant, so a group of k pods takes at most 2k steps.
//
// A pod with iters <= 0 is a SERVICE (long-running, SLO = sustained throughput): it never
// finishes, co-runs with the whole group, and its predicted throughput is its rate with every
// member active (the worst case its SLO must hold under).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

constexpr double kBig = 1e300;
constexpr int kMaxK = 64;   // pods per GPU group (CPX: 64 devices of 4 CUs would be the extreme)

// fin[i] = wall ms at which pod i finishes (kBig for a service pod); tput_ms[i] = ms per
// iteration achieved (fin / iters, or the steady-state ms/iter of a service pod).
// pin_end (optional): a member with pin_end[i] > start[i] is PINNED -- present exactly during
// [start, pin_end) (a co-runner whose interval was measured), pressing on the others but not
// simulated itself; fin[i] = pin_end[i].  Learning from a pipeline's timeline conditions the
// observed pods on what their co-runners really did, instead of re-simulating co-runners whose
// own (earlier) co-runners lie outside the observed window.
void sim_group(int k, const int32_t* w, const double* iters, const double* start, const double* alone,
               const double* C, int W, double* fin, const double* pin_end = nullptr) {
  double rem[kMaxK], st[kMaxK], pe[kMaxK];
  bool started[kMaxK], done[kMaxK], svc[kMaxK], pin[kMaxK];
  for (int i = 0; i < k; ++i) {
    svc[i] = iters[i] <= 0;
    st[i] = start ? start[i] : 0.0;
    pin[i] = pin_end && pin_end[i] > st[i];
    pe[i] = pin[i] ? pin_end[i] : 0.0;
    rem[i] = (svc[i] || pin[i]) ? kBig : std::max(alone[w[i]] * iters[i], 1e-12);
    started[i] = done[i] = false;
    fin[i] = pin[i] ? pe[i] : svc[i] ? kBig : 0.0;
  }
  double now = 0.0;
  for (int step = 0; step < 3 * k + 1; ++step) {
    bool live = false;
    for (int i = 0; i < k; ++i) live |= !done[i] && !svc[i] && !pin[i];
    if (!live) break;
    for (int i = 0; i < k; ++i)
      if (!started[i] && st[i] <= now + 1e-12) started[i] = true;
    for (int i = 0; i < k; ++i)
      if (pin[i] && started[i] && !done[i] && pe[i] <= now + 1e-12) done[i] = true;
    double rate[kMaxK];
    double dt = kBig;
    int am = -1;
    double am_t = kBig;
    for (int i = 0; i < k; ++i) {
      rate[i] = 0.0;
      if (!started[i] || done[i] || pin[i]) continue;
      double load = 1.0;
      const double* ci = C + (size_t)w[i] * W;
      for (int j = 0; j < k; ++j)
        if (j != i && started[j] && !done[j]) load += ci[w[j]];
      rate[i] = 1.0 / load;
      if (!svc[i]) {
        const double t = rem[i] / std::max(rate[i], 1e-30);
        if (t < am_t) am_t = t, am = i;
      }
    }
    dt = am_t;
    for (int i = 0; i < k; ++i) {
      if (!started[i]) dt = std::min(dt, st[i] - now);
      else if (pin[i] && !done[i]) dt = std::min(dt, pe[i] - now);
    }
    for (int i = 0; i < k; ++i)
      if (started[i] && !done[i] && !svc[i] && !pin[i]) rem[i] -= rate[i] * dt;
    now += dt;
    for (int i = 0; i < k; ++i) {
      if (!started[i] || done[i] || svc[i] || pin[i]) continue;
      const double wk = alone[w[i]] * iters[i];
      if (rem[i] <= 1e-9 * std::max(wk, 1.0) || (i == am && am_t <= dt + 1e-12)) {
        done[i] = true;
        fin[i] = now;
      }
    }
  }
}

// Steady-state ms per iteration of pod i with every member of the group active.
inline double steady_ms(int k, int i, const int32_t* w, const double* alone, const double* C, int W) {
  double load = 1.0;
  const double* ci = C + (size_t)w[i] * W;
  for (int j = 0; j < k; ++j)
    if (j != i) load += ci[w[j]];
  return alone[w[i]] * load;
}

struct GroupEval {
  int ok = 0, bad = 0;          // members meeting / missing their SLO (SLO <= 0 counts as met)
  double makespan = 0.0;        // last finish of a batch pod (services excluded)
  double deficit = 0.0;         // sum over missing members of 1 - tput / SLO (how far they are)
  double expected = 0.0;        // expected members meeting their SLO under model error (sigma)
};

// P(true throughput >= SLO) when log(true / predicted) ~ N(0, sigma^2): the planner's soft
// objective -- a plan of pods that clear their SLO by a model error's worth is worth more
// than one that meets the same number on paper by a hair.
inline double p_meet(double tput, double slo, double sigma) {
  if (slo <= 0) return 1.0;
  if (sigma <= 0) return tput >= slo ? 1.0 : 0.0;
  return 0.5 * std::erfc(-std::log(std::max(tput, 1e-12) / slo) / (sigma * std::sqrt(2.0)));
}

// Evaluate one group: SLO verdicts and makespan.  slo = minimum iterations/s.
GroupEval eval_group(int k, const int32_t* w, const double* iters, const double* slo, const double* alone,
                     const double* C, int W, double* tput_out = nullptr, double sigma = 0.0) {
  GroupEval g;
  if (k == 0) return g;
  if (k > kMaxK) throw std::runtime_error("corun: group larger than 64 pods");
  double fin[kMaxK];
  sim_group(k, w, iters, nullptr, alone, C, W, fin);
  for (int i = 0; i < k; ++i) {
    double tput;
    if (iters[i] <= 0) {
      tput = 1e3 / std::max(steady_ms(k, i, w, alone, C, W), 1e-12);
    } else {
      tput = iters[i] / std::max(fin[i], 1e-12) * 1e3;
      g.makespan = std::max(g.makespan, fin[i]);
    }
    if (tput_out) tput_out[i] = tput;
    g.expected += p_meet(tput, slo[i], sigma);
    if (slo[i] <= 0 || tput >= slo[i]) {
      ++g.ok;
    } else {
      ++g.bad;
      g.deficit += 1.0 - tput / slo[i];
    }
  }
  return g;
}

using I32 = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;
using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
using F64 = py::array_t<double, py::array::c_style | py::array::forcecast>;
using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

void check_model(const F64& alone, const F64& cmat, int& W) {
  W = (int)alone.shape(0);
  if (cmat.ndim() != 2 || cmat.shape(0) != W || cmat.shape(1) != W)
    throw std::runtime_error("corun: coupling matrix must be [W, W] for W workloads");
}

void check_wids(const int32_t* w, py::ssize_t n, int W, const char* what) {
  for (py::ssize_t i = 0; i < n; ++i)
    if (w[i] < 0 || w[i] >= W) throw std::runtime_error(std::string("corun: workload id out of range in ") + what);
}

// Batch simulation: groups of up to K pods (mask selects members); returns finish ms [G, K]
// (0 where masked out, 1e300 for service pods).
py::array_t<double> corun_times(I32 wids, F64 iters, U8 mask, F64 starts, F64 alone, F64 cmat, py::object pin_end) {
  int W;
  check_model(alone, cmat, W);
  if (wids.ndim() != 2) throw std::runtime_error("corun_times: wids must be [G, K]");
  const py::ssize_t G = wids.shape(0), K = wids.shape(1);
  if (iters.shape(0) != G || iters.shape(1) != K || mask.shape(0) != G || mask.shape(1) != K ||
      starts.shape(0) != G || starts.shape(1) != K)
    throw std::runtime_error("corun_times: array shapes differ");
  if (K > kMaxK) throw std::runtime_error("corun_times: more than 64 pods per group");
  F64 pin_a;
  const double* pp = nullptr;
  if (!pin_end.is_none()) {
    pin_a = pin_end.cast<F64>();
    if (pin_a.ndim() != 2 || pin_a.shape(0) != G || pin_a.shape(1) != K)
      throw std::runtime_error("corun_times: pin_end must be [G, K]");
    pp = pin_a.data();
  }
  py::array_t<double> out({G, K});
  const int32_t* wp = wids.data();
  const double* ip = iters.data();
  const uint8_t* mp = mask.data();
  const double* sp = starts.data();
  double* op = out.mutable_data();
  const double* A = alone.data();
  const double* Cm = cmat.data();
  {
    py::gil_scoped_release nogil;
    for (py::ssize_t g = 0; g < G; ++g) {
      int32_t w[kMaxK];
      double it[kMaxK], st[kMaxK], fin[kMaxK], pe[kMaxK];
      int idx[kMaxK], k = 0;
      for (py::ssize_t j = 0; j < K; ++j) {
        op[g * K + j] = 0.0;
        if (!mp[g * K + j]) continue;
        const int32_t x = wp[g * K + j];
        if (x < 0 || x >= W) throw std::runtime_error("corun_times: workload id out of range");
        w[k] = x;
        it[k] = ip[g * K + j];
        st[k] = sp[g * K + j];
        pe[k] = pp ? pp[g * K + j] : 0.0;
        idx[k++] = (int)j;
      }
      sim_group(k, w, it, st, A, Cm, W, fin, pp ? pe : nullptr);
      for (int i = 0; i < k; ++i) op[g * K + idx[i]] = fin[i];
    }
  }
  return out;
}

// Score-time evaluation of candidate GPUs for one incoming pod.  Residents per GPU in CSR form
// (off[g]..off[g+1]); for every candidate GPU: SLO misses before / after adding the pod,
// makespan before / after, and the incoming pod's predicted throughput there.
py::tuple corun_gpu_eval(I64 off, I32 r_wid, F64 r_iters, F64 r_slo, int x_wid, double x_iters, double x_slo,
                         I32 cand_gpu, F64 alone, F64 cmat) {
  int W;
  check_model(alone, cmat, W);
  const py::ssize_t NG = off.shape(0) - 1, NR = r_wid.shape(0), NC = cand_gpu.shape(0);
  if (NG < 0 || r_iters.shape(0) != NR || r_slo.shape(0) != NR) throw std::runtime_error("corun_gpu_eval: shapes");
  const int64_t* O = off.data();
  if (O[0] != 0 || O[NG] != NR) throw std::runtime_error("corun_gpu_eval: bad offsets");
  for (py::ssize_t g = 0; g < NG; ++g)
    if (O[g + 1] < O[g] || O[g + 1] - O[g] >= kMaxK) throw std::runtime_error("corun_gpu_eval: bad offsets");
  check_wids(r_wid.data(), NR, W, "residents");
  if (x_wid < 0 || x_wid >= W) throw std::runtime_error("corun_gpu_eval: incoming workload id out of range");
  py::array_t<int32_t> bb(NC), ba(NC);
  py::array_t<double> mb(NC), ma(NC), xt(NC);
  const int32_t* cg = cand_gpu.data();
  for (py::ssize_t c = 0; c < NC; ++c)
    if (cg[c] < 0 || cg[c] >= NG) throw std::runtime_error("corun_gpu_eval: candidate GPU out of range");
  {
    py::gil_scoped_release nogil;
    for (py::ssize_t c = 0; c < NC; ++c) {
      const int g = cg[c];
      const int n = (int)(O[g + 1] - O[g]);
      int32_t w[kMaxK];
      double it[kMaxK], sl[kMaxK], tp[kMaxK];
      for (int i = 0; i < n; ++i) {
        w[i] = r_wid.data()[O[g] + i];
        it[i] = r_iters.data()[O[g] + i];
        sl[i] = r_slo.data()[O[g] + i];
      }
      const GroupEval before = eval_group(n, w, it, sl, alone.data(), cmat.data(), W);
      w[n] = x_wid;
      it[n] = x_iters;
      sl[n] = x_slo;
      const GroupEval after = eval_group(n + 1, w, it, sl, alone.data(), cmat.data(), W, tp);
      bb.mutable_data()[c] = before.bad;
      ba.mutable_data()[c] = after.bad;
      mb.mutable_data()[c] = before.makespan;
      ma.mutable_data()[c] = after.makespan;
      xt.mutable_data()[c] = tp[n];
    }
  }
  return py::make_tuple(bb, ba, mb, ma, xt);
}

// Every group's SLO misses and makespan as it stands (CSR residents per group).
py::tuple corun_groups_eval(I64 off, I32 r_wid, F64 r_iters, F64 r_slo, F64 alone, F64 cmat) {
  int W;
  check_model(alone, cmat, W);
  const py::ssize_t NG = off.shape(0) - 1, NR = r_wid.shape(0);
  if (NG < 0 || r_iters.shape(0) != NR || r_slo.shape(0) != NR) throw std::runtime_error("corun_groups_eval: shapes");
  const int64_t* O = off.data();
  if (O[0] != 0 || O[NG] != NR) throw std::runtime_error("corun_groups_eval: bad offsets");
  for (py::ssize_t g = 0; g < NG; ++g)
    if (O[g + 1] < O[g] || O[g + 1] - O[g] > kMaxK) throw std::runtime_error("corun_groups_eval: bad offsets");
  check_wids(r_wid.data(), NR, W, "residents");
  py::array_t<int32_t> bad(NG);
  py::array_t<double> mk(NG);
  for (py::ssize_t g = 0; g < NG; ++g) {
    const int n = (int)(O[g + 1] - O[g]);
    const GroupEval e = eval_group(n, r_wid.data() + O[g], r_iters.data() + O[g], r_slo.data() + O[g], alone.data(),
                                   cmat.data(), W);
    bad.mutable_data()[g] = e.bad;
    mk.mutable_data()[g] = e.makespan;
  }
  return py::make_tuple(bad, mk);
}

// Joint placement of a burst of P pods over D devices (GPU dev_gpu[d], dev_free[d] free
// units BEFORE the burst) next to fixed residents (CSR per GPU).  dev_in = a feasible initial
// assignment.  Two phases of first-improvement local search (moves into free capacity and
// swaps of equal-unit pods across GPUs):
//   A  makespan: lower the pair's longer predicted group makespan (sum of squares as the
//      tie-break) -- the balanced plan, M0 = its longest GPU;
//   B  SLO: more members (burst + residents) predicted to meet their SLO (sigma > 0: the
//      EXPECTED number under lognormal model error of that sigma), never taking a GPU
//      above cap = (1 + tolerance) * M0 (or above its current makespan, if already over);
//      equal count -> the smaller total SLO deficit (sum of 1 - tput / SLO over the misses: a
//      gradient toward placements one swap away from meeting more), then the lower makespan.
// mode: 0 = A then B, 1 = A only (balance), 2 = B only (cap from the initial plan).
// base (optional, per GPU, ms): backlog carried from earlier bursts.  Both phases then see
// base[g] + makespan[g], and B's cap becomes the balanced plan's longest base + makespan plus
// tolerance x its longest makespan: a GPU that took extra work for SLOs in one burst gets
// lighter groups in the next ones, so the per-burst slack does not pile up on one GPU of a
// pipelined multi-GPU job (the busiest GPU's cumulative work paces it).
py::array_t<int32_t> plan_corun(I32 dev_in, I32 units, I32 wid, F64 iters, F64 slo, I32 dev_gpu, I32 dev_free,
                                I64 res_off, I32 r_wid, F64 r_iters, F64 r_slo, F64 alone, F64 cmat, int sweeps,
                                double tolerance, int mode, double sigma, py::object base_obj) {
  int W;
  check_model(alone, cmat, W);
  const py::ssize_t P = dev_in.shape(0), D = dev_gpu.shape(0), NR = r_wid.shape(0);
  if (units.shape(0) != P || wid.shape(0) != P || iters.shape(0) != P || slo.shape(0) != P)
    throw std::runtime_error("plan_corun: pod array shapes differ");
  if (dev_free.shape(0) != D) throw std::runtime_error("plan_corun: device array shapes differ");
  if (r_iters.shape(0) != NR || r_slo.shape(0) != NR) throw std::runtime_error("plan_corun: resident shapes differ");
  check_wids(wid.data(), P, W, "burst");
  check_wids(r_wid.data(), NR, W, "residents");
  int NG = 0;
  for (py::ssize_t d = 0; d < D; ++d) {
    if (dev_gpu.data()[d] < 0) throw std::runtime_error("plan_corun: negative GPU id");
    NG = std::max(NG, dev_gpu.data()[d] + 1);
  }
  if (res_off.shape(0) != NG + 1) throw std::runtime_error("plan_corun: res_off must have n_gpu + 1 entries");
  const int64_t* RO = res_off.data();
  if (RO[0] != 0 || RO[NG] != NR) throw std::runtime_error("plan_corun: bad resident offsets");
  // base[g]: GPU g's backlog in ms (work planned onto it by earlier bursts beyond the least
  // loaded GPU's); the objectives see base[g] + the group's makespan
  std::vector<double> B(NG, 0.0);
  if (!base_obj.is_none()) {
    F64 base = base_obj.cast<F64>();
    if (base.ndim() != 1 || base.shape(0) != NG) throw std::runtime_error("plan_corun: base must have n_gpu entries");
    for (int g = 0; g < NG; ++g) {
      B[g] = base.data()[g];
      if (!std::isfinite(B[g]) || B[g] < 0) throw std::runtime_error("plan_corun: base must be finite and >= 0");
    }
  }
  std::vector<int32_t> dev(dev_in.data(), dev_in.data() + P);
  std::vector<int> free(dev_free.data(), dev_free.data() + D);
  const int32_t* U = units.data();
  const int32_t* DG = dev_gpu.data();
  for (py::ssize_t p = 0; p < P; ++p) {
    if (dev[p] < 0 || dev[p] >= D) throw std::runtime_error("plan_corun: device index out of range");
    free[dev[p]] -= U[p];
  }
  for (py::ssize_t d = 0; d < D; ++d)
    if (free[d] < 0) throw std::runtime_error("plan_corun: initial assignment over capacity");
  const double* A = alone.data();
  const double* Cm = cmat.data();
  py::array_t<int32_t> out(P);
  {
    py::gil_scoped_release nogil;
    // members of each GPU: burst pods by index (>= 0), residents encoded -1 - r
    std::vector<std::vector<int>> mem(NG);
    for (int g = 0; g < NG; ++g)
      for (int64_t r = RO[g]; r < RO[g + 1]; ++r) mem[g].push_back(-1 - (int)r);
    for (py::ssize_t p = 0; p < P; ++p) mem[DG[dev[p]]].push_back((int)p);
    auto eval = [&](int g) {
      const auto& v = mem[g];
      const int k = (int)v.size();
      if (k > kMaxK) throw std::runtime_error("plan_corun: GPU group larger than 64 pods");
      int32_t w[kMaxK];
      double it[kMaxK], sl[kMaxK];
      for (int i = 0; i < k; ++i) {
        const int a = v[i];
        w[i] = a >= 0 ? wid.data()[a] : r_wid.data()[-1 - a];
        it[i] = a >= 0 ? iters.data()[a] : r_iters.data()[-1 - a];
        sl[i] = a >= 0 ? slo.data()[a] : r_slo.data()[-1 - a];
      }
      return eval_group(k, w, it, sl, A, Cm, W, nullptr, sigma);
    };
    std::vector<GroupEval> ge(NG);
    for (int g = 0; g < NG; ++g) ge[g] = eval(g);
    auto replace = [&](int g, int from, int to) {
      for (int& x : mem[g])
        if (x == from) { x = to; return; }
    };
    auto remove = [&](int g, int x) {
      auto& v = mem[g];
      v.erase(std::find(v.begin(), v.end(), x));
    };
    const double eps = 1e-9;
    // phase runner: crit(before_i, before_j, after_i, after_j) -> accept
    auto run_phase = [&](auto&& accept) {
      for (int sw = 0; sw < sweeps; ++sw) {
        bool improved = false;
        // moves into free capacity on another GPU
        for (py::ssize_t p = 0; p < P; ++p) {
          const int d0 = dev[p], g0 = DG[d0];
          for (py::ssize_t d = 0; d < D; ++d) {
            const int g1 = DG[d];
            if (g1 == g0 || free[d] < U[p]) continue;
            remove(g0, (int)p);
            mem[g1].push_back((int)p);
            const GroupEval a0 = eval(g0), a1 = eval(g1);
            if (accept(g0, g1, ge[g0], ge[g1], a0, a1)) {
              free[d0] += U[p];
              free[d] -= U[p];
              dev[p] = (int32_t)d;
              ge[g0] = a0;
              ge[g1] = a1;
              improved = true;
              break;
            }
            remove(g1, (int)p);
            mem[g0].push_back((int)p);
          }
        }
        // swaps of equal-size pods across GPUs
        for (py::ssize_t i = 0; i < P; ++i) {
          for (py::ssize_t j = i + 1; j < P; ++j) {
            const int di = dev[i], dj = dev[j], gi = DG[di], gj = DG[dj];
            if (gi == gj || U[i] != U[j]) continue;
            replace(gi, (int)i, (int)j);
            replace(gj, (int)j, (int)i);
            const GroupEval ai = eval(gi), aj = eval(gj);
            if (accept(gi, gj, ge[gi], ge[gj], ai, aj)) {
              dev[i] = dj;
              dev[j] = di;
              ge[gi] = ai;
              ge[gj] = aj;
              improved = true;
            } else {
              replace(gi, (int)j, (int)i);
              replace(gj, (int)i, (int)j);
            }
          }
        }
        if (!improved) break;
      }
    };
    auto max_mk = [&](bool eff) {
      double m = 0;
      for (int g = 0; g < NG; ++g) m = std::max(m, ge[g].makespan + (eff ? B[g] : 0.0));
      return m;
    };
    if (mode == 0 || mode == 1) {
      run_phase([&](int gi, int gj, const GroupEval& bi, const GroupEval& bj, const GroupEval& ai, const GroupEval& aj) {
        const double mb = std::max(B[gi] + bi.makespan, B[gj] + bj.makespan);
        const double ma = std::max(B[gi] + ai.makespan, B[gj] + aj.makespan);
        if (ma < mb * (1 - eps)) return true;
        if (ma > mb * (1 + eps)) return false;
        const double xi = B[gi] + bi.makespan, xj = B[gj] + bj.makespan;
        const double yi = B[gi] + ai.makespan, yj = B[gj] + aj.makespan;
        return yi * yi + yj * yj < (xi * xi + xj * xj) * (1 - 1e-6);
      });
    }
    if (mode == 0 || mode == 2) {
      // headroom of tolerance x the balanced plan's longest GROUP (not its backlog)
      const double cap = max_mk(true) + std::max(tolerance, 0.0) * max_mk(false);
      run_phase([&](int gi, int gj, const GroupEval& bi, const GroupEval& bj, const GroupEval& ai, const GroupEval& aj) {
        const bool over = (B[gi] + ai.makespan > cap * (1 + eps) && ai.makespan > bi.makespan * (1 + eps)) ||
                          (B[gj] + aj.makespan > cap * (1 + eps) && aj.makespan > bj.makespan * (1 + eps));
        if (over) return false;
        const double mb = std::max(B[gi] + bi.makespan, B[gj] + bj.makespan);
        const double ma = std::max(B[gi] + ai.makespan, B[gj] + aj.makespan);
        if (sigma > 0) {          // soft objective: expected SLOs met under model error
          const double eb = bi.expected + bj.expected, ea = ai.expected + aj.expected;
          if (ea > eb + 1e-6) return true;
          if (ea < eb - 1e-6) return false;
          return ma < mb * (1 - eps);
        }
        const int ob = bi.ok + bj.ok, oa = ai.ok + aj.ok;
        if (oa != ob) return oa > ob;
        const double fb = bi.deficit + bj.deficit, fa = ai.deficit + aj.deficit;
        if (fa < fb - 1e-6) return true;
        if (fa > fb + 1e-6) return false;
        return ma < mb * (1 - eps);
      });
    }
  }
  std::copy(dev.begin(), dev.end(), out.mutable_data());
  return out;
}

}  // namespace

void register_corun(py::module_& m) {
  m.def("corun_times", &corun_times, py::arg("wids"), py::arg("iters"), py::arg("mask"), py::arg("starts"),
        py::arg("alone_ms"), py::arg("cmat"), py::arg("pin_end") = py::none());
  m.def("corun_gpu_eval", &corun_gpu_eval, py::arg("off"), py::arg("r_wid"), py::arg("r_iters"), py::arg("r_slo"),
        py::arg("x_wid"), py::arg("x_iters"), py::arg("x_slo"), py::arg("cand_gpu"), py::arg("alone_ms"),
        py::arg("cmat"));
  m.def("corun_groups_eval", &corun_groups_eval, py::arg("off"), py::arg("r_wid"), py::arg("r_iters"),
        py::arg("r_slo"), py::arg("alone_ms"), py::arg("cmat"));
  m.def("plan_corun", &plan_corun, py::arg("dev"), py::arg("units"), py::arg("wid"), py::arg("iters"), py::arg("slo"),
        py::arg("dev_gpu"), py::arg("dev_free"), py::arg("res_off"), py::arg("r_wid"), py::arg("r_iters"),
        py::arg("r_slo"), py::arg("alone_ms"), py::arg("cmat"), py::arg("sweeps") = 8, py::arg("tolerance") = 0.03,
        py::arg("mode") = 0, py::arg("sigma") = 0.0, py::arg("base") = py::none());
}
