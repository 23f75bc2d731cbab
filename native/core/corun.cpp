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
#include <cstring>
#include <condition_variable>
#include <memory>
#include <deque>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <limits>
#include <mutex>
#include <shared_mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

constexpr double kBig = 1e300;
constexpr int kMaxK = 64;   // pods per GPU group (CPX: 64 devices of 4 CUs would be the extreme)

// A tiny fork-join pool for the planner's candidate batches (tens of microseconds each, a few
// hundred per plan): T-1 workers spin on a generation counter for the duration of one plan
// call (no sleeping: a futex wake-up costs more than a batch), the caller takes share 0.
class SpinPool {
 public:
  explicit SpinPool(int t) : T_(t) {
    for (int k = 1; k < T_; ++k)
      th_.emplace_back([this, k] {
        int seen = 0;
        for (;;) {
          int e;
          while ((e = gen_.load(std::memory_order_acquire)) == seen) __builtin_ia32_pause();
          seen = e;
          if (quit_.load(std::memory_order_acquire)) return;
          (*fn_)(k);
          left_.fetch_sub(1, std::memory_order_acq_rel);
        }
      });
  }
  void run(const std::function<void(int)>& f) {
    fn_ = &f;
    left_.store(T_ - 1, std::memory_order_relaxed);
    gen_.fetch_add(1, std::memory_order_acq_rel);
    f(0);
    while (left_.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
  }
  ~SpinPool() {
    quit_.store(true, std::memory_order_release);
    gen_.fetch_add(1, std::memory_order_acq_rel);
    for (auto& t : th_) t.join();
  }

 private:
  int T_;
  std::vector<std::thread> th_;
  std::atomic<int> gen_{0}, left_{0};
  std::atomic<bool> quit_{false};
  const std::function<void(int)>* fn_ = nullptr;
};

// Open-addressing map from 64-bit keys (already well mixed) to values kept in a deque, so a
// pointer to a value stays valid while other keys are inserted (the planner's memos: a few
// thousand inserts and several times as many lookups per plan -- a node-based map allocated per
// insert and chased a pointer per lookup).
template <class V>
class FlatMap {
 public:
  explicit FlatMap(size_t cap = 1024) { rehash(cap); }
  V* find(uint64_t k) {
    for (size_t i = k & mask_;; i = (i + 1) & mask_) {
      const int32_t x = idx_[i];
      if (x < 0) return nullptr;
      if (keys_[i] == k) return &vals_[(size_t)x];
    }
  }
  V* insert(uint64_t k, const V& v) {        // (k must not be present)
    if ((vals_.size() + 1) * 2 > idx_.size()) rehash(idx_.size() * 2);
    size_t i = k & mask_;
    while (idx_[i] >= 0) i = (i + 1) & mask_;
    keys_[i] = k;
    idx_[i] = (int32_t)vals_.size();
    vals_.push_back(v);
    return &vals_.back();
  }
  size_t size() const { return vals_.size(); }

 private:
  void rehash(size_t cap) {
    std::vector<uint64_t> ok = std::move(keys_);
    std::vector<int32_t> oi = std::move(idx_);
    keys_.assign(cap, 0);
    idx_.assign(cap, -1);
    mask_ = cap - 1;
    for (size_t j = 0; j < oi.size(); ++j) {
      if (oi[j] < 0) continue;
      size_t i = ok[j] & mask_;
      while (idx_[i] >= 0) i = (i + 1) & mask_;
      keys_[i] = ok[j];
      idx_[i] = oi[j];
    }
  }
  std::vector<uint64_t> keys_;
  std::vector<int32_t> idx_;
  std::deque<V> vals_;
  size_t mask_ = 0;
};

// fin[i] = wall ms at which pod i finishes (kBig for a service pod); tput_ms[i] = ms per
// iteration achieved (fin / iters, or the steady-state ms/iter of a service pod).
// pin_end (optional): a member with pin_end[i] > start[i] is PINNED -- present exactly during
// [start, pin_end) (a co-runner whose interval was measured), pressing on the others but not
// simulated itself; fin[i] = pin_end[i].  Learning from a pipeline's timeline conditions the
// observed pods on what their co-runners really did, instead of re-simulating co-runners whose
// own (earlier) co-runners lie outside the observed window.
void sim_group(int k, const int32_t* w, const double* iters, const double* start, const double* alone,
               const double* C, int W, double* fin, const double* pin_end = nullptr) {
  double rem[kMaxK], st[kMaxK], pe[kMaxK], load[kMaxK];
  bool started[kMaxK], done[kMaxK], svc[kMaxK], pin[kMaxK];
  for (int i = 0; i < k; ++i) {
    svc[i] = iters[i] <= 0;
    st[i] = start ? start[i] : 0.0;
    pin[i] = pin_end && pin_end[i] > st[i];
    pe[i] = pin[i] ? pin_end[i] : 0.0;
    rem[i] = (svc[i] || pin[i]) ? kBig : std::max(alone[w[i]] * iters[i], 1e-12);
    started[i] = done[i] = false;
    fin[i] = pin[i] ? pe[i] : svc[i] ? kBig : 0.0;
    load[i] = 1.0;
  }
  // load[i] = 1 + sum over ACTIVE j != i of C[w_i][w_j], kept up to date at every start / end
  // (O(k) per event instead of O(k^2) per step)
  auto press = [&](int j, double sign) {
    const double* cj = C + (size_t)w[j];
    for (int i = 0; i < k; ++i)
      if (i != j) load[i] += sign * cj[(size_t)w[i] * W];
  };
  double now = 0.0;
  for (int step = 0; step < 3 * k + 1; ++step) {
    bool live = false;
    for (int i = 0; i < k; ++i) live |= !done[i] && !svc[i] && !pin[i];
    if (!live) break;
    for (int i = 0; i < k; ++i)
      if (!started[i] && st[i] <= now + 1e-12) started[i] = true, press(i, 1.0);
    for (int i = 0; i < k; ++i)
      if (pin[i] && started[i] && !done[i] && pe[i] <= now + 1e-12) done[i] = true, press(i, -1.0);
    double rate[kMaxK];
    double dt = kBig;
    int am = -1;
    double am_t = kBig;
    for (int i = 0; i < k; ++i) {
      rate[i] = 0.0;
      if (!started[i] || done[i] || pin[i]) continue;
      rate[i] = 1.0 / load[i];
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
        press(i, -1.0);
      }
    }
  }
}

// Pipeline simulation of one GPU: members are chained per CU slot -- member i with prev[i] >= 0
// starts the moment member prev[i] finishes (a slot's stream runs its pods back to back, the
// executor's launch-ahead pipeline), but not before start[i] (its release: when the host
// enqueued it; pass a very negative value for none); a member with prev[i] < 0 at start[i].  Pinned members
// (pin_end[i] > start[i], prev[i] < 0) are present exactly in [start, pin_end): measured
// intervals of pods that already ran.  st_out[i] / fin[i] = predicted start / finish (kBig when
// it never starts, e.g. chained behind a service).
// t_stop / rem_out (optional): stop the simulation at wall time t_stop (events AT t_stop are
// processed) and report every member's remaining work there (ms of alone time; kBig for pinned
// and service members) -- plan_slots fast-forwards the shared context prefix with it.
void sim_chain(int k, const int32_t* w, const double* iters, const double* start, const int32_t* prev,
               const double* alone, const double* C, int W, double* st_out, double* fin,
               const double* pin_end = nullptr, double t_stop = kBig, double* rem_out = nullptr) {
  double rem[kMaxK], load[kMaxK];
  bool started[kMaxK], done[kMaxK], svc[kMaxK], pin[kMaxK], known[kMaxK];
  double now = kBig;
  for (int i = 0; i < k; ++i) {
    svc[i] = iters[i] <= 0;
    known[i] = prev[i] < 0;
    st_out[i] = known[i] ? start[i] : kBig;
    pin[i] = known[i] && pin_end && pin_end[i] > start[i];
    rem[i] = (svc[i] || pin[i]) ? kBig : std::max(alone[w[i]] * iters[i], 1e-12);
    started[i] = done[i] = false;
    fin[i] = pin[i] ? pin_end[i] : kBig;
    load[i] = 1.0;
    if (known[i]) now = std::min(now, st_out[i]);
  }
  if (now >= kBig) return;
  // incrementally maintained loads, as sim_group
  auto press = [&](int j, double sign) {
    const double* cj = C + (size_t)w[j];
    for (int i = 0; i < k; ++i)
      if (i != j) load[i] += sign * cj[(size_t)w[i] * W];
  };
  for (int step = 0; step < 4 * k + 2; ++step) {
    bool live = false;
    for (int i = 0; i < k; ++i) live |= !done[i] && !svc[i] && !pin[i];
    if (!live) break;
    // pinned members whose interval ends now leave first, so a pod chained behind one starts at
    // this same instant (it used to wait for the next event, one step late)
    for (int i = 0; i < k; ++i)
      if (pin[i] && started[i] && !done[i] && fin[i] <= now + 1e-12) done[i] = true, press(i, -1.0);
    for (int i = 0; i < k; ++i) {
      if (started[i]) continue;
      if (!known[i] && done[prev[i]]) {
        known[i] = true;
        st_out[i] = std::max(fin[prev[i]], start[i]);
      }
      if (known[i] && st_out[i] <= now + 1e-12) started[i] = true, press(i, 1.0);
    }
    // (a pinned member that starts now and ends now never presses)
    for (int i = 0; i < k; ++i)
      if (pin[i] && started[i] && !done[i] && fin[i] <= now + 1e-12) done[i] = true, press(i, -1.0);
    double rate[kMaxK];
    int am = -1;
    double am_t = kBig;
    for (int i = 0; i < k; ++i) {
      rate[i] = 0.0;
      if (!started[i] || done[i] || pin[i]) continue;
      rate[i] = 1.0 / load[i];
      if (!svc[i]) {
        const double t = rem[i] / std::max(rate[i], 1e-30);
        if (t < am_t) am_t = t, am = i;
      }
    }
    double dt = am_t;
    for (int i = 0; i < k; ++i) {
      if (!started[i] && known[i]) dt = std::min(dt, st_out[i] - now);
      else if (pin[i] && started[i] && !done[i]) dt = std::min(dt, fin[i] - now);
    }
    if (dt >= kBig) break;          // nothing left that can progress (chained behind a service)
    dt = std::max(dt, 0.0);
    if (now + dt > t_stop) {        // fast-forward mode: advance to t_stop and stop
      for (int i = 0; i < k; ++i)
        if (started[i] && !done[i] && !svc[i] && !pin[i]) rem[i] -= rate[i] * (t_stop - now);
      break;
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
        press(i, -1.0);
      }
    }
  }
  if (rem_out)
    for (int i = 0; i < k; ++i) rem_out[i] = done[i] ? 0.0 : rem[i];
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
// pipe (optional): each GPU's slot pipelines, for the SLO phase.  A tuple (c_off [NG+1], c_wid,
// c_start, c_end, f_off [NG+1], f_time): per GPU the in-flight pods of earlier placements with
// their (measured or predicted) intervals, pinned as co-runners, and the times its free CU slots
// become free.  With it, phase B counts SLOs met on the pipeline -- the GPU's new pods start at
// its slot free times (longest first on the earliest slot) next to the in-flight pods -- instead
// of on the group in isolation; the makespans (phase A, the cap) stay the group's own.
py::array_t<int32_t> plan_corun(I32 dev_in, I32 units, I32 wid, F64 iters, F64 slo, I32 dev_gpu, I32 dev_free,
                                I64 res_off, I32 r_wid, F64 r_iters, F64 r_slo, F64 alone, F64 cmat, int sweeps,
                                double tolerance, int mode, double sigma, py::object base_obj, py::object pipe_obj,
                                py::object hbm_obj, py::object dev_hbm_obj, int sweeps_b, py::object speed_obj) {
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
  // speed[g] (optional): GPU g's measured time / predicted time relative to its siblings
  // (planner.observe_time).  Its group makespans are scaled by it in both phases, so a burst is
  // balanced in MEASURED time -- without it a 40 %-slow GPU got balanced (model) work every
  // burst and only the carried backlog pulled it back, one burst late (shares oscillating
  // 0.34 / 0.48 / 0.57 on MI355X); the SLO counts stay the model's
  std::vector<double> S(NG, 1.0);
  if (!speed_obj.is_none()) {
    F64 sp = speed_obj.cast<F64>();
    if (sp.ndim() != 1 || sp.shape(0) != NG) throw std::runtime_error("plan_corun: speed must have n_gpu entries");
    for (int g = 0; g < NG; ++g) {
      S[g] = sp.data()[g];
      if (!std::isfinite(S[g]) || S[g] <= 0) throw std::runtime_error("plan_corun: speed must be finite and > 0");
    }
  }
  // pipeline context (see above)
  bool pipe = false, phantoms = false;
  I64 p_coff, p_foff;
  I32 p_cwid, p_hwid;
  F64 p_cst, p_cend, p_ft, p_hit;
  if (!pipe_obj.is_none()) {
    py::tuple t = pipe_obj.cast<py::tuple>();
    if (t.size() != 6 && t.size() != 8)
      throw std::runtime_error("plan_corun: pipe must be (c_off, c_wid, c_start, c_end, f_off, f_time[, h_wid, h_iters])");
    p_coff = t[0].cast<I64>();
    p_cwid = t[1].cast<I32>();
    p_cst = t[2].cast<F64>();
    p_cend = t[3].cast<F64>();
    p_foff = t[4].cast<I64>();
    p_ft = t[5].cast<F64>();
    const py::ssize_t NC = p_cwid.shape(0);
    if (p_coff.shape(0) != NG + 1 || p_foff.shape(0) != NG + 1 || p_cst.shape(0) != NC || p_cend.shape(0) != NC)
      throw std::runtime_error("plan_corun: pipe array shapes");
    if (p_coff.data()[0] != 0 || p_coff.data()[NG] != NC || p_foff.data()[0] != 0 ||
        p_foff.data()[NG] != p_ft.shape(0))
      throw std::runtime_error("plan_corun: pipe offsets");
    for (int g = 0; g < NG; ++g)
      if (p_coff.data()[g + 1] < p_coff.data()[g] || p_foff.data()[g + 1] < p_foff.data()[g])
        throw std::runtime_error("plan_corun: pipe offsets");
    check_wids(p_cwid.data(), NC, W, "pipe context");
    if (t.size() == 8) {
      // per free slot: the pod its stream runs next (-1 none), chained after the slot's new pod
      p_hwid = t[6].cast<I32>();
      p_hit = t[7].cast<F64>();
      if (p_hwid.shape(0) != p_ft.shape(0) || p_hit.shape(0) != p_ft.shape(0))
        throw std::runtime_error("plan_corun: pipe phantoms must have one entry per free slot");
      for (py::ssize_t i = 0; i < p_hwid.shape(0); ++i)
        if (p_hwid.data()[i] >= W) throw std::runtime_error("plan_corun: phantom workload id out of range");
      phantoms = true;
    }
    pipe = true;
  }
  // optional HBM: per pod GiB (hbm) and per device free GiB before the burst (dev_hbm); moves
  // and swaps then keep every device within its free HBM, as the initial assignment does
  std::vector<double> H(P, 0.0), hfree(D, 1e300);
  if (!hbm_obj.is_none() || !dev_hbm_obj.is_none()) {
    if (hbm_obj.is_none() || dev_hbm_obj.is_none()) throw std::runtime_error("plan_corun: hbm and dev_hbm go together");
    F64 hb = hbm_obj.cast<F64>(), dh = dev_hbm_obj.cast<F64>();
    if (hb.ndim() != 1 || hb.shape(0) != P || dh.ndim() != 1 || dh.shape(0) != D)
      throw std::runtime_error("plan_corun: hbm must have one entry per pod, dev_hbm one per device");
    for (py::ssize_t p = 0; p < P; ++p) H[p] = hb.data()[p];
    for (py::ssize_t d = 0; d < D; ++d) hfree[d] = dh.data()[d];
  }
  std::vector<int32_t> dev(dev_in.data(), dev_in.data() + P);
  std::vector<int> free(dev_free.data(), dev_free.data() + D);
  const int32_t* U = units.data();
  const int32_t* DG = dev_gpu.data();
  for (py::ssize_t p = 0; p < P; ++p) {
    if (dev[p] < 0 || dev[p] >= D) throw std::runtime_error("plan_corun: device index out of range");
    free[dev[p]] -= U[p];
    hfree[dev[p]] -= H[p];
  }
  for (py::ssize_t d = 0; d < D; ++d)
    if (free[d] < 0 || hfree[d] < -1e-5) throw std::runtime_error("plan_corun: initial assignment over capacity");
  const double* A = alone.data();
  const double* Cm = cmat.data();
  py::array_t<int32_t> out(P);
  {
    py::gil_scoped_release nogil;
    // members of each GPU: burst pods by index (>= 0), residents encoded -1 - r
    std::vector<std::vector<int>> mem(NG);
    for (int g = 0; g < NG; ++g)
      for (int64_t r = RO[g]; r < RO[g + 1]; ++r) mem[g].push_back(-1 - (int)r);
    std::vector<int> nburst(NG, 0);                  // burst pods per GPU
    for (py::ssize_t p = 0; p < P; ++p) mem[DG[dev[p]]].push_back((int)p), ++nburst[DG[dev[p]]];
    bool use_pipe = false, phase_b = false;
    // Simulation memos keyed by a group's WORKLOAD multiset, not by its pod indices: pods of one
    // workload and length are interchangeable in a simulation and a burst repeats workloads, so
    // most candidate moves / swaps re-evaluate a multiset that was already simulated (8-GPU bench
    // epochs: ~2.5k simulations per phase collapse to a few hundred).  A plain group simulation
    // (every member starts at once) depends on nothing else and is shared by both phases and
    // every GPU; a pipeline simulation also depends on the GPU (its in-flight context and free
    // slots) and on which members are residents.  SLO verdicts are evaluated per member on top.
    auto mix = [](uint64_t h, uint64_t x) {
      uint64_t z = h + 0x9e3779b97f4a7c15ull + x;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      return z ^ (z >> 31);
    };
    auto dbits = [](double d) {
      uint64_t u;
      std::memcpy(&u, &d, sizeof u);
      return u;
    };
    struct PlainSim {
      double makespan;
      double tput[kMaxK];          // iterations/s per member, in the canonical (w, it) order
    };
    FlatMap<PlainSim> plain_memo(2048);
    FlatMap<std::array<double, kMaxK>> pipe_memo(2048);
    std::shared_mutex sim_mu;
    std::atomic<long> n_plain{0}, n_pipe{0};
    const bool threaded = std::getenv("GPUSCHED_PLAN_THREADS") && std::atoi(std::getenv("GPUSCHED_PLAN_THREADS")) > 1;
    auto eval_raw = [&](int g, const std::vector<int>& v) {
      const int k = (int)v.size();
      if (k > kMaxK) throw std::runtime_error("plan_corun: GPU group larger than 64 pods");
      int32_t w[kMaxK];
      double it[kMaxK], sl[kMaxK];
      bool res[kMaxK];
      for (int i = 0; i < k; ++i) {
        const int a = v[i];
        w[i] = a >= 0 ? wid.data()[a] : r_wid.data()[-1 - a];
        it[i] = a >= 0 ? iters.data()[a] : r_iters.data()[-1 - a];
        sl[i] = a >= 0 ? slo.data()[a] : r_slo.data()[-1 - a];
        res[i] = a < 0;
      }
      // plain simulation on the canonical (w, it) order
      int ord[kMaxK];
      for (int i = 0; i < k; ++i) ord[i] = i;
      std::sort(ord, ord + k, [&](int a, int b) { return w[a] != w[b] ? w[a] < w[b] : it[a] < it[b]; });
      uint64_t hk = mix(0x5bd1e995ull, (uint64_t)k);
      for (int q = 0; q < k; ++q) hk = mix(mix(hk, (uint64_t)(uint32_t)w[ord[q]]), dbits(it[ord[q]]));
      // memo hits are used in place (node-based map: references stay valid across inserts)
      const PlainSim* psp = nullptr;
      {
        std::shared_lock<std::shared_mutex> lk(sim_mu, std::defer_lock);
        if (threaded) lk.lock();
        psp = plain_memo.find(hk);
      }
      if (!psp) {
        PlainSim ps;
        int32_t cw[kMaxK];
        double cit[kMaxK], fin[kMaxK];
        for (int q = 0; q < k; ++q) cw[q] = w[ord[q]], cit[q] = it[ord[q]];
        sim_group(k, cw, cit, nullptr, A, Cm, W, fin);
        ps.makespan = 0.0;
        for (int q = 0; q < k; ++q) {
          if (cit[q] <= 0) {
            ps.tput[q] = 1e3 / std::max(steady_ms(k, q, cw, A, Cm, W), 1e-12);
          } else {
            ps.tput[q] = cit[q] / std::max(fin[q], 1e-12) * 1e3;
            ps.makespan = std::max(ps.makespan, fin[q]);
          }
        }
        n_plain.fetch_add(1, std::memory_order_relaxed);
        std::unique_lock<std::shared_mutex> lk(sim_mu, std::defer_lock);
        if (threaded) lk.lock();
        psp = plain_memo.find(hk);             // (another thread may have inserted it)
        if (!psp) psp = plain_memo.insert(hk, ps);
      }
      const PlainSim& ps = *psp;
      GroupEval e;
      e.makespan = ps.makespan * S[g];
      const double sg = phase_b ? sigma : 0.0;      // phase A needs makespans only
      auto verdicts = [&](const double* tput, const int* perm) {
        e.ok = e.bad = 0;
        e.deficit = e.expected = 0.0;
        for (int q = 0; q < k; ++q) {
          const int i = perm[q];
          e.expected += p_meet(tput[q], sl[i], sg);
          if (sl[i] <= 0 || tput[q] >= sl[i]) ++e.ok;
          else ++e.bad, e.deficit += 1.0 - tput[q] / sl[i];
        }
      };
      if (!use_pipe) {
        verdicts(ps.tput, ord);
        return e;
      }
      // SLOs on the GPU's pipeline: in-flight pods pinned, new pods at the free slot times
      // (longest first onto the earliest free slot; residents already run), then (phantoms)
      // each slot's next pod chained behind its new one.  Canonical order: residents first, then
      // new pods longest first (ties by workload and length), so the result is a function of
      // the multiset
      const int64_t c0 = p_coff.data()[g], c1 = p_coff.data()[g + 1];
      const int64_t f0 = p_foff.data()[g], f1 = p_foff.data()[g + 1];
      const int nc = (int)(c1 - c0);
      int nh = 0;
      if (phantoms)
        for (int64_t q = f0; q < f1; ++q) nh += p_hwid.data()[q] >= 0;
      if (nc + k + nh > kMaxK) nh = 0;
      if (nc + k > kMaxK) {
        verdicts(ps.tput, ord);
        return e;
      }
      int po[kMaxK];
      for (int i = 0; i < k; ++i) po[i] = i;
      std::sort(po, po + k, [&](int a, int b) {
        if (res[a] != res[b]) return res[a];
        const double wa = A[w[a]] * it[a], wb = A[w[b]] * it[b];
        if (wa != wb) return wa > wb;
        return w[a] != w[b] ? w[a] < w[b] : it[a] < it[b];
      });
      uint64_t hp = mix(mix(0x27d4eb2fULL, (uint64_t)g), (uint64_t)k);
      for (int q = 0; q < k; ++q)
        hp = mix(mix(mix(hp, (uint64_t)res[po[q]]), (uint64_t)(uint32_t)w[po[q]]), dbits(it[po[q]]));
      const std::array<double, kMaxK>* ptp = nullptr;
      {
        std::shared_lock<std::shared_mutex> lk(sim_mu, std::defer_lock);
        if (threaded) lk.lock();
        ptp = pipe_memo.find(hp);
      }
      if (!ptp) {
        std::array<double, kMaxK> pt;
        int32_t pw[kMaxK], pv[kMaxK];
        double pit[kMaxK], pst[kMaxK], pen[kMaxK], pfin[kMaxK], pso[kMaxK];
        for (int c = 0; c < nc; ++c) {
          pw[c] = p_cwid.data()[c0 + c];
          pit[c] = 1.0;
          pst[c] = p_cst.data()[c0 + c];
          pen[c] = p_cend.data()[c0 + c];
          pv[c] = -1;
        }
        const double t0 = f1 > f0 ? p_ft.data()[f0] : 0.0;
        int slot_pod[kMaxK];                       // free slot q -> simulation index of its new pod
        for (int64_t q = 0; q < f1 - f0 && q < kMaxK; ++q) slot_pod[q] = -1;
        int nf = 0;
        for (int q = 0; q < k; ++q) {
          const int i = po[q];
          pw[nc + q] = w[i];
          pit[nc + q] = it[i];
          pen[nc + q] = 0.0;
          pv[nc + q] = -1;
          if (res[i]) {
            pst[nc + q] = t0;
          } else {
            const int64_t fi = std::min<int64_t>(f0 + nf, f1 - 1);
            pst[nc + q] = f1 > f0 ? p_ft.data()[fi] : 0.0;
            if (f1 > f0 && nf < f1 - f0 && fi - f0 < kMaxK) slot_pod[fi - f0] = nc + q;
            ++nf;
          }
        }
        int m = nc + k;
        if (nh > 0)
          for (int64_t q = 0; q < f1 - f0 && q < kMaxK; ++q) {
            const int32_t hw = p_hwid.data()[f0 + q];
            if (hw < 0) continue;
            pw[m] = hw;
            pit[m] = p_hit.data()[f0 + q];
            pen[m] = 0.0;
            if (slot_pod[q] >= 0) {
              pv[m] = slot_pod[q];
              pst[m] = -kBig;
            } else {
              pv[m] = -1;
              pst[m] = p_ft.data()[f0 + q];
            }
            ++m;
          }
        // the simulation clock starts at 0: shift the window (chained members keep -inf)
        double lo = kBig;
        for (int i = 0; i < m; ++i)
          if (pv[i] < 0) lo = std::min(lo, pst[i]);
        for (int i = 0; i < m; ++i) {
          if (pv[i] < 0) pst[i] -= lo;
          if (i < nc) pen[i] -= lo;
        }
        if (nh > 0) {
          sim_chain(m, pw, pit, pst, pv, A, Cm, W, pso, pfin, pen);
        } else {
          sim_group(m, pw, pit, pst, A, Cm, W, pfin, pen);
          for (int i = 0; i < m; ++i) pso[i] = pst[i];
        }
        int32_t cw[kMaxK];
        for (int q = 0; q < k; ++q) cw[q] = w[po[q]];
        for (int q = 0; q < k; ++q) {
          if (pit[nc + q] <= 0) pt[q] = 1e3 / std::max(steady_ms(k, q, cw, A, Cm, W), 1e-12);
          else pt[q] = pit[nc + q] / std::max(pfin[nc + q] - pso[nc + q], 1e-12) * 1e3;
        }
        n_pipe.fetch_add(1, std::memory_order_relaxed);
        std::unique_lock<std::shared_mutex> lk(sim_mu, std::defer_lock);
        if (threaded) lk.lock();
        ptp = pipe_memo.find(hp);
        if (!ptp) ptp = pipe_memo.insert(hp, pt);
      }
      verdicts(ptp->data(), po);
      return e;
    };
    // memo of group evaluations per phase and thread: a sweep re-evaluates mostly the same
    // (GPU, member set) pairs as the previous one -- only the two groups of an accepted move /
    // swap change.  A result is a function of the set.
    // key: an ORDER-FREE 64-bit hash of the set -- the sum of a mixed code per member, with the
    // GPU and the size mixed in -- kept per GPU as members move (Ksum), so a candidate's key is
    // one add / subtract and a memo hit needs no member list at all (a collision among the few
    // thousand sets of one plan is ~1e-12 likely)
    using Memo = FlatMap<GroupEval>;
    auto hm = [](int member) {
      uint64_t z = (uint64_t)(uint32_t)member + 0x9e3779b97f4a7c15ull;
      z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
      z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
      return z ^ (z >> 31);
    };
    auto set_key = [&](int g, uint64_t ksum, size_t k) { return mix(mix(ksum, (uint64_t)g + 0x51ull), (uint64_t)k); };
    std::vector<uint64_t> Ksum(NG, 0);
    for (int g = 0; g < NG; ++g)
      for (int x : mem[g]) Ksum[g] += hm(x);
    // candidate evaluation runs on T threads (GPUSCHED_PLAN_THREADS, default 4): each batch
    // -- every move of one pod, or every swap partner of one pod -- is evaluated in parallel on
    // the current state, then the FIRST accepted candidate in the sequential order is applied,
    // so the plan is exactly the one-thread plan
    // (default 1: at 8 GPUs a batch is 10-30 candidates, mostly memo hits, and the fork-join
    // cost more than it saved -- 21.9 vs 10.1 ms per plan with 4 threads in this container)
    int T = 1;
    if (const char* e = std::getenv("GPUSCHED_PLAN_THREADS")) T = std::max(1, std::atoi(e));
    T = std::max(1, std::min({T, (int)std::max(1u, std::thread::hardware_concurrency()), 16}));
    // one memo per phase shared by the threads (a reader-writer lock: lookups far outnumber
    // inserts once the first sweep has run)
    std::array<Memo, 2> memo{Memo(4096), Memo(4096)};
    std::shared_mutex memo_mu;
    std::atomic<long> n_evals{0};
    // build(v): fills the member list -- only called on a memo miss
    auto eval_key = [&](int g, uint64_t key, auto&& build) {
      auto& M = memo[phase_b ? 1 : 0];
      n_evals.fetch_add(1, std::memory_order_relaxed);
      if (T > 1) {
        std::shared_lock<std::shared_mutex> lk(memo_mu);
        if (const GroupEval* hit = M.find(key)) return *hit;
      } else if (const GroupEval* hit = M.find(key)) {
        return *hit;
      }
      std::vector<int> v;
      build(v);
      std::sort(v.begin(), v.end());
      const GroupEval r = eval_raw(g, v);
      if (T > 1) {
        std::unique_lock<std::shared_mutex> lk(memo_mu);
        if (!M.find(key)) M.insert(key, r);
      } else {
        M.insert(key, r);
      }
      return r;
    };
    std::vector<GroupEval> ge(NG);
    auto eval_all = [&] {
      for (int g = 0; g < NG; ++g)
        ge[g] = eval_key(g, set_key(g, Ksum[g], mem[g].size()),
                         [&](std::vector<int>& v) { v.assign(mem[g].begin(), mem[g].end()); });
    };
    eval_all();
    SpinPool pool(T);
    const double eps = 1e-9;
    // candidate c: a move (pod a -> device b) or a swap (pods a, b); its two changed groups
    struct Cand {
      int a, b, ga, gb;
    };
    struct Out {
      GroupEval ea, eb;
    };
    std::vector<Cand> cand;
    std::vector<Out> res;

    std::atomic<bool> failed{false};
    std::string err;
    std::mutex err_mu;
    auto evaluate = [&](bool swap) {
      res.resize(cand.size());
      const int n = (int)cand.size();
      // a move batch is one pod leaving one GPU for each candidate: its source group (without
      // the pod) is the same for every candidate -- evaluated once
      GroupEval src{};
      if (!swap && n > 0) {
        const Cand& x = cand[0];
        src = eval_key(x.ga, set_key(x.ga, Ksum[x.ga] - hm(x.a), mem[x.ga].size() - 1), [&](std::vector<int>& v) {
          v.assign(mem[x.ga].begin(), mem[x.ga].end());
          v.erase(std::find(v.begin(), v.end(), x.a));
        });
      }
      auto job = [&](int tid) {
        (void)tid;
        for (int c = tid; c < n; c += T) {
          const Cand& x = cand[c];
          try {
            if (swap) {
              res[c].ea = eval_key(x.ga, set_key(x.ga, Ksum[x.ga] - hm(x.a) + hm(x.b), mem[x.ga].size()),
                                   [&](std::vector<int>& v) {
                                     v.assign(mem[x.ga].begin(), mem[x.ga].end());
                                     *std::find(v.begin(), v.end(), x.a) = x.b;
                                   });
              res[c].eb = eval_key(x.gb, set_key(x.gb, Ksum[x.gb] - hm(x.b) + hm(x.a), mem[x.gb].size()),
                                   [&](std::vector<int>& v) {
                                     v.assign(mem[x.gb].begin(), mem[x.gb].end());
                                     *std::find(v.begin(), v.end(), x.b) = x.a;
                                   });
            } else {
              res[c].ea = src;
              res[c].eb = eval_key(x.gb, set_key(x.gb, Ksum[x.gb] + hm(x.a), mem[x.gb].size() + 1),
                                   [&](std::vector<int>& v) {
                                     v.assign(mem[x.gb].begin(), mem[x.gb].end());
                                     v.push_back(x.a);
                                   });
            }
          } catch (const std::exception& ex) {
            std::lock_guard<std::mutex> lk(err_mu);
            failed = true;
            err = ex.what();
          }
        }
      };
      if (T > 1 && n > 1) pool.run(job);
      else job(0);
      if (failed) throw std::runtime_error(err);
    };
    // SLO phase pruning: a move / swap between two GPUs on which every member is predicted to
    // meet its SLO is skipped -- it could only widen margins (the soft objective) or trim a
    // makespan (phase A's job).  8-GPU pipelined simulation, 4 seeds: 68.9 % SLOs met at 4,631
    // pods/s vs 69.3 % at 4,542 without the pruning, for 40 % less planning time.
    auto saturated = [&](const GroupEval& x) { return x.bad == 0; };
    // phase runner: crit(before_i, before_j, after_i, after_j) -> accept
    auto run_phase = [&](auto&& accept) {
      const int nsw = (phase_b && sweeps_b >= 0) ? sweeps_b : sweeps;
      for (int sw = 0; sw < nsw; ++sw) {
        bool improved = false;
        // moves into free capacity on another GPU (the first accepted device per pod)
        for (py::ssize_t p = 0; p < P; ++p) {
          const int d0 = dev[p], g0 = DG[d0];
          // never empty a GPU of its burst pods while the burst has a pod for every GPU: a GPU
          // with free units left idle for a whole burst is a starved pipeline (round 4's driver
          // box put a 4-pod burst on one GPU of two, GPUTEST_r04.json)
          if (P >= NG && nburst[g0] <= 1) continue;
          cand.clear();
          for (py::ssize_t d = 0; d < D; ++d) {
            const int g1 = DG[d];
            if (g1 == g0 || free[d] < U[p] || hfree[d] + 1e-6 < H[p]) continue;
            if (phase_b && saturated(ge[g0]) && saturated(ge[g1])) continue;
            cand.push_back({(int)p, (int)d, g0, g1});
          }
          if (cand.empty()) continue;
          evaluate(false);
          for (size_t c = 0; c < cand.size(); ++c) {
            const int d = cand[c].b, g1 = cand[c].gb;
            if (!accept(g0, g1, ge[g0], ge[g1], res[c].ea, res[c].eb)) continue;
            mem[g0].erase(std::find(mem[g0].begin(), mem[g0].end(), (int)p));
            mem[g1].push_back((int)p);
            Ksum[g0] -= hm((int)p);
            Ksum[g1] += hm((int)p);
            --nburst[g0];
            ++nburst[g1];
            free[d0] += U[p];
            free[d] -= U[p];
            hfree[d0] += H[p];
            hfree[d] -= H[p];
            dev[p] = (int32_t)d;
            ge[g0] = res[c].ea;
            ge[g1] = res[c].eb;
            improved = true;
            break;
          }
        }
        // swaps of equal-size pods across GPUs: partners of pod i in order; after an accepted
        // swap the remaining partners are re-evaluated against pod i's new GPU
        for (py::ssize_t i = 0; i < P; ++i) {
          py::ssize_t j0 = i + 1;
          while (j0 < P) {
            cand.clear();
            const int di = dev[i], gi = DG[di];
            for (py::ssize_t j = j0; j < P; ++j) {
              const int dj = dev[j], gj = DG[dj];
              if (gi == gj || U[i] != U[j]) continue;
              if (hfree[di] + H[i] - H[j] < -1e-6 || hfree[dj] + H[j] - H[i] < -1e-6) continue;
              if (phase_b && saturated(ge[gi]) && saturated(ge[gj])) continue;
              // same workload and length: a no-op for the makespans (phase A)
              if (!phase_b && wid.data()[i] == wid.data()[j] && iters.data()[i] == iters.data()[j]) continue;
              cand.push_back({(int)i, (int)j, gi, gj});
            }
            if (cand.empty()) break;
            evaluate(true);
            py::ssize_t next = P;
            for (size_t c = 0; c < cand.size(); ++c) {
              const int j = cand[c].b, gj = cand[c].gb, dj = dev[j];
              if (!accept(gi, gj, ge[gi], ge[gj], res[c].ea, res[c].eb)) continue;
              *std::find(mem[gi].begin(), mem[gi].end(), (int)i) = j;
              *std::find(mem[gj].begin(), mem[gj].end(), j) = (int)i;
              Ksum[gi] += hm(j) - hm((int)i);
              Ksum[gj] += hm((int)i) - hm(j);
              dev[i] = dj;
              dev[j] = di;
              hfree[di] += H[i] - H[j];
              hfree[dj] += H[j] - H[i];
              ge[gi] = res[c].ea;
              ge[gj] = res[c].eb;
              improved = true;
              next = j + 1;
              break;
            }
            j0 = next;
          }
        }
        if (!improved) break;
      }
      if (std::getenv("GPUSCHED_PLAN_DEBUG")) {
        const size_t sims = memo[phase_b ? 1 : 0].size();
        std::fprintf(stderr, "[plan_corun] phase %d evals %ld sets %zu plain sims %ld pipe sims %ld threads %d\n",
                     phase_b ? 1 : 0, n_evals.load(), sims, n_plain.load(), n_pipe.load(), T);
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
      phase_b = true;
      use_pipe = pipe;
      eval_all();
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

// One GPU's pipeline as arrays (chain_times / plan_slots): m context members -- pods already
// placed on the GPU, measured ones pinned to their interval, the rest chained per slot -- and
// n new pods to place on S CU slots.
py::tuple chain_times(I32 wid, F64 iters, F64 start, I32 prev, F64 alone, F64 cmat, py::object pin_end) {
  int W;
  check_model(alone, cmat, W);
  const py::ssize_t k = wid.shape(0);
  if (iters.shape(0) != k || start.shape(0) != k || prev.shape(0) != k)
    throw std::runtime_error("chain_times: array shapes differ");
  if (k > kMaxK) throw std::runtime_error("chain_times: more than 64 members");
  check_wids(wid.data(), k, W, "chain_times");
  for (py::ssize_t i = 0; i < k; ++i)
    if (prev.data()[i] >= (int32_t)i) throw std::runtime_error("chain_times: prev must point to an earlier member");
  F64 pin_a;
  const double* pp = nullptr;
  if (!pin_end.is_none()) {
    pin_a = pin_end.cast<F64>();
    if (pin_a.shape(0) != k) throw std::runtime_error("chain_times: pin_end must have k entries");
    pp = pin_a.data();
  }
  py::array_t<double> st(k), fin(k);
  sim_chain((int)k, wid.data(), iters.data(), start.data(), prev.data(), alone.data(), cmat.data(), W,
            st.mutable_data(), fin.mutable_data(), pp);
  return py::make_tuple(st, fin);
}

// Slot assignment of n new pods on one GPU whose CU slots already run a pipeline (context: m
// members as in chain_times; slot_tail[s] = the context member last on slot s, -1 = the slot is
// free from slot_free[s]).  New pod j on slot s starts when slot_tail[s] finishes, not before its
// release n_rel[j].  Every injective assignment (n <= S; enumerated up to max_enum, else a
// pairwise-swap local search from the longest-first / earliest-free-slot assignment) is
// simulated as a whole pipeline:
//   spread = max - min over slots of the predicted end of the slot's last pod -- a slot that
//            runs ahead of the others idles once the launch-ahead window is exhausted, so a
//            bounded spread is the throughput side;
//   expected = members (new pods and unmeasured context pods with an SLO) expected to meet
//            their SLO under lognormal model error sigma (sigma 0: hard counts).
// The choice: the most expected SLOs among assignments within spread_tol ms of the least
// spread any assignment reaches; ties -> the smaller spread.
// Returns (slot per new pod, start[m+n], fin[m+n], expected, spread, least spread).
// ph_off [S+1] / ph_wid / ph_iters (optional): per candidate slot, "phantom" pods chained after
// its last pod -- the slot's future.  Pods placed later co-run with the new pods' tails; without
// them the pipeline looks emptier than it will be and every prediction is optimistic (measured
// on MI355X bench traces: -24 % mean log error, ~0 with three phantoms per slot repeating the
// slot's recent workloads).  Phantoms press on the others; they are never counted.
// plan_slots' inputs, validated and owned (so a batch can run on another thread without the
// interpreter), and its result
struct SlotJob {
  int W = 0, m = 0, S = 0, n = 0;
  std::vector<int32_t> c_wid, c_prev, slot_tail, n_wid, PW;
  std::vector<double> c_iters, c_start, c_pin, c_slo, slot_free, n_iters, n_slo, n_rel, alone, cmat, PI;
  std::vector<int64_t> PO;
  double sigma = 0.05, spread_tol = 0.0;
  int max_enum = 720;
  bool fast_forward = true;
};
struct SlotOut {
  std::vector<int32_t> best;
  std::vector<double> st, fin;
  double best_e = 0.0, best_sp = 0.0, min_sp = 0.0;
};

SlotJob make_slot_job(I32 c_wid, F64 c_iters, F64 c_start, I32 c_prev, F64 c_pin, F64 c_slo, I32 slot_tail,
                      F64 slot_free, I32 n_wid, F64 n_iters, F64 n_slo, F64 n_rel, F64 alone, F64 cmat, double sigma,
                      double spread_tol, int max_enum, py::object ph_off_o, py::object ph_wid_o, py::object ph_it_o,
                      bool fast_forward) {
  int W;
  check_model(alone, cmat, W);
  const int m = (int)c_wid.shape(0), S = (int)slot_tail.shape(0), n = (int)n_wid.shape(0);
  if (c_iters.shape(0) != m || c_start.shape(0) != m || c_prev.shape(0) != m || c_pin.shape(0) != m ||
      c_slo.shape(0) != m)
    throw std::runtime_error("plan_slots: context shapes differ");
  if (slot_free.shape(0) != S || n_iters.shape(0) != n || n_slo.shape(0) != n || n_rel.shape(0) != n)
    throw std::runtime_error("plan_slots: slot / new-pod shapes differ");
  if (n > S) throw std::runtime_error("plan_slots: more new pods than slots");
  if (S > 64) throw std::runtime_error("plan_slots: more than 64 slots");
  if (m + n > kMaxK) throw std::runtime_error("plan_slots: more than 64 members");
  check_wids(c_wid.data(), m, W, "plan_slots context");
  check_wids(n_wid.data(), n, W, "plan_slots new pods");
  for (int i = 0; i < m; ++i)
    if (c_prev.data()[i] >= i) throw std::runtime_error("plan_slots: prev must point to an earlier member");
  for (int s = 0; s < S; ++s)
    if (slot_tail.data()[s] < -1 || slot_tail.data()[s] >= m) throw std::runtime_error("plan_slots: bad slot tail");
  SlotJob J;
  J.W = W, J.m = m, J.S = S, J.n = n;
  J.PO.assign(S + 1, 0);
  if (!ph_off_o.is_none()) {
    I64 po = ph_off_o.cast<I64>();
    I32 pw = ph_wid_o.cast<I32>();
    F64 pi = ph_it_o.cast<F64>();
    if (po.shape(0) != S + 1 || po.data()[0] != 0 || po.data()[S] != pw.shape(0) || pi.shape(0) != pw.shape(0))
      throw std::runtime_error("plan_slots: phantom arrays");
    for (int q = 0; q < S; ++q)
      if (po.data()[q + 1] < po.data()[q]) throw std::runtime_error("plan_slots: phantom offsets");
    check_wids(pw.data(), pw.shape(0), W, "plan_slots phantoms");
    J.PO.assign(po.data(), po.data() + S + 1);
    J.PW.assign(pw.data(), pw.data() + pw.shape(0));
    J.PI.assign(pi.data(), pi.data() + pi.shape(0));
  }
  if (m + n + (int)J.PW.size() > kMaxK) throw std::runtime_error("plan_slots: more than 64 members with phantoms");
  auto cp32 = [](const I32& a) { return std::vector<int32_t>(a.data(), a.data() + a.size()); };
  auto cp64 = [](const F64& a) { return std::vector<double>(a.data(), a.data() + a.size()); };
  J.c_wid = cp32(c_wid), J.c_prev = cp32(c_prev), J.slot_tail = cp32(slot_tail), J.n_wid = cp32(n_wid);
  J.c_iters = cp64(c_iters), J.c_start = cp64(c_start), J.c_pin = cp64(c_pin), J.c_slo = cp64(c_slo);
  J.slot_free = cp64(slot_free), J.n_iters = cp64(n_iters), J.n_slo = cp64(n_slo), J.n_rel = cp64(n_rel);
  J.alone = cp64(alone), J.cmat = cp64(cmat);
  J.sigma = sigma, J.spread_tol = spread_tol, J.max_enum = max_enum, J.fast_forward = fast_forward;
  return J;
}

// The slot plan itself (no Python objects: runs without the interpreter lock)
SlotOut run_slot_job(const SlotJob& J) {
  const int W = J.W, m = J.m, S = J.S, n = J.n;
  const std::vector<int64_t>& PO = J.PO;
  const std::vector<int32_t>& PW = J.PW;
  const std::vector<double>& PI = J.PI;
  const double sigma = J.sigma, spread_tol = J.spread_tol;
  const int max_enum = J.max_enum;
  const bool fast_forward = J.fast_forward;
  const int nph = (int)PW.size();
  if (m + n + nph > kMaxK) throw std::runtime_error("plan_slots: more than 64 members with phantoms");
  const int k = m + n + nph;
  int32_t w[kMaxK], pv[kMaxK];
  double it[kMaxK], s0[kMaxK], pe[kMaxK], sl[kMaxK];
  for (int i = 0; i < m; ++i) {
    w[i] = J.c_wid[i];
    it[i] = J.c_iters[i];
    s0[i] = J.c_start[i];
    pv[i] = J.c_prev[i];
    pe[i] = J.c_pin[i];
    sl[i] = J.c_slo[i];
  }
  for (int j = 0; j < n; ++j) {
    w[m + j] = J.n_wid[j];
    it[m + j] = J.n_iters[j];
    sl[m + j] = J.n_slo[j];
    pe[m + j] = 0.0;
  }
  for (int q = 0; q < nph; ++q) {
    w[m + n + q] = PW[q];
    it[m + n + q] = PI[q];
    sl[m + n + q] = 0.0;
    pe[m + n + q] = 0.0;
    s0[m + n + q] = -kBig;
  }
  const int32_t* T = J.slot_tail.data();
  const double* F = J.slot_free.data();
  const double* R = J.n_rel.data();
  const double* A = J.alone.data();
  const double* Cm = J.cmat.data();
  struct Res {
    double expected = -1.0, spread = kBig;
  };
  double st[kMaxK], fin[kMaxK];
  auto eval = [&](const int* slot, double* st_o, double* fin_o) {
    int last[64];
    for (int q = 0; q < S && q < 64; ++q) last[q] = T[q];
    for (int j = 0; j < n; ++j) {
      const int s = slot[j], t = T[s];
      pv[m + j] = t;
      s0[m + j] = t >= 0 ? R[j] : std::max(F[s], R[j]);
      if (s < 64) last[s] = m + j;
    }
    for (int q = 0; q < S && q < 64; ++q) {
      int p = last[q];
      for (int64_t x = PO[q]; x < PO[q + 1]; ++x) {
        const int i = m + n + (int)x;
        if (p >= 0) {
          pv[i] = p;
          s0[i] = -kBig;
        } else {
          pv[i] = -1;
          s0[i] = F[q];
        }
        p = i;
      }
    }
    sim_chain(k, w, it, s0, pv, A, Cm, W, st_o, fin_o, pe);
    Res r;
    r.expected = 0.0;
    for (int i = 0; i < k; ++i) {
      const bool pinned = i < m && pv[i] < 0 && pe[i] > s0[i];
      if (pinned || sl[i] <= 0 || it[i] <= 0) continue;
      const double d = fin_o[i] - st_o[i];
      r.expected += (fin_o[i] >= kBig) ? 0.0 : p_meet(it[i] / std::max(d, 1e-12) * 1e3, sl[i], sigma);
    }
    double lo = kBig, hi = -kBig;
    for (int s = 0; s < S; ++s) {
      double e = F[s];
      if (T[s] >= 0) e = fin_o[T[s]];
      for (int j = 0; j < n; ++j)
        if (slot[j] == s) e = fin_o[m + j];
      lo = std::min(lo, e);
      hi = std::max(hi, e);
    }
    r.spread = hi - lo;
    return r;
  };
  // Fast-forward of the shared context prefix: every new pod and phantom starts at or after
  // t_cut = min over slots of (its tail's finish, or its free time when it has no tail), so up
  // to t_cut every assignment simulates the context alone -- the same simulation.  It runs once;
  // members done by t_cut leave the per-assignment simulations (their SLO verdicts are a
  // constant), running ones resume at t_cut with their remaining work (scored against their real
  // start), chains behind dropped members start at their known time.  8-GPU bench epochs: ~19 of
  // 24 context members are done by t_cut, so each assignment simulates ~17 members instead of ~36.
  // Results equal the full simulations up to floating-point rounding (tests/test_corun.py).
  int mr = 0;
  int32_t rw[kMaxK], rpv[kMaxK], rmap[kMaxK], rT[64];
  double rit[kMaxK], rs0[kMaxK], rpe[kMaxK], rsl[kMaxK], rsc_it[kMaxK], rsst[kMaxK], rTfin[64];
  double ff_const = 0.0;           // SLO verdicts of the dropped (finished) context members
  bool ff = fast_forward && m > 0 && S <= 64;
  if (ff) {
    double c_st[kMaxK], c_fin[kMaxK], c_rem[kMaxK];
    sim_chain(m, w, it, s0, pv, A, Cm, W, c_st, c_fin, pe);
    double tcut = kBig;
    for (int q = 0; q < S; ++q) tcut = std::min(tcut, T[q] >= 0 ? c_fin[T[q]] : F[q]);
    if (tcut >= kBig) {
      ff = false;
    } else {
      sim_chain(m, w, it, s0, pv, A, Cm, W, c_st, c_fin, pe, tcut, c_rem);
      for (int i = 0; i < m; ++i) {
        const bool pin = pv[i] < 0 && pe[i] > s0[i];
        const bool svc = it[i] <= 0;
        const bool started = c_st[i] < kBig && c_st[i] <= tcut;
        const bool done = pin ? pe[i] <= tcut : (!svc && started && c_rem[i] <= 0.0);
        if (done) {
          rmap[i] = -1;
          if (!pin && sl[i] > 0 && it[i] > 0)
            ff_const += p_meet(it[i] / std::max(c_fin[i] - c_st[i], 1e-12) * 1e3, sl[i], sigma);
          continue;
        }
        const int r = mr++;
        rmap[i] = r;
        rw[r] = w[i];
        rsl[r] = sl[i];
        rsc_it[r] = it[i];
        rpe[r] = pin ? pe[i] : 0.0;     // (a chained member's pin value never pinned it)
        rsst[r] = std::numeric_limits<double>::quiet_NaN();     // NaN: score from the simulated start
        if (started) {
          rs0[r] = tcut;
          rpv[r] = -1;
          rit[r] = (pin || svc) ? it[i] : std::max(c_rem[i], 1e-12) / std::max(A[w[i]], 1e-300);
          if (!pin) rsst[r] = c_st[i];
        } else if (pv[i] >= 0 && rmap[pv[i]] < 0) {
          rs0[r] = std::max(c_fin[pv[i]], s0[i]);                 // its predecessor is done
          rpv[r] = -1;
          rit[r] = it[i];
        } else {
          rs0[r] = s0[i];
          rpv[r] = pv[i] >= 0 ? rmap[pv[i]] : -1;
          rit[r] = it[i];
        }
      }
      for (int q = 0; q < S; ++q) {
        rT[q] = T[q] >= 0 ? rmap[T[q]] : -1;
        rTfin[q] = (T[q] >= 0 && rmap[T[q]] < 0) ? c_fin[T[q]] : -kBig;   // a dropped tail's finish
      }
      for (int j = 0; j < n + nph; ++j) {
        rw[mr + j] = w[m + j];
        rit[mr + j] = it[m + j];
        rsc_it[mr + j] = it[m + j];
        rsl[mr + j] = sl[m + j];
        rpe[mr + j] = 0.0;
        rsst[mr + j] = std::numeric_limits<double>::quiet_NaN();
      }
    }
  }
  const int kr = mr + n + nph;
  double rst[kMaxK], rfin[kMaxK];
  auto eval_ff = [&](const int* slot) {
    int last[64];
    for (int q = 0; q < S; ++q) last[q] = rT[q];
    bool has[64];
    for (int q = 0; q < S; ++q) has[q] = false;
    for (int j = 0; j < n; ++j) {
      const int s = slot[j], t = rT[s];
      rpv[mr + j] = t;
      if (t >= 0) rs0[mr + j] = R[j];
      else rs0[mr + j] = rTfin[s] > -kBig ? std::max(rTfin[s], R[j]) : std::max(F[s], R[j]);
      last[s] = mr + j;
      has[s] = true;
    }
    for (int q = 0; q < S; ++q) {
      int p = last[q];
      for (int64_t x = PO[q]; x < PO[q + 1]; ++x) {
        const int i = mr + n + (int)x;
        if (p >= 0) {
          rpv[i] = p;
          rs0[i] = -kBig;
        } else {
          rpv[i] = -1;
          rs0[i] = (!has[q] && rTfin[q] > -kBig) ? rTfin[q] : F[q];
        }
        p = i;
      }
    }
    sim_chain(kr, rw, rit, rs0, rpv, A, Cm, W, rst, rfin, rpe);
    Res r;
    r.expected = ff_const;
    for (int i = 0; i < kr; ++i) {
      const bool pinned = i < mr && rpv[i] < 0 && rpe[i] > rs0[i];
      if (pinned || rsl[i] <= 0 || rsc_it[i] <= 0) continue;
      const double st0 = std::isnan(rsst[i]) ? rst[i] : rsst[i];
      const double d = rfin[i] - st0;
      r.expected += (rfin[i] >= kBig) ? 0.0 : p_meet(rsc_it[i] / std::max(d, 1e-12) * 1e3, rsl[i], sigma);
    }
    double lo = kBig, hi = -kBig;
    for (int s = 0; s < S; ++s) {
      double e = F[s];
      if (rT[s] >= 0) e = rfin[rT[s]];
      else if (rTfin[s] > -kBig) e = rTfin[s];
      for (int j = 0; j < n; ++j)
        if (slot[j] == s) e = rfin[mr + j];
      lo = std::min(lo, e);
      hi = std::max(hi, e);
    }
    r.spread = hi - lo;
    return r;
  };
  auto eval_any = [&](const int* slot) { return ff ? eval_ff(slot) : eval(slot, st, fin); };
  std::vector<int> best(n), cur(n);
  double best_e = -1.0, best_sp = kBig, min_sp = kBig;
  {
    // number of injective assignments S! / (S - n)!
    double count = 1.0;
    for (int j = 0; j < n; ++j) count *= (double)(S - j);
    if (n == 0) {
      best_e = 0.0;
    } else if (count <= (double)std::max(max_enum, 1)) {
      std::vector<std::pair<double, double>> all;
      std::vector<std::vector<int>> asg;
      std::vector<bool> used(S, false);
      // depth-first enumeration in lexicographic order.  Identical new pods (workload, length,
      // SLO, release) are interchangeable: of the assignments that only permute them, the
      // lexicographically first -- their slots increasing -- is the one a full enumeration meets
      // first, so only it is simulated (a Zipf burst often repeats a workload on one GPU)
      std::vector<int> twin(n, -1);
      for (int a = 0; a < n; ++a)
        for (int b = a - 1; b >= 0; --b)
          if (w[m + a] == w[m + b] && it[m + a] == it[m + b] && sl[m + a] == sl[m + b] && R[a] == R[b]) {
            twin[a] = b;
            break;
          }
      std::vector<int> pos(n, -1);
      int j = 0;
      while (j >= 0) {
        if (j == n) {
          const Res r = eval_any(cur.data());
          all.emplace_back(r.expected, r.spread);
          asg.push_back(cur);
          --j;
          if (j >= 0) used[cur[j]] = false;
          continue;
        }
        int s = pos[j] + 1;
        if (pos[j] < 0 && twin[j] >= 0) s = cur[twin[j]] + 1;
        while (s < S && used[s]) ++s;
        if (s >= S) {
          pos[j] = -1;
          --j;
          if (j >= 0) used[cur[j]] = false;
          continue;
        }
        pos[j] = s;
        cur[j] = s;
        used[s] = true;
        ++j;
      }
      for (const auto& x : all) min_sp = std::min(min_sp, x.second);
      for (size_t a = 0; a < all.size(); ++a) {
        const double e = all[a].first, sp = all[a].second;
        if (sp > min_sp + spread_tol + 1e-9) continue;
        if (e > best_e + 1e-9 || (e > best_e - 1e-9 && sp < best_sp - 1e-9)) {
          best_e = e;
          best_sp = sp;
          best = asg[a];
        }
      }
    } else {
      // longest work first onto the slot that frees first (from the context alone), then swaps
      double cst[kMaxK], cfin[kMaxK];
      if (m > 0) sim_chain(m, w, it, s0, pv, A, Cm, W, cst, cfin, pe);
      std::vector<double> free_at(S);
      for (int s = 0; s < S; ++s) free_at[s] = T[s] >= 0 ? cfin[T[s]] : F[s];
      std::vector<int> order(n);
      for (int q = 0; q < n; ++q) order[q] = q;
      std::sort(order.begin(), order.end(),
                [&](int a, int b) { return A[w[m + a]] * it[m + a] > A[w[m + b]] * it[m + b]; });
      std::vector<bool> used(S, false);
      for (int q : order) {
        int bs = -1;
        for (int s = 0; s < S; ++s)
          if (!used[s] && (bs < 0 || free_at[s] < free_at[bs])) bs = s;
        used[bs] = true;
        cur[q] = bs;
      }
      Res r = eval_any(cur.data());
      min_sp = r.spread;
      const double cap = r.spread + spread_tol;
      best = cur;
      best_e = r.expected;
      best_sp = r.spread;
      for (int sweep = 0; sweep < 8; ++sweep) {
        bool improved = false;
        for (int a = 0; a < n; ++a) {
          // swap with another new pod, or move to an unused slot
          for (int b = 0; b < n + S; ++b) {
            std::vector<int> cand = best;
            if (b < n) {
              if (b <= a) continue;
              std::swap(cand[a], cand[b]);
            } else {
              const int s = b - n;
              if (std::find(cand.begin(), cand.end(), s) != cand.end()) continue;
              cand[a] = s;
            }
            const Res x = eval_any(cand.data());
            min_sp = std::min(min_sp, x.spread);
            if (x.spread > cap + 1e-9) continue;
            if (x.expected > best_e + 1e-9 || (x.expected > best_e - 1e-9 && x.spread < best_sp - 1e-9)) {
              best = cand;
              best_e = x.expected;
              best_sp = x.spread;
              improved = true;
            }
          }
        }
        if (!improved) break;
      }
    }
  }
  SlotOut o;
  o.best.assign(best.begin(), best.end());
  o.st.assign(k, 0.0);
  o.fin.assign(k, 0.0);
  {
    const Res r = eval(best.data(), o.st.data(), o.fin.data());
    if (n == 0) best_sp = min_sp = r.spread;
  }
  o.best_e = best_e, o.best_sp = best_sp, o.min_sp = min_sp;
  return o;
}

py::tuple slot_out_tuple(const SlotOut& o) {
  py::array_t<int32_t> out((py::ssize_t)o.best.size());
  py::array_t<double> st_a((py::ssize_t)o.st.size()), fin_a((py::ssize_t)o.fin.size());
  std::copy(o.best.begin(), o.best.end(), out.mutable_data());
  std::copy(o.st.begin(), o.st.end(), st_a.mutable_data());
  std::copy(o.fin.begin(), o.fin.end(), fin_a.mutable_data());
  return py::make_tuple(out, st_a, fin_a, o.best_e, o.best_sp, o.min_sp);
}

py::tuple plan_slots(I32 c_wid, F64 c_iters, F64 c_start, I32 c_prev, F64 c_pin, F64 c_slo, I32 slot_tail,
                     F64 slot_free, I32 n_wid, F64 n_iters, F64 n_slo, F64 n_rel, F64 alone, F64 cmat, double sigma,
                     double spread_tol, int max_enum, py::object ph_off_o, py::object ph_wid_o, py::object ph_it_o,
                     bool fast_forward) {
  const SlotJob J = make_slot_job(c_wid, c_iters, c_start, c_prev, c_pin, c_slo, slot_tail, slot_free, n_wid, n_iters,
                                  n_slo, n_rel, alone, cmat, sigma, spread_tol, max_enum, ph_off_o, ph_wid_o, ph_it_o,
                                  fast_forward);
  SlotOut o;
  {
    py::gil_scoped_release nogil;
    o = run_slot_job(J);
  }
  return slot_out_tuple(o);
}

// Several GPUs' slot plans on one background thread (plan_slots_async): the burst planner needs
// the first pod's slot at once and the others only when their pods reach Reserve, so the native
// work overlaps the scheduling cycles of the burst's other pods.  result(i) waits (without the
// interpreter lock) for job i; jobs run in order.
class SlotBatch {
 public:
  explicit SlotBatch(std::vector<SlotJob> jobs)
      : jobs_(std::move(jobs)), outs_(jobs_.size()), errs_(jobs_.size()), done_(jobs_.size(), 0) {
    th_ = std::thread([this] {
      for (size_t i = 0; i < jobs_.size(); ++i) {
        try {
          outs_[i] = run_slot_job(jobs_[i]);
        } catch (const std::exception& e) {
          errs_[i] = e.what();
          if (errs_[i].empty()) errs_[i] = "plan_slots failed";
        }
        {
          std::lock_guard<std::mutex> lk(mu_);
          done_[i] = 1;
        }
        cv_.notify_all();
      }
    });
  }
  ~SlotBatch() { join(); }
  void join() {
    if (th_.joinable()) th_.join();
  }
  size_t size() const { return jobs_.size(); }
  py::tuple result(int i) {
    if (i < 0 || (size_t)i >= jobs_.size()) throw std::out_of_range("SlotBatch: job index");
    {
      py::gil_scoped_release nogil;
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return done_[(size_t)i] != 0; });
    }
    if (!errs_[(size_t)i].empty()) throw std::runtime_error(errs_[(size_t)i]);
    return slot_out_tuple(outs_[(size_t)i]);
  }

 private:
  std::vector<SlotJob> jobs_;
  std::vector<SlotOut> outs_;
  std::vector<std::string> errs_;
  std::vector<char> done_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
};

std::unique_ptr<SlotBatch> plan_slots_async(py::list jobs) {
  std::vector<SlotJob> js;
  js.reserve(jobs.size());
  for (py::handle h : jobs) {
    py::tuple a = h.cast<py::tuple>();
    if (a.size() != 21) throw std::runtime_error("plan_slots_async: each job is plan_slots' 21 arguments");
    js.push_back(make_slot_job(a[0].cast<I32>(), a[1].cast<F64>(), a[2].cast<F64>(), a[3].cast<I32>(),
                               a[4].cast<F64>(), a[5].cast<F64>(), a[6].cast<I32>(), a[7].cast<F64>(),
                               a[8].cast<I32>(), a[9].cast<F64>(), a[10].cast<F64>(), a[11].cast<F64>(),
                               a[12].cast<F64>(), a[13].cast<F64>(), a[14].cast<double>(), a[15].cast<double>(),
                               a[16].cast<int>(), py::reinterpret_borrow<py::object>(a[17]),
                               py::reinterpret_borrow<py::object>(a[18]), py::reinterpret_borrow<py::object>(a[19]),
                               a[20].cast<bool>()));
  }
  return std::make_unique<SlotBatch>(std::move(js));
}

}  // namespace

void register_corun(py::module_& m) {
  m.def("chain_times", &chain_times, py::arg("wids"), py::arg("iters"), py::arg("starts"), py::arg("prev"),
        py::arg("alone_ms"), py::arg("cmat"), py::arg("pin_end") = py::none());
  m.def("plan_slots", &plan_slots, py::arg("c_wid"), py::arg("c_iters"), py::arg("c_start"), py::arg("c_prev"),
        py::arg("c_pin"), py::arg("c_slo"), py::arg("slot_tail"), py::arg("slot_free"), py::arg("n_wid"),
        py::arg("n_iters"), py::arg("n_slo"), py::arg("n_release"), py::arg("alone_ms"), py::arg("cmat"),
        py::arg("sigma") = 0.05, py::arg("spread_tol") = 0.0, py::arg("max_enum") = 720,
        py::arg("ph_off") = py::none(), py::arg("ph_wid") = py::none(), py::arg("ph_iters") = py::none(),
        py::arg("fast_forward") = true);
  py::class_<SlotBatch>(m, "SlotBatch")
      .def("result", &SlotBatch::result, py::arg("i"))
      .def("join", &SlotBatch::join, py::call_guard<py::gil_scoped_release>())
      .def("__len__", &SlotBatch::size);
  m.def("plan_slots_async", &plan_slots_async, py::arg("jobs"),
        "Start several plan_slots jobs (tuples of its 21 positional arguments) on a background thread");
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
        py::arg("mode") = 0, py::arg("sigma") = 0.0, py::arg("base") = py::none(), py::arg("pipe") = py::none(),
        py::arg("hbm") = py::none(), py::arg("dev_hbm") = py::none(), py::arg("sweeps_b") = -1,
        py::arg("speed") = py::none());
}
