// amd-smi telemetry / topology / partition layer (host C++, links libamd_smi).
//
// Replaces the reference's NVIDIA paths:
//  * `nvidia-smi -L` UUID enumeration (pkg/profiler/parse_smi_uuids.py:6-18)
//      -> amdsmi_get_processor_handles + amdsmi_get_gpu_device_uuid (no CLI parsing);
//  * the unused `nvidia-smi --query-gpu=power.draw,utilization.gpu,temperature.gpu`
//    1 s poller (pkg/profiler/parse_smi_metrics.py:23-42) and the DCGM series the plugin
//    reads through Prometheus (pkg/prom/fetch_prom_metrics/prom_metrics.go:63-70)
//      -> a sampler thread: gfx/umc activity, VRAM used/total, socket power, hotspot
//         temperature, per-link xGMI read/write accumulators turned into byte rates;
//  * MIG layouts via the NVIDIA MIG manager (gpu_plugins.go:402-413)
//      -> amdsmi compute partition get/set (SPX/DPX/QPX/CPX) + memory partition get;
//  * new: xGMI link matrix (type, hops, weight) + NUMA node for the topology Filter, and
//    the per-process list (PID, VRAM, CU occupancy) for per-pod attribution;
//  * new: read-only partition capability probe (accelerator partition profiles = the
//    compute modes this GPU supports, and the NPS memory modes each allows) and NPS memory
//    partition set -- the agent applies only what the probe lists;
//  * new: amd-smi -> HIP enumeration map (hip_id / hsa_id / render node) and a light,
//    fast activity sampler (gfx/umc activity, VRAM, power of selected GPUs) that the
//    benchmark runs on a C++ thread across its timed region.
#include <amd_smi/amdsmi.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sampler.h"

namespace py = pybind11;

namespace {

struct Activity {                                   // light sample (benchmark sampler)
  double ts = 0;
  int index = 0;
  double gfx = -1, umc = -1, vram_used_mb = -1, power_w = -1;
};

const char* const kNps[] = {"", "NPS1", "NPS2", "", "NPS4", "", "", "", "NPS8"};

std::vector<std::string> nps_list(amdsmi_nps_caps_t c) {
  std::vector<std::string> out;
  if (c.nps_flags.nps1_cap) out.push_back("NPS1");
  if (c.nps_flags.nps2_cap) out.push_back("NPS2");
  if (c.nps_flags.nps4_cap) out.push_back("NPS4");
  if (c.nps_flags.nps8_cap) out.push_back("NPS8");
  return out;
}

const char* accel_name(amdsmi_accelerator_partition_type_t t) {
  switch (t) {
    case AMDSMI_ACCELERATOR_PARTITION_SPX: return "SPX";
    case AMDSMI_ACCELERATOR_PARTITION_DPX: return "DPX";
    case AMDSMI_ACCELERATOR_PARTITION_TPX: return "TPX";
    case AMDSMI_ACCELERATOR_PARTITION_QPX: return "QPX";
    case AMDSMI_ACCELERATOR_PARTITION_CPX: return "CPX";
    default: return "";
  }
}

struct Sample {
  double ts = 0;
  int index = 0;
  double gfx = -1, umc = -1, mm = -1;
  double vram_used_mb = -1, vram_total_mb = -1;
  double power_w = -1, temp_c = -1;
  double xgmi_read_kb = 0, xgmi_write_kb = 0;       // accumulators (sum over links)
  double xgmi_read_bps = 0, xgmi_write_bps = 0;     // rates since previous sample
  // accumulated ECC error counts (-1 = not reported by this device/driver); the node
  // agent's health monitor marks a GPU unhealthy when the uncorrectable count grows
  double ecc_correctable = -1, ecc_uncorrectable = -1, ecc_deferred = -1;
  bool responsive = false;                          // the activity/VRAM queries answered
};

const char* status_str(amdsmi_status_t s) {
  const char* msg = nullptr;
  if (amdsmi_status_code_to_string(s, &msg) == AMDSMI_STATUS_SUCCESS && msg) return msg;
  return "amdsmi error";
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

class Smi {
 public:
  Smi() = default;
  ~Smi() { shutdown(); }

  bool init() {
    std::lock_guard<std::mutex> g(mu_);
    if (inited_) return true;
    amdsmi_status_t s = amdsmi_init(AMDSMI_INIT_AMD_GPUS);
    if (s != AMDSMI_STATUS_SUCCESS) {
      err_ = status_str(s);
      return false;
    }
    inited_ = true;
    uint32_t ns = 0;
    if (amdsmi_get_socket_handles(&ns, nullptr) != AMDSMI_STATUS_SUCCESS) return true;
    std::vector<amdsmi_socket_handle> socks(ns);
    amdsmi_get_socket_handles(&ns, socks.data());
    for (auto sk : socks) {
      uint32_t np = 0;
      if (amdsmi_get_processor_handles(sk, &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
      std::vector<amdsmi_processor_handle> ps(np);
      amdsmi_get_processor_handles(sk, &np, ps.data());
      for (auto p : ps) {
        processor_type_t t;
        if (amdsmi_get_processor_type(p, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_PROCESSOR_TYPE_AMD_GPU)
          gpus_.push_back(p);
      }
    }
    prev_.assign(gpus_.size(), Sample());
    return true;
  }

  std::string error() const { return err_; }
  int count() const { return static_cast<int>(gpus_.size()); }

  py::list devices() {
    py::list out;
    for (size_t i = 0; i < gpus_.size(); ++i) {
      auto h = gpus_[i];
      py::dict d;
      d["index"] = static_cast<int>(i);
      char uuid[AMDSMI_GPU_UUID_SIZE] = {0};
      unsigned int ul = sizeof(uuid);
      if (amdsmi_get_gpu_device_uuid(h, &ul, uuid) == AMDSMI_STATUS_SUCCESS) d["uuid"] = std::string(uuid);
      amdsmi_bdf_t bdf;
      if (amdsmi_get_gpu_device_bdf(h, &bdf) == AMDSMI_STATUS_SUCCESS) {
        char b[32];
        std::snprintf(b, sizeof(b), "%04x:%02x:%02x.%x", (unsigned)bdf.domain_number, (unsigned)bdf.bus_number,
                      (unsigned)bdf.device_number, (unsigned)bdf.function_number);
        d["bdf"] = std::string(b);
      }
      uint32_t numa = 0;
      if (amdsmi_topo_get_numa_node_number(h, &numa) == AMDSMI_STATUS_SUCCESS) d["numa"] = numa;
      char part[64] = {0};
      if (amdsmi_get_gpu_compute_partition(h, part, sizeof(part)) == AMDSMI_STATUS_SUCCESS)
        d["compute_partition"] = std::string(part);
      char mpart[64] = {0};
      if (amdsmi_get_gpu_memory_partition(h, mpart, sizeof(mpart)) == AMDSMI_STATUS_SUCCESS)
        d["memory_partition"] = std::string(mpart);
      amdsmi_asic_info_t asic;
      if (amdsmi_get_gpu_asic_info(h, &asic) == AMDSMI_STATUS_SUCCESS) {
        d["market_name"] = std::string(asic.market_name);
        d["num_cu"] = asic.num_of_compute_units;
      }
      amdsmi_vram_usage_t v;
      if (amdsmi_get_gpu_vram_usage(h, &v) == AMDSMI_STATUS_SUCCESS) d["vram_total_mb"] = v.vram_total;
      out.append(d);
    }
    return out;
  }

  Sample sample_one(size_t i, double ts) {
    auto h = gpus_[i];
    Sample s;
    s.ts = ts;
    s.index = static_cast<int>(i);
    amdsmi_engine_usage_t u;
    if (amdsmi_get_gpu_activity(h, &u) == AMDSMI_STATUS_SUCCESS) {
      s.gfx = u.gfx_activity;
      s.umc = u.umc_activity;
      s.mm = u.mm_activity;
      s.responsive = true;
    }
    amdsmi_vram_usage_t v;
    if (amdsmi_get_gpu_vram_usage(h, &v) == AMDSMI_STATUS_SUCCESS) {
      s.vram_used_mb = v.vram_used;
      s.vram_total_mb = v.vram_total;
      s.responsive = true;
    }
    amdsmi_error_count_t ec;
    if (amdsmi_get_gpu_total_ecc_count(h, &ec) == AMDSMI_STATUS_SUCCESS) {
      s.ecc_correctable = static_cast<double>(ec.correctable_count);
      s.ecc_uncorrectable = static_cast<double>(ec.uncorrectable_count);
      s.ecc_deferred = static_cast<double>(ec.deferred_count);
    }
    amdsmi_power_info_t p;
    if (amdsmi_get_power_info(h, &p) == AMDSMI_STATUS_SUCCESS)
      s.power_w = (p.current_socket_power != UINT32_MAX) ? p.current_socket_power : (double)p.average_socket_power;
    int64_t t = 0;
    if (amdsmi_get_temp_metric(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS)
      s.temp_c = static_cast<double>(t);
    amdsmi_gpu_metrics_t m;
    if (amdsmi_get_gpu_metrics_info(h, &m) == AMDSMI_STATUS_SUCCESS) {
      for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
        if (m.xgmi_read_data_acc[l] != UINT64_MAX) s.xgmi_read_kb += (double)m.xgmi_read_data_acc[l];
        if (m.xgmi_write_data_acc[l] != UINT64_MAX) s.xgmi_write_kb += (double)m.xgmi_write_data_acc[l];
      }
      if (s.gfx < 0 && m.average_gfx_activity != UINT16_MAX) s.gfx = m.average_gfx_activity;
      if (s.umc < 0 && m.average_umc_activity != UINT16_MAX) s.umc = m.average_umc_activity;
    }
    const Sample& pv = prev_[i];
    if (pv.ts > 0 && ts > pv.ts) {
      s.xgmi_read_bps = (s.xgmi_read_kb - pv.xgmi_read_kb) * 1024.0 / (ts - pv.ts);
      s.xgmi_write_bps = (s.xgmi_write_kb - pv.xgmi_write_kb) * 1024.0 / (ts - pv.ts);
    }
    prev_[i] = s;
    return s;
  }

  std::vector<Sample> sample() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Sample> out;
    double ts = now_s();
    for (size_t i = 0; i < gpus_.size(); ++i) out.push_back(sample_one(i, ts));
    return out;
  }

  py::dict topology() {
    const size_t n = gpus_.size();
    std::vector<std::vector<std::string>> lt(n, std::vector<std::string>(n));
    std::vector<std::vector<int64_t>> hops(n, std::vector<int64_t>(n, 0)), w(n, std::vector<int64_t>(n, 0));
    std::vector<int> numa(n, 0);
    for (size_t i = 0; i < n; ++i) {
      uint32_t nn = 0;
      if (amdsmi_topo_get_numa_node_number(gpus_[i], &nn) == AMDSMI_STATUS_SUCCESS) numa[i] = static_cast<int>(nn);
      for (size_t j = 0; j < n; ++j) {
        if (i == j) {
          lt[i][j] = "SELF";
          continue;
        }
        uint64_t h = 0;
        amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
        if (amdsmi_topo_get_link_type(gpus_[i], gpus_[j], &h, &t) == AMDSMI_STATUS_SUCCESS) {
          lt[i][j] = t == AMDSMI_LINK_TYPE_XGMI ? "XGMI" : (t == AMDSMI_LINK_TYPE_PCIE ? "PCIE" : "OTHER");
          hops[i][j] = static_cast<int64_t>(h);
        } else {
          lt[i][j] = "UNKNOWN";
        }
        uint64_t wt = 0;
        if (amdsmi_topo_get_link_weight(gpus_[i], gpus_[j], &wt) == AMDSMI_STATUS_SUCCESS) w[i][j] = (int64_t)wt;
      }
    }
    py::dict d;
    d["n"] = static_cast<int>(n);
    d["link_type"] = lt;
    d["hops"] = hops;
    d["weight"] = w;
    d["numa"] = numa;
    return d;
  }

  py::list processes(int idx) {
    py::list out;
    if (idx < 0 || idx >= count()) return out;
    uint32_t n = 0;
    if (amdsmi_get_gpu_process_list(gpus_[idx], &n, nullptr) != AMDSMI_STATUS_SUCCESS || n == 0) return out;
    std::vector<amdsmi_proc_info_t> ps(n);
    if (amdsmi_get_gpu_process_list(gpus_[idx], &n, ps.data()) != AMDSMI_STATUS_SUCCESS) return out;
    for (uint32_t k = 0; k < n; ++k) {
      py::dict d;
      d["pid"] = static_cast<uint64_t>(ps[k].pid);
      d["name"] = std::string(ps[k].name);
      d["vram_bytes"] = ps[k].memory_usage.vram_mem;
      d["gfx_ns"] = ps[k].engine_usage.gfx;
      d["cu_occupancy"] = ps[k].cu_occupancy;
      d["container"] = std::string(ps[k].container_name);
      out.append(d);
    }
    return out;
  }

  // Read-only partition probe: current compute / memory mode, the accelerator partition
  // profiles the driver offers (compute modes with their partition counts and allowed NPS
  // modes) and the memory modes it reports as possible.  Fields that the driver or the
  // caller's privileges do not provide are absent; "errors" says why.
  py::dict partition_info(int idx) {
    py::dict d;
    py::dict errs;
    if (idx < 0 || idx >= count()) {
      errs["index"] = "bad index";
      d["errors"] = errs;
      return d;
    }
    auto h = gpus_[idx];
    char part[64] = {0};
    amdsmi_status_t st = amdsmi_get_gpu_compute_partition(h, part, sizeof(part));
    if (st == AMDSMI_STATUS_SUCCESS) d["compute_partition"] = std::string(part);
    else errs["compute_partition"] = status_str(st);
    char mpart[64] = {0};
    st = amdsmi_get_gpu_memory_partition(h, mpart, sizeof(mpart));
    if (st == AMDSMI_STATUS_SUCCESS) d["memory_partition"] = std::string(mpart);
    else errs["memory_partition"] = status_str(st);
    amdsmi_memory_partition_config_t mc;
    std::memset(&mc, 0, sizeof(mc));
    st = amdsmi_get_gpu_memory_partition_config(h, &mc);
    if (st == AMDSMI_STATUS_SUCCESS) {
      d["memory_caps"] = nps_list(mc.partition_caps);
      d["numa_ranges"] = mc.num_numa_ranges;
    } else {
      errs["memory_config"] = status_str(st);
    }
    auto* cfg = new amdsmi_accelerator_partition_profile_config_t();   // ~40 KB: keep it off the stack
    st = amdsmi_get_gpu_accelerator_partition_profile_config(h, cfg);
    if (st == AMDSMI_STATUS_SUCCESS) {
      py::list profiles;
      for (uint32_t k = 0; k < cfg->num_profiles && k < AMDSMI_MAX_ACCELERATOR_PROFILE; ++k) {
        const auto& pr = cfg->profiles[k];
        py::dict x;
        x["mode"] = std::string(accel_name(pr.profile_type));
        x["partitions"] = pr.num_partitions;
        x["memory_caps"] = nps_list(pr.memory_caps);
        x["profile_index"] = pr.profile_index;
        profiles.append(x);
      }
      d["profiles"] = profiles;
      d["default_profile_index"] = cfg->default_profile_index;
    } else {
      errs["profiles"] = status_str(st);
    }
    delete cfg;
    amdsmi_accelerator_partition_profile_t cur;
    std::memset(&cur, 0, sizeof(cur));
    uint32_t ids[AMDSMI_MAX_ACCELERATOR_PARTITIONS] = {0};
    st = amdsmi_get_gpu_accelerator_partition_profile(h, &cur, ids);
    if (st == AMDSMI_STATUS_SUCCESS) {
      d["current_profile"] = std::string(accel_name(cur.profile_type));
      d["current_partitions"] = cur.num_partitions;
      std::vector<uint32_t> v(ids, ids + std::min<uint32_t>(cur.num_partitions, AMDSMI_MAX_ACCELERATOR_PARTITIONS));
      d["partition_ids"] = v;
    } else {
      errs["current_profile"] = status_str(st);
    }
    amdsmi_kfd_info_t kfd;
    if (amdsmi_get_gpu_kfd_info(h, &kfd) == AMDSMI_STATUS_SUCCESS && kfd.current_partition_id != 0xFFFFFFFFu)
      d["kfd_partition_id"] = kfd.current_partition_id;
    d["errors"] = errs;
    return d;
  }

  py::dict enumeration(int idx) {
    py::dict d;
    if (idx < 0 || idx >= count()) return d;
    amdsmi_enumeration_info_t e;
    std::memset(&e, 0, sizeof(e));
    if (amdsmi_get_gpu_enumeration_info(gpus_[idx], &e) == AMDSMI_STATUS_SUCCESS) {
      d["hip_id"] = e.hip_id;
      d["hsa_id"] = e.hsa_id;
      d["drm_render"] = e.drm_render;
      d["drm_card"] = e.drm_card;
      d["hip_uuid"] = std::string(e.hip_uuid);
    }
    amdsmi_bdf_t bdf;
    if (amdsmi_get_gpu_device_bdf(gpus_[idx], &bdf) == AMDSMI_STATUS_SUCCESS) {
      d["pci_domain"] = static_cast<uint64_t>(bdf.domain_number);
      d["pci_bus"] = static_cast<unsigned>(bdf.bus_number);
      d["pci_device"] = static_cast<unsigned>(bdf.device_number);
    }
    return d;
  }

  std::string set_memory_partition(int idx, const std::string& mode) {
    if (idx < 0 || idx >= count()) return "bad index";
    amdsmi_memory_partition_type_t t = AMDSMI_MEMORY_PARTITION_UNKNOWN;
    for (int k = 1; k <= 8; ++k)
      if (mode == kNps[k]) t = static_cast<amdsmi_memory_partition_type_t>(k);
    if (t == AMDSMI_MEMORY_PARTITION_UNKNOWN) return "unknown mode";
    amdsmi_status_t s = amdsmi_set_gpu_memory_partition(gpus_[idx], t);
    return s == AMDSMI_STATUS_SUCCESS ? "" : status_str(s);
  }

  // ---- light activity sampler (benchmark): gfx/umc %, VRAM, power of selected GPUs ----
  std::vector<Activity> activity(const std::vector<int>& idx) {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<Activity> out;
    double ts = now_s();
    for (int i : idx) {
      if (i < 0 || i >= count()) continue;
      Activity a;
      a.ts = ts;
      a.index = i;
      amdsmi_engine_usage_t u;
      if (amdsmi_get_gpu_activity(gpus_[i], &u) == AMDSMI_STATUS_SUCCESS) {
        a.gfx = u.gfx_activity;
        a.umc = u.umc_activity;
      }
      amdsmi_vram_usage_t v;
      if (amdsmi_get_gpu_vram_usage(gpus_[i], &v) == AMDSMI_STATUS_SUCCESS) a.vram_used_mb = v.vram_used;
      amdsmi_power_info_t p;
      if (amdsmi_get_power_info(gpus_[i], &p) == AMDSMI_STATUS_SUCCESS)
        a.power_w = (p.current_socket_power != UINT32_MAX) ? p.current_socket_power : (double)p.average_socket_power;
      out.push_back(a);
    }
    return out;
  }

  void start_activity(double period_s, int capacity, std::vector<int> idx) {
    act_sampler_.start([this, idx]() { return activity(idx); }, period_s, capacity);
  }

  void stop_activity() { act_sampler_.stop(); }

  std::vector<std::vector<Activity>> drain_activity() { return act_sampler_.drain(); }

  std::string set_compute_partition(int idx, const std::string& mode) {
    if (idx < 0 || idx >= count()) return "bad index";
    amdsmi_compute_partition_type_t t = AMDSMI_COMPUTE_PARTITION_INVALID;
    if (mode == "SPX") t = AMDSMI_COMPUTE_PARTITION_SPX;
    else if (mode == "DPX") t = AMDSMI_COMPUTE_PARTITION_DPX;
    else if (mode == "QPX") t = AMDSMI_COMPUTE_PARTITION_QPX;
    else if (mode == "CPX") t = AMDSMI_COMPUTE_PARTITION_CPX;
    else return "unknown mode";
    amdsmi_status_t s = amdsmi_set_gpu_compute_partition(gpus_[idx], t);
    return s == AMDSMI_STATUS_SUCCESS ? "" : status_str(s);
  }

  // ---- background sampler with a ring buffer (sampler.h; TSan-tested on the host) -----
  void start(double period_s, int capacity) {
    sampler_.start([this]() { return sample(); }, period_s, capacity);
  }

  void stop() { sampler_.stop(); }

  std::vector<std::vector<Sample>> drain() { return sampler_.drain(); }

  void shutdown() {
    stop();
    stop_activity();
    std::lock_guard<std::mutex> g(mu_);
    if (inited_) amdsmi_shut_down();
    inited_ = false;
    gpus_.clear();
  }

 private:
  std::mutex mu_;
  bool inited_ = false;
  std::string err_;
  std::vector<amdsmi_processor_handle> gpus_;
  std::vector<Sample> prev_;
  gs::PeriodicSampler<std::vector<Activity>> act_sampler_;
  gs::PeriodicSampler<std::vector<Sample>> sampler_;   // last members: joined first on destruction
};

py::dict to_dict(const Sample& s) {
  py::dict d;
  d["ts"] = s.ts;
  d["index"] = s.index;
  d["gfx_activity"] = s.gfx;
  d["umc_activity"] = s.umc;
  d["mm_activity"] = s.mm;
  d["vram_used_mb"] = s.vram_used_mb;
  d["vram_total_mb"] = s.vram_total_mb;
  d["power_w"] = s.power_w;
  d["temp_c"] = s.temp_c;
  d["xgmi_read_bps"] = s.xgmi_read_bps;
  d["xgmi_write_bps"] = s.xgmi_write_bps;
  d["ecc_correctable"] = s.ecc_correctable;
  d["ecc_uncorrectable"] = s.ecc_uncorrectable;
  d["ecc_deferred"] = s.ecc_deferred;
  d["responsive"] = s.responsive;
  return d;
}

}  // namespace

PYBIND11_MODULE(_smi, m) {
  m.doc() = "amd-smi telemetry, topology and partition control";
  py::class_<Smi>(m, "Smi")
      .def(py::init<>())
      .def("init", &Smi::init)
      .def("error", &Smi::error)
      .def("count", &Smi::count)
      .def("devices", &Smi::devices)
      .def("sample",
           [](Smi& s) {
             py::list out;
             for (auto& x : s.sample()) out.append(to_dict(x));
             return out;
           })
      .def("topology", &Smi::topology)
      .def("processes", &Smi::processes)
      .def("set_compute_partition", &Smi::set_compute_partition)
      .def("set_memory_partition", &Smi::set_memory_partition)
      .def("partition_info", &Smi::partition_info)
      .def("enumeration", &Smi::enumeration)
      .def("start_activity", &Smi::start_activity, py::arg("period_s") = 0.005, py::arg("capacity") = 200000,
           py::arg("indices") = std::vector<int>{})
      .def("stop_activity", &Smi::stop_activity, py::call_guard<py::gil_scoped_release>())
      .def("drain_activity",
           [](Smi& s) {
             // flat rows (ts, index, gfx %, umc %, vram used MB, power W); -1 = not reported
             std::vector<std::vector<double>> out;
             for (auto& v : s.drain_activity())
               for (auto& a : v) out.push_back({a.ts, (double)a.index, a.gfx, a.umc, a.vram_used_mb, a.power_w});
             return out;
           })
      .def("start", &Smi::start, py::arg("period_s") = 1.0, py::arg("capacity") = 600)
      .def("stop", &Smi::stop, py::call_guard<py::gil_scoped_release>())
      .def("drain",
           [](Smi& s) {
             py::list out;
             for (auto& v : s.drain()) {
               py::list row;
               for (auto& x : v) row.append(to_dict(x));
               out.append(row);
             }
             return out;
           })
      .def("shutdown", &Smi::shutdown, py::call_guard<py::gil_scoped_release>());
}
