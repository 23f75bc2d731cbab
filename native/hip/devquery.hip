// Device query for every visible GPU.
//
// Reference: pkg/profiler/gpu_profiling.cpp:10-24 queries device 0 only with
// cudaMemGetInfo / cudaGetDeviceProperties / cudaDeviceGetLimit(heap, fifo, stack) and was
// never built (pkg/profiler/Makefile:13-14).  Here: all devices, HIP runtime, plus the
// MI355X facts the scheduler needs (gfx arch, CU count, XCC count via the XCD probe,
// UUID, PCI BDF, HBM free/total, clocks, L2 size).
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "api.h"
#include "common.h"

namespace gs {

static std::string hex_uuid(const hipUUID& u) {
  static const char* hx = "0123456789abcdef";
  std::string s;
  for (int i = 0; i < 16; ++i) {
    unsigned char c = static_cast<unsigned char>(u.bytes[i]);
    s += hx[c >> 4];
    s += hx[c & 15];
    if (i == 3 || i == 5 || i == 7 || i == 9) s += '-';
  }
  return s;
}

// ROCm fills hipUUID with the ASCII of the agent's unique id (16 hex digits); rocminfo,
// amd-smi's ROCm id and ROCR_VISIBLE_DEVICES all name the device "GPU-<those digits>".
static std::string rocr_uuid(const hipUUID& u) {
  std::string s;
  for (int i = 0; i < 16; ++i) {
    const char c = u.bytes[i];
    const bool hexdig = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
    if (!hexdig) return "";
    s += c;
  }
  return "GPU-" + s;
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

std::vector<DevInfo> query_all() {
  std::vector<DevInfo> out;
  int n = device_count();
  int prev = 0;
  hipGetDevice(&prev);
  for (int d = 0; d < n; ++d) {
    DevInfo di;
    di.index = d;
    hipDeviceProp_t p;
    HIP_CHECK(hipGetDeviceProperties(&p, d));
    di.name = p.name;
    di.arch = p.gcnArchName;
    di.cus = p.multiProcessorCount;
    di.clock_khz = p.clockRate;
    di.mem_clock_khz = p.memoryClockRate;
    di.warp = p.warpSize;
    di.l2_bytes = p.l2CacheSize;
    di.max_threads = p.maxThreadsPerBlock;
    di.lds_per_block = p.sharedMemPerBlock;
    di.total_mem = p.totalGlobalMem;
    di.pci_bus = p.pciBusID;
    di.pci_device = p.pciDeviceID;
    di.pci_domain = p.pciDomainID;
    char bdf[32];
    std::snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.0", p.pciDomainID, p.pciBusID, p.pciDeviceID);
    di.pci = bdf;
    hipUUID u;
    if (hipDeviceGetUuid(&u, d) == hipSuccess) {
      di.uuid = hex_uuid(u);
      di.rocr_uuid = rocr_uuid(u);
    }
    HIP_CHECK(hipSetDevice(d));
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) {
      di.free_mem = fr;
      di.total_mem = tot;
    }
    hipDeviceGetLimit(&di.heap_limit, hipLimitMallocHeapSize);
    hipDeviceGetLimit(&di.fifo_limit, hipLimitPrintfFifoSize);
    hipDeviceGetLimit(&di.stack_limit, hipLimitStackSize);
    (void)hipGetLastError();  // unsupported limits set the sticky last-error; clear it
    out.push_back(di);
  }
  if (n) hipSetDevice(prev);
  return out;
}

}  // namespace gs
