// CU-masked streams = fractional GPU sharing on MI355X.
//
// The reference shares a V100 through MPS (CUDA_MPS_ACTIVE_THREAD_PERCENTAGE 50/25 and a
// pinned memory limit, pkg/plugins/gpu_plugin/gpu_plugins.go:896-917) and an A30 through
// MIG.  The MI355X analog inside one process is a HIP stream whose hardware queue is
// restricted to a CU mask (hipExtStreamCreateWithCUMask): the GPU plugin hands each
// fractional pod a run of CU-slice units (one 32-bit mask word = 4 CUs on each of the 8
// XCDs -- a mask that leaves an XCD empty is ignored by the driver, measured), and the
// executor runs a Guaranteed pod's kernels on a stream masked to exactly those CUs.  A
// container gets the same restriction process-wide from HSA_CU_MASK="0:<cu ranges>"
// (verified in-container: profiles/r01_e2e_container_view.json).
//
// `probe_xcd` launches one workgroup per slot that records HW_REG_XCC_ID and HW_REG_HW_ID;
// the host uses it to verify which XCDs / CUs a mask really maps to.
#include <cstdint>
#include <vector>

#include "api.h"
#include "common.h"

namespace gs {

__global__ void __launch_bounds__(64) probe_kernel(uint32_t* out, int n) {
  int b = blockIdx.x;
  if (b >= n || threadIdx.x != 0) return;
  uint32_t xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  // spin a little so blocks spread over the allowed CUs instead of reusing one CU
  uint64_t t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < 20000) {
  }
  out[2 * b] = xcc;
  out[2 * b + 1] = hwid;
}

uintptr_t create_masked_stream(const std::vector<uint32_t>& mask) {
  hipStream_t s = nullptr;
  HIP_CHECK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask.size()), mask.data()));
  return reinterpret_cast<uintptr_t>(s);
}

uintptr_t create_stream(int priority) {
  hipStream_t s = nullptr;
  HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  return reinterpret_cast<uintptr_t>(s);
}

void destroy_stream(uintptr_t s) { HIP_CHECK(hipStreamDestroy(reinterpret_cast<hipStream_t>(s))); }

std::vector<uint32_t> get_stream_mask(uintptr_t s) {
  std::vector<uint32_t> m(8, 0);
  HIP_CHECK(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(s), static_cast<uint32_t>(m.size()), m.data()));
  return m;
}

// Returns 2*n words: (xcc_id, hw_id) per workgroup.
std::vector<uint32_t> probe_xcd(uintptr_t stream, int n) {
  if (n <= 0 || n > (1 << 20)) throw std::runtime_error("probe_xcd: n out of range");
  (void)hipGetLastError();
  uint32_t* d = nullptr;
  HIP_CHECK(hipMalloc(&d, sizeof(uint32_t) * 2 * n));
  HIP_CHECK(hipMemsetAsync(d, 0xff, sizeof(uint32_t) * 2 * n, reinterpret_cast<hipStream_t>(stream)));
  hipLaunchKernelGGL(probe_kernel, dim3(n), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), d, n);
  HIP_CHECK(hipGetLastError());
  std::vector<uint32_t> h(2 * n);
  HIP_CHECK(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
  HIP_CHECK(hipMemcpy(h.data(), d, sizeof(uint32_t) * 2 * n, hipMemcpyDeviceToHost));
  HIP_CHECK(hipFree(d));
  return h;
}

}  // namespace gs
