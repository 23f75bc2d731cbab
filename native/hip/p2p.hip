// xGMI peer-to-peer probes: access matrix + per-pair copy bandwidth.
//
// No reference equivalent (the reference never places multi-GPU pods).
// The topology Filter assumes every MI355X pair is one xGMI hop; this probe verifies it
// (hipDeviceCanAccessPeer) and measures the per-link copy rate (one xGMI link is
// ~153 GB/s per direction on MI355X), so a placement can be validated on the node.
#include <chrono>
#include <vector>

#include "api.h"
#include "common.h"

namespace gs {

std::vector<int> peer_access_matrix() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return {};
  std::vector<int> m(n * n, 0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      int can = (i == j);
      if (i != j) hipDeviceCanAccessPeer(&can, i, j);
      m[i * n + j] = can;
    }
  return m;
}

// Copies `bytes` from device src to device dst `iters` times; returns GB/s.
double peer_copy_gbps(int src, int dst, size_t bytes, int iters) {
  if (bytes == 0 || iters <= 0) throw std::runtime_error("peer_copy_gbps: bad args");
  int prev = 0;
  HIP_CHECK(hipGetDevice(&prev));
  void *a = nullptr, *b = nullptr;
  HIP_CHECK(hipSetDevice(src));
  HIP_CHECK(hipMalloc(&a, bytes));
  if (src != dst) hipDeviceEnablePeerAccess(dst, 0);
  HIP_CHECK(hipSetDevice(dst));
  HIP_CHECK(hipMalloc(&b, bytes));
  if (src != dst) hipDeviceEnablePeerAccess(src, 0);
  hipGetLastError();  // clear "already enabled"
  HIP_CHECK(hipSetDevice(src));
  hipStream_t s;
  HIP_CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  HIP_CHECK(hipMemcpyPeerAsync(b, dst, a, src, bytes, s));  // warm-up
  HIP_CHECK(hipEventRecord(e0, s));
  for (int i = 0; i < iters; ++i) HIP_CHECK(hipMemcpyPeerAsync(b, dst, a, src, bytes, s));
  HIP_CHECK(hipEventRecord(e1, s));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(s);
  hipFree(a);
  HIP_CHECK(hipSetDevice(dst));
  hipFree(b);
  hipSetDevice(prev);
  return (double)bytes * iters / (ms * 1e-3) / 1e9;
}

}  // namespace gs
