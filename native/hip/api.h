// Declarations shared by the HIP sources and the pybind11 bindings.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace gs {
struct DevInfo {
  int index = 0;
  std::string name, arch, uuid, rocr_uuid, pci;
  int cus = 0, clock_khz = 0, mem_clock_khz = 0, warp = 0, l2_bytes = 0, max_threads = 0;
  size_t lds_per_block = 0, total_mem = 0, free_mem = 0;
  size_t heap_limit = 0, fifo_limit = 0, stack_limit = 0;
  int pci_bus = 0, pci_device = 0, pci_domain = 0;
};
int device_count();
std::vector<DevInfo> query_all();
uintptr_t create_masked_stream(const std::vector<uint32_t>& mask);
uintptr_t create_stream(int priority);
void destroy_stream(uintptr_t s);
std::vector<uint32_t> get_stream_mask(uintptr_t s);
std::vector<uint32_t> probe_xcd(uintptr_t stream, int n);
void gemm_bf16_nt(uintptr_t a, uintptr_t bt, uintptr_t c, uintptr_t bias, int M, int N, int K, int lda, int ldb,
                  int ldc, bool relu, uintptr_t stream, int cu_budget, uintptr_t workspace = 0,
                  size_t workspace_floats = 0);
int pick_split_k(int M, int N, int K, int cu_budget);
size_t splitk_workspace_floats(int M, int N, int K, int cu_budget);
void set_split_k(int s);
void gemm_fp8_nt(uintptr_t a, uintptr_t bt, uintptr_t c, uintptr_t bias, int M, int N, int K, int lda, int ldb,
                 int ldc, bool relu, uintptr_t stream, int cu_budget);
void stream_triad(uintptr_t a, uintptr_t b, uintptr_t c, float s, size_t n_floats, int blocks, uintptr_t stream);
void set_triad_variant(int v);
void set_gemm_tile(int t);
void set_w4_probe(int mask);
void set_w4_prio(int on);
void set_gemm_policy(int p);
void set_wide_epilogue(int on);
void set_xcd_blocks(int on);
void set_lone_plain_order(int on);
void set_xcd_group(int rows);
void xcd_probe(uintptr_t out, int blocks, uintptr_t stream);
int pick_xcd_map(int tiles_m, int tiles_n);
int pick_gemm_tile(int M, int N, int cu_budget);
// workgroups of the GEMM launch this shape / CU budget gets (the kernel's CU footprint)
int gemm_workgroups(int M, int N, int K, int cu_budget, bool fp8, bool split_workspace);
std::vector<int> peer_access_matrix();
double peer_copy_gbps(int src, int dst, size_t bytes, int iters);
}  // namespace gs
