// pybind11 module `_hip`: device query, CU-masked streams, XCD probe, load kernels,
// xGMI probes.  All device pointers / streams cross the boundary as integers
// (torch.Tensor.data_ptr(), torch.cuda.Stream.cuda_stream), so the module does not link
// libtorch and builds in seconds with hipcc.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <string>
#include <vector>

#include "api.h"

namespace py = pybind11;

PYBIND11_MODULE(_hip, m) {
  m.doc() = "MI355X native HIP layer (gfx950)";
  m.attr("ARCH") = "gfx950";
  m.def("device_count", &gs::device_count);
  m.def("query_all", []() {
    py::list out;
    for (auto& d : gs::query_all()) {
      py::dict x;
      x["index"] = d.index;
      x["name"] = d.name;
      x["arch"] = d.arch;
      x["uuid"] = d.uuid;
      x["rocr_uuid"] = d.rocr_uuid;
      x["pci"] = d.pci;
      x["cus"] = d.cus;
      x["clock_khz"] = d.clock_khz;
      x["mem_clock_khz"] = d.mem_clock_khz;
      x["warp"] = d.warp;
      x["l2_bytes"] = d.l2_bytes;
      x["max_threads"] = d.max_threads;
      x["lds_per_block"] = d.lds_per_block;
      x["total_mem"] = d.total_mem;
      x["free_mem"] = d.free_mem;
      x["heap_limit"] = d.heap_limit;
      x["fifo_limit"] = d.fifo_limit;
      x["stack_limit"] = d.stack_limit;
      out.append(x);
    }
    return out;
  });
  m.def("create_masked_stream", &gs::create_masked_stream, py::arg("mask"));
  m.def("create_stream", &gs::create_stream, py::arg("priority") = 0);
  m.def("destroy_stream", &gs::destroy_stream);
  m.def("get_stream_mask", &gs::get_stream_mask);
  m.def("probe_xcd", &gs::probe_xcd, py::arg("stream"), py::arg("n"));
  m.def("gemm_bf16_nt", &gs::gemm_bf16_nt, py::arg("a"), py::arg("bt"), py::arg("c"), py::arg("bias"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("relu"),
        py::arg("stream"), py::arg("cu_budget") = 0, py::arg("workspace") = 0, py::arg("workspace_floats") = 0,
        py::call_guard<py::gil_scoped_release>());
  m.def("pick_split_k", &gs::pick_split_k, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("cu_budget") = 0);
  m.def("splitk_workspace_floats", &gs::splitk_workspace_floats, py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("cu_budget") = 0);
  m.def("set_split_k", &gs::set_split_k, py::arg("s"));
  m.def("gemm_fp8_nt", &gs::gemm_fp8_nt, py::arg("a"), py::arg("bt"), py::arg("c"), py::arg("bias"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("lda"), py::arg("ldb"), py::arg("ldc"), py::arg("relu"),
        py::arg("stream"), py::arg("cu_budget") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("stream_triad", &gs::stream_triad, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("s"),
        py::arg("n_floats"), py::arg("blocks"), py::arg("stream"), py::call_guard<py::gil_scoped_release>());
  m.def("set_triad_variant", &gs::set_triad_variant, py::arg("variant"));
  m.def("set_gemm_tile", &gs::set_gemm_tile, py::arg("tile"));
  m.def("set_w4_probe", &gs::set_w4_probe, py::arg("mask"));
  m.def("set_w4_prio", &gs::set_w4_prio, py::arg("on"));
  m.def("set_gemm_policy", &gs::set_gemm_policy, py::arg("policy"));
  m.def("set_wide_epilogue", &gs::set_wide_epilogue, py::arg("on"));
  m.def("set_xcd_blocks", &gs::set_xcd_blocks, py::arg("on"));
  m.def("set_lone_plain_order", &gs::set_lone_plain_order, py::arg("on"));
  m.def("set_xcd_group", &gs::set_xcd_group, py::arg("rows"));
  m.def("xcd_probe", &gs::xcd_probe, py::arg("out"), py::arg("blocks"), py::arg("stream"));
  m.def("pick_xcd_map", &gs::pick_xcd_map, py::arg("tiles_m"), py::arg("tiles_n"));
  m.def("pick_gemm_tile", &gs::pick_gemm_tile, py::arg("M"), py::arg("N"), py::arg("cu_budget") = 0);
  m.def("gemm_workgroups", &gs::gemm_workgroups, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("cu_budget") = 0,
        py::arg("fp8") = false, py::arg("split_workspace") = false);
  m.def("peer_access_matrix", &gs::peer_access_matrix);
  m.def("peer_copy_gbps", &gs::peer_copy_gbps, py::arg("src"), py::arg("dst"), py::arg("bytes"),
        py::arg("iters") = 10, py::call_guard<py::gil_scoped_release>());
}
