// pybind11 bindings of the native host runtime, module _penny_runtime:
//   BlockAllocator -- the paged-KV block allocator (block_allocator.h; engine-facing wrapper
//                     engine/native_block_manager.py)
//   StepRing       -- the shared-memory TP step-broadcast ring (step_ring.h; parallel/step_ring.py)
//   mark_shared_blocks -- per decode step, the shared-prefix blocks of the decode block table
//                     (ops/attention.py mark_shared_blocks, the lean decode kernel's cache policy)
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "block_allocator.h"
#include "step_ring.h"

namespace py = pybind11;
using penny::BlockAllocator;
using penny::StepRing;

namespace {

// bt [B, W] int32 (zero-padded decode block table), ctx [B] tokens.  A physical block at the same
// column of two rows' tables is shared (the prefix cache only ever shares identical prefixes, so a
// shared block's predecessors are shared too): each row's leading run of such blocks (first
// max_cols columns) is rewritten as -id - 1.  Column by column over the rows still in their run:
// sort (id, row) pairs, equal neighbours are shared.  ~B log B per column, stops when no row runs on.
void mark_shared_blocks(py::array_t<int32_t, py::array::c_style> bt, py::array_t<int32_t, py::array::c_style> ctx,
                        int max_cols, int block_size) {
  auto t = bt.mutable_unchecked<2>();
  auto c = ctx.unchecked<1>();
  const int B = (int)t.shape(0), W = (int)t.shape(1), J = std::min(W, max_cols);
  if (c.shape(0) != B) throw std::invalid_argument("ctx length != rows");
  std::vector<int> lead(B, 0), nb(B), live;
  for (int b = 0; b < B; ++b) {
    nb[b] = (c(b) + block_size - 1) / block_size;
    if (nb[b] > 0) live.push_back(b);
  }
  std::vector<std::pair<int32_t, int>> col;
  for (int j = 0; j < J && live.size() > 1; ++j) {
    col.clear();
    for (int b : live)
      if (j < nb[b]) col.emplace_back(t(b, j), b);
    std::sort(col.begin(), col.end());
    std::vector<int> next;
    for (size_t i = 0; i < col.size(); ++i) {
      const bool dup = (i > 0 && col[i - 1].first == col[i].first) ||
                       (i + 1 < col.size() && col[i + 1].first == col[i].first);
      if (dup) {
        lead[col[i].second] = j + 1;
        next.push_back(col[i].second);
      }
    }
    live.swap(next);
  }
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < lead[b]; ++j) t(b, j) = -t(b, j) - 1;
}

}  // namespace

PYBIND11_MODULE(_penny_runtime, m) {
  m.doc() = "Native host runtime for the MI355X serving engine (paged-KV block allocator, TP step ring)";
  m.def("mark_shared_blocks", &mark_shared_blocks, py::arg("bt"), py::arg("ctx"), py::arg("max_cols"),
        py::arg("block_size"));
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"), py::arg("prefix_caching"))
      .def("num_blocks", &BlockAllocator::num_blocks)
      .def("num_free", &BlockAllocator::num_free)
      .def("block_size", &BlockAllocator::block_size)
      .def("blocks_needed", &BlockAllocator::blocks_needed)
      .def("match_prefix", &BlockAllocator::match_prefix)
      .def("grow", &BlockAllocator::grow)
      .def("commit", &BlockAllocator::commit)
      .def("num_committed", &BlockAllocator::num_committed)
      .def("table", &BlockAllocator::table)
      .def("free", &BlockAllocator::free, py::arg("seq"), py::arg("keep_blocks") = -1)
      .def("usage", &BlockAllocator::usage)
      .def("check_invariants", &BlockAllocator::check_invariants)
      .def_property_readonly("hits", &BlockAllocator::hits)
      .def_property_readonly("queries", &BlockAllocator::queries)
      .def_property_readonly("evictions", &BlockAllocator::evictions);

  py::class_<StepRing>(m, "StepRing")
      .def(py::init<const std::string&, bool, uint64_t, uint64_t, uint64_t>(), py::arg("name"), py::arg("create"),
           py::arg("nslots") = 8, py::arg("slot_bytes") = 1 << 20, py::arg("nreaders") = 1)
      .def_property_readonly("name", &StepRing::name)
      .def_property_readonly("slot_bytes", &StepRing::slot_bytes)
      .def_property_readonly("nslots", &StepRing::nslots)
      .def_property_readonly("nreaders", &StepRing::nreaders)
      .def_property_readonly("closed", &StepRing::closed)
      .def_property_readonly("head", &StepRing::head)
      // writer: False if the message exceeds a slot (send it another way); raises on timeout
      .def("put",
           [](StepRing& r, py::buffer b, double timeout_s) {
             py::buffer_info info = b.request();
             const uint64_t len = (uint64_t)info.size * (uint64_t)info.itemsize;
             const void* ptr = info.ptr;
             py::gil_scoped_release nogil;
             return r.put(ptr, len, timeout_s);
           },
           py::arg("data"), py::arg("timeout_s") = 300.0)
      // reader: the next message as a uint8 array, or None on timeout
      .def("get",
           [](StepRing& r, uint64_t reader, double timeout_s) -> py::object {
             std::vector<uint8_t> buf;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = r.get(reader, buf, timeout_s);
             }
             if (!ok) return py::none();
             py::array_t<uint8_t> out((py::ssize_t)buf.size());
             if (!buf.empty()) std::memcpy(out.mutable_data(), buf.data(), buf.size());
             return std::move(out);
           },
           py::arg("reader"), py::arg("timeout_s") = -1.0)
      .def("close", &StepRing::close);
}
