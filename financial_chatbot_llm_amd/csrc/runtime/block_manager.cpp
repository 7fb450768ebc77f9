// pybind11 binding of the native paged-KV block allocator (block_allocator.h): module
// _penny_runtime, class BlockAllocator; the engine-facing wrapper is
// engine/native_block_manager.py.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_allocator.h"

namespace py = pybind11;
using penny::BlockAllocator;

PYBIND11_MODULE(_penny_runtime, m) {
  m.doc() = "Native host runtime for the MI355X serving engine (paged-KV block allocator)";
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
}
