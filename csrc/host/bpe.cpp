// Native byte-level BPE encoder (host C++, pybind11) — the framework's counterpart of the
// reference's tokenizer runtime (tiktoken's Rust core, build_components.py:278 and
// Models/Llama/Llama3.py:14-51).
//
// encode_ordinary(text) runs entirely in C++:
//   1. UTF-8 decode into code points;
//   2. pre-tokenisation with a hand-written matcher for the GPT-2 and the Llama-3 patterns
//      (the same alternation order and greedy/backtracking semantics as the regexes in
//      data/tokenizer.py), using a per-code-point class table (letter / number / whitespace /
//      other) that Python derives from the very `regex` classes the reference patterns use;
//   3. byte-pair merging of each piece by lowest rank (tiktoken semantics), with a piece cache.
// Special tokens are split off in Python before this is called (allowed_special semantics).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "bpe_core.h"

namespace py = pybind11;
using bllm_host::BPECore;

namespace {

BPECore* make_core(const py::dict& ranks, const std::string& kind, const py::bytes& classes) {
  std::unordered_map<std::string, int> r;
  r.reserve(ranks.size());
  for (auto item : ranks)
    r.emplace(py::cast<std::string>(py::reinterpret_borrow<py::bytes>(item.first)), py::cast<int>(item.second));
  return new BPECore(std::move(r), kind, std::string(classes));
}

}  // namespace

PYBIND11_MODULE(_bpe, m) {
  m.doc() = "Native byte-level BPE (GPT-2 / Llama-3 pre-tokenisation + rank merging)";
  py::class_<BPECore>(m, "BPECore")
      .def(py::init(&make_core))
      .def("encode_ordinary", &BPECore::encode_ordinary, py::call_guard<py::gil_scoped_release>())
      .def("pre_tokenize", &BPECore::pre_tokenize)
      .def("cache_size", &BPECore::cache_size);
}
