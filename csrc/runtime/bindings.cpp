// pybind11 module `llm_weighted_consensus_amd._runtime`: host runtime of the engine and the
// consensus core.  No GPU dependency (plain g++), so CPU tests load exactly this code.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "block_manager.h"
#include "consensus_core.h"

namespace py = pybind11;
using lwc::BlockManager;

namespace lwc {
void bind_json(py::module_& m);  // json_encode.cpp

// Python face of the consensus core (kept out of consensus_core.cpp so the core also builds without
// Python, e.g. the sanitizer self-test csrc/tests/runtime_selftest.cpp).
void bind_consensus_core(py::module_& m) {
  py::class_<KeyTree>(m, "KeyTree")
      .def(py::init<int, int, uint64_t>(), py::arg("source_len"), py::arg("max_branch_len"), py::arg("seed"))
      .def_property_readonly("keys", &KeyTree::keys)
      .def_property_readonly("depth", &KeyTree::depth)
      .def_property_readonly("source_len", &KeyTree::source_len)
      .def("regex_patterns", &KeyTree::regex_patterns)
      .def("find_key", &KeyTree::find_key)
      .def(
          "vote",
          [](const KeyTree& t, const std::string& content,
             std::optional<std::vector<std::pair<std::string, std::vector<std::pair<std::string, double>>>>> lp) {
            return t.vote(content, lp ? &*lp : nullptr);
          },
          py::arg("content"), py::arg("logprobs") = py::none());
  py::class_<TallyResult>(m, "TallyResult")
      .def_readonly("choice_weight", &TallyResult::choice_weight)
      .def_readonly("confidence", &TallyResult::confidence)
      .def_readonly("voter_confidence", &TallyResult::voter_confidence);
  m.def("tally", &tally, py::arg("votes"), py::arg("weights"), py::arg("num_choices"));
  m.def("unify_error_codes", &unify_error_codes);
}

}  // namespace lwc


namespace {

// Append one token to every sequence and build the padded decode batch in one call:
// returns (block_tables[B, width] int32, ctx_lens[B] int32, slots[B] int32, positions[B] int32).
// `width` >= every table length (the engine passes its captured-graph width).
py::tuple prepare_decode(BlockManager& bm, const std::vector<int64_t>& seqs, int width, int pad_to) {
  const int B = (int)seqs.size();
  const int Bp = std::max(B, pad_to);
  py::array_t<int32_t> bt({Bp, width}), ctx(Bp), slots(Bp), pos(Bp);
  auto btm = bt.mutable_unchecked<2>();
  auto cm = ctx.mutable_unchecked<1>();
  auto sm = slots.mutable_unchecked<1>();
  auto pm = pos.mutable_unchecked<1>();
  for (int i = 0; i < B; ++i) {
    const int64_t slot = bm.append_token(seqs[i]);
    const auto& tab = bm.block_table(seqs[i]);
    if ((int)tab.size() > width) throw std::runtime_error("prepare_decode: block table wider than batch width");
    for (int j = 0; j < width; ++j) btm(i, j) = j < (int)tab.size() ? tab[j] : 0;
    const int64_t len = bm.length(seqs[i]);
    cm(i) = (int32_t)len;
    sm(i) = (int32_t)slot;
    pm(i) = (int32_t)(len - 1);
  }
  for (int i = B; i < Bp; ++i) {  // padding rows: 1-token context on block 0, no cache write
    for (int j = 0; j < width; ++j) btm(i, j) = 0;
    cm(i) = 1;
    sm(i) = -1;
    pm(i) = 0;
  }
  return py::make_tuple(bt, ctx, slots, pos);
}

int32_t* writable_i32(py::array& a, int64_t need, const char* name) {
  if (a.dtype().kind() != 'i' || a.itemsize() != 4 || !(a.flags() & py::array::c_style) || !a.writeable())
    throw std::runtime_error(std::string("prepare_decode_into: ") + name + " must be a writable C-contiguous int32 array");
  if (a.size() < need) throw std::runtime_error(std::string("prepare_decode_into: ") + name + " too short");
  return static_cast<int32_t*>(a.mutable_data());
}

// Same as prepare_decode but writes straight into caller-owned arrays (views of one pinned staging
// buffer), so a decode step costs a single host->device copy.  Only the first `used_width` columns
// of each block-table row are rewritten (columns beyond a row's table are never read by the
// attention kernels, which stop at ctx_len).
void prepare_decode_into(BlockManager& bm, const std::vector<int64_t>& seqs, int width, int pad_to, py::array bt,
                         py::array ctx, py::array slots, py::array pos) {
  const int B = (int)seqs.size();
  const int Bp = std::max(B, pad_to);
  int32_t* btp = writable_i32(bt, (int64_t)Bp * width, "block_tables");
  int32_t* cp = writable_i32(ctx, Bp, "ctx_lens");
  int32_t* sp = writable_i32(slots, Bp, "slots");
  int32_t* pp = writable_i32(pos, Bp, "positions");
  for (int i = 0; i < B; ++i) {
    const int64_t slot = bm.append_token(seqs[i]);
    const auto& tab = bm.block_table(seqs[i]);
    if ((int)tab.size() > width) throw std::runtime_error("prepare_decode_into: block table wider than batch width");
    int32_t* row = btp + (size_t)i * width;
    for (size_t j = 0; j < tab.size(); ++j) row[j] = (int32_t)tab[j];
    const int64_t len = bm.length(seqs[i]);
    cp[i] = (int32_t)len;
    sp[i] = (int32_t)slot;
    pp[i] = (int32_t)(len - 1);
  }
  for (int i = B; i < Bp; ++i) {  // padding rows: 1-token context on block 0, no cache write
    btp[(size_t)i * width] = 0;
    cp[i] = 1;
    sp[i] = -1;
    pp[i] = 0;
  }
}

// Slots of positions [start, start+count) of a sequence (prefill scatter targets).
py::array_t<int32_t> slots_range(const BlockManager& bm, int64_t seq, int64_t start, int64_t count) {
  py::array_t<int32_t> out(count);
  auto m = out.mutable_unchecked<1>();
  for (int64_t i = 0; i < count; ++i) m(i) = (int32_t)bm.slot(seq, start + i);
  return out;
}

}  // namespace

PYBIND11_MODULE(_runtime, m) {
  lwc::bind_json(m);
  m.doc() = "llm_weighted_consensus_amd host runtime: paged-KV block manager and consensus core";

  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int>(), py::arg("num_blocks"), py::arg("block_size"))
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("num_free", &BlockManager::num_free)
      .def_property_readonly("num_sequences", &BlockManager::num_sequences)
      .def("has_sequence", &BlockManager::has_sequence)
      .def("blocks_for", &BlockManager::blocks_for)
      .def("can_allocate", &BlockManager::can_allocate)
      .def("add_sequence", &BlockManager::add_sequence)
      .def("fork", &BlockManager::fork)
      .def("append_token", &BlockManager::append_token)
      .def("append_cost", &BlockManager::append_cost)
      .def("free_sequence", &BlockManager::free_sequence)
      .def("set_prefix_caching", &BlockManager::set_prefix_caching)
      .def_property_readonly("prefix_caching", &BlockManager::prefix_caching)
      .def("match_prefix", &BlockManager::match_prefix)
      .def("add_sequence_cached", &BlockManager::add_sequence_cached)
      .def("cache_prefix", &BlockManager::cache_prefix)
      .def_property_readonly("num_cached_blocks", &BlockManager::num_cached_blocks)
      .def_property_readonly("num_evictable", &BlockManager::num_evictable)
      .def("length", &BlockManager::length)
      .def("block_table", &BlockManager::block_table)
      .def("slot", &BlockManager::slot)
      .def("refcount", &BlockManager::refcount)
      .def("take_copies", &BlockManager::take_copies)
      .def("append_cost_total", &BlockManager::append_cost_total)
      .def("swap_out",
           [](BlockManager& bm, const std::vector<int64_t>& seqs) {
             BlockManager::Swapped s = bm.swap_out(seqs);
             return py::make_tuple(s.blocks, s.tables, s.lens);
           })
      .def("swap_in", &BlockManager::swap_in, py::arg("seqs"), py::arg("n"), py::arg("tables"), py::arg("lens"));
  m.def("prepare_decode", &prepare_decode, py::arg("bm"), py::arg("seqs"), py::arg("width"), py::arg("pad_to") = 0);
  m.def("prepare_decode_into", &prepare_decode_into, py::arg("bm"), py::arg("seqs"), py::arg("width"),
        py::arg("pad_to"), py::arg("block_tables"), py::arg("ctx_lens"), py::arg("slots"), py::arg("positions"));
  m.def("slots_range", &slots_range);

  lwc::bind_consensus_core(m);
}
