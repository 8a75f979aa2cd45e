// Native dataset index builders (module fleetx_amd._C._native).
//
// Capability parity with reference `ppfleetx/data/data_tools/cpp/
// fast_index_map_helpers.cpp` (D03 / N-1 in SURVEY.md): the same four entry
// points with bit-identical outputs for the same seed (std::mt19937 /
// std::mt19937_64 draws in the same order), so index files built by either
// implementation are interchangeable.
//
// Design differences: single pass with geometric vector growth (the reference
// walks the corpus twice to size its buffer), one shared sentence-packing
// walker for the "mapping" and "blocks mapping" variants, GIL released for
// the heavy loops, and result buffers handed to numpy without copies.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <iostream>
#include <limits>
#include <random>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

constexpr int32_t kLongSentence = 512;

template <typename T>
py::array_t<T> to_numpy(std::vector<T>* v, int64_t rows, int64_t cols) {
  py::capsule owner(v, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>({rows, cols}, {cols * (int64_t)sizeof(T), (int64_t)sizeof(T)}, v->data(),
                        owner);
}

// ------------------------------------------------------------------ blending
void build_blending_indices(py::array_t<uint8_t>& dataset_index,
                            py::array_t<int64_t>& dataset_sample_index,
                            const py::array_t<double>& weights, int32_t num_datasets, int64_t size,
                            bool verbose) {
  auto di = dataset_index.mutable_unchecked<1>();
  auto dsi = dataset_sample_index.mutable_unchecked<1>();
  auto w = weights.unchecked<1>();
  std::vector<int64_t> used(num_datasets, 0);
  {
    py::gil_scoped_release nogil;
    for (int64_t s = 0; s < size; ++s) {
      const double t = std::max(static_cast<double>(s), 1.0);
      int64_t best = 0;
      double best_err = w[0] * t - static_cast<double>(used[0]);
      for (int64_t d = 1; d < num_datasets; ++d) {
        const double err = w[d] * t - static_cast<double>(used[d]);
        if (err > best_err) {
          best_err = err;
          best = d;
        }
      }
      di[s] = static_cast<uint8_t>(best);
      dsi[s] = used[best]++;
    }
  }
  if (verbose) {
    for (int32_t d = 0; d < num_datasets; ++d)
      std::cout << "   dataset " << d << ", input: " << w[d]
                << ", achieved: " << static_cast<double>(used[d]) / size << std::endl;
  }
}

// ------------------------------------------------------------------ GPT samples
py::array build_sample_idx(const py::array_t<int32_t>& sizes_, const py::array_t<int32_t>& doc_idx_,
                           int32_t seq_length, int32_t num_epochs, int64_t tokens_per_epoch) {
  if (seq_length <= 1 || num_epochs <= 0 || tokens_per_epoch <= 1)
    throw std::invalid_argument("build_sample_idx: bad arguments");
  auto sizes = sizes_.unchecked<1>();
  auto doc_idx = doc_idx_.unchecked<1>();
  const int64_t num_samples = (num_epochs * tokens_per_epoch - 1) / seq_length;
  const int64_t ndoc_idx = doc_idx.shape(0), nsizes = sizes.shape(0);
  auto* out = new std::vector<int32_t>(2 * (num_samples + 1));
  bool overrun = false;  // doc_idx holds fewer tokens than num_epochs * tokens_per_epoch
  {
    py::gil_scoped_release nogil;
    int32_t* o = out->data();
    int64_t d = 0;       // position in doc_idx
    int32_t offset = 0;  // token offset inside the current document
    o[0] = 0;
    o[1] = 0;
    for (int64_t s = 1; s <= num_samples && !overrun; ++s) {
      // a sample spans seq_length + 1 tokens; consecutive samples share one
      int32_t need = seq_length + 1;
      for (;;) {
        if (d >= ndoc_idx || doc_idx[d] < 0 || doc_idx[d] >= nsizes) {
          overrun = true;
          break;
        }
        const int32_t avail = sizes[doc_idx[d]] - offset;
        if (avail >= need) {
          offset += need - 1;
          break;
        }
        need -= avail;
        ++d;
        offset = 0;
      }
      o[2 * s] = static_cast<int32_t>(d);
      o[2 * s + 1] = offset;
    }
  }
  if (overrun) {
    delete out;
    throw std::invalid_argument(
        "build_sample_idx: doc_idx/sizes hold fewer tokens than num_epochs * tokens_per_epoch "
        "(or a doc id is out of range)");
  }
  return to_numpy(out, num_samples + 1, 2);
}

// ------------------------------------------------------------------ sentence packing
struct Rng32 {
  std::mt19937 gen;
  int32_t ratio;
  int32_t max_len;
  int32_t next_target() {
    if (ratio == 0) return max_len;
    const auto r = gen();
    if ((r % ratio) == 0) return 2 + r % (max_len - 1);
    return max_len;
  }
};

// Walk documents -> contiguous sentence spans.  `emit(first, last_exclusive,
// doc, block_id, target)` is called per sample.  BLOCKS selects the blocks
// variant (fixed per-document target, no short-sequence draws).
template <bool BLOCKS, typename Emit>
void pack_sentences(const py::detail::unchecked_reference<int64_t, 1>& docs,
                    const py::detail::unchecked_reference<int32_t, 1>& sizes,
                    const int32_t* title_sizes, int32_t num_epochs, uint64_t max_samples,
                    int32_t max_seq, int32_t min_sent, Rng32* rng, Emit&& emit) {
  const int64_t ndocs = docs.shape(0) - 1;
  uint64_t count = 0;
  for (int32_t epoch = 0; epoch < num_epochs; ++epoch) {
    if (count >= max_samples) break;
    int32_t block_id = 0;
    for (int64_t doc = 0; doc < ndocs; ++doc) {
      const int64_t first = docs[doc], last = docs[doc + 1];
      int64_t remain = last - first;
      bool has_long = false;
      if (remain >= (BLOCKS ? min_sent : 2)) {
        for (int64_t s = first; s < last; ++s)
          if (sizes[s] > kLongSentence) {
            has_long = true;
            break;
          }
      }
      if (remain < min_sent || has_long) continue;
      int32_t target = BLOCKS ? (max_seq - title_sizes[doc]) : rng->next_target();
      int64_t start = first;
      int32_t len = 0, nsent = 0;
      for (int64_t s = first; s < last; ++s) {
        len += sizes[s];
        ++nsent;
        --remain;
        const bool enough = BLOCKS ? (remain >= min_sent) : (remain > 1);
        if ((len >= target && enough && nsent >= min_sent) || remain == 0) {
          emit(start, s + 1, doc, block_id, target);
          ++count;
          ++block_id;
          start = s + 1;
          if (!BLOCKS) target = rng->next_target();
          len = 0;
          nsent = 0;
        }
      }
    }
  }
}

template <typename Idx>
void shuffle_rows(std::vector<Idx>& m, int width, int32_t seed) {
  const int64_t n = static_cast<int64_t>(m.size()) / width;
  std::mt19937_64 g(seed + 1);
  for (int64_t i = n - 1; i > 0; --i) {
    const int64_t j = static_cast<int64_t>(g() % (i + 1));
    for (int k = 0; k < width; ++k) std::swap(m[width * i + k], m[width * j + k]);
  }
}

template <typename Idx>
py::array build_mapping_t(const py::array_t<int64_t>& docs_, const py::array_t<int32_t>& sizes_,
                          int32_t num_epochs, uint64_t max_samples, int32_t max_seq,
                          double short_seq_prob, int32_t seed, int32_t min_sent) {
  auto docs = docs_.unchecked<1>();
  auto sizes = sizes_.unchecked<1>();
  Rng32 rng{std::mt19937(seed), short_seq_prob > 0 ? (int32_t)std::lround(1.0 / short_seq_prob) : 0,
            max_seq};
  auto* m = new std::vector<Idx>();
  {
    py::gil_scoped_release nogil;
    pack_sentences<false>(docs, sizes, nullptr, num_epochs, max_samples, max_seq, min_sent, &rng,
                          [&](int64_t a, int64_t b, int64_t, int32_t, int32_t t) {
                            m->push_back(static_cast<Idx>(a));
                            m->push_back(static_cast<Idx>(b));
                            m->push_back(static_cast<Idx>(t));
                          });
    shuffle_rows(*m, 3, seed);
  }
  const int64_t n = static_cast<int64_t>(m->size()) / 3;
  return to_numpy(m, n, 3);
}

py::array build_mapping(const py::array_t<int64_t>& docs, const py::array_t<int32_t>& sizes,
                        int32_t num_epochs, uint64_t max_samples, int32_t max_seq,
                        double short_seq_prob, int32_t seed, bool verbose, int32_t min_sent) {
  if (num_epochs <= 0 || max_seq <= 1 || short_seq_prob < 0 || short_seq_prob > 1 || seed <= 0)
    throw std::invalid_argument("build_mapping: bad arguments");
  (void)verbose;
  if (sizes.size() > std::numeric_limits<uint32_t>::max())
    return build_mapping_t<uint64_t>(docs, sizes, num_epochs, max_samples, max_seq, short_seq_prob,
                                     seed, min_sent);
  return build_mapping_t<uint32_t>(docs, sizes, num_epochs, max_samples, max_seq, short_seq_prob,
                                   seed, min_sent);
}

template <typename Idx>
py::array build_blocks_t(const py::array_t<int64_t>& docs_, const py::array_t<int32_t>& sizes_,
                         const py::array_t<int32_t>& titles_, int32_t num_epochs,
                         uint64_t max_samples, int32_t max_seq, int32_t seed, bool one_sent) {
  auto docs = docs_.unchecked<1>();
  auto sizes = sizes_.unchecked<1>();
  const int32_t* titles = titles_.data();
  auto* m = new std::vector<Idx>();
  {
    py::gil_scoped_release nogil;
    pack_sentences<true>(docs, sizes, titles, num_epochs, max_samples, max_seq, one_sent ? 1 : 2,
                         nullptr, [&](int64_t a, int64_t b, int64_t doc, int32_t blk, int32_t) {
                           m->push_back(static_cast<Idx>(a));
                           m->push_back(static_cast<Idx>(b));
                           m->push_back(static_cast<Idx>(doc));
                           m->push_back(static_cast<Idx>(blk));
                         });
    shuffle_rows(*m, 4, seed);
  }
  const int64_t n = static_cast<int64_t>(m->size()) / 4;
  return to_numpy(m, n, 4);
}

py::array build_blocks_mapping(const py::array_t<int64_t>& docs, const py::array_t<int32_t>& sizes,
                               const py::array_t<int32_t>& titles, int32_t num_epochs,
                               uint64_t max_samples, int32_t max_seq, int32_t seed, bool verbose,
                               bool use_one_sent_blocks) {
  if (num_epochs <= 0 || max_seq <= 1 || seed <= 0)
    throw std::invalid_argument("build_blocks_mapping: bad arguments");
  (void)verbose;
  if (sizes.size() > std::numeric_limits<uint32_t>::max())
    return build_blocks_t<uint64_t>(docs, sizes, titles, num_epochs, max_samples, max_seq, seed,
                                    use_one_sent_blocks);
  return build_blocks_t<uint32_t>(docs, sizes, titles, num_epochs, max_samples, max_seq, seed,
                                  use_one_sent_blocks);
}

// ------------------------------------------------------------------ bucket planner
// Greedy contiguous partition of parameter sizes into buckets of at most
// `cap` elements (a parameter never straddles buckets; oversize params get a
// bucket of their own).  Used by the RCCL gradient-bucketing layer (P02/P09).
std::vector<int64_t> plan_buckets(const std::vector<int64_t>& numels, int64_t cap) {
  std::vector<int64_t> bucket_of(numels.size());
  int64_t b = 0, fill = 0;
  for (size_t i = 0; i < numels.size(); ++i) {
    if (fill > 0 && fill + numels[i] > cap) {
      ++b;
      fill = 0;
    }
    bucket_of[i] = b;
    fill += numels[i];
  }
  return bucket_of;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "FleetX-AMD native host helpers";
  m.def("build_sample_idx", &build_sample_idx);
  m.def("build_mapping", &build_mapping);
  m.def("build_blocks_mapping", &build_blocks_mapping);
  m.def("build_blending_indices", &build_blending_indices);
  m.def("plan_buckets", &plan_buckets);
}
