// Minimal native HDF5 reader/writer for Keras-style model files.
//
// The reference persists models with `model.save(path.h5)` / `load_model`
// (AUTOENCODER-TensorFlow-IO-Kafka/cardata-v3.py:227,261) through h5py/libhdf5,
// neither of which exists on this platform.  This codec implements the subset of
// the HDF5 file format those files use (decoded from models/*.h5):
//   superblock v0/v1, version-1 object headers (+ continuation blocks),
//   "old-style" groups (symbol-table message -> v1 B-tree 'TREE' + local heap
//   'HEAP' + symbol nodes 'SNOD'), contiguous / compact datasets, attributes
//   (v1/v2/v3 messages) of numeric, fixed-length string and variable-length
//   string type (global heap 'GCOL').
// The writer emits exactly that layout (superblock v0, group leaf K 4, internal
// K 16), which is what h5py 2.x produced for the reference files.
#pragma once
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace sml {
namespace h5 {

struct Value {
  enum Kind { NUMERIC = 0, FIXED_STRING = 1, VLEN_STRING = 2 };
  Kind kind = NUMERIC;
  char dtype = 'f';            // 'f' float, 'i' signed int, 'u' unsigned int (NUMERIC)
  int itemsize = 4;            // bytes per element (NUMERIC / FIXED_STRING)
  std::vector<uint64_t> shape; // empty => scalar
  bool is_null = false;        // null dataspace
  std::string data;            // raw little-endian bytes (NUMERIC, FIXED_STRING)
  std::vector<std::string> strings;  // VLEN_STRING elements
  int str_pad = 1;             // fixed strings: 0 null-term, 1 null-pad, 2 space-pad
  int cset = 0;                // 0 ascii, 1 utf-8

  uint64_t count() const {
    uint64_t n = 1;
    for (auto d : shape) n *= d;
    return is_null ? 0 : n;
  }
};

struct Node {
  bool is_group = true;
  std::vector<std::pair<std::string, Value>> attrs;
  std::vector<std::pair<std::string, Node>> children;  // groups only
  Value value;                                          // datasets only
};

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

Node read_bytes(const std::string& bytes);
Node read_file(const std::string& path);
std::string write_bytes(const Node& root);
void write_file(const std::string& path, const Node& root);

}  // namespace h5
}  // namespace sml
