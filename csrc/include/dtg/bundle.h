// TensorBundle (TF-1.x V2 checkpoint) I/O -- see csrc/ckpt/tensor_bundle.cc.
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace dtg {
namespace ckpt {

// TF DataType enum values used by BundleEntryProto
enum TfDType { DT_FLOAT = 1, DT_DOUBLE = 2, DT_INT32 = 3, DT_INT64 = 9, DT_BFLOAT16 = 14, DT_HALF = 19 };

struct Entry {
  int dtype = DT_FLOAT;
  std::vector<int64_t> shape;
  int shard_id = 0;
  int64_t offset = 0;
  int64_t size = 0;
  uint32_t crc32c = 0;  // masked
};

struct NamedTensor {
  std::string name;
  int dtype = DT_FLOAT;
  std::vector<int64_t> shape;
  std::string bytes;
};

uint32_t crc32c(const void* data, size_t n);
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
uint32_t crc_mask(uint32_t crc);
uint32_t crc_unmask(uint32_t masked);

std::string encode_entry(const Entry& e);
Entry decode_entry(const std::string& s);

void write_bundle(const std::string& prefix, const std::vector<NamedTensor>& tensors);
std::map<std::string, Entry> read_index(const std::string& prefix);
std::vector<NamedTensor> read_bundle(const std::string& prefix, bool verify_crc);

}  // namespace ckpt
}  // namespace dtg
