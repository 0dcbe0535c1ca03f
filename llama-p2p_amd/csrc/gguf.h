// gguf.h -- minimal GGUF v2/v3 parser (mmap) for the engine's model loader.
// Replaces the GGUF parse inside Llama(model_path=...) (/root/reference/llama_p2p_network.py:19;
// SURVEY.md §8a row a2).
#pragma once
#include <stdint.h>

#include <map>
#include <string>
#include <vector>

namespace mx {

struct GGUFValue {
  int type = -1;  // GGUF value type
  double num = 0;
  std::string str;
  std::vector<double> arr_num;
  std::vector<std::string> arr_str;
  int arr_type = -1;
};

struct GGUFTensor {
  std::string name;
  std::vector<uint64_t> ne;  // ne[0] fastest
  int type = 0;              // ggml type
  uint64_t offset = 0;       // absolute file offset
  uint64_t nbytes = 0;
};

class GGUFFile {
 public:
  ~GGUFFile();
  // returns empty string on success, else an error message
  std::string open(const std::string& path);
  const GGUFValue* get(const std::string& key) const;
  double get_num(const std::string& key, double dflt) const;
  const GGUFTensor* tensor(const std::string& name) const;
  const uint8_t* data(const GGUFTensor& t) const { return base_ + t.offset; }
  std::map<std::string, GGUFValue> kv;
  std::map<std::string, GGUFTensor> tensors;
  uint64_t file_size = 0;

 private:
  uint8_t* base_ = nullptr;
  int fd_ = -1;
};

}  // namespace mx
