// gguf.cpp -- GGUF v2/v3 container parser (header, typed metadata, tensor
// infos, aligned data section), read through mmap so multi-GB models are
// never copied into host RAM before upload.
#include "gguf.h"

#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <stdexcept>

namespace mx {

namespace {
enum { T_UINT8, T_INT8, T_UINT16, T_INT16, T_UINT32, T_INT32, T_FLOAT32, T_BOOL, T_STRING, T_ARRAY, T_UINT64,
       T_INT64, T_FLOAT64 };

struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  void need(uint64_t n) {
    if ((uint64_t)(end - p) < n) throw std::runtime_error("GGUF: truncated file");
  }
  template <class T>
  T rd() {
    need(sizeof(T));
    T v;
    memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    uint64_t n = rd<uint64_t>();
    need(n);
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
};

double scalar(Cursor& c, int t) {
  switch (t) {
    case T_UINT8: return c.rd<uint8_t>();
    case T_INT8: return c.rd<int8_t>();
    case T_UINT16: return c.rd<uint16_t>();
    case T_INT16: return c.rd<int16_t>();
    case T_UINT32: return c.rd<uint32_t>();
    case T_INT32: return c.rd<int32_t>();
    case T_FLOAT32: return c.rd<float>();
    case T_BOOL: return c.rd<uint8_t>() ? 1.0 : 0.0;
    case T_UINT64: return (double)c.rd<uint64_t>();
    case T_INT64: return (double)c.rd<int64_t>();
    case T_FLOAT64: return c.rd<double>();
  }
  throw std::runtime_error("GGUF: bad scalar type " + std::to_string(t));
}

// bytes of n elements of a ggml type (n < 2^56 checked by the caller, so nothing here overflows);
// 0 for an unsupported type or a count that is not a whole number of blocks
uint64_t type_bytes(int type, uint64_t n) {
  uint64_t blk = 1, bb = 0;
  switch (type) {
    case 0: bb = 4; break;                   // F32
    case 1: bb = 2; break;                   // F16
    case 30: bb = 2; break;                  // BF16
    case 8: blk = 32, bb = 34; break;        // Q8_0
    case 2: blk = 32, bb = 18; break;        // Q4_0
    case 12: blk = 256, bb = 144; break;     // Q4_K
    case 13: blk = 256, bb = 176; break;     // Q5_K
    case 14: blk = 256, bb = 210; break;     // Q6_K
    default: return 0;
  }
  if (n % blk) return 0;
  return n / blk * bb;
}
}  // namespace

GGUFFile::~GGUFFile() {
  if (base_) munmap(base_, file_size);
  if (fd_ >= 0) close(fd_);
}

std::string GGUFFile::open(const std::string& path) {
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) return "cannot open " + path;
  struct stat st;
  if (fstat(fd_, &st) != 0) return "cannot stat " + path;
  file_size = (uint64_t)st.st_size;
  if (file_size < 24) return path + ": file too small for GGUF";
  void* m = mmap(nullptr, file_size, PROT_READ, MAP_SHARED, fd_, 0);
  if (m == MAP_FAILED) return "mmap failed for " + path;
  base_ = (uint8_t*)m;
  try {
    Cursor c{base_, base_ + file_size};
    if (memcmp(c.p, "GGUF", 4) != 0) return path + ": bad magic (not a GGUF file)";
    c.p += 4;
    uint32_t version = c.rd<uint32_t>();
    if (version != 2 && version != 3) return "unsupported GGUF version " + std::to_string(version);
    uint64_t n_t = c.rd<uint64_t>(), n_kv = c.rd<uint64_t>();
    for (uint64_t i = 0; i < n_kv; i++) {
      std::string key = c.str();
      GGUFValue v;
      v.type = (int)c.rd<uint32_t>();
      if (v.type == T_STRING) {
        v.str = c.str();
      } else if (v.type == T_ARRAY) {
        v.arr_type = (int)c.rd<uint32_t>();
        uint64_t n = c.rd<uint64_t>();
        // every element takes at least 1 byte (8 for a string's length): a count beyond what the
        // file holds is truncation, reported before any allocation of that size
        const uint64_t left = (uint64_t)(c.end - c.p);
        if (n > (v.arr_type == T_STRING ? left / 8 : left)) throw std::runtime_error("GGUF: truncated array " + key);
        if (v.arr_type == T_STRING) {
          v.arr_str.reserve(n);
          for (uint64_t j = 0; j < n; j++) v.arr_str.push_back(c.str());
        } else {
          v.arr_num.reserve(n);
          for (uint64_t j = 0; j < n; j++) v.arr_num.push_back(scalar(c, v.arr_type));
        }
      } else {
        v.num = scalar(c, v.type);
      }
      kv[key] = std::move(v);
    }
    std::vector<GGUFTensor> infos;
    for (uint64_t i = 0; i < n_t; i++) {
      GGUFTensor t;
      t.name = c.str();
      uint32_t nd = c.rd<uint32_t>();
      if (nd > 4) return "GGUF: tensor with >4 dims";
      uint64_t n = 1;
      for (uint32_t d = 0; d < nd; d++) {
        t.ne.push_back(c.rd<uint64_t>());
        if (__builtin_mul_overflow(n, t.ne.back(), &n) || n >= (1ull << 56))
          return "GGUF: tensor " + t.name + " has an element count that overflows";
      }
      t.type = (int)c.rd<uint32_t>();
      t.offset = c.rd<uint64_t>();
      t.nbytes = type_bytes(t.type, n);
      if (t.nbytes == 0 && n != 0)
        return "GGUF: tensor " + t.name + " has unsupported type " + std::to_string(t.type) +
               " (or a ragged block count)";
      infos.push_back(t);
    }
    const double al_num = get_num("general.alignment", 32);
    if (!(al_num >= 1 && al_num <= 65536)) return "GGUF: general.alignment out of range";
    const uint64_t al = (uint64_t)al_num;
    if (al & (al - 1)) return "GGUF: general.alignment " + std::to_string(al) + " is not a power of two";
    const uint64_t hdr = (uint64_t)(c.p - base_);
    const uint64_t data_start = (hdr + al - 1) / al * al;
    if (data_start > file_size) return "GGUF: data section starts past end of file";
    for (auto& t : infos) {
      // offset and size are checked against the bytes after data_start without forming sums that wrap
      const uint64_t room = file_size - data_start;
      if (t.offset > room || t.nbytes > room - t.offset)
        return "GGUF: tensor " + t.name + " extends past end of file";
      t.offset += data_start;
      tensors[t.name] = t;
    }
  } catch (const std::exception& e) {
    return e.what();
  }
  return "";
}

const GGUFValue* GGUFFile::get(const std::string& key) const {
  auto it = kv.find(key);
  return it == kv.end() ? nullptr : &it->second;
}

double GGUFFile::get_num(const std::string& key, double dflt) const {
  const GGUFValue* v = get(key);
  if (!v || v->type == T_STRING || v->type == T_ARRAY) return dflt;
  return v->num;
}

const GGUFTensor* GGUFFile::tensor(const std::string& name) const {
  auto it = tensors.find(name);
  return it == tensors.end() ? nullptr : &it->second;
}

}  // namespace mx
