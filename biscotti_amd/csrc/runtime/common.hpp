// Shared helpers for the Biscotti-AMD host runtime (C++17).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace bsc {

using u8 = uint8_t;
using u32 = uint32_t;
using u64 = uint64_t;
using i64 = int64_t;
using u128 = unsigned __int128;
using i128 = __int128;
using Bytes = std::vector<u8>;

inline Bytes to_bytes(const std::string& s) { return Bytes(s.begin(), s.end()); }

inline std::string hex(const u8* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; ++i) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}
inline std::string hex(const Bytes& b) { return hex(b.data(), b.size()); }

inline u64 load_be64(const u8* p) {
  u64 v = 0;
  for (int i = 0; i < 8; ++i) v = (v << 8) | p[i];
  return v;
}
inline void store_be64(u8* p, u64 v) {
  for (int i = 7; i >= 0; --i) { p[i] = u8(v); v >>= 8; }
}
inline u64 load_le64(const u8* p) {
  u64 v = 0;
  for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}
inline void store_le64(u8* p, u64 v) {
  for (int i = 0; i < 8; ++i) { p[i] = u8(v); v >>= 8; }
}

[[noreturn]] inline void fail(const std::string& m) { throw std::runtime_error(m); }

}  // namespace bsc
