#include "keys.hpp"

#include <fstream>

#include "hash.hpp"

namespace bsc {

static const char* B64 = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

std::string base64_encode(const Bytes& b) {
  std::string s;
  size_t i = 0;
  for (; i + 2 < b.size(); i += 3) {
    u32 v = (u32(b[i]) << 16) | (u32(b[i + 1]) << 8) | b[i + 2];
    s += B64[v >> 18]; s += B64[(v >> 12) & 63]; s += B64[(v >> 6) & 63]; s += B64[v & 63];
  }
  if (i + 1 == b.size()) {
    u32 v = u32(b[i]) << 16;
    s += B64[v >> 18]; s += B64[(v >> 12) & 63]; s += "==";
  } else if (i + 2 == b.size()) {
    u32 v = (u32(b[i]) << 16) | (u32(b[i + 1]) << 8);
    s += B64[v >> 18]; s += B64[(v >> 12) & 63]; s += B64[(v >> 6) & 63]; s += '=';
  }
  return s;
}

Bytes base64_decode(const std::string& s) {
  int rev[256];
  for (int& r : rev) r = -1;
  for (int i = 0; i < 64; ++i) rev[u8(B64[i])] = i;
  Bytes out;
  u32 acc = 0;
  int bits = 0;
  for (char c : s) {
    if (c == '=' || c == '\n' || c == '\r' || c == ' ') continue;
    int v = rev[u8(c)];
    if (v < 0) fail("base64: invalid character");
    acc = (acc << 6) | u32(v);
    bits += 6;
    if (bits >= 8) { bits -= 8; out.push_back(u8(acc >> bits)); }
  }
  return out;
}

std::string key_record_json(const KeyRecord& r) {
  return "{\"Id\":" + std::to_string(r.id) + ",\"Pkey\":\"" + base64_encode(r.pkey) + "\",\"Skey\":\"" +
         base64_encode(r.skey) + "\"}";
}

static std::string json_field(const std::string& line, const std::string& key, bool quoted) {
  std::string pat = "\"" + key + "\"";
  size_t p = line.find(pat);
  if (p == std::string::npos) fail("json: missing field " + key);
  p = line.find(':', p + pat.size());
  if (p == std::string::npos) fail("json: malformed field " + key);
  ++p;
  while (p < line.size() && (line[p] == ' ' || line[p] == '\t')) ++p;
  if (quoted) {
    if (line.compare(p, 4, "null") == 0) return "";
    if (line[p] != '"') fail("json: expected string for " + key);
    size_t e = line.find('"', p + 1);
    return line.substr(p + 1, e - p - 1);
  }
  size_t e = p;
  while (e < line.size() && (isdigit(u8(line[e])) || line[e] == '-')) ++e;
  return line.substr(p, e - p);
}

KeyRecord parse_key_record(const std::string& line) {
  KeyRecord r;
  r.id = std::stoll(json_field(line, "Id", false));
  r.pkey = base64_decode(json_field(line, "Pkey", true));
  r.skey = base64_decode(json_field(line, "Skey", true));
  return r;
}

std::vector<G1> gen_commit_key_g1(size_t d, const Scalar& s) {
  std::vector<G1> pk(d);
  G1 cur = G1::generator();
  for (size_t i = 0; i < d; ++i) {
    U256 ax, ay;
    cur.to_affine(ax, ay);
    pk[i] = G1::from_affine_mont(ax, ay);
    cur = pk[i].mul(s.v);
  }
  return pk;
}

std::vector<G2> gen_commit_key_g2(size_t d, const Scalar& s) {
  std::vector<G2> pk(d);
  G2 cur = G2::generator();
  for (size_t i = 0; i < d; ++i) {
    pk[i] = cur;
    cur = cur.mul(s.v);
    // keep coordinates small: renormalise to z = 1
    Fp2 ax, ay;
    cur.to_affine(ax, ay);
    if (!cur.is_inf()) { cur.x = ax; cur.y = ay; cur.z = Fp2::one(); }
  }
  return pk;
}

void write_commit_key(const std::string& path, size_t d, const Scalar& s) {
  auto g1 = gen_commit_key_g1(d, s);
  auto g2 = gen_commit_key_g2(d, s);
  std::ofstream f(path, std::ios::trunc);
  if (!f) fail("cannot open " + path);
  for (size_t i = 0; i < d; ++i) {
    KeyRecord r{i64(i), g1[i].marshal(), g2[i].marshal()};
    f << key_record_json(r) << "\n";
  }
}

std::vector<G1> read_commit_key(const std::string& path, size_t d, bool check_g2) {
  std::ifstream f(path);
  if (!f) fail("cannot open " + path);
  std::vector<G1> pk(d, G1::infinity());
  std::vector<bool> seen(d, false);
  std::string line;
  while (std::getline(f, line)) {
    if (line.find_first_not_of(" \r\n\t") == std::string::npos) continue;
    KeyRecord r = parse_key_record(line);
    if (r.id < 0 || size_t(r.id) >= d) continue;  // keys beyond d are ignored
    pk[size_t(r.id)] = G1::unmarshal(r.pkey);
    if (check_g2) (void)G2::unmarshal(r.skey);
    seen[size_t(r.id)] = true;
  }
  for (size_t i = 0; i < d; ++i)
    if (!seen[i]) fail("commit key file lacks id " + std::to_string(i));
  return pk;
}

std::pair<Scalar, G1> client_key_from_entropy(const Bytes& entropy) {
  Blake2Xb x(entropy);
  Scalar sk = pick_scalar_from_xof(x);
  G1 pk = gen_table().mul(sk.v);
  return {sk, pk};
}

void write_client_keys(const std::string& path, const std::vector<std::pair<Scalar, G1>>& keys) {
  std::ofstream f(path, std::ios::trunc);
  if (!f) fail("cannot open " + path);
  for (size_t i = 0; i < keys.size(); ++i) {
    KeyRecord r{i64(i), keys[i].second.marshal(), keys[i].first.to_be()};
    f << key_record_json(r) << "\n";
  }
}

std::vector<std::pair<Scalar, G1>> read_client_keys(const std::string& path) {
  std::ifstream f(path);
  if (!f) fail("cannot open " + path);
  std::vector<std::pair<Scalar, G1>> out;
  std::string line;
  while (std::getline(f, line)) {
    if (line.find_first_not_of(" \r\n\t") == std::string::npos) continue;
    KeyRecord r = parse_key_record(line);
    if (size_t(r.id) >= out.size()) out.resize(static_cast<size_t>(r.id) + 1);
    out[size_t(r.id)] = {Scalar::from_be(r.skey), G1::unmarshal(r.pkey)};
  }
  return out;
}

}  // namespace bsc
