#include "ledger.hpp"

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>

#include "bn256.hpp"
#include "hash.hpp"

namespace bsc {

// ------------------------------------------------------------------ gob primitives
// uint: <128 -> one byte; otherwise negated byte count followed by big-endian bytes.
void gob_put_uint(Bytes& b, u64 x) {
  if (x < 128) { b.push_back(u8(x)); return; }
  u8 tmp[8];
  int n = 0;
  while (x) { tmp[n++] = u8(x); x >>= 8; }
  b.push_back(u8(256 - n));
  for (int i = n - 1; i >= 0; --i) b.push_back(tmp[i]);
}
void gob_put_int(Bytes& b, i64 x) {
  u64 u = x < 0 ? ((~u64(x)) << 1) | 1 : u64(x) << 1;
  gob_put_uint(b, u);
}
void gob_put_float(Bytes& b, double f) {
  u64 bits;
  memcpy(&bits, &f, 8);
  u64 rev = 0;
  for (int i = 0; i < 8; ++i) { rev = (rev << 8) | (bits & 0xff); bits >>= 8; }
  gob_put_uint(b, rev);
}
static void gob_put_string(Bytes& b, const std::string& s) {
  gob_put_uint(b, s.size());
  b.insert(b.end(), s.begin(), s.end());
}
static void gob_put_bytes(Bytes& b, const Bytes& s) {
  gob_put_uint(b, s.size());
  b.insert(b.end(), s.begin(), s.end());
}
static void gob_message(Bytes& out, const Bytes& payload) {
  gob_put_uint(out, payload.size());
  out.insert(out.end(), payload.begin(), payload.end());
}

// Predefined gob type ids.
enum : i64 { T_BOOL = 1, T_INT = 2, T_FLOAT = 4, T_BYTES = 5 };
// User type ids as a fresh process assigns them while building BlockData's type info.
enum : i64 { T_BLOCKDATA = 65, T_F64S = 66, T_UPDATE = 67, T_BYTESS = 68, T_UPDATES = 69 };

static void common_type(Bytes& p, const std::string& name, i64 id) {
  gob_put_uint(p, 1);  // CommonType.Name
  gob_put_string(p, name);
  gob_put_uint(p, 1);  // CommonType.Id
  gob_put_int(p, id);
  gob_put_uint(p, 0);
}

static Bytes struct_def(i64 id, const std::string& name,
                        const std::vector<std::pair<std::string, i64>>& fields) {
  Bytes p;
  gob_put_int(p, -id);
  gob_put_uint(p, 3);  // wireType.StructT (field index 2)
  gob_put_uint(p, 1);  // structType.CommonType
  common_type(p, name, id);
  gob_put_uint(p, 1);  // structType.Field
  gob_put_uint(p, fields.size());
  for (auto& f : fields) {
    gob_put_uint(p, 1);
    gob_put_string(p, f.first);
    gob_put_uint(p, 1);
    gob_put_int(p, f.second);
    gob_put_uint(p, 0);
  }
  gob_put_uint(p, 0);  // end structType
  gob_put_uint(p, 0);  // end wireType
  return p;
}

static Bytes slice_def(i64 id, const std::string& name, i64 elem) {
  Bytes p;
  gob_put_int(p, -id);
  gob_put_uint(p, 2);  // wireType.SliceT (field index 1)
  gob_put_uint(p, 1);  // sliceType.CommonType
  common_type(p, name, id);
  gob_put_uint(p, 1);  // sliceType.Elem
  gob_put_int(p, elem);
  gob_put_uint(p, 0);
  gob_put_uint(p, 0);
  return p;
}

static const Bytes& gob_type_prefix() {
  static const Bytes pre = [] {
    Bytes out;
    gob_message(out, struct_def(T_BLOCKDATA, "BlockData",
                                {{"Iteration", T_INT}, {"GlobalW", T_F64S}, {"Deltas", T_UPDATES}}));
    gob_message(out, slice_def(T_F64S, "[]float64", T_FLOAT));
    gob_message(out, slice_def(T_UPDATES, "[]main.Update", T_UPDATE));
    gob_message(out, struct_def(T_UPDATE, "Update",
                                {{"SourceID", T_INT},
                                 {"Iteration", T_INT},
                                 {"Delta", T_F64S},
                                 {"Commitment", T_BYTES},
                                 {"Noise", T_F64S},
                                 {"NoisedDelta", T_F64S},
                                 {"Accepted", T_BOOL},
                                 {"SignatureList", T_BYTESS}}));
    gob_message(out, slice_def(T_BYTESS, "[][]uint8", T_BYTES));
    return out;
  }();
  return pre;
}

// A float64 travels as the uint of its byte-reversed bits (gob_put_float); for a model vector that is
// ~9 bytes per value.  One reservation, raw writes: block hashing sits on the round's host path
// (each round's block is encoded to be hashed).
static inline u8* gob_uint_raw(u8* o, u64 x) {
  if (x < 128) {
    *o++ = u8(x);
    return o;
  }
  const int n = 8 - (__builtin_clzll(x) >> 3);   // bytes of x without leading zeros
  *o++ = u8(256 - n);
  // the n low bytes of x, big-endian, as ONE 8-byte store (the caller reserves 9 bytes per value,
  // so the bytes past the n valid ones land in space the next value overwrites or the final resize
  // drops)
  const u64 be = __builtin_bswap64(x << (8 * (8 - n)));
  memcpy(o, &be, 8);
  return o + n;
}

static void put_f64s(Bytes& p, const std::vector<double>& v) {
  gob_put_uint(p, v.size());
  const size_t at = p.size();
  p.resize(at + 9 * v.size());
  u8* o = p.data() + at;
  for (double x : v) {
    u64 bits;
    memcpy(&bits, &x, 8);
    o = gob_uint_raw(o, __builtin_bswap64(bits));
  }
  p.resize(size_t(o - p.data()));
}

static void encode_update(Bytes& p, const Update& u) {
  int last = -1;
  auto field = [&](int idx) { gob_put_uint(p, u64(idx - last)); last = idx; };
  if (u.source_id != 0) { field(0); gob_put_int(p, u.source_id); }
  if (u.iteration != 0) { field(1); gob_put_int(p, u.iteration); }
  if (!u.delta.empty()) { field(2); put_f64s(p, u.delta); }
  if (!u.commitment.empty()) { field(3); gob_put_bytes(p, u.commitment); }
  if (!u.noise.empty()) { field(4); put_f64s(p, u.noise); }
  if (!u.noised_delta.empty()) { field(5); put_f64s(p, u.noised_delta); }
  if (u.accepted) { field(6); gob_put_uint(p, 1); }
  if (!u.signatures.empty()) {
    field(7);
    gob_put_uint(p, u.signatures.size());
    for (auto& s : u.signatures) gob_put_bytes(p, s);
  }
  gob_put_uint(p, 0);
}

Bytes gob_encode_blockdata(const BlockData& d) {
  Bytes out = gob_type_prefix();
  Bytes p;
  size_t est = 16 + 9 * d.global_w.size();
  for (auto& u : d.deltas)
    est += 48 + u.commitment.size() + 9 * (u.delta.size() + u.noise.size() + u.noised_delta.size()) +
           80 * u.signatures.size();
  p.reserve(est);
  out.reserve(out.size() + est + 10);
  gob_put_int(p, T_BLOCKDATA);
  int last = -1;
  auto field = [&](int idx) { gob_put_uint(p, u64(idx - last)); last = idx; };
  if (d.iteration != 0) { field(0); gob_put_int(p, d.iteration); }
  if (!d.global_w.empty()) { field(1); put_f64s(p, d.global_w); }
  if (!d.deltas.empty()) {
    field(2);
    gob_put_uint(p, d.deltas.size());
    for (auto& u : d.deltas) encode_update(p, u);
  }
  gob_put_uint(p, 0);
  gob_message(out, p);
  return out;
}

// bytes put_f64s writes for the values of v (the count excluded)
static size_t f64s_payload_len(const std::vector<double>& v) {
  size_t n = 0;
  for (double x : v) {
    u64 bits;
    memcpy(&bits, &x, 8);
    const u64 r = __builtin_bswap64(bits);
    n += r < 128 ? 1 : size_t(9 - (__builtin_clzll(r) >> 3));
  }
  return n;
}

// ------------------------------------------------------------------ Block
// sha256(prev_hash || timestamp || gob(data)) -- the same bytes as hashing gob_encode_blockdata(data), but
// the ~70 KB of GlobalW values are encoded straight into the hash in L1-sized pieces (no message buffer):
// the gob message's length prefix comes from a length pass over the values.  The block hash sits on the
// round's host path between the recovery's read-back and the next round's speculative launch.
Bytes Block::compute_hash() const {
  Sha256 s;
  s.update(prev_hash);
  std::string ts = std::to_string(timestamp);
  s.update(reinterpret_cast<const u8*>(ts.data()), ts.size());
  const BlockData& d = data;
  Bytes head, tail;   // the message payload = head | GlobalW values | tail
  head.reserve(32);
  int last = -1;
  auto field = [&](Bytes& p, int idx) { gob_put_uint(p, u64(idx - last)); last = idx; };
  gob_put_int(head, T_BLOCKDATA);
  if (d.iteration != 0) { field(head, 0); gob_put_int(head, d.iteration); }
  size_t wlen = 0;
  if (!d.global_w.empty()) {
    field(head, 1);
    gob_put_uint(head, d.global_w.size());
    wlen = f64s_payload_len(d.global_w);
  }
  if (!d.deltas.empty()) {
    field(tail, 2);
    gob_put_uint(tail, d.deltas.size());
    for (auto& u : d.deltas) encode_update(tail, u);
  }
  gob_put_uint(tail, 0);
  s.update(gob_type_prefix());
  Bytes len;
  gob_put_uint(len, head.size() + wlen + tail.size());
  s.update(len);
  s.update(head);
  constexpr size_t CH = 448;   // values per piece: <= 448 * 9 bytes, plus the 8-byte store's slack
  u8 buf[CH * 9 + 8];
  const size_t nw = d.global_w.size();
  for (size_t i = 0; i < nw; i += CH) {
    u8* o = buf;
    const size_t e = std::min(nw, i + CH);
    for (size_t k = i; k < e; ++k) {
      u64 bits;
      memcpy(&bits, &d.global_w[k], 8);
      o = gob_uint_raw(o, __builtin_bswap64(bits));
    }
    s.update(buf, size_t(o - buf));
  }
  s.update(tail);
  Bytes out(32);
  s.final(out.data());
  return out;
}
void Block::set_hash() { hash = compute_hash(); }

// ------------------------------------------------------------------ Go float formatting
std::string go_format_float(double v) {
  if (std::isnan(v)) return "NaN";
  if (std::isinf(v)) return v > 0 ? "+Inf" : "-Inf";
  if (v == 0) return std::signbit(v) ? "-0" : "0";
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  std::string s(buf, res.ptr);
  bool neg = s[0] == '-';
  if (neg) s = s.substr(1);
  size_t e = s.find('e');
  std::string mant = s.substr(0, e);
  int exp = std::stoi(s.substr(e + 1));
  std::string digs;
  for (char c : mant) if (c != '.') digs.push_back(c);
  while (digs.size() > 1 && digs.back() == '0') digs.pop_back();
  std::string out = neg ? "-" : "";
  // strconv 'g' with shortest digits: exponent form iff exp < -4 || exp >= 6 (eprec = 6).
  if (exp < -4 || exp >= 6) {
    out += digs[0];
    if (digs.size() > 1) { out += '.'; out += digs.substr(1); }
    out += 'e';
    out += exp < 0 ? '-' : '+';
    int ae = std::abs(exp);
    if (ae < 10) out += '0';
    out += std::to_string(ae);
    return out;
  }
  // %f style with exactly the shortest digits
  int dp = exp + 1;  // digits before the decimal point
  if (dp <= 0) {
    out += "0.";
    out += std::string(-dp, '0');
    out += digs;
  } else if (dp >= int(digs.size())) {
    out += digs;
    out += std::string(dp - digs.size(), '0');
  } else {
    out += digs.substr(0, dp);
    out += '.';
    out += digs.substr(dp);
  }
  return out;
}

std::string go_format_float_slice(const std::vector<double>& v) {
  std::string s = "[";
  for (size_t i = 0; i < v.size(); ++i) {
    if (i) s += ",";
    s += go_format_float(v[i]);
  }
  s += "]";
  return s;
}

static std::string gfp_hex(const U256& x) {
  char b[80];
  snprintf(b, sizeof(b), "%16.16llx%16.16llx%16.16llx%16.16llx", (unsigned long long)x.w[3],
           (unsigned long long)x.w[2], (unsigned long long)x.w[1], (unsigned long long)x.w[0]);
  return b;
}

std::string update_string(const Update& u) {
  std::string pt;
  U256 x, y;
  bool inf = true;
  if (u.commitment.size() >= 64) {
    x = Fp().reduce(U256::from_be(u.commitment.data()));
    y = Fp().reduce(U256::from_be(u.commitment.data() + 32));
    inf = x.is_zero() && y.is_zero();
  }
  if (inf) { x = U256(); y = U256::from_u64(1); }
  pt = "bn256.G1:(" + gfp_hex(x) + ", " + gfp_hex(y) + ")";
  return "{Iteration:" + std::to_string(u.iteration) + ", " + "Commitment:" + pt + ", " +
         "Deltas:" + go_format_float_slice(u.delta) + "}";
}

std::string blockdata_string(const BlockData& d) {
  std::string ups = "[";
  for (size_t i = 0; i < d.deltas.size(); ++i) {
    ups += update_string(d.deltas[i]);
    if (i + 1 != d.deltas.size()) ups += " ,";
  }
  ups += "]";
  return "Iteration: " + std::to_string(d.iteration) + ", GlobalW: " + go_format_float_slice(d.global_w) +
         ", deltas: " + ups;
}

// ------------------------------------------------------------------ Blockchain
Block Blockchain::genesis(size_t nf) {
  Block b;
  b.timestamp = 0;
  b.data.iteration = -1;
  b.data.global_w.assign(nf, 0.0);
  b.set_hash();
  return b;
}
Blockchain Blockchain::with_genesis(size_t nf) {
  Blockchain c;
  c.blocks.push_back(genesis(nf));
  return c;
}
Block Blockchain::make_block(const BlockData& d, const std::map<i64, i64>& stake, i64 now_unix) const {
  return make_block(BlockData(d), std::map<i64, i64>(stake), now_unix);
}
Block Blockchain::make_block(BlockData&& d, std::map<i64, i64>&& stake, i64 now_unix) const {
  Block b;
  b.timestamp = d.deltas.empty() ? 0 : now_unix;
  b.data = std::move(d);
  b.prev_hash = latest().hash;
  b.stake = std::move(stake);
  b.set_hash();
  return b;
}
const Block* Blockchain::get(i64 it) const {
  if (i64(blocks.size()) >= it + 2 && it + 1 >= 0) {
    const Block& b = blocks[size_t(it + 1)];
    if (b.data.iteration != it) fail("ledger: blocks for multiple iterations appended");
    return &b;
  }
  return nullptr;
}
void Blockchain::append(const Block& b) { blocks.push_back(b); }
bool Blockchain::better_block(const Block& b) const {
  const Block* mine = get(b.data.iteration);
  const Block* prev = get(b.data.iteration - 1);
  if (!mine || !prev) return false;
  if (b.prev_hash != prev->hash) return false;
  if (b.data.deltas.empty() || !mine->data.deltas.empty()) return false;
  return true;
}
int Blockchain::add_block(const Block& b) {
  if (get(b.data.iteration) != nullptr) {
    if (!better_block(b)) return -1;
    blocks[size_t(b.data.iteration + 1)] = b;
    return 1;
  }
  append(b);
  return 0;
}
bool Blockchain::verify(std::string* why) const { return verify_range(0, blocks.size(), why); }

// blocks [from, to): re-hash each one (SHA-256 over prev || timestamp || gob(BlockData)) and check its
// link to the block before it -- what a rejoining peer checks on the chain it adopts
bool Blockchain::verify_range(size_t from, size_t to, std::string* why) const {
  to = std::min(to, blocks.size());
  for (size_t i = from; i < to; ++i) {
    const Block& b = blocks[i];
    if (b.compute_hash() != b.hash) {
      if (why) *why = "hash mismatch at index " + std::to_string(i);
      return false;
    }
    if (i > 0 && b.prev_hash != blocks[i - 1].hash) {
      if (why) *why = "broken link at index " + std::to_string(i);
      return false;
    }
    if (b.data.iteration != i64(i) - 1) {
      if (why) *why = "iteration mismatch at index " + std::to_string(i);
      return false;
    }
  }
  return true;
}
std::string Blockchain::print_chain() const {
  std::string s;
  for (auto& b : blocks) {
    s += "Prev. hash: " + hex(b.prev_hash) + "\n";
    s += "Data: " + blockdata_string(b.data) + "\n";
    s += "Hash: " + hex(b.hash) + "\n\n";
  }
  return s;
}

// ------------------------------------------------------------------ persistence
namespace {
void put_u64(Bytes& b, u64 v) { u8 t[8]; store_le64(t, v); b.insert(b.end(), t, t + 8); }
void put_blob(Bytes& b, const Bytes& v) { put_u64(b, v.size()); b.insert(b.end(), v.begin(), v.end()); }
void put_f64s_raw(Bytes& b, const std::vector<double>& v) {
  put_u64(b, v.size());
  size_t o = b.size();
  b.resize(o + 8 * v.size());
  if (!v.empty()) memcpy(b.data() + o, v.data(), 8 * v.size());
}
struct Reader {
  const u8* p; size_t n, o = 0;
  u64 u() { if (o + 8 > n) fail("chain file: truncated"); u64 v = load_le64(p + o); o += 8; return v; }
  Bytes blob() { u64 k = u(); if (o + k > n) fail("chain file: truncated"); Bytes b(p + o, p + o + k); o += k; return b; }
  std::vector<double> f64s() {
    u64 k = u();
    if (o + 8 * k > n) fail("chain file: truncated");
    std::vector<double> v(k);
    if (k) memcpy(v.data(), p + o, 8 * k);
    o += 8 * k;
    return v;
  }
};
const char MAGIC[8] = {'B', 'S', 'C', 'C', 'H', 'N', '0', '1'};
}  // namespace

Bytes Blockchain::serialize_block(const Block& b) {
  Bytes r;
  put_u64(r, u64(b.timestamp));
  put_blob(r, b.prev_hash);
  put_blob(r, b.hash);
  put_u64(r, b.stake.size());
  for (auto& kv : b.stake) { put_u64(r, u64(kv.first)); put_u64(r, u64(kv.second)); }
  put_u64(r, u64(b.data.iteration));
  put_f64s_raw(r, b.data.global_w);
  put_u64(r, b.data.deltas.size());
  for (auto& u : b.data.deltas) {
    put_u64(r, u64(u.source_id));
    put_u64(r, u64(u.iteration));
    put_f64s_raw(r, u.delta);
    put_blob(r, u.commitment);
    put_f64s_raw(r, u.noise);
    put_f64s_raw(r, u.noised_delta);
    put_u64(r, u.accepted ? 1 : 0);
    put_u64(r, u.signatures.size());
    for (auto& s : u.signatures) put_blob(r, s);
  }
  Bytes framed;
  put_u64(framed, r.size());
  framed.insert(framed.end(), r.begin(), r.end());
  return framed;
}

Block Blockchain::deserialize_block(const u8* p, size_t n, size_t* used) {
  Reader hdr{p, n};
  u64 len = hdr.u();
  if (8 + len > n) fail("chain file: truncated record");
  Reader r{p + 8, size_t(len)};
  Block b;
  b.timestamp = i64(r.u());
  b.prev_hash = r.blob();
  b.hash = r.blob();
  u64 ns = r.u();
  for (u64 i = 0; i < ns; ++i) { i64 k = i64(r.u()); b.stake[k] = i64(r.u()); }
  b.data.iteration = i64(r.u());
  b.data.global_w = r.f64s();
  u64 nd = r.u();
  for (u64 i = 0; i < nd; ++i) {
    Update u;
    u.source_id = i64(r.u());
    u.iteration = i64(r.u());
    u.delta = r.f64s();
    u.commitment = r.blob();
    u.noise = r.f64s();
    u.noised_delta = r.f64s();
    u.accepted = r.u() != 0;
    u64 nsg = r.u();
    for (u64 j = 0; j < nsg; ++j) u.signatures.push_back(r.blob());
    b.data.deltas.push_back(std::move(u));
  }
  if (used) *used = 8 + len;
  return b;
}

void Blockchain::save(const std::string& path) const {
  std::ofstream f(path, std::ios::binary | std::ios::trunc);
  if (!f) fail("cannot open " + path);
  f.write(MAGIC, 8);
  for (auto& b : blocks) {
    Bytes r = serialize_block(b);
    f.write(reinterpret_cast<const char*>(r.data()), std::streamsize(r.size()));
  }
}

void Blockchain::append_to_file(const std::string& path, const Block& b) {
  std::ifstream probe(path, std::ios::binary);
  bool exists = bool(probe);
  probe.close();
  std::ofstream f(path, std::ios::binary | std::ios::app);
  if (!f) fail("cannot open " + path);
  if (!exists) f.write(MAGIC, 8);
  Bytes r = serialize_block(b);
  f.write(reinterpret_cast<const char*>(r.data()), std::streamsize(r.size()));
  f.flush();
}

Blockchain Blockchain::load(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) fail("cannot open " + path);
  Bytes all((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  if (all.size() < 8 || memcmp(all.data(), MAGIC, 8) != 0) fail("chain file: bad magic");
  Blockchain c;
  size_t o = 8;
  while (o < all.size()) {
    // a process killed mid-append leaves a torn final record (length prefix or body cut short):
    // the chain up to it is intact, resume from there (the next save/append rewrites the tail)
    const size_t rest = all.size() - o;
    if (rest < 8 || load_le64(all.data() + o) > rest - 8) break;
    size_t used = 0;
    c.blocks.push_back(deserialize_block(all.data() + o, all.size() - o, &used));
    o += used;
  }
  std::string why;
  if (!c.verify(&why)) fail("chain file failed verification: " + why);
  return c;
}

}  // namespace bsc
