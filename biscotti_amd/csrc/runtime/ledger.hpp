// Ledger: Update / BlockData / Block / Blockchain, with the reference's hash rule
//   Hash = SHA256(PrevBlockHash || decimal(Timestamp) || gob(BlockData))   (DistSys/block.go:23-28)
// gob(BlockData) is produced by a hand-written encoder of Go's encoding/gob wire format for
// exactly these types, as a fresh gob.Encoder emits them (DistSys/blockData.go:31-41): the four
// type-definition messages (BlockData=65, []float64=66, Update=67, [][]uint8=68, []Update=69)
// followed by the value message.
//
// Data model (DistSys/update.go:13-22, blockData.go:10-14, block.go:14-20):
//   Update    {SourceID int, Iteration int, Delta []float64, Commitment []byte,
//              Noise []float64, NoisedDelta []float64, Accepted bool, SignatureList [][]byte}
//   BlockData {Iteration int, GlobalW []float64, Deltas []Update}
//   Block     {Timestamp int64, Data BlockData, PrevBlockHash []byte, Hash []byte, StakeMap map[int]int}
#pragma once
#include <map>
#include <string>

#include "common.hpp"

namespace bsc {

struct Update {
  i64 source_id = 0;
  i64 iteration = 0;
  std::vector<double> delta;
  Bytes commitment;
  std::vector<double> noise;
  std::vector<double> noised_delta;
  bool accepted = false;
  std::vector<Bytes> signatures;
};

struct BlockData {
  i64 iteration = 0;
  std::vector<double> global_w;
  std::vector<Update> deltas;
};

struct Block {
  i64 timestamp = 0;
  BlockData data;
  Bytes prev_hash;
  Bytes hash;
  std::map<i64, i64> stake;
  void set_hash();
  Bytes compute_hash() const;
};

// gob encoding helpers (exposed for tests)
void gob_put_uint(Bytes& b, u64 x);
void gob_put_int(Bytes& b, i64 x);
void gob_put_float(Bytes& b, double f);
Bytes gob_encode_blockdata(const BlockData& d);

// Go fmt %v of a float64 (shortest repr, %g-style exponent rule) -- for PrintChain parity.
std::string go_format_float(double v);
std::string go_format_float_slice(const std::vector<double>& v);  // arrayToString (blockData.go)
std::string update_string(const Update& u);                        // Update.String()
std::string blockdata_string(const BlockData& d);                  // BlockData.String()

struct Blockchain {
  std::vector<Block> blocks;
  static Blockchain with_genesis(size_t num_features);
  static Block genesis(size_t num_features);
  // NewBlock semantics: timestamp 0 for empty blocks, else `now_unix` (block.go:30-44)
  Block make_block(const BlockData& d, const std::map<i64, i64>& stake, i64 now_unix) const;
  Block make_block(BlockData&& d, std::map<i64, i64>&& stake, i64 now_unix) const;   // no copies
  const Block& latest() const { return blocks.back(); }
  // getBlock(iteration) (blockchain.go:77-96): index iteration+1 if present
  const Block* get(i64 iteration) const;
  bool has(i64 iteration) const { return get(iteration) != nullptr; }
  void append(const Block& b);
  // evaluateBlockQuality (honest.go:631-647): same parent, non-empty, replacing an empty block
  bool better_block(const Block& b) const;
  // addBlock (honest.go:515-540): append / replace-if-better. Returns 0 appended, 1 replaced, -1 refused.
  int add_block(const Block& b);
  // chain validity: linkage + recomputed hashes
  bool verify(std::string* why = nullptr) const;
  bool verify_range(size_t from, size_t to, std::string* why = nullptr) const;
  std::string print_chain() const;  // PrintChain (blockchain.go:43-54)
  // Persistence: append-only file of length-prefixed records (checkpoint/resume).
  static Bytes serialize_block(const Block& b);
  static Block deserialize_block(const u8* p, size_t n, size_t* used);
  void save(const std::string& path) const;
  static Blockchain load(const std::string& path);
  static void append_to_file(const std::string& path, const Block& b);
};

}  // namespace bsc
