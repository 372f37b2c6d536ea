// Key material and the reference's bootstrap file formats.
//
//   commitKey.json : JSON lines {"Id":i,"Pkey":base64(G1 64B),"Skey":base64(G2 129B)}, i < d
//                    PK_G1[i] = s^i * G1, PK_G2[i] = s^i * G2 with the hard-coded s = 2
//                    (DistSys/publicKey.go:26-61, keyGeneration/generateBootstrapFile.go:102-133)
//   pKeyG1.json    : JSON lines {"Id":i,"Pkey":base64(G1 64B),"Skey":base64(scalar 32B BE)}
//                    (generateBootstrapFile.go:141-191, publicKey.go:81-99)
//   peersfile.txt  : one IP:port per line; the line index is the peer id
//
// Go's encoding/json writes []byte as standard base64 with padding, fields in struct order,
// one object per line (json.Encoder.Encode appends '\n').
#pragma once
#include <string>

#include "bn256.hpp"

namespace bsc {

std::string base64_encode(const Bytes& b);
Bytes base64_decode(const std::string& s);

struct KeyRecord {
  i64 id = 0;
  Bytes pkey;
  Bytes skey;
};
std::string key_record_json(const KeyRecord& r);
KeyRecord parse_key_record(const std::string& line);  // tolerant of whitespace / field order

// commit key generation: PK_G1[i] = s^i G1 (and G2 if with_g2)
std::vector<G1> gen_commit_key_g1(size_t d, const Scalar& s);
std::vector<G2> gen_commit_key_g2(size_t d, const Scalar& s);
void write_commit_key(const std::string& path, size_t d, const Scalar& s);
// returns G1 commit key from commitKey.json (G2 parts are validated but only G1 is returned)
std::vector<G1> read_commit_key(const std::string& path, size_t d, bool check_g2);

// client keys: sk derived from `entropy` (32 B) with the kyber Pick rule; pk = sk*G1
std::pair<Scalar, G1> client_key_from_entropy(const Bytes& entropy);
void write_client_keys(const std::string& path, const std::vector<std::pair<Scalar, G1>>& keys);
std::vector<std::pair<Scalar, G1>> read_client_keys(const std::string& path);

}  // namespace bsc
