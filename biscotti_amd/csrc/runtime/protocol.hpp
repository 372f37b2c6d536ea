// Biscotti round protocol: configuration, committee lottery and the per-round state machine.
//
// The reference runs one Go process per peer whose goroutines race over TCP RPCs
// (DistSys/main.go).  Here the decision logic of a round is a deterministic state machine that
// every rank replicates; data movement between phases is done by the Python driver with device
// kernels and torch.distributed collectives.  Network races of the reference ("first N arrivals")
// are modelled by a seeded arrival order, timeouts by liveness masks with the same
// empty-block semantics.
//
//   flags/derived sizes      DistSys/main.go:613-684, 825
//   roles lottery            DistSys/vrf.go:54-182, main.go:497-565
//   krum threshold/accept    DistSys/krum.go:100-166,227-365 ; ML/Pytorch/client_obj.py:114-143
//   signature quorum         DistSys/main.go:1686   (>= nv/2, integer division)
//   share partition quirk    DistSys/main.go:1875-1931 (miner index advances only on success)
//   miner threshold          DistSys/main.go:360     (NUM_SAMPLES/2)
//   leader + quorum          DistSys/main.go:2027-2045, 2072-2142, 2237-2277
//   block creation / stake   DistSys/honest.go:346-440
//   FedSys                   FedSys/main.go:27-48,192-375 ; FedSys/honest.go:130-163,311-337
#pragma once
#include <map>
#include <set>
#include <string>

#include "ledger.hpp"

namespace bsc {

struct ProtocolConfig {
  i64 num_nodes = 0;
  i64 num_verifiers = 3;   // -nv
  i64 num_miners = 3;      // -na
  i64 num_noisers = 2;     // -nn
  bool secure_agg = true;  // -sa
  bool noising = true;     // -np
  bool verification = true;  // -vp
  double epsilon = 2.0;    // -ep
  double poisoning = 0.0;  // -po
  i64 perc_samples = 70;   // -ns
  bool rand_sample = false;  // -rs
  i64 colluders = 0;       // -c (percent)
  std::string defense = "KRUM";
  i64 poly_size = 10;
  i64 precision = 4;
  i64 max_iterations = 100;
  i64 default_stake = 10;
  i64 stake_unit = 5;
  u64 seed = 0;            // arrival-order / sampling seed
  bool shared_inbox = false;  // every verifier sees the same inbox (round-1 model; the reference's
  //                             verifiers each keep their own first-arrivals list)
  bool miner_cap = true;   // leader fires at NUM_SAMPLES/2 shares (main.go:360): block = first arrivals
  i64 miner_block_div = 0;  // 0: the NUM_SAMPLES/2 rule (main.go:360); k > 0: the leader fires at num_nodes / k
  //                           shares, at least 2 (minBlockSize, main.go:348-352 with k = 8)
  // derived (call derive())
  i64 num_samples = 0, krum_thresh = 0, total_shares = 0, shares_per_miner = 0;
  i64 miner_share_thresh = 0, poisoning_index = 0, collusion_thresh = 0;
  void derive();
};

// Stake lottery over 2-byte windows of `input`, SHA-256 re-hash when exhausted (vrf.go).
// The reference materialises one ticket per stake unit (its list grows by 5 per contribution
// every round); the same draw is an upper_bound over stake prefix sums: O(n) memory, O(log n).
struct Lottery {
  std::vector<i64> ids, cum;  // holders with stake > 0 (ascending id) and inclusive prefix sums
  Bytes input;
  size_t i = 0;
  Lottery(const std::map<i64, i64>& stake, i64 total_nodes, const Bytes& in);
  i64 total() const { return cum.empty() ? 0 : cum.back(); }
  i64 ticket(i64 idx) const;  // owner of ticket #idx in the reference's list order
  i64 draw();
};
void select_roles(const std::map<i64, i64>& stake, const Bytes& block_hash, i64 nv, i64 na, i64 n,
                  std::vector<i64>* verifiers, std::vector<i64>* miners);
std::vector<i64> select_noisers(const std::map<i64, i64>& stake, const Bytes& vrf_output, i64 source_id,
                                i64 nn, i64 n);
// the same draw from a prebuilt ticket table (`table`'s input is ignored): a batch over every worker
// builds the stake prefix sums once instead of once per worker
std::vector<i64> select_noisers(const Lottery& table, const Bytes& vrf_output, i64 source_id, i64 nn);

// Multi-Krum (client_obj.py:114-143) -- host reference; X is row-major [n, d] float64.
std::vector<double> krum_scores(const double* X, i64 n, i64 d, i64 groupsize);
std::vector<i64> krum_select(const std::vector<double>& scores, i64 n_accept);

u64 splitmix64(u64& s);
std::vector<i64> seeded_permutation(i64 n, u64 seed);

struct RoundPlan {
  i64 iteration = -1;
  std::vector<i64> verifiers, miners, workers;
  i64 leader = -1;
  std::vector<u8> live;  // [num_nodes]
  bool done = false;     // MAX_ITERATIONS reached
};

class RoundFSM {
 public:
  ProtocolConfig cfg;
  Blockchain chain;
  std::map<i64, i64> stake;
  i64 iteration = -1;
  RoundPlan plan;
  std::vector<std::string> addresses;  // peer table (IP:port) for sort-order rules

  RoundFSM(const ProtocolConfig& c, i64 num_features);
  // prepareForNextIteration: roles from the latest block hash + stake
  const RoundPlan& begin_round(const std::vector<u8>& live);
  // The updates each online verifier collects: first krum_thresh arrivals (seeded order),
  // sorted by SourceID, optional random sampling (krum.go:296-312,368-388).
  std::vector<i64> verifier_inbox(const std::vector<i64>& submitted) const;
  // Every verifier's own inbox (plan.verifiers order): each verifier receives the updates in its own
  // seeded arrival order and keeps the first krum_thresh (krum.go:284-322 runs per verifier process).
  std::vector<std::vector<i64>> verifier_inboxes(const std::vector<i64>& submitted) const;
  // Arrival order of the workers' shares / updates at the leader miner (a permutation of
  // plan.workers); the leader builds its block from the first miner_share_thresh approved ones.
  std::vector<i64> leader_arrivals() const;
  // approved workers the leader's block can carry: the first miner_share_thresh in leader arrival
  // order (all of them when miner_cap is off), returned sorted
  std::vector<i64> leader_cap(const std::vector<i64>& candidates) const;
  i64 leader_cap_size() const;  // 0: no cap
  i64 krum_clip(i64 n) const { return i64(0.5 * double(n)); }
  // accepted[v] = SourceIDs verifier v accepted; returns approved workers (>= nv/2 signatures)
  std::vector<i64> approve(const std::map<i64, std::vector<i64>>& accepted, bool* verifiers_online) const;
  // Share routing: for each approved worker, part index each online miner receives.
  // Returns map miner -> list of (worker, part_index).
  std::map<i64, std::vector<std::pair<i64, i64>>> route_shares(const std::vector<i64>& approved) const;
  // Leader's view: node list (intersection over responding miners) and which miners' aggregated
  // parts are available; quorum per main.go:2079.
  struct LeaderView {
    bool leader_online = false;
    bool quorum = false;
    std::vector<i64> node_list;            // sorted
    std::vector<i64> contributing_miners;  // leader first, then responders
  };
  LeaderView leader_view(const std::map<i64, std::vector<std::pair<i64, i64>>>& routes) const;
  // Non-secure-agg path: miner each approved worker reaches (first online in seeded order).
  std::map<i64, std::vector<i64>> route_updates(const std::vector<i64>& approved) const;
  // Block creation.  Secure-agg: deltas = [{Iteration, Commitment, Accepted}] per node, +stake.
  Block make_secagg_block(const std::vector<double>& new_w, const std::vector<i64>& node_list,
                          const std::vector<Bytes>& commitments, i64 now_unix);
  // the same from a raw model pointer (the pinned read-back of the recovery): one copy of W, into the block
  Block make_secagg_block(const double* new_w, size_t n, const std::vector<i64>& node_list,
                          std::vector<Bytes>&& commitments, i64 now_unix);
  // Plain path (createBlock): full updates, stake +/- per Accepted flag.
  Block make_plain_block(const std::vector<double>& new_w, const std::vector<Update>& updates, i64 now_unix);
  Block make_empty_block();
  // append (append/replace-if-better); adopts the block's stake map (main.go:1346-1349)
  int commit_block(const Block& b);
  bool is_poisoner(i64 id, bool fedsys = false) const;
  bool is_colluder(i64 id) const { return cfg.colluders > 0 && id >= cfg.collusion_thresh; }
  u64 round_seed(u64 salt) const;
  // The FSM as it will be once `b` is committed (its stake adopted), with a chain holding only b's hash:
  // begin_round / verifier_inboxes / leader_arrivals on it give the next round's plan before `b`'s
  // commit (the engine launches the next round's share MSM while it still reads the audit).
  RoundFSM successor(const Block& b);
};

// FedSys (centralized FL baseline): server node 0 collects NUM_SAMPLES updates.
struct FedSysConfig {
  i64 num_nodes = 0;
  i64 perc_samples = 35;
  bool rand_sample = false;
  double poisoning = 0.0;
  i64 num_samples = 0, random_samples = 0;
  void derive();
};
// Which worker updates the server aggregates this round (with replacement when rand_sample).
std::vector<i64> fedsys_select(const FedSysConfig& c, const std::vector<i64>& submitted, u64 seed);

}  // namespace bsc
