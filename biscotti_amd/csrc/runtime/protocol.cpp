#include "protocol.hpp"

#include <algorithm>
#include <cmath>
#include <iterator>

#include "hash.hpp"

namespace bsc {

void ProtocolConfig::derive() {
  if (num_nodes <= 0) fail("protocol: num_nodes must be > 0");
  num_samples = i64(double(num_nodes) * (double(perc_samples) / 100.0));
  if (num_samples > num_nodes - num_verifiers - num_miners) num_samples = num_nodes - num_verifiers - num_miners;
  krum_thresh = rand_sample ? num_nodes - num_verifiers - num_miners : num_samples;
  total_shares = i64(std::ceil(double(poly_size * 2) / double(num_miners))) * num_miners;
  shares_per_miner = total_shares / num_miners;
  miner_share_thresh = miner_block_div > 0 ? std::max<i64>(num_nodes / miner_block_div, 2) : num_samples / 2;
  poisoning_index = i64(std::ceil(double(num_nodes) * (1.0 - poisoning)));
  collusion_thresh = i64(std::ceil(double(num_nodes) * (1.0 - double(colluders) / 100.0)));
}

// ------------------------------------------------------------------ lottery
Lottery::Lottery(const std::map<i64, i64>& stake, i64 total, const Bytes& in) : input(in) {
  i64 acc = 0;
  for (i64 id = 0; id < total; ++id) {
    auto it = stake.find(id);
    const i64 s = it == stake.end() ? 0 : it->second;
    if (s <= 0) continue;
    acc += s;
    ids.push_back(id);
    cum.push_back(acc);
  }
  if (ids.empty()) fail("lottery: no stake");
}
i64 Lottery::ticket(i64 idx) const {
  return ids[size_t(std::upper_bound(cum.begin(), cum.end(), idx) - cum.begin())];
}
i64 Lottery::draw() {
  if (i + 1 >= input.size()) {
    input = Sha256::digest(input);
    i = 0;
  }
  const i64 idx = i64((size_t(input[i]) * 256 + size_t(input[i + 1])) % size_t(total()));
  ++i;
  return ticket(idx);
}

static size_t distinct_holders(const Lottery& l) { return l.ids.size(); }

void select_roles(const std::map<i64, i64>& stake, const Bytes& hash, i64 nv, i64 na, i64 n,
                  std::vector<i64>* verifiers, std::vector<i64>* miners) {
  Lottery l(stake, n, hash);
  if (i64(distinct_holders(l)) < std::max(nv, na)) fail("lottery: not enough staked peers for committees");
  std::set<i64> vs, ms;
  verifiers->clear();
  miners->clear();
  while (i64(verifiers->size()) < nv) {
    i64 w = l.draw();
    if (vs.insert(w).second) verifiers->push_back(w);
  }
  while (i64(miners->size()) < na) {
    i64 w = l.draw();
    if (ms.insert(w).second) miners->push_back(w);
  }
}

std::vector<i64> select_noisers(const std::map<i64, i64>& stake, const Bytes& out, i64 self, i64 nn, i64 n) {
  return select_noisers(Lottery(stake, n, Bytes{}), out, self, nn);
}

std::vector<i64> select_noisers(const Lottery& table, const Bytes& out, i64 self, i64 nn) {
  Lottery l = table;
  l.input = out;
  l.i = 0;
  const i64 others = i64(l.ids.size()) - (std::binary_search(l.ids.begin(), l.ids.end(), self) ? 1 : 0);
  if (others < nn) fail("lottery: not enough peers for noisers");
  std::set<i64> seen;
  std::vector<i64> res;
  while (i64(res.size()) < nn) {
    i64 w = l.draw();
    if (w != self && seen.insert(w).second) res.push_back(w);
  }
  return res;
}

// ------------------------------------------------------------------ krum
std::vector<double> krum_scores(const double* X, i64 n, i64 d, i64 groupsize) {
  std::vector<double> sq(static_cast<size_t>(n), 0.0), dist(static_cast<size_t>(n * n));
  for (i64 i = 0; i < n; ++i) {
    double s = 0;
    for (i64 k = 0; k < d; ++k) s += X[i * d + k] * X[i * d + k];
    sq[size_t(i)] = s;
  }
  for (i64 i = 0; i < n; ++i)
    for (i64 j = 0; j < n; ++j) {
      double g = 0;
      for (i64 k = 0; k < d; ++k) g += X[i * d + k] * X[j * d + k];
      dist[size_t(i * n + j)] = sq[size_t(i)] + sq[size_t(j)] - 2 * g;
    }
  std::vector<double> scores(static_cast<size_t>(n), 0.0);
  for (i64 i = 0; i < n; ++i) {
    std::vector<double> row(dist.begin() + i * n, dist.begin() + (i + 1) * n);
    std::sort(row.begin(), row.end());
    double s = 0;
    for (i64 k = 1; k < groupsize - 1 && k < n; ++k) s += row[size_t(k)];
    scores[size_t(i)] = s;
  }
  return scores;
}

std::vector<i64> krum_select(const std::vector<double>& scores, i64 n_accept) {
  std::vector<i64> idx(scores.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i64(i);
  std::stable_sort(idx.begin(), idx.end(), [&](i64 a, i64 b) { return scores[size_t(a)] < scores[size_t(b)]; });
  if (n_accept < i64(idx.size())) idx.resize(static_cast<size_t>(std::max<i64>(n_accept, 0)));
  std::sort(idx.begin(), idx.end());
  return idx;
}

u64 splitmix64(u64& s) {
  u64 z = (s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

std::vector<i64> seeded_permutation(i64 n, u64 seed) {
  std::vector<i64> p(static_cast<size_t>(n));
  for (i64 i = 0; i < n; ++i) p[size_t(i)] = i;
  u64 s = seed;
  for (i64 i = n - 1; i > 0; --i) {
    i64 j = i64(splitmix64(s) % u64(i + 1));
    std::swap(p[size_t(i)], p[size_t(j)]);
  }
  return p;
}

// ------------------------------------------------------------------ FSM
RoundFSM::RoundFSM(const ProtocolConfig& c, i64 nf) : cfg(c) {
  cfg.derive();
  chain = Blockchain::with_genesis(static_cast<size_t>(nf));
  for (i64 i = 0; i < cfg.num_nodes; ++i) {
    stake[i] = cfg.default_stake;
    addresses.push_back("127.0.0.1:" + std::to_string(8000 + i));
  }
}

u64 RoundFSM::round_seed(u64 salt) const {
  const Bytes& h = chain.latest().hash;
  u64 s = cfg.seed ^ (u64(iteration) * 0x9e3779b97f4a7c15ULL) ^ (salt * 0xd1b54a32d192ed03ULL);
  for (size_t i = 0; i + 8 <= h.size(); i += 8) s ^= load_le64(h.data() + i) + (i << 3);
  splitmix64(s);
  return s;
}

const RoundPlan& RoundFSM::begin_round(const std::vector<u8>& live) {
  if (i64(live.size()) != cfg.num_nodes) fail("begin_round: live mask size mismatch");
  plan = RoundPlan();
  if (iteration > cfg.max_iterations) { plan.done = true; plan.iteration = iteration; return plan; }
  select_roles(stake, chain.latest().hash, cfg.num_verifiers, cfg.num_miners, cfg.num_nodes, &plan.verifiers,
               &plan.miners);
  std::set<i64> committee(plan.verifiers.begin(), plan.verifiers.end());
  committee.insert(plan.miners.begin(), plan.miners.end());
  for (i64 i = 0; i < cfg.num_nodes; ++i)
    if (!committee.count(i)) plan.workers.push_back(i);
  plan.leader = *std::max_element(plan.miners.begin(), plan.miners.end());
  plan.live = live;
  ++iteration;
  plan.iteration = iteration;
  return plan;
}

std::vector<i64> RoundFSM::verifier_inbox(const std::vector<i64>& submitted) const {
  std::vector<i64> order = seeded_permutation(i64(submitted.size()), round_seed(1));
  std::vector<i64> inbox;
  for (i64 k : order) {
    if (i64(inbox.size()) >= cfg.krum_thresh) break;
    inbox.push_back(submitted[size_t(k)]);
  }
  std::sort(inbox.begin(), inbox.end());
  if (cfg.rand_sample) {
    std::vector<i64> perm = seeded_permutation(i64(inbox.size()), round_seed(2));
    std::vector<i64> s;
    for (i64 k : perm) {
      if (i64(s.size()) >= cfg.num_samples) break;
      s.push_back(inbox[size_t(k)]);
    }
    inbox = s;  // sampled order (krum.go:368-388 keeps permutation order)
  }
  return inbox;
}

std::vector<std::vector<i64>> RoundFSM::verifier_inboxes(const std::vector<i64>& submitted) const {
  std::vector<std::vector<i64>> out;
  if (cfg.shared_inbox) {
    std::vector<i64> one = verifier_inbox(submitted);
    out.assign(plan.verifiers.size(), one);
    return out;
  }
  for (size_t k = 0; k < plan.verifiers.size(); ++k) {
    // verifier k's own arrival order (the network race each verifier process sees)
    std::vector<i64> order = seeded_permutation(i64(submitted.size()), round_seed(1000 + u64(plan.verifiers[k])));
    std::vector<i64> inbox;
    for (i64 j : order) {
      if (i64(inbox.size()) >= cfg.krum_thresh) break;
      inbox.push_back(submitted[size_t(j)]);
    }
    std::sort(inbox.begin(), inbox.end());  // sort.Slice by SourceID (krum.go:304-306)
    if (cfg.rand_sample) {
      // sampleUpdates seeds with the iteration, so every verifier draws the same positions
      std::vector<i64> perm = seeded_permutation(i64(inbox.size()), round_seed(2));
      std::vector<i64> s;
      for (i64 j : perm) {
        if (i64(s.size()) >= cfg.num_samples) break;
        s.push_back(inbox[size_t(j)]);
      }
      inbox = s;
    }
    out.push_back(inbox);
  }
  return out;
}

std::vector<i64> RoundFSM::leader_arrivals() const {
  std::vector<i64> perm = seeded_permutation(i64(plan.workers.size()), round_seed(3));
  std::vector<i64> out;
  out.reserve(perm.size());
  for (i64 j : perm) out.push_back(plan.workers[size_t(j)]);
  return out;
}

i64 RoundFSM::leader_cap_size() const {
  if (!cfg.miner_cap) return 0;
  // NUM_SAMPLES/2 (main.go:360) or num_nodes / miner_block_div (minBlockSize, main.go:348-352), at least 2:
  // the leader only builds a block from > 1 node
  // (main.go:2079) -- in the reference a second share lands while the leader queries the other
  // miners; the same floor as its minBlockSize rule (main.go:347-351)
  return std::max<i64>(cfg.miner_share_thresh, 2);
}

std::vector<i64> RoundFSM::leader_cap(const std::vector<i64>& candidates) const {
  std::vector<i64> out;
  const i64 cap = leader_cap_size();
  if (cap <= 0 || i64(candidates.size()) <= cap) {
    out = candidates;
  } else {
    std::vector<u8> cand(size_t(cfg.num_nodes), 0);   // a flag per peer instead of a node-based set
    for (i64 w : candidates)
      if (w >= 0 && w < cfg.num_nodes) cand[size_t(w)] = 1;
    for (i64 w : leader_arrivals()) {
      if (i64(out.size()) >= cap) break;
      if (cand[size_t(w)]) out.push_back(w);
    }
  }
  std::sort(out.begin(), out.end());
  return out;
}

std::vector<i64> RoundFSM::approve(const std::map<i64, std::vector<i64>>& accepted, bool* verifiers_online) const {
  std::map<i64, i64> sigs;
  bool any = false;
  for (i64 v : plan.verifiers) {
    if (!plan.live[size_t(v)]) continue;
    any = true;
    auto it = accepted.find(v);
    if (it == accepted.end()) continue;
    for (i64 w : it->second) sigs[w]++;
  }
  if (verifiers_online) *verifiers_online = any;
  std::vector<i64> out;
  i64 need = i64(plan.verifiers.size()) / 2;
  for (i64 w : plan.workers) {
    if (!plan.live[size_t(w)]) continue;
    if (!cfg.verification) { out.push_back(w); continue; }
    auto it = sigs.find(w);
    i64 c = it == sigs.end() ? 0 : it->second;
    if (c >= need) out.push_back(w);  // reference rule, incl. its nv=1 quirk (0 >= 0)
  }
  return out;
}

std::map<i64, std::vector<std::pair<i64, i64>>> RoundFSM::route_shares(const std::vector<i64>& approved) const {
  std::vector<i64> ms = plan.miners;
  std::sort(ms.begin(), ms.end(), [&](i64 a, i64 b) { return addresses[size_t(a)] < addresses[size_t(b)]; });
  std::map<i64, std::vector<std::pair<i64, i64>>> routes;
  for (i64 w : approved) {
    i64 part = 0;
    for (i64 m : ms) {
      if (!plan.live[size_t(m)]) continue;  // dial failure: index does not advance
      routes[m].push_back({w, part});
      ++part;
    }
  }
  return routes;
}

RoundFSM::LeaderView RoundFSM::leader_view(const std::map<i64, std::vector<std::pair<i64, i64>>>& routes) const {
  LeaderView lv;
  i64 L = plan.leader;
  lv.leader_online = plan.live[size_t(L)] != 0;
  if (!lv.leader_online) return lv;
  auto own = routes.find(L);
  if (own == routes.end() || own->second.empty()) return lv;  // leader has no shares -> empty block
  // sorted vectors, not node-based sets: this sits on the round's host path between the committee's selection
  // and the block build (std::set allocations made it ~30 us at 60 approved workers)
  auto sorted_ids = [](const std::vector<std::pair<i64, i64>>& v) {
    std::vector<i64> ids;
    ids.reserve(v.size());
    for (auto& wp : v) ids.push_back(wp.first);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    return ids;
  };
  std::vector<i64> inter = sorted_ids(own->second), theirs, nx;
  lv.contributing_miners.push_back(L);
  for (i64 m : plan.miners) {
    if (m == L || !plan.live[size_t(m)]) continue;
    auto it = routes.find(m);
    if (it == routes.end() || it->second.empty()) continue;
    theirs = sorted_ids(it->second);
    nx.clear();
    std::set_intersection(inter.begin(), inter.end(), theirs.begin(), theirs.end(), std::back_inserter(nx));
    inter.swap(nx);
    lv.contributing_miners.push_back(m);
  }
  // the leader fires at NUM_SAMPLES/2 received shares (main.go:360): its list is the first arrivals
  lv.node_list = leader_cap(inter);
  lv.quorum = cfg.shares_per_miner * i64(lv.contributing_miners.size()) >= cfg.poly_size &&
              lv.node_list.size() > 1;
  return lv;
}

std::map<i64, std::vector<i64>> RoundFSM::route_updates(const std::vector<i64>& approved) const {
  std::map<i64, std::vector<i64>> r;
  for (i64 w : approved) {
    std::vector<i64> perm = seeded_permutation(i64(plan.miners.size()), round_seed(100 + u64(w)));
    for (i64 k : perm) {
      i64 m = plan.miners[size_t(k)];
      if (plan.live[size_t(m)]) { r[m].push_back(w); break; }
    }
  }
  // the leader creates its block at NUM_SAMPLES/2 received updates (processUpdate, main.go:1222-1230)
  auto it = r.find(plan.leader);
  if (it != r.end()) it->second = leader_cap(it->second);
  return r;
}

Block RoundFSM::make_secagg_block(const std::vector<double>& new_w, const std::vector<i64>& node_list,
                                  const std::vector<Bytes>& commitments, i64 now_unix) {
  return make_secagg_block(new_w.data(), new_w.size(), node_list, std::vector<Bytes>(commitments), now_unix);
}

Block RoundFSM::make_secagg_block(const double* new_w, size_t n, const std::vector<i64>& node_list,
                                  std::vector<Bytes>&& commitments, i64 now_unix) {
  if (commitments.size() != node_list.size()) fail("make_secagg_block: commitments/node_list mismatch");
  BlockData d;
  d.iteration = iteration;
  if (node_list.empty())
    d.global_w = chain.latest().data.global_w;
  else
    d.global_w.assign(new_w, new_w + n);
  std::map<i64, i64> st = stake;
  d.deltas.resize(node_list.size());
  for (size_t k = 0; k < node_list.size(); ++k) {
    st[node_list[k]] += cfg.stake_unit;
    Update& u = d.deltas[k];
    u.iteration = iteration;
    u.commitment = std::move(commitments[k]);
    u.accepted = true;
  }
  return chain.make_block(std::move(d), std::move(st), now_unix);
}

Block RoundFSM::make_plain_block(const std::vector<double>& new_w, const std::vector<Update>& updates, i64 now_unix) {
  BlockData d;
  d.iteration = iteration;
  d.global_w = new_w;
  std::map<i64, i64> st = stake;
  for (auto& u : updates) st[u.source_id] += u.accepted ? cfg.stake_unit : -cfg.stake_unit;
  d.deltas = updates;
  return chain.make_block(d, st, now_unix);
}

Block RoundFSM::make_empty_block() {
  BlockData d;
  d.iteration = iteration;
  d.global_w = chain.latest().data.global_w;
  return chain.make_block(d, stake, 0);
}

RoundFSM RoundFSM::successor(const Block& b) {
  Blockchain saved = std::move(chain);  // the copy below must not duplicate the whole chain
  chain = Blockchain();
  Block head;                            // the plan reads only the latest hash (roles, round seeds)
  head.hash = b.hash;
  chain.blocks.push_back(std::move(head));
  RoundFSM s = *this;
  chain = std::move(saved);
  if (!b.stake.empty()) s.stake = b.stake;
  s.plan = RoundPlan();
  return s;
}

int RoundFSM::commit_block(const Block& b) {
  int r = chain.add_block(b);
  if (r >= 0 && !b.stake.empty()) stake = b.stake;
  return r;
}

bool RoundFSM::is_poisoner(i64 id, bool fedsys) const {
  if (cfg.poisoning <= 0) return false;
  return fedsys ? id >= cfg.poisoning_index : id > cfg.poisoning_index;
}

void FedSysConfig::derive() {
  num_samples = i64(double(num_nodes) * (double(perc_samples) / 100.0));
  random_samples = 0;
  if (rand_sample) {
    random_samples = num_samples;
    num_samples = num_nodes - 1;
  }
}

std::vector<i64> fedsys_select(const FedSysConfig& c, const std::vector<i64>& submitted, u64 seed) {
  std::vector<i64> perm = seeded_permutation(i64(submitted.size()), seed);
  std::vector<i64> got;
  for (i64 k : perm) {
    if (i64(got.size()) >= c.num_samples) break;
    got.push_back(submitted[size_t(k)]);
  }
  std::sort(got.begin(), got.end());
  if (!c.rand_sample || got.empty()) return got;
  std::vector<i64> s;
  u64 st = seed ^ 0x5851f42d4c957f2dULL;
  for (i64 i = 0; i < c.random_samples; ++i) s.push_back(got[size_t(splitmix64(st) % got.size())]);
  return s;
}

}  // namespace bsc
